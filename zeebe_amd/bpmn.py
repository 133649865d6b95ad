"""A small fluent BPMN builder producing the same XML document order as the
reference's model API (bpmn-model/src/main/java/io/camunda/zeebe/model/bpmn/builder/
AbstractFlowNodeBuilder.java:92-179): ``createTarget`` appends the target node
first and then the connecting sequence flow, unless ``sequenceFlowId`` /
``condition`` created the flow earlier.  Document order matters: the engine
connects sequence flows in reverse document order (ModelWalker.java:75-79),
which fixes every ``getOutgoing()`` order.

Usage mirrors ``Bpmn.createExecutableProcess(id).startEvent()...done()``.
"""
from xml.sax.saxutils import escape, quoteattr

BPMN_NS = "http://www.omg.org/spec/BPMN/20100524/MODEL"
ZEEBE_NS = "http://camunda.org/schema/zeebe/1.0"


class _Node:
    def __init__(self, kind, id_, **attrs):
        self.kind = kind
        self.id = id_
        self.attrs = attrs
        self.job_type = None
        self.retries = None
        self.default = None
        self.condition = None
        self.source = None
        self.target = None
        self.message = None  # (message id, name, correlation key expression) of a message catch event
        self.timer = None    # timeDuration of a timer catch event
        self.attached_to = None     # boundary event: the activity it is attached to
        self.cancel_activity = True  # boundary event: interrupting (BoundaryEvent default)
        self.multi = None    # activity: (isSequential, inputCollection, inputElement, extra attrs)
        self.mappings = []   # zeebe:ioMapping entries: ("input" | "output", source, target)


class ProcessBuilder:
    def __init__(self, process_id):
        self.process_id = process_id
        self.root = []       # the process's children, document order
        self.children = self.root  # the container being built (the process or an embedded sub-process)
        self.nodes = {}
        self._container_of = {}  # node id -> the children list it lives in
        self._stack = []     # enclosing containers while building a sub-process
        self.current = None
        self._pending_flow = None
        self._counter = 0

    # ---- helpers ----
    def _gen_id(self, kind):
        self._counter += 1
        return "%s_%d" % (kind, self._counter)

    def _flow(self):
        if self._pending_flow is None:
            f = _Node("sequenceFlow", self._gen_id("sequenceFlow"))
            self.children.append(f)
            self._pending_flow = f
        return self._pending_flow

    def _add_node(self, kind, id_):
        id_ = id_ or self._gen_id(kind)
        n = _Node(kind, id_)
        self.children.append(n)
        self.nodes[id_] = n
        self._container_of[id_] = self.children
        if self.current is not None:
            self._connect(n)
        self.current = n
        return n

    def _connect(self, target):
        f = self._flow()
        f.source = self.current.id
        f.target = target.id
        self._pending_flow = None

    # ---- fluent API ----
    def startEvent(self, id_=None):
        self._add_node("startEvent", id_)
        return self

    def endEvent(self, id_=None):
        self._add_node("endEvent", id_)
        return self

    def serviceTask(self, id_=None, job_type=None, retries=None):
        n = self._add_node("serviceTask", id_)
        n.job_type = job_type if job_type is not None else "task"
        n.retries = retries
        return self

    def jobWorkerTask(self, kind, id_=None, job_type=None, retries=None):
        """sendTask / scriptTask / businessRuleTask with a zeebe:taskDefinition (job workers, like
        serviceTask: BpmnElementProcessors.java:46-60)."""
        n = self._add_node(kind, id_)
        n.job_type = job_type if job_type is not None else "task"
        n.retries = retries
        return self

    def zeebeJobType(self, t):
        self.current.job_type = t
        return self

    def zeebeTaskHeader(self, key, value):
        """AbstractJobWorkerTaskBuilder.zeebeTaskHeader: a <zeebe:header> in the task's <zeebe:taskHeaders>."""
        self.current.headers = getattr(self.current, "headers", []) + [(key, value)]
        return self

    def task(self, id_=None):
        self._add_node("task", id_)
        return self

    def manualTask(self, id_=None):
        self._add_node("manualTask", id_)
        return self

    def intermediateThrowEvent(self, id_=None):
        self._add_node("intermediateThrowEvent", id_)
        return self

    def intermediateCatchEvent(self, id_=None):
        self._add_node("intermediateCatchEvent", id_)
        return self

    def message(self, name, correlation_key=None):
        """IntermediateCatchEventBuilder.message(m -> m.name(name).zeebeCorrelationKeyExpression(key)):
        a <message> with a zeebe:subscription under the definitions (ZeebeExpression: "=" prefix);
        StartEventBuilder.message(name): a message start event, no correlation key."""
        expr = None if correlation_key is None else \
            correlation_key if correlation_key.startswith("=") else "=" + correlation_key
        self.current.message = ("Message_%s" % self.current.id, name, expr)
        return self

    def subProcess(self, id_=None):
        """AbstractFlowNodeBuilder.subProcess(id).embeddedSubProcess(): the sub-process node and its
        incoming flow in the current container, then its children inside it (startEvent() there
        starts a new path); ``subProcessDone()`` continues after the sub-process."""
        n = self._add_node("subProcess", id_)
        n.children = []
        self._stack.append((self.children, n))
        self.children = n.children
        self.current = None
        self._pending_flow = None
        return self

    def subProcessDone(self):
        self.children, n = self._stack.pop()
        self.current = n
        self._pending_flow = None
        return self

    def eventSubProcess(self, id_=None):
        """AbstractFlowNodeBuilder / ProcessBuilder.eventSubProcess(id, e -> ...): a subProcess with
        triggeredByEvent="true" in the current container, not connected; its children follow (its start
        event: startEvent(..).error(code)); ``eventSubProcessDone()`` returns to where the builder was."""
        id_ = id_ or self._gen_id("eventSubProcess")
        n = _Node("subProcess", id_, triggeredByEvent="true")
        n.children = []
        self.children.append(n)
        self.nodes[id_] = n
        self._container_of[id_] = self.children
        self._stack.append((self.children, self.current))
        self.children = n.children
        self.current = None
        self._pending_flow = None
        return self

    def eventSubProcessDone(self):
        self.children, self.current = self._stack.pop()
        self._pending_flow = None
        return self

    def boundaryEvent(self, id_=None):
        """AbstractActivityBuilder.boundaryEvent(id): a boundaryEvent sibling of the current activity
        appended to its container (no connecting flow), attachedToRef = the activity; the builder
        continues from the boundary event."""
        activity = self.current
        id_ = id_ or self._gen_id("boundaryEvent")
        n = _Node("boundaryEvent", id_)
        n.attached_to = activity.id
        self.children.append(n)
        self.nodes[id_] = n
        self._container_of[id_] = self.children
        self.current = n
        self._pending_flow = None
        return self

    def error(self, error_code=None):
        """BoundaryEventBuilder / StartEventBuilder.error(code): an <errorEventDefinition> referring to an
        <error errorCode>; no code: a catch-all errorEventDefinition without errorRef."""
        self.current.error = error_code if error_code is not None else ""
        return self

    def multiInstance(self, input_collection, input_element=None, sequential=False, **extra):
        """AbstractActivityBuilder.multiInstance(b -> b.zeebeInputCollectionExpression(..)
        .zeebeInputElement(..).sequential()/.parallel()): a <multiInstanceLoopCharacteristics> with a
        zeebe:loopCharacteristics (MultiInstanceLoopCharacteristicsBuilder); `extra` adds attributes
        (outputCollection, outputElement) or a completionCondition."""
        expr = input_collection if input_collection.startswith("=") else "=" + input_collection
        self.current.multi = (bool(sequential), expr, input_element, extra)
        return self

    # ZeebeVariablesMappingBuilder (bpmn-model/.../builder/ZeebeVariablesMappingBuilder.java): the
    # *Expression forms prefix the source with "=" (asZeebeExpression); the plain forms keep a static
    # source.  They apply to the current node (after subProcessDone(): the sub-process).
    def _mapping(self, kind, source, target):
        self.current.mappings.append((kind, source, target))
        return self

    def zeebeInputExpression(self, source, target):
        return self._mapping("input", source if source.startswith("=") else "=" + source, target)

    def zeebeOutputExpression(self, source, target):
        return self._mapping("output", source if source.startswith("=") else "=" + source, target)

    def zeebeInput(self, source, target):
        return self._mapping("input", source, target)

    def zeebeOutput(self, source, target):
        return self._mapping("output", source, target)

    def cancelActivity(self, cancel):
        self.current.cancel_activity = bool(cancel)
        return self

    def moveToActivity(self, id_):
        return self.moveToNode(id_)

    def timerWithCycle(self, cycle):
        """BoundaryEventBuilder.timerWithCycle: <timerEventDefinition><timeCycle>."""
        self.current.timer = ("cycle", cycle)
        return self

    def timerWithDuration(self, duration):
        """IntermediateCatchEventBuilder.timerWithDuration: <timerEventDefinition><timeDuration>."""
        self.current.timer = duration
        return self

    def timerWithDurationExpression(self, expression):
        """AbstractTimerEventDefinitionBuilder.timerWithDurationExpression: the FEEL expression as
        `=expression` in <timeDuration>."""
        return self.timerWithDuration("=" + expression)

    def timerWithCycleExpression(self, expression):
        """BoundaryEventBuilder.timerWithCycleExpression: `=expression` in <timeCycle>."""
        return self.timerWithCycle("=" + expression)

    def exclusiveGateway(self, id_=None):
        self._add_node("exclusiveGateway", id_)
        return self

    def parallelGateway(self, id_=None):
        self._add_node("parallelGateway", id_)
        return self

    def sequenceFlowId(self, id_):
        f = self._flow()
        f.id = id_
        return self

    def conditionExpression(self, expr):
        # AbstractFlowNodeBuilder.conditionExpression -> asZeebeExpression: "=" prefix
        self._flow().condition = expr if expr.startswith("=") else "=" + expr
        return self

    def condition(self, expr):
        self._flow().condition = expr
        return self

    def defaultFlow(self):
        # AbstractExclusiveGatewayBuilder.defaultFlow: the current flow is created now
        self.current.default = self._flow()
        return self

    def moveToLastExclusiveGateway(self):
        for c in reversed(self.children):
            if c.kind == "exclusiveGateway":
                self.current = c
                return self
        raise ValueError("no exclusive gateway")

    def moveToLastGateway(self):
        # AbstractFlowNodeBuilder.findLastGateway: walk unique predecessors from the current node
        node = self.current
        while True:
            prev = [c.source for c in self._container_of[node.id] if c.kind == "sequenceFlow" and c.target == node.id]
            if len(prev) != 1:
                raise ValueError("Unable to determine an unique previous gateway of " + node.id)
            node = self.nodes[prev[0]]
            if node.kind in ("exclusiveGateway", "parallelGateway"):
                self.current = node
                return self

    def moveToNode(self, id_):
        self.current = self.nodes[id_]
        self.children = self._container_of[id_]
        return self

    def connectTo(self, id_):
        self._connect(self.nodes[id_])
        self.current = self.nodes[id_]
        return self

    def done(self):
        out = ['<?xml version="1.0" encoding="UTF-8" standalone="no"?>',
               '<definitions xmlns="%s" xmlns:zeebe="%s" id="definitions" targetNamespace="%s">'
               % (BPMN_NS, ZEEBE_NS, BPMN_NS),
               '  <process id=%s isExecutable="true">' % quoteattr(self.process_id)]
        catches = []
        errors = []

        def render(children, ind):
            for c in children:
                if c.kind == "sequenceFlow":
                    attrs = 'id=%s sourceRef=%s targetRef=%s' % (quoteattr(c.id), quoteattr(c.source), quoteattr(c.target))
                    if c.condition is None:
                        out.append("%s<sequenceFlow %s/>" % (ind, attrs))
                    else:
                        out.append("%s<sequenceFlow %s><conditionExpression>%s</conditionExpression></sequenceFlow>"
                                   % (ind, attrs, escape(c.condition)))
                elif c.kind in ("serviceTask", "sendTask", "scriptTask", "businessRuleTask"):
                    retries = ' retries="%s"' % c.retries if c.retries is not None else ""
                    hs = getattr(c, "headers", [])
                    th = "<zeebe:taskHeaders>%s</zeebe:taskHeaders>" % "".join(
                        "<zeebe:header key=%s value=%s/>" % (quoteattr(k), quoteattr(v)) for k, v in hs) if hs else ""
                    out.append('%s<%s id=%s><extensionElements><zeebe:taskDefinition type=%s%s/>%s%s'
                               '</extensionElements>%s</%s>' % (ind, c.kind, quoteattr(c.id), quoteattr(c.job_type),
                                                               retries, th, io(c), loop(c), c.kind))
                elif c.kind == "intermediateCatchEvent" and c.message:
                    catches.append(c)
                    out.append('%s<intermediateCatchEvent id=%s><messageEventDefinition id=%s messageRef=%s/>'
                               '</intermediateCatchEvent>' % (ind, quoteattr(c.id), quoteattr(c.id + "_med"),
                                                              quoteattr(c.message[0])))
                elif c.kind == "endEvent" and getattr(c, "error", None) is not None:
                    errors.append(c)  # EndEventBuilder.error(code): an error end event (a code is required)
                    out.append('%s<endEvent id=%s><errorEventDefinition id=%s errorRef=%s/></endEvent>'
                               % (ind, quoteattr(c.id), quoteattr(c.id + "_eed"), quoteattr("Error_" + c.id)))
                elif c.kind == "startEvent" and getattr(c, "error", None) is not None:
                    ref = ' errorRef=%s' % quoteattr("Error_" + c.id) if c.error else ""
                    if c.error:
                        errors.append(c)
                    out.append('%s<startEvent id=%s><errorEventDefinition id=%s%s/></startEvent>'
                               % (ind, quoteattr(c.id), quoteattr(c.id + "_eed"), ref))
                elif c.kind == "startEvent" and c.message:
                    catches.append(c)
                    out.append('%s<startEvent id=%s><messageEventDefinition id=%s messageRef=%s/></startEvent>'
                               % (ind, quoteattr(c.id), quoteattr(c.id + "_med"), quoteattr(c.message[0])))
                elif c.kind == "intermediateCatchEvent" and c.timer:
                    out.append('%s<intermediateCatchEvent id=%s><timerEventDefinition id=%s><timeDuration>%s'
                               '</timeDuration></timerEventDefinition></intermediateCatchEvent>'
                               % (ind, quoteattr(c.id), quoteattr(c.id + "_ted"), escape(c.timer)))
                elif c.kind == "boundaryEvent":
                    cancel = "" if c.cancel_activity else ' cancelActivity="false"'
                    body = ""
                    if isinstance(c.timer, tuple):
                        body = ('<timerEventDefinition id=%s><timeCycle>%s</timeCycle></timerEventDefinition>'
                                % (quoteattr(c.id + "_ted"), escape(c.timer[1])))
                    elif c.timer:
                        body = ('<timerEventDefinition id=%s><timeDuration>%s</timeDuration></timerEventDefinition>'
                                % (quoteattr(c.id + "_ted"), escape(c.timer)))
                    elif c.message:
                        catches.append(c)
                        body = '<messageEventDefinition id=%s messageRef=%s/>' % (quoteattr(c.id + "_med"),
                                                                                quoteattr(c.message[0]))
                    elif getattr(c, "error", None) is not None:
                        ref = ' errorRef=%s' % quoteattr("Error_" + c.id) if c.error else ""
                        if c.error:
                            errors.append(c)
                        body = '<errorEventDefinition id=%s%s/>' % (quoteattr(c.id + "_eed"), ref)
                    out.append('%s<boundaryEvent id=%s attachedToRef=%s%s>%s</boundaryEvent>'
                               % (ind, quoteattr(c.id), quoteattr(c.attached_to), cancel, body))
                elif c.kind == "exclusiveGateway" and c.default:
                    out.append("%s<exclusiveGateway id=%s default=%s/>" % (ind, quoteattr(c.id), quoteattr(c.default.id)))
                elif c.kind == "subProcess":
                    ext = "<extensionElements>%s</extensionElements>" % io(c) if c.mappings else ""
                    trig = ' triggeredByEvent="true"' if c.attrs.get("triggeredByEvent") else ""
                    out.append("%s<subProcess id=%s%s>%s" % (ind, quoteattr(c.id), trig, ext))
                    render(c.children, ind + "  ")
                    out.append("%s</subProcess>" % ind)
                elif c.multi:
                    out.append("%s<%s id=%s>%s</%s>" % (ind, c.kind, quoteattr(c.id), loop(c), c.kind))
                else:
                    out.append("%s<%s id=%s/>" % (ind, c.kind, quoteattr(c.id)))

        def io(c):
            if not c.mappings:
                return ""
            return "<zeebe:ioMapping>%s</zeebe:ioMapping>" % "".join(
                "<zeebe:%s source=%s target=%s/>" % (k, quoteattr(src), quoteattr(t)) for k, src, t in c.mappings)

        def loop(c):
            if not c.multi:
                return ""
            seq, coll, elem, extra = c.multi
            attrs = 'inputCollection=%s' % quoteattr(coll)
            if elem:
                attrs += ' inputElement=%s' % quoteattr(elem)
            for k in ("outputCollection", "outputElement"):
                if k in extra:
                    attrs += ' %s=%s' % (k, quoteattr(extra[k]))
            cc = ('<completionCondition>%s</completionCondition>' % escape(extra["completionCondition"])
                  if "completionCondition" in extra else "")
            return ('<multiInstanceLoopCharacteristics isSequential="%s">%s<extensionElements>'
                    '<zeebe:loopCharacteristics %s/></extensionElements></multiInstanceLoopCharacteristics>'
                    % ("true" if seq else "false", cc, attrs))

        render(self.root, "    ")
        out.append("  </process>")
        for c in catches:
            if c.message[2] is None:
                out.append('  <message id=%s name=%s/>' % tuple(quoteattr(x) for x in c.message[:2]))
                continue
            out.append('  <message id=%s name=%s><extensionElements><zeebe:subscription correlationKey=%s/>'
                       '</extensionElements></message>' % tuple(quoteattr(x) for x in c.message))
        for c in errors:
            out.append('  <error id=%s errorCode=%s/>' % (quoteattr("Error_" + c.id), quoteattr(c.error)))
        out.append("</definitions>")
        return "\n".join(out) + "\n"


def createExecutableProcess(process_id):
    return ProcessBuilder(process_id)


# ---- the BASELINE.json workloads -------------------------------------------------------------

def linear_process(n_tasks=10, process_id="linear", job_type="benchmark-task"):
    """Config 2: start -> task1 .. taskN -> end."""
    b = createExecutableProcess(process_id).startEvent("start")
    for i in range(1, n_tasks + 1):
        b.serviceTask("task%d" % i, job_type)
    return b.endEvent("end").done()


def xor_process(process_id="xorProcess", condition="= amount > 1000"):
    """Config 3: start -> xor -> [high: condition -> endHigh] [default -> endLow]."""
    return (createExecutableProcess(process_id).startEvent("start").exclusiveGateway("xor")
            .sequenceFlowId("high").conditionExpression(condition).endEvent("endHigh")
            .moveToNode("xor").sequenceFlowId("low").defaultFlow().endEvent("endLow").done())


def fork_join_process(branches=8, process_id="forkjoin", tasks=False, job_type="branch"):
    """Config 4: start -> fork(parallel, N out) -> N flows [-> task_i] -> join(parallel, N in) -> end."""
    b = createExecutableProcess(process_id).startEvent("start").parallelGateway("fork")
    for i in range(1, branches + 1):
        b.moveToNode("fork").sequenceFlowId("f%d" % i)
        if tasks:
            b.serviceTask("t%d" % i, job_type)
            b.sequenceFlowId("j%d" % i)
        if i == 1:
            b.parallelGateway("join")
        else:
            b.connectTo("join")
    b.moveToNode("join").sequenceFlowId("toEnd").endEvent("end")
    return b.done()


def sub_process_process(inner="task", process_id="process", job_type="task"):
    """EmbeddedSubProcessTest.java:41-80 shapes: start -> sub-process(start -> [inner] -> end) -> end.
    inner: "none" (NO_TASK_SUB_PROCESS), "task" (ONE_TASK_SUB_PROCESS), "parallel"
    (PARALLEL_TASKS_SUB_PROCESS: fork -> task-1 / task-2 -> join), "nested" (a nested sub-process)."""
    b = createExecutableProcess(process_id).startEvent().subProcess("sub-process").startEvent()
    if inner == "task":
        b.serviceTask("task", job_type)
    elif inner == "parallel":
        (b.parallelGateway("fork").serviceTask("task-1", "task-1").sequenceFlowId("join-1").parallelGateway("join")
         .moveToNode("fork").serviceTask("task-2", "task-2").sequenceFlowId("join-2").connectTo("join"))
    elif inner == "nested":
        b.subProcess("nestedSubProcess").startEvent().endEvent().subProcessDone()
    b.endEvent().subProcessDone()
    return b.endEvent().done()


def message_catch_process(process_id="process", message_name="msg", correlation_key="key", catch_id="catch"):
    """Config 5: start -> message catch (name, `= correlation_key`) -> end
    (MessageCorrelationMultiplePartitionsTest.java:43-49 shape)."""
    return (createExecutableProcess(process_id).startEvent("start").intermediateCatchEvent(catch_id)
            .message(message_name, correlation_key).endEvent("end").done())


def message_boundary_process(process_id="boundaryEventProcess", message_name="msg", correlation_key="key",
                             task_id="task", job_type="type", flow_id="to-end2", interrupting=True):
    """MessageCatchElementTest.BOUNDARY_EVENT_PROCESS (engine/src/test/.../message/MessageCatchElementTest.java:
    71-80): start -> service task with an interrupting message boundary event (-> end2) -> end;
    interrupting=False: NON_INT_BOUNDARY_EVENT_PROCESS (:81-91, cancelActivity(false))."""
    b = createExecutableProcess(process_id).startEvent("start").serviceTask(task_id, job_type)
    b.boundaryEvent("boundary")
    if not interrupting:
        b.cancelActivity(False)
    b.message(message_name, correlation_key).sequenceFlowId(flow_id).endEvent("end2")
    return b.moveToActivity(task_id).endEvent("end").done()


def multi_instance_process(items=(10, 20, 30), sequential=False, input_element="item", process_id="process",
                           element_id="task", job_type="task", inner="serviceTask", after=None):
    """MultiInstanceActivityTest.process (engine/src/test/.../multiinstance/MultiInstanceActivityTest.java:
    98-108): start -> a multi-instance activity over a static collection -> [after: a service task] ->
    end.  `items` is the FEEL list (a sequence of ints / strings, or the literal text)."""
    if isinstance(items, str):
        coll = items
    else:
        lit = lambda v: ('"%s"' % v if isinstance(v, str) else "null" if v is None  # noqa: E731
                         else ("true" if v else "false") if isinstance(v, bool) else str(v))
        coll = "= [" + ", ".join(lit(v) for v in items) + "]"
    b = createExecutableProcess(process_id).startEvent("start")
    if inner == "serviceTask":
        b.serviceTask(element_id, job_type)
    else:
        getattr(b, inner)(element_id)
    b.multiInstance(coll, input_element, sequential)
    if after:
        b.serviceTask(after, after)
    return b.endEvent("end").done()


def job_types_of(xml):
    """Static job types (zeebe:taskDefinition type) a BPMN XML declares."""
    import re
    if isinstance(xml, bytes):
        xml = xml.decode()
    return set(m for m in re.findall(r'taskDefinition[^>]*?\stype="([^"=][^"]*)"', xml))


def message_start_names_of(xml):
    """Message names of the message start events a BPMN XML declares (startEvent > messageEventDefinition
    messageRef -> <message name>)."""
    import re
    if isinstance(xml, bytes):
        xml = xml.decode()
    refs = set(re.findall(r'<(?:\w+:)?startEvent\b[^>]*>\s*<(?:\w+:)?messageEventDefinition\b[^>]*?\smessageRef="([^"]*)"',
                          xml))
    names = dict(re.findall(r'<(?:\w+:)?message\b[^>]*?\sid="([^"]*)"[^>]*?\sname="([^"]*)"', xml))
    names.update((i, n) for n, i in re.findall(r'<(?:\w+:)?message\b[^>]*?\sname="([^"]*)"[^>]*?\sid="([^"]*)"', xml))
    return {names[r] for r in refs if r in names}


def message_names_of(xml):
    """Static message names (<message name="...">) a BPMN XML declares."""
    import re
    if isinstance(xml, bytes):
        xml = xml.decode()
    return set(re.findall(r'<(?:\w+:)?message\b[^>]*?\sname="([^"=][^"]*)"', xml))
