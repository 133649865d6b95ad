"""Random structured BPMN processes inside the executor's subset (the idea of the reference's
test-util/.../bpmn/random generator: blocks of tasks, exclusive split/merge and parallel fork/join,
nested).  Used to drive the GPU executor and the CPU oracle with the same inputs.

Bounds keep every process inside the device limits (<= 8 waiting elements per instance, <= 16
join counters, a default flow on every exclusive split so no incident is raised).  With
``sub_processes`` a block can be an embedded sub-process holding a nested sequence (start ->
blocks -> end), never inside a parallel branch (one active instance per sub-process element).
With ``boundaries`` a task outside parallel branches may carry a timer boundary event whose path
ends in an end event or (interrupting ones) merges back after the task (one timer per instance at a
time; a sub-process may carry one too, with none inside it).  With ``multi_instance`` a task outside parallel branches may be a multi-instance activity over
a static list (MultiInstanceActivityTest's shapes): parallel or sequential, the inputElement `x`, an
outputCollection (its own name) of `= x` or `= loopCounter`, and a completionCondition.  With ``errors`` a
task outside parallel branches may carry an error boundary event (code E1 or E2, or a catch-all) and a
sub-process without a timer boundary event one of its own (sometimes a second one with the other code);
its path ends in an end event or (always interrupting) merges back after the activity."""
from xml.sax.saxutils import escape, quoteattr

BPMN_NS = "http://www.omg.org/spec/BPMN/20100524/MODEL"
ZEEBE_NS = "http://camunda.org/schema/zeebe/1.0"


class _Gen:
    def __init__(self, rng, max_depth, max_blocks, messages, pass_through=False, tasks=True, sub_processes=False,
                 task_kinds=False, boundaries=False, multi_instance=False, errors=False):
        self.rng = rng
        self.errors = errors
        self.error_codes = set()
        self.multi_instance = multi_instance
        self.boundaries = boundaries
        self.task_kinds = task_kinds
        self.sub_processes = sub_processes
        self.scope = None  # the sub-process being filled (None: the process)
        self.subs = 0
        self.tasks = tasks
        self.pass_through = pass_through
        self.max_depth = max_depth
        self.max_blocks = max_blocks
        self.messages = messages
        self.nodes = []   # (kind, id, extra)
        self.flows = []   # [id, src, tgt, condition or None]
        self.defaults = {}
        self.n = 0
        self.join_slots = 0
        self.catches = 0

    def _id(self, kind):
        self.n += 1
        return "%s_%d" % (kind, self.n)

    def node(self, kind, **extra):
        nid = self._id(kind)
        self.nodes.append((kind, nid, dict(extra, scope=self.scope)))
        return nid

    def flow(self, src, tgt, cond=None):
        fid = self._id("flow")
        self.flows.append([fid, src, tgt, cond, self.scope])
        return fid

    def condition(self):
        r = self.rng
        a = int(r.integers(0, 1000))
        kind = int(r.integers(0, 4))
        if kind == 0:
            return "= amount > %d" % a
        if kind == 1:
            return "= amount <= %d" % a
        if kind == 2:
            b = int(r.integers(a, 1001))
            return "= amount >= %d and amount < %d" % (a, b)
        return "= amount = %d or amount > %d" % (a, int(r.integers(500, 1000)))

    def error_boundary(self, activity):
        r = self.rng
        code = ("E1", "E2", "")[int(r.integers(0, 3))]
        if code:
            self.error_codes.add(code)
        b = self.node("boundaryEvent", attached=activity, error=code, cancel=True)
        if int(r.integers(0, 3)) == 0:  # a second error boundary event with another code, to its own end
            other = "E2" if code == "E1" else "E1"
            self.error_codes.add(other)
            self.flow(self.node("boundaryEvent", attached=activity, error=other, cancel=True), self.node("endEvent"))
        if int(r.integers(0, 2)):
            self.flow(b, self.node("endEvent"))
            return activity
        merge = self.node("exclusiveGateway")
        self.flow(activity, merge)
        self.flow(b, merge)
        return merge

    def sequence(self, cur, depth, width):
        for _ in range(int(self.rng.integers(0, self.max_blocks + 1))):
            cur = self.block(cur, depth, width)
        return cur

    def block(self, cur, depth, width):
        r = self.rng
        choices = ["task", "task"] if self.tasks else ["pass"]
        if depth < self.max_depth:
            choices += ["xor", "xor"]
            if width * 2 <= 8 and self.join_slots + 4 <= 16:
                choices.append("par")
        if self.messages and self.catches < 1 and width == 1:
            choices.append("catch")
        if self.pass_through:
            choices.append("pass")
        if self.sub_processes and width == 1 and depth < self.max_depth and self.subs < 3:
            choices.append("sub")
        c = choices[int(r.integers(0, len(choices)))]
        if c == "sub":  # embedded sub-process: start -> blocks -> end inside, one persistent slot
            self.subs += 1
            sp = self.node("subProcess")
            self.flow(cur, sp)
            outer, self.scope = self.scope, sp
            # a timer boundary event on the sub-process (then none inside it: one timer per instance)
            timed = self.boundaries and int(r.integers(0, 3)) == 0
            inner_b, self.boundaries = self.boundaries, self.boundaries and not timed
            st = self.node("startEvent")
            end = self.sequence(st, depth + 1, width)
            en = self.node("endEvent")
            self.flow(end, en)
            self.scope = outer
            self.boundaries = inner_b
            if not timed and self.errors and int(r.integers(0, 3)) == 0:
                return self.error_boundary(sp)
            if timed:
                cancel = bool(int(r.integers(0, 3)))
                b = self.node("boundaryEvent", attached=sp, duration="PT%dS" % int(r.integers(1, 120)), cancel=cancel)
                if not cancel or int(r.integers(0, 2)):
                    self.flow(b, self.node("endEvent"))
                    return sp
                merge = self.node("exclusiveGateway")
                self.flow(sp, merge)
                self.flow(b, merge)
                return merge
            return sp
        if c == "pass":  # elements without behaviour: undefined / manual task, none throw event
            t = self.node(("task", "manualTask", "intermediateThrowEvent")[int(r.integers(0, 3))])
            self.flow(cur, t)
            return t
        if c == "task":
            kind = "serviceTask"
            if self.task_kinds:  # the job worker tasks (JobWorkerTaskBlockBuilder's choices)
                kind = ("serviceTask", "sendTask", "scriptTask", "businessRuleTask")[int(r.integers(0, 4))]
            t = self.node(kind, job_type="job%d" % int(r.integers(0, 3)))
            self.flow(cur, t)
            if self.multi_instance and width == 1 and int(r.integers(0, 2)):
                seq = bool(int(r.integers(0, 2)))
                items = [int(v) for v in r.integers(1, 5, int(r.integers(1, 4)))]
                loop = {"seq": seq, "coll": "= [%s]" % ", ".join(map(str, items))}
                if int(r.integers(0, 2)):
                    loop["out"] = ("= x", "= loopCounter")[int(r.integers(0, 2))]
                if int(r.integers(0, 2)):
                    loop["cond"] = ("= x >= 3", "= numberOfCompletedInstances >= 2", "= loopCounter = 2")[int(r.integers(0, 3))]
                self.nodes[-1][2]["loop"] = loop
                return t
            if self.boundaries and width == 1 and int(r.integers(0, 2)):
                # an interrupting timer boundary event: its own end, or back through an XOR merge
                cancel = bool(int(r.integers(0, 3)))
                timer = "PT%dS" % int(r.integers(1, 120))
                if not cancel and int(r.integers(0, 2)):  # a cycle (non-interrupting only)
                    timer = ("R/" if int(r.integers(0, 2)) else "R%d/" % int(r.integers(1, 4))) + timer
                b = self.node("boundaryEvent", attached=t, duration=timer, cancel=cancel)
                # a non-interrupting one always ends on its own (merging back would double the token)
                if int(r.integers(0, 2)) or not self.nodes[-1][2]["cancel"]:
                    self.flow(b, self.node("endEvent"))
                    return t
                merge = self.node("exclusiveGateway")
                self.flow(t, merge)
                self.flow(b, merge)
                return merge
            if self.errors and width == 1 and int(r.integers(0, 2)):
                return self.error_boundary(t)
            return t
        if c == "catch":
            self.catches += 1
            e = self.node("intermediateCatchEvent")
            self.flow(cur, e)
            return e
        if c == "xor":
            split = self.node("exclusiveGateway")
            self.flow(cur, split)
            merge = self.node("exclusiveGateway")
            k = int(r.integers(2, 4))
            dflt = int(r.integers(0, k))
            for b in range(k):
                first = len(self.flows)
                end = self.sequence(split, depth + 1, width)
                if end == split:  # empty branch: direct flow to the merge
                    fid = self.flow(split, merge, None if b == dflt else self.condition())
                else:
                    fid = next(f[0] for f in self.flows[first:] if f[1] == split)  # the branch's first flow
                    next(f for f in self.flows[first:] if f[1] == split)[3] = None if b == dflt else self.condition()
                    self.flow(end, merge)
                if b == dflt:
                    self.defaults[split] = fid
            return merge
        fork = self.node("parallelGateway")
        self.flow(cur, fork)
        join = self.node("parallelGateway")
        k = int(r.integers(2, 4)) if width * 3 <= 8 and self.join_slots + 4 <= 16 else 2
        self.join_slots += k + 1  # the flows into the join and the one into the fork
        for _ in range(k):
            end = self.sequence(fork, depth + 1, width * k)
            self.flow(end, join)
        return join


def random_process(rng, process_id="random", max_depth=2, max_blocks=3, messages=False, pass_through=False,
                   tasks=True, sub_processes=False, task_kinds=False, boundaries=False, multi_instance=False,
                   errors=False, event_sub_processes=False):
    """tasks=False: no wait states (the CREATE batch runs the instance to its end); task_kinds: job
    worker tasks among service / send / script / business-rule tasks."""
    g = _Gen(rng, max_depth, max_blocks, messages, pass_through or not tasks, tasks, sub_processes, task_kinds,
             boundaries, multi_instance, errors)
    # event_sub_processes: one or two error-start event sub-processes of the process (E1 / E2 / catch-all), each
    # a recovery task or none before its end event (drawn first: the rest of the process keeps its draws
    # relative to each other)
    esps = []
    if event_sub_processes:
        for i in range(int(rng.integers(1, 3))):
            code = ("E1", "E2", "")[int(rng.integers(0, 3))]
            if code:
                g.error_codes.add(code)
            esps.append(("esp_%d" % i, code, bool(int(rng.integers(0, 2)))))
    start = g.node("startEvent")
    cur = g.sequence(start, 0, 1)
    end = g.node("endEvent")
    g.flow(cur, end)
    out = ['<?xml version="1.0" encoding="UTF-8"?>',
           '<definitions xmlns="%s" xmlns:zeebe="%s" id="d" targetNamespace="%s">' % (BPMN_NS, ZEEBE_NS, BPMN_NS),
           '  <process id=%s isExecutable="true">' % quoteattr(process_id)]
    def render(scope, ind):
        for kind, nid, extra in g.nodes:
            if extra["scope"] != scope:
                continue
            if kind in ("serviceTask", "sendTask", "scriptTask", "businessRuleTask"):
                loop = extra.get("loop")
                lc = ""
                if loop:
                    lc = ('<multiInstanceLoopCharacteristics isSequential="%s"><extensionElements>'
                          '<zeebe:loopCharacteristics inputCollection=%s inputElement="x"%s/></extensionElements>%s'
                          '</multiInstanceLoopCharacteristics>'
                          % ("true" if loop["seq"] else "false", quoteattr(loop["coll"]),
                             ' outputCollection=%s outputElement=%s' % (quoteattr("out_" + nid), quoteattr(loop["out"]))
                             if "out" in loop else "",
                             "<completionCondition>%s</completionCondition>" % escape(loop["cond"]) if "cond" in loop else ""))
                # with task kinds, every other task has static task headers (derived from its id, no draw from
                # the generator: the campaigns' processes keep their shapes)
                th = ""
                if g.task_kinds and sum(map(ord, nid)) % 2:
                    th = "<zeebe:taskHeaders>%s</zeebe:taskHeaders>" % "".join(
                        "<zeebe:header key=%s value=%s/>" % (quoteattr(k), quoteattr(v))
                        for k, v in (("workerVersion", "42"), (nid, "h-" + nid), ("Aa", "1"), ("BB", "2")))
                out.append('%s<%s id=%s><extensionElements><zeebe:taskDefinition type=%s/>%s'
                           '</extensionElements>%s</%s>' % (ind, kind, quoteattr(nid), quoteattr(extra["job_type"]), th,
                                                            lc, kind))
            elif kind == "exclusiveGateway" and nid in g.defaults:
                out.append('%s<exclusiveGateway id=%s default=%s/>' % (ind, quoteattr(nid), quoteattr(g.defaults[nid])))
            elif kind == "intermediateCatchEvent":
                out.append('%s<intermediateCatchEvent id=%s><messageEventDefinition messageRef="msg_def"/>'
                           '</intermediateCatchEvent>' % (ind, quoteattr(nid)))
            elif kind == "boundaryEvent" and "error" in extra:
                ref = ' errorRef="err_%s"' % extra["error"] if extra["error"] else ""
                out.append('%s<boundaryEvent id=%s attachedToRef=%s><errorEventDefinition%s/></boundaryEvent>'
                           % (ind, quoteattr(nid), quoteattr(extra["attached"]), ref))
            elif kind == "boundaryEvent":
                tag = "timeCycle" if extra["duration"].startswith("R") else "timeDuration"
                out.append('%s<boundaryEvent id=%s attachedToRef=%s%s><timerEventDefinition><%s>%s'
                           '</%s></timerEventDefinition></boundaryEvent>'
                           % (ind, quoteattr(nid), quoteattr(extra["attached"]),
                              "" if extra["cancel"] else ' cancelActivity="false"', tag, extra["duration"], tag))
            elif kind == "subProcess":
                out.append("%s<subProcess id=%s>" % (ind, quoteattr(nid)))
                render(nid, ind + "  ")
                out.append("%s</subProcess>" % ind)
            else:
                out.append("%s<%s id=%s/>" % (ind, kind, quoteattr(nid)))
        for fid, src, tgt, cond, fscope in g.flows:
            if fscope != scope:
                continue
            attrs = "id=%s sourceRef=%s targetRef=%s" % (quoteattr(fid), quoteattr(src), quoteattr(tgt))
            if cond is None:
                out.append("%s<sequenceFlow %s/>" % (ind, attrs))
            else:
                out.append("%s<sequenceFlow %s><conditionExpression>%s</conditionExpression></sequenceFlow>"
                           % (ind, attrs, escape(cond)))

    for eid, code, task in esps:
        ref = ' errorRef="err_%s"' % code if code else ""
        out.append('    <subProcess id="%s" triggeredByEvent="true">' % eid)
        out.append('      <startEvent id="%s_start"><errorEventDefinition%s/></startEvent>' % (eid, ref))
        out.append('      <endEvent id="%s_end"/>' % eid)
        if task:
            out.append('      <serviceTask id="%s_task"><extensionElements><zeebe:taskDefinition type="recover"/>'
                       '</extensionElements></serviceTask>' % eid)
            out.append('      <sequenceFlow id="%s_f1" sourceRef="%s_start" targetRef="%s_task"/>' % (eid, eid, eid))
            out.append('      <sequenceFlow id="%s_f2" sourceRef="%s_task" targetRef="%s_end"/>' % (eid, eid, eid))
        else:
            out.append('      <sequenceFlow id="%s_f1" sourceRef="%s_start" targetRef="%s_end"/>' % (eid, eid, eid))
        out.append('    </subProcess>')
    render(None, "    ")
    out.append("  </process>")
    if messages:
        out.append('  <message id="msg_def" name="msg"><extensionElements>'
                   '<zeebe:subscription correlationKey="= key"/></extensionElements></message>')
    for code in sorted(g.error_codes):
        out.append('  <error id="err_%s" errorCode="%s"/>' % (code, code))
    out.append("</definitions>")
    return "\n".join(out) + "\n"
