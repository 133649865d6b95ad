"""Embedded sub-processes on the CPU oracle, pinned by the assertions of the
reference's EmbeddedSubProcessTest (engine/src/test/java/io/camunda/zeebe/engine/processing/bpmn/
subprocess/EmbeddedSubProcessTest.java), and the product compiler's element numbering / flow order
for nested containers against the oracle's."""
import pytest

from helpers import complete_commands, create_commands
from oracle.oracle import Oracle, OracleError
from test_compiler import Compiled
from zeebe_amd import abi, bpmn
from zeebe_amd.native import ZbhipError

BASE = 1 << 51
ET = {n: i for i, n in enumerate(abi.ELEMENT_TYPES)}
PI_ACTIVATED = abi.PI_INTENT_IDS["ELEMENT_ACTIVATED"]
PI_ACTIVATING = abi.PI_INTENT_IDS["ELEMENT_ACTIVATING"]


def _run(o, cmds):
    o.clear_records()
    o.submit(cmds)
    o.run()
    return o.records()


def _types(o, recs, proc=0):
    """(bpmnElementType, intent) of every PROCESS_INSTANCE record, as the tests extract them."""
    out = []
    for r in recs:
        if r["value_type"] != abi.VT_PROCESS_INSTANCE or r["record_type"] == abi.RT_REJECTION:
            continue
        out.append((abi.ELEMENT_TYPES[o.element_type(proc, int(r["element_idx"]))], abi.PI_INTENTS[int(r["intent"])]))
    return out


def _subsequence(seq, sub):
    it = iter(seq)
    return all(any(x == y for x in it) for y in sub)


def _create(o, xml):
    proc = o.deploy(xml)
    return _run(o, create_commands(1, proc))


def test_should_activate_sub_process():
    # EmbeddedSubProcessTest.shouldActivateSubProcess (:82-115)
    o = Oracle()
    recs = _create(o, bpmn.sub_process_process("none"))
    assert _subsequence(_types(o, recs), [
        ("SEQUENCE_FLOW", "SEQUENCE_FLOW_TAKEN"),
        ("SUB_PROCESS", "ELEMENT_ACTIVATING"),
        ("SUB_PROCESS", "ELEMENT_ACTIVATED"),
        ("START_EVENT", "ACTIVATE_ELEMENT"),
        ("START_EVENT", "ELEMENT_ACTIVATING"),
        ("START_EVENT", "ELEMENT_ACTIVATED")])
    pik = BASE + 1
    act = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == PI_ACTIVATING
           and o.element_type(0, int(r["element_idx"])) == ET["SUB_PROCESS"]][0]
    assert int(act["scope_key"]) == pik  # hasFlowScopeKey(processInstanceKey)
    assert o.element_id(0, int(act["element_idx"])) == "sub-process"


def test_should_complete_sub_process():
    # EmbeddedSubProcessTest.shouldCompleteSubProcess (:243-271)
    o = Oracle()
    recs = _create(o, bpmn.sub_process_process("none"))
    t = _types(o, recs)
    assert _subsequence(t, [
        ("END_EVENT", "ELEMENT_COMPLETED"),
        ("SUB_PROCESS", "ELEMENT_COMPLETING"),
        ("SUB_PROCESS", "ELEMENT_COMPLETED"),
        ("SEQUENCE_FLOW", "SEQUENCE_FLOW_TAKEN"),
        ("END_EVENT", "ACTIVATE_ELEMENT")])
    assert ("PROCESS", "ELEMENT_COMPLETED") in t
    assert o.state() == ["KEY|latestKey|%d" % (BASE + 10)]


def test_should_create_job_for_inner_task():
    # EmbeddedSubProcessTest.shouldCreateJobForInnerTask (:273-300)
    o = Oracle()
    recs = _create(o, bpmn.sub_process_process("task"))
    task = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == PI_ACTIVATED
            and o.element_type(0, int(r["element_idx"])) == ET["SERVICE_TASK"]][0]
    job = [r for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED][0]
    assert o.element_id(0, int(job["element_idx"])) == "task"
    assert int(job["scope_key"]) == int(task["key"])  # hasElementInstanceKey(serviceTaskActivated.getKey())
    assert int(job["process_idx"]) == int(task["process_idx"])
    # the task's flow scope is the sub-process instance, whose flow scope is the process instance
    sub = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == PI_ACTIVATED
           and o.element_type(0, int(r["element_idx"])) == ET["SUB_PROCESS"]][0]
    assert int(task["scope_key"]) == int(sub["key"]) and int(sub["scope_key"]) == BASE + 1
    st = o.state()
    assert any(r.startswith("ELEMENT_INSTANCE_KEY|%d|parentKey=%d,childCount=1," % (int(sub["key"]), BASE + 1))
               for r in st)
    assert "ELEMENT_INSTANCE_PARENT_CHILD|%d|%d" % (int(sub["key"]), int(task["key"])) in st


def test_should_complete_nested_sub_process():
    # EmbeddedSubProcessTest.shouldCompleteNestedSubProcess (:386-420)
    o = Oracle()
    recs = _create(o, bpmn.sub_process_process("nested"))
    assert _subsequence(_types(o, recs), [
        ("SUB_PROCESS", "ELEMENT_ACTIVATED"),
        ("SUB_PROCESS", "ELEMENT_ACTIVATED"),
        ("END_EVENT", "ELEMENT_COMPLETED"),
        ("SUB_PROCESS", "ELEMENT_COMPLETED"),
        ("END_EVENT", "ELEMENT_COMPLETED"),
        ("SUB_PROCESS", "ELEMENT_COMPLETED"),
        ("END_EVENT", "ELEMENT_COMPLETED"),
        ("PROCESS", "ELEMENT_COMPLETED")])


def test_should_complete_sub_process_with_parallel_flow():
    # EmbeddedSubProcessTest.shouldCompleteSubProcessWithParallelFlow (:422-467): fork inside the
    # sub-process, task-1 -> end and task-2 -> end (no join), task-1 completed first
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("sub-process").startEvent()
    (b.parallelGateway("fork").serviceTask("task-1", "task-1").endEvent()
     .moveToLastGateway().serviceTask("task-2", "task-2").endEvent().subProcessDone().endEvent())
    o = Oracle()
    recs = list(_create(o, b.done()))
    jobs = {o.element_id(0, int(r["element_idx"])): int(r["key"]) for r in recs
            if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED}
    inst = 0
    for name in ("task-1", "task-2"):
        recs += list(_run(o, complete_commands([inst], [jobs[name] - BASE - 1])))
    assert _subsequence(_types(o, recs), [
        ("PARALLEL_GATEWAY", "ELEMENT_COMPLETED"),
        ("SERVICE_TASK", "ELEMENT_COMPLETED"),
        ("END_EVENT", "ELEMENT_COMPLETED"),
        ("SERVICE_TASK", "ELEMENT_COMPLETED"),
        ("END_EVENT", "ELEMENT_COMPLETED"),
        ("SUB_PROCESS", "ELEMENT_COMPLETING"),
        ("SUB_PROCESS", "ELEMENT_COMPLETED"),
        ("PROCESS", "ELEMENT_COMPLETED")])
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


def test_join_counters_of_a_sub_process_are_keyed_by_its_instance():
    # NUMBER_OF_TAKEN_SEQUENCE_FLOWS [flowScopeKey, gateway, flow]: the sub-process instance is the
    # flow scope of its gateways (PARALLEL_TASKS_SUB_PROCESS, EmbeddedSubProcessTest.java:49-62)
    o = Oracle()
    recs = _create(o, bpmn.sub_process_process("parallel"))
    sub = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == PI_ACTIVATED
           and o.element_type(0, int(r["element_idx"])) == ET["SUB_PROCESS"]][0]
    jobs = {o.element_id(0, int(r["element_idx"])): int(r["key"]) for r in recs
            if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED}
    _run(o, complete_commands([0], [jobs["task-1"] - BASE - 1]))
    assert "NUMBER_OF_TAKEN_SEQUENCE_FLOWS|%d|join|join-1|1" % int(sub["key"]) in o.state()
    _run(o, complete_commands([0], [jobs["task-2"] - BASE - 1]))
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


def test_compiler_numbers_nested_containers_like_the_oracle():
    for xml in [bpmn.sub_process_process(k) for k in ("none", "task", "parallel", "nested")]:
        c = Compiled(xml)
        o = Oracle()
        p = o.deploy(xml)
        ids = [c.id(i) for i in range(len(c.els))]
        assert ids == [o.element_id(p, i) for i in range(len(c.els))]
        for i, e in enumerate(c.els):
            if e["element_type"] == ET["SUB_PROCESS"]:
                assert c.els[e["start_event"]]["element_type"] == ET["START_EVENT"]
                assert c.els[e["start_event"]]["flow_scope"] == i
        assert c.els[0]["start_event"] == ids.index("startEvent_1")
    c = Compiled(bpmn.sub_process_process("parallel"))
    ids = [c.id(i) for i in range(len(c.els))]
    sub = ids.index("sub-process")
    assert all(c.els[ids.index(x)]["flow_scope"] == sub for x in ("fork", "join", "task-1", "task-2", "join-1"))
    assert c.els[sub]["flow_scope"] == 0
    # getOutgoing() of the fork: reverse document order within the sub-process (the flow to task-2
    # comes later in the document)
    out = c.outgoing("fork")
    assert [c.id(int(c.els[ids.index(f)]["flow_target"])) for f in out] == ["task-2", "task-1"]


@pytest.mark.parametrize("inner", [
    '<subProcess id="s" triggeredByEvent="true"><startEvent id="s0"/></subProcess>',
    '<subProcess id="s"><multiInstanceLoopCharacteristics/><startEvent id="s0"/></subProcess>',
    '<subProcess id="s"><endEvent id="s1"/></subProcess>',
])
def test_sub_processes_outside_the_subset_are_refused(inner):
    xml = ('<definitions xmlns="http://www.omg.org/spec/BPMN/20100524/MODEL"><process id="p" isExecutable="true">'
           '<startEvent id="a"/>%s<sequenceFlow id="f" sourceRef="a" targetRef="s"/></process></definitions>' % inner)
    with pytest.raises(ZbhipError):
        Compiled(xml)
    with pytest.raises(OracleError):
        Oracle().deploy(xml)


def _job_worker_chain():
    b = bpmn.createExecutableProcess("process").startEvent("start")
    for kind in ("serviceTask", "sendTask", "scriptTask", "businessRuleTask"):
        b.jobWorkerTask(kind, kind + "-1", kind)
    return b.endEvent("end").done()


def test_job_worker_tasks_create_jobs():
    # BpmnElementProcessors.java:46-60: send tasks and script / business-rule tasks with a
    # zeebe:taskDefinition run JobWorkerTaskProcessor -- JOB:CREATED with the element's type and id
    o = Oracle()
    recs = list(_create(o, _job_worker_chain()))
    kinds = ["SERVICE_TASK", "SEND_TASK", "SCRIPT_TASK", "BUSINESS_RULE_TASK"]
    for step, kind in enumerate(kinds):
        job = [r for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED][-1]
        assert abi.ELEMENT_TYPES[o.element_type(0, int(job["element_idx"]))] == kind
        assert ("JOBS|%d|type=%s," % (int(job["key"]), o.element_id(0, int(job["element_idx"])).split("-")[0])
                in "\n".join(o.state()))
        recs = list(_run(o, complete_commands([0], [int(job["key"]) - BASE - 1])))
    assert ("PROCESS", "ELEMENT_COMPLETED") in _types(o, recs)


@pytest.mark.parametrize("ext", ['<zeebe:script expression="=1" resultVariable="x"/>',
                                 '<zeebe:calledDecision decisionId="d" resultVariable="x"/>'])
def test_script_and_decision_tasks_without_a_job_are_refused(ext):
    tag = "scriptTask" if "script" in ext else "businessRuleTask"
    xml = ('<definitions xmlns="http://www.omg.org/spec/BPMN/20100524/MODEL" xmlns:zeebe="http://camunda.org/schema/zeebe/1.0">'
           '<process id="p" isExecutable="true"><startEvent id="a"/><%s id="t"><extensionElements>%s'
           '</extensionElements></%s><sequenceFlow id="f" sourceRef="a" targetRef="t"/></process></definitions>'
           % (tag, ext, tag))
    with pytest.raises(ZbhipError):
        Compiled(xml)
    with pytest.raises(OracleError):
        Oracle().deploy(xml)
