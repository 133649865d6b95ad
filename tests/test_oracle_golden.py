"""Pins the CPU oracle against the golden vectors: the hand-derived
Appendix-A sequences and the assertions of the reference's own engine tests,
transcribed into the same EngineRule-like style."""
import numpy as np
import pytest

from helpers import (amount_docs, complete_commands, create_commands, load_appendix_a, process_xml,
                     split_batches, symbolic)
from oracle.oracle import Oracle, OracleError
from zeebe_amd import abi, bpmn

BASE = 1 << 51


def _sym(o, recs):
    return symbolic(recs, o.element_id, o.name, o.reason)


def _run_single(o, cmds, docs=None):
    o.clear_records()
    o.submit(cmds, docs)
    o.run()
    return o.records()


CASES = load_appendix_a()


@pytest.mark.parametrize("name", sorted(CASES))
def test_appendix_a_sequences(name):
    case = CASES[name]
    o = Oracle()
    proc = o.deploy(process_xml(case["process"]))
    docs = None
    if "amount" in case:
        docs = amount_docs([case["amount"]], o.intern("amount"))
        cmds = create_commands(1, proc)
        cmds["doc_count"] = 1
    else:
        cmds = create_commands(1, proc)
    got = [_sym(o, _run_single(o, cmds, docs))]
    for _ in case["batches"][1:]:
        # complete the job created by the previous batch (JobClient.complete)
        prev = o.records()
        job_keys = [int(r["key"]) for r in prev if r["value_type"] == abi.VT_JOB and r["intent"] == 0]
        assert len(job_keys) == 1
        got.append(_sym(o, _run_single(o, complete_commands([0], [job_keys[0] - BASE - 1]))))
    assert got == case["batches"]


def test_one_task_final_state_is_empty_after_completion():
    o = Oracle()
    proc = o.deploy(process_xml({"fixture": "one_task.bpmn"}))
    _run_single(o, create_commands(1, proc))
    st = o.state()
    # waiting state: process + task instances, the job and its activatable row (DbJobState.create)
    assert any(r.startswith("JOBS|%d|type=benchmark-task,retries=3" % (BASE + 6)) for r in st)
    assert "JOB_STATES|%d|ACTIVATABLE" % (BASE + 6) in st
    assert "JOB_ACTIVATABLE|benchmark-task|<default>|%d" % (BASE + 6) in st
    assert "EVENT_SCOPE|%d|accepting=1,interrupted=0,interrupting=,boundaryElementIds=" % (BASE + 5) in st
    assert "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY|2251799813685249|%d" % (BASE + 1) in st
    _run_single(o, complete_commands([0], [5]))
    # everything removed on completion; only the key generator remains
    assert o.state() == ["KEY|latestKey|%d" % (BASE + 9)]


def test_create_process_instance_sequence():
    # CreateProcessInstanceTest.java:173-211 -- start COMPLETED -> SFT -> ACTIVATE(end);
    # SFT flowScopeKey = PI key
    xml = bpmn.createExecutableProcess("process").startEvent("start").endEvent("end").done()
    o = Oracle()
    recs = _run_single(o, create_commands(1, o.deploy(xml)))
    s = _sym(o, recs)
    i = s.index(["E", "PI", "ELEMENT_COMPLETED", "start", "k3", "k1"])
    assert s[i + 1][:3] == ["E", "PI", "SEQUENCE_FLOW_TAKEN"] and s[i + 1][5] == "k1"
    assert s[i + 2][:4] == ["C", "PI", "ACTIVATE_ELEMENT", "end"]
    assert s[-1][:4] == ["E", "PI", "ELEMENT_COMPLETED", "process"]


def _pairs(o, recs, only_events=False):
    return [(o.element_id(int(r["process_idx"]), int(r["element_idx"])), abi.intent_name(5, int(r["intent"])))
            for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE
            and (not only_events or r["record_type"] == abi.RT_EVENT)]


def _contains_sequence(seq, sub):
    return any(seq[i:i + len(sub)] == sub for i in range(len(seq) - len(sub) + 1))


def _contains_subsequence(seq, sub):
    it = iter(seq)
    return all(any(x == s for x in it) for s in sub)


def test_parallel_gateway_pass_through():
    # ParallelGatewayTest.shouldPassThroughParallelGateway (:142-180)
    xml = (bpmn.createExecutableProcess("process").startEvent("start").sequenceFlowId("flow1")
           .parallelGateway("fork").sequenceFlowId("flow2").endEvent("end").done())
    o = Oracle()
    p = _pairs(o, _run_single(o, create_commands(1, o.deploy(xml))), only_events=True)
    assert _contains_sequence(p, [
        ("fork", "ELEMENT_ACTIVATING"), ("fork", "ELEMENT_ACTIVATED"), ("fork", "ELEMENT_COMPLETING"),
        ("fork", "ELEMENT_COMPLETED"), ("flow2", "SEQUENCE_FLOW_TAKEN"), ("end", "ELEMENT_ACTIVATING"),
        ("end", "ELEMENT_ACTIVATED"), ("end", "ELEMENT_COMPLETING"), ("end", "ELEMENT_COMPLETED"),
        ("process", "ELEMENT_COMPLETING"), ("process", "ELEMENT_COMPLETED")])


def test_parallel_gateway_completes_scope():
    # ParallelGatewayTest.shouldCompleteScopeOnParallelGateway (:182-208)
    xml = (bpmn.createExecutableProcess("process").startEvent("start").sequenceFlowId("flow1")
           .parallelGateway("fork").done())
    o = Oracle()
    p = _pairs(o, _run_single(o, create_commands(1, o.deploy(xml))))
    assert _contains_sequence(p, [("fork", "ELEMENT_COMPLETED"), ("process", "COMPLETE_ELEMENT")])


def test_parallel_gateway_merge_once():
    # ParallelGatewayTest.shouldMergeParallelBranches (:210-233)
    xml = (bpmn.createExecutableProcess("process").startEvent("start").parallelGateway("fork")
           .sequenceFlowId("flow1").parallelGateway("join").endEvent("end").moveToNode("fork")
           .sequenceFlowId("flow2").connectTo("join").done())
    o = Oracle()
    recs = _run_single(o, create_commands(1, o.deploy(xml)))
    p = _pairs(o, recs)
    assert _contains_subsequence(p, [("flow1", "SEQUENCE_FLOW_TAKEN"), ("join", "ELEMENT_ACTIVATING")])
    assert _contains_subsequence(p, [("flow2", "SEQUENCE_FLOW_TAKEN"), ("join", "ELEMENT_ACTIVATING")])
    assert p.count(("join", "ELEMENT_ACTIVATING")) == 1


def test_parallel_gateway_rejects_activate_when_flow_taken_twice():
    # ParallelGatewayTest.shouldRejectActivateCommandWhenSequenceFlowIsTakenTwice (:354-401)
    xml = (bpmn.createExecutableProcess("process").startEvent().parallelGateway("splitting")
           .parallelGateway("joining").moveToNode("splitting").exclusiveGateway("exclusive")
           .moveToNode("splitting").connectTo("exclusive").moveToNode("exclusive").connectTo("joining")
           .moveToNode("joining").endEvent("endEvent").done())
    o = Oracle()
    recs = _run_single(o, create_commands(1, o.deploy(xml)))
    rej = [(i, r) for i, r in enumerate(recs) if r["record_type"] == abi.RT_REJECTION]
    assert len(rej) == 2
    for i, r in rej:
        assert r["rejection_type"] == abi.REJ_INVALID_STATE
        assert o.reason(i) == ("Expected to be able to activate parallel gateway 'joining', "
                               "but not all sequence flows have been taken.")
    p = _pairs(o, recs)
    assert p.count(("joining", "ELEMENT_ACTIVATED")) == 1


def test_parallel_gateway_scope_completes_when_all_paths_completed():
    # ParallelGatewayTest.shouldCompleteScopeWhenAllPathsCompleted (:85-106)
    xml = (bpmn.createExecutableProcess("process").startEvent("start").parallelGateway("fork")
           .serviceTask("task1", "type1").endEvent("end1").moveToNode("fork")
           .serviceTask("task2", "type2").endEvent("end2").done())
    o = Oracle()
    recs = _run_single(o, create_commands(1, o.deploy(xml)))
    jobs = {o.element_id(int(r["process_idx"]), int(r["element_idx"])): int(r["key"])
            for r in recs if r["value_type"] == abi.VT_JOB}
    out = []
    for t in ("task1", "task2"):
        out.extend(_pairs(o, _run_single(o, complete_commands([0], [jobs[t] - BASE - 1]))))
    ends = [e for e, i in out if e.startswith("end") and i == "ELEMENT_COMPLETED"]
    assert ends == ["end1", "end2"]
    assert ("process", "ELEMENT_COMPLETED") in out and out.count(("process", "ELEMENT_COMPLETED")) == 1


def test_parallel_gateway_only_triggers_when_all_branches_activated():
    # ParallelGatewayTest.shouldOnlyTriggerGatewayWhenAllBranchesAreActivated (:235-286)
    xml = (bpmn.createExecutableProcess("process").startEvent().parallelGateway("fork")
           .exclusiveGateway("exclusiveJoin").moveToLastGateway().connectTo("exclusiveJoin")
           .sequenceFlowId("joinFlow1").parallelGateway("join").moveToNode("fork")
           .serviceTask("waitState", "type").sequenceFlowId("joinFlow2").connectTo("join").endEvent().done())
    o = Oracle()
    recs = _run_single(o, create_commands(1, o.deploy(xml)))
    p1 = _pairs(o, recs)
    assert p1.count(("joinFlow1", "SEQUENCE_FLOW_TAKEN")) == 2
    assert ("join", "ELEMENT_ACTIVATING") not in p1
    job = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB][0]
    p2 = _pairs(o, _run_single(o, complete_commands([0], [job - BASE - 1])))
    assert _contains_subsequence(p1 + p2, [("joinFlow1", "SEQUENCE_FLOW_TAKEN"), ("joinFlow1", "SEQUENCE_FLOW_TAKEN"),
                                           ("joinFlow2", "SEQUENCE_FLOW_TAKEN"), ("join", "ELEMENT_ACTIVATING")])


def _xor_split_model():
    return (bpmn.createExecutableProcess("process").startEvent().exclusiveGateway("xor").sequenceFlowId("s1")
            .conditionExpression("foo < 5").endEvent("a").moveToLastGateway().sequenceFlowId("s2")
            .conditionExpression("foo >= 5 and foo < 10").endEvent("b").moveToLastExclusiveGateway()
            .defaultFlow().sequenceFlowId("s3").endEvent("c").done())


def test_exclusive_gateway_split():
    # ExclusiveGatewayTest.shouldSplitOnExclusiveGateway (:40-86)
    o = Oracle()
    proc = o.deploy(_xor_split_model())
    foo = o.intern("foo")
    cmds = create_commands(3, proc)
    cmds["doc_count"] = 1
    cmds["doc_begin"] = [0, 1, 2]
    recs = _run_single(o, cmds, amount_docs([4, 8, 12], foo))
    ends = {}
    for r in recs:
        if r["value_type"] == 5 and r["intent"] == 5 and r["record_type"] == 0:
            e = o.element_id(int(r["process_idx"]), int(r["element_idx"]))
            if e in ("a", "b", "c"):
                ends[int(r["source_index"])] = e
    assert ends == {0: "a", 1: "b", 2: "c"}


def test_exclusive_gateway_decimal_and_boundaries():
    # `= amount > 1000` over int and scaled-decimal inputs (config 3 / 3b)
    o = Oracle()
    proc = o.deploy(bpmn.xor_process())
    amount = o.intern("amount")
    vals = [999, 1000, 1001, 0, 2000]
    cmds = create_commands(len(vals), proc)
    cmds["doc_count"] = 1
    cmds["doc_begin"] = np.arange(len(vals))
    recs = _run_single(o, cmds, amount_docs(vals, amount))
    taken = [o.element_id(int(r["process_idx"]), int(r["element_idx"])) for r in recs
             if r["value_type"] == 5 and r["intent"] == 1 and
             o.element_id(int(r["process_idx"]), int(r["element_idx"])) in ("high", "low")]
    assert taken == ["low", "low", "high", "low", "high"]
    # decimals (scale 1e6): 1000.01 > 1000, 1000.00 not
    o2 = Oracle()
    proc = o2.deploy(bpmn.xor_process())
    amount = o2.intern("amount")
    dec = [1000_010000, 1000_000000, 999_990000]
    cmds = create_commands(3, proc)
    cmds["doc_count"] = 1
    cmds["doc_begin"] = np.arange(3)
    recs = _run_single(o2, cmds, amount_docs(dec, amount, decimal=True))
    taken = [o2.element_id(int(r["process_idx"]), int(r["element_idx"])) for r in recs
             if r["value_type"] == 5 and r["intent"] == 1 and
             o2.element_id(int(r["process_idx"]), int(r["element_idx"])) in ("high", "low")]
    assert taken == ["high", "low", "low"]


def test_exclusive_gateway_missing_variable_raises_an_incident():
    # a null operand of `>` makes the result NULL, not a boolean -> incident EXTRACT_VALUE_ERROR
    # (ExpressionProcessor.java:356-368; tests/test_oracle_incidents.py pins the records)
    o = Oracle()
    proc = o.deploy(bpmn.xor_process())
    o.submit(create_commands(1, proc))
    o.run()
    recs = o.records()
    assert int(recs[-1]["value_type"]) == abi.VT_INCIDENT and int(recs[-1]["partition"]) == abi.ERR_EXTRACT_VALUE_ERROR


def test_exclusive_gateway_no_outgoing_flow_completes_scope():
    # ExclusiveGatewayTest (:289-320): a gateway without outgoing flows is an implicit end
    xml = bpmn.createExecutableProcess("process").startEvent().exclusiveGateway("xor").done()
    o = Oracle()
    p = _pairs(o, _run_single(o, create_commands(1, o.deploy(xml))))
    assert _contains_sequence(p, [("xor", "ELEMENT_COMPLETED"), ("process", "COMPLETE_ELEMENT")])


def test_complete_job_twice_is_rejected():
    # JobCommandPreconditionChecker NOT_FOUND text
    o = Oracle()
    proc = o.deploy(process_xml({"fixture": "one_task.bpmn"}))
    _run_single(o, create_commands(1, proc))
    _run_single(o, complete_commands([0], [5]))
    recs = _run_single(o, complete_commands([0], [5]))
    assert len(recs) == 1 and recs[0]["record_type"] == abi.RT_REJECTION
    assert recs[0]["rejection_type"] == abi.REJ_NOT_FOUND
    assert o.reason(0) == "Expected to complete job with key '%d', but no such job was found" % (BASE + 6)


def test_complete_job_with_variables_merges_into_process_scope():
    # CompleteJobTest (:49-150): variables of the job are propagated to the process scope
    o = Oracle()
    proc = o.deploy(process_xml({"fixture": "one_task.bpmn"}))
    _run_single(o, create_commands(1, proc))
    x = o.intern("x")
    cmds = complete_commands([0], [5])
    cmds["doc_count"] = 1
    recs = _run_single(o, cmds, amount_docs([7], x))
    s = _sym(o, recs)
    # JOB:COMPLETED, PROCESS_EVENT:TRIGGERING, COMPLETE cmd, COMPLETING, VARIABLE:CREATED (scope PI), COMPLETED ...
    assert s[4] == ["E", "VAR", "CREATED", "x", "k8", "k1"]
    assert s[5][:4] == ["E", "PI", "ELEMENT_COMPLETED", "task"]


def test_batch_limit_overflow_goes_to_log():
    # ProcessingStateMachine.java:345-417: with maxCommandsInBatch=3 the follow-up commands beyond the
    # limit are written to the log and processed later as their own batches; per-instance order holds.
    xml = process_xml({"fixture": "one_task.bpmn"})
    full = Oracle()
    full_recs = _run_single(full, create_commands(1, full.deploy(xml)))
    small = Oracle(max_commands_in_batch=3)
    small_recs = _run_single(small, create_commands(1, small.deploy(xml)))
    assert len(set(int(r["source_index"]) for r in small_recs)) > 1
    strip = lambda s: [t[:4] for t in s]  # noqa: E731
    assert strip(_sym(small, small_recs)) == strip(_sym(full, full_recs))


def test_many_instances_are_independent():
    # per-instance sequences do not depend on the other instances in the window
    xml = bpmn.linear_process(3)
    o = Oracle()
    proc = o.deploy(xml)
    recs = _run_single(o, create_commands(50, proc))
    batches = split_batches(recs)
    assert len(batches) == 50
    shapes = {tuple((int(recs[i]["record_type"]), int(recs[i]["intent"])) for i in b) for b in batches}
    assert len(shapes) == 1
    keys = [int(recs[b[0]]["key"]) - BASE for b in batches]
    assert keys == [1 + 6 * i for i in range(50)]


# ---- elements without behaviour: undefined task, manual task, none
# intermediate throw event -- UndefinedTaskProcessor / ManualTaskProcessor (task/*.java) and
# IntermediateThrowEventProcessor.NoneIntermediateThrowEventBehavior (event/*.java:113-138)

PASS_THROUGH = {"task": ("TASK", "UNSPECIFIED"), "manualTask": ("MANUAL_TASK", "UNSPECIFIED"),
                "intermediateThrowEvent": ("INTERMEDIATE_THROW_EVENT", "NONE")}


def _types(o, recs, elem_id):
    from oracle import logserial as LS
    tables = o.process_tables()
    out = set()
    for r in recs:
        if r["value_type"] != abi.VT_PROCESS_INSTANCE:
            continue
        p, e = int(r["process_idx"]), int(r["element_idx"])
        if o.element_id(p, e) == elem_id:
            el = tables[p]["elements"][e]
            out.add((LS.ELEMENT_TYPE[el[0]], LS.EVENT_TYPE[el[1]]))
    return out


@pytest.mark.parametrize("kind", sorted(PASS_THROUGH))
def test_pass_through_element_types(kind):
    # BpmnElementTypeTest (:367-396): every record of the element carries its element type;
    # BpmnEventTypeTest (:54-62, :415-424): NONE for the none throw event, UNSPECIFIED for tasks
    b = bpmn.createExecutableProcess("process").startEvent("start")
    xml = getattr(b, kind)("elem").endEvent("end").done()
    o = Oracle()
    recs = _run_single(o, create_commands(1, o.deploy(xml)))
    assert _types(o, recs, "elem") == {PASS_THROUGH[kind]}
    p = _pairs(o, recs)
    assert _contains_sequence(p, [
        ("elem", "ACTIVATE_ELEMENT"), ("elem", "ELEMENT_ACTIVATING"), ("elem", "ELEMENT_ACTIVATED"),
        ("elem", "COMPLETE_ELEMENT"), ("elem", "ELEMENT_COMPLETING"), ("elem", "ELEMENT_COMPLETED")])
    assert p[-1] == ("process", "ELEMENT_COMPLETED")
    assert o.state() == ["KEY|latestKey|%d" % (BASE + 7)]


def test_none_throw_event_ends_the_path():
    # BpmnEventTypeTest "None Throw Event" model: start -> throw, no end event; the throw event's
    # completion ends the execution path and completes the process
    xml = bpmn.createExecutableProcess("process").startEvent("start").intermediateThrowEvent("elem").done()
    o = Oracle()
    p = _pairs(o, _run_single(o, create_commands(1, o.deploy(xml))), only_events=True)
    assert p[-4:] == [("elem", "ELEMENT_COMPLETING"), ("elem", "ELEMENT_COMPLETED"),
                      ("process", "ELEMENT_COMPLETING"), ("process", "ELEMENT_COMPLETED")]


def test_pass_through_elements_mixed_with_jobs_and_gateways():
    xml = (bpmn.createExecutableProcess("process").startEvent("start").task("t1")
           .parallelGateway("fork").manualTask("m1").serviceTask("s1", "job").parallelGateway("join")
           .moveToNode("fork").intermediateThrowEvent("e1").connectTo("join")
           .moveToNode("join").endEvent("end").done())
    o = Oracle()
    recs = _run_single(o, create_commands(1, o.deploy(xml)))
    jobs = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB]
    assert len(jobs) == 1
    p = _pairs(o, recs, only_events=True)
    assert ("e1", "ELEMENT_COMPLETED") in p and ("m1", "ELEMENT_COMPLETED") in p and ("t1", "ELEMENT_COMPLETED") in p
    assert ("process", "ELEMENT_COMPLETED") not in p
    recs = _run_single(o, complete_commands([0], [jobs[0] - BASE - 1]))
    assert _pairs(o, recs, only_events=True)[-1] == ("process", "ELEMENT_COMPLETED")
