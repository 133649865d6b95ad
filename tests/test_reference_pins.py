"""Pins the CPU oracle (and, under -m gpu, the gfx950 path against it) with the remaining
known-answer tests of SURVEY §8c:

* NumberOfTakenSequenceFlowsStateTest.java:45-188 -- the join-counter algebra, observed through
  the engine as NUMBER_OF_TAKEN_SEQUENCE_FLOWS rows [flowScopeKey | gatewayId | flowId -> n]
  (ProcessInstanceSequenceFlowTakenApplier.java:54-60 increments,
  ProcessInstanceElementActivatingApplier.java:80-98 decrements one per incoming flow);
* FeelExpressionTest.java:79-109,190-230 -- comparison / conjunction / disjunction / null checks
  on msgpack inputs, observed as the exclusive gateway's routing (ExclusiveGatewayProcessor
  .findSequenceFlowToTake, :86-126); expressions outside the int64/decimal/bool/null subset
  (path expressions, `is defined`) are refused at deploy and left to the CPU engine;
* StreamProcessorTest.java:314-384 -- every follow-up record of a processing batch, including the
  records of follow-up commands processed in the same batch, carries the initial command's
  position as its source position (ProcessingStateMachine.java:328-417).
"""
import struct

import pytest

from helpers import complete_commands, create_commands
from oracle.oracle import Oracle, OracleError
from zeebe_amd import abi, bpmn

BASE = 1 << 51


def _run(o, cmds, docs=None):
    o.clear_records()
    o.submit(cmds, docs)
    o.run()
    return o.records()


def _taken_rows(o):
    return sorted(r for r in o.state() if r.startswith("NUMBER_OF_TAKEN_SEQUENCE_FLOWS|"))


def _job_keys(recs):
    return [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]


def _pairs(o, recs):
    return [(o.element_id(int(r["process_idx"]), int(r["element_idx"])), abi.intent_name(5, int(r["intent"])))
            for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["record_type"] == abi.RT_EVENT]


# ---- NumberOfTakenSequenceFlowsStateTest ------------------------------------------------------
def repeated_flow_join():
    # ParallelGatewayTest.shouldOnlyTriggerGatewayWhenAllBranchesAreActivated's model: joinFlow1
    # is taken twice (both fork branches pass the exclusive merge) before joinFlow2 once
    return (bpmn.createExecutableProcess("process").startEvent().parallelGateway("fork")
            .exclusiveGateway("exclusiveJoin").moveToLastGateway().connectTo("exclusiveJoin")
            .sequenceFlowId("joinFlow1").parallelGateway("join").moveToNode("fork")
            .serviceTask("waitState", "type").sequenceFlowId("joinFlow2").connectTo("join").endEvent().done())


def two_branch_join():
    return (bpmn.createExecutableProcess("process").startEvent().parallelGateway("fork")
            .serviceTask("ta", "type").sequenceFlowId("fa").parallelGateway("join").moveToNode("fork")
            .sequenceFlowId("fb").connectTo("join").moveToNode("join").endEvent("end").done())


def test_taken_flows_counted_per_flow_and_kept_after_decrement():
    o = Oracle()
    recs = _run(o, create_commands(1, o.deploy(repeated_flow_join())))
    pi = BASE + 1
    # shouldReturnNumberPerTakenSequenceFlows: joinFlow1 twice -> one row with n = 2;
    # shouldReturnZeroIfNoSequenceFlowIsTaken: no row for joinFlow2 yet
    assert _taken_rows(o) == ["NUMBER_OF_TAKEN_SEQUENCE_FLOWS|%d|join|joinFlow1|2" % pi]
    assert ("join", "ELEMENT_ACTIVATING") not in _pairs(o, recs)
    recs = _run(o, complete_commands([0], [_job_keys(recs)[0] - BASE - 1]))
    assert _pairs(o, recs).count(("join", "ELEMENT_ACTIVATED")) == 1
    # shouldDecrementNumbersButKeepRemaining: one per incoming flow, the repeat stays
    assert _taken_rows(o) == ["NUMBER_OF_TAKEN_SEQUENCE_FLOWS|%d|join|joinFlow1|1" % pi]
    # the remaining taken flow keeps the scope alive (activeSequenceFlows 3 - 2 incoming = 1)
    assert ("process", "ELEMENT_COMPLETED") not in _pairs(o, recs)


def test_taken_flows_are_per_scope_and_removed_when_decremented_to_zero():
    o = Oracle()
    recs = _run(o, create_commands(2, o.deploy(two_branch_join())))
    pis = sorted(int(r["key"]) for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE
                 and r["intent"] == 3 and r["element_idx"] == 0)
    assert len(pis) == 2
    # shouldIncrementNumber: one row per flow scope, the other scope's counter is separate
    assert _taken_rows(o) == ["NUMBER_OF_TAKEN_SEQUENCE_FLOWS|%d|join|fb|1" % k for k in pis]
    km0 = {o.resolve(0, n): n for n in range(32)}
    job0 = [j for j in _job_keys(recs) if j in km0]
    assert len(job0) == 1
    recs = _run(o, complete_commands([0], [km0[job0[0]]]))
    assert ("process", "ELEMENT_COMPLETED") in _pairs(o, recs)
    # shouldRemoveNumbersWhenDecrementing / shouldDecrementNumbers: instance 0's rows are gone,
    # instance 1's counter is untouched
    assert _taken_rows(o) == ["NUMBER_OF_TAKEN_SEQUENCE_FLOWS|%d|join|fb|1" % pis[1]]


# ---- FeelExpressionTest ------------------------------------------------------------------------
def feel_gateway(expr):
    return (bpmn.createExecutableProcess("process").startEvent().exclusiveGateway("xor")
            .sequenceFlowId("yes").conditionExpression(expr).endEvent("isTrue").moveToLastExclusiveGateway()
            .defaultFlow().sequenceFlowId("no").endEvent("isFalse").done())


def _docs(o, entries):
    d = abi.make_docs(len(entries))
    for i, (name, typ, value) in enumerate(entries):
        d[i]["name_id"] = o.intern(name)
        d[i]["type"] = typ
        d[i]["value"] = value
    return d


# (test name in FeelExpressionTest, expression, context, expected boolean)
FEEL_CASES = {
    "comparison": ("x < 4", [("x", abi.DOC_INT, 2)], True),
    # the reference binds y = false as a second variable; documents with more than one entry are
    # outside the subset (agrona iteration order unpinned), so y's value is written as a literal
    "conjunction": ("x and false", [("x", abi.DOC_BOOL, 1)], False),
    "disjunction": ("x or false", [("x", abi.DOC_BOOL, 1)], True),
    "nullCheckWithNonExistingVariable": ("x = null", [], True),
}


def feel_route(o, expr, entries):
    proc = o.deploy(feel_gateway(expr))
    docs = _docs(o, entries)
    cmds = create_commands(1, proc)
    cmds["doc_count"] = len(entries)
    return cmds, docs


def _taken(o, recs):
    return [e for e, i in _pairs(o, recs) if i == "SEQUENCE_FLOW_TAKEN" and e in ("yes", "no")]


@pytest.mark.parametrize("case", sorted(FEEL_CASES))
def test_feel_expression_routing(case):
    expr, entries, want = FEEL_CASES[case]
    o = Oracle()
    cmds, docs = feel_route(o, expr, entries)
    assert _taken(o, _run(o, cmds, docs)) == (["yes"] if want else ["no"])


@pytest.mark.parametrize("expr", ["x.y = null", "is defined(x)", "is defined(x.y)", "upper case(x) = \"FOO\""])
def test_feel_outside_subset_is_refused_at_deploy(expr):
    # nullCheckWithNestedNonExistingVariable / checkIfDefined* / builtinFunctionInvocation: path
    # expressions and built-in functions are outside the compiled subset; deployment refuses them,
    # so such processes stay on the CPU engine (ZBHIP_EPARSE from zbhip_deploy)
    with pytest.raises(OracleError):
        Oracle().deploy(feel_gateway(expr))


# ---- StreamProcessorTest.shouldProcessFollowUpEventsAndCommands ------------------------------
def test_follow_up_records_carry_the_initial_command_position():
    from zeebe_amd.logwriter import LogSerializer, split_entries
    xml = bpmn.createExecutableProcess("process").startEvent("start").endEvent("end").done()
    o = Oracle()
    ser = LogSerializer()
    assert o.deploy(xml) == ser.deploy(xml) == 0
    cmds = create_commands(1, 0)
    recs = _run(o, cmds)
    # the batch processes follow-up commands (ACTIVATE_ELEMENT, COMPLETE_ELEMENT) in the same call
    assert int((recs["record_type"] == abi.RT_COMMAND).sum()) >= 4
    assert set(recs["source_index"].tolist()) == {0}
    command_position = 1
    buf = ser.serialize(recs, cmds, source_positions=[command_position], first_position=2)
    entries = list(split_entries(buf))
    assert len(entries) == len(recs)
    for i, (off, framed) in enumerate(entries):
        _, _, _, pos, src, _, _, _, _ = struct.unpack_from("<HBBqqqqHH", buf, off + 12)
        assert (pos, src) == (2 + i, command_position)


# ---- the same pins on the gfx950 path (through the C ABI), records and state == oracle ---------
def _gpu_both(xml, windows, names=()):
    """windows: list of fn(part, orc) -> (cmds, docs); runs each on both, compares every record
    field and the exported state after every window."""
    from test_gpu_parity import run_both
    from zeebe_amd.engine import Partition
    part, orc = Partition(max_instances=8, max_commands=8), Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    for n in names:
        assert part.intern(n) == orc.intern(n)
    for w in windows:
        cmds, docs = w(part, orc)
        run_both(part, orc, cmds, docs)
        assert part.state() == orc.state()
    assert part.stats()["fallback"] == 0
    return part, orc


def _complete_open_jobs(part, orc):
    keys = sorted(int(r.split("|")[1]) for r in part.state() if r.startswith("JOBS|"))
    ref = [part.resolve_key(k) for k in keys[:1]]
    return complete_commands([i for i, _ in ref], [o for _, o in ref]), None


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["repeated_flow_join", "two_branch_join"])
def test_gpu_taken_flow_counters(model):
    xml = {"repeated_flow_join": repeated_flow_join, "two_branch_join": two_branch_join}[model]()
    n = 1 if model == "repeated_flow_join" else 2
    part, orc = _gpu_both(xml, [lambda p, o: (create_commands(n, 0), None), _complete_open_jobs])
    assert _taken_rows(orc)  # a counter is left in both cases (see the CPU tests above)


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(FEEL_CASES))
def test_gpu_feel_expression_routing(case):
    expr, entries, want = FEEL_CASES[case]

    def window(part, orc):
        cmds = create_commands(1, 0)
        cmds["doc_count"] = len(entries)
        return cmds, _docs(orc, entries)

    part, orc = _gpu_both(feel_gateway(expr), [window], names=[e[0] for e in entries])
    assert _taken(orc, orc.records()) == (["yes"] if want else ["no"])
