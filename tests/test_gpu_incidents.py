"""Incidents of exclusive gateways on the gfx950 path (BpmnIncidentBehavior.createIncident, :51-71):
records, log bytes (the incident messages of ExclusiveGatewayProcessor.java:121-125 and
ExpressionProcessor.java:356-368) and zb-db bytes of the state (INCIDENTS,
INCIDENT_PROCESS_INSTANCES, the gateway's ELEMENT_ACTIVATING instance) equal to the CPU oracle,
which tests/test_oracle_incidents.py pins on ConditionIncidentTest / ExclusiveGatewayTest.  The
instance stays on the device with its gateway waiting; later windows of the same instances
(parallel branches, job completions) run on the device too."""
import numpy as np
import pytest

from helpers import complete_commands, create_commands
from oracle import statedb as SD
from test_gpu_logserial import Pair
from test_oracle_incidents import condition_process, missing_variable_process
from zeebe_amd import abi, bpmn

pytestmark = pytest.mark.gpu


def _docs(pair, rng, n, name="foo"):
    """one `foo` per instance: ints 0..15 (s1 < 5, s2 > 10, else no flow), decimals, strings, nil,
    booleans, or none at all (a missing variable)"""
    nid = pair.part.intern(name)
    assert nid == pair.orc.intern(name)
    sid = pair.part.intern_string("bar")
    assert sid == pair.orc.intern_string("bar")
    kinds = rng.integers(0, 6, n)
    cmds = create_commands(n, 0)
    docs = abi.make_docs(n)
    m = 0
    for i in range(n):
        k = kinds[i]
        if k == 5:
            continue  # no document: `foo` missing -> NULL
        d = docs[m]
        d["name_id"] = nid
        if k <= 1:
            d["type"], d["value"] = abi.DOC_INT, rng.integers(0, 16)
        elif k == 2:
            d["type"], d["value"] = abi.DOC_DEC, rng.integers(0, 16_000_000)
        elif k == 3:
            d["type"], d["value"] = abi.DOC_STR, sid
        else:
            d["type"], d["value"] = abi.DOC_NIL, 0
        cmds[i]["doc_count"] = 1
        cmds[i]["doc_begin"] = m
        m += 1
    return cmds, docs[:m]


def _incidents(recs):
    return recs[recs["value_type"] == abi.VT_INCIDENT]


@pytest.mark.parametrize("seed", [1, 2])
def test_condition_incidents_match_oracle(seed):
    rng = np.random.default_rng(seed)
    pair = Pair(condition_process(), 400)
    cmds, docs = _docs(pair, rng, 400)
    recs = pair.window(cmds, docs)
    inc = _incidents(recs)
    assert len(inc) > 100
    errs = set(inc["partition"].tolist())
    assert errs == {abi.ERR_CONDITION_ERROR, abi.ERR_EXTRACT_VALUE_ERROR}
    # the messages through the C ABI equal the ones the oracle's serialiser writes
    msgs = {pair.part.incident_message(r) for r in inc}
    assert "Expected at least one condition to evaluate to true, or to have a default flow" in msgs
    assert "Expected result of the expression 'foo > 10' to be 'BOOLEAN', but was 'NULL'." in msgs
    assert pair.part.stats()["fallback"] == 0


def test_missing_variable_incident_and_default_flow():
    pair = Pair(missing_variable_process(), 64)
    cmds = create_commands(64, 0)
    recs = pair.window(cmds)
    assert len(_incidents(recs)) == 64


def parallel_branch_process():
    # fork -> [exclusive gateway on `foo` -> end] + [service task -> end]: a branch with an incident
    # keeps the process instance active after the other branch completes
    return (bpmn.createExecutableProcess("process").startEvent().parallelGateway("fork")
            .exclusiveGateway("xor").sequenceFlowId("s1").conditionExpression("foo < 5").endEvent("e1")
            .moveToLastExclusiveGateway().sequenceFlowId("s2").conditionExpression("foo > 10").endEvent("e2")
            .moveToNode("fork").serviceTask("task", "work").endEvent("e3").done())


def test_incident_on_one_branch_keeps_the_instance_active():
    rng = np.random.default_rng(7)
    pair = Pair(parallel_branch_process(), 200)
    cmds, docs = _docs(pair, rng, 200)
    recs = pair.window(cmds, docs)
    assert len(_incidents(recs)) > 0
    jobs = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    res = [pair.part.resolve_key(k) for k in jobs]
    recs = pair.window(complete_commands([r[0] for r in res], [r[1] for r in res]))
    done = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == abi.PI_INTENT_IDS[
        "ELEMENT_COMPLETED"] and r["element_idx"] == 0]
    assert 0 < len(done) < 200  # instances with an incident stay active
    assert pair.part.stats()["fallback"] == 0


def test_incident_inside_a_sub_process():
    xml = (bpmn.createExecutableProcess("process").startEvent().subProcess("sub").startEvent()
           .exclusiveGateway("xor").sequenceFlowId("s1").conditionExpression("foo < 5").endEvent()
           .moveToLastExclusiveGateway().sequenceFlowId("s2").conditionExpression("foo > 10").endEvent()
           .subProcessDone().serviceTask("after", "work").endEvent().done())
    rng = np.random.default_rng(3)
    pair = Pair(xml, 128)
    cmds, docs = _docs(pair, rng, 128)
    recs = pair.window(cmds, docs)
    assert len(_incidents(recs)) > 0
    assert pair.part.stats()["fallback"] == 0


def test_incidents_with_templates_and_batch_limit():
    # config 3's process: `= amount > 1000` with a default flow; string / nil / missing amounts are
    # NULL conditions.  The second window replays CREATE templates for the boolean outcomes and takes
    # the general path for the incidents.
    rng = np.random.default_rng(11)
    pair = Pair(bpmn.xor_process(), 600)
    for w in range(2):
        cmds, docs = _docs(pair, rng, 300, name="amount")
        cmds["instance"] += 300 * w
        recs = pair.window(cmds, docs)
        assert len(_incidents(recs)) > 0
    assert pair.part.stats()["fallback"] == 0


def test_incident_instances_hand_off_through_zb_db_bytes():
    # the fallback hand-off exports an instance with an incident: its rows are the CPU engine's and
    # its zb-db entries equal the oracle's encoding of them
    rng = np.random.default_rng(5)
    pair = Pair(condition_process(), 32)
    cmds, docs = _docs(pair, rng, 32)
    recs = pair.window(cmds, docs)
    inc = _incidents(recs)
    assert len(inc) > 0
    insts = sorted({pair.part.resolve_key(int(r["scope_key"]))[0] for r in inc})
    strings = pair.orc.strings()
    rows = pair.part.export_instances(insts[:4])
    assert any(r.startswith("INCIDENTS|") for r in rows) and set(rows) <= set(pair.orc.state())
    assert pair.part.export_instances_db(insts[:4]) == SD.encode_rows(rows, pair.orc.process_tables(),
                                                                      lambda i: strings[i])
