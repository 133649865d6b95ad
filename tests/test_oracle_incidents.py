"""Incidents of exclusive gateways on the CPU oracle (and, under -m gpu, the gfx950 path against
it), pinned on the reference's tests:

* ConditionIncidentTest.java:42-123 -- no condition true and no default flow: INCIDENT:CREATED with
  CONDITION_ERROR "Expected at least one condition to evaluate to true, or to have a default flow";
  a condition that does not evaluate to a boolean (`foo > 10` with foo = "bar" is NULL):
  EXTRACT_VALUE_ERROR "Expected result of the expression 'foo > 10' to be 'BOOLEAN', but was
  'NULL'." -- which also pins the evaluation order of the outgoing flows (s2 before s1: reverse
  document order, ModelWalker.java:75-79); bpmnProcessId / processInstanceKey / elementId of the
  gateway's ELEMENT_ACTIVATING, elementInstanceKey = variableScopeKey = its key, tenant <default>;
* ExclusiveGatewayTest.shouldResolveIncidentsWhenTerminating (:323-346): a condition naming a
  missing variable raises an incident (its result is NULL, cf. the reference's other incident
  tests: "... to be 'STRING', but was 'NULL'." for missing variables);
* BpmnIncidentBehavior.createIncident (:51-71) / IncidentCreatedApplier: the incident key is the
  next key after the gateway's, the gateway stays ELEMENT_ACTIVATING (no ACTIVATED), its rows
  INCIDENTS and INCIDENT_PROCESS_INSTANCES exist, the process instance stays active.
"""
import pytest

from helpers import create_commands
from oracle import logserial as LS
from oracle import statedb as SD
from oracle.oracle import Oracle
from zeebe_amd import abi, bpmn



def mp_decode(b, i=0):
    """(value, next offset) of the msgpack value at b[i] (maps, strings, ints, bools, nil, bin)."""
    t = b[i]
    if t <= 0x7F:
        return t, i + 1
    if t >= 0xE0:
        return t - 0x100, i + 1
    if 0x80 <= t <= 0x8F or t in (0xDE, 0xDF):
        n, i = (t & 0x0F, i + 1) if t <= 0x8F else (int.from_bytes(b[i + 1:i + 3 if t == 0xDE else i + 5], "big"),
                                                     i + (3 if t == 0xDE else 5))
        out = {}
        for _ in range(n):
            k, i = mp_decode(b, i)
            v, i = mp_decode(b, i)
            out[k] = v
        return out, i
    if 0xA0 <= t <= 0xBF or t in (0xD9, 0xDA, 0xDB):
        if t <= 0xBF:
            n, i = t & 0x1F, i + 1
        else:
            w = {0xD9: 1, 0xDA: 2, 0xDB: 4}[t]
            n, i = int.from_bytes(b[i + 1:i + 1 + w], "big"), i + 1 + w
        return bytes(b[i:i + n]).decode(), i + n
    if t in (0xC4, 0xC5, 0xC6):
        w = {0xC4: 1, 0xC5: 2, 0xC6: 4}[t]
        n = int.from_bytes(b[i + 1:i + 1 + w], "big")
        return bytes(b[i + 1 + w:i + 1 + w + n]), i + 1 + w + n
    if t in (0xC0, 0xC2, 0xC3):
        return {0xC0: None, 0xC2: False, 0xC3: True}[t], i + 1
    w = {0xCC: 1, 0xCD: 2, 0xCE: 4, 0xCF: 8, 0xD0: 1, 0xD1: 2, 0xD2: 4, 0xD3: 8}[t]
    return int.from_bytes(b[i + 1:i + 1 + w], "big", signed=t >= 0xD0), i + 1 + w


def decode_object(b):
    return mp_decode(bytes(b))[0]


def condition_process():
    # ConditionIncidentTest.PROCESS
    return (bpmn.createExecutableProcess("process").startEvent().exclusiveGateway("xor")
            .sequenceFlowId("s1").conditionExpression("foo < 5").endEvent()
            .moveToLastGateway().sequenceFlowId("s2").conditionExpression("foo > 10").endEvent().done())


def missing_variable_process():
    # ExclusiveGatewayTest.shouldResolveIncidentsWhenTerminating
    return (bpmn.createExecutableProcess("process").startEvent().exclusiveGateway("xor")
            .sequenceFlowId("s1").defaultFlow().endEvent("default-end")
            .moveToLastGateway().sequenceFlowId("s2").conditionExpression("nonexisting_variable")
            .endEvent("non-default-end").done())


def _create(o, proc, entries):
    d = abi.make_docs(len(entries))
    for i, (name, typ, value) in enumerate(entries):
        d[i]["name_id"] = o.intern(name)
        d[i]["type"] = typ
        d[i]["value"] = value
    cmds = create_commands(1, proc)
    cmds["doc_count"] = len(entries)
    return cmds, d


def _run(o, cmds, docs):
    o.clear_records()
    o.submit(cmds, docs)
    o.run()
    return o.records()


def _incident(o, recs):
    inc = recs[recs["value_type"] == abi.VT_INCIDENT]
    assert len(inc) == 1
    r = inc[0]
    assert r["record_type"] == abi.RT_EVENT and r["intent"] == abi.INCIDENT_CREATED
    gw = [x for x in recs if x["value_type"] == abi.VT_PROCESS_INSTANCE and x["record_type"] == abi.RT_EVENT
          and o.element_id(int(x["process_idx"]), int(x["element_idx"])) == "xor"]
    # the gateway stays ELEMENT_ACTIVATING
    assert [int(x["intent"]) for x in gw] == [abi.PI_ELEMENT_ACTIVATING]
    assert int(r["scope_key"]) == int(gw[0]["key"])                     # elementInstanceKey
    assert int(r["process_instance_key"]) == int(gw[0]["process_instance_key"])
    assert o.element_id(int(r["process_idx"]), int(r["element_idx"])) == "xor"
    assert int(r["key"]) == int(gw[0]["key"]) + 1                       # keyGenerator.nextKey()
    assert r is recs[-1] or int(recs[-1]["value_type"]) == abi.VT_INCIDENT
    return r, gw[0]


def _value(o, r):
    tables = LS.Tables(o.process_tables(), o.name, lambda i: b"")
    return decode_object(LS.record_value(r, tables, lambda s: [], lambda i: None))


@pytest.mark.parametrize("foo,error,message", [
    ((abi.DOC_INT, 9), "CONDITION_ERROR",
     "Expected at least one condition to evaluate to true, or to have a default flow"),
    ((abi.DOC_STR, "bar"), "EXTRACT_VALUE_ERROR",
     "Expected result of the expression 'foo > 10' to be 'BOOLEAN', but was 'NULL'."),
])
def test_condition_incident(foo, error, message):
    o = Oracle()
    proc = o.deploy(condition_process())
    typ, v = foo
    if typ == abi.DOC_STR:
        v = o.intern_string(v)
    cmds, docs = _create(o, proc, [("foo", typ, v)])
    recs = _run(o, cmds, docs)
    r, gw = _incident(o, recs)
    val = _value(o, r)
    assert val["errorType"] == error
    assert val["errorMessage"] == message
    assert val["bpmnProcessId"] == "process"
    assert val["elementId"] == "xor"
    assert val["elementInstanceKey"] == val["variableScopeKey"] == int(gw["key"])
    assert val["processInstanceKey"] == int(gw["process_instance_key"])
    assert val["jobKey"] == -1 and val["tenantId"] == "<default>"
    state = o.state()
    ik, ek = int(r["key"]), int(gw["key"])
    assert any(s.startswith("INCIDENTS|%d|" % ik) for s in state)
    assert "INCIDENT_PROCESS_INSTANCES|%d|%d" % (ek, ik) in state
    gw_row = [s for s in state if s.startswith("ELEMENT_INSTANCE_KEY|%d|" % ek)]
    assert len(gw_row) == 1 and ",state=2," in gw_row[0]
    # the process instance stays active with the gateway as its child
    pi_row = [s for s in state if s.startswith("ELEMENT_INSTANCE_KEY|%d|" % int(gw["process_instance_key"]))]
    assert len(pi_row) == 1 and ",childCount=1," in pi_row[0] and ",state=3," in pi_row[0]
    # zb-db bytes of the incident rows
    db = SD.encode_rows(state, o.process_tables(), lambda i: b"bar")
    inc = [e for e in db if e[0] == 34]
    assert len(inc) == 1
    assert decode_object(inc[0][2])["incidentRecord"]["errorMessage"] == message


def test_missing_variable_condition_raises_incident():
    o = Oracle()
    proc = o.deploy(missing_variable_process())
    cmds, docs = _create(o, proc, [("foo", abi.DOC_INT, 10)])
    recs = _run(o, cmds, docs)
    r, _ = _incident(o, recs)
    assert _value(o, r)["errorMessage"] == (
        "Expected result of the expression 'nonexisting_variable' to be 'BOOLEAN', but was 'NULL'.")


@pytest.mark.parametrize("value,taken", [((abi.DOC_INT, 3), "s1"), ((abi.DOC_INT, 11), "s2")])
def test_condition_process_routes_without_incident(value, taken):
    o = Oracle()
    proc = o.deploy(condition_process())
    cmds, docs = _create(o, proc, [("foo", value[0], value[1])])
    recs = _run(o, cmds, docs)
    assert not (recs["value_type"] == abi.VT_INCIDENT).any()
    flows = [o.element_id(int(x["process_idx"]), int(x["element_idx"])) for x in recs
             if x["value_type"] == abi.VT_PROCESS_INSTANCE and x["intent"] == abi.PI_SEQUENCE_FLOW_TAKEN]
    assert taken in flows


def test_number_result_names_its_type():
    # a condition whose result is a number: typeCheck's "... but was 'NUMBER'."
    xml = (bpmn.createExecutableProcess("process").startEvent().exclusiveGateway("xor")
           .sequenceFlowId("s1").conditionExpression("foo").endEvent().done())
    o = Oracle()
    proc = o.deploy(xml)
    cmds, docs = _create(o, proc, [("foo", abi.DOC_INT, 7)])
    r, _ = _incident(o, _run(o, cmds, docs))
    assert _value(o, r)["errorMessage"] == "Expected result of the expression 'foo' to be 'BOOLEAN', but was 'NUMBER'."
