"""Multi-instance activities on the CPU oracle, pinned by the assertions of the
reference's MultiInstanceActivityTest (engine/src/test/java/io/camunda/zeebe/engine/processing/bpmn/
multiinstance/MultiInstanceActivityTest.java), both parameterisations (parallel, sequential).

The reference test's process reads its inputCollection from a variable (`items`) and collects an
output collection: tests/test_oracle_mi_collections.py pins that form; the tests below drive the static
list literal (`= [10, 20, 30]`: the same items) through the lifecycle, job, loop-variable and skip
assertions.  completeJobs (:1579-1613) activates one job at a time
(JOB_BATCH:ACTIVATE, maxJobsToActivate 1) and completes it with a `result` variable."""
import numpy as np
import pytest

from helpers import complete_commands, create_commands
from oracle.oracle import Oracle, OracleError
from zeebe_amd import abi, bpmn

BASE = 1 << 51
PI = abi.PI_INTENTS
ITEMS = (10, 20, 30)
MODES = [("parallel", False), ("sequential", True)]


def _run(o, cmds, docs=None):
    o.clear_records()
    o.submit(cmds, docs)
    o.run()
    return o.records()


def _types(o, recs, elem_id=None):
    out = []
    for r in recs:
        if r["value_type"] != abi.VT_PROCESS_INSTANCE or r["record_type"] == abi.RT_REJECTION:
            continue
        if elem_id is not None and o.element_id(0, int(r["element_idx"])) != elem_id:
            continue
        out.append((abi.ELEMENT_TYPES[o.element_type(0, int(r["element_idx"]))], PI[int(r["intent"])]))
    return out


def _subsequence(seq, sub):
    it = iter(seq)
    return all(any(x == y for x in it) for y in sub)


def drive(xml, job_type="task", results=(11, 22, 33), limit=100):
    """Create one instance, then completeJobs: activate one job, complete it with result=results[i]."""
    o = Oracle(max_commands_in_batch=limit)
    proc = o.deploy(xml)
    res = o.intern("result")
    recs = list(_run(o, create_commands(1, proc)))
    activated = []
    for i in range(len(results)):
        _, jobs, reason = o.activate_jobs(job_type, max_jobs=1)
        assert reason == 0 and len(jobs) == 1, "job %d" % i
        activated.append(jobs[0])
        ordinal = o.ordinal_of(0, int(jobs[0]["key"]))
        d = abi.make_docs(1)
        d["name_id"], d["type"], d["value"] = res, abi.DOC_INT, results[i]
        c = complete_commands([0], [ordinal])
        c["doc_count"] = 1
        recs += list(_run(o, c, d))
    return o, recs, activated


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_activate_activities_with_loop_characteristics(mode, seq):
    # shouldActivateActivitiesWithLoopCharacteristics (:160-183) with parallelLifecycle /
    # sequentialLifecycle (:124-157)
    o, recs, _ = drive(bpmn.multi_instance_process(ITEMS, sequential=seq))
    st = ("SERVICE_TASK", "ELEMENT_ACTIVATING"), ("SERVICE_TASK", "ELEMENT_ACTIVATED")
    en = ("SERVICE_TASK", "ELEMENT_COMPLETING"), ("SERVICE_TASK", "ELEMENT_COMPLETED")
    want = (list(st) * 3 + list(en) * 3) if not seq else (list(st) + list(en)) * 3
    t = _types(o, recs, "task")
    assert _subsequence(t, want)
    if not seq:  # the parallel form activates all three before any completes
        assert not _subsequence(t, list(st) + list(en) + list(st))


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_activate_activities_for_each_element(mode, seq):
    # shouldActivateActivitiesForEachElement (:185-212)
    o, recs, _ = drive(bpmn.multi_instance_process(ITEMS, sequential=seq))
    assert _subsequence(_types(o, recs, "task"), [
        ("MULTI_INSTANCE_BODY", "ELEMENT_ACTIVATING"), ("MULTI_INSTANCE_BODY", "ELEMENT_ACTIVATED"),
        ("SERVICE_TASK", "ELEMENT_ACTIVATED"), ("SERVICE_TASK", "ELEMENT_ACTIVATED")])


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_create_one_job_for_each_element(mode, seq):
    # shouldCreateOneJobForEachElement (:214-238)
    o, recs, _ = drive(bpmn.multi_instance_process(ITEMS, sequential=seq))
    created = [r for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    assert len(created) == 3 and {o.element_id(0, int(r["element_idx"])) for r in created} == {"task"}


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_complete_body_when_all_jobs_are_completed(mode, seq):
    # shouldCompleteBodyWhenAllJobsAreCompleted (:240-269)
    o, recs, _ = drive(bpmn.multi_instance_process(ITEMS, sequential=seq))
    assert _subsequence(_types(o, recs, "task"), [("SERVICE_TASK", "ELEMENT_COMPLETED")] * 3 + [
        ("MULTI_INSTANCE_BODY", "COMPLETE_ELEMENT"), ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETING"),
        ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED")])


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_go_through_multi_instance_activity(mode, seq):
    # shouldGoThroughMultiInstanceActivity (:458-489)
    o, recs, _ = drive(bpmn.multi_instance_process(ITEMS, sequential=seq))
    assert _subsequence(_types(o, recs), [
        ("START_EVENT", "ELEMENT_COMPLETED"), ("SEQUENCE_FLOW", "SEQUENCE_FLOW_TAKEN"),
        ("MULTI_INSTANCE_BODY", "ELEMENT_ACTIVATING"), ("MULTI_INSTANCE_BODY", "ELEMENT_ACTIVATED"),
        ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETING"), ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED"),
        ("SEQUENCE_FLOW", "SEQUENCE_FLOW_TAKEN"), ("END_EVENT", "ELEMENT_COMPLETED"),
        ("PROCESS", "ELEMENT_COMPLETED")])
    assert o.state() == ["KEY|latestKey|%d" % (BASE + o.key_counter())]


def _var_records(o, recs, name):
    nid = o.intern(name)
    return [r for r in recs if r["value_type"] == abi.VT_VARIABLE and int(r["element_idx"]) == nid]


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_set_input_element_variable(mode, seq):
    # shouldSetInputElementVariable (:491-523): the activated jobs carry `item`, and the item
    # VARIABLE:CREATED records carry the collection's values, in order
    o, recs, jobs = drive(bpmn.multi_instance_process(ITEMS, sequential=seq))
    item = o.intern("item")
    got = []
    for j in jobs:
        vs = {int(v["name_id"]): int(v["value"]) for v in j["variables"][: int(j["n_variables"])]}
        got.append(vs[item])
    assert got == list(ITEMS)
    created = [r for r in _var_records(o, recs, "item") if r["intent"] == 0]
    assert [int(r["message_key"]) for r in created] == list(ITEMS)
    assert all(int(r["aux"]) == abi.AUX_INLINE and int(r["partition"]) == abi.DOC_INT for r in created)


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_not_propagate_input_element_variable(mode, seq):
    # shouldNotPropagateInputElementVariable (:525-548): no `item` record at the process scope
    o, recs, _ = drive(bpmn.multi_instance_process(ITEMS, sequential=seq))
    pik = BASE + 1
    assert all(int(r["scope_key"]) != pik for r in _var_records(o, recs, "item"))
    # the job's `result` goes to the process scope (mergeDocument through the body, no local match)
    res = _var_records(o, recs, "result")
    assert [int(r["scope_key"]) for r in res] == [pik] * 3 and [int(r["intent"]) for r in res] == [0, 1, 1]


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_skip_if_collection_is_empty(mode, seq):
    # shouldSkipIfCollectionIsEmpty (:622-655): exactly these six records of the element
    o = Oracle()
    o.deploy(bpmn.multi_instance_process((), sequential=seq))
    recs = _run(o, create_commands(1, 0))
    assert _types(o, recs, "task") == [
        ("MULTI_INSTANCE_BODY", "ACTIVATE_ELEMENT"), ("MULTI_INSTANCE_BODY", "ELEMENT_ACTIVATING"),
        ("MULTI_INSTANCE_BODY", "ELEMENT_ACTIVATED"), ("MULTI_INSTANCE_BODY", "COMPLETE_ELEMENT"),
        ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETING"), ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED")]
    assert ("PROCESS", "ELEMENT_COMPLETED") in _types(o, recs)


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_ignore_input_element_variable_if_not_defined(mode, seq):
    # shouldIgnoreInputElementVariableIfNotDefined (:657-688)
    o, recs, jobs = drive(bpmn.multi_instance_process(ITEMS, sequential=seq, input_element=None))
    item = o.intern("item")
    assert all(item not in [int(v["name_id"]) for v in j["variables"][: int(j["n_variables"])]] for j in jobs)
    assert not _var_records(o, recs, "item")


@pytest.mark.parametrize("mode,seq", MODES)
def test_should_set_loop_counter_variable(mode, seq):
    # shouldSetLoopCounterVariable (:1075-1111): loopCounter 1, 2, 3 local to the inner instances in
    # their activation order
    o, recs, _ = drive(bpmn.multi_instance_process(ITEMS, sequential=seq))
    inner = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and
             r["intent"] == abi.PI_INTENT_IDS["ELEMENT_ACTIVATED"] and
             o.element_type(0, int(r["element_idx"])) == abi.ELEMENT_TYPES.index("SERVICE_TASK")]
    lc = _var_records(o, recs, "loopCounter")
    assert [(int(r["scope_key"]), int(r["message_key"])) for r in lc] == list(zip(inner[:3], (1, 2, 3)))


def test_parallel_batch_command_and_counters():
    # the parallel body writes PROCESS_INSTANCE_BATCH:ACTIVATE (activateChildInstancesInBatches,
    # BpmnStateTransitionBehavior.java:315-324): key = the next key, batchElementInstanceKey = the
    # body, index = the collection size; its processing writes one ACTIVATE_ELEMENT per item, each
    # with a new key (ActivateProcessInstanceBatchProcessor.java:44-60).  The body's ElementInstance
    # counts its children (ProcessInstanceElementActivatingApplier.manageMultiInstance :237-253,
    # ProcessInstanceElementCompletedApplier.manageMultiInstance :104-110).
    o = Oracle()
    o.deploy(bpmn.multi_instance_process(ITEMS))
    recs = _run(o, create_commands(1, 0))
    pib = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE_BATCH]
    assert len(pib) == 1 and pib[0]["record_type"] == abi.RT_COMMAND and pib[0]["intent"] == abi.PIB_ACTIVATE
    body_key = int([r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and
                    r["intent"] == abi.PI_INTENT_IDS["ELEMENT_ACTIVATED"] and
                    o.element_type(0, int(r["element_idx"])) == abi.ELEMENT_TYPES.index("MULTI_INSTANCE_BODY")][0]["key"])
    assert int(pib[0]["scope_key"]) == body_key and int(pib[0]["partition"]) == 3
    i = list(recs).index(pib[0])
    acts = [r for r in recs[i + 1:] if r["record_type"] == abi.RT_COMMAND and r["value_type"] == abi.VT_PROCESS_INSTANCE]
    assert [int(r["key"]) for r in acts[:3]] == [int(pib[0]["key"]) + 1 + k for k in range(3)]
    assert all(int(r["scope_key"]) == body_key for r in acts[:3])
    body = [r for r in o.state() if r.startswith("ELEMENT_INSTANCE_KEY|%d|" % body_key)][0]
    assert "childCount=3,childActivatedCount=3,childCompletedCount=0" in body and "multiInstanceLoopCounter=3" in body
    inner = sorted(r for r in o.state() if r.startswith("ELEMENT_INSTANCE_KEY|") and "bpmnElementType=9," in r)
    assert ["multiInstanceLoopCounter=%d" % (k + 1) in r for k, r in enumerate(inner)] == [True] * 3


def test_strings_and_limits():
    # string items into the value dictionary (interned at deploy, in item order); a batch limit of 3
    # pushes the parallel activations past the limit (written unprocessed, their own batches later)
    o, recs, jobs = drive(bpmn.multi_instance_process(("a", "bb", "c"), job_type="s"), job_type="s", limit=3)
    item = o.intern("item")
    vals = [o.string_value(int({int(v["name_id"]): v["value"] for v in j["variables"][: int(j["n_variables"])]}[item]))
            for j in jobs]
    assert vals == [b"a", b"bb", b"c"]
    assert any(r["unprocessed"] for r in recs)


@pytest.mark.parametrize("bad", [
    '= items.nested', '= [1.5]', '= [x]', '= [1] + [2]', '= [1, 2', '= ["a\\\\b"]'])
def test_refused_input_collections(bad):
    o = Oracle()
    with pytest.raises(OracleError, match="inputCollection"):
        o.deploy(bpmn.multi_instance_process(bad))


@pytest.mark.parametrize("extra,match", [
    (dict(outputCollection="results"), "outputCollection"),                           # no outputElement
    (dict(outputCollection="results", outputElement="= result.nested"), "outputCollection"),  # a path
    (dict(completionCondition="x"), "completionCondition"),                          # static text
    (dict(completionCondition="= count(items) > 1"), "completionCondition")])        # a function call
def test_refused_output_collection_and_condition(extra, match):
    # (outputCollection / outputElement / completionCondition themselves: test_oracle_mi_collections.py)
    b = bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "t")
    b.multiInstance("= [1]", "item", **extra)
    with pytest.raises(OracleError, match=match):
        Oracle().deploy(b.endEvent().done())


@pytest.mark.parametrize("seq", [False, True])
def test_undefined_task_inner(seq):
    # an inner activity without a wait state completes in its activation's batch
    o = Oracle()
    o.deploy(bpmn.multi_instance_process(ITEMS, sequential=seq, inner="task"))
    recs = _run(o, create_commands(1, 0))
    t = _types(o, recs, "task")
    assert t.count(("TASK", "ELEMENT_COMPLETED")) == 3 and t[-1] == ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED")
    assert o.state() == ["KEY|latestKey|%d" % (BASE + o.key_counter())]


def test_zb_db_round_trip():
    # the state rows of waiting multi-instance bodies / inner instances (counters, loop variables
    # with an interned string item) through the product's zb-db encoder and decoder (host code)
    from zeebe_amd.logwriter import LogSerializer
    xml = bpmn.multi_instance_process((10, "twenty", 30), after="after")
    o = Oracle()
    o.deploy(xml)
    _run(o, create_commands(2))
    rows = sorted(r for r in o.state() if not r.startswith("KEY|"))
    assert any("bpmnElementType=19," in r and "childActivatedCount=3" in r for r in rows)
    s = LogSerializer()
    s.deploy(xml)
    for n in o.names():
        s.intern(n)
    for v in o.strings():
        s.intern_string(v)
    back = s.decode_state_entries(s.encode_state_rows(rows), intern=lambda b: s.intern_string(b))
    assert back == rows
    # and the product encoder's bytes are oracle/statedb.py's
    from oracle import statedb as SD
    strings = o.strings()
    assert s.encode_state_rows(rows) == SD.encode_rows(rows, o.process_tables(), lambda i: strings[i])
