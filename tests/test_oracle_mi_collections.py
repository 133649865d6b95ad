"""Multi-instance activities as the reference writes them, on the CPU oracle: the inputCollection a list
variable (`= items`), an outputCollection collecting an outputElement, and a completionCondition --
MultiInstanceBodyProcessor.java:83-394 and MultiInstanceOutputCollectionBehavior.java:43-141.

Pinned by the assertions of MultiInstanceActivityTest (engine/src/test/java/io/camunda/zeebe/engine/
processing/bpmn/multiinstance/MultiInstanceActivityTest.java), both parameterisations, through the restated
processing loop over the oracle engine (tests/psm.py).  Its process (:98-108, INPUT_VARIABLE_BUILDER
:71-77): start -> service task `task` (inputCollection `= items`, inputElement `item`, outputElement
`= result`, outputCollection `results`) -> end; completeJobs (:1579-1613) activates one job at a time and
completes it with `result` = 11, 22, 33.  Documents hold one entry here (the oracle refuses multi-entry
documents: their agrona iteration order is unpinned), so the reference's `x` of the `= x` conditions
comes from a preceding task's completion, and the other conditions read `item` and the numberOf*
variables."""
import pytest

from psm import Client, Log, OracleEngine, StreamProcessor
from zeebe_amd import abi, bpmn

KEY = 2251799813685249
ITEMS = (10, 20, 30)
RESULTS = (11, 22, 33)
MODES = [("parallel", False), ("sequential", True)]


def process(seq, before=False, **extra):
    loop = dict(outputCollection="results", outputElement="= result")
    loop.update(extra)
    b = bpmn.createExecutableProcess("process").startEvent("start")
    if before:
        b.serviceTask("setup", "setup")
    b.serviceTask("task", "task").multiInstance("= items", "item", seq, **loop)
    return b.endEvent("end").done()


class Run:
    def __init__(self, xml, limit=100):
        self.log = Log()
        self.eng = OracleEngine(max_commands_in_batch=limit)
        self.eng.deploy(xml, KEY, 1)
        self.sp = StreamProcessor(self.log, [self.eng], limit)

    def write(self, *recs):
        start = len(self.log.entries)
        Client(self.log).write(*recs)
        self.sp.run()
        return self.log.entries[start:]

    def complete_jobs(self, count, results=RESULTS, job_type="task"):
        """completeJobs: one job activated at a time, completed with `result`."""
        for i in range(count):
            batch = self.write(Client.activate_jobs(job_type, max_jobs=1))[-1]
            assert len(batch.value["jobKeys"]) == 1, "job %d" % i
            self.write(Client.complete_job(batch.value["jobKeys"][0], (("result", results[i]),)))

    def pi(self, element_id=None):
        return [(r.value["bpmnElementType"], abi.PI_INTENTS[r.intent]) for r in self.log.entries
                if r.value_type == abi.VT_PROCESS_INSTANCE and r.record_type != abi.RT_REJECTION
                and (element_id is None or r.value["elementId"] == element_id)]

    def variables(self, name, intent=None, scope=None):
        return [r for r in self.log.entries if r.value_type == abi.VT_VARIABLE and r.value["name"] == name
                and (intent is None or r.intent == intent) and (scope is None or r.value["scopeKey"] == scope)]

    def key_of(self, element_type, intent=abi.PI_ELEMENT_COMPLETED):
        return next(r.key for r in self.log.entries if r.value_type == abi.VT_PROCESS_INSTANCE
                    and r.intent == intent and r.value["bpmnElementType"] == element_type)


def subsequence(seq, sub):
    it = iter(seq)
    return all(any(x == y for x in it) for y in sub)


def create(run, items=ITEMS):
    return run.write(Client.create("process", (("items", items),)))


@pytest.mark.parametrize("mode,seq", MODES)
def test_activities_and_jobs_for_each_element(mode, seq):
    # shouldActivateActivitiesForEachElement (:185-212), shouldCreateOneJobForEachElement (:214-238),
    # shouldCompleteBodyWhenAllJobsAreCompleted (:240-269), shouldSetInputElementVariable (:491-523)
    r = Run(process(seq))
    create(r)
    r.complete_jobs(3)
    jobs = [e for e in r.log.entries if e.value_type == abi.VT_JOB and e.intent == abi.JOB_CREATED]
    assert len(jobs) == 3
    batches = [e for e in r.log.entries if e.value_type == abi.VT_JOB_BATCH and e.intent == 1]
    assert [dict(b.value["jobs"][0]["variables"])["item"] for b in batches] == list(ITEMS)
    t = r.pi("task")
    assert t[-3:] == [("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETING"), ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED"),
                      ("SERVICE_TASK", "SEQUENCE_FLOW_TAKEN")] or \
        ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED") in t
    assert [v.value["value"] for v in r.variables("item", abi.VAR_CREATED)] == list(ITEMS)
    assert r.pi()[-1] == ("PROCESS", "ELEMENT_COMPLETED")


@pytest.mark.parametrize("mode,seq", MODES)
def test_output_collection(mode, seq):
    # shouldSetOutputCollectionVariable (:809-832), shouldCollectOutputInVariable (:834-864),
    # shouldSetOutputElementVariable (:866-896)
    r = Run(process(seq))
    create(r)
    r.complete_jobs(3)
    pik = r.key_of("PROCESS")
    body = r.key_of("MULTI_INSTANCE_BODY")
    assert [v.value["value"] for v in r.variables("results", scope=pik)] == [RESULTS]
    assert [v.value["value"] for v in r.variables("results", scope=body)] == [
        (None, None, None), (11, None, None), (11, 22, None), (11, 22, 33)]
    assert [v.value["value"] for v in r.variables("result", abi.VAR_CREATED)] == [None, None, None]
    assert [v.value["value"] for v in r.variables("result", abi.VAR_UPDATED)] == list(RESULTS)
    # the element variables are local to the inner instances: none reaches the process scope
    assert not r.variables("item", scope=pik) and not r.variables("result", scope=pik)


@pytest.mark.parametrize("mode,seq", MODES)
@pytest.mark.parametrize("elem,want", [("= item", ITEMS), ("= loopCounter", (1, 2, 3))])
def test_output_element_is_the_input_element_or_the_loop_counter(mode, seq, elem, want):
    # shouldNotInitializeOutputElementVariableIfSameNameAsInputElement (:898-944),
    # shouldNotInitializeOutputElementVariableIfSetToLoopCounter (:946-985): no nil-initialised variable,
    # the collection collects the unchanged values (the jobs' `result` goes to the process scope)
    r = Run(process(seq, outputElement=elem))
    create(r)
    r.complete_jobs(3)
    name = elem[2:]
    assert not [v for v in r.variables(name, abi.VAR_CREATED) if v.value["value"] is None]
    assert r.variables("results", abi.VAR_UPDATED)[-1].value["value"] == want
    assert [v.value["value"] for v in r.variables("results", scope=r.key_of("PROCESS"))] == [want]


@pytest.mark.parametrize("mode,seq", MODES)
def test_empty_collection(mode, seq):
    # shouldSkipIfCollectionIsEmpty (:622-656), shouldSetEmptyOutputCollectionIfSkip (:987-1012)
    r = Run(process(seq))
    create(r, ())
    t = r.pi("task")
    assert ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED") in t and ("SERVICE_TASK", "ELEMENT_ACTIVATED") not in t
    assert [v.value["value"] for v in r.variables("results", scope=r.key_of("PROCESS"))] == [()]
    assert r.pi()[-1] == ("PROCESS", "ELEMENT_COMPLETED")


@pytest.mark.parametrize("mode,seq", MODES)
def test_completion_condition_on_the_input_element(mode, seq):
    # shouldCompleteBodyWhenCompleteConditionAccessInputDataItemEvaluateTrue (:366-422): two jobs
    # completed, then the body completes; the parallel form terminates the third inner instance
    r = Run(process(seq, completionCondition="= item = 20"))
    create(r)
    r.complete_jobs(2)
    t = r.pi("task")
    assert subsequence(t, [("SERVICE_TASK", "ELEMENT_COMPLETED"), ("SERVICE_TASK", "ELEMENT_COMPLETED"),
                           ("MULTI_INSTANCE_BODY", "COMPLETE_ELEMENT"), ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETING"),
                           ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED")])
    if not seq:
        assert t.count(("SERVICE_TASK", "ELEMENT_TERMINATED")) == 1
        batch = [e for e in r.log.entries if e.value_type == abi.VT_PROCESS_INSTANCE_BATCH]
        assert [(e.intent, e.value["index"]) for e in batch][-1] == (abi.PIB_TERMINATE, -1)
        canceled = [e for e in r.log.entries if e.value_type == abi.VT_JOB and e.intent == abi.JOB_CANCELED]
        assert len(canceled) == 1
    else:
        assert t.count(("SERVICE_TASK", "ELEMENT_ACTIVATED")) == 2
    assert r.variables("results", scope=r.key_of("PROCESS"))[0].value["value"] == (11, 22, None)
    assert r.pi()[-1] == ("PROCESS", "ELEMENT_COMPLETED")
    # the body's counters in the state rows (childTerminatedCount of the parallel form)
    assert not [row for row in r.eng.state() if row.startswith("ELEMENT_INSTANCE_KEY")]


@pytest.mark.parametrize("mode,seq", MODES)
@pytest.mark.parametrize("x,completed", [(True, 1), (False, 3)])
def test_completion_condition_on_a_variable(mode, seq, x, completed):
    # shouldCompleteBodyWhenCompleteConditionEvaluateTrue (:271-326) / ...EvaluateFalse (:424-457): `= x`;
    # x comes from the completion of a task before the multi-instance activity
    r = Run(process(seq, before=True, completionCondition="= x"))
    create(r)
    batch = r.write(Client.activate_jobs("setup", max_jobs=1))[-1]
    r.write(Client.complete_job(batch.value["jobKeys"][0], (("x", x),)))
    r.complete_jobs(completed)
    t = r.pi("task")
    assert subsequence(t, [("SERVICE_TASK", "ELEMENT_COMPLETED")] * completed +
                       [("MULTI_INSTANCE_BODY", "COMPLETE_ELEMENT"), ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED")])
    if x and not seq:
        assert t.count(("SERVICE_TASK", "ELEMENT_TERMINATED")) == 2
    elif x:
        assert t.count(("SERVICE_TASK", "ELEMENT_ACTIVATED")) == 1
    assert r.pi()[-1] == ("PROCESS", "ELEMENT_COMPLETED")


@pytest.mark.parametrize("mode,seq", MODES)
def test_completion_condition_on_number_of_completed_instances(mode, seq):
    r = Run(process(seq, completionCondition="= numberOfCompletedInstances >= 2 and numberOfInstances > 0"))
    create(r)
    r.complete_jobs(2)
    t = r.pi("task")
    assert ("MULTI_INSTANCE_BODY", "ELEMENT_COMPLETED") in t
    assert t.count(("SERVICE_TASK", "ELEMENT_TERMINATED")) == (0 if seq else 1)
    assert r.pi()[-1] == ("PROCESS", "ELEMENT_COMPLETED")


def test_state_rows_of_list_variables_round_trip():
    # a list variable and a body's output collection in the state rows, back through import
    r = Run(process(False))
    create(r)
    r.complete_jobs(1)
    rows = [row for row in r.eng.state() if not row.startswith("KEY|")]
    lists = [row for row in rows if row.startswith("VARIABLES|") and "type=6" in row]
    assert len(lists) == 2  # items (process scope) and results (the body)
    fresh = OracleEngine()
    fresh.deploy(process(False), KEY, 1)
    fresh.upsert(rows)
    assert [row for row in fresh.state() if not row.startswith("KEY|")] == rows
