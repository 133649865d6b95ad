"""Input / output mappings (zeebe:ioMapping) on the CPU oracle, pinned by the
reference's ActivityInputMappingTest / ActivityOutputMappingTest (engine/src/test/java/io/camunda/zeebe/
engine/processing/variable/mapping/) cases whose initial document has one variable (documents with
several entries iterate in agrona order: parity unpinned), plus the record order of
BpmnVariableMappingBehavior (behavior/BpmnVariableMappingBehavior.java:53-156) around the job and the
element lifecycle, which the product's tests compare against."""
import pytest

from helpers import complete_commands, create_commands
from oracle.oracle import Oracle, OracleError
from zeebe_amd import abi, bpmn

BASE = 1 << 51


def typed(t, v):
    return (None if t == abi.DOC_NIL else bool(v) if t == abi.DOC_BOOL else int(v) if t == abi.DOC_INT
            else int(v) / 10 ** abi.DEC_SCALE if t == abi.DOC_DEC else ("str", int(v)))


class Run:
    def __init__(self, xml):
        self.o = Oracle()
        self.o.deploy(xml)
        self.docs = abi.make_docs(0)
        self.records = []

    def window(self, cmds, docs=None):
        self.o.clear_records()
        base = len(self.docs)
        if docs is not None:
            self.docs = docs if not base else __import__("numpy").concatenate([self.docs, docs])
        self.o.submit(cmds, docs)
        self.o.run()
        recs = self.o.records()
        self.records.extend(recs)
        return recs

    def create(self, variables=()):
        c = create_commands(1)
        d = abi.make_docs(len(variables))
        for j, (n, v) in enumerate(variables):
            d[j]["name_id"] = self.o.intern(n)
            d[j]["type"], d[j]["value"] = abi.DOC_INT, v
        c["doc_count"] = len(variables)
        return self.window(c, d)

    def complete_jobs(self):
        jobs = [int(r["key"]) for r in self.records if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
        done = {int(r["key"]) for r in self.records if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_COMPLETED}
        jobs = [k for k in jobs if k not in done]
        return self.window(complete_commands([0] * len(jobs), [self.o.ordinal_of(0, k) for k in jobs]))

    def variables(self, scope=None, after=0):
        out = []
        for r in self.records[after:]:
            if r["value_type"] != abi.VT_VARIABLE or (scope is not None and int(r["scope_key"]) != scope):
                continue
            aux = int(r["aux"])
            v = typed(int(r["partition"]), int(r["message_key"])) if aux == abi.AUX_INLINE else \
                typed(int(self.docs[aux]["type"]), int(self.docs[aux]["value"]))
            out.append((abi.VAR_INTENTS[int(r["intent"])], self.o.name(int(r["element_idx"])), v))
        return out

    def key_of(self, elem_id, intent="ELEMENT_ACTIVATED"):
        for r in self.records:
            if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == abi.PI_INTENT_IDS[intent] and \
                    self.o.element_id(0, int(r["element_idx"])) == elem_id:
                return int(r["key"])
        raise KeyError(elem_id)


def sub_process(mappings, task=False):
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("sub").startEvent()
    if task:
        b.serviceTask("task", "task")
    b.endEvent().subProcessDone()
    for kind, src, tgt in mappings:
        b._mapping(kind, src, tgt)
    return b.endEvent().done()


@pytest.mark.parametrize("mapping, expected", [
    (("=x", "x"), ("x", 1)),   # ActivityInputMappingTest parameters 0
    (("=x", "y"), ("y", 1)),   # parameters 1
])
def test_activity_input_mapping(mapping, expected):
    # ActivityInputMappingTest.shouldApplyInputMappings: the sub-process's variables (scopeKey = its key)
    r = Run(sub_process([("input",) + mapping]))
    r.create([("x", 1)])
    sub = r.key_of("sub")
    assert [v[1:] for v in r.variables(scope=sub)] == [expected]


@pytest.mark.parametrize("mappings, expected", [
    ([("output", "=x", "y")], ("y", 1)),                            # ActivityOutputMappingTest parameters 0
    ([("input", "=x", "y"), ("output", "=y", "z")], ("z", 1)),      # parameters 2
    ([("input", "=x", "y"), ("output", "=x", "z")], ("z", 1)),      # parameters 3
])
def test_activity_output_mapping(mappings, expected):
    # ActivityOutputMappingTest.shouldApplyOutputMappings: variables of the process scope written after
    # the inner task completed
    r = Run(sub_process(mappings, task=True))
    recs = r.create([("x", 1)])
    pik = BASE + 1
    n = len(r.records)
    r.complete_jobs()
    done = next(i for i, x in enumerate(r.records) if x["value_type"] == abi.VT_PROCESS_INSTANCE and
                x["intent"] == abi.PI_INTENT_IDS["ELEMENT_COMPLETED"] and r.o.element_id(0, int(x["element_idx"])) == "task")
    assert [v[1:] for v in r.variables(scope=pik, after=done)] == [expected]
    # the sub-process scope's own variables went with it (no VARIABLES rows left but the process's)
    assert all(row.split("|")[1] == str(pik) for row in r.o.state() if row.startswith("VARIABLES|"))


def test_task_mapping_order_and_local_scope():
    # applyInputMappings before the job (JobWorkerTaskProcessor.onActivate :50-61): VARIABLE:CREATED in
    # the task's scope between ELEMENT_ACTIVATING and JOB:CREATED; the job's variables become local when
    # an output mapping exists (mergeLocalDocument), the mapping result goes to the flow scope
    # (mergeDocument), and the task's local variables are removed with it
    xml = (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "t")
           .zeebeInputExpression("x", "local").zeebeOutputExpression("local", "result").endEvent().done())
    r = Run(xml)
    recs = r.create([("x", 7)])
    seq = [(abi.VT_SHORT if hasattr(abi, "VT_SHORT") else int(x["value_type"]), int(x["intent"])) for x in recs]
    task = r.key_of("task")
    i_act = next(i for i, x in enumerate(recs) if x["value_type"] == abi.VT_PROCESS_INSTANCE and
                 x["intent"] == abi.PI_INTENT_IDS["ELEMENT_ACTIVATING"] and int(x["key"]) == task)
    assert recs[i_act + 1]["value_type"] == abi.VT_VARIABLE and int(recs[i_act + 1]["scope_key"]) == task
    assert recs[i_act + 2]["value_type"] == abi.VT_JOB
    assert r.variables(scope=task) == [("CREATED", "local", 7)]
    r.complete_jobs()
    pik = BASE + 1
    assert ("CREATED", "result", 7) in r.variables(scope=pik)
    assert not [row for row in r.o.state() if row.startswith("VARIABLES|%d|" % task)]


def test_output_mapping_updates_an_existing_variable_and_whole_decimals():
    # mergeDocument updates the variable where it exists (VARIABLE:UPDATED, its key); a whole decimal
    # is written as an integer (FeelToMessagePackTransformer.scala:35-39); a static source is a string
    xml = (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "t")
           .zeebeOutputExpression("2", "x").zeebeInput("static", "s").endEvent().done())
    r = Run(xml)
    r.create([("x", 1)])
    r.complete_jobs()
    pik = BASE + 1
    vs = r.variables(scope=pik)
    assert vs[0] == ("CREATED", "x", 1) and vs[-1] == ("UPDATED", "x", 2)
    task = r.key_of("task")
    assert r.variables(scope=task)[0][:2] == ("CREATED", "s")


def test_missing_source_variable_is_outside_the_subset():
    r = Run(bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "t")
            .zeebeInputExpression("missing", "y").endEvent().done())
    with pytest.raises(OracleError):
        r.create()


@pytest.mark.parametrize("mappings", [
    [("input", "=a", "x"), ("input", "=b", "y")],   # two entries: agrona document order unpinned
    [("input", "=a.b", "x")],                       # a path
    [("input", "=a", "x.y")],                       # a nested target
    [("output", "=a + 1", "x")],                    # an expression
])
def test_mappings_outside_the_subset(mappings):
    b = bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "t")
    for m in mappings:
        b._mapping(*m)
    with pytest.raises(OracleError):
        Oracle().deploy(b.endEvent().done())
