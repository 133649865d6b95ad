"""zeebe:ioMapping on the gfx950 path (the KScopeIO variant: variables in element-instance scopes)
against the CPU oracle (tests/test_oracle_io_mapping.py pins it on ActivityInputMappingTest /
ActivityOutputMappingTest): every record (the mapped VARIABLE records with their values inline),
the exported state after every window, log bytes and zb-db bytes, job activation variables, export ->
import -> continue, and the adapter inside the processing loop.

BpmnVariableMappingBehavior.java:53-156, VariableMappingTransformer.java:73-200, VariableBehavior.java:
60-200, FeelToMessagePackTransformer.scala:35-39."""
import numpy as np
import pytest

from helpers import create_commands
from test_gpu_parity import assert_same_records, run_both
from oracle.oracle import Oracle
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu


def _sub(mappings, inner="none"):
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("sub").startEvent()
    if inner == "task":
        b.serviceTask("task", "task")
    b.endEvent().subProcessDone()
    for m in mappings:
        b._mapping(*m)
    return b.endEvent().done()


def _task_in_out():
    return (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "t")
            .zeebeInputExpression("x", "local").zeebeOutputExpression("local", "result").endEvent().done())


def _two_tasks():
    return (bpmn.createExecutableProcess("process").startEvent().serviceTask("a", "a")
            .zeebeInputExpression("x", "t").zeebeOutputExpression("t", "r")
            .serviceTask("b", "b").zeebeInputExpression("r", "u").zeebeOutput("done", "status").endEvent().done())


def _literals():
    return (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "t")
            .zeebeOutputExpression("2", "x").zeebeInput("static", "s").serviceTask("t2", "t2")
            .zeebeInputExpression("true", "flag").zeebeOutputExpression("null", "x").endEvent().done())


def _xor_in_sub():
    # a condition inside the sub-process reads the sub-process's input-mapped variable (the scope chain)
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("sub").startEvent().exclusiveGateway("xor")
    (b.sequenceFlowId("high").conditionExpression("= y > 5").serviceTask("approve", "approve")
     .zeebeOutputExpression("y", "approved").endEvent("e1")
     .moveToNode("xor").sequenceFlowId("low").defaultFlow().endEvent("e2").subProcessDone()
     .zeebeInputExpression("x", "y").endEvent())
    return b.done()


def _nested():
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("outer").startEvent()
    b.subProcess("inner").startEvent().serviceTask("task", "task").zeebeOutputExpression("b", "c").endEvent()
    b.subProcessDone().zeebeInputExpression("a", "b").endEvent().subProcessDone().zeebeInputExpression("x", "a")
    return b.endEvent().done()


def _boundary():
    # applyInputMappings before subscribeToEvents: VARIABLE:CREATED, TIMER:CREATED, JOB:CREATED
    b = bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "t").zeebeInputExpression("x", "y")
    b.boundaryEvent("timer").timerWithDuration("PT1M").endEvent("timeout")
    return b.moveToActivity("task").endEvent("end").done()


SHAPES = {
    "sub_in_same": lambda: _sub([("input", "=x", "x")]),
    "sub_in": lambda: _sub([("input", "=x", "y")]),
    "sub_out": lambda: _sub([("output", "=x", "y")], "task"),
    "sub_in_out": lambda: _sub([("input", "=x", "y"), ("output", "=y", "z")], "task"),
    "sub_in_out_x": lambda: _sub([("input", "=x", "y"), ("output", "=x", "z")], "task"),
    "task_in_out": _task_in_out,
    "two_tasks": _two_tasks,
    "literals": _literals,
    "xor_in_sub": _xor_in_sub,
    "nested": _nested,
    "boundary": _boundary,
}
# document names of JOB:COMPLETE commands: a process variable, and a local one of some scope (merged where
# it exists: the task's or a sub-process's), within the device's 4 variables per instance
# (a job document merged locally by an output mapping is one variable more: "nested" and "two_tasks" would
# pass the 4, which falls back -- tested on its own below)
JOB_VARS = {"task_in_out": ("x", "local"), "sub_in_out": ("x", "y"), "sub_in_out_x": ("x", "y"), "sub_out": ("x", "y"),
            "xor_in_sub": ("x", "y"), "boundary": ("x", "y"), "nested": (), "two_tasks": ()}


class Both:
    def __init__(self, xml, n):
        self.part = Partition(max_instances=n, max_commands=max(n, 8), max_records_per_batch=128)
        self.orc = Oracle()
        assert self.part.deploy(xml) == self.orc.deploy(xml) == 0
        self.names = {}
        self.strings = []

    def name(self, nm):
        if nm not in self.names:
            a, b = self.part.intern(nm), self.orc.intern(nm)
            assert a == b
            self.names[nm] = a
        return self.names[nm]

    def value(self, rng, entry, nm, numbers=False):
        """a random value of every device type (decimals whole and not: whole ones become INT); numbers:
        ints and decimals only (a FEEL ordering comparison over other types is outside the subset)"""
        entry["name_id"] = self.name(nm)
        k = int(rng.choice([0, 1, 2, 6])) if numbers else int(rng.integers(0, 7))
        if k == 0:
            entry["type"], entry["value"] = abi.DOC_INT, int(rng.integers(-20, 20))
        elif k == 1:
            entry["type"], entry["value"] = abi.DOC_DEC, int(rng.integers(-20, 20)) * 10 ** abi.DEC_SCALE
        elif k == 2:
            entry["type"], entry["value"] = abi.DOC_DEC, int(rng.integers(-2000000, 2000000)) * 10 ** 4
        elif k == 3:
            s = "s%d" % rng.integers(0, 5)
            a, b = self.part.intern_string(s), self.orc.intern_string(s)
            assert a == b
            entry["type"], entry["value"] = abi.DOC_STR, a
        elif k == 4:
            entry["type"], entry["value"] = abi.DOC_BOOL, int(rng.integers(0, 2))
        elif k == 5:
            entry["type"], entry["value"] = abi.DOC_NIL, 0
        else:
            entry["type"], entry["value"] = abi.DOC_INT, int(rng.integers(0, 12))

    def window(self, cmds, docs=None):
        got = run_both(self.part, self.orc, cmds, docs)
        assert self.part.state() == self.orc.state()
        return got


def drive(xml, n, seed, phases=8, job_vars=("x",), numbers=False):
    rng = np.random.default_rng(seed)
    B = Both(xml, n)
    cmds = create_commands(n, 0)
    docs = abi.make_docs(n)
    for i in range(n):
        B.value(rng, docs[i], "x", numbers)
    cmds["doc_count"] = 1
    cmds["doc_begin"] = np.arange(n)
    B.window(cmds, docs)
    for _ in range(phases):
        keys = sorted(int(r.split("|")[1]) for r in B.part.state() if r.startswith("JOBS|"))
        if not keys:
            break
        by_inst = {}
        for k in keys:
            inst, ordv = B.part.resolve_key(k)
            by_inst.setdefault(inst, ordv)
        insts = sorted(by_inst)
        c = abi.make_commands(len(insts))
        c["instance"] = insts
        c["ref"] = [by_inst[i] for i in insts]
        c["kind"] = abi.CMD_JOB_COMPLETE
        d = abi.make_docs(len(insts))
        for j in range(len(insts)):
            if job_vars and rng.integers(0, 2):
                B.value(rng, d[j], job_vars[int(rng.integers(0, len(job_vars)))], numbers)
                c[j]["doc_count"], c[j]["doc_begin"] = 1, j
        B.window(c, d)
    assert B.part.stats()["fallback"] == 0
    return B


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_gpu_io_mapping_parity(shape):
    drive(SHAPES[shape](), 160, seed=len(shape), job_vars=JOB_VARS.get(shape, ("x",)), numbers=shape == "xor_in_sub")


def test_gpu_io_mapping_record_values_inline():
    # the input mapping's VARIABLE:CREATED carries the source's value inline, scopeKey = the task
    B = Both(_task_in_out(), 4)
    c = create_commands(1, 0)
    d = abi.make_docs(1)
    d[0]["name_id"], d[0]["type"], d[0]["value"] = B.name("x"), abi.DOC_DEC, 2500000  # 2.5
    c["doc_count"] = 1
    recs = B.window(c, d)
    v = [r for r in recs if r["value_type"] == abi.VT_VARIABLE]
    task = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and B.part.element_id(0, int(r["element_idx"])) == "task"]
    assert int(v[1]["scope_key"]) == int(task[-1]["key"]) and int(v[1]["aux"]) == abi.AUX_INLINE
    assert (int(v[1]["partition"]), int(v[1]["message_key"])) == (abi.DOC_DEC, 2500000)


def test_gpu_missing_source_variable_falls_back():
    B = Both(_task_in_out(), 4)
    B.part.submit(create_commands(1, 0))
    B.part.run()
    assert B.part.command_status(0)[0] != 0 and B.part.drain().size == 0


@pytest.mark.parametrize("shape", ["task_in_out", "sub_in_out", "nested", "two_tasks"])
def test_gpu_io_mapping_log_and_db_bytes(shape):
    # the host serialiser writes the inline VARIABLE values (== oracle/logserial.py), zb-db bytes of
    # the element-scope VARIABLES rows (== oracle/statedb.py)
    from test_gpu_logserial import Pair, drive as drive_log
    pair = Pair(SHAPES[shape](), 100, names=["x"])
    d = abi.make_docs(100)
    d["name_id"], d["type"], d["value"] = 0, abi.DOC_INT, np.arange(100)
    drive_log(pair, 100, d)


def test_gpu_io_mapping_job_activation_variables():
    # JOB_BATCH:ACTIVATE: the task's local (input-mapped) variable first, then the enclosing scopes'
    # (a sub-process's own variables included), names once (DbVariableState.getVariablesAsDocument)
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("sub").startEvent()
    b.serviceTask("task", "act").zeebeInputExpression("y", "x").endEvent().subProcessDone().zeebeInputExpression("x", "y")
    B = Both(b.endEvent().done(), 8)
    c = create_commands(4, 0)
    d = abi.make_docs(4)
    d["name_id"], d["type"], d["value"] = B.name("x"), abi.DOC_INT, np.arange(4) + 10
    c["doc_count"], c["doc_begin"] = 1, np.arange(4)
    B.window(c, d)
    gk, gj, _ = B.part.activate_jobs("act", max_jobs=4)
    ok, oj, _ = B.orc.activate_jobs("act", max_jobs=4)
    assert gk == ok and len(gj) == len(oj) == 4
    for g, o in zip(gj, oj):
        gv = [(int(v["name_id"]), int(v["type"]), int(v["value"])) for v in g["variables"][:int(g["n_variables"])]]
        ov = [(int(v["name_id"]), int(v["type"]), int(v["value"])) for v in o["variables"][:int(o["n_variables"])]]
        assert gv == ov and len(gv) == 2
    assert B.part.state() == B.orc.state()


def test_gpu_io_mapping_restart():
    from test_gpu_import import _same

    # export -> fresh handle -> import -> continue equals the uninterrupted partition and the oracle
    # (task- and sub-process-scope variables restored into their scopes)
    xml = _sub([("input", "=x", "y"), ("output", "=y", "z")], "task")
    B = Both(xml, 64)
    c = create_commands(64, 0)
    d = abi.make_docs(64)
    d["name_id"], d["type"], d["value"] = B.name("x"), abi.DOC_INT, np.arange(64)
    c["doc_count"], c["doc_begin"] = 1, np.arange(64)
    B.window(c, d)
    entries = B.part.state_db()
    fresh = Partition(max_instances=64, max_commands=64, max_records_per_batch=128)
    assert fresh.deploy(xml) == 0
    assert fresh.intern("x") == B.name("x")
    assert fresh.import_state_db(entries) == 64
    assert fresh.state() == B.part.state()
    # the same JOB:COMPLETE commands, each side addressing the job by its own key ordinals (the import
    # numbers an instance's keys in key order)
    keys = sorted(int(r.split("|")[1]) for r in fresh.state() if r.startswith("JOBS|"))
    refs = [fresh.resolve_key(k) for k in keys]
    cc = abi.make_commands(len(refs))
    cc["instance"], cc["ref"], cc["kind"] = [r[0] for r in refs], [r[1] for r in refs], abi.CMD_JOB_COMPLETE
    co = cc.copy()
    co["ref"] = [B.orc.ordinal_of(int(r[0]), k) for r, k in zip(refs, keys)]
    fresh.submit(cc)
    fresh.run()
    got = fresh.drain()
    B.orc.clear_records()
    B.orc.submit(co)
    B.orc.run()
    _same(got, B.orc.records())  # (source_index / aux bases are each handle's own counters)
    assert fresh.state() == B.orc.state()
    assert [r for r in fresh.state() if not r.startswith("KEY|")] == []


def test_gpu_io_mapping_variable_capacity_falls_back():
    # a fifth variable of an instance (zb_internal.h kVars): the job's document merged into the task's
    # scope next to four others -- the command falls back, its instance untouched
    B = Both(_nested(), 4)
    c = create_commands(1, 0)
    d = abi.make_docs(1)
    d[0]["name_id"], d[0]["type"], d[0]["value"] = B.name("x"), abi.DOC_INT, 3
    c["doc_count"] = 1
    B.window(c, d)
    before = B.part.state()
    job = next(int(r.split("|")[1]) for r in before if r.startswith("JOBS|"))
    inst, ordv = B.part.resolve_key(job)
    cc = abi.make_commands(1)
    cc["instance"], cc["ref"], cc["kind"], cc["doc_count"] = inst, ordv, abi.CMD_JOB_COMPLETE, 1
    B.part.submit(cc, d)
    B.part.run()
    assert B.part.command_status(0) == (1, "vars") and B.part.state() == before
