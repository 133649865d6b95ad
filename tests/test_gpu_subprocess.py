"""Embedded sub-processes on the gfx950 path (KScope: flow scopes below the process, SURVEY §8(f)
row 4) against the CPU oracle: records (flowScopeKey of every element inside a sub-process = the
sub-process instance's key), exported state (the sub-process's childCount / activeSequenceFlows,
parent-child rows, taken-flow counters keyed by the sub-process instance), log bytes (host and
device serialisers) and zb-db bytes.  Shapes from EmbeddedSubProcessTest.java:41-62,386-467 and
random structured processes with nested sub-processes (tests/random_bpmn.py).  Also the other job
worker tasks (send / script / business-rule tasks with a zeebe:taskDefinition)."""
import numpy as np
import pytest

from helpers import amount_docs, create_commands
from random_bpmn import random_process
from test_gpu_logdev import Log, job_completions
from test_gpu_logserial import Pair
from test_gpu_logserial import drive as drive_log
from test_gpu_parity import drive
from oracle.oracle import Oracle
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu

ET = {n: i for i, n in enumerate(abi.ELEMENT_TYPES)}


def _parallel_no_join():
    # EmbeddedSubProcessTest.shouldCompleteSubProcessWithParallelFlow (:422-467)
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("sub-process").startEvent()
    (b.parallelGateway("fork").serviceTask("task-1", "task-1").endEvent()
     .moveToLastGateway().serviceTask("task-2", "task-2").endEvent().subProcessDone().endEvent())
    return b.done()


def _xor_inside():
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("sub").startEvent().exclusiveGateway("xor")
    (b.sequenceFlowId("high").conditionExpression("= amount > 1000").serviceTask("approve", "approve").endEvent("e1")
     .moveToNode("xor").sequenceFlowId("low").defaultFlow().endEvent("e2").subProcessDone()
     .serviceTask("after", "after").endEvent())
    return b.done()


def _sub_then_task_then_sub():
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("s1").startEvent().serviceTask("a", "a")
    b.endEvent().subProcessDone().serviceTask("mid", "mid").subProcess("s2").startEvent()
    b.subProcess("s3").startEvent().serviceTask("b", "b").endEvent().subProcessDone().endEvent().subProcessDone()
    return b.endEvent().done()


SHAPES = {
    "none": lambda: bpmn.sub_process_process("none"),
    "task": lambda: bpmn.sub_process_process("task"),
    "parallel": lambda: bpmn.sub_process_process("parallel"),
    "nested": lambda: bpmn.sub_process_process("nested"),
    "parallel_no_join": _parallel_no_join,
    "chain": _sub_then_task_then_sub,
}


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_gpu_sub_process_parity(shape):
    part, orc = drive(SHAPES[shape](), 200, phases=20, rng_seed=7)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []
    assert part.stats()["fallback"] == 0


def test_gpu_sub_process_flow_scope_keys():
    # shouldActivateSubProcess (:82-115): the sub-process's flowScopeKey is the process instance;
    # its children's is the sub-process instance
    part = Partition(max_instances=4, max_commands=4)
    part.deploy(bpmn.sub_process_process("task"))
    part.submit(create_commands(1, 0))
    part.run()
    recs = part.drain()
    pi = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE]
    sub = [r for r in pi if part.element_id(0, int(r["element_idx"])) == "sub-process"]
    task = [r for r in pi if part.element_id(0, int(r["element_idx"])) == "task"]
    pik = int(recs[0]["key"])
    assert all(int(r["scope_key"]) == pik for r in sub)
    assert all(int(r["scope_key"]) == int(sub[0]["key"]) for r in task if r["record_type"] != abi.RT_COMMAND)


def test_gpu_sub_process_xor_inside():
    rng = np.random.default_rng(11)
    part, orc = drive(_xor_inside(), 300, lambda n: amount_docs(rng.integers(0, 2001, n), 0), phases=10)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


RANDOM_SEEDS = [s for s in range(40) if random_process(np.random.default_rng(3000 + s), sub_processes=True)
                .count("<subProcess") > 0]


@pytest.mark.parametrize("seed", RANDOM_SEEDS)
def test_gpu_random_sub_process_parity(seed):
    rng = np.random.default_rng(3000 + seed)
    xml = random_process(rng, sub_processes=True)
    part, orc = drive(xml, 96, lambda n: amount_docs(rng.integers(0, 1000, n), 0), phases=60, rng_seed=seed,
                      max_records=256)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


@pytest.mark.parametrize("shape", ["task", "parallel", "chain"])
def test_gpu_sub_process_log_and_db_bytes(shape):
    # host serialiser over the drained records == oracle/logserial.py; zb-db bytes == oracle/statedb.py
    drive_log(Pair(SHAPES[shape](), 120), 120)


@pytest.mark.parametrize("shape", ["task", "parallel", "nested", "chain"])
def test_gpu_sub_process_device_log_bytes(shape):
    log = Log(SHAPES[shape](), 150)
    recs = log.window(create_commands(150, 0))
    rng = np.random.default_rng(5)
    for _ in range(12):
        c = job_completions(recs, log.part, rng)
        if c is None or len(c) == 0:
            break
        recs = log.window(c)


def test_gpu_second_active_instance_of_a_sub_process_falls_back():
    # two tokens reach one sub-process element (a fork with two flows into it): outside the device
    # subset (one active instance per sub-process element) -> the whole CREATE batch falls back,
    # nothing written, the instance fenced
    b = bpmn.createExecutableProcess("process").startEvent().parallelGateway("fork").subProcess("sub")
    b.startEvent().serviceTask("t", "t").endEvent().subProcessDone().endEvent("end").moveToNode("fork").connectTo("sub")
    xml = b.done()
    part = Partition(max_instances=8, max_commands=8)
    part.deploy(xml)
    part.submit(create_commands(4, 0))
    part.run()
    assert part.stats()["fallback"] == 4
    assert len(part.drain()) == 0
    assert [r for r in part.state() if not r.startswith("KEY|")] == []
    # the oracle runs it (two sub-process instances in one scope)
    o = Oracle()
    o.deploy(xml)
    o.submit(create_commands(1, 0))
    o.run()
    subs = [r for r in o.records() if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == 3
            and o.element_type(0, int(r["element_idx"])) == ET["SUB_PROCESS"]]
    assert len(subs) == 2


# ---- job worker tasks: send / script / business-rule tasks with a zeebe:taskDefinition ----------
def test_gpu_job_worker_task_kinds_linear():
    # a linear chain of the four job worker kinds: KLinear's straight-line segments cover them
    from test_oracle_subprocess import _job_worker_chain
    part, orc = drive(_job_worker_chain(), 500, phases=6)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


def test_gpu_job_worker_task_kinds_log_bytes():
    from test_oracle_subprocess import _job_worker_chain
    drive_log(Pair(_job_worker_chain(), 100), 100)


@pytest.mark.parametrize("seed", range(8))
def test_gpu_random_job_worker_kinds_with_sub_processes(seed):
    rng = np.random.default_rng(4000 + seed)
    xml = random_process(rng, sub_processes=True, task_kinds=True)
    part, orc = drive(xml, 96, lambda n: amount_docs(rng.integers(0, 1000, n), 0), phases=60, rng_seed=seed,
                      max_records=256)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []
