"""Interrupting timer boundary events on the gfx950 path (KScope) against the CPU oracle with the same
clock: the boundary timer created with the task (before its job), canceled when the job completes
first (TIMER:CANCELED with the stored dueDate), or triggered first -- TERMINATE_ELEMENT of the task,
JOB:CANCELED, ELEMENT_TERMINATED, PROCESS_EVENT:TRIGGERED and the boundary event's activation and
outgoing flows; each instance's open job or timer is chosen at random every round.  Records, state,
host log bytes, zb-db bytes and restart through zb-db bytes.  Reference: BoundaryEventTest.java:48-139,
ActivityTest.java:150-199, JobWorkerTaskProcessor.java:77-104, EventTriggerBehavior.java:191-244."""
import pytest

from test_gpu_logserial import Pair
from test_gpu_timers import _open_work, drive_timers, part_key
from test_oracle_boundary import cycle_process, multiple_sequence_flows, non_interrupting_process, sub_process_boundary
from test_oracle_timers import NOW
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition
from helpers import create_commands
import numpy as np

pytestmark = pytest.mark.gpu


def _linear_with_boundary():
    # a -> b, a's timer escalates to c
    b = bpmn.createExecutableProcess("process").startEvent("s").serviceTask("a", "a").boundaryEvent("late")
    b.timerWithDuration("PT5M").serviceTask("c", "c").endEvent("ce").moveToActivity("a").serviceTask("b", "b")
    return b.endEvent("e").done()


def _boundary_in_sub_process():
    b = bpmn.createExecutableProcess("process").startEvent().parallelGateway("fork").subProcess("sub").startEvent()
    b.serviceTask("inner", "inner").boundaryEvent("late").timerWithDuration("PT1M").endEvent("lateEnd")
    b.moveToActivity("inner").endEvent().subProcessDone().parallelGateway("join").moveToNode("fork")
    b.serviceTask("other", "other").connectTo("join")
    return b.endEvent("e").done()


def _boundary_then_catch():
    # the boundary timer's row is reused by the catch event after the task (one timer at a time)
    b = bpmn.createExecutableProcess("process").startEvent("s").jobWorkerTask("scriptTask", "a", "a")
    b.boundaryEvent("late").timerWithDuration("PT2H").endEvent("le").moveToActivity("a")
    b.intermediateCatchEvent("wait").timerWithDuration("PT1S").serviceTask("z", "z")
    return b.endEvent("e").done()


def _boundary_to_gateway():
    # the boundary event leaves through a parallel gateway into two tasks
    b = bpmn.createExecutableProcess("process").startEvent("s").serviceTask("a", "a").boundaryEvent("late")
    b.timerWithDuration("PT10S").parallelGateway("fork").serviceTask("x", "x").parallelGateway("join")
    b.moveToNode("fork").serviceTask("y", "y").connectTo("join").endEvent("je").moveToActivity("a")
    return b.endEvent("e").done()


def _non_interrupting_escalation():
    # a non-interrupting reminder that runs a task of its own while the activity waits
    b = bpmn.createExecutableProcess("process").startEvent("s").serviceTask("a", "a").boundaryEvent("remind")
    b.cancelActivity(False).timerWithDuration("PT1H").serviceTask("r", "r").endEvent("re").moveToActivity("a")
    return b.serviceTask("b", "b").endEvent("e").done()


def _sub_process_parallel(interrupting=True):
    # a timer boundary event on a sub-process whose fork keeps two tasks active: PROCESS_INSTANCE_BATCH
    # :TERMINATE terminates both (key order), then the sub-process, then the boundary event
    b = bpmn.createExecutableProcess("process").startEvent("s").subProcess("sub").startEvent("ss").parallelGateway("fork")
    b.serviceTask("x", "x").parallelGateway("join").moveToNode("fork").serviceTask("y", "y").connectTo("join")
    b.endEvent("se").subProcessDone().boundaryEvent("late").cancelActivity(interrupting).timerWithDuration("PT20S")
    b.serviceTask("late_task", "late").endEvent("le")
    return b.moveToActivity("sub").serviceTask("after", "after").endEvent("e").done()


def _nested_sub_processes():
    # the boundary event on the outer sub-process: its termination reaches the inner one's task
    b = bpmn.createExecutableProcess("process").startEvent("s").subProcess("outer").startEvent("os")
    b.serviceTask("a", "a").subProcess("inner").startEvent("is").serviceTask("b", "b").endEvent("ie").subProcessDone()
    b.endEvent("oe").subProcessDone().boundaryEvent("late").timerWithDuration("PT15S").endEvent("le")
    return b.moveToActivity("outer").endEvent("e").done()


def _sub_process_multi_instance():
    # a multi-instance task inside a sub-process whose boundary timer terminates it: the body's inner
    # instances through PROCESS_INSTANCE_BATCH:TERMINATE, then the body, then the sub-process
    # (MultiInstanceBodyProcessor.onTerminate / onChildTerminated / terminate)
    b = bpmn.createExecutableProcess("process").startEvent("start").subProcess("sub").startEvent("ss")
    b.serviceTask("task", "task")
    b.multiInstance("= [1, 2, 3]", "item", False)
    b.endEvent("se").subProcessDone().boundaryEvent("late").timerWithDuration("PT2S")
    b.sequenceFlowId("to-canceled").endEvent("canceled")
    return b.moveToActivity("sub").endEvent("end").done()


def _interrupting_cycle(sub=False):
    # an interrupting boundary event with a timeCycle (TriggerTimerProcessor.shouldReschedule does not look at
    # the activity: the next timer is created after the TERMINATE_ELEMENT command and canceled with the
    # activity); on a task or on a sub-process
    b = bpmn.createExecutableProcess("process").startEvent("s")
    if sub:
        b.subProcess("sub").startEvent("ss").serviceTask("a", "a").endEvent("se").subProcessDone()
        act = "sub"
    else:
        b.serviceTask("a", "a")
        act = "a"
    b.boundaryEvent("late").timerWithCycle("R3/PT20S").serviceTask("c", "c").endEvent("ce").moveToActivity(act)
    return b.endEvent("e").done()


SHAPES = {"multiple_sequence_flows": lambda: multiple_sequence_flows("PT30S"), "linear": _linear_with_boundary,
          "interrupting_cycle": _interrupting_cycle, "interrupting_cycle_sub": lambda: _interrupting_cycle(True),
          "sub_process_multi_instance": _sub_process_multi_instance,
          "sub_process": lambda: sub_process_boundary(True, "PT10S"),
          "sub_process_non_interrupting": lambda: sub_process_boundary(False, "PT10S"),
          "sub_process_parallel": _sub_process_parallel,
          "sub_process_parallel_non_interrupting": lambda: _sub_process_parallel(False),
          "nested_sub_processes": _nested_sub_processes,
          "non_interrupting": lambda: non_interrupting_process("PT30S"),
          "non_interrupting_escalation": _non_interrupting_escalation,
          "cycle_infinite": lambda: cycle_process("R/PT30S"), "cycle_r3": lambda: cycle_process("R3/PT10S"),
          "in_sub_process": _boundary_in_sub_process, "then_catch": _boundary_then_catch,
          "to_gateway": _boundary_to_gateway}


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("seed", [3, 8])
def test_gpu_boundary_parity(shape, seed):
    part, orc = drive_timers(SHAPES[shape](), 200, seed=seed)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


def test_gpu_boundary_both_outcomes():
    # every instance's first move: even instances complete the job, odd ones fire the timer
    xml = multiple_sequence_flows("PT30S")
    n = 64
    part = Partition(max_instances=n, max_commands=n, max_records_per_batch=128)
    from oracle.oracle import Oracle
    from test_gpu_parity import run_both
    orc = Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    for e in (part, orc):
        e.set_clock(NOW)
    run_both(part, orc, create_commands(n, 0))
    rows = part.state()
    c = abi.make_commands(n)
    for r in rows:
        p = r.split("|")
        if r.startswith("JOBS|"):
            inst, ordv = part.resolve_key(int(p[1]))
            if inst % 2 == 0:
                c[inst]["instance"], c[inst]["kind"], c[inst]["ref"] = inst, abi.CMD_JOB_COMPLETE, ordv
        elif r.startswith("TIMERS|"):
            inst, ordv = part.resolve_key(int(p[2]))
            due = int(dict(kv.split("=") for kv in p[3].split(","))["dueDate"])
            if inst % 2 == 1:
                c[inst]["instance"], c[inst]["kind"], c[inst]["ref"] = inst, abi.CMD_TIMER_TRIGGER, ordv
                c[inst]["doc_begin"], c[inst]["pad"] = due & 0xFFFFFFFF, due >> 32
    for e in (part, orc):
        e.set_clock(NOW + 30000)
    got = run_both(part, orc, c)
    assert part.state() == orc.state() == [r for r in part.state() if r.startswith("KEY|")]
    assert (got["value_type"] == abi.VT_TIMER).sum() == n  # CANCELED for even, TRIGGERED for odd
    assert ((got["value_type"] == abi.VT_JOB) & (got["intent"] == abi.JOB_CANCELED)).sum() == n // 2
    assert part.stats()["fallback"] == 0


# (141, 312: a batch cancels the task's stored timer, then creates and cancels a sub-process's
# boundary timer of its own -- two TIMER:CANCELED with different dueDates in one batch; found by
# scripts/fuzz_random.py)
@pytest.mark.parametrize("seed", list(range(8)) + [141, 312])
def test_gpu_random_processes_with_boundary_events(seed):
    # tests/random_bpmn.py: random structured processes (sub-processes, job worker kinds) whose
    # tasks outside parallel branches may carry a timer boundary event; each round completes a job
    # or fires a timer per instance at random
    from helpers import amount_docs
    from random_bpmn import random_process
    rng = np.random.default_rng(6000 + seed)
    xml = random_process(rng, sub_processes=True, task_kinds=True, boundaries=True)
    part, orc = drive_timers(xml, 96, seed=seed, phases=60, max_records=256,
                             docs_fn=lambda n: amount_docs(rng.integers(0, 1000, n), 0))
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


# (140, 151: multi-instance bodies terminated with their sub-process; 228, 271: see above)
@pytest.mark.parametrize("seed", list(range(8)) + [140, 151, 228, 271])
def test_gpu_random_processes_with_multi_instance_activities(seed):
    # the same with multi-instance tasks among them (static collections, parallel or sequential, an
    # outputCollection, sequential completion conditions): each round completes inner instances' jobs
    from helpers import amount_docs
    from random_bpmn import random_process
    rng = np.random.default_rng(7000 + seed)
    xml = random_process(rng, sub_processes=True, task_kinds=True, boundaries=True, multi_instance=True)
    part, orc = drive_timers(xml, 96, seed=seed, phases=80, max_records=256,
                             docs_fn=lambda n: amount_docs(rng.integers(0, 1000, n), 0))
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


@pytest.mark.parametrize("shape", ["multiple_sequence_flows", "in_sub_process", "then_catch", "non_interrupting_escalation",
                                   "cycle_r3", "sub_process", "sub_process_parallel", "nested_sub_processes",
                                   "interrupting_cycle", "interrupting_cycle_sub"])
def test_gpu_boundary_log_and_db_bytes(shape):
    pair = Pair(SHAPES[shape](), 100)
    for e in (pair.part, pair.orc):
        e.set_clock(NOW)
    pair.window(create_commands(100, 0))
    rng = np.random.default_rng(5)
    for step in range(8):
        c = _open_work(pair.part, rng)
        if c is None:
            break
        for e in (pair.part, pair.orc):
            e.set_clock(NOW + 1000 * (step + 1))
        pair.window(c)


@pytest.mark.parametrize("shape", ["linear", "in_sub_process", "non_interrupting_escalation", "cycle_infinite",
                                   "sub_process", "sub_process_parallel_non_interrupting"])
def test_gpu_boundary_restart_equivalence(shape):
    xml = SHAPES[shape]()
    n = 48
    part, orc = drive_timers(xml, n, phases=1)
    fresh = Partition(max_instances=n, max_commands=n, max_records_per_batch=128)
    assert fresh.deploy(xml) == 0
    entries = part.state_db()
    fresh.import_state_db(entries)
    assert fresh.state() == part.state() and fresh.state_db() == entries
    rng = np.random.default_rng(11)
    clock = NOW + 100000
    for _ in range(10):
        c = _open_work(part, rng)
        if c is None:
            break
        clock += 1000
        c2 = c.copy()
        for j, cmd in enumerate(c):
            c2[j]["instance"], c2[j]["ref"] = fresh.resolve_key(part_key(part, int(cmd["instance"]), int(cmd["ref"])))
        for p, cc in ((part, c), (fresh, c2)):
            p.set_clock(clock)
            p.submit(cc)
            p.run()
            p.drain()
        orc.set_clock(clock)
        orc.clear_records()
        orc.submit(c)
        orc.run()
        assert part.state() == orc.state() == fresh.state()
    assert [r for r in fresh.state() if not r.startswith("KEY|")] == []


@pytest.mark.parametrize("shape", ["multiple_sequence_flows", "non_interrupting_escalation", "cycle_r3", "to_gateway"])
def test_gpu_boundary_batch_limit(shape):
    # maxCommandsInBatch = 3: the boundary event's follow-ups (its COMPLETE_ELEMENT, the flows'
    # ACTIVATEs) are written to the log unprocessed and run as continuation batches
    # (ProcessingStateMachine.java:388-417), records (`unprocessed` flags included) and state equal
    from oracle.oracle import Oracle
    from test_gpu_parity import run_both
    n = 32
    part = Partition(max_instances=n, max_commands=64 * n, max_records_per_batch=256, max_commands_in_batch=3)
    orc = Oracle(max_commands_in_batch=3)
    xml = SHAPES[shape]()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    clock = NOW
    for e in (part, orc):
        e.set_clock(clock)
    run_both(part, orc, create_commands(n, 0))
    rng = np.random.default_rng(12)
    unprocessed = 0
    for _ in range(20):
        c = _open_work(part, rng)
        if c is None:
            break
        clock += 1000
        for e in (part, orc):
            e.set_clock(clock)
        got = run_both(part, orc, c)
        unprocessed += int(got["unprocessed"].sum())
        assert part.state() == orc.state()
    assert part.stats()["fallback"] == 0 and unprocessed > 0
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


def test_gpu_late_cycle_triggers():
    # TriggerTimerProcessor.refreshTimer + Interval.toEpochMilli (Interval.java:77-93): the next
    # timer of a cycle starts at dueDate + interval unless that is not after the clock, then clock +
    # interval.  Four groups of instances are triggered in four windows, each later past its dueDate
    # (0, 999, 1000 and 2500 ms late, PT1S cycle); records and state equal the oracle's and the device
    # log bytes equal the host serialiser's
    from oracle.oracle import Oracle
    from test_gpu_logdev import Log
    from test_gpu_parity import assert_same_records
    xml = cycle_process("R/PT1S")
    n = 4 * 64
    log = Log(xml, n)
    orc = Oracle()
    assert orc.deploy(xml) == 0
    for e in (log.part, orc):
        e.set_clock(NOW)
    orc.submit(create_commands(n, 0))
    orc.run()
    assert_same_records(log.window(create_commands(n, 0)), orc.records())
    timers = {}
    for r in log.part.state():
        if r.startswith("TIMERS|"):
            p = r.split("|")
            timers[log.part.resolve_key(int(p[2]))] = int(dict(kv.split("=") for kv in p[3].split(","))["dueDate"])
    assert len(timers) == n
    for g, late in enumerate((0, 999, 1000, 2500)):
        mine = [(i, o) for (i, o) in sorted(timers) if i // 64 == g]
        c = abi.make_commands(len(mine))
        for j, (i, o) in enumerate(mine):
            due = timers[(i, o)]
            c[j]["instance"], c[j]["kind"], c[j]["ref"] = i, abi.CMD_TIMER_TRIGGER, o
            c[j]["doc_begin"], c[j]["pad"] = due & 0xFFFFFFFF, due >> 32
        for e in (log.part, orc):
            e.set_clock(NOW + 1000 + late)
        orc.clear_records()
        orc.submit(c)
        orc.run()
        got = log.window(c)
        assert_same_records(got, orc.records())
        nxt = got[(got["value_type"] == abi.VT_TIMER) & (got["intent"] == abi.TIMER_CREATED)]
        want_due = NOW + 2000 if late < 1000 else NOW + 1000 + late + 1000
        assert len(nxt) == 64 and (nxt["aux"] == want_due).all()
        assert log.part.state() == orc.state()
