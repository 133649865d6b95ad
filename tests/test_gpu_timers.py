"""Timer intermediate catch events on the gfx950 path (KScope; the instance's timer row in HBM)
against the CPU oracle with the same clock: TIMER:CREATED (dueDate = clock + duration), TIMER:TRIGGER
commands (the due-date checker's, built from the exported TIMERS rows) -> TIMER:TRIGGERED, PROCESS_EVENT
:TRIGGERING and the catch event's completion; NOT_FOUND rejections of stale triggers; records, state
(TIMERS, TIMER_DUE_DATES, EVENT_SCOPE rows), host log bytes and zb-db bytes; restart through zb-db
bytes.  Reference: TimerCatchEventTest.java:122-296, TriggerTimerProcessor.java:81-114,
CatchEventBehavior.java:303-330."""
import numpy as np
import pytest

from oracle.oracle import Oracle
from test_gpu_logserial import Pair
from test_gpu_parity import run_both
from test_oracle_timers import NOW, timer_process, trigger_commands
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition
from helpers import create_commands

pytestmark = pytest.mark.gpu


def _open_work(part, rng):
    """One command per instance for its open jobs / timer (chosen at random): JOB:COMPLETE or
    TIMER:TRIGGER with the timer's dueDate (what DueDateTimerChecker writes)."""
    items = {}
    for r in part.state():
        if r.startswith("JOBS|"):
            k = int(r.split("|")[1])
            inst, ordv = part.resolve_key(k)
            items.setdefault(inst, []).append((abi.CMD_JOB_COMPLETE, ordv, 0))
        elif r.startswith("TIMERS|"):
            parts = r.split("|")
            k = int(parts[2])
            due = int(dict(kv.split("=") for kv in parts[3].split(","))["dueDate"])
            inst, ordv = part.resolve_key(k)
            items.setdefault(inst, []).append((abi.CMD_TIMER_TRIGGER, ordv, due))
    if not items:
        return None
    insts = sorted(items)
    c = abi.make_commands(len(insts))
    for i, inst in enumerate(insts):
        kind, ordv, due = items[inst][rng.integers(len(items[inst]))]
        c[i]["instance"], c[i]["kind"], c[i]["ref"] = inst, kind, ordv
        c[i]["doc_begin"], c[i]["pad"] = due & 0xFFFFFFFF, due >> 32
    return c


def drive_timers(xml, n, seed=0, phases=30, docs_fn=None, max_records=128):
    part = Partition(max_instances=n, max_commands=max(n, 8), max_records_per_batch=max_records)
    orc = Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    clock = NOW
    for e in (part, orc):
        e.set_clock(clock)
    cmds, docs = create_commands(n, 0), None
    if docs_fn is not None:  # an `amount` per instance (random processes' conditions)
        assert part.intern("amount") == orc.intern("amount")
        docs = docs_fn(n)
        cmds["doc_count"] = 1
        cmds["doc_begin"] = np.arange(n)
    run_both(part, orc, cmds, docs)
    assert part.state() == orc.state()
    rng = np.random.default_rng(seed)
    for _ in range(phases):
        c = _open_work(part, rng)
        if c is None:
            break
        clock += 1000
        for e in (part, orc):
            e.set_clock(clock)
        run_both(part, orc, c)
        assert part.state() == orc.state()
    assert part.stats()["fallback"] == 0
    return part, orc


def _task_timer_task():
    return (bpmn.createExecutableProcess("process").startEvent("s").serviceTask("a", "a").intermediateCatchEvent("wait")
            .timerWithDuration("PT15M").serviceTask("b", "b").endEvent("e").done())


def _timer_in_branch():
    # a fork: one branch waits on a timer, the other on a job; join
    b = bpmn.createExecutableProcess("process").startEvent("s").parallelGateway("fork").intermediateCatchEvent("t1")
    b.timerWithDuration("PT1H").parallelGateway("join").moveToNode("fork").serviceTask("job", "job").connectTo("join")
    return b.endEvent("e").done()


def _timer_in_sub_process():
    b = bpmn.createExecutableProcess("process").startEvent("s").subProcess("sub").startEvent()
    b.intermediateCatchEvent("t").timerWithDuration("PT30S").serviceTask("x", "x").endEvent().subProcessDone()
    return b.endEvent("e").done()


SHAPES = {"timer": lambda: timer_process("PT10S"), "task_timer_task": _task_timer_task,
          "timer_in_branch": _timer_in_branch, "timer_in_sub_process": _timer_in_sub_process,
          "zero": lambda: timer_process("PT0S"),
          # constant FEEL expressions (BoundaryEventTest.java:48-69's forms)
          "feel_duration": lambda: timer_process('=duration("PT0.1S")'),
          "feel_cycle_boundary": lambda: (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "type")
                                          .boundaryEvent("event").cancelActivity(False)
                                          .timerWithCycleExpression('cycle(3, duration("PT1S"))').endEvent()
                                          .moveToActivity("task").endEvent().done())}


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_gpu_timer_parity(shape):
    part, orc = drive_timers(SHAPES[shape](), 200, seed=3)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


def test_gpu_stale_timer_trigger_is_rejected():
    part, orc = drive_timers(timer_process("PT1M"), 32, phases=0)
    rows = [r.split("|") for r in part.state() if r.startswith("TIMERS|")]
    keys = [(int(p[2]), int(dict(kv.split("=") for kv in p[3].split(","))["dueDate"])) for p in rows]
    res = [part.resolve_key(k) for k, _ in keys]
    c = trigger_commands([i for i, _ in res], [o for _, o in res], [d for _, d in keys])
    run_both(part, orc, c)
    got = run_both(part, orc, c)  # every timer already triggered: NOT_FOUND rejections
    assert (got["record_type"] == abi.RT_REJECTION).all() and (got["value_type"] == abi.VT_TIMER).all()
    assert part.state() == orc.state()


def test_gpu_second_timer_in_an_instance_falls_back():
    b = bpmn.createExecutableProcess("process").startEvent("s").parallelGateway("fork").intermediateCatchEvent("t1")
    b.timerWithDuration("PT1H").parallelGateway("join").moveToNode("fork").intermediateCatchEvent("t2")
    b.timerWithDuration("PT2H").connectTo("join")
    part = Partition(max_instances=8, max_commands=8)
    part.deploy(b.endEvent("e").done())
    part.submit(create_commands(4, 0))
    part.run()
    assert part.stats()["fallback"] == 4


@pytest.mark.parametrize("shape", ["timer", "task_timer_task", "timer_in_sub_process"])
def test_gpu_timer_log_and_db_bytes(shape):
    pair = Pair(SHAPES[shape](), 100)
    for e in (pair.part, pair.orc):
        e.set_clock(NOW)
    pair.window(create_commands(100, 0))
    rng = np.random.default_rng(1)
    for step in range(8):
        c = _open_work(pair.part, rng)
        if c is None:
            break
        for e in (pair.part, pair.orc):
            e.set_clock(NOW + 1000 * (step + 1))
        pair.window(c)


@pytest.mark.parametrize("shape", ["task_timer_task", "timer_in_sub_process"])
def test_gpu_timer_restart_equivalence(shape):
    # export -> import into a fresh handle with open timers; both continue like the oracle
    xml = SHAPES[shape]()
    n = 48
    part, orc = drive_timers(xml, n, phases=1)
    fresh = Partition(max_instances=n, max_commands=n, max_records_per_batch=128)
    assert fresh.deploy(xml) == 0
    entries = part.state_db()
    fresh.import_state_db(entries)
    assert fresh.state() == part.state() and fresh.state_db() == entries
    rng = np.random.default_rng(9)
    clock = NOW + 100000
    for _ in range(10):
        c = _open_work(part, rng)
        if c is None:
            break
        clock += 1000
        # the same commands for the fresh handle, by key (an imported instance's ordinals are its own)
        c2 = c.copy()
        for j, cmd in enumerate(c):
            c2[j]["instance"], c2[j]["ref"] = fresh.resolve_key(part_key(part, int(cmd["instance"]), int(cmd["ref"])))
        outs = []
        for p, cc in ((part, c), (fresh, c2)):
            p.set_clock(clock)
            p.submit(cc)
            p.run()
            outs.append(p.drain())
        orc.set_clock(clock)
        orc.clear_records()
        orc.submit(c)
        orc.run()
        want = orc.records()
        timer = want["value_type"] == abi.VT_TIMER
        for got in outs:
            assert len(got) == len(want)
            for f in abi.PARITY_FIELDS:
                if f in ("source_index", "aux"):
                    continue
                assert np.array_equal(got[f], want[f]), f
            assert np.array_equal(got["aux"][timer], want["aux"][timer])  # dueDates
        assert part.state() == orc.state() == fresh.state()
    assert [r for r in fresh.state() if not r.startswith("KEY|")] == []


def part_key(part, inst, ordv):
    """The key of (instance, ordinal) on a handle: the key history through the exported state."""
    for r in part.state():
        if r.startswith("JOBS|") or r.startswith("TIMERS|"):
            k = int(r.split("|")[2] if r.startswith("TIMERS|") else r.split("|")[1])
            if part.resolve_key(k) == (inst, ordv):
                return k
    raise KeyError((inst, ordv))


def test_gpu_activated_jobs_canceled_by_a_boundary_timer(monkeypatch):
    # an interrupting boundary timer fires on ACTIVATED jobs: JOB:CANCELED is the stored job (deadline
    # and worker), in the records, the host serialiser's bytes and the device writer's bytes alike
    from test_gpu_logdev import Log
    monkeypatch.setenv("ZBHIP_DEVICE_ACTIVATIONS", "1")
    xml = (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "type")
           .boundaryEvent("timer").cancelActivity(True).timerWithDuration("PT1M").endEvent("te")
           .moveToActivity("task").endEvent().done())
    pair = Pair(xml, 40)
    log = Log(xml, 40)
    for e in (pair.part, pair.orc, log.part):
        e.set_clock(NOW)
    pair.window(create_commands(40, 0))
    log.window(create_commands(40, 0))
    for e in (pair.part, pair.orc, log.part):
        e.activate_jobs("type", worker="boundary-w", timeout=999, max_jobs=25, timestamp=5)
    rows = [r.split("|") for r in pair.part.state() if r.startswith("TIMERS|")]
    keys = [(int(p[2]), int(dict(kv.split("=") for kv in p[3].split(","))["dueDate"])) for p in rows]
    res = [pair.part.resolve_key(k) for k, _ in keys]
    c = trigger_commands([i for i, _ in res], [o for _, o in res], [d for _, d in keys])
    got = pair.window(c)
    canceled = got[(got["value_type"] == abi.VT_JOB) & (got["intent"] == abi.JOB_CANCELED)]
    assert len(canceled) == 40 and (canceled["message_key"] == 1004).sum() == 25
    log.window(c)
    assert log.declined == 0
