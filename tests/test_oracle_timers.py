"""Timer intermediate catch events on the CPU oracle, pinned by the assertions of
the reference's TimerCatchEventTest (engine/src/test/java/io/camunda/zeebe/engine/processing/timer/
TimerCatchEventTest.java:122-296) with a fixed clock; the static-duration parser (Interval.parse
subset) of oracle and product compiler; and the product's log serializer / zb-db encoder against
the oracle's restatements on the CPU engine's timer records and state."""
import numpy as np
import pytest

from helpers import create_commands
from oracle.oracle import Oracle, OracleError
from test_compiler import Compiled
from test_logserial import Run
from zeebe_amd import abi, bpmn
from zeebe_amd.native import ZbhipError

BASE = 1 << 51
NOW = 1700000000000


def timer_process(duration="PT10S", pid="process"):
    return (bpmn.createExecutableProcess(pid).startEvent("start").intermediateCatchEvent("timer")
            .timerWithDuration(duration).endEvent("end").done())


def trigger_commands(instances, ordinals, dues):
    c = abi.make_commands(len(instances))
    c["instance"] = instances
    c["ref"] = ordinals
    c["kind"] = abi.CMD_TIMER_TRIGGER
    dues = np.asarray(dues, dtype=np.int64)
    c["doc_begin"] = dues & 0xFFFFFFFF
    c["pad"] = dues >> 32
    return c


def _run(o, cmds):
    o.clear_records()
    o.submit(cmds)
    o.run()
    return list(o.records())


def _timer_records(recs):
    return [r for r in recs if r["value_type"] == abi.VT_TIMER]


def _trigger_all(o, recs, instance=0):
    created = [r for r in _timer_records(recs) if r["intent"] == abi.TIMER_CREATED]
    return _run(o, trigger_commands([instance] * len(created), [int(r["key"]) - BASE - 1 for r in created],
                                    [int(r["aux"]) for r in created]))


def test_life_cycle():
    # TimerCatchEventTest.testLifeCycle (:122-155): PT0S; the timer element's PI intents and the
    # timer record sequence (TIMER:TRIGGER is the due-date checker's command, submitted here)
    o = Oracle()
    o.set_clock(NOW)
    o.deploy(timer_process("PT0S", "testLifeCycle"))
    recs = _run(o, create_commands(1, 0))
    recs += _trigger_all(o, recs)
    timer_el = [i for i, e in enumerate(o.process_tables()[0]["elements"]) if e[2] == "timer"][0]
    intents = [abi.PI_INTENTS[int(r["intent"])] for r in recs
               if r["value_type"] == abi.VT_PROCESS_INSTANCE and int(r["element_idx"]) == timer_el]
    assert intents == ["ACTIVATE_ELEMENT", "ELEMENT_ACTIVATING", "ELEMENT_ACTIVATED", "COMPLETE_ELEMENT",
                       "ELEMENT_COMPLETING", "ELEMENT_COMPLETED"]
    assert [abi.TIMER_INTENTS[int(r["intent"])] for r in _timer_records(recs)] == ["CREATED", "TRIGGERED"]
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


def test_should_create_timer():
    # TimerCatchEventTest.shouldCreateTimer (:157-193): elementInstanceKey = the ACTIVATED timer
    # element's key, processInstanceKey, dueDate = clock + 10 s (fixed clock: exactly)
    o = Oracle()
    o.set_clock(NOW)
    o.deploy(timer_process("PT10S"))
    recs = _run(o, create_commands(1, 0))
    activated = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == 3
                 and o.element_id(0, int(r["element_idx"])) == "timer"][0]
    created = _timer_records(recs)[0]
    assert int(created["scope_key"]) == int(activated["key"])
    assert int(created["process_instance_key"]) == BASE + 1
    assert int(created["aux"]) == NOW + 10000
    st = o.state()
    assert "TIMER_DUE_DATES|%d|%d|%d" % (NOW + 10000, int(activated["key"]), int(created["key"])) in st
    assert "EVENT_SCOPE|%d|accepting=1,interrupted=0,interrupting=timer,boundaryElementIds=" % int(activated["key"]) in st


def test_should_trigger_and_complete_timer_event():
    # shouldTriggerTimer (:233-264): TRIGGERED key and value equal CREATED's; shouldCompleteTimerEvent
    # (:266-296): the timer element's COMPLETED key equals its ACTIVATED key
    o = Oracle()
    o.set_clock(NOW)
    o.deploy(timer_process("PT1M"))
    recs = _run(o, create_commands(1, 0))
    created = _timer_records(recs)[0]
    o.set_clock(NOW + 60000)
    recs2 = _trigger_all(o, recs)
    triggered = _timer_records(recs2)[0]
    assert abi.TIMER_INTENTS[int(triggered["intent"])] == "TRIGGERED"
    for f in ("key", "scope_key", "process_instance_key", "aux", "element_idx", "process_idx"):
        assert triggered[f] == created[f], f
    act = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == 3
           and o.element_id(0, int(r["element_idx"])) == "timer"][0]
    done = [r for r in recs2 if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == 5
            and o.element_id(0, int(r["element_idx"])) == "timer"][0]
    assert int(done["key"]) == int(act["key"]) and int(done["scope_key"]) == int(act["scope_key"])
    # a second trigger of the same timer: NOT_FOUND (TriggerTimerProcessor.java:86-90)
    again = _run(o, trigger_commands([0], [int(created["key"]) - BASE - 1], [int(created["aux"])]))
    assert len(again) == 1 and again[0]["record_type"] == abi.RT_REJECTION
    assert again[0]["rejection_type"] == abi.REJ_NOT_FOUND
    assert o.reason(0) == "Expected to trigger timer with key '%d', but no such timer was found" % int(created["key"])


@pytest.mark.parametrize("text,ms", [("PT10S", 10000), ("PT1M30.5S", 90500), ("P0DT2H", 7200000), ("PT0S", 0),
                                     ("PT0.001S", 1), (" PT2H3M ", 7380000), ("PT48H", 172800000)])
def test_static_durations(text, ms):
    o = Oracle()
    o.set_clock(NOW)
    o.deploy(timer_process(text))
    assert int(_timer_records(_run(o, create_commands(1, 0)))[0]["aux"]) == NOW + ms
    c = Compiled(timer_process(text))
    assert int(c.els[[c.id(i) for i in range(len(c.els))].index("timer")]["duration_ms"]) == ms


# constant FEEL expressions (ExpressionProcessor.evaluateIntervalExpression): a day-time duration is a
# java.time.Duration -- days of 24 h (new Interval(duration)), unlike the calendar days of the string
# form; a string goes through Interval.parse.  BoundaryEventTest.java:54 uses duration("PT0.1S").
@pytest.mark.parametrize("text,ms", [('=duration("PT0.1S")', 100), ('= duration( "PT2M" )', 120000),
                                     ('=duration("P1D")', 86400000), ('=duration("P1DT1H")', 90000000),
                                     ('="PT5S"', 5000)])
def test_constant_feel_durations(text, ms):
    test_static_durations(text, ms)


# days are a Period (Interval.isCalendarBased): added in the broker's system zone, so a DST change
# moves the due date -- refused rather than assuming a UTC zone
@pytest.mark.parametrize("text", ["P1Y", "P1M", "P1W", "PT-1S", "PT", "R3/PT1S", "P60D", "P1DT2H", "P2D",
                                  "=timeout", "=duration(d)", '=duration("P1M")', '="P1D"', '=date("2020-01-01")'])
def test_durations_outside_the_subset_are_refused(text):
    with pytest.raises(ZbhipError):
        Compiled(timer_process(text))
    with pytest.raises(OracleError):
        Oracle().deploy(timer_process(text))


def test_product_serializer_and_state_encoder_on_timer_records():
    # the product's host log serializer and zb-db encoder (+ decoder) over the CPU engine's timer
    # windows equal the oracle restatements (oracle/logserial.py, oracle/statedb.py) byte for byte:
    # TIMER:CREATED / TRIGGERED values, a NOT_FOUND rejection, TIMERS and TIMER_DUE_DATES rows
    from oracle import statedb as SD
    from test_statedb import _check_state
    run = Run([timer_process("PT30S"), bpmn.createExecutableProcess("p2").startEvent("s").serviceTask("t", "t")
               .intermediateCatchEvent("wait").timerWithDuration("PT5M").endEvent("e").done()])
    run.orc.set_clock(NOW)
    cmds = create_commands(6, 0)
    cmds["ref"] = [0, 1, 0, 1, 0, 1]
    recs = run.window(cmds)
    encoded = _check_state(run)
    assert {SD.CF["TIMERS"], SD.CF["TIMER_DUE_DATES"]} <= encoded
    entries = run.ser.encode_state_rows(run.orc.state())
    assert sorted(run.ser.decode_state_entries(entries)) == sorted(
        r for r in run.orc.state() if r.split("|")[0] in SD.CF)
    # complete the jobs of the p2 instances (their timers start), then trigger every timer
    jobs = [r for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    insts = [int(r["source_index"]) for r in jobs]  # CREATE i went into instance slot i
    c = abi.make_commands(len(jobs))
    c["instance"] = insts
    c["ref"] = [_ord(run.orc, i, int(r["key"])) for i, r in zip(insts, jobs)]
    c["kind"] = abi.CMD_JOB_COMPLETE
    run.window(c)
    _check_state(run)
    timers = {}
    for row in run.orc.state():
        if row.startswith("TIMERS|"):
            parts = row.split("|")
            f = dict(kv.split("=") for kv in parts[3].split(","))
            timers[int(parts[2])] = (int(f["processInstanceKey"]), int(f["dueDate"]))
    assert len(timers) == 6
    pis = {pk: i for i, pk in enumerate(sorted({v[0] for v in timers.values()}))}  # slot i: PI key order
    keys = sorted(timers)
    cmds = trigger_commands([pis[timers[k][0]] for k in keys], [_ord(run.orc, pis[timers[k][0]], k) for k in keys],
                            [timers[k][1] for k in keys])
    run.orc.set_clock(NOW + 300000)
    recs = run.window(np.concatenate([cmds, cmds[:1]]))  # the last one: already triggered -> NOT_FOUND
    assert recs[-1]["record_type"] == abi.RT_REJECTION and recs[-1]["value_type"] == abi.VT_TIMER
    _check_state(run)
    assert [r for r in run.orc.state() if r.startswith("TIMER")] == []


def _ord(o, instance, key):
    """The ordinal of `key` among the instance's keys (the oracle's per-instance key history)."""
    for i in range(64):
        if o.resolve(instance, i) == key:
            return i
    raise KeyError(key)


def boundary_process(cycle=None, duration=None, interrupting=False):
    b = (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "type")
         .boundaryEvent("event").cancelActivity(interrupting))
    b = b.timerWithCycleExpression(cycle) if cycle else b.timerWithDurationExpression(duration)
    return b.endEvent().moveToActivity("task").endEvent().done()


# BoundaryEventTest.java:48-69's constant expressions: a duration("PT0.1S") interrupting timer and a
# cycle(duration("PT1S")) non-interrupting one (FeelFunctionProvider.cycle -> "R/PT1S": infinite);
# cycle(3, ...) -> "R3/..."
@pytest.mark.parametrize("cycle,duration,interrupting,ms,reps", [
    (None, 'duration("PT0.1S")', True, 100, 1),
    ('cycle(duration("PT1S"))', None, False, 1000, -1),
    ('cycle(3, duration("PT2S"))', None, False, 2000, 3),
    ('"R2/PT3S"', None, False, 3000, 2),
])
def test_constant_feel_boundary_timers(cycle, duration, interrupting, ms, reps):
    xml = boundary_process(cycle, duration, interrupting)
    o = Oracle()
    o.set_clock(NOW)
    o.deploy(xml)
    created = [r for r in _timer_records(_run(o, create_commands(1, 0))) if r["intent"] == abi.TIMER_CREATED]
    assert len(created) == 1 and int(created[0]["aux"]) == NOW + ms and int(created[0]["partition"]) == reps
    c = Compiled(xml)
    e = c.els[[c.id(i) for i in range(len(c.els))].index("event")]
    assert int(e["duration_ms"]) == ms and int(e["job_retries"]) >> 8 == (255 if reps == -1 else reps)


@pytest.mark.parametrize("cycle", ['cycle(x)', 'cycle(0, duration("PT1S"))', 'cycle(duration(d))', '"PT1S"'])
def test_feel_cycles_outside_the_subset(cycle):
    with pytest.raises(ZbhipError):
        Compiled(boundary_process(cycle))
    with pytest.raises(OracleError):
        Oracle().deploy(boundary_process(cycle))
