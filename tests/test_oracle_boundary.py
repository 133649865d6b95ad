"""Interrupting timer boundary events on job worker tasks on the CPU oracle,
pinned by the reference's BoundaryEventTest (engine/src/test/java/io/camunda/zeebe/engine/processing/
bpmn/boundary/BoundaryEventTest.java:48-139) and ActivityTest (processing/bpmn/activity/ActivityTest.java:
150-199, 260-280; its WITH_BOUNDARY_EVENTS model has two timers on one task, the device subset one --
the assertions are the same per timer); the model subset shared by oracle and product compiler; the
product's log serializer and zb-db encoder against the oracle restatements on boundary windows."""
import numpy as np
import pytest

from helpers import create_commands
from oracle.oracle import Oracle, OracleError
from test_compiler import Compiled
from test_logserial import Run
from test_oracle_timers import BASE, NOW, _run, trigger_commands
from zeebe_amd import abi, bpmn
from zeebe_amd.native import ZbhipError


def multiple_sequence_flows(duration="PT0.1S", job_type="type"):
    """BoundaryEventTest.MULTIPLE_SEQUENCE_FLOWS (:48-60) with the static duration its expression
    evaluates to: the boundary timer leaves through two flows, the task through one."""
    return (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", job_type).boundaryEvent("timer")
            .cancelActivity(True).timerWithDuration(duration).endEvent("end1").moveToNode("timer").endEvent("end2")
            .moveToActivity("task").endEvent("taskEnd").done())


def with_boundary_event():
    """ActivityTest.WITH_BOUNDARY_EVENTS (:49-61) with its first timer."""
    return (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "type").boundaryEvent("timer1")
            .timerWithDuration("PT10S").endEvent().moveToActivity("task").endEvent("taskEnd").done())


def non_interrupting_process(duration="PT1S"):
    """BoundaryEventTest.NON_INTERRUPTING_PROCESS (:61-69) with a static timeDuration in place of
    its cycle expression (one trigger, no reschedule)."""
    return (bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "type").boundaryEvent("event")
            .cancelActivity(False).timerWithDuration(duration).endEvent("eventEnd").moveToActivity("task")
            .endEvent("taskEnd").done())


def _eid(o, r):
    e = int(r["element_idx"])
    return o.element_id(0, e) if e >= 0 else None


def _tuple(o, r):
    return abi.VALUE_TYPES.get(int(r["value_type"]), int(r["value_type"])), \
        abi.intent_name(int(r["value_type"]), int(r["intent"])), _eid(o, r)


def _between(o, recs, start, stop):
    """RecordingExporter.records().between(task `start`, task `stop`) as (value type, intent, element)."""
    out, on = [], False
    for r in recs:
        t = _tuple(o, r)
        if t == ("PROCESS_INSTANCE", start, "task"):
            on = True
        if on:
            out.append(t)
        if on and t == ("PROCESS_INSTANCE", stop, "task"):
            break
    return out


def _trigger_all(o, recs):
    created = [r for r in recs if r["value_type"] == abi.VT_TIMER and r["intent"] == abi.TIMER_CREATED]
    return _run(o, trigger_commands([0] * len(created), [int(r["key"]) - BASE - 1 for r in created],
                                    [int(r["aux"]) for r in created]))


def _complete_jobs(o, recs):
    jobs = [r for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    c = abi.make_commands(len(jobs))
    c["kind"] = abi.CMD_JOB_COMPLETE
    c["ref"] = [int(r["key"]) - BASE - 1 for r in jobs]
    return _run(o, c)


def _started(xml):
    o = Oracle()
    o.set_clock(NOW)
    o.deploy(xml)
    return o, _run(o, create_commands(1, 0))


def test_subscribe_on_activation():
    # ActivityTest.shouldSubscribeToBoundaryEventTriggersOnReady (:150-180): the boundary timer is
    # created between the task's ACTIVATING and ACTIVATED, before the job
    o, recs = _started(with_boundary_event())
    assert [t[1] for t in _between(o, recs, "ELEMENT_ACTIVATING", "ELEMENT_ACTIVATED")] == [
        "ELEMENT_ACTIVATING", "CREATED", "CREATED", "ELEMENT_ACTIVATED"]
    seq = _between(o, recs, "ELEMENT_ACTIVATING", "ELEMENT_ACTIVATED")
    assert seq[1] == ("TIMER", "CREATED", "timer1") and seq[2] == ("JOB", "CREATED", "task")
    timer = [r for r in recs if r["value_type"] == abi.VT_TIMER][0]
    assert int(timer["aux"]) == NOW + 10000
    task_key = [r for r in recs if _tuple(o, r) == ("PROCESS_INSTANCE", "ELEMENT_ACTIVATED", "task")][0]["key"]
    assert int(timer["scope_key"]) == int(task_key)  # elementInstanceKey = the activity's instance
    st = o.state()
    assert "EVENT_SCOPE|%d|accepting=1,interrupted=0,interrupting=timer1,boundaryElementIds=timer1" % int(task_key) in st
    assert any(r.startswith("TIMERS|%d|" % int(task_key)) and "handlerNodeId=timer1" in r for r in st)


def test_unsubscribe_on_completing():
    # ActivityTest.shouldUnsubscribeFromBoundaryEventTriggersOnCompleting (:184-199, :260-280):
    # TIMER:CANCELED between the task's COMPLETING and COMPLETED, with the timer's key and value
    o, recs = _started(with_boundary_event())
    created = [r for r in recs if r["value_type"] == abi.VT_TIMER][0]
    done = _complete_jobs(o, recs)
    seq = _between(o, done, "ELEMENT_COMPLETING", "ELEMENT_COMPLETED")
    assert seq[0][1] == "ELEMENT_COMPLETING" and seq[-1][1] == "ELEMENT_COMPLETED"
    assert ("TIMER", "CANCELED", "timer1") in seq
    canceled = [r for r in done if r["value_type"] == abi.VT_TIMER][0]
    for f in ("key", "scope_key", "process_instance_key", "aux", "element_idx"):
        assert canceled[f] == created[f], f
    assert [r for r in o.state() if not r.startswith("KEY|")] == []
    # the canceled timer can no longer be triggered (TriggerTimerProcessor.java:86-90)
    again = _run(o, trigger_commands([0], [int(created["key"]) - BASE - 1], [int(created["aux"])]))
    assert len(again) == 1 and again[0]["record_type"] == abi.RT_REJECTION
    assert again[0]["rejection_type"] == abi.REJ_NOT_FOUND


def test_activate_boundary_event_when_triggered():
    # BoundaryEventTest.shouldActivateBoundaryEventWhenEventTriggered (:100-139): containsSubsequence
    # TIMER TRIGGERED, task ELEMENT_TERMINATING, JOB CANCELED, task ELEMENT_TERMINATED, timer ACTIVATING
    o, recs = _started(multiple_sequence_flows())
    fired = _trigger_all(o, recs)
    seq = [_tuple(o, r) for r in fired]
    want = [("TIMER", "TRIGGERED", "timer"), ("PROCESS_INSTANCE", "ELEMENT_TERMINATING", "task"),
            ("JOB", "CANCELED", "task"), ("PROCESS_INSTANCE", "ELEMENT_TERMINATED", "task"),
            ("PROCESS_INSTANCE", "ELEMENT_ACTIVATING", "timer")]
    it = iter(seq)
    assert all(w in it for w in want), seq
    # the full batch head (EventHandle.activateElement, JobWorkerTaskProcessor.onTerminate,
    # EventTriggerBehavior.activateTriggeredEvent)
    assert seq[:10] == [
        ("TIMER", "TRIGGERED", "timer"), ("PROCESS_EVENT", "TRIGGERING", "timer"),
        ("PROCESS_INSTANCE", "TERMINATE_ELEMENT", "task"), ("PROCESS_INSTANCE", "ELEMENT_TERMINATING", "task"),
        ("JOB", "CANCELED", "task"), ("PROCESS_INSTANCE", "ELEMENT_TERMINATED", "task"),
        ("PROCESS_EVENT", "TRIGGERED", "timer"), ("PROCESS_INSTANCE", "ELEMENT_ACTIVATING", "timer"),
        ("PROCESS_INSTANCE", "ELEMENT_ACTIVATED", "timer"), ("PROCESS_INSTANCE", "COMPLETE_ELEMENT", "timer")]
    pe = [r for r in fired if r["value_type"] == abi.VT_PROCESS_EVENT]
    assert pe[0]["key"] == pe[1]["key"]  # TRIGGERED under the trigger's key
    task = [r for r in fired if _tuple(o, r)[2] == "task" and r["value_type"] == abi.VT_PROCESS_INSTANCE][0]
    act = [r for r in fired if _tuple(o, r) == ("PROCESS_INSTANCE", "ELEMENT_ACTIVATING", "timer")][0]
    assert int(act["scope_key"]) == int(task["scope_key"])  # the boundary event's flow scope: the task's
    assert int(act["key"]) > int(pe[0]["key"])


def test_take_all_outgoing_sequence_flows_if_triggered():
    # BoundaryEventTest.shouldTakeAllOutgoingSequenceFlowsIfTriggered (:75-98)
    o, recs = _started(multiple_sequence_flows())
    fired = _trigger_all(o, recs)
    ends = [_eid(o, r) for r in fired if r["value_type"] == abi.VT_PROCESS_INSTANCE and
            abi.PI_INTENTS[int(r["intent"])] == "ELEMENT_COMPLETED" and _eid(o, r) in ("end1", "end2", "taskEnd")]
    assert sorted(ends) == ["end1", "end2"]
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


def test_non_interrupting_boundary_keeps_the_activity():
    # BoundaryEventTest.shouldNotTerminateActivityForNonInterruptingBoundaryEvents (:274-313): the
    # subsequence TIMER TRIGGERED ... JOB COMPLETED, task COMPLETING, task COMPLETED (its cycle's
    # re-created timer and the CANCELED of it do not occur for a duration); the boundary event's
    # path runs while the task stays ACTIVATED (EventHandle.activateElement, not interrupting)
    o, recs = _started(non_interrupting_process())
    task_key = [r for r in recs if _tuple(o, r) == ("PROCESS_INSTANCE", "ELEMENT_ACTIVATED", "task")][0]["key"]
    st = o.state()
    assert "EVENT_SCOPE|%d|accepting=1,interrupted=0,interrupting=,boundaryElementIds=event" % int(task_key) in st
    fired = _trigger_all(o, recs)
    seq = [_tuple(o, r) for r in fired]
    assert seq[:7] == [
        ("TIMER", "TRIGGERED", "event"), ("PROCESS_EVENT", "TRIGGERING", "event"),
        ("PROCESS_EVENT", "TRIGGERED", "event"), ("PROCESS_INSTANCE", "ELEMENT_ACTIVATING", "event"),
        ("PROCESS_INSTANCE", "ELEMENT_ACTIVATED", "event"), ("PROCESS_INSTANCE", "COMPLETE_ELEMENT", "event"),
        ("PROCESS_INSTANCE", "ELEMENT_COMPLETING", "event")]
    assert not any(t[1].startswith(("TERMINATE", "ELEMENT_TERMINAT")) or t[1] == "CANCELED" for t in seq)
    assert ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "eventEnd") in seq
    assert any(r.startswith("ELEMENT_INSTANCE_KEY|%d|" % int(task_key)) and "state=3" in r for r in o.state())
    done = _complete_jobs(o, recs)
    it = iter([_tuple(o, r) for r in recs + fired + done])
    want = [("TIMER", "TRIGGERED", "event"), ("JOB", "COMPLETED", "task"),
            ("PROCESS_INSTANCE", "ELEMENT_COMPLETING", "task"), ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "task")]
    assert all(w in it for w in want)
    assert not any(_tuple(o, r) == ("TIMER", "CANCELED", "event") for r in done)
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


def test_job_of_a_terminated_task_is_not_found():
    o, recs = _started(multiple_sequence_flows())
    _trigger_all(o, recs)
    rej = _complete_jobs(o, recs)
    assert len(rej) == 1 and rej[0]["record_type"] == abi.RT_REJECTION
    assert rej[0]["rejection_type"] == abi.REJ_NOT_FOUND


def test_boundary_in_sub_process_and_parallel_branch():
    # the timer-or-job race inside a sub-process, next to a plain job in a parallel branch
    b = bpmn.createExecutableProcess("process").startEvent().parallelGateway("fork").subProcess("sub").startEvent()
    b.serviceTask("inner", "inner").boundaryEvent("late").timerWithDuration("PT1M").endEvent("lateEnd")
    b.moveToActivity("inner").endEvent().subProcessDone().parallelGateway("join").moveToNode("fork")
    b.serviceTask("other", "other").connectTo("join")
    o, recs = _started(b.endEvent("e").done())
    fired = _trigger_all(o, recs)
    assert ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "late") in [_tuple(o, r) for r in fired]
    _complete_jobs(o, recs)  # inner: NOT_FOUND; other: completes the join
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


def _boundary_model(attrs="", body=None, on="serviceTask"):
    body = body if body is not None else ('<timerEventDefinition id="t"><timeDuration>PT1S</timeDuration>'
                                          '</timerEventDefinition>')
    task = ('<serviceTask id="a"><extensionElements><zeebe:taskDefinition type="a"/></extensionElements></serviceTask>'
            if on == "serviceTask" else '<task id="a"/>')
    return ('<?xml version="1.0" encoding="UTF-8"?><definitions xmlns="http://www.omg.org/spec/BPMN/20100524/MODEL" '
            'xmlns:zeebe="http://camunda.org/schema/zeebe/1.0" id="d" targetNamespace="x"><process id="p" '
            'isExecutable="true"><startEvent id="s"/>%s<sequenceFlow id="f1" sourceRef="s" targetRef="a"/>'
            '<boundaryEvent id="b" attachedToRef="a"%s>%s</boundaryEvent><endEvent id="e"/>'
            '<sequenceFlow id="f2" sourceRef="b" targetRef="e"/></process></definitions>' % (task, attrs, body))


def test_boundary_model_subset():
    for xml in (_boundary_model(), _boundary_model(' cancelActivity="false"'), multiple_sequence_flows(),
                with_boundary_event(), non_interrupting_process()):
        Compiled(xml)
        Oracle().deploy(xml)
    # (an interrupting timeCycle is accepted since round 6: test_interrupting_cycle_reschedules_then_cancels)
    Compiled(_boundary_model(body='<timerEventDefinition id="t"><timeCycle>R3/PT1S</timeCycle></timerEventDefinition>'))
    refused = [_boundary_model(body='<messageEventDefinition id="m" messageRef="x"/>'),
               _boundary_model(on="task"),
               (bpmn.createExecutableProcess("p").startEvent().serviceTask("a", "a").boundaryEvent("b1")
                .timerWithDuration("PT1S").endEvent().moveToActivity("a").boundaryEvent("b2").timerWithDuration("PT2S")
                .endEvent().moveToActivity("a").endEvent().done())]
    for xml in refused:
        with pytest.raises(ZbhipError):
            Compiled(xml)
        with pytest.raises(OracleError):
            Oracle().deploy(xml)
    c = Compiled(multiple_sequence_flows("PT2M"))
    ids = [c.id(i) for i in range(len(c.els))]
    task, timer = ids.index("task"), ids.index("timer")
    assert int(c.els[timer]["element_type"]) == abi.ELEMENT_TYPES.index("BOUNDARY_EVENT")
    assert int(c.els[timer]["flow_source"]) == task and int(c.els[task]["start_event"]) == timer
    # job_retries of a boundary event: interrupting | repetitions << 8
    assert int(c.els[timer]["duration_ms"]) == 120000 and int(c.els[timer]["job_retries"]) == 1 | (1 << 8)
    c = Compiled(non_interrupting_process())
    ids = [c.id(i) for i in range(len(c.els))]
    assert int(c.els[ids.index("event")]["job_retries"]) == 0 | (1 << 8)  # cancelActivity="false"
    for cycle, reps in (("R/PT1S", 255), ("R3/PT2M", 3), ("R254/PT1S", 254)):
        c = Compiled(_boundary_model(' cancelActivity="false"', _cycle(cycle)))
        ids = [c.id(i) for i in range(len(c.els))]
        assert int(c.els[ids.index("b")]["job_retries"]) == reps << 8, cycle
        Oracle().deploy(_boundary_model(' cancelActivity="false"', _cycle(cycle)))
    for xml in (_boundary_model(' cancelActivity="false"', _cycle("R0/PT1S")),
                _boundary_model(' cancelActivity="false"', _cycle("R255/PT1S")),
                _boundary_model(' cancelActivity="false"', _cycle("R/2024-01-01T00:00:00Z/PT1S"))):
        with pytest.raises(ZbhipError):
            Compiled(xml)
        with pytest.raises(OracleError):
            Oracle().deploy(xml)


def _cycle(text):
    return '<timerEventDefinition id="t"><timeCycle>%s</timeCycle></timerEventDefinition>' % text


def cycle_process(cycle="R/PT1S"):
    """BoundaryEventTest.NON_INTERRUPTING_PROCESS (:61-69) with the static cycle its
    `cycle(duration("PT1S"))` expression evaluates to (R/PT1S: infinite repetitions)."""
    b = bpmn.createExecutableProcess("process").startEvent().serviceTask("task", "type").boundaryEvent("event")
    b.cancelActivity(False).timerWithCycle(cycle).endEvent("eventEnd").moveToActivity("task")
    return b.endEvent("taskEnd").done()


def test_non_interrupting_cycle_reschedules():
    # BoundaryEventTest.shouldNotTerminateActivityForNonInterruptingBoundaryEvents (:274-313), exactly:
    # TIMER TRIGGERED, TIMER CREATED (the cycle's next), JOB COMPLETED, task COMPLETING,
    # TIMER CANCELED, task COMPLETED
    o, recs = _started(cycle_process())
    created = [r for r in recs if r["value_type"] == abi.VT_TIMER][0]
    assert int(created["partition"]) == -1  # TimerRecord.repetitions: RepeatingInterval.INFINITE
    fired = _trigger_all(o, recs)
    timers = [r for r in fired if r["value_type"] == abi.VT_TIMER]
    assert [abi.TIMER_INTENTS[int(r["intent"])] for r in timers] == ["TRIGGERED", "CREATED"]
    nxt = timers[1]
    assert int(nxt["aux"]) == int(created["aux"]) + 1000 and int(nxt["key"]) > int(created["key"])
    assert int(nxt["scope_key"]) == int(created["scope_key"]) and int(nxt["partition"]) == -1
    # the rescheduled CREATED follows the boundary event's activation (TriggerTimerProcessor.java:109-116)
    seq = [_tuple(o, r) for r in fired]
    assert seq.index(("TIMER", "CREATED", "event")) > seq.index(("PROCESS_INSTANCE", "COMPLETE_ELEMENT", "event"))
    done = _complete_jobs(o, recs)
    it = iter([_tuple(o, r) for r in recs + fired + done])
    want = [("TIMER", "TRIGGERED", "event"), ("TIMER", "CREATED", "event"), ("JOB", "COMPLETED", "task"),
            ("PROCESS_INSTANCE", "ELEMENT_COMPLETING", "task"), ("TIMER", "CANCELED", "event"),
            ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "task")]
    assert all(w in it for w in want)
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


@pytest.mark.parametrize("late_ms,next_due", [(0, NOW + 2000), (999, NOW + 2000), (1000, NOW + 1000 + 1000 + 1000),
                                              (2500, NOW + 1000 + 2500 + 1000)])
def test_late_cycle_trigger_counts_from_the_clock(late_ms, next_due):
    # TriggerTimerProcessor.refreshTimer (:161-175): Interval.withStart(dueDate) starts at dueDate +
    # interval; subscribeToTimerEvent takes Interval.toEpochMilli(now) (Interval.java:77-93), which is
    # that start unless start <= now, then now + interval -- a trigger processed a period or more late
    # does not schedule a dueDate in the past
    o, recs = _started(cycle_process("R/PT1S"))
    created = [r for r in recs if r["value_type"] == abi.VT_TIMER][0]
    assert int(created["aux"]) == NOW + 1000
    o.set_clock(NOW + 1000 + late_ms)
    fired = _trigger_all(o, recs)
    nxt = [r for r in fired if r["value_type"] == abi.VT_TIMER and r["intent"] == abi.TIMER_CREATED][0]
    assert int(nxt["aux"]) == next_due
    assert any(r.startswith("TIMER_DUE_DATES|%d|" % next_due) for r in o.state())


def test_cycle_with_repetitions_stops():
    # R3: three triggers (repetitions 3, 2, 1 in the records), then no timer is left
    o, recs = _started(cycle_process("R3/PT10S"))
    seen = []
    for _ in range(4):
        open_timers = [r for r in o.state() if r.startswith("TIMERS|")]
        if not open_timers:
            break
        created = [r for r in recs if r["value_type"] == abi.VT_TIMER and r["intent"] == abi.TIMER_CREATED][-1:]
        fired = _trigger_all(o, created)
        seen += [(abi.TIMER_INTENTS[int(r["intent"])], int(r["partition"])) for r in fired
                 if r["value_type"] == abi.VT_TIMER]
        recs = fired
    assert seen == [("TRIGGERED", 3), ("CREATED", 2), ("TRIGGERED", 2), ("CREATED", 1), ("TRIGGERED", 1)]
    assert any(r.startswith("JOBS|") for r in o.state())  # the activity is still waiting


def test_product_serializer_and_state_encoder_on_boundary_records():
    # the product's host log serializer and zb-db encoder (+ decoder) over the CPU engine's boundary
    # windows equal the oracle restatements byte for byte: TIMER:CREATED / CANCELED / TRIGGERED,
    # JOB:CANCELED, PROCESS_EVENT:TRIGGERED, TERMINATE_ELEMENT / ELEMENT_TERMINATING / TERMINATED,
    # EVENT_SCOPE rows with boundary ids
    from oracle import statedb as SD
    from test_statedb import _check_state
    run = Run([multiple_sequence_flows("PT30S")])
    run.orc.set_clock(NOW)
    recs = run.window(create_commands(6, 0))
    encoded = _check_state(run)
    assert {SD.CF["TIMERS"], SD.CF["EVENT_SCOPE"]} <= encoded
    entries = run.ser.encode_state_rows(run.orc.state())
    assert sorted(run.ser.decode_state_entries(entries)) == sorted(
        r for r in run.orc.state() if r.split("|")[0] in SD.CF)
    # instances 0..2: the job completes (TIMER:CANCELED); 3..5: the timer fires (termination)
    jobs = [r for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    timers = [r for r in recs if r["value_type"] == abi.VT_TIMER and r["intent"] == abi.TIMER_CREATED]
    c = abi.make_commands(6)
    for i in range(6):
        c[i]["instance"] = i
        if i < 3:
            c[i]["kind"], c[i]["ref"] = abi.CMD_JOB_COMPLETE, _ord(run.orc, i, int(jobs[i]["key"]))
        else:
            due = int(timers[i]["aux"])
            c[i]["kind"], c[i]["ref"] = abi.CMD_TIMER_TRIGGER, _ord(run.orc, i, int(timers[i]["key"]))
            c[i]["doc_begin"], c[i]["pad"] = due & 0xFFFFFFFF, due >> 32
    run.orc.set_clock(NOW + 30000)
    out = run.window(c)
    kinds = {(int(r["value_type"]), int(r["intent"])) for r in out}
    assert {(abi.VT_TIMER, abi.TIMER_CANCELED), (abi.VT_JOB, abi.JOB_CANCELED),
            (abi.VT_PROCESS_EVENT, abi.PE_TRIGGERED)} <= kinds
    _check_state(run)
    assert [r for r in run.orc.state() if not r.startswith("KEY|")] == []


def _ord(o, instance, key):
    for i in range(64):
        if o.resolve(instance, i) == key:
            return i
    raise KeyError(key)


def sub_process_boundary(interrupting=True, duration="PT1S"):
    """BoundaryEventTest.shouldTerminateSubProcessBeforeTriggeringBoundaryEvent (:218-273): a timer
    boundary event on an embedded sub-process holding a service task."""
    b = bpmn.createExecutableProcess("process").startEvent().subProcess("sub").startEvent("subStart")
    b.serviceTask("task", "type").endEvent("subEnd").subProcessDone()
    b.boundaryEvent("timer").cancelActivity(interrupting).timerWithDuration(duration).endEvent("endTimer")
    return b.moveToActivity("sub").endEvent("end").done()


def test_terminate_sub_process_before_triggering_boundary_event():
    # the golden tail of BoundaryEventTest.shouldTerminateSubProcessBeforeTriggeringBoundaryEvent: the
    # timer (subscribed when the sub-process's start event completes) terminates the sub-process --
    # PROCESS_INSTANCE_BATCH:TERMINATE of its children, the task's job canceled -- then the boundary event
    o, recs = _started(sub_process_boundary())
    created = [r for r in recs if r["value_type"] == abi.VT_TIMER and r["intent"] == abi.TIMER_CREATED]
    assert len(created) == 1 and _eid(o, created[0]) == "timer"
    out = _trigger_all(o, recs)
    want = [("TIMER", "TRIGGERED", "timer"), ("PROCESS_EVENT", "TRIGGERING", "timer"),
            ("PROCESS_INSTANCE", "TERMINATE_ELEMENT", "sub"), ("PROCESS_INSTANCE", "ELEMENT_TERMINATING", "sub"),
            ("PROCESS_INSTANCE_BATCH", "TERMINATE", "sub"), ("PROCESS_INSTANCE", "TERMINATE_ELEMENT", "task"),
            ("PROCESS_INSTANCE", "ELEMENT_TERMINATING", "task"), ("JOB", "CANCELED", "task"),
            ("PROCESS_INSTANCE", "ELEMENT_TERMINATED", "task"), ("PROCESS_INSTANCE", "ELEMENT_TERMINATED", "sub"),
            ("PROCESS_EVENT", "TRIGGERED", "timer"), ("PROCESS_INSTANCE", "ELEMENT_ACTIVATING", "timer"),
            ("PROCESS_INSTANCE", "ELEMENT_ACTIVATED", "timer"), ("PROCESS_INSTANCE", "COMPLETE_ELEMENT", "timer"),
            ("PROCESS_INSTANCE", "ELEMENT_COMPLETING", "timer"), ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "timer")]
    got = [_tuple(o, r) for r in out]
    end = got.index(("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "timer")) + 1
    assert got[end - len(want):end] == want
    assert got[-1] == ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "process")
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


def test_sub_process_boundary_timer_cancelled_on_completion():
    # SubProcessProcessor.onComplete: unsubscribeFromEvents -- the job completes, the sub-process
    # completes and its boundary timer is canceled (TIMER:CANCELED before ELEMENT_COMPLETED of sub)
    o, recs = _started(sub_process_boundary())
    out = _complete_jobs(o, recs)
    got = [_tuple(o, r) for r in out]
    i = got.index(("TIMER", "CANCELED", "timer"))
    assert got[i - 1] == ("PROCESS_INSTANCE", "ELEMENT_COMPLETING", "sub")
    assert got[i + 1] == ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "sub")
    assert got[-1] == ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "process")
    assert [r for r in o.state() if not r.startswith("KEY|")] == []


def test_non_interrupting_sub_process_boundary_keeps_the_sub_process():
    o, recs = _started(sub_process_boundary(False))
    out = _trigger_all(o, recs)
    got = [_tuple(o, r) for r in out]
    assert ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "endTimer") in got
    assert not any(t[1] in ("TERMINATE_ELEMENT", "ELEMENT_TERMINATING") for t in got)
    st = o.state()
    assert any("elementId=task" in r for r in st if r.startswith("ELEMENT_INSTANCE_KEY"))
    out = _complete_jobs(o, recs)
    assert _tuple(o, out[-1]) == ("PROCESS_INSTANCE", "ELEMENT_COMPLETED", "process")


def test_multi_instance_body_terminated_with_its_sub_process():
    # MultiInstanceActivityTest.shouldTerminateInstancesOnTerminatingBody (:584-620)'s subsequence --
    # body TERMINATING, the open inner instance TERMINATING / TERMINATED, body TERMINATED -- with the
    # body terminated by its flow scope: a sub-process around the multi-instance task whose timer
    # boundary event fires after all but one inner job completed (MultiInstanceBodyProcessor.onTerminate
    # :116-125, onChildTerminated :240-253, terminate :282-315; SubProcessProcessor.onChildTerminated)
    b = bpmn.createExecutableProcess("process").startEvent("start").subProcess("sub").startEvent("ss")
    b.serviceTask("task", "task")
    b.multiInstance("= [1, 2, 3]", "item", False)
    b.endEvent("se").subProcessDone().boundaryEvent("late").timerWithDuration("PT10S")
    b.sequenceFlowId("to-canceled").endEvent("canceled")
    xml = b.moveToActivity("sub").endEvent("end").done()
    o, recs = _started(xml)
    jobs = [r for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    assert len(jobs) == 3
    c = abi.make_commands(2)
    c["kind"] = abi.CMD_JOB_COMPLETE
    c["ref"] = [int(r["key"]) - BASE - 1 for r in jobs[:2]]
    _run(o, c)
    rows = [x for x in o.state() if x.startswith("TIMERS|")]
    assert len(rows) == 1  # the sub-process's boundary timer
    due = int(dict(kv.split("=") for kv in rows[0].split("|")[3].split(","))["dueDate"])
    tkey = int(rows[0].split("|")[2])
    recs = _run(o, trigger_commands([0], [tkey - BASE - 1], [due]))
    seq = [(abi.intent_name(int(r["value_type"]), int(r["intent"])), _eid(o, r)) for r in recs
           if r["value_type"] == abi.VT_PROCESS_INSTANCE]
    want = [("ELEMENT_TERMINATING", "sub"), ("ELEMENT_TERMINATING", "task"), ("ELEMENT_TERMINATING", "task"),
            ("ELEMENT_TERMINATED", "task"), ("ELEMENT_TERMINATED", "task"), ("ELEMENT_TERMINATED", "sub"),
            ("SEQUENCE_FLOW_TAKEN", "to-canceled"), ("ELEMENT_COMPLETED", "canceled"), ("ELEMENT_COMPLETED", "process")]
    it = iter(seq)
    assert all(any(x == w for x in it) for w in want), seq  # containsSubsequence
    assert sum(1 for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CANCELED) == 1
    assert [x for x in o.state() if not x.startswith("KEY|")] == []


def test_interrupting_cycle_reschedules_then_cancels():
    # TriggerTimerProcessor.processRecord (:80-114) + shouldReschedule (:128-130): an interrupting boundary
    # timer with a cycle writes TIMER:TRIGGERED, PROCESS_EVENT:TRIGGERING, the activity's TERMINATE_ELEMENT
    # and the cycle's next TIMER:CREATED (one repetition fewer, due from the trigger's dueDate); the
    # termination then cancels that timer (JOB:CANCELED, TIMER:CANCELED) before the boundary event runs
    from zeebe_amd import bpmn as B
    b = B.createExecutableProcess("process").startEvent("s").serviceTask("a", "a").boundaryEvent("late")
    xml = b.timerWithCycle("R3/PT20S").endEvent("ce").moveToActivity("a").endEvent("e").done()
    o, recs = _started(xml)
    timers = [r for r in recs if r["value_type"] == abi.VT_TIMER and r["intent"] == abi.TIMER_CREATED]
    assert len(timers) == 1 and int(timers[0]["partition"]) == 3
    got = _trigger_all(o, recs)
    seq = [(int(r["value_type"]), int(r["intent"])) for r in got]
    created = [i for i, r in enumerate(got) if r["value_type"] == abi.VT_TIMER and r["intent"] == abi.TIMER_CREATED]
    canceled = [i for i, r in enumerate(got) if r["value_type"] == abi.VT_TIMER and r["intent"] == abi.TIMER_CANCELED]
    assert len(created) == 1 and len(canceled) == 1 and created[0] < canceled[0]
    assert int(got[created[0]]["partition"]) == 2 and got[created[0]]["key"] == got[canceled[0]]["key"]
    assert int(got[canceled[0]]["aux"]) == int(got[created[0]]["aux"])  # the same dueDate
    assert (abi.VT_JOB, abi.JOB_CANCELED) in seq
