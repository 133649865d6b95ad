"""The oracle's error boundary events and JOB:THROW_ERROR (zb_oracle.cpp throw_error; JobThrowErrorProcessor
.java:84-176, CatchEventAnalyzer.java:55-160, JobErrorThrownApplier, BpmnEventPublicationBehavior
.throwErrorEvent -> EventHandle.activateElement, EventTriggerBehavior.activateTriggeredEvent) pinned on the
reference's ErrorEventTest, ErrorEventIncidentTest and JobThrowErrorTest (engine/src/test/.../processing/
{bpmn/error,incident,job}), run through the restated processing loop (tests/psm.py, one partition over the
oracle engine).  One boundary event per activity (job worker tasks and embedded sub-processes): the cases with two error boundary events on one task
(shouldCatchErrorEventsByErrorCode, ...WithSpecificErrorCode) are outside the subset."""
from psm import Client
from test_gpu_scheduled import KEY_A
from test_oracle_message_ttl import cluster, of, write
from zeebe_amd import abi, bpmn

JOB_TYPE, ERROR_CODE = "test", "ERROR"


def process(code=ERROR_CODE, boundary=True):
    # ErrorEventTest.process(...) with serviceTask.boundaryEvent("error", b -> b.error(code)).endEvent()
    b = bpmn.createExecutableProcess("wf").startEvent("start").serviceTask("task", JOB_TYPE)
    if boundary:
        b.boundaryEvent("error").error(code).endEvent("end-error").moveToActivity("task")
    return b.endEvent("end").done()


def started(cl, xml):
    e = write(cl, Client.create("wf"))
    job = of(e, abi.VT_JOB, abi.JOB_CREATED)[0]
    pik = job.value["processInstanceKey"]
    return job, pik


def pi_of(cl, pik):
    return [(r.value["bpmnElementType"], abi.PI_INTENTS[r.intent]) for r in cl.parts[0].log.entries
            if r.value_type == abi.VT_PROCESS_INSTANCE and r.value["processInstanceKey"] == pik]


def subsequence(got, want):
    it = iter(got)
    return all(w in it for w in want)


def test_error_boundary_event_is_triggered():
    # ErrorEventTest.shouldTriggerEvent (:60-97) and shouldNotCancelJob (:429-448)
    cl = cluster((process(), KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, ERROR_CODE))
    thrown = of(e, abi.VT_JOB, abi.JOB_ERROR_THROWN)
    assert len(thrown) == 1 and thrown[0].key == job.key
    assert thrown[0].value["errorCode"] == ERROR_CODE and thrown[0].value["elementId"] == "task"
    assert subsequence(pi_of(cl, pik), [
        ("SERVICE_TASK", "ELEMENT_TERMINATING"), ("SERVICE_TASK", "ELEMENT_TERMINATED"),
        ("BOUNDARY_EVENT", "ELEMENT_ACTIVATING"), ("BOUNDARY_EVENT", "ELEMENT_ACTIVATED"),
        ("BOUNDARY_EVENT", "COMPLETE_ELEMENT"), ("BOUNDARY_EVENT", "ELEMENT_COMPLETING"),
        ("BOUNDARY_EVENT", "ELEMENT_COMPLETED"), ("SEQUENCE_FLOW", "SEQUENCE_FLOW_TAKEN"),
        ("END_EVENT", "ELEMENT_ACTIVATING"), ("END_EVENT", "ELEMENT_ACTIVATED"), ("END_EVENT", "ELEMENT_COMPLETING"),
        ("END_EVENT", "ELEMENT_COMPLETED"), ("PROCESS", "COMPLETE_ELEMENT"), ("PROCESS", "ELEMENT_COMPLETING"),
        ("PROCESS", "ELEMENT_COMPLETED")])
    jobs = [abi.JOB_INTENTS[r.intent] for r in cl.parts[0].log.entries if r.value_type == abi.VT_JOB]
    assert jobs == ["CREATED", "THROW_ERROR", "ERROR_THROWN"]
    # the boundary event was triggered through the task's event scope: TRIGGERING then TRIGGERED
    pe = [r for r in e if r.value_type == abi.VT_PROCESS_EVENT]
    assert [r.intent for r in pe] == [abi.PE_TRIGGERING, abi.PE_TRIGGERED] and pe[0].value["targetElementId"] == "error"
    assert not [r for r in cl.parts[0].state() if r.startswith(("JOBS|", "JOB_STATES|"))]


def test_numeric_and_catch_all_error_codes():
    # shouldCatchErrorEventsByNumericErrorCode (:148-191); ...OnBoundaryEventWithoutErrorRef (:194-224);
    # ...WithoutErrorCode (:227-254)
    for code, thrown in (("404", "404"), ("", "error"), (None, "error")):
        xml = process(code) if code is not None else process("").replace(' errorRef="Error_error"', "")
        cl = cluster((xml, KEY_A, 1))
        job, pik = started(cl, None)
        write(cl, Client.throw_error(job.key, thrown))
        assert ("BOUNDARY_EVENT", "ELEMENT_COMPLETED") in pi_of(cl, pik)
        assert pi_of(cl, pik)[-1] == ("PROCESS", "ELEMENT_COMPLETED")


def test_uncaught_error_creates_an_incident():
    # ErrorEventIncidentTest.shouldCreateIncidentWhenThrownErrorIsUncaught (:92-123) and
    # shouldCreateIncidentWithDefaultErrorMessage (:125-156); JobThrowErrorTest (:397-445) without a boundary
    cl = cluster((process("error"), KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, "other-error", "error thrown"))
    thrown = of(e, abi.VT_JOB, abi.JOB_ERROR_THROWN)[0]
    assert thrown.value["elementId"] == "NO_CATCH_EVENT_FOUND" and thrown.value["errorMessage"] == "error thrown"
    inc = of(e, abi.VT_INCIDENT, abi.INCIDENT_CREATED)[0].value
    assert inc["errorType"] == "UNHANDLED_ERROR_EVENT"
    assert inc["errorMessage"] == ("Expected to throw an error event with the code 'other-error' with message 'error thrown', "
                                   "but it was not caught. Available error events are [error]")
    assert (inc["elementId"], inc["elementInstanceKey"], inc["variableScopeKey"], inc["jobKey"], inc["processInstanceKey"]) == \
        (thrown.value["elementId"], thrown.value["elementInstanceKey"], thrown.value["elementInstanceKey"], thrown.key, pik)
    # the job stays, ERROR_THROWN: a second throw is rejected (JobThrowErrorTest.shouldRejectIfErrorIsThrown :100-114)
    e = write(cl, Client.throw_error(job.key, "error"))
    rej = [r for r in e if r.record_type == abi.RT_REJECTION]
    assert rej and rej[0].rejection_type == abi.REJ_INVALID_STATE and "it is in state 'ERROR_THROWN'" in rej[0].rejection_reason
    state = cl.parts[0].state()
    assert "JOB_STATES|%d|ERROR_THROWN" % job.key in state
    # FailJobTest.shouldRejectFailIfErrorThrown (:265-280); completion the same (DefaultJobCommand
    # PreconditionGuard: ACTIVATABLE or ACTIVATED)
    for cmd, verb in ((Client.fail_job(job.key, 3), "fail"), (Client.complete_job(job.key), "complete")):
        rej = [r for r in write(cl, cmd) if r.record_type == abi.RT_REJECTION]
        assert rej[0].rejection_type == abi.REJ_INVALID_STATE and rej[0].rejection_reason == (
            "Expected to %s job with key '%d', but it is in state 'ERROR_THROWN'" % (verb, job.key))
    assert cl.parts[0].state() == state
    cl = cluster((process(boundary=False), KEY_A, 1))
    job, _ = started(cl, None)
    e = write(cl, Client.throw_error(job.key, "other-error"))
    assert of(e, abi.VT_INCIDENT, abi.INCIDENT_CREATED)[0].value["errorMessage"] == \
        "Expected to throw an error event with the code 'other-error', but it was not caught. No error events are available in the scope."


def test_rejections_and_truncation():
    # JobThrowErrorTest.shouldRejectIfJobNotFound (:70-81), shouldRejectIfJobIsFailed (:83-98),
    # shouldTruncateErrorMessage (:396-419)
    cl = cluster((process(), KEY_A, 1))
    e = write(cl, Client.throw_error(123, "error"))
    assert e[-1].record_type == abi.RT_REJECTION and e[-1].rejection_type == abi.REJ_NOT_FOUND
    assert e[-1].rejection_reason == "Expected to throw an error for job with key '123', but no such job was found"
    job, _ = started(cl, None)
    write(cl, Client.fail_job(job.key, 0))
    e = write(cl, Client.throw_error(job.key, "error"))
    assert e[-1].rejection_type == abi.REJ_INVALID_STATE and "it is in state 'FAILED'" in e[-1].rejection_reason
    # shouldTruncateErrorMessage (:395-419) / shouldNotTruncateErrorMessage (:421-445): limitString to 10 000
    # characters and "...", no error code
    for n, want in ((10001, "*" * 10000 + "..."), (10000, "*" * 10000)):
        cl = cluster((process(boundary=False), KEY_A, 1))
        job, _ = started(cl, None)
        e = write(cl, Client.throw_error(job.key, "", "*" * n))
        assert of(e, abi.VT_JOB, abi.JOB_ERROR_THROWN)[0].value["errorMessage"] == want
        assert of(e, abi.VT_INCIDENT, abi.INCIDENT_CREATED)[0].value["errorMessage"] == (
            "Expected to throw an error event with the code '' with message '" + want +
            "', but it was not caught. No error events are available in the scope.")


def test_error_variables_are_local_to_the_catch_event():
    # JobThrowErrorTest.shouldThrowErrorWithVariables (:116-167): one VARIABLE:CREATED, at the error catch event
    cl = cluster((process(), KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, ERROR_CODE, "error-message", variables=[("foo", "bar")]))
    thrown = of(e, abi.VT_JOB, abi.JOB_ERROR_THROWN)[0]
    assert dict(thrown.value["variables"]) == {"foo": "bar"} and thrown.value["errorMessage"] == "error-message"
    boundary = [r for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_ACTIVATING
                and r.value["elementId"] == "error"][0]
    var = [r for r in e if r.value_type == abi.VT_VARIABLE]
    assert [(r.value["name"], r.value["value"], r.value["scopeKey"], r.intent) for r in var] == \
        [("foo", "bar", boundary.key, abi.VAR_CREATED)]


def sub_process_boundaries():
    # ErrorEventIncidentTest.BOUNDARY_EVENT_SUBPROCESS (:69-89)
    b = bpmn.createExecutableProcess("wf").startEvent("start").subProcess("subprocess").startEvent("start_subprocess")
    b.serviceTask("task_in_subprocess", JOB_TYPE).boundaryEvent("error_in_subprocess").error("error_in_subprocess")
    b.endEvent("end_boundary_in_subprocess").moveToActivity("task_in_subprocess").endEvent("end_subprocess")
    b.subProcessDone().boundaryEvent("error").error("error").endEvent("end_boundary").moveToActivity("subprocess")
    return b.endEvent("end").done()


def test_error_boundary_event_on_a_sub_process():
    # ErrorEventIncidentTest.shouldCreateIncidentIfErrorIsThrownFromSubprocessWithoutCatchEvent... (:379-409):
    # the walk through the flow scopes lists every error event it passes
    cl = cluster((sub_process_boundaries(), KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, "unknown_error_code", "error message"))
    assert of(e, abi.VT_INCIDENT, abi.INCIDENT_CREATED)[0].value["errorMessage"] == (
        "Expected to throw an error event with the code 'unknown_error_code' with message 'error message', but it "
        "was not caught. Available error events are [error_in_subprocess, error]")
    # caught at the sub-process's boundary event: the sub-process terminates (its task first), then the
    # boundary event activates in the process scope (as ErrorEventTest.shouldCatchErrorOutsideMultiInstance
    # Subprocess :570-616, without the body)
    cl = cluster((sub_process_boundaries(), KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, "error", variables=[("foo", "bar")]))
    assert of(e, abi.VT_JOB, abi.JOB_ERROR_THROWN)[0].value["elementId"] == "task_in_subprocess"
    boundary = [r for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_ACTIVATING
                and r.value["elementId"] == "error"][0]
    assert [(r.value["name"], r.value["scopeKey"]) for r in e if r.value_type == abi.VT_VARIABLE] == \
        [("foo", boundary.key)]
    assert subsequence(pi_of(cl, pik), [
        ("SUB_PROCESS", "ELEMENT_TERMINATING"), ("SERVICE_TASK", "ELEMENT_TERMINATING"),
        ("SERVICE_TASK", "ELEMENT_TERMINATED"), ("SUB_PROCESS", "ELEMENT_TERMINATED"),
        ("BOUNDARY_EVENT", "ELEMENT_ACTIVATING"), ("BOUNDARY_EVENT", "ELEMENT_COMPLETED"),
        ("END_EVENT", "ELEMENT_COMPLETED"), ("PROCESS", "ELEMENT_COMPLETED")])
    ids = [r.value["elementId"] for r in cl.parts[0].log.entries if r.value_type == abi.VT_PROCESS_INSTANCE
           and r.intent == abi.PI_ELEMENT_COMPLETED]
    assert ids[-3:] == ["error", "end_boundary", "wf"]
    pe = [r for r in e if r.value_type == abi.VT_PROCESS_EVENT]
    assert [r.intent for r in pe] == [abi.PE_TRIGGERING, abi.PE_TRIGGERED] and pe[0].value["targetElementId"] == "error"
    # caught inside: the sub-process continues
    cl = cluster((sub_process_boundaries(), KEY_A, 1))
    job, pik = started(cl, None)
    write(cl, Client.throw_error(job.key, "error_in_subprocess"))
    ids = [r.value["elementId"] for r in cl.parts[0].log.entries if r.value_type == abi.VT_PROCESS_INSTANCE
           and r.intent == abi.PI_ELEMENT_COMPLETED]
    assert ids[-5:] == ["error_in_subprocess", "end_boundary_in_subprocess", "subprocess", "end", "wf"]
    assert not [r for r in cl.parts[0].state() if r.startswith(("JOBS|", "EVENT_SCOPE|"))]


def test_random_processes_with_error_boundary_events_on_the_engine():
    # the GPU campaign's workloads (tests/test_gpu_error_events.py) through the engine alone: the oracle takes
    # every throw (caught, or an incident) and every completion without refusing
    import numpy as np
    from random_bpmn import random_process
    from test_gpu_error_events import random_error_campaign
    caught = incidents = 0
    for seed in (3, 19):
        xml = random_process(np.random.default_rng(9000 + seed), sub_processes=True, task_kinds=True, errors=True)
        cl = cluster((xml, KEY_A, 1))
        random_error_campaign(seed, cl, lambda *r: write(cl, *r), xml)
        log = cl.parts[0].log.entries
        caught += sum(1 for r in log if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_COMPLETED
                      and r.value["bpmnElementType"] == "BOUNDARY_EVENT")
        incidents += sum(1 for r in log if r.value_type == abi.VT_INCIDENT)
    assert caught >= 10 and incidents >= 10


def two_boundaries(first=("error-1", "error-1"), second=("error-2", "error-2"), timer=None):
    # ErrorEventTest.process(serviceTask -> two boundaryEvent(..).error(..).endEvent()); with `timer` a
    # timer boundary event (the activity's one timer) besides them
    b = bpmn.createExecutableProcess("wf").startEvent("start").serviceTask("task", JOB_TYPE)
    for bid, code in (first, second):
        b.boundaryEvent(bid).error(code).endEvent("end-" + bid).moveToActivity("task")
    if timer:
        b.boundaryEvent("timer").timerWithDuration(timer).endEvent("end-timer").moveToActivity("task")
    return b.endEvent("end").done()


def boundary_path(cl, pik):
    return [r.value["elementId"] for r in cl.parts[0].log.entries if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.value["processInstanceKey"] == pik and r.value["bpmnElementType"] == "BOUNDARY_EVENT"]


def test_two_error_boundary_events_by_error_code():
    # ErrorEventTest.shouldCatchErrorEventsByErrorCode (:99-146): each code its own boundary event
    cl = cluster((two_boundaries(), KEY_A, 1))
    j1, p1 = started(cl, None)
    j2, p2 = started(cl, None)
    write(cl, Client.throw_error(j1.key, "error-1"), Client.throw_error(j2.key, "error-2"))
    assert set(boundary_path(cl, p1)) == {"error-1"} and set(boundary_path(cl, p2)) == {"error-2"}
    assert pi_of(cl, p1)[-1] == pi_of(cl, p2)[-1] == ("PROCESS", "ELEMENT_COMPLETED")


def test_code_specific_error_boundary_event_wins():
    # ErrorEventTest.shouldCatchErrorEventsOnBoundaryEventWithSpecificErrorCode (:256-287): the catch-all is
    # attached first, the code-specific one catches (ERROR_CODE_COMPARATOR orders codes descending)
    cl = cluster((two_boundaries(("catch-all", None), ("code-specific", ERROR_CODE)), KEY_A, 1))
    job, pik = started(cl, None)
    write(cl, Client.throw_error(job.key, ERROR_CODE))
    assert set(boundary_path(cl, pik)) == {"code-specific"}
    # another code: the catch-all
    job, pik = started(cl, None)
    write(cl, Client.throw_error(job.key, "other"))
    assert set(boundary_path(cl, pik)) == {"catch-all"}


def test_available_error_codes_in_comparator_order():
    # findErrorCatchEventInScope visits the codes in ERROR_CODE_COMPARATOR order (reversed byte order) and
    # lists each visited one; the event scope holds every boundary event in attach order
    cl = cluster((two_boundaries(("b1", "A-1"), ("b2", "B-2")), KEY_A, 1))
    job, pik = started(cl, None)
    state = [r for r in cl.parts[0].state() if r.startswith("EVENT_SCOPE|")]
    assert any("interrupting=b1;b2,boundaryElementIds=b1;b2" in r for r in state)
    e = write(cl, Client.throw_error(job.key, "C-3"))
    assert of(e, abi.VT_INCIDENT, abi.INCIDENT_CREATED)[0].value["errorMessage"] == (
        "Expected to throw an error event with the code 'C-3', but it was not caught. "
        "Available error events are [B-2, A-1]")


def test_error_boundary_events_beside_a_timer_boundary_event():
    # a timer and two error boundary events on one task: the timer fires, or an error is caught (the timer
    # canceled with the task's termination)
    cl = cluster((two_boundaries(timer="PT10S"), KEY_A, 1))
    job, pik = started(cl, None)
    assert [r for r in cl.parts[0].state() if r.startswith("TIMERS|")]
    e = write(cl, Client.throw_error(job.key, "error-2"))
    assert of(e, abi.VT_TIMER, abi.TIMER_CANCELED)
    assert set(boundary_path(cl, pik)) == {"error-2"}
    assert not [r for r in cl.parts[0].state() if r.startswith(("TIMERS|", "JOBS|", "EVENT_SCOPE|"))]


def test_error_boundary_event_on_a_multi_instance_task():
    # ErrorCatchEventTest["boundary event on multi-instance service task"] (:103-116): the boundary event
    # attaches to the body; shouldTriggerEvent's subsequence (:191-218) and shouldThrowErrorWithVariables
    # (:220-273: the variable local to the boundary event)
    b = bpmn.createExecutableProcess("wf").startEvent().serviceTask("task", JOB_TYPE).multiInstance("= [1]")
    xml = b.boundaryEvent("error-boundary-event").error(ERROR_CODE).endEvent("be").moveToActivity("task").endEvent("end").done()
    cl = cluster((xml, KEY_A, 1))
    job, pik = started(cl, None)
    body = [r for r in cl.parts[0].state() if r.startswith("EVENT_SCOPE|") and "error-boundary-event" in r]
    assert len(body) == 1
    e = write(cl, Client.throw_error(job.key, ERROR_CODE, variables=[("foo", "bar")]))
    ids = [(r.value["elementId"], abi.PI_INTENTS[r.intent]) for r in cl.parts[0].log.entries
           if r.value_type == abi.VT_PROCESS_INSTANCE and r.value["processInstanceKey"] == pik]
    assert subsequence(ids, [("task", "ELEMENT_TERMINATING"), ("task", "ELEMENT_TERMINATED"),
                             ("error-boundary-event", "ELEMENT_ACTIVATING"), ("error-boundary-event", "ELEMENT_COMPLETED"),
                             ("wf", "ELEMENT_COMPLETED")])
    bk = [r.key for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_ACTIVATING
          and r.value["elementId"] == "error-boundary-event"][0]
    assert [(r.value["name"], r.value["scopeKey"]) for r in e if r.value_type == abi.VT_VARIABLE] == [("foo", bk)]
    assert [r for r in cl.parts[0].state() if not r.startswith("KEY|")] == []
