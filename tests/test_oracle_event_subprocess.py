"""The oracle's error-start event sub-processes (zb_oracle.cpp trigger_event_sub_process /
activate_event_sub_process; EventHandle.activateElement -> EventTriggerBehavior.triggerEventSubProcess
:74-118 and activateTriggeredEvent :191-264, EventSubProcessProcessor, EventSubProcessInterruptionMarker,
ProcessInstanceElementActivatingApplier.moveVariablesToNewEventScope :102-116,
ProcessProcessor / SubProcessProcessor.onChildTerminated, CatchEventAnalyzer's event order) pinned on the
reference's ErrorEventTest (error start events :288-427), ErrorCatchEventTest (its event sub-process
parameters :118-188 and shouldThrowErrorWithVariables :220-273) and JobThrowErrorTest
.shouldThrowErrorWithVariablesWithEventSubProcess (:350-393), through the restated processing loop."""
from psm import Client
from test_gpu_scheduled import KEY_A
from test_oracle_error_events import JOB_TYPE, ERROR_CODE, pi_of, started, subsequence
from test_oracle_message_ttl import cluster, of, write
from zeebe_amd import abi, bpmn


def esp_process(*esps, boundary=None):
    """ErrorEventTest's processes: event sub-processes (id, start id, code; None = a catch-all) before the
    start event, a service task (with an error boundary event of `boundary`'s code when given)."""
    b = bpmn.createExecutableProcess("wf")
    for sid, start, code in esps:
        b.eventSubProcess(sid).startEvent(start).error(code).endEvent(sid + "-end").eventSubProcessDone()
    b.startEvent("start").serviceTask("task", JOB_TYPE)
    if boundary is not None:
        b.boundaryEvent("error-boundary-event").error(boundary).endEvent("boundary-end").moveToActivity("task")
    return b.endEvent("end").done()


def completed_starts(cl, pik):
    return [r.value["elementId"] for r in cl.parts[0].log.entries if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.value["processInstanceKey"] == pik and r.intent == abi.PI_ELEMENT_COMPLETED
            and r.value["bpmnElementType"] == "START_EVENT"]


def ids_of(cl, pik):
    return [(r.value["elementId"], abi.PI_INTENTS[r.intent]) for r in cl.parts[0].log.entries
            if r.value_type == abi.VT_PROCESS_INSTANCE and r.value["processInstanceKey"] == pik]


def test_error_start_events():
    # ErrorEventTest.shouldCatchErrorEventsOnErrorStartEventWithoutErrorRef / ...WithEmptyErrorCode /
    # ...WithoutErrorCode (:288-391): a catch-all error start event; ...WithSpecificErrorCode (:393-427): the
    # code-specific one of two
    for esps, code, want in ((( ("sub", "error", None), ), "errorCode", "error"),
                             ((("sub", "error", ""), ), "errorCode", "error"),
                             ((("sub-1", "catch-all", None), ("sub-2", "code-specific", ERROR_CODE)), ERROR_CODE,
                              "code-specific")):
        cl = cluster((esp_process(*esps), KEY_A, 1))
        job, pik = started(cl, None)
        write(cl, Client.throw_error(job.key, code))
        assert subsequence(completed_starts(cl, pik), ["start", want])
        assert pi_of(cl, pik)[-1] == ("PROCESS", "ELEMENT_COMPLETED")


def test_error_event_sub_process_record_sequence():
    # ErrorCatchEventTest.shouldTriggerEvent["error event subprocess"] (:118-131, :191-218): the task
    # terminated, the event sub-process activated and completed, then the process
    cl = cluster((esp_process(("error-event-subprocess", "error-start-event", ERROR_CODE)), KEY_A, 1))
    job, pik = started(cl, None)
    state = [r for r in cl.parts[0].state() if r.startswith("EVENT_SCOPE|%d|" % pik)]
    assert state == ["EVENT_SCOPE|%d|accepting=1,interrupted=0,interrupting=error-start-event,boundaryElementIds=" % pik]
    e = write(cl, Client.throw_error(job.key, ERROR_CODE))
    assert subsequence(ids_of(cl, pik), [
        ("task", "ELEMENT_TERMINATING"), ("task", "ELEMENT_TERMINATED"),
        ("error-event-subprocess", "ELEMENT_ACTIVATING"), ("error-event-subprocess", "ELEMENT_COMPLETED"),
        ("wf", "ELEMENT_COMPLETED")])
    # the event sub-process is activated by a new command (key -1), its start event completes before its end
    # event; TRIGGERING only (no TRIGGERED: the trigger moves to the start event for its output mappings)
    act = [r for r in e if r.record_type == abi.RT_COMMAND and r.value_type == abi.VT_PROCESS_INSTANCE
           and r.intent == abi.PI_INTENT_IDS["ACTIVATE_ELEMENT"] and r.value["elementId"] == "error-event-subprocess"]
    assert len(act) == 1 and act[0].key == -1 and act[0].value["flowScopeKey"] == pik
    assert [r.intent for r in e if r.value_type == abi.VT_PROCESS_EVENT] == [abi.PE_TRIGGERING]
    assert subsequence(ids_of(cl, pik), [("error-start-event", "ELEMENT_COMPLETED"),
                                         ("error-event-subprocess-end", "ELEMENT_COMPLETED"),
                                         ("error-event-subprocess", "ELEMENT_COMPLETED")])
    assert [r for r in cl.parts[0].state() if not r.startswith("KEY|")] == []


def test_error_variables_go_to_the_process_instance():
    # JobThrowErrorTest.shouldThrowErrorWithVariablesWithEventSubProcess (:350-393), ErrorCatchEventTest
    # .shouldThrowErrorWithVariables["error event subprocess"]: VARIABLE:CREATED at the process instance
    cl = cluster((esp_process(("error-event-subprocess", "error-start-event", ERROR_CODE)), KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, ERROR_CODE, variables=[("foo", "bar")]))
    var = [(r.value["name"], r.value["value"], r.value["scopeKey"], r.intent) for r in e if r.value_type == abi.VT_VARIABLE]
    assert var == [("foo", "bar", pik, abi.VAR_CREATED)]


def test_catch_event_precedence():
    # ErrorCatchEventTest "favor boundary event on task over error event subprocess" (:153-165): the task's
    # scope comes first
    cl = cluster((esp_process(("error-event-subprocess", "esp-start", ERROR_CODE), boundary=ERROR_CODE), KEY_A, 1))
    job, pik = started(cl, None)
    write(cl, Client.throw_error(job.key, ERROR_CODE))
    assert ("error-boundary-event", "ELEMENT_COMPLETED") in ids_of(cl, pik)
    assert ("error-event-subprocess", "ELEMENT_ACTIVATING") not in ids_of(cl, pik)
    # "favor error event subprocess over boundary event on subprocess" (:166-186): inside the sub-process the
    # event sub-process's start event comes before the sub-process's boundary event
    b = bpmn.createExecutableProcess("wf").startEvent().subProcess("sub")
    b.eventSubProcess("error-event-subprocess").startEvent("error-start-event").error(ERROR_CODE).endEvent("ee")
    b.eventSubProcessDone().startEvent("s2").serviceTask("task", JOB_TYPE).endEvent("e2").subProcessDone()
    xml = b.boundaryEvent("error").error(ERROR_CODE).endEvent("be").moveToActivity("sub").endEvent("end").done()
    cl = cluster((xml, KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, ERROR_CODE))
    assert subsequence(ids_of(cl, pik), [
        ("task", "ELEMENT_TERMINATING"), ("task", "ELEMENT_TERMINATED"),
        ("error-event-subprocess", "ELEMENT_ACTIVATING"), ("error-event-subprocess", "ELEMENT_COMPLETED"),
        ("sub", "ELEMENT_COMPLETED"), ("end", "ELEMENT_COMPLETED"), ("wf", "ELEMENT_COMPLETED")])
    assert ("error", "ELEMENT_ACTIVATING") not in ids_of(cl, pik)


def test_uncaught_error_lists_the_error_start_events():
    # CatchEventAnalyzer: the available codes in getEvents order (event sub-processes first, the last
    # attached first) sorted by ERROR_CODE_COMPARATOR per scope
    cl = cluster((esp_process(("s1", "st1", "A"), ("s2", "st2", "B")), KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, "C"))
    assert of(e, abi.VT_INCIDENT, abi.INCIDENT_CREATED)[0].value["errorMessage"] == (
        "Expected to throw an error event with the code 'C', but it was not caught. Available error events are [B, A]")


def test_parallel_branches_are_terminated():
    # an interrupting event sub-process terminates every active child (one TERMINATE_ELEMENT each, key
    # order): the other branch's job is canceled; the event sub-process runs once none is left
    b = bpmn.createExecutableProcess("wf")
    b.eventSubProcess("esp").startEvent("esp-start").error(ERROR_CODE).serviceTask("recover", "recover")
    b.endEvent("esp-end").eventSubProcessDone()
    b.startEvent("start").parallelGateway("fork").serviceTask("task", JOB_TYPE).parallelGateway("join")
    xml = b.moveToNode("fork").serviceTask("other", "other").connectTo("join").endEvent("end").done()
    cl = cluster((xml, KEY_A, 1))
    e = write(cl, Client.create("wf"))
    jobs = {r.value["type"]: r for r in of(e, abi.VT_JOB, abi.JOB_CREATED)}
    pik = jobs[JOB_TYPE].value["processInstanceKey"]
    e = write(cl, Client.throw_error(jobs[JOB_TYPE].key, ERROR_CODE))
    terms = [r for r in e if r.record_type == abi.RT_COMMAND and r.value_type == abi.VT_PROCESS_INSTANCE
             and r.intent == abi.PI_INTENT_IDS["TERMINATE_ELEMENT"]]
    assert sorted(r.value["elementId"] for r in terms) == ["other", "task"]
    assert [r.key for r in terms] == sorted(r.key for r in terms)  # getChildren: key order
    assert [r.key for r in of(e, abi.VT_JOB, abi.JOB_CANCELED)] == [jobs["other"].key]
    rec = of(e, abi.VT_JOB, abi.JOB_CREATED)
    assert [r.value["type"] for r in rec] == ["recover"]
    write(cl, Client.complete_job(rec[0].key))
    assert pi_of(cl, pik)[-1] == ("PROCESS", "ELEMENT_COMPLETED")
    assert [r for r in cl.parts[0].state() if not r.startswith("KEY|")] == []


def test_error_end_event_caught_by_a_sub_process_boundary_event():
    # ErrorEventTest.shouldThrowErrorOnEndEvent (:618-656)
    b = bpmn.createExecutableProcess("wf").startEvent().subProcess("subProcess").startEvent()
    b.endEvent("throw-error").error(ERROR_CODE).subProcessDone()
    xml = b.boundaryEvent("catch-error").error(ERROR_CODE).endEvent("end-error").moveToActivity("subProcess").endEvent("end").done()
    cl = cluster((xml, KEY_A, 1))
    e = write(cl, Client.create("wf"))
    pik = e[-1].value["processInstanceKey"] if e[-1].value_type == abi.VT_PROCESS_INSTANCE else \
        of(e, abi.VT_PROCESS_INSTANCE, abi.PI_ELEMENT_ACTIVATED)[0].value["processInstanceKey"]
    events = [(t, i) for t, i in pi_of(cl, pik) if not i.endswith("_ELEMENT") and i != "SEQUENCE_FLOW_TAKEN"]
    assert subsequence(events, [
        ("END_EVENT", "ELEMENT_ACTIVATED"), ("SUB_PROCESS", "ELEMENT_TERMINATING"), ("END_EVENT", "ELEMENT_TERMINATING"),
        ("END_EVENT", "ELEMENT_TERMINATED"), ("SUB_PROCESS", "ELEMENT_TERMINATED"), ("BOUNDARY_EVENT", "ELEMENT_ACTIVATING"),
        ("BOUNDARY_EVENT", "ELEMENT_COMPLETED"), ("PROCESS", "ELEMENT_COMPLETED")])


def test_uncaught_error_end_event_raises_an_incident():
    # ErrorEventIncidentTest.shouldCreateIncidentOnErrorEndEvent (:264-297): on the end event itself
    xml = bpmn.createExecutableProcess("wf").startEvent().endEvent("error").error("error").done()
    cl = cluster((xml, KEY_A, 1))
    e = write(cl, Client.create("wf"))
    inc = of(e, abi.VT_INCIDENT, abi.INCIDENT_CREATED)[0].value
    # (the reference takes the first END_EVENT record, the ACTIVATE_ELEMENT command: the same key)
    end = [r for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.value["bpmnElementType"] == "END_EVENT"
           and r.record_type == abi.RT_EVENT][-1]
    assert inc["errorType"] == "UNHANDLED_ERROR_EVENT" and inc["errorMessage"] == (
        "Expected to throw an error event with the code 'error', but it was not caught. "
        "No error events are available in the scope.")
    assert (inc["elementId"], inc["elementInstanceKey"], inc["variableScopeKey"], inc["jobKey"]) == \
        ("error", end.key, end.key, -1)
    assert abi.PI_INTENTS[end.intent] == "ELEMENT_ACTIVATING"


def test_error_inside_a_triggered_event_sub_process_is_not_caught_by_its_container():
    # ErrorEventIncidentTest.shouldCreateIncidentIfErrorIsThrownFromInterruptingEventSubprocess (:190-228): the
    # interrupted process is not searched
    b = bpmn.createExecutableProcess("wf")
    b.eventSubProcess("error").startEvent("error-start").error(ERROR_CODE).serviceTask("task-in-subprocess", JOB_TYPE)
    b.endEvent("esp-end").eventSubProcessDone()
    xml = b.startEvent("start").serviceTask("task", JOB_TYPE).endEvent("end").done()
    cl = cluster((xml, KEY_A, 1))
    job, pik = started(cl, None)
    e = write(cl, Client.throw_error(job.key, ERROR_CODE))
    inner = of(e, abi.VT_JOB, abi.JOB_CREATED)[0]
    assert inner.value["elementId"] == "task-in-subprocess"
    e = write(cl, Client.throw_error(inner.key, ERROR_CODE))
    inc = of(e, abi.VT_INCIDENT, abi.INCIDENT_CREATED)[0].value
    assert inc["errorType"] == "UNHANDLED_ERROR_EVENT" and inc["elementId"] == "NO_CATCH_EVENT_FOUND"
    assert inc["errorMessage"] == ("Expected to throw an error event with the code '%s', but it was not caught. "
                                   "No error events are available in the scope." % ERROR_CODE)


def test_error_end_event_caught_by_an_event_sub_process():
    # an error end event inside a sub-process, caught by the process's event sub-process: the process's
    # children terminate (the sub-process with its end event), then the event sub-process runs
    b = bpmn.createExecutableProcess("wf")
    b.eventSubProcess("esp").startEvent("esp-start").error("E").endEvent("esp-end").eventSubProcessDone()
    b.startEvent("start").subProcess("sub").startEvent("ss").endEvent("throw").error("E").subProcessDone()
    xml = b.endEvent("end").done()
    cl = cluster((xml, KEY_A, 1))
    write(cl, Client.create("wf"))
    ids = [(r.value["elementId"], abi.PI_INTENTS[r.intent]) for r in cl.parts[0].log.entries
           if r.value_type == abi.VT_PROCESS_INSTANCE]
    assert subsequence(ids, [("throw", "ELEMENT_ACTIVATED"), ("sub", "ELEMENT_TERMINATING"), ("throw", "ELEMENT_TERMINATED"),
                             ("sub", "ELEMENT_TERMINATED"), ("esp", "ELEMENT_ACTIVATING"), ("esp-end", "ELEMENT_COMPLETED"),
                             ("esp", "ELEMENT_COMPLETED"), ("wf", "ELEMENT_COMPLETED")])
    assert [r for r in cl.parts[0].state() if not r.startswith("KEY|")] == []
