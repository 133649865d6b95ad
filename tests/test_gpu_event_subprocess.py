"""Error-start event sub-processes in the reference's processing loop.  A process (or an embedded
sub-process) with event sub-processes whose start events catch errors runs on the device -- they subscribe
to nothing; the instance's (the sub-process's) event scope lists their start events among its interrupting
ids, as the state export writes it -- and a JOB:THROW_ERROR of a device job moves the instance to the engine
(the adapter's held-instance hand-off), which terminates the flow scope's children and runs the event
sub-process (oracle pinned by tests/test_oracle_event_subprocess.py).  The same workload through the loop
over the engine alone and through [adapter, engine]: every log and state equal, at batch limits 3 and 100."""
import pytest

from psm import Client, open_jobs
from test_gpu_scheduled import KEY_A, KEY_B, KEY_C, check, single, write
from zeebe_amd import abi, bpmn

pytestmark = pytest.mark.gpu


def processes():
    # the process's event sub-processes (code-specific with a recovery task, catch-all) and two branches
    a = bpmn.createExecutableProcess("esp")
    a.eventSubProcess("on-e1").startEvent("e1-start").error("E1").serviceTask("recover", "recover").endEvent("e1-end")
    a.eventSubProcessDone().eventSubProcess("on-any").startEvent("any-start").error().endEvent("any-end")
    a.eventSubProcessDone().startEvent("start").parallelGateway("fork").serviceTask("work", "work")
    a = a.parallelGateway("join").moveToNode("fork").serviceTask("other", "other").connectTo("join").endEvent("end").done()
    # an event sub-process inside an embedded sub-process, beside the sub-process's own error boundary
    b = bpmn.createExecutableProcess("nested").startEvent("s").subProcess("sub")
    b.eventSubProcess("inner").startEvent("inner-start").error("E2").endEvent("inner-end").eventSubProcessDone()
    b.startEvent("sub-start").serviceTask("work", "work").endEvent("sub-end").subProcessDone()
    b = b.boundaryEvent("outer").error("E2").endEvent("outer-end").moveToActivity("sub").endEvent("end").done()
    # the task's own boundary event first, then the process's event sub-process
    c = bpmn.createExecutableProcess("both").eventSubProcess("proc-esp").startEvent("ps").error("E3").endEvent("pe")
    c.eventSubProcessDone().startEvent("s").serviceTask("work", "work").boundaryEvent("b").error("E1").endEvent("be")
    c = c.moveToActivity("work").endEvent("end").done()
    return a, b, c


@pytest.mark.parametrize("limit", [3, 100])
def test_error_event_sub_processes_in_the_processing_loop(limit):
    a, b, c = processes()
    deps = [(a, KEY_A, 1), (b, KEY_B, 1), (c, KEY_C, 1)]
    ref, gpu = single(deps, deps, limit=limit)
    write(ref, gpu, *([Client.create("esp") for _ in range(6)] + [Client.create("nested") for _ in range(3)] +
                      [Client.create("both") for _ in range(3)]))
    ad = gpu.parts[0].adapter
    assert ad.counts["device_commands"] >= 12
    # the jobs by instance (instance keys follow the CREATE order at every batch limit)
    by = {}
    for k, r in open_jobs(ref.parts[0].log).items():
        by.setdefault(r.value["processInstanceKey"], {})[r.value["elementId"]] = k
    inst = [by[p] for p in sorted(by)]
    esp, nested, both = inst[:6], inst[6:9], inst[9:]
    write(ref, gpu, Client.throw_error(esp[0]["work"], "E1", "", variables=(("why", "x"),)),
          Client.throw_error(esp[1]["work"], "Z"), Client.throw_error(esp[2]["other"], "E1"),
          Client.complete_job(esp[3]["work"]), Client.complete_job(esp[3]["other"]),
          Client.throw_error(nested[0]["work"], "E2"), Client.throw_error(nested[1]["work"], "nope"),
          Client.throw_error(both[0]["work"], "E1"), Client.throw_error(both[1]["work"], "E3"),
          Client.complete_job(both[2]["work"]))
    for _ in range(3):
        dead = {r.key for r in ref.parts[0].log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_ERROR_THROWN}
        live = sorted(k for k in open_jobs(ref.parts[0].log) if k not in dead)
        if not live:
            break
        write(ref, gpu, *[Client.complete_job(k) for k in live])
    check(ref, gpu)
    log = gpu.parts[0].log.entries
    done = [r.value["elementId"] for r in log if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.intent == abi.PI_ELEMENT_COMPLETED]
    assert done.count("on-e1") == 2 and done.count("on-any") == 1 and done.count("inner") == 1
    assert done.count("b") == 1 and done.count("proc-esp") == 1
    assert [r for r in log if r.value_type == abi.VT_VARIABLE and r.value["name"] == "why"]
    assert not ad.fallback_reasons


# (random processes with error boundary events and one or two error-start event sub-processes; seeds whose
# campaigns run event sub-processes the most)
@pytest.mark.parametrize("seed", [1, 5, 10, 13, 16, 35, 37])
def test_random_processes_with_event_sub_processes(seed):
    import numpy as np
    from random_bpmn import random_process
    from test_gpu_error_events import random_error_campaign
    xml = random_process(np.random.default_rng(9000 + seed), sub_processes=True, task_kinds=True, errors=True,
                         event_sub_processes=True)
    deps = [(xml, KEY_A, 1)]
    ref, gpu = single(deps, deps, limit=100)
    random_error_campaign(seed, ref, lambda *r: write(ref, gpu, *r), xml)
    check(ref, gpu)
    assert gpu.parts[0].adapter.counts["device_commands"] >= 24 and not gpu.parts[0].adapter.fallback_reasons


def end_event_processes():
    # an error end event inside a sub-process caught by the sub-process's boundary event; one caught by the
    # process's event sub-process; an uncaught one (an incident on the end event)
    a = bpmn.createExecutableProcess("endBoundary").startEvent().subProcess("sub").startEvent("ss")
    a.serviceTask("work", "work").endEvent("throw").error("E").subProcessDone()
    a = a.boundaryEvent("caught").error("E").endEvent("caught-end").moveToActivity("sub").endEvent("end").done()
    b = bpmn.createExecutableProcess("endEsp")
    b.eventSubProcess("esp").startEvent("esp-start").error("E").serviceTask("recover", "recover").endEvent("esp-end")
    b = b.eventSubProcessDone().startEvent("s").serviceTask("work", "work").endEvent("throw").error("E").done()
    c = bpmn.createExecutableProcess("endUncaught").startEvent().serviceTask("work", "work").endEvent("throw").error("X").done()
    return a, b, c


@pytest.mark.parametrize("limit", [3, 100])
def test_error_end_events_in_the_processing_loop(limit):
    # the job completion that reaches an error end event hands the instance to the engine (the device
    # declines the command before any record), which throws the error: caught by a boundary event, by an
    # event sub-process, or an UNHANDLED_ERROR_EVENT incident on the end event
    a, b, c = end_event_processes()
    deps = [(a, KEY_A, 1), (b, KEY_B, 1), (c, KEY_C, 1)]
    ref, gpu = single(deps, deps, limit=limit)
    write(ref, gpu, *([Client.create("endBoundary") for _ in range(3)] + [Client.create("endEsp") for _ in range(3)] +
                      [Client.create("endUncaught") for _ in range(2)]))
    ad = gpu.parts[0].adapter
    assert ad.counts["device_commands"] >= 8
    for _ in range(3):
        live = sorted(open_jobs(ref.parts[0].log))
        if not live:
            break
        write(ref, gpu, *[Client.complete_job(k) for k in live])
    check(ref, gpu)
    log = gpu.parts[0].log.entries
    done = [r.value["elementId"] for r in log if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.intent == abi.PI_ELEMENT_COMPLETED]
    assert done.count("caught") == 3 and done.count("esp") == 3
    inc = [r for r in log if r.value_type == abi.VT_INCIDENT and r.intent == abi.INCIDENT_CREATED]
    assert len(inc) == 2 and all(r.value["elementId"] == "throw" for r in inc)
    assert ad.fallback_reasons and set(ad.fallback_reasons) == {"unsupported"}
