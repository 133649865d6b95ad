"""Error boundary events in the reference's processing loop.  A process whose job worker tasks carry error
boundary events runs on the device (the boundary subscribes to nothing); a JOB:THROW_ERROR of a device job
moves the instance to the engine first (the adapter's held-instance hand-off: its zb-db rows -- the task's
event scope with the boundary event among its interrupting and boundary ids -- into the engine's state),
whose JobThrowErrorProcessor then catches it at the boundary event or raises UNHANDLED_ERROR_EVENT
(oracle pinned by tests/test_oracle_error_events.py).  The same workload through the loop over the engine
alone and through [adapter, engine]: every log and state equal, at batch limits 3 and 100."""
import pytest

from psm import Client, open_jobs
from test_gpu_scheduled import KEY_A, KEY_B, check, single, write
from zeebe_amd import abi, bpmn

pytestmark = pytest.mark.gpu


def processes():
    a = (bpmn.createExecutableProcess("errors").startEvent("start").serviceTask("task", "work")
         .boundaryEvent("on-error").error("E1").serviceTask("recover", "recover").endEvent("end-error")
         .moveToActivity("task").serviceTask("next", "work-2").endEvent("end").done())
    b = (bpmn.createExecutableProcess("catchAll").startEvent("s").serviceTask("t", "work")
         .boundaryEvent("any").error().endEvent("e2").moveToActivity("t").endEvent("e1").done())
    return a, b


@pytest.mark.parametrize("limit", [3, 100])
def test_error_boundary_events_in_the_processing_loop(limit):
    a, b = processes()
    deps = [(a, KEY_A, 1), (b, KEY_B, 1)]
    ref, gpu = single(deps, deps, limit=limit)
    write(ref, gpu, *([Client.create("errors") for _ in range(10)] + [Client.create("catchAll") for _ in range(4)]))
    assert gpu.parts[0].adapter.counts["device_commands"] >= 14
    jobs = sorted(k for k, r in open_jobs(ref.parts[0].log).items() if r.value["type"] == "work")
    # caught (code-specific / catch-all), with variables, uncaught (incident), rejections, completions
    write(ref, gpu, Client.throw_error(jobs[0], "E1"), Client.throw_error(jobs[1], "E1", "with message"),
          Client.throw_error(jobs[2], "E1", "", variables=(("reason", "bad"),)),
          Client.throw_error(jobs[3], "other", "not caught"), Client.throw_error(jobs[10], "anything"),
          Client.throw_error(123, "E1"), Client.complete_job(jobs[4]))
    write(ref, gpu, Client.throw_error(jobs[3], "E1"), Client.complete_job(jobs[5]), Client.throw_error(jobs[4], "E1"))
    # the recovering and the remaining tasks complete
    for _ in range(3):
        live = sorted(k for k, r in open_jobs(ref.parts[0].log).items() if r.value["type"] != "work" or k in jobs[6:10])
        if not live:
            break
        write(ref, gpu, *[Client.complete_job(k) for k in live])
    check(ref, gpu)
    log = gpu.parts[0].log.entries
    thrown = [r for r in log if r.value_type == abi.VT_JOB and r.intent == abi.JOB_ERROR_THROWN]
    assert len(thrown) == 5
    assert any(r.value["elementId"] == "NO_CATCH_EVENT_FOUND" for r in thrown)
    assert [r for r in log if r.value_type == abi.VT_INCIDENT and r.value["errorType"] == "UNHANDLED_ERROR_EVENT"]
    assert [r for r in log if r.value_type == abi.VT_VARIABLE and r.value["name"] == "reason"]
    done = sum(1 for r in log if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_COMPLETED
               and r.value["bpmnElementType"] == "PROCESS")
    assert done == 10  # (the incident instance waits; three catchAll tasks stay open)
    ad = gpu.parts[0].adapter
    # one hand-off per thrown error (a throw for a completed job still resolving to its running instance moves
    # that instance too: the engine rejects it, NOT_FOUND), no declines
    assert 5 <= len(ad.handed_off) <= 6 and not ad.fallback_reasons


@pytest.mark.parametrize("limit", [3, 100])
def test_error_boundary_events_on_sub_processes_in_the_processing_loop(limit):
    # ErrorEventIncidentTest.BOUNDARY_EVENT_SUBPROCESS: caught inside, at the sub-process, or nowhere; the
    # hand-off carries the sub-process's event scope (its boundary event among its interrupting ids)
    from test_oracle_error_events import sub_process_boundaries
    deps = [(sub_process_boundaries(), KEY_A, 1)]
    ref, gpu = single(deps, deps, limit=limit)
    write(ref, gpu, *[Client.create("wf") for _ in range(6)])
    assert gpu.parts[0].adapter.counts["device_commands"] >= 6
    jobs = sorted(open_jobs(ref.parts[0].log))
    write(ref, gpu, Client.throw_error(jobs[0], "error_in_subprocess"), Client.throw_error(jobs[1], "error"),
          Client.throw_error(jobs[2], "error", "", variables=(("why", "x"),)), Client.throw_error(jobs[3], "nope"),
          Client.complete_job(jobs[4]))
    write(ref, gpu, *[Client.complete_job(k) for k in sorted(open_jobs(ref.parts[0].log))])
    check(ref, gpu)
    log = gpu.parts[0].log.entries
    done = [r.value["elementId"] for r in log if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.intent == abi.PI_ELEMENT_COMPLETED]
    assert done.count("wf") == 5 and done.count("end_boundary") == 2 and done.count("end_boundary_in_subprocess") == 1
    assert [r for r in log if r.value_type == abi.VT_VARIABLE and r.value["name"] == "why"]
    ad = gpu.parts[0].adapter
    assert len(ad.handed_off) == 4 and not ad.fallback_reasons


def random_error_campaign(seed, ref, emit, xml, rounds=30, n=24):
    """tests/random_bpmn.py processes with error boundary events (tasks, sub-processes; codes E1 / E2 or
    catch-all): every round each open job is completed, left, or gets an error thrown with E1, E2 or E3
    (caught by its code, by a catch-all, or nowhere: an incident) -- half of the jobs of tasks with an error
    boundary event, one in twelve of the others."""
    import re
    import numpy as np
    from psm import Client as C
    guarded = set(re.findall(r'attachedToRef="([^"]+)"><errorEventDefinition', xml))
    rng = np.random.default_rng(seed)
    emit(*[C.create("random", variables=(("amount", int(a)),)) for a in rng.integers(0, 1000, n)])
    thrown = 0
    for _ in range(rounds):
        log = ref.parts[0].log
        dead = {r.key for r in log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_ERROR_THROWN}
        jobs = sorted((k, r.value["elementId"]) for k, r in open_jobs(log).items() if k not in dead)
        if not jobs:
            break
        cmds = []
        for k, elem in jobs:
            m = int(rng.integers(0, 12))
            if m == 0:
                continue
            if m <= (6 if elem in guarded else 1):
                thrown += 1
                cmds.append(C.throw_error(k, ("E1", "E1", "E2", "E2", "E3")[int(rng.integers(0, 5))]))
            else:
                cmds.append(C.complete_job(k))
        emit(*cmds)
    return thrown


# (seeds whose processes hold three or more error boundary events; 3, 4, 9, 29: on sub-processes too)
@pytest.mark.parametrize("seed", [0, 3, 4, 7, 9, 19, 29, 36])
def test_random_processes_with_error_boundary_events(seed):
    import numpy as np
    from random_bpmn import random_process
    xml = random_process(np.random.default_rng(9000 + seed), sub_processes=True, task_kinds=True, errors=True)
    deps = [(xml, KEY_A, 1)]
    ref, gpu = single(deps, deps, limit=100)
    random_error_campaign(seed, ref, lambda *r: write(ref, gpu, *r), xml)
    check(ref, gpu)
    assert not gpu.parts[0].adapter.fallback_reasons


@pytest.mark.parametrize("limit", [3, 100])
def test_several_boundary_events_on_one_task_in_the_processing_loop(limit):
    # two error boundary events (a catch-all and a code-specific one) and a timer boundary event on one task:
    # the timer stays the device's (TIMER:CREATED with the task), the event scope lists all three; thrown
    # errors go to the code-specific or the catch-all boundary event, canceling the timer; some timers fire
    from test_oracle_error_events import two_boundaries
    deps = [(two_boundaries(("catch-all", None), ("code-specific", "E"), timer="PT10S"), KEY_A, 1)]
    ref, gpu = single(deps, deps, limit=limit)
    write(ref, gpu, *[Client.create("wf") for _ in range(8)])
    jobs = sorted(open_jobs(ref.parts[0].log))
    write(ref, gpu, Client.throw_error(jobs[0], "E"), Client.throw_error(jobs[1], "other"),
          Client.complete_job(jobs[2]))
    from test_gpu_scheduled import step
    step(ref, gpu, 11000)
    check(ref, gpu)
    log = gpu.parts[0].log.entries
    caught = [r.value["elementId"] for r in log if r.value_type == abi.VT_PROCESS_INSTANCE
              and r.intent == abi.PI_ELEMENT_COMPLETED and r.value["bpmnElementType"] == "BOUNDARY_EVENT"]
    assert sorted(caught) == ["catch-all", "code-specific"] + ["timer"] * 5
    ad = gpu.parts[0].adapter
    assert len(ad.handed_off) == 2 and not ad.fallback_reasons


@pytest.mark.parametrize("limit", [3, 100])
def test_error_boundary_events_on_multi_instance_activities_in_the_processing_loop(limit):
    # an error boundary event of a multi-instance task attaches to its body (ErrorCatchEventTest "boundary event
    # on multi-instance service task"): parallel and sequential bodies; a throw terminates the body with its
    # other inner instances (their jobs canceled) and activates the boundary event
    par = (bpmn.createExecutableProcess("par").startEvent().serviceTask("task", "work").multiInstance("= [1, 2, 3]", "x")
           .boundaryEvent("caught").error("E").endEvent("ce").moveToActivity("task").endEvent("end").done())
    seq = (bpmn.createExecutableProcess("seq").startEvent().serviceTask("task", "work").multiInstance("= [1, 2]", "x", True)
           .boundaryEvent("caught").error().endEvent("ce").moveToActivity("task").endEvent("end").done())
    deps = [(par, KEY_A, 1), (seq, KEY_B, 1)]
    ref, gpu = single(deps, deps, limit=limit)
    write(ref, gpu, *([Client.create("par") for _ in range(4)] + [Client.create("seq") for _ in range(4)]))
    by = {}
    for k, r in open_jobs(ref.parts[0].log).items():
        by.setdefault(r.value["processInstanceKey"], []).append(k)
    inst = [sorted(by[p]) for p in sorted(by)]
    write(ref, gpu, Client.throw_error(inst[0][1], "E", "", variables=(("why", "x"),)), Client.throw_error(inst[1][0], "Z"),
          Client.complete_job(inst[2][0]), Client.throw_error(inst[4][0], "any"), Client.complete_job(inst[5][0]))
    for _ in range(4):
        dead = {r.key for r in ref.parts[0].log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_ERROR_THROWN}
        live = sorted(k for k in open_jobs(ref.parts[0].log) if k not in dead)
        if not live:
            break
        write(ref, gpu, *[Client.complete_job(k) for k in live])
    check(ref, gpu)
    log = gpu.parts[0].log.entries
    done = [r.value["elementId"] for r in log if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.intent == abi.PI_ELEMENT_COMPLETED]
    assert done.count("caught") == 2
    assert [r for r in log if r.value_type == abi.VT_JOB and r.intent == abi.JOB_CANCELED]
    assert not gpu.parts[0].adapter.fallback_reasons
