"""Job push of device jobs in the reference's processing loop (BpmnJobActivationBehavior.publishWork
:61-100; ActivatableJobsPushTest.java, pinned on the oracle by tests/test_oracle_job_push.py).

With a job stream open for a type (zbhip_set_job_stream on the device, the engine's JobStreamer on the
oracle engine), every job of that type the device creates is activated for the stream in the same batch:
the step kernel writes the push record right after JOB:CREATED, the host stores the activation (the
stream's worker and deadline) and expands the record into JOB_BATCH:ACTIVATED.  Time-outs and failures
with retries left push again.  The same workload runs through the loop over the engine alone and over
[adapter, engine]; every log and state equal, the pushed jobs completed and timed out like polled ones."""
import numpy as np
import pytest

from psm import Client, RecordingJobStream, open_jobs
from test_gpu_scheduled import KEY_A, KEY_B, check, single, step, write
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import JOB_BATCH_ACTIVATED, VT_JOB_BATCH

pytestmark = pytest.mark.gpu


def streams(ref, gpu, job_type, worker, timeout, on=True, fetch=()):
    """One job stream per side (the gateway's): the engine and the adapter of a partition push into it."""
    sinks = []
    for side, procs in ((ref, [ref.parts[0].engine]), (gpu, [gpu.parts[0].adapter, gpu.parts[0].engine])):
        stream = side.__dict__.setdefault("job_stream", RecordingJobStream())
        for p in procs:
            p.set_job_stream(job_type, worker, timeout, on, fetch_variables=fetch, push=stream.push)
        sinks.append(stream)
    return sinks


def pushed_equal(ref, gpu):
    assert gpu.job_stream.activated_jobs == ref.job_stream.activated_jobs


def notifiers(ref, gpu):
    """RecordingJobStreamer per side: the engine's and the adapter's notifyWorkAvailable side effects."""
    from psm import RecordingJobStreamer
    out = []
    for side, procs in ((ref, [ref.parts[0].engine]), (gpu, [gpu.parts[0].adapter, gpu.parts[0].engine])):
        side.streamer = RecordingJobStreamer()
        for p in procs:
            p.job_streamer = side.streamer
        out.append(side.streamer)
    return out


def notified_equal(ref, gpu):
    assert gpu.streamer.notifications == ref.streamer.notifications


def pushes(log):
    return [r for r in log.entries if r.value_type == VT_JOB_BATCH and r.intent == JOB_BATCH_ACTIVATED
            and r.value["maxJobsToActivate"] == -1]


def test_job_push_in_the_processing_loop():
    a = bpmn.linear_process(3)  # benchmark-task x3
    b = bpmn.linear_process(2, process_id="engineOnly", job_type="engine-task")
    deps = [(a, KEY_A, 1), (b, KEY_B, 1)]
    ref, gpu = single(deps, deps[:1])
    notifiers(ref, gpu)  # publishWork without a stream: JobStreamer.notifyWorkAvailable
    write(ref, gpu, *[Client.create("linear") for _ in range(4)])  # polled jobs, no stream yet
    notified_equal(ref, gpu)
    assert gpu.streamer.notifications == {"benchmark-task": 4}
    streams(ref, gpu, "benchmark-task", "pusher", 20000)
    streams(ref, gpu, "engine-task", "pusher", 20000, fetch=("n",))
    write(ref, gpu, *([Client.create("linear", (("n", i),) if i % 3 else ()) for i in range(12)] +
                      [Client.create("engineOnly", (("n", 7),)) for _ in range(2)]))
    pushed_equal(ref, gpu)
    assert any(j["variables"] == (("n", 4),) for _, j in gpu.job_stream.activated_jobs)
    log = gpu.parts[0].log
    pushed = pushes(log)
    assert len(pushed) == 14
    # pushed jobs are ACTIVATED: a poll only finds the four jobs created before the stream opened
    write(ref, gpu, Client.activate_jobs("benchmark-task", worker="poller", timeout=60000, max_jobs=50,
                                         timestamp=ref.clock.now))
    polled = [r for r in log.entries if r.value_type == VT_JOB_BATCH and r.value["maxJobsToActivate"] == 50][-1]
    assert len(polled.value["jobKeys"]) == 4
    # complete pushed jobs: the next task's job is pushed too
    keys = sorted(k for p in pushed for k in p.value["jobKeys"])
    write(ref, gpu, *[Client.complete_job(k, (("m", k % 5),)) for k in keys[:6]])
    assert len(pushes(log)) > 14
    pushed_equal(ref, gpu)
    # failures with retries left push again; without retries: the incident, no push
    live = sorted(k for p in pushes(log) for k in p.value["jobKeys"] if k in open_jobs(ref.parts[0].log))
    write(ref, gpu, Client.fail_job(live[0], 2, "retry me"), Client.fail_job(live[1], 0))
    # the deadlines pass: TIMED_OUT, then pushed again with a fresh deadline
    step(ref, gpu, 30000)
    timed_out = [r for r in log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_TIMED_OUT]
    assert timed_out
    pushed_equal(ref, gpu)
    # the stream closes: created jobs are activatable again
    streams(ref, gpu, "benchmark-task", "pusher", 20000, on=False)
    n = len(pushes(log))
    write(ref, gpu, *[Client.create("linear") for _ in range(3)])
    assert len(pushes(log)) == n
    rng = np.random.default_rng(5)
    for _ in range(6):
        live = sorted(open_jobs(ref.parts[0].log))
        if not live:
            break
        rng.shuffle(live)
        write(ref, gpu, *[Client.complete_job(k) for k in live])
    check(ref, gpu)
    pushed_equal(ref, gpu)
    notified_equal(ref, gpu)  # creations, time-outs and failures with retries after the stream closed
    assert gpu.streamer.notifications["benchmark-task"] > 4


def test_push_survives_a_restart():
    """The stored activation of a pushed job (worker, deadline) is in the exported state."""
    a = bpmn.linear_process(2)
    ref, gpu = single([(a, KEY_A, 1)], [(a, KEY_A, 1)])
    streams(ref, gpu, "benchmark-task", "pusher", 15000)
    write(ref, gpu, *[Client.create("linear") for _ in range(5)])
    from zeebe_amd.engine import Partition
    part = gpu.parts[0].adapter.part
    fresh = Partition(max_instances=256, max_commands=48)
    fresh.deploy(a, process_definition_key=KEY_A)
    fresh.import_state_db(part.state_db())
    assert fresh.state() == part.state()
    assert any("|ACTIVATED" in r for r in part.state() if r.startswith("JOB_STATES|"))


def test_push_reads_the_variables_at_its_creation():
    """publishWork collects the pushed job's variables when JOB:CREATED is written (BpmnJobActivationBehavior
    .java:83): a later command of the same instance -- here a parallel branch's completion with a document,
    read in the same log window -- must not leak into the pushed job.  The adapter keeps such commands out
    of the pushing window (adapter.py _push_fenced)."""
    xml = (bpmn.createExecutableProcess("forked").startEvent("start").parallelGateway("fork")
           .serviceTask("a", "a").serviceTask("p", "pushed").sequenceFlowId("j1").parallelGateway("join")
           .moveToNode("fork").serviceTask("b", "b").sequenceFlowId("j2").connectTo("join")
           .moveToNode("join").endEvent("end").done())
    ref, gpu = single([(xml, KEY_A, 1)], [(xml, KEY_A, 1)])
    streams(ref, gpu, "pushed", "pusher", 20000)
    write(ref, gpu, *[Client.create("forked", (("n", i),)) for i in range(6)])
    jobs = open_jobs(ref.parts[0].log)
    by_type = {}
    for k, r in sorted(jobs.items()):
        by_type.setdefault(r.value["type"], []).append((r.value["processInstanceKey"], k))
    a, b = dict(by_type["a"]), dict(by_type["b"])
    # one window: task a's completion (task p's job created and pushed), then b's with a document
    recs = []
    for pik in sorted(a):
        recs += [Client.complete_job(a[pik]), Client.complete_job(b[pik], (("n", 1000 + pik % 7),))]
    write(ref, gpu, *recs)
    pushed_equal(ref, gpu)
    assert len(gpu.job_stream.activated_jobs) == 6
    assert all(dict(j["variables"])["n"] < 1000 for _, j in gpu.job_stream.activated_jobs)
    assert gpu.parts[0].adapter.counts["windows"] >= 6
    live = sorted(open_jobs(ref.parts[0].log))
    write(ref, gpu, *[Client.complete_job(k) for k in live])
    check(ref, gpu)
