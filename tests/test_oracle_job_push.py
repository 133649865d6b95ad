"""The oracle's job push (zb_oracle.cpp publish_work; BpmnJobActivationBehavior.publishWork :61-100) pinned
on the reference's ActivatableJobsPushTest (engine/src/test/.../processing/job/ActivatableJobsPushTest.java):
with a job stream of the type open, a created job is activated for the stream in the same batch
(JOB:CREATED then JOB_BATCH:ACTIVATED), and again after a time-out (:155-170) and after a failure with
retries left (:172-187).  Run through the restated processing loop over the oracle engine (tests/psm.py)."""
from psm import Client, Clock, Log, OracleEngine, Rec, RecordingJobStream, StreamProcessor
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import JOB_BATCH_ACTIVATED, VT_JOB_BATCH

KEY = 2251799813685249
TIMEOUT = 30000  # ActivatableJobsPushTest.setUp: timeout 30000L, worker "test", fetchVariables a, b, c
# (the reference's Map.of("a", .., "b", .., "c", ..) document: one entry here -- the oracle refuses
# multi-entry documents, whose msgpack iteration order is unpinned)
VARIABLES = (("a", "valA"),)


def loop(clock=None):
    log = Log()
    eng = OracleEngine(clock=clock or 0)
    eng.deploy(bpmn.linear_process(1, process_id="process", job_type="pushed"), KEY, 1)
    eng.job_stream = RecordingJobStream()
    eng.set_job_stream("pushed", "test", TIMEOUT, fetch_variables=("a", "b", "c"), push=eng.job_stream.push)
    sp = StreamProcessor(log, [eng])
    return log, eng, sp


def assert_activated_job(eng, job_key, activation_count):
    # assertActivatedJob (:258-272): every push of the job, the stream's worker, the variables
    jobs = eng.job_stream.activated_jobs
    assert len(jobs) == activation_count
    for key, job in jobs:
        assert key == job_key
        assert (job["worker"], dict(job["variables"]), job["tenantId"]) == ("test", dict(VARIABLES), "<default>")


def run(log, sp, *recs):
    start = len(log.entries)
    Client(log).write(*recs)
    sp.run()
    return log.entries[start:]


def order(entries):
    return [(r.value_type, r.intent) for r in entries if r.record_type == abi.RT_EVENT
            and r.value_type in (abi.VT_JOB, VT_JOB_BATCH)]


def pushes(entries):
    return [r for r in entries if r.value_type == VT_JOB_BATCH and r.intent == JOB_BATCH_ACTIVATED]


def test_push_when_job_created():
    # shouldPushWhenJobCreated (:101-118): one job in the batch, CREATED before ACTIVATED
    log, eng, sp = loop()
    entries = run(log, sp, Client.create("process", VARIABLES))
    assert order(entries) == [(abi.VT_JOB, abi.JOB_CREATED), (VT_JOB_BATCH, JOB_BATCH_ACTIVATED)]
    created = [r for r in entries if r.value_type == abi.VT_JOB][0]
    batch = pushes(entries)[0]
    v = batch.value
    assert v["jobKeys"] == (created.key,) and len(v["jobs"]) == 1
    assert (v["type"], v["worker"], v["timeout"], v["maxJobsToActivate"]) == ("pushed", "test", TIMEOUT, -1)
    job = v["jobs"][0]
    assert (job["worker"], job["deadline"]) == ("test", TIMEOUT)
    assert "JOB_STATES|%d|ACTIVATED" % created.key in eng.state()
    assert_activated_job(eng, created.key, 1)
    # the pushed job is not activatable: a poll finds nothing
    polled = run(log, sp, Client.activate_jobs("pushed"))[-1]
    assert polled.value["jobKeys"] == ()


def test_push_for_multiple_jobs_created():
    # shouldPushForMultipleJobsCreated (:120-153): every job its own push
    log, eng, sp = loop()
    entries = run(log, sp, *[Client.create("process") for _ in range(3)])
    created = [r.key for r in entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_CREATED]
    assert [p.value["jobKeys"] for p in pushes(entries)] == [(k,) for k in created]
    assert len({p.key for p in pushes(entries)}) == 3


def test_push_when_job_times_out():
    # shouldPushWhenJobTimesOut (:155-170): TIME_OUT, TIMED_OUT, ACTIVATED
    clock = Clock(0)
    log, eng, sp = loop(clock)
    job_key = pushes(run(log, sp, Client.create("process", VARIABLES)))[0].value["jobKeys"][0]
    clock.now += TIMEOUT + 1
    entries = run(log, sp, _time_out(job_key))
    assert order(entries)[-2:] == [(abi.VT_JOB, abi.JOB_TIMED_OUT), (VT_JOB_BATCH, JOB_BATCH_ACTIVATED)]
    again = pushes(entries)[0].value["jobs"][0]
    assert again["deadline"] == clock.now + TIMEOUT
    assert_activated_job(eng, job_key, 2)


def _time_out(job_key):
    # JobTimeoutTrigger's command (JobTimeoutCheckerScheduler: JOB:TIME_OUT with the job's value)
    return Rec(abi.RT_COMMAND, abi.VT_JOB, abi.JOB_TIME_OUT, job_key, {"tenantId": "<default>"})


def test_push_after_job_failed():
    # shouldPushAfterJobFailed (:172-187): FAIL, FAILED, ACTIVATED; no push without retries
    log, eng, sp = loop()
    run(log, sp, Client.create("process", VARIABLES), Client.create("process", VARIABLES))
    a, b = [p.value["jobKeys"][0] for p in pushes(log.entries)]
    entries = run(log, sp, Client.fail_job(a, 5, "again"))
    assert order(entries) == [(abi.VT_JOB, abi.JOB_FAILED), (VT_JOB_BATCH, JOB_BATCH_ACTIVATED)]
    job = pushes(entries)[0].value["jobs"][0]
    assert (job["retries"], job["errorMessage"]) == (5, "again")
    assert [k for k, _ in eng.job_stream.activated_jobs] == [a, b, a]
    entries = run(log, sp, Client.fail_job(b, 0))
    assert not pushes(entries) and [r for r in entries if r.value_type == abi.VT_INCIDENT]


def test_no_push_once_the_stream_is_gone():
    log, eng, sp = loop()
    eng.set_job_stream("pushed", "test", TIMEOUT, on=False)
    entries = run(log, sp, Client.create("process"))
    assert order(entries) == [(abi.VT_JOB, abi.JOB_CREATED)]


# ---- notifyWorkAvailable: ActivatableJobsNotificationTests.java (engine/src/test/.../processing/job/) -------
def notifying_loop(clock=None, job_type="task"):
    from psm import RecordingJobStreamer
    log = Log()
    eng = OracleEngine(clock=clock or 0)
    eng.deploy(bpmn.linear_process(1, process_id="process", job_type=job_type), KEY, 1)
    eng.job_streamer = RecordingJobStreamer()
    return log, eng, StreamProcessor(log, [eng])


def test_notify_when_job_created():
    # shouldNotifyWhenJobCreated (:67-74): three jobs, three notifications of the type
    log, eng, sp = notifying_loop()
    run(log, sp, *[Client.create("process") for _ in range(3)])
    assert eng.job_streamer.notifications == {"task": 3}


def test_notify_when_jobs_available_again_and_after_time_out():
    # shouldNotifyWhenJobsAvailableAgain (:76-87): create, activate, create -> 2;
    # shouldNotifyWhenJobsAvailableAfterTimeOut (:101-113): the time-out makes it activatable -> 2
    clock = Clock(0)
    log, eng, sp = notifying_loop(clock)
    run(log, sp, Client.create("process"))
    job_key = run(log, sp, Client.activate_jobs("task", timeout=10))[-1].value["jobKeys"][0]
    run(log, sp, Client.create("process"))
    assert eng.job_streamer.notifications == {"task": 2}
    clock.now += 100
    run(log, sp, _time_out(job_key))
    assert eng.job_streamer.notifications == {"task": 3}


def test_notify_when_jobs_fail_with_retries_available():
    # shouldNotifyWhenJobsFailWithRetryAvailable (:129-141): FAIL with retries -> 2; none left: no notification
    log, eng, sp = notifying_loop()
    run(log, sp, Client.create("process"), Client.create("process"))
    a, b = [r.key for r in log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_CREATED]
    run(log, sp, Client.fail_job(a, 10))
    assert eng.job_streamer.notifications == {"task": 3}
    run(log, sp, Client.fail_job(b, 0))
    assert eng.job_streamer.notifications == {"task": 3}


def test_notify_per_job_type_and_not_with_a_stream():
    # shouldNotifyForMultipleJobTypes (:164-175); a type with a stream is pushed instead (publishWork)
    log, eng, sp = notifying_loop(job_type="first")
    eng.deploy(bpmn.linear_process(1, process_id="second", job_type="second"), KEY + 1, 1)
    eng.set_job_stream("second", "w", TIMEOUT)
    run(log, sp, Client.create("process"), Client.create("second"))
    assert eng.job_streamer.notifications == {"first": 1}
