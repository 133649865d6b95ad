"""JOB:FAIL of device jobs in the reference's processing loop (JobFailProcessor.java:79-162 through
zbhip_fail_job; JobFailedApplier -> DbJobState.fail).

The same workload runs through the loop over the engine alone (the oracle engine, pinned on FailJobTest
and JobFailIncidentTest by tests/test_oracle_job_failures.py) and through [adapter, engine] with the
scheduled tasks of tests/test_gpu_scheduled.py: failures with retries left (ACTIVATABLE again, the next
activation and the later JOB:COMPLETED / JOB:TIMED_OUT records carry the stored retries and errorMessage),
failures without (JOB:FAILED + INCIDENT:CREATED JOB_NO_RETRIES on the device, then the instance waits for
the incident's resolution on the engine), failures outside the device subset (variables: the engine's,
after the hand-off), and the rejections.  Every log and state equal; a restart keeps the stored fields."""
import numpy as np
import pytest

from psm import Client, open_jobs
from test_gpu_scheduled import KEY_A, KEY_B, check, single, step, write
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import JOB_BATCH_ACTIVATED, VT_JOB_BATCH

pytestmark = pytest.mark.gpu


def test_job_failures_in_the_processing_loop():
    a = bpmn.linear_process(3)
    b = bpmn.linear_process(2, process_id="engineOnly", job_type="engine-task")
    deps = [(a, KEY_A, 1), (b, KEY_B, 1)]
    ref, gpu = single(deps, deps[:1])
    from test_gpu_job_push import notified_equal, notifiers
    notifiers(ref, gpu)  # failures with retries left (and time-outs) notify the job type again
    write(ref, gpu, *([Client.create("linear") for _ in range(12)] + [Client.create("engineOnly") for _ in range(2)]))
    clock = ref.clock
    write(ref, gpu, Client.activate_jobs("benchmark-task", worker="w1", timeout=60000, max_jobs=6, timestamp=clock.now))
    jobs = sorted(k for k, r in open_jobs(ref.parts[0].log).items() if r.value["bpmnProcessId"] == "linear")
    # retries left (activated / never activated), none left (incidents), outside the subset, rejections
    write(ref, gpu, Client.fail_job(jobs[0], 2, "boom, with|separators"), Client.fail_job(jobs[1], 0),
          Client.fail_job(jobs[7], 1), Client.fail_job(jobs[8], 0, "custom message"),
          Client.fail_job(jobs[9], 3, "", variables=(("reason", 7),)), Client.fail_job(123, 3),
          # StringUtil.limitString counts UTF-16 code units: the cut falls inside a surrogate pair
          Client.fail_job(jobs[3], 1, "a" + "\U0001D11E" * 5000))
    write(ref, gpu, Client.fail_job(jobs[1], 3), Client.complete_job(jobs[8]))
    log = gpu.parts[0].log
    incidents = [r for r in log.entries if r.value_type == abi.VT_INCIDENT]
    assert len(incidents) == 2 and {r.value["errorMessage"] for r in incidents} == {"No more retries left.",
                                                                                      "custom message"}
    assert any(r.value.get("errorMessage", "").endswith("?...") for r in log.entries
               if r.value_type == abi.VT_JOB and r.intent == abi.JOB_FAILED)
    rej = [r for r in log.entries if r.record_type == abi.RT_REJECTION and r.value_type == abi.VT_JOB]
    assert len(rej) == 3
    ad = gpu.parts[0].adapter
    assert ad.counts["job_failures"] == 5 and len(ad.handed_off) == 3  # two incidents + the variables' failure
    # the failed jobs with retries left are activated again (their retries), completed or timed out
    write(ref, gpu, Client.activate_jobs("benchmark-task", worker="w2", timeout=10000, max_jobs=20, timestamp=clock.now))
    batch = [r for r in log.entries if r.value_type == VT_JOB_BATCH and r.intent == JOB_BATCH_ACTIVATED]
    assert any(j["retries"] == 2 for r in batch for j in r.value["jobs"])
    # restart: the stored retries / errorMessage of ACTIVATABLE and ACTIVATED failed jobs survive
    from zeebe_amd.engine import Partition
    part = ad.part
    fresh = Partition(max_instances=256, max_commands=48)
    fresh.deploy(a, process_definition_key=KEY_A)
    fresh.import_state_db(part.state_db())
    assert fresh.state() == part.state()
    step(ref, gpu, 30000)  # the w2 activations time out: TIMED_OUT carries the failure's fields
    timed_out = [r for r in log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_TIMED_OUT]
    assert any(r.value.get("errorMessage") == "boom, with|separators" for r in timed_out)
    rng = np.random.default_rng(3)
    for _ in range(4):
        live = sorted(k for k, r in open_jobs(ref.parts[0].log).items())
        if not live:
            break
        rng.shuffle(live)
        write(ref, gpu, *[Client.complete_job(k) for k in live])
    completed = [r for r in log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_COMPLETED]
    assert any(r.value.get("retries") == 2 and r.value.get("errorMessage") for r in completed)
    check(ref, gpu)
    notified_equal(ref, gpu)
