"""Job activation on the CPU oracle, pinned to the reference's ActivateJobsTest
(engine/src/test/java/io/camunda/zeebe/engine/processing/job/ActivateJobsTest.java): the three
rejection texts (:74-115), one job with its variables (:141-187), batches in job-key order
(:190-218, :247-265), completing activated jobs (:230-244); and the state the activation leaves
(JobBatchActivatedApplier -> DbJobState.activate: JOB_STATES ACTIVATED, JOB_DEADLINES, no
JOB_ACTIVATABLE).  The product's rejection text function (host code) is checked here too."""
import ctypes as C

import numpy as np

from helpers import create_commands, string_docs
from oracle.oracle import Oracle
from zeebe_amd import abi, bpmn
from zeebe_amd.native import load

TYPE = "test-task"


def _engine(n, xml=None, docs=None):
    o = Oracle()
    o.deploy(xml or bpmn.linear_process(1, job_type=TYPE))
    c = create_commands(n)
    if docs is not None:
        c["doc_count"] = 1
        c["doc_begin"] = np.arange(n)
    o.submit(c, docs)
    o.run()
    recs = o.records()
    o.clear_records()
    jobs = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    return o, jobs


def _reason(max_jobs, timeout, job_type):
    L = load()
    t = job_type.encode()
    cmd = abi.JobActivation(type=t, type_len=len(t), worker=b"w", worker_len=1, timeout=timeout, max_jobs=max_jobs)
    reason = 1 if max_jobs < 1 else 2 if timeout < 1 else 3
    res = abi.JobBatch(key=-1, rejection_type=abi.REJ_INVALID_ARGUMENT, reason=reason)
    buf = C.create_string_buffer(256)
    L.zbhip_job_batch_rejection_reason(C.byref(cmd), C.byref(res), buf, 256)
    return reason, buf.value.decode()


def test_rejections():
    o, _ = _engine(1)
    assert o.activate_jobs(TYPE, max_jobs=0)[2] == 1
    assert o.activate_jobs(TYPE, timeout=0)[2] == 2
    assert o.activate_jobs("", max_jobs=3)[2] == 3
    assert _reason(0, 1000, TYPE)[1] == (
        "Expected to activate job batch with max jobs to activate to be greater than zero, but it was '0'")
    assert _reason(3, 0, TYPE)[1] == "Expected to activate job batch with timeout to be greater than zero, but it was '0'"
    assert _reason(3, 1000, "")[1] == "Expected to activate job batch with type to be present, but it was blank"
    # a rejected command generates no key
    assert o.key_counter() == _engine(1)[0].key_counter()


def test_activate_single_job_with_variables():
    # shouldActivateSingleJob: three instances with {'foo': 'bar'}, maxJobsToActivate 1
    o = Oracle()
    o.deploy(bpmn.linear_process(1, job_type=TYPE))
    foo = o.intern("foo")
    bar = o.intern_string("bar")
    c = create_commands(3)
    c["doc_count"] = 1
    c["doc_begin"] = np.arange(3)
    o.submit(c, string_docs(foo, [bar] * 3))
    o.run()
    recs = o.records()
    first = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED][0]
    key, jobs, reason = o.activate_jobs(TYPE, worker="myTestWorker", timeout=12 * 60 * 1000, max_jobs=1, timestamp=1000)
    assert reason == 0 and key > 0 and len(jobs) == 1
    j = jobs[0]
    assert int(j["key"]) == first and int(j["retries"]) == 3
    assert int(j["deadline"]) == 1000 + 12 * 60 * 1000
    assert int(j["n_variables"]) == 1
    v = j["variables"][0]
    assert (int(v["name_id"]), int(v["type"]), int(v["value"])) == (foo, abi.DOC_STR, bar)
    state = o.state()
    assert "JOB_STATES|%d|ACTIVATED" % first in state
    assert "JOB_DEADLINES|%d|%d" % (1000 + 720000, first) in state
    assert not any(r.startswith("JOB_ACTIVATABLE|") and r.endswith("|%d" % first) for r in state)
    assert any(r.startswith("JOBS|%d|" % first) and r.endswith("worker=myTestWorker") for r in state)


def test_activate_job_batches_in_key_order():
    # shouldActivateJobBatches: 12 jobs, batches of 3, 4, 3 take them in order
    o, keys = _engine(12)
    got = [[int(j["key"]) for j in o.activate_jobs(TYPE, max_jobs=m)[1]] for m in (3, 4, 3)]
    assert got == [keys[0:3], keys[3:7], keys[7:10]]
    # shouldReturnEmptyBatchIfNoJobsAvailable
    key, jobs, reason = o.activate_jobs("no-such-type", max_jobs=3)
    assert reason == 0 and key > 0 and len(jobs) == 0


def test_only_jobs_of_the_type():
    # shouldOnlyReturnJobsOfCorrectType: the jobs of the type, in key order
    o = Oracle()
    o.deploy(bpmn.linear_process(1, process_id="a", job_type=TYPE))
    o.deploy(bpmn.linear_process(1, process_id="b", job_type="different" + TYPE))
    o.submit(np.concatenate([create_commands(3, 0), create_commands(5, 1, 3), create_commands(4, 0, 8)]))
    o.run()
    recs = o.records()
    want = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED
            and int(r["process_idx"]) == 0]
    assert [int(j["key"]) for j in o.activate_jobs(TYPE, max_jobs=7)[1]] == want


def test_complete_activated_jobs():
    o, keys = _engine(5)
    jobs = o.activate_jobs(TYPE, max_jobs=5)[1]
    c = abi.make_commands(5)
    c["instance"] = np.arange(5)
    c["kind"] = abi.CMD_JOB_COMPLETE
    c["ref"] = 5  # the job key ordinal of linear-1 (App. A.1)
    o.clear_records()
    o.submit(c)
    o.run()
    recs = o.records()
    done = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_COMPLETED]
    assert sorted(done) == sorted(keys) == sorted(int(j["key"]) for j in jobs)
    assert [r for r in o.state() if r.startswith(("JOBS|", "JOB_STATES|", "JOB_DEADLINES|"))] == []
