"""Job activation on the gfx950 path: JOB_BATCH:ACTIVATE over the GPU-resident
job rows (zbhip_activate_jobs: the host's JOB_ACTIVATABLE index picks the jobs, k_activate_jobs marks
them ACTIVATED and gathers their element instances and variables) against the CPU oracle
(JobBatchActivateProcessor.java:60-143, JobBatchCollector.java:67-123, JobBatchActivatedApplier.java,
DbJobState.activate :118-133; the oracle is pinned by tests/test_oracle_jobs.py on ActivateJobsTest).

Bar: batch key, job keys (in order), element instance / process instance keys, deadline, retries,
variables, and afterwards every window's records and the exported state (canonical rows and zb-db
bytes, JOB_STATES ACTIVATED / JOB_DEADLINES included) equal to the oracle's."""
import numpy as np
import pytest

from helpers import amount_docs, create_commands, string_docs
from oracle import statedb as SD
from oracle.oracle import Oracle
from test_gpu_parity import assert_same_records
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu

JOB_FIELDS = ["key", "element_instance_key", "process_instance_key", "deadline", "process_idx", "element_idx",
              "retries", "n_variables"]


def same_batch(g, o):
    gk, gj, gr = g
    ok_, oj, orr = o
    assert (gk, gr) == (ok_, orr)
    assert len(gj) == len(oj)
    for f in JOB_FIELDS:
        assert np.array_equal(gj[f], oj[f]), f
    for a, b in zip(gj, oj):
        n = int(a["n_variables"])
        for f in ("name_id", "type", "value"):
            assert np.array_equal(a["variables"][:n][f], b["variables"][:n][f]), f


def window(part, orc, cmds, docs=None):
    part.submit(cmds, docs)
    part.run()
    got = part.drain()
    orc.clear_records()
    orc.submit(cmds, docs)
    orc.run()
    assert_same_records(got, orc.records(), part, orc)
    assert part.fallback() == []
    return got


def same_state(part, orc):
    assert part.state() == orc.state()
    strings = orc.strings()
    assert part.state_db() == SD.encode_rows(orc.state(), orc.process_tables(), lambda i: strings[i])


def completions(part, keys):
    c = abi.make_commands(len(keys))
    for i, k in enumerate(keys):
        c[i]["instance"], c[i]["ref"] = part.resolve_key(int(k))
    c["kind"] = abi.CMD_JOB_COMPLETE
    return c


def test_activate_single_job_with_variables():
    part, orc = Partition(max_instances=8, max_commands=8), Oracle()
    for e in (part, orc):
        e.deploy(bpmn.linear_process(1, job_type="test-task"))
    foo = part.intern("foo")
    assert orc.intern("foo") == foo
    bar = part.intern_string("bar")
    assert orc.intern_string("bar") == bar
    c = create_commands(3)
    c["doc_count"] = 1
    c["doc_begin"] = np.arange(3)
    window(part, orc, c, string_docs(foo, [bar] * 3))
    args = dict(worker="myTestWorker", timeout=720000, max_jobs=1, timestamp=1000)
    same_batch(part.activate_jobs("test-task", **args), orc.activate_jobs("test-task", **args))
    same_state(part, orc)
    # invalid commands: INVALID_ARGUMENT, no key
    for bad in (dict(max_jobs=0), dict(timeout=0)):
        same_batch(part.activate_jobs("test-task", **bad), orc.activate_jobs("test-task", **bad))
    same_batch(part.activate_jobs("", max_jobs=3), orc.activate_jobs("", max_jobs=3))


def test_batches_in_key_order_then_complete():
    n = 24
    part, orc = Partition(max_instances=n, max_commands=n), Oracle()
    for e in (part, orc):  # distinct definition keys (the deployment's keys)
        e.deploy(bpmn.linear_process(3, process_id="a", job_type="t"), process_definition_key=2251799813685249)
        e.deploy(bpmn.linear_process(2, process_id="b", job_type="u"), process_definition_key=2251799813685250)
    c = np.concatenate([create_commands(10, 0), create_commands(8, 1, 10), create_commands(6, 0, 18)])
    window(part, orc, c)
    taken = []
    for m, ts in ((3, 10), (4, 20), (3, 30)):
        g = part.activate_jobs("t", worker="w%d" % m, timeout=5000, max_jobs=m, timestamp=ts)
        same_batch(g, orc.activate_jobs("t", worker="w%d" % m, timeout=5000, max_jobs=m, timestamp=ts))
        taken += [int(k) for k in g[1]["key"]]
    same_state(part, orc)
    same_batch(part.activate_jobs("none"), orc.activate_jobs("none"))
    # complete some activated and some activatable jobs in one window (ACTIVATED is completable,
    # DefaultJobCommandPreconditionGuard); the next task's job is activatable again
    open_keys = sorted(int(r.split("|")[1]) for r in part.state() if r.startswith("JOBS|"))
    pick = taken[::2] + [k for k in open_keys if k not in taken][:5]
    window(part, orc, completions(part, pick))
    same_state(part, orc)
    g = part.activate_jobs("t", max_jobs=50, timestamp=99)
    same_batch(g, orc.activate_jobs("t", max_jobs=50, timestamp=99))
    same_batch(part.activate_jobs("u", max_jobs=50, timestamp=99), orc.activate_jobs("u", max_jobs=50, timestamp=99))
    same_state(part, orc)
    # restart: the activated jobs' state survives export -> import
    fresh = Partition(max_instances=n, max_commands=n)
    fresh.deploy(bpmn.linear_process(3, process_id="a", job_type="t"), process_definition_key=2251799813685249)
    fresh.deploy(bpmn.linear_process(2, process_id="b", job_type="u"), process_definition_key=2251799813685250)
    fresh.import_state_db(part.state_db())
    assert fresh.state() == part.state()
    # drain every job
    for _ in range(6):
        keys = sorted(int(r.split("|")[1]) for r in part.state() if r.startswith("JOBS|"))
        if not keys:
            break
        window(part, orc, completions(part, keys))
        same_state(part, orc)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


def test_variables_scopes_and_requested_names():
    n = 16
    xml = (bpmn.createExecutableProcess("p").startEvent("s").serviceTask("t1", "a").exclusiveGateway("x")
           .sequenceFlowId("hi").conditionExpression("= amount > 500").serviceTask("t2", "b").endEvent("e1")
           .moveToNode("x").sequenceFlowId("lo").defaultFlow().serviceTask("t3", "b").endEvent("e2").done())
    part, orc = Partition(max_instances=n, max_commands=n), Oracle()
    for e in (part, orc):
        e.deploy(xml)
    names = [part.intern(x) for x in ("amount", "z", "yy", "b")]
    assert [orc.intern(x) for x in ("amount", "z", "yy", "b")] == names
    rng = np.random.default_rng(11)
    c = create_commands(n)
    c["doc_count"] = 1
    c["doc_begin"] = np.arange(n)
    window(part, orc, c, amount_docs(rng.integers(0, 1000, n), names[0]))
    same_batch(part.activate_jobs("a", max_jobs=4), orc.activate_jobs("a", max_jobs=4))
    # complete every "a" job with one more variable (merged into the process scope)
    keys = sorted(int(r.split("|")[1]) for r in part.state() if r.startswith("JOBS|"))
    cm = completions(part, keys)
    cm["doc_count"] = 1
    cm["doc_begin"] = np.arange(len(keys))
    d = abi.make_docs(len(keys))
    d["name_id"] = [names[1 + (i % 3)] for i in range(len(keys))]
    d["type"] = abi.DOC_INT
    d["value"] = np.arange(len(keys))
    window(part, orc, cm, d)
    same_state(part, orc)
    # all variables (DbString order: length, then bytes) and a requested subset
    same_batch(part.activate_jobs("b", max_jobs=5), orc.activate_jobs("b", max_jobs=5))
    same_batch(part.activate_jobs("b", max_jobs=5, variables=("yy", "amount")),
               orc.activate_jobs("b", max_jobs=5, variables=("yy", "amount")))
    same_state(part, orc)


def test_parallel_branches_and_eviction():
    n = 12
    xml = bpmn.fork_join_process(3, tasks=True, job_type="branch")
    part, orc = Partition(max_instances=n, max_commands=n), Oracle()
    for e in (part, orc):
        e.deploy(xml)
    window(part, orc, create_commands(n))
    same_batch(part.activate_jobs("branch", max_jobs=10, timestamp=5), orc.activate_jobs("branch", max_jobs=10, timestamp=5))
    same_state(part, orc)
    # an evicted instance's jobs are the CPU engine's: never activated on the device again
    part.evict_instances([n - 1])
    g = part.activate_jobs("branch", max_jobs=100)
    assert all(int(j["instance"]) != n - 1 for j in g[1])
    assert len(g[1]) == 3 * n - 10 - 3
