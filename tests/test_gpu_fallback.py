"""Fallback hand-off at the boundary (Engine.java:134 onProcessingError, ProcessingStateMachine.java:
276-310): a command the device does not process goes to the CPU engine in log order, later commands
of its subject in the window are fenced (FB_FENCED) and follow it there, the instance's rows move to
the CPU engine (zbhip_export_instances_db + zbhip_evict_instances), and the keys the CPU engine
generates are declared (zbhip_key_before / zbhip_set_external_keys) so the device-processed commands
after them relabel to the reference's keys.

The CPU engine here is a second oracle kept in lockstep with the device partition; the reference is
a third oracle that processes every window itself.  Bar: the merged record stream (device records
of the processed commands, CPU-engine records of the fallback commands, in log order) and the final
state equal the reference's."""
import numpy as np
import pytest

from helpers import complete_commands, create_commands
from oracle import statedb as SD
from oracle.oracle import Oracle
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition
from zeebe_amd.native import ZbhipError

pytestmark = pytest.mark.gpu

FIELDS = abi.PARITY_FIELDS
XML = bpmn.linear_process(5)
N = 8


def _docs(entries):
    d = abi.make_docs(len(entries))
    for j, (name, value) in enumerate(entries):
        d[j]["name_id"], d[j]["type"], d[j]["value"] = name, abi.DOC_INT, value
    return d


def _open_jobs(part, recs):
    """{instance: job key ordinal} of the JOB:CREATED records of a drained window."""
    jobs = recs[(recs["value_type"] == abi.VT_JOB) & (recs["intent"] == abi.JOB_CREATED)]
    return dict(part.resolve_key(int(k)) for k in jobs["key"])


def _lockstep(gpu, *oracles):
    """Deploys linear-5 on every engine and drives N instances: create, then jobs 1..4, instance 0
    completing each job with a document holding one new variable v1..v4 (4 variables: the device's
    per-instance capacity, zb_internal.h kVars).  Returns the variable names and the open jobs."""
    engines = (gpu,) + oracles
    names = None
    for e in engines:
        assert e.deploy(XML) == 0
        ids = [e.intern("v%d" % k) for k in range(1, 6)]
        assert names is None or ids == names
        names = ids
    cmds, docs = create_commands(N), None
    for task in range(5):
        for e in engines:
            e.submit(cmds, docs)
            e.run()
        got = gpu.drain()
        assert gpu.fallback() == []
        for o in oracles:
            want = o.records()
            o.clear_records()
            for f in FIELDS:
                assert np.array_equal(got[f], want[f]), f
        jobs = _open_jobs(gpu, got)
        if task == 4:
            return names, jobs
        cmds = complete_commands(np.arange(N), [jobs[i] for i in range(N)])
        cmds[0]["doc_count"], cmds[0]["doc_begin"] = 1, 0
        docs = _docs([(names[task], 10 + task)])


def test_fallback_fences_the_subject_and_hands_it_to_the_cpu_engine():
    gpu = Partition(max_instances=2 * N, max_commands=2 * N, max_records_per_batch=64)
    cpu, ref = Oracle(), Oracle()
    names, jobs = _lockstep(gpu, cpu, ref)
    # the window: instance 0's 5th variable exceeds the device's variable slots (FB_VARS); the same
    # job completed again later in the window (a stale command) must follow it on the CPU engine
    w = np.concatenate([complete_commands([1], [jobs[1]]), complete_commands([0], [jobs[0]]),
                        complete_commands([2], [jobs[2]]), complete_commands([0], [jobs[0]]),
                        create_commands(1, 0, first_instance=N)])
    w[1]["doc_count"], w[1]["doc_begin"] = 1, 0
    docs = _docs([(names[4], 99)])
    ref.submit(w, docs)
    ref.run()
    want = ref.records()

    gpu.submit(w, docs)
    gpu.run()
    status = [gpu.command_status(i) for i in range(len(w))]
    assert status == [(0, 0), (1, "vars"), (0, 0), (1, "fenced"), (0, 0)], status
    # hand-off: the instance's rows are what the CPU engine holds for it (zb-db bytes)
    rows = gpu.export_instances([0])
    assert rows and set(rows) <= set(cpu.state())
    strings = cpu.strings()
    assert gpu.export_instances_db([0]) == SD.encode_rows(rows, cpu.process_tables(), lambda i: strings[i])
    job0 = [int(r.split("|")[1]) for r in rows if r.startswith("JOBS|")]
    assert len(job0) == 1 and gpu.resolve_key(job0[0])[0] == 0
    gpu.evict_instances([0])
    with pytest.raises(ZbhipError):  # evicted: the adapter routes its keys to the CPU engine
        gpu.resolve_key(job0[0])
    # the CPU engine processes the fallback commands in log order, keys continuing the device's
    pbits = 1 << 51
    cpu_recs = {}
    for i in (1, 3):
        before = gpu.key_before(i) - pbits
        cpu.set_key_counter(before)
        cpu.clear_records()
        cpu.submit(w[i:i + 1], docs if w[i]["doc_count"] else None)
        cpu.run()
        cpu_recs[i] = cpu.records()
        gpu.set_external_keys(i, cpu.key_counter() - before)
    got = gpu.drain()
    base = int(want["source_index"][0])
    merged = []
    for i in range(len(w)):
        if i in cpu_recs:
            r = cpu_recs[i].copy()
            r["source_index"] = base + i
            merged.append(r)
        else:
            merged.append(got[got["source_index"] == base + i])
    merged = np.concatenate(merged)
    assert len(merged) == len(want)
    for f in FIELDS:
        assert np.array_equal(merged[f], want[f]), (f, merged[f], want[f])
    # the stale completion was rejected by the CPU engine (the job was completed before it)
    assert [int(x) for x in cpu_recs[3]["record_type"]] == [abi.RT_REJECTION]
    # instance 0 ended on the CPU engine; every other row is the device's, and the key counter
    # (KEY latestKey) includes the CPU engine's keys
    assert gpu.state() == ref.state()


def test_completed_instance_keys_do_not_resolve_and_reuse_in_window_is_refused():
    part = Partition(max_instances=4, max_commands=8)
    orc = Oracle()
    part.deploy(bpmn.linear_process(1))
    orc.deploy(bpmn.linear_process(1))
    part.submit(create_commands(2))
    part.run()
    recs = part.drain()
    jobs = recs[(recs["value_type"] == abi.VT_JOB) & (recs["intent"] == abi.JOB_CREATED)]
    inst, ordv = part.resolve_key(int(jobs[0]["key"]))
    assert inst == 0
    # complete instance 0; a CREATE into its slot in the same window is refused
    w = np.concatenate([complete_commands([0], [ordv]), create_commands(1)])
    with pytest.raises(ZbhipError):
        part.submit(w)
    part.submit(complete_commands([0], [ordv]))
    part.run()
    part.drain()
    # the completed instance's job key no longer resolves (a stale JOB:COMPLETE goes to the CPU
    # engine, which rejects it NOT_FOUND); the slot is reused by the next window
    with pytest.raises(ZbhipError):
        part.resolve_key(int(jobs[0]["key"]))
    part.submit(create_commands(1))
    part.run()
    recs = part.drain()
    new_job = recs[(recs["value_type"] == abi.VT_JOB) & (recs["intent"] == abi.JOB_CREATED)]
    assert part.resolve_key(int(new_job[0]["key"]))[0] == 0
    assert int(new_job[0]["key"]) != int(jobs[0]["key"])
    # instance 1 still waits on its job
    assert part.resolve_key(int(jobs[1]["key"]))[0] == 1


def test_device_window_with_duplicate_subjects_is_planned_like_a_host_window():
    import torch
    xml = bpmn.linear_process(3)
    host, dev_p = Partition(max_instances=16, max_commands=32), Partition(max_instances=16, max_commands=32)
    for p in (host, dev_p):
        p.deploy(xml)
        p.submit(create_commands(8))
        p.run()
        p.drain()
    # two commands for instances 0..3 (the second one stale), once for 4..7
    c = np.concatenate([complete_commands(np.arange(8), np.full(8, 5)), complete_commands(np.arange(4), np.full(4, 5))])
    host.submit(c)
    host.run()
    want = host.drain()
    t = torch.from_numpy(c.view(np.uint8).copy()).to("cuda")
    dev_p.submit_device(t.data_ptr(), len(c))
    dev_p.run()
    got = dev_p.drain()
    for f in FIELDS:
        assert np.array_equal(got[f], want[f]), f
    assert dev_p.state() == host.state()
    # a subject out of range refuses the device window (the speculative check reports it at the run)
    bad = complete_commands([99], [5])
    tb = torch.from_numpy(bad.view(np.uint8).copy()).to("cuda")
    with pytest.raises(ZbhipError):
        dev_p.submit_device(tb.data_ptr(), 1)
        dev_p.run()


def test_speculative_subject_check_replays_a_window_with_repeats():
    """Untrusted device windows launch before their subject check is read back: k_step runs guarded by
    the check's verdict (the guard word of the window's stamp), and the next call that depends on the
    window reads it.  A window with a repeated subject did nothing on the device; it is replanned on the
    host and run again before the next window -- the statistics (transitions, records, completed
    instances) equal the host-planned run's."""
    import torch
    xml = bpmn.linear_process(3)
    host = Partition(max_instances=16, max_commands=32)
    dev_p = Partition(max_instances=16, max_commands=32)
    for p in (host, dev_p):
        p.deploy(xml)
        p.submit(create_commands(8))
        p.run()
        p.drain()
    # faulty (a repeat), clean, faulty, clean: the jobs of tasks 1, 2, 3
    windows = [np.concatenate([complete_commands(np.arange(8), np.full(8, 5)), complete_commands(np.arange(4), np.full(4, 5))]),
               complete_commands(np.arange(8), np.full(8, 9)),
               np.concatenate([complete_commands(np.arange(4), np.full(4, 13)), complete_commands(np.arange(2), np.full(2, 13))]),
               complete_commands(np.arange(4, 8), np.full(4, 13))]
    for k, w in enumerate(windows):
        host.submit(w)
        host.run(abi.RUN_NO_RESULTS | (abi.RUN_ACCUMULATE if k else 0))
    want = host.stats()
    ts = [torch.from_numpy(c.view(np.uint8).copy()).to("cuda") for c in windows]
    torch.cuda.synchronize()
    for k, t in enumerate(ts):
        dev_p.submit_device(t.data_ptr(), len(windows[k]))  # reads the last window's verdict: replays it
        dev_p.run(abi.RUN_NO_RESULTS | (abi.RUN_ACCUMULATE if k else 0))
    got = dev_p.stats()  # reads the last window's verdict (clean)
    for k in ("transitions", "records", "completed_instances", "fallback"):
        assert got[k] == want[k], k
    assert want["completed_instances"] == 8 and want["transitions"] > 0
