"""Log bytes written on the device (zbhip_serialize_log_device, logdev.hip): for every window, the
bytes equal the host serialiser's (zbhip_serialize_log over the drained records -- itself equal to
the oracle's, tests/test_gpu_logserial.py) byte for byte: frames, LogEntryDescriptor headers, SBE
RecordMetadata with rejection texts, msgpack values with documents; keys relabelled on the device
(batch key bases, the previous command of the instance in the window, the per-instance key ring).

SequencedBatchSerializer.java:33-67, LogAppendEntrySerializer.java:40-111, protocol.xml:137-152."""
import numpy as np
import pytest

from helpers import amount_docs, create_commands
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition
from zeebe_amd.native import ZbhipError

pytestmark = pytest.mark.gpu

TS = 1700000000123


class Log:
    def __init__(self, xml, n, names=(), max_records=128, **kw):
        self.part = Partition(max_instances=n, max_commands=16 * n, max_records_per_batch=max_records, **kw)
        assert self.part.deploy(xml) == 0
        self.names = [self.part.intern(x) for x in names]
        self.ser = self.part.log_serializer()
        self.source_base = self.doc_base = 0
        self.position = 100
        self.windows = 0
        self.declined = 0

    def window(self, cmds, docs=None, device=True, flags=0, allow_host=False):
        """allow_host: a window the device path declines (ZBHIP_EUNSUPP: e.g. a key older than the
        instance's key ring) is checked on the host serialiser only; self.declined counts them."""
        docs = docs if docs is not None else abi.make_docs(0)
        self.part.submit(cmds, docs)
        self.part.run(flags)
        pos = self.position + 2 * np.arange(len(cmds), dtype=np.int64)
        first = int(pos[-1]) + 1 if len(cmds) else self.position
        dev = None
        if device:
            try:
                dev = self.part.serialize_log_device(pos, first, TS)
            except ZbhipError as e:
                if not (allow_host and e.code == -5):
                    raise
                self.declined += 1
                device = False
        recs = self.part.drain()
        host = self.ser.serialize(recs, cmds, docs, self.source_base, self.doc_base, pos, first, TS)
        if device:
            assert len(dev) == len(host)
            if dev != host:
                bad = next(i for i in range(len(host)) if dev[i] != host[i])
                raise AssertionError("byte %d of %d differs: device %r host %r" % (bad, len(host), dev[bad - 8:bad + 24],
                                                                                 host[bad - 8:bad + 24]))
        self.source_base += len(cmds)
        self.doc_base += len(docs)
        self.position = first + len(recs)
        self.windows += 1
        return recs


def job_completions(recs, part, rng=None, limit=None):
    jobs = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    if rng is not None:
        rng.shuffle(jobs)
    jobs = jobs[:limit] if limit else jobs
    c = abi.make_commands(len(jobs))
    for i, k in enumerate(jobs):
        c[i]["instance"], c[i]["ref"] = part.resolve_key(k)
    c["kind"] = abi.CMD_JOB_COMPLETE
    return c


@pytest.mark.parametrize("tasks", [1, 5])
def test_linear_windows(tasks):
    n = 300
    log = Log(bpmn.linear_process(tasks), n)
    recs = log.window(create_commands(n))
    for _ in range(tasks):
        recs = log.window(job_completions(recs, log.part))
    assert log.windows == tasks + 1


def test_exclusive_gateway_documents():
    # int, decimal, bool and nil values, both outcomes, and the template path on later windows
    n = 256
    log = Log(bpmn.xor_process(), n, names=("amount",))
    rng = np.random.default_rng(3)
    for w in range(4):
        c = create_commands(n)
        c["doc_count"] = 1
        c["doc_begin"] = np.arange(n)
        if w == 0:
            d = amount_docs(rng.integers(0, 2000, n), log.names[0])
        elif w == 1:
            d = amount_docs(rng.integers(0, 200000, n) / 100.0, log.names[0], decimal=True)
        else:
            d = amount_docs(rng.integers(-5000, 5000000000, n), log.names[0])
        log.window(c, d)


def test_fork_join_rejections_and_tasks():
    # join rejections (reason texts with element ids); branch tasks completed in random order, several
    # jobs of an instance in one window (rounds: the previous-command chain)
    n = 64
    log = Log(bpmn.fork_join_process(8), n)
    for _ in range(3):
        log.window(create_commands(n))
    log2 = Log(bpmn.fork_join_process(4, tasks=True), n)
    recs = log2.window(create_commands(n))
    rng = np.random.default_rng(9)
    for _ in range(6):
        c = job_completions(recs, log2.part, rng)
        if len(c) == 0:
            break
        recs = log2.window(c)


def test_stale_job_complete_rejection():
    # JOB:COMPLETE of a job completed in an earlier window: NOT_FOUND rejection with the job key
    n = 32
    log = Log(bpmn.linear_process(2), n)
    recs = log.window(create_commands(n))
    c = job_completions(recs, log.part)
    log.window(c)
    log.window(c)  # the same commands again: every one rejected


def test_a_skipped_window_turns_the_device_path_off():
    n = 16
    log = Log(bpmn.linear_process(2), n)
    recs = log.window(create_commands(n), device=False)
    with pytest.raises(ZbhipError, match="EUNSUPP"):
        log.window(job_completions(recs, log.part))


def test_records_left_in_hbm_and_device_windows():
    # ZBHIP_RUN_DEVICE_RECORDS: the records stay in HBM for the device writer; a later drain copies
    # them (the bytes and the drained records agree with the host path); windows submitted from
    # device memory take the same path
    import torch

    n = 200
    log = Log(bpmn.linear_process(3), n)
    recs = log.window(create_commands(n), flags=abi.RUN_DEVICE_RECORDS)
    recs = log.window(job_completions(recs, log.part), flags=abi.RUN_DEVICE_RECORDS)
    c = job_completions(recs, log.part)
    dev = torch.from_numpy(c.view(np.uint8).copy()).cuda()
    log.part.submit_device(dev.data_ptr(), len(c))
    log.part.run(abi.RUN_DEVICE_RECORDS)
    pos = log.position + 2 * np.arange(len(c), dtype=np.int64)
    first = int(pos[-1]) + 1
    got = log.part.serialize_log_device(pos, first, TS)
    recs = log.part.drain()
    assert got == log.ser.serialize(recs, c, abi.make_docs(0), log.source_base, log.doc_base, pos, first, TS)


@pytest.mark.parametrize("shape", ["timer", "task_timer_task", "boundary", "non_interrupting_escalation", "cycle_r3",
                                   "cycle_infinite", "in_sub_process"])
def test_timer_and_boundary_windows(shape):
    # KScope windows with timer records (CREATED from the clock, a cycle's next from the TRIGGER
    # command, TRIGGERED, CANCELED from cmd_due), JOB:CANCELED, PROCESS_EVENT:TRIGGERED and the
    # terminate intents: device bytes == host serialiser; a stale TRIGGER's rejection text too
    from test_gpu_boundary import SHAPES as BSHAPES
    from test_gpu_timers import SHAPES as TSHAPES, _open_work
    from test_oracle_boundary import multiple_sequence_flows
    from test_oracle_timers import NOW, trigger_commands
    shapes = dict(TSHAPES, **BSHAPES, boundary=lambda: multiple_sequence_flows("PT30S"))
    log = Log(shapes[shape](), 64)
    log.part.set_clock(NOW)
    recs = log.window(create_commands(64, 0))
    rng = np.random.default_rng(4)
    stale_done = False
    for step in range(8):
        c = _open_work(log.part, rng)
        if c is None:
            break
        log.part.set_clock(NOW + 1000 * (step + 1))
        # cycles pile up keys between a job's creation and its completion: past the 16-entry key
        # ring the device path declines the window (the host serialiser writes it)
        recs = log.window(c, allow_host=shape.startswith("cycle"))
        timers = c[c["kind"] == abi.CMD_TIMER_TRIGGER]
        if len(timers) and not stale_done:
            # triggered just now: a repeated TRIGGER is rejected NOT_FOUND, its reason text (with the
            # timer key, still in the device's key ring) written on the device
            recs = log.window(timers[:1].copy())
            assert recs[0]["record_type"] == abi.RT_REJECTION
            stale_done = True
    assert log.declined < log.windows - 1  # the device wrote the timer windows


def test_window_past_two_gigabytes():
    # a CREATE window of linear-10 whose log bytes pass 2^31 (byte offsets in 64 bits end to end: the
    # wave-cooperative writer reads every entry's offset across lanes); the tail's bytes equal the host
    # serialiser's for the tail's records
    n = 450_000
    part = Partition(max_instances=n, max_commands=n, max_records_per_batch=64)
    assert part.deploy(bpmn.linear_process(10)) == 0
    ser = part.log_serializer()
    cmds = create_commands(n)
    part.submit(cmds)
    part.run()
    pos = 100 + 2 * np.arange(n, dtype=np.int64)
    first = int(pos[-1]) + 1
    ptr, used = part.serialize_log_device(pos, first, TS, copy=False)
    assert used > (1 << 31)
    recs = part.drain()
    k = 64  # the last k commands' records
    tail_src = n - k
    at = int(np.searchsorted(recs["source_index"], tail_src))
    host = ser.serialize(recs[at:], cmds[tail_src:], abi.make_docs(0), tail_src, 0, pos[tail_src:], first + at, TS)
    import ctypes as C
    buf = C.create_string_buffer(used)
    part.L.zbhip_log_device_copy(part.h, buf, used)
    assert buf.raw[used - len(host):used] == host


def test_declined_window_past_earlier_windows_and_after_a_redeploy():
    # a window the size pass declines (string variables: the host serialiser writes them) whose
    # records reach far past every earlier window's per-record info: the speculative write pass must
    # write nothing for it (its entry info is incomplete); the next windows -- also after another
    # process was deployed -- are written on the device again
    log = Log(bpmn.linear_process(2), 600, names=("s",))
    log.window(create_commands(4))
    log.window(create_commands(4, first_instance=4))
    n = 400
    c = create_commands(n, first_instance=8)
    c["doc_count"] = 1
    c["doc_begin"] = np.arange(n)
    d = abi.make_docs(n)
    d["name_id"] = log.names[0]
    d["type"] = abi.DOC_STR
    d["value"] = [log.part.intern_string("v%d" % i) for i in range(n)]
    log.window(c, d, allow_host=True)
    assert log.declined == 1
    recs = log.window(create_commands(64, first_instance=420))
    assert log.part.deploy(bpmn.linear_process(3, process_id="later")) == 1
    log.window(create_commands(32, process_idx=1, first_instance=484))
    log.window(job_completions(recs, log.part))
    assert log.declined == 1


def test_activated_job_completions_on_the_device(monkeypatch):
    # JOB:COMPLETED / CANCELED of an ACTIVATED job carry the stored deadline and worker
    # (DbJobState.activate): the device writer composes them from the batch's activation word and the
    # value dictionary's bytes -- a plain, an empty and a 40-byte worker (msgpack str8 header)
    monkeypatch.setenv("ZBHIP_DEVICE_ACTIVATIONS", "1")
    n = 96
    log = Log(bpmn.linear_process(3, job_type="t"), n)
    recs = log.window(create_commands(n))
    log.part.activate_jobs("t", worker="w", timeout=1000, max_jobs=30, timestamp=10)
    log.part.activate_jobs("t", worker="", timeout=2000, max_jobs=20, timestamp=20)
    log.part.activate_jobs("t", worker="worker-" + "x" * 33, timeout=3000, max_jobs=20, timestamp=30)
    recs = log.window(job_completions(recs, log.part))
    done = recs[(recs["value_type"] == abi.VT_JOB) & (recs["intent"] == abi.JOB_COMPLETED)]
    assert sorted(set(done["message_key"].tolist())) == [-1, 1010, 2020, 3030]
    # the next tasks' jobs, activated again and completed; then the rest without activation
    log.part.activate_jobs("t", worker="again", timeout=500, max_jobs=50, timestamp=40)
    recs = log.window(job_completions(recs, log.part))
    log.window(job_completions(recs, log.part))
    assert log.declined == 0


def test_log_bytes_copied_asynchronously_into_pinned_buffers():
    # zbhip_log_copy_async: window k's bytes cross PCIe into one of the handle's two pinned buffers while
    # window k+1 is submitted, run and serialised into the other device buffer; once waited for they equal
    # the host serialiser's bytes of window k (and stay valid until the second next copy)
    n = 300
    part = Partition(max_instances=n, max_commands=16 * n, max_records_per_batch=128)
    part.deploy(bpmn.linear_process(4))
    ser = part.log_serializer()
    cmds, source_base, position, pending, landings = create_commands(n), 0, 100, None, []
    for _ in range(5):
        part.submit(cmds)
        part.run(abi.RUN_DEVICE_RECORDS)
        pos = position + 2 * np.arange(len(cmds), dtype=np.int64)
        first = int(pos[-1]) + 1
        _, used = part.serialize_log_device(pos, first, TS, copy=False)
        landing = part.log_copy_async(used)
        landings.append(landing)
        recs = part.drain()
        want = ser.serialize(recs, cmds, abi.make_docs(0), source_base, 0, pos, first, TS)
        if pending is not None:
            assert part.log_copy_wait(pending[0], pending[1]) == pending[2]
        pending = (landing, used, want)
        source_base += len(cmds)
        position = first + len(recs)
        cmds = job_completions(recs, part)
    assert part.log_copy_wait(pending[0], pending[1]) == pending[2]
    assert len(set(landings)) == 2 and landings[0] == landings[2] != landings[1]
