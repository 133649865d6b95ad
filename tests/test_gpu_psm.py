"""The drop-in boundary inside the reference's processing loop: ProcessingStateMachine (restated in
tests/psm.py, pinned against the oracle's batch driver by tests/test_psm_oracle.py) runs
[GpuBatchProcessor (zeebe_amd/adapter.py, the Python mirror of the Java adapter), engine] over one log,
and the whole log -- every record, its position, source position and processed flag -- and the final
state equal the same loop over the engine alone (the CPU oracle, one command at a time).

This is what the adapter must get right inside ProcessingStateMachine.batchProcessing /
collectBatchProcessingStepResult (stream-platform/.../ProcessingStateMachine.java:328-417):
follow-up commands the platform feeds back after a device batch answered from the builder (not
re-processed by the engine), continuations past maxCommandsInBatch run at their own log position
after whatever the log holds before them (ZBHIP_OPEN_DEFER_CONTINUATIONS), one key generator across
device windows and the engine's commands (DbKeyGenerator.setKeyIfHigher), the fallback hand-off,
JOB_BATCH:ACTIVATE on the device, rejections carrying the command's value, and restart through the
engine's state (on_recovered -> zbhip_import_state)."""
import numpy as np
import pytest

from psm import Client, Log, OracleEngine, StreamProcessor, open_jobs
from test_oracle_timers import NOW
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import GpuBatchProcessor

pytestmark = pytest.mark.gpu

KEY_A, KEY_B, KEY_C = 2251799813685249, 2251799813685250, 2251799813685251


class Ref:
    """The reference: the processing loop over the engine alone."""

    def __init__(self, deployments, limit):
        self.log = Log()
        self.engine = OracleEngine(max_commands_in_batch=limit, clock=NOW)
        for xml, key, version in deployments:
            self.engine.deploy(xml, key, version)
        self.sp = StreamProcessor(self.log, [self.engine], limit)

    def state(self):
        return self.engine.state()


class Mixed:
    """The same loop over [the device behind the adapter, the engine].  `device` = the deployments the
    adapter knows (a process deployed later, or outside the device subset, is the engine's)."""

    def __init__(self, deployments, device, limit, window=48, instances=256, log=None, engine=None):
        device_keys = {k for _, k, _ in device}
        self.log = log or Log()
        if engine is None:
            engine = OracleEngine(max_commands_in_batch=limit, clock=NOW)
            for xml, key, version in deployments:
                engine.deploy(xml, key, version)
        self.engine = engine
        self.adapter = GpuBatchProcessor(engine, self.log.reader(), device, zeebe_db=engine, key_generator=engine,
                                         instances=instances, window=window, max_commands_in_batch=limit,
                                         clock=lambda: NOW,
                                         engine_deployments=[d for d in deployments if d[1] not in device_keys])
        self.adapter.init()
        self.sp = StreamProcessor(self.log, [self.adapter, engine], limit)
        self.sp.read = len(self.log.entries)

    def state(self):
        part = self.adapter.part
        dev = [r for r in part.state() if not r.startswith("KEY|")]
        eng = self.engine.state()
        key = [r for r in eng if r.startswith("KEY|")]
        # one key generator: the device's is level with the engine's
        assert part.current_key() <= self.engine.current_key()
        return sorted(dev + [r for r in eng if not r.startswith("KEY|")] + key)


def phase(ref, mixed, recs):
    Client(ref.log, mixed.log).write(*recs)
    ref.sp.run()
    mixed.sp.run()
    want, got = ref.log.canonical(), mixed.log.canonical()
    if got != want:
        bad = next(i for i in range(min(len(got), len(want))) if got[i] != want[i]) if got[:len(want)] != want[:len(got)] \
            else min(len(got), len(want))
        raise AssertionError("log entry %d of %d/%d:\n got  %s\n want %s" % (
            bad, len(got), len(want), got[bad] if bad < len(got) else None, want[bad] if bad < len(want) else None))
    assert mixed.state() == ref.state()


def completions(ref, rng, variables=None, skip=()):
    jobs = sorted(k for k in open_jobs(ref.log) if k not in skip)
    rng.shuffle(jobs)
    return [Client.complete_job(k, variables(k) if variables else ()) for k in jobs]


@pytest.mark.parametrize("limit", [3, 100])
def test_adapter_in_the_processing_loop(limit):
    # device processes A (linear-4) and C (fork/join-4 with tasks, fan-out past a limit of 3), and B
    # (linear-2) deployed for the engine only: its CREATEs generate keys between device windows;
    # JOB_BATCH:ACTIVATE of a device job type in between
    a, b, c = bpmn.linear_process(4), bpmn.linear_process(2, process_id="engineOnly", job_type="engine-task"), \
        bpmn.fork_join_process(4, tasks=True, process_id="forkjoin")
    deps = [(a, KEY_A, 1), (c, KEY_C, 1), (b, KEY_B, 1)]
    ref, mixed = Ref(deps, limit), Mixed(deps, deps[:2], limit)
    rng = np.random.default_rng(limit)
    first = [Client.create("linear") for _ in range(30)] + [Client.create("engineOnly")] + \
            [Client.create("forkjoin", (("n", k),)) for k in range(20)] + [Client.create("engineOnly")] + \
            [Client.create("linear") for _ in range(10)]
    phase(ref, mixed, first)
    for p in range(12):
        recs = completions(ref, rng, lambda k: (("done", int(k) % 7),) if k % 3 == 0 else ())
        if not recs:
            break
        mid = len(recs) // 2
        extra = [Client.create("engineOnly")]
        if p % 2 == 0:
            extra.append(Client.activate_jobs("benchmark-task", max_jobs=5))
            extra.append(Client.activate_jobs("engine-task", max_jobs=2))
        phase(ref, mixed, recs[:mid] + extra + recs[mid:])
    c = mixed.adapter.counts
    assert c["fallbacks"] == 0 and c["activations"] == 6 and c["followups_answered"] > 100
    # the device ran every CREATE / COMPLETE of A and C (the engine only B's commands and follow-ups);
    # with a limit of 3 the continuations came back from the log after engine commands in between
    assert c["device_commands"] >= 300 and c["windows"] > 12
    assert (c["continuations"] > 100) == (limit == 3)


def test_fallback_hand_off_in_the_processing_loop():
    # instance 0 collects one new variable per job (the device holds 4 per instance, zb_internal.h
    # kVars): its 5th falls back, the instance moves to the engine with its rows, later commands of
    # it in the window follow (fenced), and its later jobs are the engine's
    xml = bpmn.linear_process(6)
    deps = [(xml, KEY_A, 1)]
    ref, mixed = Ref(deps, 100), Mixed(deps, deps, 100)
    phase(ref, mixed, [Client.create("linear") for _ in range(8)])
    rng = np.random.default_rng(5)
    first_pi = min(r.value["processInstanceKey"] for r in ref.log.entries
                   if r.value_type == abi.VT_PROCESS_INSTANCE_CREATION and r.intent == 1)
    for task in range(6):
        jobs = open_jobs(ref.log)
        recs = []
        for k in sorted(jobs):
            v = (("v%d" % task, task),) if jobs[k].value["processInstanceKey"] == first_pi else ()
            recs.append(Client.complete_job(k, v))
        rng.shuffle(recs)
        if task == 4:  # a stale completion of the handed-off instance's job in the same window
            stale = [r for r in recs if jobs[r.key].value["processInstanceKey"] == first_pi][0]
            recs.append(Client.complete_job(stale.key))
        phase(ref, mixed, recs + [Client.create("linear")])
    assert mixed.adapter.handed_off


def test_restart_imports_device_instances():
    # the engine ran everything up to a restart; after recovery (replay -> the engine's state) the
    # adapter moves the instances of device processes into HBM and the loop continues on the device
    xml = bpmn.fork_join_process(3, tasks=True)
    deps = [(xml, KEY_A, 1)]
    ref = Ref(deps, 100)
    Client(ref.log).write(*[Client.create("forkjoin") for _ in range(16)])
    ref.sp.run()
    rng = np.random.default_rng(3)
    Client(ref.log).write(*completions(ref, rng)[:20])
    ref.sp.run()
    # restart: a fresh engine from the reference's state (its zb-db entries), the device from the
    # adapter's recovery; the engine keeps what the device does not take
    from oracle import statedb as SD
    rows = ref.state()
    tables, strings = ref.engine.o.process_tables(), ref.engine.o.strings()
    pairs = [(r, e) for r in rows for e in SD.encode_rows([r], tables, lambda i: strings[i])]
    log = Log()
    log.entries = [r for r in ref.log.entries]
    engine = OracleEngine(max_commands_in_batch=100, clock=NOW)
    engine.deploy(xml, KEY_A, 1)
    mixed = Mixed(deps, deps, 100, log=log, engine=engine)
    take = mixed.adapter.on_recovered([e for _, e in pairs], resume_position=len(log.entries) + 1)
    moved = {r for (r, _), t in zip(pairs, take) if t}
    assert moved and any(r.startswith("ELEMENT_INSTANCE_KEY|") for r in moved)
    engine.upsert([r for r in rows if r not in moved and not r.startswith("KEY|")])
    engine.set_key_if_higher(ref.engine.current_key())
    mixed.adapter.part.set_key_if_higher(engine.current_key())
    assert mixed.state() == ref.state()
    for _ in range(4):
        recs = completions(ref, rng)
        if not recs:
            break
        phase(ref, mixed, recs)
    assert not open_jobs(ref.log)


@pytest.mark.parametrize("limit", [3, 100])
def test_multi_instance_in_the_processing_loop(limit):
    # parallel and sequential bodies behind the adapter: PROCESS_INSTANCE_BATCH:ACTIVATE and the inner
    # activations as follow-ups answered from the builder or, past a limit of 3, continuations read
    # back from the log (matched by key, value type, intent and value); job activations carry the
    # loop variables
    a = bpmn.multi_instance_process((1, "two", 3), process_id="par", job_type="mi-par", after="after")
    b = bpmn.multi_instance_process((4, 5), sequential=True, process_id="seq", job_type="mi-seq")
    deps = [(a, KEY_A, 1), (b, KEY_B, 1)]
    ref, mixed = Ref(deps, limit), Mixed(deps, deps, limit)
    phase(ref, mixed, [Client.create("par") for _ in range(8)] + [Client.create("seq") for _ in range(8)])
    rng = np.random.default_rng(17 + limit)
    for p in range(12):
        recs = completions(ref, rng, lambda k: (("r", int(k) % 5),) if k % 2 else ())
        if not recs:
            break
        extra = [Client.activate_jobs("mi-par", max_jobs=3)] if p % 2 == 0 else []
        phase(ref, mixed, recs + extra)
    c = mixed.adapter.counts
    assert c["fallbacks"] == 0 and c["device_commands"] > 40
    assert (c["continuations"] > 0) == (limit == 3)
    assert not open_jobs(ref.log)


def test_io_mappings_in_the_processing_loop():
    # zeebe:ioMapping behind the adapter (KScopeIO): the mapped VARIABLE records' values inline in the
    # log, task- and sub-process-scope variables in the state, job activations with the local variables
    from test_gpu_io_mapping import _sub, _task_in_out
    a = _task_in_out()
    b = _sub([("input", "=x", "y"), ("output", "=y", "z")], "task").replace('id="process"', 'id="subproc"', 1)
    deps = [(a, KEY_A, 1), (b, KEY_B, 1)]
    ref, mixed = Ref(deps, 100), Mixed(deps, deps, 100)
    phase(ref, mixed, [Client.create("process", (("x", k),)) for k in range(10)] +
          [Client.create("subproc", (("x", 2.5 if k % 2 else k),)) for k in range(10)])
    rng = np.random.default_rng(21)
    for p in range(4):
        recs = completions(ref, rng, lambda k: (("local", int(k) % 3),) if k % 2 else ())
        if not recs:
            break
        phase(ref, mixed, recs + [Client.activate_jobs("t", max_jobs=3)])
    c = mixed.adapter.counts
    assert c["fallbacks"] == 0 and c["device_commands"] >= 30, c
