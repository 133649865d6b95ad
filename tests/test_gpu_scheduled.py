"""The engine's scheduled tasks over device-held state, in the reference's processing loop.

The reference's checkers read RocksDB: DueDateTimerChecker (engine/.../processing/timer/
DueDateTimerChecker.java:86-129) writes TIMER:TRIGGER for due timers, JobTimeoutTrigger (processing/job/
JobTimeoutTrigger.java:74-87) JOB:TIME_OUT for activated jobs past their deadline, and the pending-
subscription checkers (PendingProcessMessageSubscriptionChecker.java:78-128, MessageObserver.java:61-73 ->
PendingMessageSubscriptionChecker) send the subscription commands again that got no answer.  Behind the
adapter they read the merged views of zeebe_amd/adapter.py (the engine's state + the device's:
zbhip_due_timers, zbhip_timed_out_jobs, the adapter's pending-subscription states), and JOB:TIME_OUT of a
device job runs through zbhip_time_out_job.

Each test runs the same workload, with the same controlled clock (EngineRule.increaseTime), through the
loop over the engine alone (tests/psm.py: the oracle engine, its own state views) and through the loop over
[adapter, engine]; nobody but the checkers writes triggers, time-outs or resends.  The bar: every log
(every record, position, source position, processed flag) and every state equal."""
import numpy as np
import pytest

from psm import (Client, Clock, DueDateTimerChecker, canon_strings, EngineJobState, EngineMessageState, EngineTimerState,
                 InterPartitionCommandSender, JobTimeoutTrigger, Log, MessageTimeToLiveChecker, OracleEngine,
                 PendingMessageSubscriptionChecker,
                 PendingProcessMessageSubscriptionChecker, Rec, ScheduleService, StreamProcessor, open_jobs, run_cluster)
from test_oracle_boundary import cycle_process, multiple_sequence_flows
from test_oracle_timers import NOW, timer_process
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import DeviceJobState, DevicePendingSubscriptionState, DeviceTimerInstanceState, GpuBatchProcessor

pytestmark = pytest.mark.gpu

KEY_A, KEY_B, KEY_C, KEY_D = 2251799813685249, 2251799813685250, 2251799813685251, 2251799813685252


class PartitionLoop:
    """One partition: its log, processing loop, schedule service and the checkers the engine registers
    (EngineProcessors: DueDateTimerChecker, JobTimeoutTrigger, and for message partitions the pending
    subscription checkers), over the engine's state -- or, with `device`, over the adapter's merged views."""

    def __init__(self, clock, deployments, device_deployments=None, limit=100, partition_id=1, partition_count=1,
                 sender=None, log=None, correlation_keys=0):
        self.clock = clock
        self.log = log if log is not None else Log()
        self.engine = OracleEngine(partition_id=partition_id, max_commands_in_batch=limit, clock=clock,
                                   partition_count=partition_count, command_sender=sender)
        for xml, key, version in deployments:
            self.engine.deploy(xml, key, version)
        timers, jobs, pending = EngineTimerState(self.engine), EngineJobState(self.engine), self.engine.pending
        self.adapter = None
        procs = [self.engine]
        if device_deployments is not None:
            dkeys = {k for _, k, _ in device_deployments}
            self.adapter = GpuBatchProcessor(
                self.engine, self.log.reader(), device_deployments, zeebe_db=self.engine, key_generator=self.engine,
                partition_id=partition_id, partition_count=partition_count, instances=256, window=48,
                max_commands_in_batch=limit, clock=clock, correlation_keys=correlation_keys, command_sender=sender,
                engine_deployments=[d for d in deployments if d[1] not in dkeys])
            self.adapter.init()
            procs = [self.adapter, self.engine]
            timers, jobs = DeviceTimerInstanceState(self.adapter, timers), DeviceJobState(self.adapter, jobs)
            pending = DevicePendingSubscriptionState(self.adapter, pending)
        self.sp = StreamProcessor(self.log, procs, limit)
        self.service = ScheduleService(clock, self.log)
        self.timer_checker = DueDateTimerChecker(timers, clock)
        self.engine.due_date_checker = self.timer_checker
        if self.adapter:
            self.adapter.due_date_checker = self.timer_checker
        # StreamProcessorLifecycleAware.onRecovered, in registration order
        self.timer_checker.on_recovered(self.service)
        JobTimeoutTrigger(jobs, clock).on_recovered(self.service)
        # MessageObserver.onRecovered (:47-66): the TTL checker over the engine's MESSAGE_DEADLINES (the
        # device buffers no messages: a key with a buffered message is the engine's)
        MessageTimeToLiveChecker(EngineMessageState(self.engine), clock).on_recovered(self.service)
        if sender is not None:
            PendingProcessMessageSubscriptionChecker(pending, clock, sender).on_recovered(self.service)
            PendingMessageSubscriptionChecker(pending, clock, sender, partition_id).on_recovered(self.service)

    def state(self):
        # (string variables spelled out: the engine's and the device's dictionaries intern in their own order)
        eng = canon_strings(self.engine.state(), lambda i: self.engine.o.string_value(i).decode())
        if self.adapter is None:
            return sorted(eng)
        part = self.adapter.part
        assert part.current_key() <= self.engine.current_key()  # one key generator
        rows = canon_strings([r for r in part.state() if not r.startswith("KEY|")], part.string_value) + eng
        # MESSAGE_STATS: one messagesDeadlineCount row, the buffered messages of both (the device's are 0)
        stats = [r for r in rows if r.startswith("MESSAGE_STATS|")]
        if len(stats) > 1:
            rows = [r for r in rows if not r.startswith("MESSAGE_STATS|")] + \
                ["MESSAGE_STATS|messagesDeadlineCount|%d" % sum(int(r.rsplit("|", 1)[1]) for r in stats)]
        return sorted(rows)


class Cluster:
    def __init__(self, parts, clock):
        self.parts, self.clock = parts, clock

    def settle(self):
        """Every log processed and every due task run, until the partitions are quiet."""
        while True:
            run_cluster([p.sp for p in self.parts])
            if not any(p.service.run_one() for p in self.parts):
                return

    def increase_time(self, ms):
        """EngineRule.increaseTime: the clock moves on, the due scheduled tasks run."""
        self.clock.now += ms
        self.settle()


def check(ref, gpu):
    for p, (a, b) in enumerate(zip(ref.parts, gpu.parts), 1):
        want, got = a.log.canonical(), b.log.canonical()
        if got != want:
            n = min(len(got), len(want))
            bad = next((i for i in range(n) if got[i] != want[i]), n)
            ctx = "".join("\n  %d got  %s\n  %d want %s" % (i, got[i] if i < len(got) else None, i,
                                                          want[i] if i < len(want) else None)
                          for i in range(max(0, bad - 3), bad))
            raise AssertionError("partition %d log entry %d of %d/%d:\n got  %s\n want %s\n before:%s" % (
                p, bad, len(got), len(want), got[bad] if bad < len(got) else None, want[bad] if bad < len(want) else None,
                ctx))
        assert b.state() == a.state(), p


def write(ref, gpu, *recs, partition=0):
    Client(ref.parts[partition].log, gpu.parts[partition].log).write(*recs)
    ref.settle()
    gpu.settle()
    check(ref, gpu)


def step(ref, gpu, ms):
    ref.increase_time(ms)
    gpu.increase_time(ms)
    check(ref, gpu)


def single(deployments, device_deployments, limit=100):
    ref_clock, gpu_clock = Clock(NOW), Clock(NOW)
    ref = Cluster([PartitionLoop(ref_clock, deployments, limit=limit)], ref_clock)
    gpu = Cluster([PartitionLoop(gpu_clock, deployments, device_deployments, limit=limit)], gpu_clock)
    ref.settle()
    gpu.settle()
    return ref, gpu


def checker_commands(log, value_type, intent):
    """Commands of the log a scheduled task wrote (no source position)."""
    return [r for r in log.entries if r.record_type == abi.RT_COMMAND and r.value_type == value_type
            and r.intent == intent and r.source_position == -1]


def test_due_date_timer_checker_triggers_device_timers():
    # timer catch events, interrupting boundary timers and a non-interrupting cycle on the device, a
    # timer catch event of a process only the engine runs: the one checker task writes TIMER:TRIGGER for
    # all of them in TIMER_DUE_DATES order (dueDate, elementInstanceKey, key), reschedules itself at the
    # next dueDate, and some jobs complete first (their timers are canceled, never triggered)
    deps = [(timer_process("PT10S", pid="catch"), KEY_A, 1), (multiple_sequence_flows("PT30S"), KEY_B, 1),
            (cycle_process("R3/PT10S"), KEY_C, 1), (timer_process("PT15S", pid="engineTimer"), KEY_D, 1)]
    ref, gpu = single(deps, deps[:3])
    rng = np.random.default_rng(11)
    for wave in range(3):
        write(ref, gpu, *([Client.create("catch") for _ in range(4)] +
                          [Client.create("process", key=KEY_B if k % 2 else KEY_C) for k in range(8)] +
                          [Client.create("engineTimer") for _ in range(2)]))
        step(ref, gpu, 4000 + 1000 * wave)
    for t in range(8):
        jobs = sorted(open_jobs(ref.parts[0].log))
        done = [Client.complete_job(k) for k in jobs if rng.integers(0, 3) == 0]
        if done:
            write(ref, gpu, *done)
        step(ref, gpu, 7000)
    log = gpu.parts[0].log
    triggers = checker_commands(log, abi.VT_TIMER, abi.TIMER_TRIGGER)
    triggered = [r for r in log.entries if r.value_type == abi.VT_TIMER and r.intent == abi.TIMER_TRIGGERED]
    assert len(triggers) >= 30 and len(triggered) >= 30
    assert not [r for r in log.entries if r.value_type == abi.VT_TIMER and r.intent == abi.TIMER_TRIGGER
                and r.source_position != -1]
    c = gpu.parts[0].adapter.counts
    assert c["fallbacks"] == 0 and c["device_commands"] > 60
    # every catch timer fired: those instances completed
    assert not [k for k, r in open_jobs(ref.parts[0].log).items() if r.value["bpmnProcessId"] == "catch"]


def race(ref, gpu, recs, ms):
    """Commands reach the log, then the clock moves on and the due tasks run before the processing loop
    reads them (the actor runs the scheduled task first): a TIMER:TRIGGER written after a JOB:COMPLETE that
    cancels its timer is rejected NOT_FOUND, with the command's TimerRecord (TypedRejectionWriter)."""
    for cl in (ref, gpu):
        Client(cl.parts[0].log).write(*recs)
        cl.clock.now += ms
        while any(p.service.run_one() for p in cl.parts):
            pass
        cl.settle()
    check(ref, gpu)


def test_boundary_timers_racing_job_completions():
    # interrupting boundary timers and a non-interrupting cycle (R3/PT10S); some jobs complete in the
    # same instant their timers fire: the trigger is processed after the completion that canceled it
    deps = [(multiple_sequence_flows("PT30S"), KEY_A, 1), (cycle_process("R3/PT10S"), KEY_B, 1)]
    ref, gpu = single(deps, deps)
    write(ref, gpu, *[Client.create("process", key=KEY_A if k % 2 else KEY_B) for k in range(24)])
    rng = np.random.default_rng(9)
    for _ in range(6):
        jobs = sorted(open_jobs(ref.parts[0].log))
        if not jobs:
            break
        race(ref, gpu, [Client.complete_job(k) for k in jobs if rng.integers(0, 2)], 10000)
    log = gpu.parts[0].log
    rejected = [r for r in log.entries if r.record_type == abi.RT_REJECTION and r.value_type == abi.VT_TIMER]
    assert rejected and all(r.value["elementInstanceKey"] > 0 and r.value["targetElementId"] for r in rejected)
    assert gpu.parts[0].adapter.counts["fallbacks"] == 0


def test_job_timeout_trigger_times_out_device_jobs():
    # JobTimeOutTest: activated jobs past their deadline time out (JOB:TIME_OUT from the trigger with the
    # stored job, JOB:TIMED_OUT, ACTIVATABLE again with deadline and worker kept), are activated again and
    # completed -- their COMPLETED records carry the latest activation; device and engine jobs (a process
    # only the engine runs) in one deadline order; time-outs the processor rejects
    a = bpmn.linear_process(3)
    b = bpmn.linear_process(2, process_id="engineOnly", job_type="engine-task")
    deps = [(a, KEY_A, 1), (b, KEY_B, 1)]
    ref, gpu = single(deps, deps[:1])
    write(ref, gpu, *([Client.create("linear") for _ in range(10)] + [Client.create("engineOnly") for _ in range(4)]))
    clock = ref.clock
    write(ref, gpu, Client.activate_jobs("benchmark-task", worker="w1", timeout=10000, max_jobs=6,
                                         timestamp=clock.now),
          Client.activate_jobs("engine-task", worker="e1", timeout=5000, max_jobs=2, timestamp=clock.now))
    step(ref, gpu, 12000)
    write(ref, gpu, Client.activate_jobs("benchmark-task", worker="w2", timeout=40000, max_jobs=3,
                                         timestamp=clock.now))
    step(ref, gpu, 20000)  # the first time-out run (30 s after recovery)
    log = gpu.parts[0].log
    assert len(checker_commands(log, abi.VT_JOB, abi.JOB_TIME_OUT)) == 8
    timed_out = [r for r in log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_TIMED_OUT]
    assert len(timed_out) == 8 and all(r.value["worker"] in ("w1", "e1") for r in timed_out)
    # restart: timed-out jobs (JOB_STATES ACTIVATABLE, the record's deadline and worker kept) survive
    # export -> import, and the fresh handle activates them again
    from zeebe_amd.engine import Partition
    part = gpu.parts[0].adapter.part
    fresh = Partition(max_instances=256, max_commands=48)
    fresh.deploy(a, process_definition_key=KEY_A)
    fresh.import_state_db(part.state_db())
    assert fresh.state() == part.state()
    assert len(fresh.timed_out_jobs(clock.now + 10 ** 9)) == 3  # the three w2 activations
    key, jobs, _ = fresh.activate_jobs("benchmark-task", worker="again", max_jobs=20, timestamp=clock.now)
    assert key > 0 and len(jobs) == 10 - 3
    # timed-out jobs are activatable again: a new worker, then some complete, the rest time out again
    write(ref, gpu, Client.activate_jobs("benchmark-task", worker="w3", timeout=10000, max_jobs=10,
                                         timestamp=clock.now))
    jobs = sorted(open_jobs(ref.parts[0].log))
    write(ref, gpu, *[Client.complete_job(k) for k in jobs[::3]])
    # the rejections JobTimeOutProcessor writes: a completed job, an ACTIVATABLE one, one not timed out yet
    live = open_jobs(ref.parts[0].log)
    gone = jobs[0]
    activatable = next(k for k, r in sorted(live.items()) if r.value["bpmnProcessId"] == "engineOnly")
    value = {"type": "benchmark-task", "retries": 3, "tenantId": "<default>", "variables": ()}
    write(ref, gpu, Rec(abi.RT_COMMAND, abi.VT_JOB, abi.JOB_TIME_OUT, gone, value),
          Rec(abi.RT_COMMAND, abi.VT_JOB, abi.JOB_TIME_OUT, sorted(live)[0], value),
          Rec(abi.RT_COMMAND, abi.VT_JOB, abi.JOB_TIME_OUT, activatable, value))
    rej = [r for r in log.entries if r.record_type == abi.RT_REJECTION and r.intent == abi.JOB_TIME_OUT]
    assert len(rej) == 3 and "no such job was found" in rej[0].rejection_reason
    step(ref, gpu, 30000)
    for _ in range(4):
        jobs = sorted(open_jobs(ref.parts[0].log))
        if not jobs:
            break
        write(ref, gpu, Client.activate_jobs("benchmark-task", worker="w4", timeout=1000, max_jobs=4,
                                             timestamp=clock.now))
        write(ref, gpu, *[Client.complete_job(k) for k in jobs])
        step(ref, gpu, 30000)
    completed = [r for r in log.entries if r.value_type == abi.VT_JOB and r.intent == abi.JOB_COMPLETED]
    assert any(r.value.get("worker") == "w3" for r in completed)
    assert gpu.parts[0].adapter.counts["time_outs"] >= 8 and gpu.parts[0].adapter.counts["fallbacks"] == 0


# ---- config 5: sends lost between partitions, sent again by the pending-subscription checkers ----
P = 3
MSG_XML = bpmn.message_catch_process(message_name="message", correlation_key="key", catch_id="receive-message")
KEYS = ["item-2", "item-1", "item-0"] + ["order-%d" % j for j in range(7)]


class LossySender(InterPartitionCommandSender):
    """TestInterPartitionCommandSender that loses the first send of some subscriptions' commands (every
    third element instance key, per value type and intent): the receiver never sees them."""

    def __init__(self, logs, lose):
        super().__init__(logs)
        self.lose = lose
        self.seen = set()
        self.lost = 0

    def send_command(self, receiver_partition, value_type, intent, value, key=-1):
        k = (value_type, intent, value["elementInstanceKey"])
        if (value_type, intent) in self.lose and k not in self.seen and value["elementInstanceKey"] % 3 == 0:
            self.seen.add(k)
            self.lost += 1
            return
        self.seen.add(k)
        super().send_command(receiver_partition, value_type, intent, value, key)


def message_clusters(lose):
    def make(device):
        clock = Clock(NOW)
        logs = {p: Log() for p in range(1, P + 1)}
        sender = LossySender(logs, lose)
        parts = [PartitionLoop(clock, [(MSG_XML, KEY_A, 1)], [(MSG_XML, KEY_A, 1)] if device else None,
                               partition_id=p, partition_count=P, sender=sender, log=logs[p],
                               correlation_keys=64) for p in range(1, P + 1)]
        cl = Cluster(parts, clock)
        cl.sender = sender
        cl.settle()
        return cl
    return make(False), make(True)


@pytest.mark.parametrize("lose", ["open", "correlate"])
def test_pending_subscription_checkers_resend_lost_commands(lose):
    # "open": MESSAGE_SUBSCRIPTION:CREATE lost -> the PI partition's subscription stays OPENING and
    # PendingProcessMessageSubscriptionChecker sends it again; "correlate": PROCESS_MESSAGE_SUBSCRIPTION:
    # CORRELATE lost -> the message partition's subscription stays CORRELATING and the MessageObserver's
    # checker correlates again.  Then every instance completes, on every partition as in the reference.
    from oracle.oracle import subscription_partition
    kinds = {"open": {(abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_CREATE)},
             "correlate": {(abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CORRELATE)}}[lose]
    ref, gpu = message_clusters(kinds)
    for cl in (ref, gpu):
        for i in range(30):
            Client(cl.parts[(i + i // 10) % 3].log).write(Client.create("process", (("key", KEYS[i % 10]),)))
        cl.settle()
    check(ref, gpu)
    if lose == "open":
        step(ref, gpu, 15000)
        step(ref, gpu, 20000)  # the checker's run 30 s after recovery: OPENING for more than 10 s
    pubs = {p: [] for p in range(1, P + 1)}
    for k in KEYS:
        pubs[subscription_partition(k, P)] += [Client.publish_message("message", k) for _ in range(3)]
    for p, recs in sorted(pubs.items()):
        Client(ref.parts[p - 1].log, gpu.parts[p - 1].log).write(*recs)
    ref.settle()
    gpu.settle()
    check(ref, gpu)
    for _ in range(3):
        step(ref, gpu, 30000)
    assert ref.sender.lost == gpu.sender.lost > 0
    done = sum(1 for p in gpu.parts for r in p.log.entries
               if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == 5 and r.value["bpmnElementType"] == "PROCESS")
    assert done == 30
    c = [p.adapter.counts for p in gpu.parts]
    assert all(x["fallbacks"] == 0 for x in c), [p.adapter.fallback_reasons for p in gpu.parts]


def test_sub_process_boundary_timers_in_the_processing_loop():
    """Timer boundary events on embedded sub-processes behind the adapter: the DueDateTimerChecker's
    TIMER:TRIGGER terminates a sub-process (PROCESS_INSTANCE_BATCH:TERMINATE of its children, their jobs
    canceled) before its boundary event, or -- non-interrupting -- runs the boundary path beside it;
    jobs completed first cancel the timers.  Logs and state equal the engine-only loop's."""
    from test_oracle_boundary import sub_process_boundary
    from test_gpu_boundary import _sub_process_parallel
    deps = [(sub_process_boundary(True, "PT10S"), KEY_A, 1), (_sub_process_parallel(False), KEY_B, 1)]
    ref, gpu = single(deps, deps)
    rng = np.random.default_rng(5)
    write(ref, gpu, *([Client.create("process", key=KEY_A) for _ in range(6)] +
                      [Client.create("process", key=KEY_B) for _ in range(6)]))
    for t in range(6):
        jobs = sorted(open_jobs(ref.parts[0].log))
        done = [Client.complete_job(k) for k in jobs if rng.integers(0, 3) == 0]
        if done:
            write(ref, gpu, *done)
        step(ref, gpu, 7000)
    check(ref, gpu)
    log = gpu.parts[0].log
    assert any(r.value_type == abi.VT_PROCESS_INSTANCE_BATCH for r in log.entries)
    assert gpu.parts[0].adapter.counts["fallbacks"] == 0, gpu.parts[0].adapter.fallback_reasons


def test_truncated_device_scans_keep_the_checkers_order():
    """zbhip_due_timers / zbhip_timed_out_jobs return at most a cap of rows; a truncated device list may
    leave out a row ordered before engine entries past its last returned row, so the merged views stop
    there (DeviceTimerInstanceState / DeviceJobState) and the checkers' next runs take the rest.  With the
    cap forced to 4, the TIMER:TRIGGER and JOB:TIME_OUT commands reach the log in the engine-only loop's
    order (TIMER_DUE_DATES [dueDate, elementInstanceKey, timerKey], JOB_DEADLINES [deadline, jobKey]),
    over several checker runs instead of one, and every instance ends in the same state."""
    deps = [(timer_process("PT10S", pid="catch"), KEY_A, 1), (timer_process("PT10S", pid="engineTimer"), KEY_D, 1),
            (bpmn.linear_process(1), KEY_B, 1), (bpmn.linear_process(1, process_id="engineOnly", job_type="engine-task"),
                                                 KEY_C, 1)]
    ref, gpu = single(deps, deps[:1] + deps[2:3])
    gpu.parts[0].adapter.scheduled_cap = 4
    # timers with one dueDate, device and engine instances interleaved in key order
    write(ref, gpu, *[Client.create("catch" if k % 3 else "engineTimer") for k in range(18)])
    write(ref, gpu, *[Client.create("linear" if k % 3 else "engineOnly") for k in range(15)])
    clock = ref.clock
    write(ref, gpu, Client.activate_jobs("benchmark-task", worker="w", timeout=5000, max_jobs=20, timestamp=clock.now),
          Client.activate_jobs("engine-task", worker="e", timeout=5000, max_jobs=20, timestamp=clock.now))
    for cl in (ref, gpu):
        cl.increase_time(15000)
        for _ in range(12):  # the checkers' later runs (100 ms / 30 s apart)
            cl.increase_time(30000)

    def order(cl, vt, it):
        return [r.key for r in checker_commands(cl.parts[0].log, vt, it)]
    triggers = order(gpu, abi.VT_TIMER, abi.TIMER_TRIGGER)
    assert len(triggers) == 18 and triggers == order(ref, abi.VT_TIMER, abi.TIMER_TRIGGER)
    time_outs = order(gpu, abi.VT_JOB, abi.JOB_TIME_OUT)
    assert len(time_outs) == 15 and time_outs == order(ref, abi.VT_JOB, abi.JOB_TIME_OUT)
    # the truncated scans spread them over several checker runs (batches without a source position)
    runs = {r.position - i for i, r in enumerate(checker_commands(gpu.parts[0].log, abi.VT_TIMER, abi.TIMER_TRIGGER))}
    assert len(runs) > 1
    for cl in (ref, gpu):
        live = sorted(open_jobs(cl.parts[0].log))
        Client(cl.parts[0].log).write(*[Client.complete_job(k) for k in live])
        cl.settle()
    assert gpu.parts[0].state() == ref.parts[0].state()
