"""TEST INFRASTRUCTURE -- a restatement of stream-platform's processing loop over an in-memory log, the
harness the reference's own platform tests use (stream-platform/src/test/.../StreamPlatform.java:63-85:
ListLogStorage + SyncLogStream, a mocked RecordProcessor), with the CPU oracle as the engine behind
the RecordProcessor interface.

* :class:`Log` / :class:`Reader` -- the log stream: entries with positions, source positions and the
  processed flag (LogAppendEntry.ofProcessed, LogEntryDescriptor skipProcessing).
* :class:`StreamProcessor` -- ProcessingStateMachine.processCommand / batchProcessing /
  collectBatchProcessingStepResult (stream-platform/.../stream/impl/ProcessingStateMachine.java:
  247-417): one batch per unprocessed command read from the log, a FIFO of follow-up commands fed back
  as UnwrittenRecords while pending + processed + new < maxCommandsInBatch, the rest written
  unprocessed; the batch is appended to the log with sourceRecordPosition = the initial command's
  position, then its post-commit tasks run (executeSideEffects, :546-590).
* :class:`OracleEngine` -- the reference engine (oracle/zb_oracle.cpp process_one: Engine.process for
  one command) as a RecordProcessor, with the partition's key generator (DbKeyGenerator) and the
  RawDbWriter of a hand-off (import_rows).
* :class:`Client` -- the EngineRule test clients writing commands to the log.
* :class:`Clock` / :class:`ScheduleService` and the checkers -- ActorClock under test control
  (EngineRule.increaseTime) and ProcessingScheduleServiceImpl: tasks run between batches, a task's
  commands are written to the log as one batch; DueDateChecker / DueDateTimerChecker, JobTimeoutTrigger,
  PendingProcessMessageSubscriptionChecker and MessageObserver's PendingMessageSubscriptionChecker
  restated over a state view (the engine's, or the adapter's merged device + engine view).

Only tests use this module (it loads the oracle)."""
import numpy as np

from oracle.oracle import Oracle
from zeebe_amd import abi
from zeebe_amd.adapter import (JOB_BATCH_ACTIVATE, JOB_BATCH_ACTIVATED, MESSAGE_VALUE_TYPES, VT_JOB_BATCH, XPART_COMMAND,
                               RecordValues, doc_entries, push_side_effects, typed_value, xpart_value)
from zeebe_amd.engine import ProcessDefinition, msgpack_string_map


class RecordingJobStream:
    """RecordingJobStreamer's stream (engine/src/test/.../util/RecordingJobStreamer.java): the pushed
    ActivatedJobs, (jobKey, job record value) in push order."""

    def __init__(self):
        self.activated_jobs = []

    def push(self, job_key, job):
        self.activated_jobs.append((job_key, job))


class RecordingJobStreamer:
    """RecordingJobStreamer's notifications (engine/src/test/.../util/RecordingJobStreamer.java:22-32):
    notifyWorkAvailable(jobType) counted per type -- publishWork's side effect for a job made activatable
    with no stream for its type (BpmnJobActivationBehavior.java:97-111)."""

    def __init__(self):
        self.notifications = {}

    def notify_work_available(self, job_type):
        self.notifications[job_type] = self.notifications.get(job_type, 0) + 1


class Rec:
    """A logged record (LoggedEvent + TypedRecord); position None = UnwrittenRecord."""
    __slots__ = ("position", "source_position", "record_type", "value_type", "intent", "key", "rejection_type",
                 "rejection_reason", "value", "processed", "timestamp")

    def __init__(self, record_type, value_type, intent, key, value, rejection_type=abi.REJ_NONE, rejection_reason="",
                 position=None, source_position=-1, processed=False, timestamp=0):
        self.record_type, self.value_type, self.intent, self.key = record_type, value_type, intent, key
        self.value, self.rejection_type, self.rejection_reason = value, rejection_type, rejection_reason
        self.position, self.source_position, self.processed, self.timestamp = position, source_position, processed, timestamp

    def canonical(self):
        return (self.position, self.source_position, self.record_type, self.value_type, self.intent, self.key,
                self.rejection_type, self.rejection_reason, self.processed, _canon(self.value))

    def __repr__(self):
        return "Rec(%s)" % (self.canonical(),)


def _canon(v):
    if isinstance(v, dict):
        return tuple(sorted((k, _canon(x)) for k, x in v.items()))
    if isinstance(v, (list, tuple)):
        return tuple(_canon(x) for x in v)
    return v


class Log:
    def __init__(self):
        self.entries = []

    def append(self, recs, source_position=-1):
        for r in recs:
            r.position = len(self.entries) + 1
            r.source_position = source_position
            self.entries.append(r)

    def reader(self):
        return Reader(self)

    def canonical(self):
        return [r.canonical() for r in self.entries]


class Reader:
    def __init__(self, log):
        self.log = log
        self.i = 0

    def seek(self, position):
        self.i = position - 1

    def has_next(self):
        return self.i < len(self.log.entries)

    def next(self):
        r = self.log.entries[self.i]
        self.i += 1
        return r


class Builder:
    """BufferedProcessingResultBuilder (+ the ProcessingResult it builds)."""

    def __init__(self):
        self.entries = []
        self.post_commit = []

    def append_record(self, key, record_type, value_type, intent, rejection_type, rejection_reason, value):
        self.entries.append(Rec(record_type, value_type, intent, key, value, rejection_type, rejection_reason))

    def append_post_commit_task(self, task):
        self.post_commit.append(task)

    def build(self):
        return self


class StreamProcessor:
    """ProcessingStateMachine (stream-platform/.../stream/impl/ProcessingStateMachine.java:247-417)."""

    def __init__(self, log, processors, max_commands_in_batch=100):
        self.log = log
        self.processors = processors
        self.limit = max_commands_in_batch
        self.read = 0
        self.batches = 0

    def run(self):
        """Processes the log to its end (readNextRecord -> processCommand, :199-310)."""
        while self.read < len(self.log.entries):
            rec = self.log.entries[self.read]
            self.read += 1
            if rec.record_type == abi.RT_COMMAND and not rec.processed:
                self._process_command(rec)

    def _process_command(self, initial):
        builder = Builder()
        pending, writes = [initial], []
        processed = last_size = 0
        while pending and processed < self.limit:
            command = pending.pop(0)
            proc = next((p for p in self.processors if p.accepts(command.value_type)), None)
            if proc is not None:
                result = proc.process(command, builder)
                # collectBatchProcessingStepResult (:388-417)
                to_process = []
                current = len(pending) + processed + 1
                for e in result.entries[last_size:]:
                    w = Rec(e.record_type, e.value_type, e.intent, e.key, e.value, e.rejection_type, e.rejection_reason)
                    if e.record_type == abi.RT_COMMAND and current + len(to_process) < self.limit:
                        to_process.append(Rec(e.record_type, e.value_type, e.intent, e.key, e.value))
                        w.processed = True  # LogAppendEntry.ofProcessed
                    writes.append(w)
                pending.extend(to_process)
                last_size = len(result.entries)
            processed += 1
        self.log.append(writes, initial.position)
        self.batches += 1
        for task in builder.post_commit:  # executeSideEffects: post-commit tasks after the write
            task()


def oracle_tables(o):
    """The oracle's deployments as ProcessDefinitions (the adapter's RecordValues input)."""
    out = []
    for i, t in enumerate(o.process_tables()):
        els = t["elements"]
        out.append(ProcessDefinition(i, t["bpmn_process_id"], [e[2] for e in els], [abi.ELEMENT_TYPES[e[0]] for e in els],
                                     [e[3] or None for e in els], [abi.EVENT_TYPES[e[1]] for e in els],
                                     [e[4] for e in els], t["version"], t["key"],
                                     [msgpack_string_map(h) if h else () for h in t["headers"]]))
    return out


class Clock:
    """ActorClock (the controlled clock of EngineRule: increaseTime)."""

    def __init__(self, now=0):
        self.now = now

    def __call__(self):
        return self.now


class TaskResultBuilder:
    """stream-platform's TaskResultBuilder: appendCommandRecord(key, intent, value) of a scheduled task."""

    def __init__(self):
        self.records = []

    def append_command_record(self, key, value_type, intent, value):
        self.records.append(Rec(abi.RT_COMMAND, value_type, intent, key, value))
        return True


class ScheduleService:
    """ProcessingScheduleServiceImpl (stream-platform/.../scheduling/ProcessingScheduleServiceImpl.java):
    runDelayed / runAtFixedRate on the partition's actor; a task's result (its commands) is written to
    the log as one batch without a source position.  run_due() runs the tasks due at the clock's time,
    earliest first (same time: scheduling order)."""

    def __init__(self, clock, log):
        self.clock, self.log = clock, log
        self.tasks = []
        self.seq = 0

    def run_delayed(self, delay, task):
        self.seq += 1
        self.tasks.append((self.clock.now + max(delay, 0), self.seq, task, None))

    def run_at_fixed_rate(self, delay, runnable):
        self.seq += 1
        self.tasks.append((self.clock.now + delay, self.seq, runnable, delay))

    def next_due(self):
        return min((t[0], t[1]) for t in self.tasks) if self.tasks else None

    def run_one(self):
        """Runs the earliest due task; False when none is due."""
        due = [t for t in self.tasks if t[0] <= self.clock.now]
        if not due:
            return False
        t = min(due, key=lambda x: (x[0], x[1]))
        self.tasks.remove(t)
        _, _, task, rate = t
        if rate is not None:  # a Runnable at fixed rate: no result, rescheduled
            task()
            self.seq += 1
            self.tasks.append((self.clock.now + rate, self.seq, task, rate))
            return True
        builder = TaskResultBuilder()
        task(builder)
        self.log.append(builder.records)
        return True


class DueDateTimerChecker:
    """DueDateTimerChecker + DueDateChecker (engine/.../processing/timer/DueDateTimerChecker.java:24-130,
    processing/scheduled/DueDateChecker.java): one task for all timers, scheduled at the earliest known
    dueDate (TIMER_RESOLUTION 100 ms floor); it writes TIMER:TRIGGER for every timer due (key = the
    timer, the TimerInstance's TimerRecord) and reschedules itself at the first dueDate left."""
    TIMER_RESOLUTION = 100

    def __init__(self, timer_state, clock):
        self.state, self.clock = timer_state, clock
        self.service = None
        self.running = False
        self.next_due = -1

    def on_recovered(self, service):
        self.service = service
        service.run_delayed(0, self._task)  # timers due after a restart

    def _delay(self, due):
        return max(due - self.clock.now, self.TIMER_RESOLUTION)

    def schedule_timer(self, due):
        if not self.running:
            self.service.run_delayed(self._delay(due), self._task)
            self.next_due, self.running = due, True
        elif self.next_due - due > self.TIMER_RESOLUTION:
            self.service.run_delayed(self._delay(due), self._task)
            self.next_due = due

    def _task(self, builder):
        def visit(key, value):
            return builder.append_command_record(key, abi.VT_TIMER, abi.TIMER_TRIGGER, dict(value))
        self.next_due = self.state.process_timers_with_due_date_before(self.clock.now, visit)
        if self.next_due > 0:
            self.service.run_delayed(self._delay(self.next_due), self._task)
            self.running = True
        else:
            self.running = False


class JobTimeoutTrigger:
    """JobTimeoutTrigger (engine/.../processing/job/JobTimeoutTrigger.java:21-88): every 30 s, JOB:TIME_OUT
    for each job in JOB_DEADLINES with deadline < now (key = the job, value = the stored job)."""
    INTERVAL = 30000

    def __init__(self, job_state, clock):
        self.state, self.clock = job_state, clock

    def on_recovered(self, service):
        self.service = service
        service.run_delayed(self.INTERVAL, self._task)

    def _task(self, builder):
        self.state.for_each_timed_out_entry(
            self.clock.now, lambda key, value: builder.append_command_record(key, abi.VT_JOB, abi.JOB_TIME_OUT, dict(value)))
        self.service.run_delayed(self.INTERVAL, self._task)


class EngineMessageState:
    """The engine's MessageState for the MessageTimeToLiveChecker (its MESSAGE_DEADLINES rows):
    DbMessageState.visitMessagesWithDeadlineBeforeTimestamp (:408-434), [deadline, messageKey] order."""

    def __init__(self, engine):
        self.engine = engine

    def deadlines(self):
        out = []
        for r in self.engine.state():
            if r.startswith("MESSAGE_DEADLINES|"):
                _, d, k = r.split("|")
                out.append((int(d), int(k)))
        return sorted(out)

    def visit_messages_with_deadline_before(self, timestamp, visitor):
        for deadline, key in self.deadlines():
            if deadline > timestamp or not visitor(deadline, key):
                return


class MessageTimeToLiveChecker:
    """MessageTimeToLiveChecker (engine/.../processing/message/MessageTimeToLiveChecker.java:35-124),
    scheduled by MessageObserver.onRecovered (:47-66) after messagesTtlCheckerInterval (EngineConfiguration:
    1 min; batch limit Integer.MAX_VALUE): one MESSAGE_BATCH:EXPIRE with the keys of every message whose
    deadline <= now, then again after the interval."""
    INTERVAL = 60000

    def __init__(self, message_state, clock):
        self.state, self.clock = message_state, clock

    def on_recovered(self, service):
        self.service = service
        service.run_delayed(self.INTERVAL, self._task)

    def _task(self, builder):
        keys = []
        self.state.visit_messages_with_deadline_before(self.clock.now, lambda d, k: keys.append(k) or True)
        if keys:
            builder.append_command_record(-1, abi.VT_MESSAGE_BATCH, abi.MESSAGE_BATCH_EXPIRE,
                                          {"messageKeys": tuple(keys)})
        self.service.run_delayed(self.INTERVAL, self._task)


def open_message_subscription_value(r):
    """SubscriptionCommandSender.sendDirectOpenMessageSubscription (:83-110) from the stored
    ProcessMessageSubscriptionRecord."""
    return {"processInstanceKey": r["processInstanceKey"], "elementInstanceKey": r["elementInstanceKey"],
            "messageKey": -1, "messageName": r["messageName"], "correlationKey": r["correlationKey"],
            "interrupting": r["interrupting"], "bpmnProcessId": r["bpmnProcessId"], "variables": (),
            "tenantId": "<default>"}


def close_message_subscription_value(r):
    """SubscriptionCommandSender.sendDirectCloseMessageSubscription (:236-264)."""
    return {"processInstanceKey": r["processInstanceKey"], "elementInstanceKey": r["elementInstanceKey"],
            "messageKey": -1, "messageName": r["messageName"], "correlationKey": "", "interrupting": True,
            "bpmnProcessId": "", "variables": (), "tenantId": "<default>"}


def correlate_process_message_subscription_value(r, sender):
    """SubscriptionCommandSender.sendDirectCorrelateProcessMessageSubscription (:160-198)."""
    return {"subscriptionPartitionId": sender, "processInstanceKey": r["processInstanceKey"],
            "elementInstanceKey": r["elementInstanceKey"], "messageKey": r["messageKey"],
            "messageName": r["messageName"], "variables": tuple(r.get("variables", ())), "interrupting": True,
            "bpmnProcessId": r["bpmnProcessId"], "correlationKey": r["correlationKey"], "elementId": "",
            "tenantId": "<default>"}


class PendingProcessMessageSubscriptionChecker:
    """PendingProcessMessageSubscriptionChecker (engine/.../message/PendingProcessMessageSubscriptionChecker
    .java:20-129): every 30 s, subscriptions still OPENING / CLOSING 10 s after they were last sent are
    sent again directly (MESSAGE_SUBSCRIPTION:CREATE / DELETE to the subscription partition)."""
    TIMEOUT, INTERVAL = 10000, 30000

    def __init__(self, pending, clock, sender):
        self.pending, self.clock, self.sender = pending, clock, sender

    def on_recovered(self, service):
        self.service = service
        service.run_delayed(self.INTERVAL, self._task)

    def _task(self, builder):
        for _, sub, r, opening in self.pending.pending_process_message_subscriptions(self.clock.now - self.TIMEOUT):
            if opening:
                self.sender.send_command(r["subscriptionPartitionId"], abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_CREATE,
                                         open_message_subscription_value(r))
            else:
                self.sender.send_command(r["subscriptionPartitionId"], abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_DELETE,
                                         close_message_subscription_value(r))
            self.pending.on_sent_pms(sub, self.clock.now)
        self.service.run_delayed(self.INTERVAL, self._task)


class PendingMessageSubscriptionChecker:
    """MessageObserver's PendingMessageSubscriptionChecker (engine/.../message/MessageObserver.java:61-73,
    PendingMessageSubscriptionChecker.java:15-57): at a fixed rate of 30 s, CORRELATING subscriptions
    last sent 10 s ago or earlier are correlated again (PROCESS_MESSAGE_SUBSCRIPTION:CORRELATE to the
    process instance's partition)."""
    TIMEOUT, INTERVAL = 10000, 30000

    def __init__(self, pending, clock, sender, partition_id):
        self.pending, self.clock, self.sender, self.partition_id = pending, clock, sender, partition_id

    def on_recovered(self, service):
        service.run_at_fixed_rate(self.INTERVAL, self.run)

    def run(self):
        for _, sub, r in self.pending.pending_message_subscriptions(self.clock.now - self.TIMEOUT):
            self.sender.send_command(r["processInstanceKey"] >> 51, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION,
                                     abi.PMS_CORRELATE, correlate_process_message_subscription_value(r, self.partition_id))
            self.pending.on_sent_ms(sub, self.clock.now)


def _row_fields(text):
    out = {}
    for kv in text.split(","):
        k, _, v = kv.partition("=")
        out[k] = v
    return out


class EngineTimerState:
    """The engine's TimerInstanceState (its TIMERS / TIMER_DUE_DATES rows): due(now) -> [(dueDate,
    elementInstanceKey, key, TimerRecord)], next_after(now); process_timers_with_due_date_before for the
    engine-only loop."""

    def __init__(self, engine):
        self.engine = engine

    def _timers(self):
        out = []
        for r in self.engine.state():
            if r.startswith("TIMERS|"):
                _, eik, key, f = r.split("|", 3)
                f = _row_fields(f)
                out.append((int(f["dueDate"]), int(eik), int(key),
                            {"elementInstanceKey": int(eik), "processInstanceKey": int(f["processInstanceKey"]),
                             "dueDate": int(f["dueDate"]), "repetitions": int(f["repetitions"]),
                             "targetElementId": f["handlerNodeId"],
                             "processDefinitionKey": int(f["processDefinitionKey"]), "tenantId": "<default>"}))
        return sorted(out, key=lambda t: t[:3])

    def due(self, now):
        return [t for t in self._timers() if t[0] <= now]

    def next_after(self, now):
        later = [t[0] for t in self._timers() if t[0] > now]
        return min(later) if later else -1

    def process_timers_with_due_date_before(self, now, visitor):
        for due, _, key, value in self._timers():
            if due > now or not visitor(key, value):
                return due
        return -1


class EngineJobState:
    """The engine's JobState (JOBS / JOB_STATES / JOB_DEADLINES rows): timed_out(now) -> [(deadline, key,
    JobRecord)]; for_each_timed_out_entry for the engine-only loop."""

    def __init__(self, engine):
        self.engine = engine

    def timed_out(self, now):
        rows = self.engine.state()
        jobs = {}
        for r in rows:
            if r.startswith("JOBS|"):
                _, key, f = r.split("|", 2)
                jobs[int(key)] = _row_fields(f)
        out = []
        for r in rows:
            if r.startswith("JOB_DEADLINES|"):
                _, deadline, key = r.split("|")
                deadline, key = int(deadline), int(key)
                if deadline < now:
                    f = jobs[key]
                    out.append((deadline, key, {
                        "tenantId": "<default>", "variables": (), "type": f["type"], "retries": int(f["retries"]),
                        "elementId": f["elementId"], "elementInstanceKey": int(f["elementInstanceKey"]),
                        "processInstanceKey": int(f["processInstanceKey"]), "bpmnProcessId": f["bpmnProcessId"],
                        "processDefinitionVersion": int(f["processDefinitionVersion"]),
                        "processDefinitionKey": int(f["processDefinitionKey"]), "deadline": int(f["deadline"]),
                        "worker": f["worker"]}))
                    if "errorMessageHex" in f:  # a failed job's stored errorMessage
                        out[-1][2]["errorMessage"] = bytes.fromhex(f["errorMessageHex"]).decode()
        return sorted(out, key=lambda t: t[:2])

    def for_each_timed_out_entry(self, now, callback):
        for _, key, value in self.timed_out(now):
            if not callback(key, value):
                return


class PendingStates:
    """The engine's TransientPendingSubscriptionState pair, kept by its appliers (DbProcessMessage
    SubscriptionState.java:82-124,180-222, DbMessageSubscriptionState.java:157-222): OPENING / CLOSING
    process message subscriptions and CORRELATING message subscriptions with their last sent time."""

    def __init__(self, clock):
        self.clock = clock
        self.pms, self.ms = {}, {}

    def track(self, rt, vt, it, value):
        if rt != abi.RT_EVENT:
            return
        if vt == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION:
            sub = (value["elementInstanceKey"], value["messageName"])
            if it in (abi.PMS_CREATING, abi.PMS_DELETING):
                self.pms[sub] = [self.clock.now, dict(value), it == abi.PMS_CREATING]
            elif it in (abi.PMS_CREATED, abi.PMS_DELETED, abi.PMS_CORRELATED):
                self.pms.pop(sub, None)
        elif vt == abi.VT_MESSAGE_SUBSCRIPTION:
            sub = (value["elementInstanceKey"], value["messageName"])
            if it == abi.MS_CORRELATING:
                self.ms[sub] = [self.clock.now, dict(value)]
            elif it in (abi.MS_CORRELATED, abi.MS_DELETED):
                self.ms.pop(sub, None)

    def pending_process_message_subscriptions(self, deadline):
        return sorted(((t, sub, r, op) for sub, (t, r, op) in self.pms.items() if t < deadline), key=lambda x: x[0])

    def add_pms(self, sub, sent, record, opening):
        """TransientPendingSubscriptionState.add of a subscription whose row came in with a hand-off."""
        self.pms[sub] = [sent, record, opening]

    def pending_message_subscriptions(self, deadline):
        return sorted(((t, sub, r) for sub, (t, r) in self.ms.items() if t < deadline), key=lambda x: x[0])

    def add_ms(self, sub, sent, record):
        """TransientPendingSubscriptionState.add of a CORRELATING subscription whose row came in with a
        correlation key's move to the engine."""
        self.ms[sub] = [sent, record]

    def on_sent_pms(self, sub, when):
        if sub in self.pms:
            self.pms[sub][0] = when

    def on_sent_ms(self, sub, when):
        if sub in self.ms:
            self.ms[sub][0] = when


class OracleEngine:
    """The reference engine as a RecordProcessor (Engine.java:71-131), one command per process call;
    also the partition's DbKeyGenerator (KeyGeneratorControls) and the RawDbWriter of a hand-off."""

    ACCEPTS = (abi.VT_PROCESS_INSTANCE_CREATION, abi.VT_JOB, abi.VT_TIMER, abi.VT_PROCESS_INSTANCE, VT_JOB_BATCH,
               abi.VT_PROCESS_INSTANCE_BATCH, abi.VT_MESSAGE_BATCH) + MESSAGE_VALUE_TYPES

    def __init__(self, partition_id=1, max_commands_in_batch=100, clock=0, partition_count=1, command_sender=None):
        self.o = Oracle(partition_id=partition_id, partition_count=partition_count,
                        max_commands_in_batch=max_commands_in_batch)
        self.command_sender = command_sender  # InterPartitionCommandSender of config 5
        self.clock = clock if isinstance(clock, Clock) else None  # a controlled ActorClock, or a fixed time
        self.o.set_clock(clock.now if self.clock else clock)
        self.due_date_checker = None  # DueDateTimerChecker.scheduleTimer (TIMER:CREATED side effects)
        self.pending = PendingStates(self.clock or Clock(clock))
        self.pbits = partition_id << 51
        self.slot_of = {}
        self.next_slot = 0
        self.doc_values = []  # client value of every document entry the oracle holds (its doc indices)
        self.tables = []
        self.streams = {}  # job streams: type -> (worker, timeout)
        self.stream_sinks = {}  # job type -> (fetchVariables, push)
        self.job_streamer = None  # JobStreamer.notifyWorkAvailable of publishWork without a stream
        self.o.take_notified()  # (the oracle keeps its notifications from now on)
        self.values = RecordValues([], self.o.name, lambda i: self.o.string_value(i).decode(),
                                   list_items=self.o.list_items, streams=self.streams)

    def deploy(self, xml, key, version=1):
        idx = self.o.deploy(xml, key, version)
        self.tables = oracle_tables(self.o)
        self.values = RecordValues(self.tables, self.o.name, lambda i: self.o.string_value(i).decode(),
                                   list_items=self.o.list_items,
                                   streams=self.streams)
        return idx

    def set_job_stream(self, job_type, worker, timeout, on=True, fetch_variables=(), push=None):
        """A job stream (JobStreamer.streamFor) of `job_type`: created jobs are pushed -- JOB_BATCH:ACTIVATED,
        and after the commit push(jobKey, job) with its `fetch_variables`."""
        self.o.set_job_stream(job_type, worker, timeout, on)
        if on:
            self.streams[job_type] = (worker, timeout)
            if push is not None:
                self.stream_sinks[job_type] = (tuple(fetch_variables), push)
        else:
            self.streams.pop(job_type, None)
            self.stream_sinks.pop(job_type, None)

    def set_clock(self, now):
        self.o.set_clock(now)

    # KeyGeneratorControls
    def current_key(self):
        return self.pbits + self.o.key_counter()

    def set_key_if_higher(self, key):
        if key - self.pbits > self.o.key_counter():
            self.o.set_key_counter(key - self.pbits)

    # RawDbWriter
    def upsert(self, rows, string_value=None):
        """The rows of a hand-off into the engine's state.  The text rows name STRING variable values (and
        list items) by the writer's value-dictionary ids; with `string_value` (the writer's id -> bytes)
        they are re-interned into this engine's dictionary (zb-db bytes carry the strings themselves)."""
        if string_value is not None:
            rows = [self._reintern(r, string_value) if r.startswith("VARIABLES|") else r for r in rows]
        self.o.import_rows(rows)

    def _reintern(self, row, string_value):
        head, _, f = row.rpartition("|")
        fields = dict(kv.split("=", 1) for kv in f.split(","))
        mine = lambda i: str(self.o.intern_string(string_value(int(i))))  # noqa: E731
        if fields["type"] == str(abi.DOC_STR):
            fields["value"] = mine(fields["value"])
        elif fields["type"] == str(abi.DOC_LIST) and fields["value"]:
            fields["value"] = ";".join(t + ":" + (mine(v) if t == str(abi.DOC_STR) else v)
                                       for t, v in (it.split(":", 1) for it in fields["value"].split(";")))
        return head + "|" + ",".join("%s=%s" % kv for kv in fields.items())

    def state(self):
        return self.o.state()

    def activatable_jobs(self, job_type):
        """JobState.forEachActivatableJobs of `job_type`: the JOB_ACTIVATABLE [[type, jobKey], tenant] keys."""
        return sorted(int(r.rsplit("|", 1)[1]) for r in self.o.state()
                      if r.startswith("JOB_ACTIVATABLE|") and r.split("|")[1] == job_type)

    def accepts(self, vt):
        return vt in self.ACCEPTS

    def replay(self, record):
        pass

    def _proc_index(self, v):
        pdk = v.get("processDefinitionKey", -1)
        best = -1
        for i, p in enumerate(self.tables):
            if pdk is not None and pdk > 0:
                if p.definition_key == pdk:
                    return i
            elif p.bpmn_process_id == v.get("bpmnProcessId") and (best < 0 or p.version > self.tables[best].version):
                best = i
        return best

    def process(self, record, out):
        vt, it, v = record.value_type, record.intent, record.value
        if vt == VT_JOB_BATCH:
            return self._activate(record, out)
        if vt == abi.VT_MESSAGE_BATCH:
            return self._expire(record, out)
        r = np.zeros(1, dtype=abi.RECORD_DTYPE)[0]
        r["record_type"], r["value_type"], r["intent"], r["key"] = abi.RT_COMMAND, vt, it, record.key
        r["process_idx"] = r["element_idx"] = -1
        r["scope_key"] = r["process_instance_key"] = r["aux"] = r["message_key"] = -1
        r["correlation_key"], r["message_name"], r["bpmn_process_id"] = abi.NO_STRING, 0xFFFF, 0xFFFF
        r["rejection_type"] = abi.REJ_NONE
        slot = 0xFFFFFF
        variables = tuple(v.get("variables", ())) if isinstance(v, dict) else ()
        if vt == abi.VT_PROCESS_INSTANCE_CREATION:
            r["process_idx"] = self._proc_index(v)
            slot = self.next_slot
            self.next_slot += 1
        elif vt == abi.VT_TIMER:
            r["aux"] = v["dueDate"]
        elif vt == abi.VT_JOB and it == abi.JOB_THROW_ERROR:  # zb_oracle.cpp throw_error's command fields
            r["partition"] = self.o.intern_string(v.get("errorCode", ""))
            r["correlation_key"] = self.o.intern_string(v["errorMessage"]) if v.get("errorMessage") else abi.NO_STRING
        elif vt == abi.VT_JOB and it == abi.JOB_FAIL:  # zb_oracle.cpp fail_job's command fields
            r["partition"] = v.get("retries", 0)
            r["message_key"] = v.get("retryBackoff", 0)
            r["correlation_key"] = self.o.intern_string(v["errorMessage"]) if v.get("errorMessage") else abi.NO_STRING
        elif vt == abi.VT_PROCESS_INSTANCE:
            p = self._proc_index(v)
            r["process_idx"] = p
            t = self.tables[p]  # by id and type: a multi-instance body and its inner activity share the id
            r["element_idx"] = next(e for e, (i, ty) in enumerate(zip(t.element_ids, t.element_types))
                                    if i == v["elementId"] and ty == v["bpmnElementType"])
            r["scope_key"], r["process_instance_key"] = v["flowScopeKey"], v["processInstanceKey"]
            slot = self.slot_of.setdefault(v["processInstanceKey"], 0xFFFFF0 - len(self.slot_of))
        elif vt == abi.VT_PROCESS_INSTANCE_BATCH:
            r["scope_key"], r["process_instance_key"] = v["batchElementInstanceKey"], v["processInstanceKey"]
            r["partition"] = v["index"]
            slot = self.slot_of.setdefault(v["processInstanceKey"], 0xFFFFF0 - len(self.slot_of))
        elif vt == abi.VT_MESSAGE:
            r["message_name"] = self.o.intern(v["name"])
            r["correlation_key"] = self.o.intern_string(v["correlationKey"])
            # (zb_oracle.cpp process_one: timeToLive in aux, the command's timestamp in scope_key, the
            # messageId's string id in process_instance_key)
            r["aux"] = v.get("timeToLive", 0)
            r["scope_key"] = record.timestamp
            r["process_instance_key"] = self.o.intern_string(v["messageId"]) if v.get("messageId") else -1
            slot = int(r["correlation_key"])
            variables = ()
        elif vt in MESSAGE_VALUE_TYPES:
            r["scope_key"], r["process_instance_key"] = v["elementInstanceKey"], v["processInstanceKey"]
            r["message_key"] = v["messageKey"]
            r["message_name"] = self.o.intern(v["messageName"])
            r["bpmn_process_id"] = self.o.intern(v["bpmnProcessId"]) if v["bpmnProcessId"] else 0xFFFF
            r["correlation_key"] = self.o.intern_string(v["correlationKey"]) if v["correlationKey"] else abi.NO_STRING
            r["interrupting"] = int(v["interrupting"])
            r["partition"] = v.get("subscriptionPartitionId", 0)
            variables = ()
            if vt == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION:
                slot = self.slot_of.setdefault(v["processInstanceKey"], 0xFFFFF0 - len(self.slot_of))
            else:
                slot = 0xFFFFFF  # (the correlation slot: only the oracle's key bookkeeping uses it)
        docs = doc_entries(variables, self.o.intern, self.o.intern_string, self.o.intern_list)
        base = len(self.doc_values)
        self.doc_values.extend(val for _, val in variables)
        self.o.clear_records()
        if self.clock:
            self.o.set_clock(self.clock.now)
        self.o.process_one(r, slot, docs, record.position or 0, len(out.entries))
        recs = self.o.records()
        pushes = []
        for k, x in enumerate(recs):
            rt, xvt, xit = int(x["record_type"]), int(x["value_type"]), int(x["intent"])
            if rt == abi.RT_REJECTION and k == 0 and xvt == vt and xit == it:
                value = dict(v)  # TypedRejectionWriter: the command's value
            else:
                value = self.values.value(x, variables, lambda aux: self.doc_values[aux], record.timestamp)
            if xvt == abi.VT_PROCESS_INSTANCE_CREATION:
                self.slot_of[int(x["scope_key"])] = slot
            out.append_record(int(x["key"]), rt, xvt, xit, int(x["rejection_type"]),
                              self.o.reason(k) if rt == abi.RT_REJECTION else "", value)
            self.pending.track(rt, xvt, xit, value)
            if rt == abi.RT_EVENT and xvt == VT_JOB_BATCH:
                pushes.append((int(x["aux"]), value))
            if rt == abi.RT_EVENT and xvt == abi.VT_TIMER and xit == abi.TIMER_CREATED and self.due_date_checker:
                out.append_post_commit_task(lambda d=value["dueDate"]: self.due_date_checker.schedule_timer(d) or True)
        if pushes:
            strings = self.o.strings()
            push_side_effects(out, pushes, self.stream_sinks, self.o.job_variables, self.values, self.o.name,
                              lambda i: strings[i].decode())
        notified = self.o.take_notified()
        if notified and self.job_streamer is not None:
            out.append_post_commit_task(lambda types=notified: [self.job_streamer.notify_work_available(t)
                                                                for t in types] and True)
        sends = self.o.outbox()  # SubscriptionCommandSender's side effects of this command
        if len(sends):
            strings = self.o.strings()
            cmds = [(int(x["target_partition"]),) + XPART_COMMAND[int(x["kind"])] +
                    (xpart_value(x, self.o.name, lambda i: strings[i].decode()),) for x in sends]

            def task():
                for target, svt, sit, value in cmds:
                    self.command_sender.send_command(target, svt, sit, value)
                return True
            out.append_post_commit_task(task)
        return out.build()

    def _expire(self, record, out):
        """MESSAGE_BATCH:EXPIRE (MessageBatchExpireProcessor.java:33-52): MESSAGE:EXPIRED per message key, in
        the batch's order (the oracle's MESSAGE:EXPIRE of one key each)."""
        for mk in record.value["messageKeys"]:
            r = np.zeros(1, dtype=abi.RECORD_DTYPE)[0]
            r["record_type"], r["value_type"], r["intent"], r["key"] = abi.RT_COMMAND, abi.VT_MESSAGE, abi.MSG_EXPIRE, mk
            r["process_idx"] = r["element_idx"] = -1
            r["scope_key"] = r["process_instance_key"] = r["aux"] = r["message_key"] = -1
            r["correlation_key"], r["message_name"], r["bpmn_process_id"] = abi.NO_STRING, 0xFFFF, 0xFFFF
            r["rejection_type"] = abi.REJ_NONE
            self.o.clear_records()
            self.o.process_one(r, 0xFFFFFF, abi.make_docs(0), record.position or 0, len(out.entries))
            for x in self.o.records():
                out.append_record(int(x["key"]), int(x["record_type"]), int(x["value_type"]), int(x["intent"]),
                                  abi.REJ_NONE, "", self.values.value(x))
        return out.build()

    def _activate(self, record, out):
        v = record.value
        key, jobs, reason = self.o.activate_jobs(v["type"], v["worker"], v["timeout"], v["maxJobsToActivate"],
                                                 v.get("timestamp", 0))
        if key < 0:
            out.append_record(record.key, abi.RT_REJECTION, VT_JOB_BATCH, JOB_BATCH_ACTIVATE,
                              abi.REJ_INVALID_ARGUMENT, "reason %d" % reason, dict(v))
            return out.build()
        strings = self.o.strings()
        out.append_record(key, abi.RT_EVENT, VT_JOB_BATCH, JOB_BATCH_ACTIVATED, abi.REJ_NONE, "",
                          self.values.job_batch(v, key, jobs, self.o.name, lambda i: strings[i].decode()))
        return out.build()


class Client:
    """EngineRule's test clients (util/client/*Client.java): commands written to the log."""

    def __init__(self, *logs):
        self.logs = logs

    def write(self, *recs):
        for log in self.logs:
            log.append([Rec(r.record_type, r.value_type, r.intent, r.key, r.value, timestamp=r.timestamp) for r in recs])

    @staticmethod
    def create(bpmn_process_id, variables=(), key=-1):
        return Rec(abi.RT_COMMAND, abi.VT_PROCESS_INSTANCE_CREATION, 0, -1,
                   {"bpmnProcessId": bpmn_process_id, "processDefinitionKey": key, "version": -1,
                    "variables": tuple(variables), "tenantId": "<default>"})

    @staticmethod
    def complete_job(key, variables=()):
        return Rec(abi.RT_COMMAND, abi.VT_JOB, abi.JOB_COMPLETE, key, {"variables": tuple(variables),
                                                                       "tenantId": "<default>"})

    @staticmethod
    def fail_job(key, retries, error_message="", variables=()):
        """JobClient.fail (util/client/JobClient.java): JOB:FAIL with retries and an errorMessage."""
        return Rec(abi.RT_COMMAND, abi.VT_JOB, abi.JOB_FAIL, key,
                   {"retries": retries, "errorMessage": error_message, "retryBackoff": 0, "variables": tuple(variables),
                    "tenantId": "<default>"})

    @staticmethod
    def throw_error(key, error_code, error_message="", variables=()):
        """JobClient.withErrorCode(..).throwError (util/client/JobClient.java): JOB:THROW_ERROR."""
        return Rec(abi.RT_COMMAND, abi.VT_JOB, abi.JOB_THROW_ERROR, key,
                   {"errorCode": error_code, "errorMessage": error_message, "variables": tuple(variables),
                    "tenantId": "<default>"})

    @staticmethod
    def publish_message(name, correlation_key, timestamp=0, time_to_live=0, message_id=""):
        """MessageClient.publish (MessageRecord.java:37-43): time-to-live 0 unless given, an optional message
        id; `timestamp` = the command's record timestamp (the broker's clock when it was written)."""
        return Rec(abi.RT_COMMAND, abi.VT_MESSAGE, abi.MSG_PUBLISH, -1,
                   {"name": name, "correlationKey": correlation_key, "timeToLive": time_to_live, "variables": (),
                    "messageId": message_id, "deadline": -1, "tenantId": "<default>"}, timestamp=timestamp)

    @staticmethod
    def activate_jobs(job_type, worker="w", timeout=300000, max_jobs=10, timestamp=0):
        return Rec(abi.RT_COMMAND, VT_JOB_BATCH, JOB_BATCH_ACTIVATE, -1,
                   {"type": job_type, "worker": worker, "timeout": timeout, "maxJobsToActivate": max_jobs,
                    "timestamp": timestamp})


def open_jobs(log):
    """Job keys created and not completed / canceled so far (RecordingExporter over the log)."""
    alive = {}
    for r in log.entries:
        if r.value_type == abi.VT_JOB and r.record_type == abi.RT_EVENT:
            if r.intent == abi.JOB_CREATED:
                alive[r.key] = r
            elif r.intent in (abi.JOB_COMPLETED, abi.JOB_CANCELED):
                alive.pop(r.key, None)
    return alive


class InterPartitionCommandSender:
    """TestInterPartitionCommandSender (engine/src/test/.../util/TestInterPartitionCommandSender.java:
    23-59): a sent command is written to the receiving partition's log as a COMMAND with key -1
    (LogAppendEntry.of(metadata, command))."""

    def __init__(self, logs):
        self.logs = logs  # partition id -> Log

    def send_command(self, receiver_partition, value_type, intent, value, key=-1):
        self.logs[receiver_partition].append([Rec(abi.RT_COMMAND, value_type, intent, key, value)])


def canon_strings(rows, string_value):
    """State rows with STRING variable values (and string list items) spelled out instead of value-
    dictionary ids: each engine and each device interns strings in the order it meets them, so ids differ
    between a cluster and its reference while the strings are the same.  `string_value`: id -> str."""
    out = []
    for r in rows:
        if r.startswith("VARIABLES|"):
            head, _, f = r.rpartition("|")
            fields = dict(kv.split("=", 1) for kv in f.split(","))
            sv = lambda i: "'" + string_value(int(i)) + "'"  # noqa: E731
            if fields["type"] == str(abi.DOC_STR):
                fields["value"] = sv(fields["value"])
            elif fields["type"] == str(abi.DOC_LIST) and fields["value"]:
                fields["value"] = ";".join(t + ":" + (sv(v) if t == str(abi.DOC_STR) else v)
                                           for t, v in (it.split(":", 1) for it in fields["value"].split(";")))
            r = head + "|" + ",".join("%s=%s" % kv for kv in fields.items())
        out.append(r)
    return out


def run_cluster(processors):
    """Every partition's processing loop, round robin, until no partition has an unprocessed command
    (EngineRule.multiplePartition: one stream processor per partition)."""
    while True:
        busy = False
        for sp in processors:
            if sp.read < len(sp.log.entries):
                sp.run()
                busy = True
        if not busy:
            return
