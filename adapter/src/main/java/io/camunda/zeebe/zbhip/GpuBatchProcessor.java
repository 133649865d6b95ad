/*
 * The host adapter a maintainer adds to the broker: a stream-platform RecordProcessor placed before
 * the engine (StreamProcessorTransitionStep.java:135-147: List.of(gpu, engine, checkpointProcessor))
 * that answers the hot-path commands from libzbhip.so and hands everything else -- and every
 * command the device falls back on -- to the unchanged engine.
 *
 * Inside ProcessingStateMachine.batchProcessing / collectBatchProcessingStepResult
 * (stream-platform/.../stream/impl/ProcessingStateMachine.java:328-417) it behaves as the engine:
 *  - a device batch is appended whole when the platform processes its initial command; the
 *    follow-up commands the platform then feeds back (UnwrittenRecord) were already processed on the
 *    device and return the builder unchanged (out.build(), never EmptyProcessingResult: the platform
 *    skips the builder's entries by their count);
 *  - follow-ups written unprocessed past maxCommandsInBatch are device continuations
 *    (ZBHIP_OPEN_DEFER_CONTINUATIONS): they run when the platform reads them back, at their own log
 *    position (ZBHIP_CMD_CONTINUE), after whatever the log holds before them;
 *  - one key generator: after each device command DbKeyGenerator.setKeyIfHigher(device keys),
 *    before each window zbhip_set_key_if_higher(DbKeyGenerator's key);
 *  - the fallback hand-off declares the engine's keys after its batch (a post-commit task);
 *  - JOB_BATCH:ACTIVATE of job types only device instances hold goes to zbhip_activate_jobs;
 *  - after recovery the instances of device processes move from RocksDB into HBM (onRecovered);
 *  - config 5 (correlationSlots > 0): MESSAGE:PUBLISH, MESSAGE_SUBSCRIPTION:CREATE/CORRELATE and
 *    PROCESS_MESSAGE_SUBSCRIPTION:CREATE/CORRELATE run on the device (Messages), and the commands a
 *    device batch sends to other partitions go to InterPartitionCommandSender in a post-commit task of
 *    that batch (SubscriptionCommandSender.handleFollowUpCommandBasedOnPartition, :320-338);
 *  - the engine's scheduled tasks read device-held state through DeviceScheduledState (timerState,
 *    jobState, pending*State below, passed to the checkers EngineProcessors builds), device TIMER:CREATED
 *    records schedule the DueDateTimerChecker as the engine's do (a side effect), and JOB:TIME_OUT of a
 *    device job runs through zbhip_time_out_job (JobTimeOutProcessor.java:46-73), JOB:FAIL through
 *    zbhip_fail_job (JobFailProcessor.java:79-162);
 *  - job push (BpmnJobActivationBehavior.publishWork): the broker's JobStreamer mirrored per device job
 *    type into zbhip_set_job_stream before each window (JobStreams), the stream's push a post-commit task.
 * The Python mirror zeebe_amd/adapter.py is this class line for line in behaviour; tests/test_gpu_psm.py
 * runs it inside a restatement of ProcessingStateMachine against the engine alone.
 *
 * Not compiled in this image (no JDK); written against the reference's interfaces:
 *   RecordProcessor                stream-platform/.../stream/api/RecordProcessor.java:17-108
 *   ProcessingResultBuilder        stream-platform/.../stream/api/ProcessingResultBuilder.java:22-80
 *   RecordProcessorContext         stream-platform/.../stream/api/RecordProcessorContext.java:18-32
 *   KeyGeneratorControls           stream-platform/.../stream/api/state/KeyGeneratorControls.java:11-19
 *   DbKeyGenerator                 stream-platform/.../stream/impl/state/DbKeyGenerator.java:17-61
 *   UnwrittenRecord                stream-platform/.../stream/impl/records/UnwrittenRecord.java:19-40
 *   StreamProcessorLifecycleAware  stream-platform/.../stream/api/StreamProcessorLifecycleAware.java:13
 *   LogStreamReader / LoggedEvent  logstreams/.../log/LogStreamReader.java, LoggedEvent.java
 * See INTEGRATION.md for the contract of every zbhip call used here.
 */
package io.camunda.zeebe.zbhip;

import io.camunda.zeebe.engine.Engine;
import io.camunda.zeebe.logstreams.log.LogStreamReader;
import io.camunda.zeebe.logstreams.log.LoggedEvent;
import io.camunda.zeebe.protocol.impl.record.RecordMetadata;
import io.camunda.zeebe.protocol.impl.record.value.job.JobBatchRecord;
import io.camunda.zeebe.protocol.impl.record.value.incident.IncidentRecord;
import io.camunda.zeebe.protocol.impl.record.value.job.JobRecord;
import io.camunda.zeebe.protocol.impl.record.value.processinstance.ProcessInstanceCreationRecord;
import io.camunda.zeebe.protocol.impl.record.value.processinstance.ProcessInstanceBatchRecord;
import io.camunda.zeebe.protocol.impl.record.value.processinstance.ProcessInstanceRecord;
import io.camunda.zeebe.protocol.record.intent.ProcessInstanceBatchIntent;
import io.camunda.zeebe.protocol.impl.record.value.timer.TimerRecord;
import io.camunda.zeebe.protocol.record.RecordType;
import io.camunda.zeebe.protocol.record.ValueType;
import io.camunda.zeebe.protocol.record.intent.JobBatchIntent;
import io.camunda.zeebe.protocol.record.intent.JobIntent;
import io.camunda.zeebe.protocol.record.intent.ProcessInstanceCreationIntent;
import io.camunda.zeebe.protocol.record.intent.ProcessInstanceIntent;
import io.camunda.zeebe.protocol.record.intent.TimerIntent;
import io.camunda.zeebe.scheduler.clock.ActorClock;
import io.camunda.zeebe.stream.api.InterPartitionCommandSender;
import io.camunda.zeebe.stream.api.ProcessingResult;
import io.camunda.zeebe.stream.api.ProcessingResultBuilder;
import io.camunda.zeebe.stream.api.ReadonlyStreamProcessorContext;
import io.camunda.zeebe.stream.api.RecordProcessor;
import io.camunda.zeebe.stream.api.RecordProcessorContext;
import io.camunda.zeebe.stream.api.StreamProcessorLifecycleAware;
import io.camunda.zeebe.stream.api.records.TypedRecord;
import io.camunda.zeebe.stream.impl.records.UnwrittenRecord;
import io.camunda.zeebe.stream.impl.state.DbKeyGenerator;
import io.camunda.zeebe.protocol.record.value.TenantOwned;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.nio.charset.StandardCharsets;
import org.agrona.concurrent.UnsafeBuffer;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.BitSet;
import java.util.HashMap;
import java.util.HashSet;
import java.util.Iterator;
import java.util.List;
import java.util.Map;
import java.util.Set;

public final class GpuBatchProcessor implements RecordProcessor, StreamProcessorLifecycleAware {

  /** Deployed processes the adapter knows: bpmnProcessId (latest version) / definition key. */
  public interface Deployments {
    /** BPMN XML of every deployed process, in deployment order (DbProcessState). */
    List<DeployedResource> all();

    record DeployedResource(long definitionKey, String bpmnProcessId, int version, byte[] xml) {}
  }

  /** Raw column-family access of a hand-off and of recovery; the broker binds it to its ZeebeDb transaction. */
  public interface RawDb {
    void upsert(int columnFamily, byte[] key, byte[] value);

    void delete(int columnFamily, byte[] key);

    /** Every entry of the hot-path column families (ZbColumnFamilies ordinals), in key order. */
    void forEach(Entry consumer);

    interface Entry {
      void entry(int columnFamily, byte[] key, byte[] value);
    }
  }

  /**
   * A follow-up a device batch wrote unprocessed (a PROCESS_INSTANCE command or a multi-instance
   * body's PROCESS_INSTANCE_BATCH:ACTIVATE): matched against the log in the order written.
   */
  record Continuation(long id, int slot, long key, int valueType, int intent, String elementId, long flowScopeKey,
      long batchElementInstanceKey, long piKey) {
    boolean matches(final TypedRecord record) {
      if (record.getKey() != key || record.getValueType().value() != valueType || record.getIntent().value() != intent) {
        return false;
      }
      if (record.getValue() instanceof final ProcessInstanceRecord v) {
        return v.getElementId().equals(elementId) && v.getFlowScopeKey() == flowScopeKey
            && v.getProcessInstanceKey() == piKey;
      }
      return record.getValue() instanceof final ProcessInstanceBatchRecord v
          && v.getBatchElementInstanceKey() == batchElementInstanceKey && v.getProcessInstanceKey() == piKey;
    }
  }

  private static final int WINDOW = 1 << 16; // commands per submitted window (zbhip_config.max_commands)
  private static final int INSTANCES = 1 << 22; // instance slots in HBM (288 GB holds ~2.5e9)

  private final Engine engine;
  private final LogStreamReader reader;
  private final Deployments deployments;
  private final RawDb zeebeDb;
  private final int partitionCount;
  private final int device;
  private final int correlationSlots; // config 5: correlation slots in HBM (0: messages stay with the engine)
  private final Set<String> messageNames = new HashSet<>();
  // names of every deployed process's message start events: their publishes (and keys) are the engine's
  private final Set<String> startMessageNames = new HashSet<>();
  private int partitionId;
  private InterPartitionCommandSender sender;
  private Messages messages;

  private final Arena arena = Arena.ofShared();
  private MemorySegment handle;
  private DbKeyGenerator keyGenerator;
  private final Map<Long, ZbHip.Deployed> byKey = new HashMap<>();
  private final Map<String, ZbHip.Deployed> latestById = new HashMap<>();
  private final List<ZbHip.Deployed> byIndex = new ArrayList<>();
  private final Set<String> engineJobTypes = new HashSet<>();
  private final BitSet usedSlots = new BitSet(INSTANCES);
  private final Set<Integer> ended = new HashSet<>(); // ended instances whose continuations still wait
  private int nextFreeSlot;

  // the window read ahead from the log
  private final Window window = new Window();
  private final Set<Integer> handedOff = new HashSet<>();
  private final ArrayDeque<Continuation> continuations = new ArrayDeque<>();
  private int followUps; // follow-ups of the current device batch the platform feeds back
  private boolean windowDone = true; // every command of the current window was emitted
  private io.camunda.zeebe.engine.processing.timer.DueDateTimerChecker dueDateTimerChecker;
  private JobStreams jobStreams = new JobStreams(null);
  private io.camunda.zeebe.engine.state.immutable.JobState engineJobState; // the engine's (jobState(...))
  // the engine's transient pending-subscription states: entries of subscriptions that move to the engine go
  // there at once (its appliers clear them when its batches close the subscriptions)
  io.camunda.zeebe.engine.state.message.TransientPendingSubscriptionState engineProcessTransient;
  io.camunda.zeebe.engine.state.message.TransientPendingSubscriptionState engineMessageTransient;

  public GpuBatchProcessor(
      final Engine engine,
      final LogStreamReader reader,
      final Deployments deployments,
      final RawDb zeebeDb,
      final int partitionCount,
      final int device) {
    this(engine, reader, deployments, zeebeDb, partitionCount, device, 0);
  }

  public GpuBatchProcessor(
      final Engine engine,
      final LogStreamReader reader,
      final Deployments deployments,
      final RawDb zeebeDb,
      final int partitionCount,
      final int device,
      final int correlationSlots) {
    this.engine = engine;
    this.reader = reader;
    this.deployments = deployments;
    this.zeebeDb = zeebeDb;
    this.partitionCount = partitionCount;
    this.device = device;
    this.correlationSlots = correlationSlots;
  }

  @Override
  public void init(final RecordProcessorContext ctx) {
    engine.init(ctx);
    // the platform's key generator is the DbKeyGenerator (StreamProcessor.java:368)
    keyGenerator = (DbKeyGenerator) ctx.getKeyGenerator();
    partitionId = ctx.getPartitionId();
    sender = ctx.getPartitionCommandSender();
    final long partitionBits = (long) partitionId << 51;
    handle =
        ZbHip.open(
            arena, ctx.getPartitionId(), partitionCount, device, /* maxCommandsInBatch */ 100, INSTANCES, WINDOW,
            keyGenerator.getCurrentKey() - partitionBits, correlationSlots, ZbHip.OPEN_DEFER_CONTINUATIONS);
    for (final var d : deployments.all()) {
      deploy(d);
    }
    messages = new Messages(partitionId, correlationSlots, messageNames, startMessageNames);
    window.init(arena);
    ctx.addLifecycleListeners(List.of(this));
  }

  private void deploy(final Deployments.DeployedResource d) {
    final ZbHip.Deployed p = ZbHip.deploy(handle, d.xml(), d.definitionKey(), d.version());
    startMessageNames.addAll(JobTypes.messageStartNames(d.xml()));
    if (p == null) {
      // outside the device subset: its instances (and their job types) stay on the CPU engine
      engineJobTypes.addAll(JobTypes.of(d.xml()));
      return;
    }
    messageNames.addAll(JobTypes.messageNames(d.xml()));
    byKey.put(d.definitionKey(), p);
    byIndex.add(p);
    final var prev = latestById.get(d.bpmnProcessId());
    if (prev == null || prev.version() < d.version()) {
      latestById.put(d.bpmnProcessId(), p);
    }
  }

  @Override
  public boolean accepts(final ValueType valueType) {
    return valueType == ValueType.PROCESS_INSTANCE_CREATION || valueType == ValueType.JOB
        || valueType == ValueType.TIMER || valueType == ValueType.JOB_BATCH
        || (correlationSlots > 0 && Messages.isMessageCommand(valueType)) || engine.accepts(valueType);
  }

  @Override
  public void replay(final TypedRecord record) {
    // events only; the appliers write RocksDB.  Instances restored this way move into HBM in onRecovered
    engine.replay(record);
  }

  /**
   * After replay the engine's state holds every instance: those of device processes move into HBM
   * (zbhip_import_state_db) and leave RocksDB, except instances a command still waiting in the log
   * addresses by its own record (a follow-up written unprocessed before the restart).
   */
  @Override
  public void onRecovered(final ReadonlyStreamProcessorContext context) {
    final RecoveredState state = RecoveredState.collect(handle, zeebeDb, reader);
    if (state.size() > 0) {
      final int first = nextFreeSlot;
      final int n = ZbHip.importStateDb(handle, state.entries(arena), state.bytes(), first);
      usedSlots.set(first, first + n);
      nextFreeSlot = first + n;
      state.forEachMoved(zeebeDb::delete);
    }
    ZbHip.setKeyIfHigher(handle, keyGenerator.getCurrentKey());
  }

  @Override
  public ProcessingResult process(final TypedRecord record, final ProcessingResultBuilder out) {
    if (record instanceof UnwrittenRecord) {
      // a follow-up command the platform feeds back within the current batch
      if (followUps > 0) {
        followUps--;
        return out.build(); // already processed on the device: its records are in the builder
      }
      return engine.process(record, out);
    }
    followUps = 0;
    if (record.getValueType() == ValueType.JOB_BATCH && record.getIntent() == JobBatchIntent.ACTIVATE) {
      final JobBatchRecord batch = (JobBatchRecord) record.getValue();
      if (!engineJobTypes.contains(batch.getType())) {
        return activateJobs(record, batch, out);
      }
      return deviceProcessJobTypes().contains(batch.getType()) ? activateJobsMerged(record, batch, out)
          : engine.process(record, out);
    }
    if (record.getValueType() == ValueType.JOB && record.getIntent() == JobIntent.TIME_OUT
        && ZbHip.resolveKey(handle, record.getKey()) >= 0) {
      return timeOutJob(record, out);
    }
    if (record.getValueType() == ValueType.JOB && record.getIntent() == JobIntent.FAIL
        && ZbHip.resolveKey(handle, record.getKey()) >= 0) {
      return failJob(record, out);
    }
    int i = window.covers(record.getPosition()) ? window.indexOf(record.getPosition()) : -1;
    if (i < 0) {
      if (!isHotPath(record, continuations.iterator())) {
        if (messages.enabled() && record.getValueType() == ValueType.MESSAGE
            && record.getIntent() == io.camunda.zeebe.protocol.record.intent.MessageIntent.PUBLISH) {
          // a publish the engine processes: its correlation key's message state goes there first
          messages.toEngine(((io.camunda.zeebe.protocol.impl.record.value.message.MessageRecord) record.getValue())
              .getCorrelationKey(), this, zeebeDb::upsert);
        }
        // a command the device does not run for an instance it holds (INCIDENT:RESOLVE of a gateway's
        // incident, PROCESS_INSTANCE:CANCEL, ...): the instance moves to RocksDB first
        final int held = heldInstance(record);
        if (held >= 0) {
          handOff(held);
          keyGenerator.setKeyIfHigher(ZbHip.currentKey(handle));
        }
        return engine.process(record, out);
      }
      fillWindow(record);
      i = window.indexOf(record.getPosition());
      if (i < 0) {
        return engine.process(record, out); // the read-ahead stopped before it
      }
    }
    windowDone = i == window.size() - 1;
    if (ZbHip.commandStatus(handle, i) != 0) {
      return fallBack(i, record, out);
    }
    followUps = window.emit(i, record, out, this);
    if (messages.enabled()) {
      messages.send(handle, i, out, sender, this); // the batch's cross-partition commands, post-commit
    }
    // DbKeyGenerator after this command: the device's keys so far (the engine's next command, a
    // fallback in this window or whatever follows the window, continues after them)
    keyGenerator.setKeyIfHigher(ZbHip.keyBefore(handle, i + 1));
    return out.build();
  }

  @Override
  public ProcessingResult onProcessingError(
      final Throwable error, final TypedRecord record, final ProcessingResultBuilder out) {
    return engine.onProcessingError(error, record, out);
  }

  // ---- the window ------------------------------------------------------------------------------

  private ZbHip.Deployed createTarget(final ProcessInstanceCreationRecord create) {
    return create.getProcessDefinitionKey() > 0
        ? byKey.get(create.getProcessDefinitionKey())
        : latestById.get(create.getBpmnProcessId());
  }

  /**
   * Would the device take this log command?  {@code next}: the continuations not yet claimed by the
   * read-ahead (a log PI command is one when it is the next one written).
   */
  private boolean isHotPath(final TypedRecord record, final Iterator<Continuation> next) {
    if (record.getRecordType() != RecordType.COMMAND) {
      return false;
    }
    final ValueType vt = record.getValueType();
    if (vt == ValueType.PROCESS_INSTANCE_CREATION) {
      return record.getIntent() == ProcessInstanceCreationIntent.CREATE
          && createTarget((ProcessInstanceCreationRecord) record.getValue()) != null;
    }
    if ((vt == ValueType.JOB && record.getIntent() == JobIntent.COMPLETE)
        || (vt == ValueType.TIMER && record.getIntent() == TimerIntent.TRIGGER)) {
      // JOB:COMPLETE of a device job; TIMER:TRIGGER (DueDateTimerChecker's command) of a device timer
      return ZbHip.resolveKey(handle, record.getKey()) >= 0;
    }
    if ((vt == ValueType.PROCESS_INSTANCE
            && (record.getIntent() == ProcessInstanceIntent.ACTIVATE_ELEMENT
                || record.getIntent() == ProcessInstanceIntent.COMPLETE_ELEMENT
                || record.getIntent() == ProcessInstanceIntent.TERMINATE_ELEMENT))
        || (vt == ValueType.PROCESS_INSTANCE_BATCH && record.getIntent() == ProcessInstanceBatchIntent.ACTIVATE)) {
      return next.hasNext() && next.next().matches(record);
    }
    if (messages.enabled() && Messages.isMessageCommand(vt)) {
      try (Arena a = Arena.ofConfined()) {
        return messages.of(record, this, a) != null;
      }
    }
    return false;
  }

  /**
   * Reads consecutive hot-path commands from the log starting at {@code first}, converts them to
   * zbhip_command rows (+ variable document entries), submits and runs them once, and drains the
   * window's records (keys relabelled to DbKeyGenerator's, ordered by source command).
   */
  private void fillWindow(final TypedRecord first) {
    freeEndedSlots();
    window.reset(first.getPosition());
    reader.seek(first.getPosition());
    final RecordMetadata meta = new RecordMetadata();
    final Iterator<Continuation> next = continuations.iterator();
    int claimed = 0;
    jobStreams.sync(handle, deviceJobTypes()); // the streams open now (pushFenced reads them)
    while (reader.hasNext() && window.size() < WINDOW) {
      final LoggedEvent event = reader.next();
      event.readMetadata(meta);
      if (meta.getRecordType() != RecordType.COMMAND || event.shouldSkipProcessing()) {
        continue; // follow-up events and processed follow-up commands of earlier batches
      }
      final TypedRecord rec = Window.typed(event, meta, partitionId);
      final Iterator<Continuation> peek = continuations.stream().skip(claimed).iterator();
      if (!isHotPath(rec, peek)) {
        break; // the engine's: the window ends before it (log order is kept)
      }
      final ValueType vt = meta.getValueType();
      if (pushFenced(rec, vt, claimed)) {
        break; // the next window takes it
      }
      if (vt == ValueType.PROCESS_INSTANCE_CREATION) {
        final ProcessInstanceCreationRecord create = (ProcessInstanceCreationRecord) rec.getValue();
        final int slot = takeSlot();
        if (slot < 0 || !window.addCreate(event.getPosition(), rec, createTarget(create).index(), slot, this)) {
          if (slot >= 0) {
            usedSlots.clear(slot); // the document is outside the subset: the slot stays free
          }
          break; // the engine takes this CREATE
        }
      } else if (vt == ValueType.JOB) {
        final long ref = ZbHip.resolveKey(handle, event.getKey());
        if (!window.addJobComplete(event.getPosition(), rec, ref, this)) {
          break;
        }
      } else if (vt == ValueType.TIMER) {
        final long ref = ZbHip.resolveKey(handle, event.getKey());
        window.addTimerTrigger(event.getPosition(), rec, ref, ((TimerRecord) rec.getValue()).getDueDate());
      } else if (Messages.isMessageCommand(vt)) {
        window.addMessageCommand(event.getPosition(), rec, messages.of(rec, this, window.arena()));
      } else {
        final Continuation c = next.next();
        claimed++;
        window.addContinuation(event.getPosition(), rec, c.slot(), c.id());
      }
      if (messages.enabled() && messages.ownsKeys() && !Messages.isSlotCommand(vt, rec)) {
        // a correlation key of this partition is the engine's: a process-instance command may subscribe to
        // it locally and fall back with engine keys, which a message window takes only after its last device
        // key (zbhip_set_external_keys) -- such a command ends its window
        break;
      }
    }
    for (int k = 0; k < claimed; k++) {
      continuations.removeFirst();
    }
    // keys the engine generated since the last window come first (setKeyIfHigher)
    ZbHip.setKeyIfHigher(handle, keyGenerator.getCurrentKey());
    // the window's clock: TIMER:CREATED dueDates (CatchEventBehavior.java:310, ActorClock), pushed jobs'
    // deadlines (the job streams were synced before the read-ahead: publishWork asks JobStreamer per job)
    ZbHip.setClock(handle, ActorClock.currentTimeMillis());
    window.submitRun(handle);
    windowDone = false;
  }

  /**
   * A job stream's push gathers the job's variables when the push record is appended (JobStreams.push:
   * zbhip_job_variables), after the whole window ran; the reference gathers them in publishWork, at
   * JOB:CREATED (BpmnJobActivationBehavior.java:83).  While a stream pushes, a window holds at most one
   * command per process instance, so no later command of the window changes what a push reads or ends
   * its job (adapter.py _push_fenced).
   */
  private boolean pushFenced(final TypedRecord rec, final ValueType vt, final int claimed) {
    if (!jobStreams.pushing()) {
      return false;
    }
    final int instance;
    if (vt == ValueType.JOB || vt == ValueType.TIMER) {
      instance = (int) (ZbHip.resolveKey(handle, rec.getKey()) >>> 16);
    } else if (vt == ValueType.PROCESS_INSTANCE || vt == ValueType.PROCESS_INSTANCE_BATCH) {
      instance = continuations.stream().skip(claimed).findFirst().orElseThrow().slot();
    } else if (vt == ValueType.PROCESS_MESSAGE_SUBSCRIPTION) {
      try (Arena a = Arena.ofConfined()) {
        instance = messages.of(rec, this, a).instance();
      }
    } else {
      return false;
    }
    return window.addresses(instance);
  }

  /** A process instance completed (Window.emit): its slot is free once its continuations ran. */
  void instanceEnded(final int slot) {
    ended.add(slot);
  }

  private void freeEndedSlots() {
    for (final Iterator<Integer> it = ended.iterator(); it.hasNext(); ) {
      final int slot = it.next();
      if (ZbHip.pendingContinuations(handle, slot) == 0 && (messages == null || !messages.closing(slot))) {
        usedSlots.clear(slot);
        it.remove();
      }
    }
  }

  /** A continuation the window's command i wrote unprocessed (Window.emit, in log order). */
  void expectContinuation(final Continuation c) {
    continuations.addLast(c);
  }

  int internName(final String name) {
    return ZbHip.intern(handle, name);
  }

  long internString(final byte[] value) {
    return ZbHip.internString(handle, value);
  }

  /** zbhip_resolve_key: (slot << 16 | key ordinal) of a device key, or -1. */
  long resolve(final long key) {
    return key < 0 ? -1 : ZbHip.resolveKey(handle, key);
  }

  Messages messages() {
    return messages;
  }

  private int takeSlot() {
    int s = usedSlots.nextClearBit(nextFreeSlot);
    if (s >= INSTANCES) {
      s = usedSlots.nextClearBit(0);
    }
    while (s < INSTANCES && window.addresses(s)) {
      s = usedSlots.nextClearBit(s + 1);
    }
    if (s >= INSTANCES) {
      return -1;
    }
    usedSlots.set(s);
    nextFreeSlot = s + 1;
    return s;
  }

  ZbHip.Deployed process(final int index) {
    return byIndex.get(index);
  }

  /** A value-dictionary string (string variables). */
  byte[] stringValue(final long id) {
    return ZbHip.stringValue(handle, id);
  }

  /** The partition's name dictionary (variable names of VARIABLE records). */
  String name(final int id) {
    return ZbHip.name(handle, id);
  }

  String incidentMessage(final MemorySegment rec) {
    return ZbHip.incidentMessage(handle, rec);
  }

  String rejectionReason(final MemorySegment rec) {
    return ZbHip.rejectionReason(handle, rec);
  }

  // ---- fallback hand-off (INTEGRATION.md §8; Engine.java:134, ProcessingStateMachine.java:276-310) ----

  /** The device instance slot a non-hot-path command addresses by its key or its value's process instance, or -1. */
  private int heldInstance(final TypedRecord record) {
    long ref = record.getKey() >= 0 ? ZbHip.resolveKey(handle, record.getKey()) : -1;
    if (ref < 0) {
      final long pik = record.getValue() instanceof final ProcessInstanceRecord v ? v.getProcessInstanceKey()
          : record.getValue() instanceof final IncidentRecord v ? v.getProcessInstanceKey() : -1;
      ref = pik >= 0 ? ZbHip.resolveKey(handle, pik) : -1;
    }
    return ref < 0 ? -1 : (int) (ref >>> 16);
  }

  /** Hands the device instance of process instance key {@code pik} to the engine (if the device holds it). */
  void handOffInstanceOf(final long pik) {
    final long ref = ZbHip.resolveKey(handle, pik);
    if (ref >= 0) {
      handOff((int) (ref >>> 16));
      keyGenerator.setKeyIfHigher(ZbHip.currentKey(handle));
    }
  }

  private void handOff(final int instance) {
    if (handedOff.add(instance)) {
      // the instance's zb-db entries into RocksDB (the platform's transaction), then off the device
      // with its waiting continuations (the engine reads them back from the log)
      ZbHip.handOff(handle, instance, (cf, key, value) -> {
        if (cf == JobTypes.JOBS_COLUMN_FAMILY) {
          engineJobTypes.add(JobTypes.typeOfJobsValue(value));
        }
        zeebeDb.upsert(cf, key, value);
      });
      continuations.removeIf(c -> c.slot() == instance);
      usedSlots.clear(instance);
      ended.remove(instance);
      if (messages != null && messages.enabled()) {
        messages.handedOff(instance, engineProcessTransient);
      }
    }
  }

  private ProcessingResult fallBack(final int i, final TypedRecord record, final ProcessingResultBuilder out) {
    final int instance = window.instanceOf(i);
    if (Messages.isMessageCommand(record.getValueType()) && record.getValueType() != ValueType.PROCESS_MESSAGE_SUBSCRIPTION) {
      // a message-partition command the device declined: its correlation key's state moves to the engine
      messages.toEngine(new String(stringValue(instance), StandardCharsets.UTF_8), this, zeebeDb::upsert);
    } else {
      handOff(instance);
    }
    final long before = ZbHip.keyBefore(handle, i);
    keyGenerator.setKeyIfHigher(before);
    // the keys the engine's batch generates (follow-ups included) are declared after it
    out.appendPostCommitTask(() -> {
      ZbHip.setExternalKeys(handle, i, (int) (keyGenerator.getCurrentKey() - before));
      return true;
    });
    return engine.process(record, out);
  }

  // ---- the engine's scheduled tasks over device-held state (DeviceScheduledState, INTEGRATION.md §8) ----

  /** What EngineProcessors passes to DueDateTimerChecker instead of the engine's TimerInstanceState. */
  public io.camunda.zeebe.engine.state.immutable.TimerInstanceState timerState(
      final io.camunda.zeebe.engine.state.immutable.TimerInstanceState engineTimers) {
    return new DeviceScheduledState.Timers(this, engineTimers);
  }

  /**
   * ... to JobTimeoutTrigger instead of the engine's JobState (kept: merged activations read the engine's
   * JOB_ACTIVATABLE through it).
   */
  public io.camunda.zeebe.engine.state.immutable.JobState jobState(
      final io.camunda.zeebe.engine.state.immutable.JobState engineJobs) {
    engineJobState = engineJobs;
    return new DeviceScheduledState.Jobs(this, engineJobs);
  }

  /**
   * ... to PendingProcessMessageSubscriptionChecker; {@code engineTransient} is the engine's
   * TransientPendingSubscriptionState (the pending entries of handed-off instances move into it).
   */
  public io.camunda.zeebe.engine.state.immutable.PendingProcessMessageSubscriptionState pendingProcessSubscriptionState(
      final io.camunda.zeebe.engine.state.immutable.PendingProcessMessageSubscriptionState engineState,
      final io.camunda.zeebe.engine.state.message.TransientPendingSubscriptionState engineTransient) {
    engineProcessTransient = engineTransient;
    return new DeviceScheduledState.PendingProcessSubscriptions(this, engineState, engineTransient);
  }

  /**
   * ... to MessageObserver (PendingMessageSubscriptionChecker); {@code engineTransient} is the message
   * side's TransientPendingSubscriptionState (CORRELATING entries of subscriptions moved with their
   * correlation key go into it).
   */
  public io.camunda.zeebe.engine.state.immutable.PendingMessageSubscriptionState pendingMessageSubscriptionState(
      final io.camunda.zeebe.engine.state.immutable.PendingMessageSubscriptionState engineState,
      final io.camunda.zeebe.engine.state.message.TransientPendingSubscriptionState engineTransient) {
    engineMessageTransient = engineTransient;
    return new DeviceScheduledState.PendingMessageSubscriptions(this, engineState, engineTransient);
  }

  /** The broker's JobStreamer (the one EngineProcessors gets): device jobs of streamed types are pushed. */
  public void setJobStreamer(final io.camunda.zeebe.engine.processing.streamprocessor.JobStreamer streamer) {
    jobStreams = new JobStreams(streamer);
  }

  /** The DueDateTimerChecker device TIMER:CREATED records schedule (CatchEventBehavior's side effect). */
  public void setDueDateTimerChecker(final io.camunda.zeebe.engine.processing.timer.DueDateTimerChecker checker) {
    dueDateTimerChecker = checker;
  }

  void timerCreated(final ProcessingResultBuilder out, final long dueDate) {
    if (dueDateTimerChecker != null) {
      out.appendPostCommitTask(() -> {
        dueDateTimerChecker.scheduleTimer(dueDate);
        return true;
      });
    }
  }

  /** The device state equals the log's: the current window's commands were all emitted. */
  boolean scheduledReady() {
    return windowDone;
  }

  MemorySegment handle() {
    return handle;
  }

  /** The stored JobRecord of a zbhip_record JOB row (zbhip_timed_out_jobs / zbhip_time_out_job). */
  JobRecord storedJob(final MemorySegment row) {
    return (JobRecord) window.valueOf(row, this);
  }

  // ---- JOB:TIME_OUT of a device job (JobTimeOutProcessor.java:46-73) ------------------------------

  private ProcessingResult timeOutJob(final TypedRecord record, final ProcessingResultBuilder out) {
    jobStreams.sync(handle, deviceJobTypes());
    ZbHip.setKeyIfHigher(handle, keyGenerator.getCurrentKey());
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment r = a.allocate(ZbHip.RECORD.byteSize() * 2, 8);
      final long n = ZbHip.timeOutJob(handle, record.getKey(), ActorClock.currentTimeMillis(), r);
      if (r.get(java.lang.foreign.ValueLayout.JAVA_BYTE, ZbHip.Rec.RECORD_TYPE) == RecordType.COMMAND_REJECTION.value()) {
        final RecordMetadata meta = new RecordMetadata().valueType(ValueType.JOB);
        meta.recordType(RecordType.COMMAND_REJECTION).intent(JobIntent.TIME_OUT)
            .rejectionType(io.camunda.zeebe.protocol.record.RejectionType.NOT_FOUND)
            .rejectionReason(rejectionReason(r));
        out.appendRecord(record.getKey(), (JobRecord) record.getValue(), meta);
        return out.build();
      }
      // JOB:TIMED_OUT with the stored job; publishWork: the push (JOB_BATCH:ACTIVATED) of a job stream's
      // type, else notifyWorkAvailable (a side effect, no record)
      appendDeviceRecords(r, n, out);
    }
    keyGenerator.setKeyIfHigher(ZbHip.currentKey(handle));
    return out.build();
  }

  // ---- JOB:FAIL of a device job (JobFailProcessor.java:79-162) -------------------------------------

  private ProcessingResult failJob(final TypedRecord record, final ProcessingResultBuilder out) {
    final JobRecord v = (JobRecord) record.getValue();
    jobStreams.sync(handle, deviceJobTypes());
    ZbHip.setKeyIfHigher(handle, keyGenerator.getCurrentKey());
    final int slot = (int) (ZbHip.resolveKey(handle, record.getKey()) >>> 16);
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment r = a.allocate(ZbHip.RECORD.byteSize() * 2, 8);
      final byte[] message = new byte[v.getErrorMessageBuffer().capacity()];
      v.getErrorMessageBuffer().getBytes(0, message);
      final long n = ZbHip.failJob(handle, record.getKey(), v.getRetries(), v.getRetryBackoff(), message,
          v.getVariablesBuffer().capacity() > 1 ? 1 : 0, ActorClock.currentTimeMillis(), r);
      if (n < 0) {
        // outside the device subset (variables, a retry back-off): the engine's, with the instance
        handOff(slot);
        keyGenerator.setKeyIfHigher(ZbHip.currentKey(handle));
        return engine.process(record, out);
      }
      if (r.get(java.lang.foreign.ValueLayout.JAVA_BYTE, ZbHip.Rec.RECORD_TYPE) == RecordType.COMMAND_REJECTION.value()) {
        final RecordMetadata meta = new RecordMetadata().valueType(ValueType.JOB);
        meta.recordType(RecordType.COMMAND_REJECTION).intent(JobIntent.FAIL)
            .rejectionType(io.camunda.zeebe.protocol.record.RejectionType.get(
                (short) (r.get(java.lang.foreign.ValueLayout.JAVA_BYTE, ZbHip.Rec.REJECTION_TYPE) & 0xFF)))
            .rejectionReason(rejectionReason(r));
        out.appendRecord(record.getKey(), v, meta);
        return out.build();
      }
      // JOB:FAILED, then the push (retries left) or INCIDENT:CREATED JOB_NO_RETRIES
      final boolean incident = appendDeviceRecords(r, n, out);
      keyGenerator.setKeyIfHigher(ZbHip.currentKey(handle));
      if (incident) {
        // the instance waits for the incident's resolution (JOB:UPDATE_RETRIES, INCIDENT:RESOLVE): the
        // engine's, with the job's FAILED state and the incident rows
        handOff(slot);
      }
    }
    return out.build();
  }

  /**
   * Event rows of a host-side job call (TIMED_OUT / FAILED / JOB_BATCH push / INCIDENT); true if an incident.
   * A job made activatable again (TIMED_OUT, FAILED with retries left) went through publishWork: pushed, or
   * without a stream notifyJobAvailable (BpmnJobActivationBehavior.java:97-111).
   */
  private boolean appendDeviceRecords(final MemorySegment rows, final long n, final ProcessingResultBuilder out) {
    boolean incident = false, pushed = false;
    JobRecord activatable = null;
    for (long k = 0; k < n; k++) {
      final MemorySegment r = rows.asSlice(ZbHip.RECORD.byteSize() * k, ZbHip.RECORD.byteSize());
      final ValueType vt = ValueType.get((short) r.get(java.lang.foreign.ValueLayout.JAVA_BYTE, ZbHip.Rec.VALUE_TYPE));
      final byte intent = r.get(java.lang.foreign.ValueLayout.JAVA_BYTE, ZbHip.Rec.INTENT);
      final RecordMetadata meta = new RecordMetadata().recordType(RecordType.EVENT).valueType(vt)
          .intent(io.camunda.zeebe.protocol.record.intent.Intent.fromProtocolValue(vt, intent));
      final var value = window.valueOf(r, this);
      out.appendRecord(r.get(java.lang.foreign.ValueLayout.JAVA_LONG, ZbHip.Rec.KEY), value, meta);
      if (vt == ValueType.JOB_BATCH) {
        jobStreams.push(out, handle, (JobBatchRecord) value, this);
        pushed = true;
      } else if (vt == ValueType.JOB && (intent == JobIntent.TIMED_OUT.value()
          || (intent == JobIntent.FAILED.value() && ((JobRecord) value).getRetries() > 0))) {
        activatable = (JobRecord) value;
      }
      incident |= vt == ValueType.INCIDENT;
    }
    if (activatable != null && !pushed) {
      jobStreams.notifyAvailable(out, activatable.getType());
    }
    return incident;
  }

  JobStreams jobStreams() {
    return jobStreams;
  }

  /** The job types of device processes (the streams the device must know of). */
  private Set<String> deviceJobTypes() {
    final Set<String> types = deviceProcessJobTypes();
    types.removeAll(engineJobTypes);
    return types;
  }

  /** Every job type a device process declares (some may be held by the engine too). */
  private Set<String> deviceProcessJobTypes() {
    final Set<String> types = new HashSet<>();
    for (final ZbHip.Deployed d : byIndex) {
      for (final String t : d.jobTypes()) {
        if (t != null && !t.isEmpty()) {
          types.add(t);
        }
      }
    }
    return types;
  }

  // ---- job activation (JobBatchActivateProcessor.java:60-143) --------------------------------------

  private ProcessingResult activateJobs(
      final TypedRecord record, final JobBatchRecord batch, final ProcessingResultBuilder out) {
    ZbHip.setKeyIfHigher(handle, keyGenerator.getCurrentKey());
    final JobActivation activation = JobActivation.of(arena, batch, record.getTimestamp(), this);
    ZbHip.activateJobs(handle, activation.command(), activation.jobs(), activation.capacity(), activation.result());
    activation.emit(record, out, this);
    if (activation.key() >= 0) {
      keyGenerator.setKeyIfHigher(activation.key());
    }
    return out.build();
  }

  /**
   * JOB_BATCH:ACTIVATE of a job type both the engine and the device hold jobs of (handed-off instances,
   * engine-only processes of a device type): JobBatchCollector.collectJobs (:67-123) walks JOB_ACTIVATABLE
   * [type, jobKey] in key order over both.  The first maxJobsToActivate keys of the two lists (the engine's
   * JobState.forEachActivatableJobs, zbhip_activatable_jobs) split into each side's share; the engine
   * activates its share first (its nextKey is the batch key: the engine's record and response are caught
   * in a scratch builder), the device its own with the same key (its key counter is one behind), and the
   * one JOB_BATCH:ACTIVATED record -- and the engine's response -- list both in key order
   * (adapter.py _activate_jobs_merged).
   */
  private ProcessingResult activateJobsMerged(
      final TypedRecord record, final JobBatchRecord batch, final ProcessingResultBuilder out) {
    final int max = batch.getMaxJobsToActivate();
    if (max < 1 || batch.getTimeout() < 1 || batch.getType().isEmpty() || engineJobState == null) {
      return engine.process(record, out); // the rejection (or no view of the engine's jobs)
    }
    ZbHip.setKeyIfHigher(handle, keyGenerator.getCurrentKey());
    final long[] device = ZbHip.activatableJobs(handle, batch.getType().getBytes(StandardCharsets.UTF_8), max);
    if (device.length == 0) {
      return engine.process(record, out);
    }
    final List<Long> picked = new ArrayList<>();
    engineJobState.forEachActivatableJobs(batch.getTypeBuffer(), List.of(TenantOwned.DEFAULT_TENANT_IDENTIFIER),
        (key, job) -> {
          picked.add(key);
          return picked.size() < max;
        });
    for (final long k : device) {
      picked.add(k);
    }
    picked.sort(Long::compare);
    final Set<Long> mine = new HashSet<>();
    for (final long k : device) {
      mine.add(k);
    }
    final List<Long> first = picked.subList(0, Math.min(max, picked.size()));
    final int onDevice = (int) first.stream().filter(mine::contains).count();
    if (onDevice == first.size()) {
      return activateJobs(record, batch, out);
    }
    // the command as written (the engine's processor adds its jobs to the command's value)
    final UnsafeBuffer asWritten = new UnsafeBuffer(new byte[batch.getLength()]);
    batch.write(asWritten, 0);
    final ScratchResult share = new ScratchResult();
    batch.setMaxJobsToActivate(first.size() - onDevice);
    engine.process(record, share);
    final JobBatchRecord engineBatch = (JobBatchRecord) share.value;
    final java.util.TreeMap<Long, JobRecord> jobs = new java.util.TreeMap<>();
    final Iterator<JobRecord> engineJobs = engineBatch.jobs().iterator();
    for (final var k : engineBatch.jobKeys()) {
      final JobRecord copy = new JobRecord();
      copy.wrap(engineJobs.next());
      jobs.put(k.getValue(), copy);
    }
    final boolean engineTruncated = engineBatch.getTruncated();
    // the device's share, with the batch key the engine generated
    final JobBatchRecord deviceCmd = new JobBatchRecord();
    deviceCmd.wrap(asWritten);
    deviceCmd.setMaxJobsToActivate(onDevice);
    final JobActivation activation = JobActivation.of(arena, deviceCmd, record.getTimestamp(), this);
    ZbHip.activateJobs(handle, activation.command(), activation.jobs(), activation.capacity(), activation.result());
    if (activation.key() != share.key) {
      throw new IllegalStateException("merged activation: batch keys " + share.key + " / " + activation.key());
    }
    jobs.putAll(activation.activated(this));
    final JobBatchRecord merged = new JobBatchRecord();
    merged.wrap(asWritten);
    for (final var e : jobs.entrySet()) {
      merged.jobKeys().add().setValue(e.getKey());
      merged.jobs().add().wrap(e.getValue());
    }
    merged.setTruncated(engineTruncated || activation.truncated());
    keyGenerator.setKeyIfHigher(share.key);
    out.appendRecord(share.key, merged, share.metadata);
    if (share.response != null) {
      share.response.replay(out, merged);
    }
    for (final var task : share.postCommit) {
      out.appendPostCommitTask(task);
    }
    return out.build();
  }

  /** The engine's share of a merged activation: its one record, response and side effects, held back. */
  private static final class ScratchResult implements ProcessingResultBuilder, ProcessingResult {
    long key = -1;
    io.camunda.zeebe.protocol.record.RecordValue value;
    final RecordMetadata metadata = new RecordMetadata();
    Response response;
    final List<io.camunda.zeebe.stream.api.PostCommitTask> postCommit = new ArrayList<>();

    record Response(RecordType type, long key, io.camunda.zeebe.protocol.record.intent.Intent intent,
        ValueType valueType, io.camunda.zeebe.protocol.record.RejectionType rejectionType, String reason,
        long requestId, int requestStreamId) {
      void replay(final ProcessingResultBuilder out, final io.camunda.zeebe.msgpack.UnpackedObject value) {
        out.withResponse(type, key, intent, value, valueType, rejectionType, reason, requestId, requestStreamId);
      }
    }

    @Override
    public io.camunda.zeebe.util.Either<RuntimeException, ProcessingResultBuilder> appendRecordReturnEither(
        final long key, final io.camunda.zeebe.protocol.record.RecordValue value, final RecordMetadata metadata) {
      this.key = key;
      this.value = value;
      this.metadata.wrap(metadata);
      return io.camunda.zeebe.util.Either.right(this);
    }

    @Override
    public ProcessingResultBuilder withResponse(final RecordType type, final long key,
        final io.camunda.zeebe.protocol.record.intent.Intent intent, final io.camunda.zeebe.msgpack.UnpackedObject value,
        final ValueType valueType, final io.camunda.zeebe.protocol.record.RejectionType rejectionType,
        final String rejectionReason, final long requestId, final int requestStreamId) {
      response = new Response(type, key, intent, valueType, rejectionType, rejectionReason, requestId, requestStreamId);
      return this;
    }

    @Override
    public ProcessingResultBuilder appendPostCommitTask(final io.camunda.zeebe.stream.api.PostCommitTask task) {
      postCommit.add(task);
      return this;
    }

    @Override
    public ProcessingResultBuilder resetPostCommitTasks() {
      postCommit.clear();
      return this;
    }

    @Override
    public ProcessingResult build() {
      return this;
    }

    @Override
    public boolean canWriteEventOfLength(final int eventLength) {
      return true;
    }

    // ProcessingResult (ProcessingResult.java:17-51): never handed to the platform
    @Override
    public io.camunda.zeebe.stream.api.records.ImmutableRecordBatch getRecordBatch() {
      throw new UnsupportedOperationException();
    }

    @Override
    public java.util.Optional<io.camunda.zeebe.stream.api.ProcessingResponse> getProcessingResponse() {
      throw new UnsupportedOperationException();
    }

    @Override
    public boolean executePostCommitTasks() {
      throw new UnsupportedOperationException();
    }

    @Override
    public boolean isEmpty() {
      return key < 0;
    }
  }

  public void close() {
    if (handle != null) {
      ZbHip.close(handle);
      handle = null;
    }
    arena.close();
  }
}
