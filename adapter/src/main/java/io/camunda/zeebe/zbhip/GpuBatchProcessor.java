/*
 * The host adapter a maintainer adds to the broker: a stream-platform RecordProcessor placed before
 * the engine (StreamProcessorTransitionStep.java:135-147: List.of(gpu, engine, checkpointProcessor))
 * that answers the hot-path commands from libzbhip.so and hands everything else -- and every
 * command the device falls back on -- to the unchanged engine.
 *
 * Not compiled in this image (no JDK); written against the reference's interfaces:
 *   RecordProcessor                stream-platform/.../stream/api/RecordProcessor.java:17-108
 *   ProcessingResultBuilder        stream-platform/.../stream/api/ProcessingResultBuilder.java:22-80
 *   RecordProcessorContext         stream-platform/.../stream/api/RecordProcessorContext.java:18-32
 *   KeyGeneratorControls           stream-platform/.../stream/impl/state/DbKeyGenerator.java:40-60
 *   LogStreamReader / LoggedEvent  logstreams/.../log/LogStreamReader.java, LoggedEvent.java
 * See INTEGRATION.md for the contract of every zbhip call used here.
 */
package io.camunda.zeebe.zbhip;

import io.camunda.zeebe.engine.Engine;
import io.camunda.zeebe.logstreams.log.LogStreamReader;
import io.camunda.zeebe.logstreams.log.LoggedEvent;
import io.camunda.zeebe.protocol.impl.record.RecordMetadata;
import io.camunda.zeebe.protocol.impl.record.value.job.JobRecord;
import io.camunda.zeebe.protocol.impl.record.value.processinstance.ProcessInstanceCreationRecord;
import io.camunda.zeebe.protocol.impl.record.value.timer.TimerRecord;
import io.camunda.zeebe.protocol.record.RecordType;
import io.camunda.zeebe.protocol.record.ValueType;
import io.camunda.zeebe.protocol.record.intent.JobIntent;
import io.camunda.zeebe.protocol.record.intent.ProcessInstanceCreationIntent;
import io.camunda.zeebe.protocol.record.intent.TimerIntent;
import io.camunda.zeebe.scheduler.clock.ActorClock;
import io.camunda.zeebe.stream.api.ProcessingResult;
import io.camunda.zeebe.stream.api.ProcessingResultBuilder;
import io.camunda.zeebe.stream.api.RecordProcessor;
import io.camunda.zeebe.stream.api.RecordProcessorContext;
import io.camunda.zeebe.stream.api.records.TypedRecord;
import io.camunda.zeebe.stream.impl.state.KeyGeneratorControls;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.BitSet;
import java.util.HashMap;
import java.util.HashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;

public final class GpuBatchProcessor implements RecordProcessor {

  /** Deployed processes the adapter knows: bpmnProcessId (latest version) / definition key. */
  public interface Deployments {
    /** BPMN XML of every deployed process, in deployment order (DbProcessState). */
    List<DeployedResource> all();

    record DeployedResource(long definitionKey, String bpmnProcessId, int version, byte[] xml) {}
  }

  private static final int WINDOW = 1 << 16; // commands per submitted window (zbhip_config.max_commands)
  private static final int INSTANCES = 1 << 22; // instance slots in HBM (288 GB holds ~2.5e9)

  private final Engine engine;
  private final LogStreamReader reader;
  private final Deployments deployments;
  private final RawDbWriter zeebeDb;
  private final int partitionCount;
  private final int device;

  private final Arena arena = Arena.ofShared();
  private MemorySegment handle;
  private KeyGeneratorControls keyGenerator;
  private final Map<Long, ZbHip.Deployed> byKey = new HashMap<>();
  private final Map<String, ZbHip.Deployed> latestById = new HashMap<>();
  private final List<ZbHip.Deployed> byIndex = new ArrayList<>();
  private final BitSet usedSlots = new BitSet(INSTANCES);
  private int nextFreeSlot;

  // the window read ahead from the log
  private final Window window = new Window();
  private final Set<Integer> handedOff = new HashSet<>();

  public GpuBatchProcessor(
      final Engine engine,
      final LogStreamReader reader,
      final Deployments deployments,
      final RawDbWriter zeebeDb,
      final int partitionCount,
      final int device) {
    this.engine = engine;
    this.reader = reader;
    this.deployments = deployments;
    this.zeebeDb = zeebeDb;
    this.partitionCount = partitionCount;
    this.device = device;
  }

  @Override
  public void init(final RecordProcessorContext ctx) {
    engine.init(ctx);
    keyGenerator = (KeyGeneratorControls) ctx.getKeyGenerator();
    handle =
        ZbHip.open(
            arena, ctx.getPartitionId(), partitionCount, device, /* maxCommandsInBatch */ 100, INSTANCES, WINDOW,
            keyGenerator.getCurrentKey(), /* correlation slots: config 5 only */ 0);
    for (final var d : deployments.all()) {
      deploy(d);
    }
    window.init(arena);
  }

  private void deploy(final Deployments.DeployedResource d) {
    final ZbHip.Deployed p = ZbHip.deploy(handle, d.xml(), d.definitionKey(), d.version());
    if (p == null) {
      return; // outside the device subset: its instances run on the CPU engine
    }
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
        || valueType == ValueType.TIMER || engine.accepts(valueType);
  }

  @Override
  public void replay(final TypedRecord record) {
    // events only; the appliers write RocksDB.  Instances restored this way are loaded into HBM
    // after recovery with ZbHip.importStateDb over the hot-path column families.
    engine.replay(record);
  }

  @Override
  public ProcessingResult process(final TypedRecord record, final ProcessingResultBuilder out) {
    if (!isHotPath(record)) {
      return engine.process(record, out);
    }
    if (!window.covers(record.getPosition())) {
      fillWindow(record);
    }
    final int i = window.indexOf(record.getPosition());
    if (i < 0) {
      return engine.process(record, out); // the read-ahead stopped before it (e.g. a CPU-resident instance)
    }
    if (ZbHip.commandStatus(handle, i) != 0) {
      return fallBack(i, record, out);
    }
    window.emit(i, out, this);
    return out.build();
  }

  @Override
  public ProcessingResult onProcessingError(
      final Throwable error, final TypedRecord record, final ProcessingResultBuilder out) {
    return engine.onProcessingError(error, record, out);
  }

  // ---- the window ------------------------------------------------------------------------------

  private boolean isHotPath(final TypedRecord record) {
    if (record.getRecordType() != RecordType.COMMAND) {
      return false;
    }
    if (record.getValueType() == ValueType.PROCESS_INSTANCE_CREATION) {
      return record.getIntent() == ProcessInstanceCreationIntent.CREATE;
    }
    // JOB:COMPLETE of a device job; TIMER:TRIGGER (DueDateTimerChecker's command) of a device timer
    return ((record.getValueType() == ValueType.JOB && record.getIntent() == JobIntent.COMPLETE)
            || (record.getValueType() == ValueType.TIMER && record.getIntent() == TimerIntent.TRIGGER))
        && ZbHip.resolveKey(handle, record.getKey()) >= 0;
  }

  /**
   * Reads consecutive hot-path commands from the log starting at {@code first}, converts them to
   * zbhip_command rows (+ variable document entries), submits and runs them once, and drains the
   * window's records (keys relabelled to DbKeyGenerator's, ordered by source command).
   */
  private void fillWindow(final TypedRecord first) {
    window.reset(first.getPosition());
    reader.seek(first.getPosition());
    final RecordMetadata meta = new RecordMetadata();
    final ProcessInstanceCreationRecord create = new ProcessInstanceCreationRecord();
    final JobRecord job = new JobRecord();
    final TimerRecord timer = new TimerRecord();
    while (reader.hasNext() && window.size() < WINDOW) {
      final LoggedEvent event = reader.next();
      event.readMetadata(meta);
      if (meta.getRecordType() != RecordType.COMMAND) {
        continue; // follow-up events of earlier batches between the commands
      }
      if (meta.getValueType() == ValueType.PROCESS_INSTANCE_CREATION
          && meta.getIntent() == ProcessInstanceCreationIntent.CREATE) {
        event.readValue(create);
        final ZbHip.Deployed p =
            create.getProcessDefinitionKey() > 0
                ? byKey.get(create.getProcessDefinitionKey())
                : latestById.get(create.getBpmnProcessId());
        if (p == null || !window.addCreate(event.getPosition(), p.index(), takeSlot(), create.getVariablesBuffer(), this)) {
          break; // a process on the CPU engine: the window ends before it (log order is kept)
        }
      } else if (meta.getValueType() == ValueType.JOB && meta.getIntent() == JobIntent.COMPLETE) {
        event.readValue(job);
        final long ref = ZbHip.resolveKey(handle, event.getKey());
        if (ref < 0 || !window.addJobComplete(event.getPosition(), ref, job.getVariablesBuffer(), this)) {
          break; // a job of a CPU-resident instance
        }
      } else if (meta.getValueType() == ValueType.TIMER && meta.getIntent() == TimerIntent.TRIGGER) {
        event.readValue(timer);
        final long ref = ZbHip.resolveKey(handle, event.getKey());
        if (ref < 0) {
          break; // a timer of a CPU-resident instance
        }
        window.addTimerTrigger(event.getPosition(), ref, timer.getDueDate());
      } else {
        break; // any other command ends the window
      }
    }
    // the window's clock: TIMER:CREATED dueDates (CatchEventBehavior.java:310, ActorClock)
    ZbHip.setClock(handle, ActorClock.currentTimeMillis());
    window.submitRunDrain(handle);
    // instances that ended in this window free their slots for later CREATEs
    window.forEachEndedInstance(slot -> usedSlots.clear(slot));
  }

  int internName(final String name) {
    return ZbHip.intern(handle, name);
  }

  long internString(final byte[] value) {
    return ZbHip.internString(handle, value);
  }

  private int takeSlot() {
    int s = usedSlots.nextClearBit(nextFreeSlot);
    if (s >= INSTANCES) {
      s = usedSlots.nextClearBit(0);
    }
    usedSlots.set(s);
    nextFreeSlot = s + 1;
    return s;
  }

  ZbHip.Deployed process(final int index) {
    return byIndex.get(index);
  }

  /** The partition's name dictionary (variable names of VARIABLE records). */
  String name(final int id) {
    return ZbHip.name(handle, id);
  }

  String rejectionReason(final MemorySegment rec) {
    return ZbHip.rejectionReason(handle, rec);
  }

  // ---- fallback hand-off (INTEGRATION.md §8; Engine.java:134, ProcessingStateMachine.java:276-310) ----

  private ProcessingResult fallBack(final int i, final TypedRecord record, final ProcessingResultBuilder out) {
    final int instance = window.instanceOf(i);
    if (handedOff.add(instance)) {
      // the instance's zb-db entries into RocksDB (the platform's transaction), then off the device
      ZbHip.handOff(handle, instance, zeebeDb::upsert);
      usedSlots.clear(instance);
    }
    final long before = ZbHip.keyBefore(handle, i);
    keyGenerator.setKeyIfHigher(before);
    final ProcessingResult result = engine.process(record, out);
    ZbHip.setExternalKeys(handle, i, (int) (keyGenerator.getCurrentKey() - before));
    return result;
  }

  /** Raw column-family writes of a hand-off; the broker binds this to its ZeebeDb transaction. */
  public interface RawDbWriter {
    void upsert(int columnFamily, byte[] key, byte[] value);
  }

  public void close() {
    if (handle != null) {
      ZbHip.close(handle);
      handle = null;
    }
    arena.close();
  }
}
