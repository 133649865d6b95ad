/*
 * Config 5 on the adapter: the message commands of the log as device commands, and the commands a
 * device batch sends to other partitions as the reference's record values.  The Python mirror is
 * zeebe_amd/adapter.py (GpuBatchProcessor._message_command, xpart_value); tests/test_gpu_psm_messages.py
 * runs it on three partitions inside a restatement of ProcessingStateMachine against the engine alone.
 *
 *  - MESSAGE:PUBLISH (MessagePublishProcessor) with time-to-live 0, no message id and no variables,
 *    of a message name a device catch event waits for -> ZBHIP_CMD_PUBLISH on the correlation slot
 *    (the value-dictionary id of the correlation key);
 *  - one owner per correlation key: a publish the engine processes (outside that subset) first moves its
 *    key's subscriptions from the device into RocksDB (toEngine: zbhip_export_correlation_slots_db +
 *    zbhip_evict_correlation_slots), and every later message command of the key is the engine's -- it
 *    buffers messages with a time-to-live, correlates them when a subscription opens and expires them
 *    (MessagePublishProcessor.java:83-185, MessageCorrelator.java:41-96, MessageTimeToLiveChecker);
 *  - MESSAGE_SUBSCRIPTION:CREATE / CORRELATE (the message partition's side) and
 *    PROCESS_MESSAGE_SUBSCRIPTION:CREATE / CORRELATE (the process instance partition's side) ->
 *    zbhip_xpart_cmd rows of the window (ZBHIP_CMD_MSG_SUB_* / ZBHIP_CMD_PMS_*).
 *  - zbhip_outbox_command rows -> the value SubscriptionCommandSender sets for each kind
 *    (SubscriptionCommandSender.java:54-218), sent by InterPartitionCommandSender.sendCommand in a
 *    post-commit task of the sending batch (handleFollowUpCommandBasedOnPartition, :320-338).
 *
 * Not compiled in this image (no JDK).  Value classes: MessageRecord.java:37-43,
 * MessageSubscriptionRecord.java:40-48, ProcessMessageSubscriptionRecord.java:44-54.
 */
package io.camunda.zeebe.zbhip;

import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

import io.camunda.zeebe.protocol.Protocol;
import io.camunda.zeebe.protocol.impl.record.UnifiedRecordValue;
import io.camunda.zeebe.protocol.impl.record.value.message.MessageRecord;
import io.camunda.zeebe.protocol.impl.record.value.message.MessageSubscriptionRecord;
import io.camunda.zeebe.protocol.impl.record.value.message.ProcessMessageSubscriptionRecord;
import io.camunda.zeebe.protocol.record.ValueType;
import io.camunda.zeebe.protocol.record.intent.Intent;
import io.camunda.zeebe.protocol.record.intent.MessageIntent;
import io.camunda.zeebe.protocol.record.intent.MessageSubscriptionIntent;
import io.camunda.zeebe.protocol.record.intent.ProcessMessageSubscriptionIntent;
import io.camunda.zeebe.stream.api.InterPartitionCommandSender;
import io.camunda.zeebe.stream.api.ProcessingResultBuilder;
import io.camunda.zeebe.stream.api.records.TypedRecord;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import java.util.Set;
import org.agrona.DirectBuffer;
import org.agrona.concurrent.UnsafeBuffer;

final class Messages {

  static final int NO_STRING = 0xFFFFFFFF;
  private static final String TENANT = "<default>";

  /** A log command as a device command: zbhip_command fields and, for subscription commands, its xpart row. */
  record DeviceCommand(int instance, byte kind, int ref, MemorySegment xpart) {}

  private final int partitionId;
  private final int correlationSlots;
  private final Set<String> messageNames;
  // message start event names of every deployment: a publish of such a name starts instances
  // (MessagePublishProcessor.correlateToMessageStartEvents, :157-180), so it is the engine's
  private final Set<String> startMessageNames;
  // MESSAGE_SUBSCRIPTION_BY_KEY [elementInstanceKey, messageName] -> correlation slot of an open
  // subscription: a MESSAGE_SUBSCRIPTION:CORRELATE's value carries no correlation key
  private final Map<SubscriptionKey, Integer> subscriptions = new HashMap<>();
  // correlation keys whose message state the engine holds (toEngine)
  private final Set<String> engineOwned = new java.util.HashSet<>();
  // CORRELATING entries of subscriptions moved with their key, for the engine's transient state
  final List<Map.Entry<SubscriptionKey, PendingSubscription>> movedPendingMessage = new ArrayList<>();
  // (elementInstanceKey, messageName) -> routing handle (slot << 16 | ordinal) of a device subscription
  private final Map<SubscriptionKey, Long> handles = new HashMap<>();
  private final java.util.Set<Integer> closingSlots = new java.util.HashSet<>();
  // the transient pending states the appliers of the device's records keep in the reference
  // (DbProcessMessageSubscriptionState.java:82-124,180-222, DbMessageSubscriptionState.java:157-222):
  // OPENING / CLOSING process message subscriptions and CORRELATING message subscriptions, with the time
  // they were last sent (insertion order kept: TransientPendingSubscriptionState.entriesBefore sorts by it)
  final Map<SubscriptionKey, PendingProcessSubscription> pendingProcess = new java.util.LinkedHashMap<>();
  final Map<SubscriptionKey, PendingSubscription> pendingMessage = new java.util.LinkedHashMap<>();

  record SubscriptionKey(long elementInstanceKey, String messageName) {}

  static final class PendingProcessSubscription {
    long sentTime;
    final ProcessMessageSubscriptionRecord record = new ProcessMessageSubscriptionRecord();
    boolean opening;
  }

  static final class PendingSubscription {
    long sentTime;
    final MessageSubscriptionRecord record = new MessageSubscriptionRecord();
  }

  Messages(
      final int partitionId,
      final int correlationSlots,
      final Set<String> messageNames,
      final Set<String> startMessageNames) {
    this.partitionId = partitionId;
    this.correlationSlots = correlationSlots;
    this.messageNames = messageNames;
    this.startMessageNames = startMessageNames;
  }

  boolean enabled() {
    return correlationSlots > 0;
  }

  /** Whether the engine owns a correlation key of this partition (toEngine ran). */
  boolean ownsKeys() {
    return !engineOwned.isEmpty();
  }

  /** A message-partition command (its subject a correlation slot, not an instance). */
  static boolean isSlotCommand(final ValueType vt, final TypedRecord record) {
    return vt == ValueType.MESSAGE || vt == ValueType.MESSAGE_SUBSCRIPTION;
  }

  static boolean isMessageCommand(final ValueType vt) {
    return vt == ValueType.MESSAGE || vt == ValueType.MESSAGE_SUBSCRIPTION
        || vt == ValueType.PROCESS_MESSAGE_SUBSCRIPTION;
  }

  /**
   * The device form of a message command, or null when the engine keeps it: a PUBLISH outside the
   * subset (or of a message start event's name), PROCESS_MESSAGE_SUBSCRIPTION commands of an instance the device does not hold,
   * MESSAGE_SUBSCRIPTION commands of a local instance the device does not hold.
   */
  DeviceCommand of(final TypedRecord record, final GpuBatchProcessor p, final Arena arena) {
    if (record.getValueType() == ValueType.MESSAGE) {
      final MessageRecord v = (MessageRecord) record.getValue();
      if (record.getIntent() != MessageIntent.PUBLISH || v.getTimeToLive() != 0 || !v.getMessageId().isEmpty()
          || v.getVariablesBuffer().capacity() > 1 || !messageNames.contains(v.getName())
          || startMessageNames.contains(v.getName()) || engineOwned.contains(v.getCorrelationKey())) {
        return null;
      }
      final long corr = p.internString(v.getCorrelationKey().getBytes(StandardCharsets.UTF_8));
      if (corr >= correlationSlots) {
        return null;
      }
      return new DeviceCommand((int) corr, ZbHip.CMD_PUBLISH, p.internName(v.getName()), null);
    }
    final MemorySegment x = arena.allocate(ZbHip.XPART);
    final long pik, eik;
    final byte kind;
    if (record.getValueType() == ValueType.PROCESS_MESSAGE_SUBSCRIPTION) {
      // the process instance partition's side: the subscribing element instance of a device instance
      final ProcessMessageSubscriptionRecord v = (ProcessMessageSubscriptionRecord) record.getValue();
      kind = record.getIntent() == ProcessMessageSubscriptionIntent.CREATE ? ZbHip.CMD_PMS_CREATE
          : record.getIntent() == ProcessMessageSubscriptionIntent.CORRELATE ? ZbHip.CMD_PMS_CORRELATE
          : record.getIntent() == ProcessMessageSubscriptionIntent.DELETE ? ZbHip.CMD_PMS_DELETE : 0;
      if (kind == 0 || v.getVariablesBuffer().capacity() > 1) {
        return null;
      }
      pik = v.getProcessInstanceKey();
      eik = v.getElementInstanceKey();
      long pi = p.resolve(pik), el = p.resolve(eik);
      if ((pi < 0 || el < 0) && kind == ZbHip.CMD_PMS_DELETE) {
        // a closing subscription's acknowledgement may arrive after its instance ended: the routing
        // handle kept since PROCESS_MESSAGE_SUBSCRIPTION:CREATING
        pi = el = handles.getOrDefault(new SubscriptionKey(eik, v.getMessageName()), -1L);
      }
      if (pi < 0 || el < 0 || (pi >>> 16) != (el >>> 16)) {
        return null;
      }
      fill(x, pik, eik, v.getMessageKey(), p.internName(v.getMessageName()),
          v.getBpmnProcessId().isEmpty() ? 0xFFFF : p.internName(v.getBpmnProcessId()),
          v.getCorrelationKey().isEmpty() ? NO_STRING : (int) p.internString(bytes(v.getCorrelationKeyBuffer())),
          kind, v.isInterrupting(), (int) (el >>> 16), (int) (el & 0xFFFF), v.getSubscriptionPartitionId());
      return new DeviceCommand((int) (el >>> 16), kind, 0, x);
    }
    // the message partition's side
    final MessageSubscriptionRecord v = (MessageSubscriptionRecord) record.getValue();
    kind = record.getIntent() == MessageSubscriptionIntent.CREATE ? ZbHip.CMD_MSG_SUB_CREATE
        : record.getIntent() == MessageSubscriptionIntent.CORRELATE ? ZbHip.CMD_MSG_SUB_CORRELATE
        : record.getIntent() == MessageSubscriptionIntent.DELETE ? ZbHip.CMD_MSG_SUB_DELETE : 0;
    if (kind == 0 || v.getVariablesBuffer().capacity() > 1) {
      return null;
    }
    pik = v.getProcessInstanceKey();
    eik = v.getElementInstanceKey();
    // a key the engine owns: a CREATE by its key, a CORRELATE / DELETE (no key in the value) when the
    // device holds no such subscription
    final SubscriptionKey sk = new SubscriptionKey(eik, v.getMessageName());
    if (kind == ZbHip.CMD_MSG_SUB_CREATE ? engineOwned.contains(v.getCorrelationKey()) : !subscriptions.containsKey(sk)) {
      return null;
    }
    // the routing handle of the subscribing element instance: its slot and key ordinal when the
    // instance lives here (a local correlation enters it in the same batch), else an id derived from
    // the element instance key -- unique per subscription like the reference's
    // [elementInstanceKey, messageName]; the process instance partition resolves the keys itself
    final int src = Protocol.decodePartitionId(pik);
    final int inst, ord;
    if (src == partitionId) {
      final long el = p.resolve(eik);
      if (el < 0) {
        return null;
      }
      inst = (int) (el >>> 16);
      ord = (int) (el & 0xFFFF);
    } else {
      final long n = eik - ((long) Protocol.decodePartitionId(eik) << Protocol.KEY_BITS);
      inst = (int) n;
      ord = (int) ((n >>> 32) & 0xFFFF);
    }
    int corr = v.getCorrelationKey().isEmpty() ? NO_STRING : (int) p.internString(bytes(v.getCorrelationKeyBuffer()));
    if (kind == ZbHip.CMD_MSG_SUB_CORRELATE || kind == ZbHip.CMD_MSG_SUB_DELETE) {
      // no correlation key in the value: the slot of the subscription it names
      corr = subscriptions.get(sk);
    }
    if (Integer.toUnsignedLong(corr) >= correlationSlots) {
      return null;
    }
    if (kind == ZbHip.CMD_MSG_SUB_CREATE) {
      subscriptions.putIfAbsent(sk, corr); // a DELETE read into the same window finds the slot
    }
    fill(x, pik, eik, v.getMessageKey(), p.internName(v.getMessageName()),
        v.getBpmnProcessId().isEmpty() ? 0xFFFF : p.internName(v.getBpmnProcessId()), corr, kind,
        v.isInterrupting(), inst, ord, src);
    return new DeviceCommand(corr, kind, 0, x);
  }

  private void fill(final MemorySegment x, final long pik, final long eik, final long messageKey, final int name,
      final int bpmn, final int corr, final byte kind, final boolean interrupting, final int instance,
      final int ord, final int source) {
    x.set(JAVA_LONG, 0, eik);
    x.set(JAVA_LONG, 8, pik);
    x.set(JAVA_LONG, 16, messageKey);
    x.set(JAVA_INT, 24, corr);
    x.set(JAVA_INT, 28, instance);
    x.set(JAVA_SHORT, 32, (short) ord);
    x.set(JAVA_SHORT, 34, (short) name);
    x.set(JAVA_SHORT, 36, (short) bpmn);
    x.set(JAVA_BYTE, 38, kind);
    x.set(JAVA_BYTE, 39, (byte) (interrupting ? 1 : 0));
    x.set(JAVA_SHORT, 40, (short) source);
    x.set(JAVA_SHORT, 42, (short) partitionId);
  }

  /** An emitted MESSAGE_SUBSCRIPTION event: keeps MESSAGE_SUBSCRIPTION_BY_KEY's slot map current. */
  void onSubscriptionEvent(final Intent intent, final MessageSubscriptionRecord v, final int correlationSlot) {
    final SubscriptionKey k = new SubscriptionKey(v.getElementInstanceKey(), v.getMessageName());
    if (intent == MessageSubscriptionIntent.CREATED) {
      subscriptions.put(k, correlationSlot);
    } else if (intent == MessageSubscriptionIntent.CORRELATED || intent == MessageSubscriptionIntent.DELETED) {
      // (a non-interrupting subscription stays open after its correlation: updateToCorrelatedState)
      if (intent == MessageSubscriptionIntent.DELETED || v.isInterrupting()) {
        subscriptions.remove(k);
      }
      pendingMessage.remove(k);
    } else if (intent == MessageSubscriptionIntent.CORRELATING) {  // updateToCorrelatingState
      final PendingSubscription ps = pendingMessage.computeIfAbsent(k, x -> new PendingSubscription());
      ps.sentTime = io.camunda.zeebe.scheduler.clock.ActorClock.currentTimeMillis();
      ps.record.wrap(v);
    }
  }

  /**
   * An emitted PROCESS_MESSAGE_SUBSCRIPTION event of instance slot `slot`: the routing handle of a device
   * subscription is kept from CREATING until it is gone, and a slot with a closing subscription stays
   * taken until its DELETED (the device row outlives the instance).
   */
  void onProcessSubscriptionEvent(final Intent intent, final ProcessMessageSubscriptionRecord v, final int slot,
      final GpuBatchProcessor p) {
    final SubscriptionKey k = new SubscriptionKey(v.getElementInstanceKey(), v.getMessageName());
    if (intent == ProcessMessageSubscriptionIntent.CREATING || intent == ProcessMessageSubscriptionIntent.DELETING) {
      // put (OPENING) / updateToClosingState: pending since now
      final PendingProcessSubscription ps = pendingProcess.computeIfAbsent(k, x -> new PendingProcessSubscription());
      ps.sentTime = io.camunda.zeebe.scheduler.clock.ActorClock.currentTimeMillis();
      ps.record.wrap(v);
      ps.opening = intent == ProcessMessageSubscriptionIntent.CREATING;
    }
    if (intent == ProcessMessageSubscriptionIntent.CREATING) {
      handles.put(k, p.resolve(v.getElementInstanceKey()));
    } else if (intent == ProcessMessageSubscriptionIntent.DELETING) {
      closingSlots.add(slot);
    } else if (intent == ProcessMessageSubscriptionIntent.CREATED) {
      pendingProcess.remove(k);  // updateToOpenedState
    } else if (intent == ProcessMessageSubscriptionIntent.CORRELATED || intent == ProcessMessageSubscriptionIntent.DELETED) {
      // (a non-interrupting subscription stays open after its correlation: updateToOpenedState)
      if (intent == ProcessMessageSubscriptionIntent.DELETED || v.isInterrupting()) {
        handles.remove(k);
      }
      pendingProcess.remove(k);
      if (intent == ProcessMessageSubscriptionIntent.DELETED) {
        closingSlots.remove(slot);
      }
    }
  }

  // pending entries of handed-off instances, moved into the engine's transient state by
  // DeviceScheduledState.PendingProcessSubscriptions (the hand-off writes RocksDB rows only)
  final List<Map.Entry<SubscriptionKey, PendingProcessSubscription>> movedPending = new ArrayList<>();

  /**
   * Instance slot `slot` was handed off to the engine: its subscriptions are the engine's now -- no
   * closing row holds the slot, no routing handle points into it, their pending entries move.
   */
  void handedOff(final int slot) {
    handedOff(slot, null);
  }

  void handedOff(final int slot, final io.camunda.zeebe.engine.state.message.TransientPendingSubscriptionState engine) {
    closingSlots.remove(slot);
    for (final var it = handles.entrySet().iterator(); it.hasNext(); ) {
      final var e = it.next();
      if (e.getValue() >= 0 && (int) (e.getValue() >>> 16) == slot) {
        final PendingProcessSubscription ps = pendingProcess.remove(e.getKey());
        if (ps != null && engine != null) {  // the engine's transient state now
          engine.add(new io.camunda.zeebe.engine.state.message.TransientPendingSubscriptionState.PendingSubscription(
              e.getKey().elementInstanceKey(), e.getKey().messageName(), ps.record.getTenantId()), ps.sentTime);
        } else if (ps != null) {
          movedPending.add(Map.entry(e.getKey(), ps));
        }
        it.remove();
      }
    }
  }

  /**
   * One owner per correlation key: before the engine processes a publish of {@code correlationKey} (or a
   * message command of it the device declined), the key's subscriptions move from its correlation slot
   * into RocksDB and off the device, their CORRELATING entries into the engine's transient state, and
   * the key's later message commands go to the engine (adapter.py _message_state_to_engine).
   */
  void toEngine(final String correlationKey, final GpuBatchProcessor p, final ZbHip.DbSink rocksDb) {
    if (!engineOwned.add(correlationKey)) {
      return;
    }
    final long slot = p.internString(correlationKey.getBytes(StandardCharsets.UTF_8));
    if (slot < 0 || slot >= correlationSlots) {
      return;
    }
    // subscribers on this partition: the engine's correlations reach them as follow-ups of its own batches,
    // so their instances go with the key (a later local subscription to the key falls back the same way)
    final List<Long> local = new ArrayList<>();
    for (final String row : ZbHip.exportCorrelationSlotRows(p.handle(), (int) slot)) {
      if (row.startsWith("MESSAGE_SUBSCRIPTION_BY_KEY|")) {
        final long pik = Long.parseLong(row.split("processInstanceKey=", 2)[1].split(",", 2)[0]);
        if (Protocol.decodePartitionId(pik) == partitionId) {
          local.add(pik);
        }
      }
    }
    ZbHip.correlationSlotToEngine(p.handle(), (int) slot, rocksDb);
    if (p.scheduledReady()) {
      for (final long pik : local) {
        p.handOffInstanceOf(pik);
      }
    }
    for (final var it = subscriptions.entrySet().iterator(); it.hasNext(); ) {
      final var e = it.next();
      if (e.getValue() == slot) {
        final PendingSubscription ps = pendingMessage.remove(e.getKey());
        if (ps != null && p.engineMessageTransient != null) {  // the engine's transient state now
          p.engineMessageTransient.add(new io.camunda.zeebe.engine.state.message.TransientPendingSubscriptionState
              .PendingSubscription(e.getKey().elementInstanceKey(), e.getKey().messageName(), ps.record.getTenantId()),
              ps.sentTime);
        } else if (ps != null) {
          movedPendingMessage.add(Map.entry(e.getKey(), ps));
        }
        it.remove();
      }
    }
  }

  /** Whether the instance slot waits for a closing subscription's PROCESS_MESSAGE_SUBSCRIPTION:DELETE. */
  boolean closing(final int slot) {
    return closingSlots.contains(slot);
  }

  /** Window command i's sends, handed to InterPartitionCommandSender once its batch is committed. */
  void send(final MemorySegment handle, final int i, final ProcessingResultBuilder out,
      final InterPartitionCommandSender sender, final GpuBatchProcessor p) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment rows = ZbHip.outboxCommand(handle, i, a);
      final long n = rows.byteSize() / ZbHip.XPART.byteSize();
      if (n == 0) {
        return;
      }
      final List<Runnable> sends = new ArrayList<>();
      for (long j = 0; j < n; j++) {
        final MemorySegment x = rows.asSlice(j * ZbHip.XPART.byteSize(), ZbHip.XPART.byteSize());
        final int target = x.get(JAVA_SHORT, 42);
        final byte kind = x.get(JAVA_BYTE, 38);
        final UnifiedRecordValue value = value(x, p);
        sends.add(() -> sender.sendCommand(target, valueType(kind), intent(kind), value));
      }
      out.appendPostCommitTask(() -> {
        sends.forEach(Runnable::run);
        return true;
      });
    }
  }

  static ValueType valueType(final byte kind) {
    return kind == ZbHip.CMD_MSG_SUB_CREATE || kind == ZbHip.CMD_MSG_SUB_CORRELATE || kind == ZbHip.CMD_MSG_SUB_DELETE
        ? ValueType.MESSAGE_SUBSCRIPTION : ValueType.PROCESS_MESSAGE_SUBSCRIPTION;
  }

  static Intent intent(final byte kind) {
    return switch (kind) {
      case ZbHip.CMD_MSG_SUB_CREATE -> MessageSubscriptionIntent.CREATE;
      case ZbHip.CMD_MSG_SUB_CORRELATE -> MessageSubscriptionIntent.CORRELATE;
      case ZbHip.CMD_PMS_CREATE -> ProcessMessageSubscriptionIntent.CREATE;
      case ZbHip.CMD_MSG_SUB_DELETE -> MessageSubscriptionIntent.DELETE;
      case ZbHip.CMD_PMS_DELETE -> ProcessMessageSubscriptionIntent.DELETE;
      default -> ProcessMessageSubscriptionIntent.CORRELATE;
    };
  }

  /**
   * The value of a sent command exactly as the SubscriptionCommandSender method that sends it sets it
   * (:54-218); properties it does not set keep their declared defaults.
   */
  static UnifiedRecordValue value(final MemorySegment x, final GpuBatchProcessor p) {
    final long eik = x.get(JAVA_LONG, 0), pik = x.get(JAVA_LONG, 8), messageKey = x.get(JAVA_LONG, 16);
    final int corrId = x.get(JAVA_INT, 24);
    final DirectBuffer name = buf(p.name(x.get(JAVA_SHORT, 34) & 0xFFFF));
    final int bpmnId = x.get(JAVA_SHORT, 36) & 0xFFFF;
    final DirectBuffer bpmn = bpmnId == 0xFFFF ? buf("") : buf(p.name(bpmnId));
    final DirectBuffer corr = new UnsafeBuffer(corrId == NO_STRING ? new byte[0] : p.stringValue(corrId));
    final boolean interrupting = x.get(JAVA_BYTE, 39) != 0;
    final int sender = x.get(JAVA_SHORT, 40);
    switch (x.get(JAVA_BYTE, 38)) {
      case ZbHip.CMD_MSG_SUB_CREATE: // openMessageSubscription
        return new MessageSubscriptionRecord().setProcessInstanceKey(pik).setElementInstanceKey(eik)
            .setBpmnProcessId(bpmn).setMessageKey(-1).setMessageName(name).setCorrelationKey(corr)
            .setInterrupting(interrupting).setTenantId(TENANT);
      case ZbHip.CMD_MSG_SUB_CORRELATE: // correlateMessageSubscription
        return new MessageSubscriptionRecord().setProcessInstanceKey(pik).setElementInstanceKey(eik)
            .setBpmnProcessId(bpmn).setMessageKey(-1).setMessageName(name).setTenantId(TENANT);
      case ZbHip.CMD_MSG_SUB_DELETE: // closeMessageSubscription (:220-236)
        return new MessageSubscriptionRecord().setProcessInstanceKey(pik).setElementInstanceKey(eik)
            .setMessageKey(-1).setMessageName(name).setTenantId(TENANT);
      case ZbHip.CMD_PMS_DELETE: // closeProcessMessageSubscription (:267-283)
        return new ProcessMessageSubscriptionRecord().setSubscriptionPartitionId(sender).setProcessInstanceKey(pik)
            .setElementInstanceKey(eik).setMessageKey(-1).setMessageName(name).setTenantId(TENANT);
      case ZbHip.CMD_PMS_CREATE: // openProcessMessageSubscription
        return new ProcessMessageSubscriptionRecord().setSubscriptionPartitionId(sender).setProcessInstanceKey(pik)
            .setElementInstanceKey(eik).setMessageKey(-1).setMessageName(name).setInterrupting(interrupting)
            .setTenantId(TENANT);
      default: // correlateProcessMessageSubscription (the subset's messages carry no variables)
        return new ProcessMessageSubscriptionRecord().setSubscriptionPartitionId(sender).setProcessInstanceKey(pik)
            .setElementInstanceKey(eik).setBpmnProcessId(bpmn).setMessageKey(messageKey).setMessageName(name)
            .setCorrelationKey(corr).setTenantId(TENANT);
    }
  }

  private static DirectBuffer buf(final String s) {
    return new UnsafeBuffer(s.getBytes(StandardCharsets.UTF_8));
  }

  private static byte[] bytes(final DirectBuffer b) {
    final byte[] out = new byte[b.capacity()];
    b.getBytes(0, out);
    return out;
  }
}
