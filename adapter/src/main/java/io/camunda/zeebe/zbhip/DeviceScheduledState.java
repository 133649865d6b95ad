/*
 * The state the engine's scheduled tasks read, with the device's part added (INTEGRATION.md §8).
 *
 * The reference's checkers scan RocksDB, which does not hold the instances HBM holds:
 *   DueDateTimerChecker            engine/.../processing/timer/DueDateTimerChecker.java:30-38,86-129
 *   JobTimeoutTrigger              engine/.../processing/job/JobTimeoutTrigger.java:30-33,74-87
 *   PendingProcessMessageSubscriptionChecker  engine/.../processing/message/
 *                                  PendingProcessMessageSubscriptionChecker.java:30-37,78-128
 *   MessageObserver -> PendingMessageSubscriptionChecker  MessageObserver.java:28-42,61-73
 * EngineProcessors builds each of them over a state interface; the maintainer passes these wrappers
 * instead (GpuBatchProcessor.timerState(...) etc.), so the unchanged checkers see one merged state:
 *   - timers: the engine's TIMER_DUE_DATES and the device's due timers (zbhip_due_timers, a device
 *     scan) merged in [dueDate, elementInstanceKey, timerKey] order
 *     (DbTimerInstanceState.processTimersWithDueDateBefore, :87-116);
 *   - jobs: the engine's JOB_DEADLINES and the device's activated jobs (zbhip_timed_out_jobs) merged in
 *     [deadline, jobKey] order (DbJobState.forEachTimedOutEntry, :286-298);
 *   - pending subscriptions: the engine's transient states, then the device's (kept by Messages from
 *     the device's records, as the appliers keep the engine's).
 * While a window is only partly emitted the device is ahead of the log; the device part then answers
 * nothing and the timer view asks for a run one timer resolution later (what actor scheduling allows).
 * The Python mirror is zeebe_amd/adapter.py (DeviceTimerInstanceState, DeviceJobState,
 * DevicePendingSubscriptionState); tests/test_gpu_scheduled.py runs the restated checkers over it.
 *
 * Not compiled in this image (no JDK); written against
 *   TimerInstanceState, JobState, PendingProcessMessageSubscriptionState,
 *   PendingMessageSubscriptionState   engine/.../state/immutable/*.java
 *   TimerInstance                     engine/.../state/instance/TimerInstance.java
 */
package io.camunda.zeebe.zbhip;

import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

import io.camunda.zeebe.engine.state.immutable.JobState;
import io.camunda.zeebe.engine.state.immutable.PendingMessageSubscriptionState;
import io.camunda.zeebe.engine.state.immutable.PendingProcessMessageSubscriptionState;
import io.camunda.zeebe.engine.state.immutable.TimerInstanceState;
import io.camunda.zeebe.engine.state.instance.TimerInstance;
import io.camunda.zeebe.engine.state.message.MessageSubscription;
import io.camunda.zeebe.engine.state.message.ProcessMessageSubscription;
import io.camunda.zeebe.engine.state.message.TransientPendingSubscriptionState;
import io.camunda.zeebe.protocol.impl.record.value.job.JobRecord;
import io.camunda.zeebe.protocol.impl.record.value.message.ProcessMessageSubscriptionRecord;
import io.camunda.zeebe.protocol.impl.record.value.timer.TimerRecord;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.Comparator;
import java.util.List;
import java.util.Map;
import java.util.function.BiPredicate;
import java.util.function.Consumer;
import org.agrona.DirectBuffer;
import org.agrona.concurrent.UnsafeBuffer;

final class DeviceScheduledState {

  private static final int CAP = 1 << 16; // rows per scan (the rest comes with the next run)

  private DeviceScheduledState() {}

  /** TimerInstanceState over the engine's timers and the device's. */
  static final class Timers implements TimerInstanceState {
    private final GpuBatchProcessor gpu;
    private final TimerInstanceState engine;

    Timers(final GpuBatchProcessor gpu, final TimerInstanceState engine) {
      this.gpu = gpu;
      this.engine = engine;
    }

    @Override
    public long processTimersWithDueDateBefore(final long timestamp, final TimerVisitor consumer) {
      if (!gpu.scheduledReady()) {
        return timestamp; // mid-window: DueDateChecker runs again after TIMER_RESOLUTION
      }
      final List<TimerInstance> due = new ArrayList<>();
      final long engineNext = engine.processTimersWithDueDateBefore(timestamp, t -> {
        final TimerInstance copy = new TimerInstance();
        copy.copyFrom(t);
        due.add(copy);
        return true;
      });
      final long[] deviceNext = {-1};
      TimerInstance last = null;
      try (Arena a = Arena.ofConfined()) {
        final MemorySegment out = a.allocate(ZbHip.RECORD.byteSize() * CAP, 16);
        final long n = ZbHip.dueTimers(gpu.handle(), timestamp, out, CAP, deviceNext);
        for (long r = 0; r < n; r++) {
          last = timerInstance(out.asSlice(ZbHip.RECORD.byteSize() * r, ZbHip.RECORD.byteSize()));
          due.add(last);
        }
      }
      // TIMER_DUE_DATES order: [dueDate, [elementInstanceKey, timerKey]]
      final Comparator<TimerInstance> order = Comparator.comparingLong(TimerInstance::getDueDate)
          .thenComparingLong(TimerInstance::getElementInstanceKey).thenComparingLong(TimerInstance::getKey);
      due.sort(order);
      // a truncated device scan (due rows left out): the first row left out may precede engine timers
      // ordered after the last row returned, so the visit stops there and the checker runs again at the
      // date returned (processTimersWithDueDateBefore stops at any timer its visitor refuses, :87-116)
      final TimerInstance bound = last != null && deviceNext[0] >= 0 && deviceNext[0] <= timestamp ? last : null;
      for (final TimerInstance t : due) {
        if (bound != null && order.compare(t, bound) > 0) {
          return Math.min(t.getDueDate(), deviceNext[0]);
        }
        if (!consumer.visit(t)) {
          return t.getDueDate();
        }
      }
      final long e = engineNext, d = deviceNext[0];
      return e < 0 ? d : d < 0 ? e : Math.min(e, d);
    }

    /** A TIMER:TRIGGER row of zbhip_due_timers as the TimerInstance the visitor writes it from. */
    private TimerInstance timerInstance(final MemorySegment r) {
      final ZbHip.Deployed d = gpu.process(r.get(JAVA_INT, ZbHip.Rec.PROCESS_IDX));
      final TimerInstance t = new TimerInstance();
      t.setKey(r.get(JAVA_LONG, ZbHip.Rec.KEY));
      t.setElementInstanceKey(r.get(JAVA_LONG, ZbHip.Rec.SCOPE_KEY));
      t.setProcessInstanceKey(r.get(JAVA_LONG, ZbHip.Rec.PROCESS_INSTANCE_KEY));
      t.setDueDate(r.get(JAVA_LONG, ZbHip.Rec.AUX));
      t.setHandlerNodeId(new UnsafeBuffer(d.elementIds()[r.get(JAVA_INT, ZbHip.Rec.ELEMENT_IDX)].getBytes()));
      t.setRepetitions(r.get(JAVA_INT, ZbHip.Rec.PARTITION)); // zbhip_due_timers: repetitions in partition
      t.setProcessDefinitionKey(d.definitionKey());
      t.setTenantId(TimerRecord.DEFAULT_TENANT_ID);
      return t;
    }

    @Override
    public void forEachTimerForElementInstance(final long elementInstanceKey, final Consumer<TimerInstance> action) {
      engine.forEachTimerForElementInstance(elementInstanceKey, action);
    }

    @Override
    public TimerInstance get(final long elementInstanceKey, final long timerKey) {
      return engine.get(elementInstanceKey, timerKey);
    }
  }

  /** JobState whose time-out scan covers the device's activated jobs too. */
  static final class Jobs implements JobState {
    private final GpuBatchProcessor gpu;
    private final JobState engine;

    Jobs(final GpuBatchProcessor gpu, final JobState engine) {
      this.gpu = gpu;
      this.engine = engine;
    }

    private record Due(long deadline, long key, JobRecord job) {}

    @Override
    public void forEachTimedOutEntry(final long upperBound, final BiPredicate<Long, JobRecord> callback) {
      final List<Due> due = new ArrayList<>();
      engine.forEachTimedOutEntry(upperBound, (key, job) -> {
        final JobRecord copy = new JobRecord();
        copy.wrap(job);
        due.add(new Due(copy.getDeadline(), key, copy));
        return true;
      });
      Due last = null;
      final long[] deviceNext = {-1};
      if (gpu.scheduledReady()) {
        try (Arena a = Arena.ofConfined()) {
          final MemorySegment out = a.allocate(ZbHip.RECORD.byteSize() * CAP, 16);
          final long n = ZbHip.timedOutJobs(gpu.handle(), upperBound, out, CAP, deviceNext);
          for (long r = 0; r < n; r++) {
            final MemorySegment row = out.asSlice(ZbHip.RECORD.byteSize() * r, ZbHip.RECORD.byteSize());
            last = new Due(row.get(JAVA_LONG, ZbHip.Rec.MESSAGE_KEY), row.get(JAVA_LONG, ZbHip.Rec.KEY), gpu.storedJob(row));
            due.add(last);
          }
        }
      }
      final Comparator<Due> order = Comparator.comparingLong(Due::deadline).thenComparingLong(Due::key);
      due.sort(order); // [deadline, jobKey]
      // a truncated device list: engine entries past its last row wait for the trigger's next run
      final Due bound = last != null && deviceNext[0] >= 0 ? last : null;
      for (final Due d : due) {
        if (bound != null && order.compare(d, bound) > 0) {
          return;
        }
        if (!callback.test(d.key(), d.job())) {
          return;
        }
      }
    }

    @Override
    public boolean exists(final long jobKey) {
      return engine.exists(jobKey);
    }

    @Override
    public State getState(final long key) {
      return engine.getState(key);
    }

    @Override
    public boolean isInState(final long key, final State state) {
      return engine.isInState(key, state);
    }

    @Override
    public void forEachActivatableJobs(final DirectBuffer type, final List<String> tenantIds,
        final BiPredicate<Long, JobRecord> callback) {
      engine.forEachActivatableJobs(type, tenantIds, callback);
    }

    @Override
    public JobRecord getJob(final long key) {
      return engine.getJob(key);
    }

    @Override
    public JobRecord getJob(final long key, final Map<String, Object> authorizations) {
      return engine.getJob(key, authorizations);
    }

    @Override
    public long findBackedOffJobs(final long timestamp, final BiPredicate<Long, JobRecord> callback) {
      return engine.findBackedOffJobs(timestamp, callback);
    }
  }

  /** PendingProcessMessageSubscriptionState: the engine's pending subscriptions, then the device's. */
  static final class PendingProcessSubscriptions implements PendingProcessMessageSubscriptionState {
    private final GpuBatchProcessor gpu;
    private final PendingProcessMessageSubscriptionState engine;
    private final TransientPendingSubscriptionState engineTransient;

    PendingProcessSubscriptions(final GpuBatchProcessor gpu, final PendingProcessMessageSubscriptionState engine,
        final TransientPendingSubscriptionState engineTransient) {
      this.gpu = gpu;
      this.engine = engine;
      this.engineTransient = engineTransient;
    }

    @Override
    public void visitPending(final long deadline, final ProcessMessageSubscriptionVisitor visitor) {
      // subscriptions of handed-off instances: pending in the engine's state now
      for (final var e : gpu.messages().movedPending) {
        engineTransient.add(new TransientPendingSubscriptionState.PendingSubscription(
            e.getKey().elementInstanceKey(), e.getKey().messageName(), e.getValue().record.getTenantId()),
            e.getValue().sentTime);
      }
      gpu.messages().movedPending.clear();
      engine.visitPending(deadline, visitor);
      if (!gpu.scheduledReady()) {
        return;
      }
      final List<Messages.PendingProcessSubscription> due = new ArrayList<>();
      for (final var e : gpu.messages().pendingProcess.values()) {
        if (e.sentTime < deadline) {
          due.add(e);
        }
      }
      due.sort(Comparator.comparingLong(e -> e.sentTime)); // stable: ties keep insertion order
      for (final var e : due) {
        final ProcessMessageSubscription s = new ProcessMessageSubscription();
        s.setRecord(e.record);
        if (e.opening) {
          s.setOpening();
        } else {
          s.setClosing();
        }
        visitor.visit(s);
      }
    }

    @Override
    public void onSent(final ProcessMessageSubscriptionRecord record, final long timestampMs) {
      engine.onSent(record, timestampMs);
      final var e = gpu.messages().pendingProcess.get(
          new Messages.SubscriptionKey(record.getElementInstanceKey(), record.getMessageName()));
      if (e != null) {
        e.sentTime = timestampMs;
      }
    }
  }

  /** PendingMessageSubscriptionState: the engine's correlating subscriptions, then the device's. */
  static final class PendingMessageSubscriptions implements PendingMessageSubscriptionState {
    private final GpuBatchProcessor gpu;
    private final PendingMessageSubscriptionState engine;
    private final TransientPendingSubscriptionState engineTransient;

    PendingMessageSubscriptions(final GpuBatchProcessor gpu, final PendingMessageSubscriptionState engine,
        final TransientPendingSubscriptionState engineTransient) {
      this.gpu = gpu;
      this.engine = engine;
      this.engineTransient = engineTransient;
    }

    @Override
    public void visitPending(final long deadline, final MessageSubscriptionVisitor visitor) {
      // subscriptions moved with their correlation key (Messages.toEngine): pending in the engine's state now
      for (final var e : gpu.messages().movedPendingMessage) {
        engineTransient.add(new TransientPendingSubscriptionState.PendingSubscription(
            e.getKey().elementInstanceKey(), e.getKey().messageName(), e.getValue().record.getTenantId()),
            e.getValue().sentTime);
      }
      gpu.messages().movedPendingMessage.clear();
      engine.visitPending(deadline, visitor);
      if (!gpu.scheduledReady()) {
        return;
      }
      final List<Messages.PendingSubscription> due = new ArrayList<>();
      for (final var e : gpu.messages().pendingMessage.values()) {
        if (e.sentTime < deadline) {
          due.add(e);
        }
      }
      due.sort(Comparator.comparingLong(e -> e.sentTime));
      for (final var e : due) {
        final MessageSubscription s = new MessageSubscription();
        s.setRecord(e.record);
        s.setCorrelating(true);
        visitor.visit(s);
      }
    }

    @Override
    public void onSent(final long elementInstanceKey, final String messageName, final String tenantId,
        final long timestampMs) {
      engine.onSent(elementInstanceKey, messageName, tenantId, timestampMs);
      final var e = gpu.messages().pendingMessage.get(new Messages.SubscriptionKey(elementInstanceKey, messageName));
      if (e != null) {
        e.sentTime = timestampMs;
      }
    }
  }
}
