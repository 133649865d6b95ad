/*
 * The engine's JobStreamer behind the adapter (engine/.../processing/streamprocessor/JobStreamer.java:28-73;
 * BpmnJobActivationBehavior.publishWork :61-100).  The reference asks the streamer for every job it makes
 * activatable; the device decides per job type inside the step kernel, so before each window (and before
 * a time-out or failure of a device job) the adapter mirrors the streamer's current stream per device job
 * type into zbhip_set_job_stream.  The push side effect of every JOB_BATCH:ACTIVATED the device wrote is
 * the stream's push(ActivatedJob) after the commit, with the job's variables collected when the record is
 * appended (zbhip_job_variables over the stream's fetchVariables).  Not compiled in this image (no JDK).
 */
package io.camunda.zeebe.zbhip;

import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

import io.camunda.zeebe.engine.processing.streamprocessor.JobStreamer;
import io.camunda.zeebe.engine.processing.streamprocessor.JobStreamer.JobStream;
import io.camunda.zeebe.protocol.impl.record.value.job.JobBatchRecord;
import io.camunda.zeebe.protocol.impl.record.value.job.JobRecord;
import io.camunda.zeebe.protocol.impl.stream.job.ActivatedJobImpl;
import io.camunda.zeebe.stream.api.ProcessingResultBuilder;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.nio.charset.StandardCharsets;
import java.util.Collection;
import java.util.HashMap;
import java.util.Map;
import java.util.Optional;
import org.agrona.DirectBuffer;
import org.agrona.concurrent.UnsafeBuffer;

final class JobStreams {
  private static final String TENANT = "<default>";
  private static final int JOB_BYTES = 144; // zbhip_activated_job

  private final JobStreamer streamer;
  private final Map<String, JobStream> onDevice = new HashMap<>(); // device job type -> the stream set

  JobStreams(final JobStreamer streamer) {
    this.streamer = streamer == null ? JobStreamer.noop() : streamer;
  }

  /** zbhip_set_job_stream for every device job type whose stream opened, changed or closed. */
  void sync(final MemorySegment handle, final Collection<String> deviceJobTypes) {
    for (final String type : deviceJobTypes) {
      final DirectBuffer typeBuffer = new UnsafeBuffer(type.getBytes(StandardCharsets.UTF_8));
      final Optional<JobStream> stream = streamer.streamFor(typeBuffer, p -> p.tenantIds().contains(TENANT));
      final JobStream prev = onDevice.get(type);
      if (stream.isPresent() && stream.get() != prev) {
        final var props = stream.get().properties();
        final byte[] worker = new byte[props.worker().capacity()];
        props.worker().getBytes(0, worker);
        ZbHip.setJobStream(handle, type.getBytes(StandardCharsets.UTF_8), worker, props.timeout(), true);
        onDevice.put(type, stream.get());
      } else if (stream.isEmpty() && prev != null) {
        ZbHip.setJobStream(handle, type.getBytes(StandardCharsets.UTF_8), new byte[0], 0, false);
        onDevice.remove(type);
      }
    }
  }

  /**
   * publishWork without a stream for the job's type: notifyJobAvailable's side effect, post-commit
   * (BpmnJobActivationBehavior.java:97-111) -- long-polling workers of that type are woken.
   */
  void notifyAvailable(final ProcessingResultBuilder out, final String type) {
    out.appendPostCommitTask(() -> {
      streamer.notifyWorkAvailable(type);
      return true;
    });
  }

  /** Whether a device job type has a stream now (the device pushes its jobs). */
  boolean pushing() {
    return !onDevice.isEmpty();
  }

  /** The stream's timeout of a push record's JobBatchRecord (createJobBatchRecord :122-131). */
  long timeout(final String type) {
    final JobStream s = onDevice.get(type);
    return s == null ? -1 : s.properties().timeout();
  }

  /**
   * The push side effect of one JOB_BATCH:ACTIVATED the device wrote: the job's variables now, the
   * stream's push after the commit (publishWork :83-97).
   */
  void push(final ProcessingResultBuilder out, final MemorySegment handle, final JobBatchRecord batch,
      final GpuBatchProcessor p) {
    final JobRecord job = batch.jobs().iterator().next();
    final long jobKey = batch.jobKeys().iterator().next().getValue();
    final JobStream stream = onDevice.get(job.getType());
    if (stream == null) {
      return;
    }
    try (Arena a = Arena.ofConfined()) {
      final var fetch = stream.properties().fetchVariables();
      final int[] ids = new int[fetch.size()];
      int k = 0;
      for (final DirectBuffer name : fetch) {
        ids[k++] = p.internName(name.getStringWithoutLengthUtf8(0, name.capacity()));
      }
      final MemorySegment keys = a.allocate(JAVA_LONG, 1);
      keys.set(JAVA_LONG, 0, jobKey);
      final MemorySegment row = a.allocate(JOB_BYTES, 8);
      ZbHip.jobVariables(handle, keys, 1, k == 0 ? MemorySegment.NULL : a.allocateArray(JAVA_INT, ids), k, row);
      final JobRecord pushable = new JobRecord();
      pushable.wrap(job); // (a copy: the batch record is reused by the platform)
      pushable.setVariables(JobActivation.variables(row, p));
      final var activated = new ActivatedJobImpl().setJobKey(jobKey).setRecord(pushable);
      out.appendPostCommitTask(() -> {
        stream.push(activated);
        return true;
      });
    }
  }
}
