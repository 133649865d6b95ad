/*
 * JOB_BATCH:ACTIVATE on the device (JobBatchActivateProcessor.java:60-143): the zbhip_job_activation
 * command, room for the activated jobs, and the JOB_BATCH:ACTIVATED event (or the INVALID_ARGUMENT
 * rejection) the adapter appends -- JobBatchRecord with jobKeys and jobs (JobRecord with deadline,
 * worker and the collected variables, JobBatchCollector.java:67-123).  Struct layouts: include/zbhip.h
 * (zbhip_job_activation 72 B, zbhip_job_batch 16 B, zbhip_activated_job 144 B).  Not compiled in this
 * image (no JDK).
 */
package io.camunda.zeebe.zbhip;

import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

import io.camunda.zeebe.msgpack.spec.MsgPackWriter;
import io.camunda.zeebe.protocol.impl.record.RecordMetadata;
import io.camunda.zeebe.protocol.impl.record.value.job.JobBatchRecord;
import io.camunda.zeebe.protocol.impl.record.value.job.JobRecord;
import io.camunda.zeebe.protocol.record.RecordType;
import io.camunda.zeebe.protocol.record.RejectionType;
import io.camunda.zeebe.protocol.record.ValueType;
import io.camunda.zeebe.protocol.record.intent.JobBatchIntent;
import io.camunda.zeebe.stream.api.ProcessingResultBuilder;
import io.camunda.zeebe.stream.api.records.TypedRecord;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.nio.charset.StandardCharsets;
import org.agrona.ExpandableArrayBuffer;
import org.agrona.concurrent.UnsafeBuffer;

record JobActivation(MemorySegment command, MemorySegment jobs, long capacity, MemorySegment result, JobBatchRecord batch) {
  private static final byte DOC_NIL = 0, DOC_BOOL = 1, DOC_INT = 2, DOC_DEC = 3, DOC_STR = 5;
  private static final int JOB_BYTES = 144;

  static JobActivation of(final Arena arena, final JobBatchRecord batch, final long timestamp, final GpuBatchProcessor p) {
    final byte[] type = batch.getType().getBytes(StandardCharsets.UTF_8);
    final byte[] worker = batch.getWorker().getBytes(StandardCharsets.UTF_8);
    final MemorySegment cmd = arena.allocate(72, 8);
    cmd.set(java.lang.foreign.ValueLayout.ADDRESS, 0, arena.allocateArray(JAVA_BYTE, type));
    cmd.set(JAVA_LONG, 8, type.length);
    cmd.set(java.lang.foreign.ValueLayout.ADDRESS, 16, arena.allocateArray(JAVA_BYTE, worker));
    cmd.set(JAVA_LONG, 24, worker.length);
    cmd.set(JAVA_LONG, 32, batch.getTimeout());
    cmd.set(JAVA_INT, 40, batch.getMaxJobsToActivate());
    cmd.set(JAVA_INT, 44, 0);
    cmd.set(JAVA_LONG, 48, timestamp); // deadline = the command's timestamp + timeout
    final var names = batch.variables();
    final int[] ids = new int[names.size()];
    int k = 0;
    for (final var v : names) {
      final var b = v.getValue();
      ids[k++] = p.internName(b.getStringWithoutLengthUtf8(0, b.capacity()));
    }
    cmd.set(java.lang.foreign.ValueLayout.ADDRESS, 56, k == 0 ? MemorySegment.NULL : arena.allocateArray(JAVA_INT, ids));
    cmd.set(JAVA_LONG, 64, k);
    final long cap = Math.max(1, batch.getMaxJobsToActivate());
    return new JobActivation(cmd, arena.allocate(JOB_BYTES * cap, 8), cap, arena.allocate(16, 8), batch);
  }

  long key() {
    return result.get(JAVA_LONG, 0);
  }

  /** The JOB_BATCH:ACTIVATED event with the activated jobs, or the command's rejection. */
  void emit(final TypedRecord command, final ProcessingResultBuilder out, final GpuBatchProcessor p) {
    final RecordMetadata meta = new RecordMetadata().valueType(ValueType.JOB_BATCH);
    if (key() < 0) {
      final int reason = result.get(JAVA_BYTE, 13);
      meta.recordType(RecordType.COMMAND_REJECTION).intent(JobBatchIntent.ACTIVATE)
          .rejectionType(RejectionType.INVALID_ARGUMENT).rejectionReason(rejection(batch, reason));
      out.appendRecord(command.getKey(), batch, meta);
      return;
    }
    for (final var e : activated(p).entrySet()) {
      batch.jobKeys().add().setValue(e.getKey());
      batch.jobs().add().wrap(e.getValue());
    }
    batch.setTruncated(truncated());
    meta.recordType(RecordType.EVENT).intent(JobBatchIntent.ACTIVATED);
    out.appendRecord(key(), batch, meta);
  }

  boolean truncated() {
    return result.get(JAVA_BYTE, 14) != 0;
  }

  /** The activated device jobs in key order: job key -> JobRecord (JobBatchCollector's jobs). */
  java.util.LinkedHashMap<Long, JobRecord> activated(final GpuBatchProcessor p) {
    final java.util.LinkedHashMap<Long, JobRecord> out = new java.util.LinkedHashMap<>();
    final int n = result.get(JAVA_INT, 8);
    for (int i = 0; i < n; i++) {
      final MemorySegment j = jobs.asSlice((long) JOB_BYTES * i, JOB_BYTES);
      final ZbHip.Deployed d = p.process(j.get(JAVA_INT, 36));
      final int elem = j.get(JAVA_INT, 40);
      final JobRecord job = new JobRecord();
      job.setType(batch.getType())
          .setWorker(batch.getWorker())
          .setDeadline(j.get(JAVA_LONG, 24))
          .setRetries(j.get(JAVA_SHORT, 44) & 0xFFFF)
          .setElementId(d.elementIds()[elem])
          .setElementInstanceKey(j.get(JAVA_LONG, 8))
          .setProcessInstanceKey(j.get(JAVA_LONG, 16))
          .setBpmnProcessId(d.bpmnProcessId())
          .setProcessDefinitionKey(d.definitionKey())
          .setProcessDefinitionVersion(d.version())
          .setVariables(variables(j, p))
          .setTenantId("<default>");
      out.put(j.get(JAVA_LONG, 0), job);
    }
    return out;
  }

  /** The job's collected variables (zbhip_doc_entry rows) as a msgpack document. */
  static UnsafeBuffer variables(final MemorySegment job, final GpuBatchProcessor p) {
    final int n = job.get(JAVA_SHORT, 46) & 0xFFFF;
    final ExpandableArrayBuffer buf = new ExpandableArrayBuffer();
    final MsgPackWriter w = new MsgPackWriter().wrap(buf, 0);
    w.writeMapHeader(n);
    for (int v = 0; v < n; v++) {
      final long o = 48L + 16L * v;
      w.writeString(new UnsafeBuffer(p.name(job.get(JAVA_INT, o)).getBytes(StandardCharsets.UTF_8)));
      final long value = job.get(JAVA_LONG, o + 8);
      switch (job.get(JAVA_BYTE, o + 4)) {
        case DOC_BOOL -> w.writeBoolean(value != 0);
        case DOC_INT -> w.writeInteger(value);
        case DOC_DEC -> w.writeFloat(value / 1_000_000d);
        case DOC_STR -> w.writeString(new UnsafeBuffer(p.stringValue(value)));
        default -> w.writeNil();
      }
    }
    return new UnsafeBuffer(buf, 0, w.getOffset());
  }

  /** JobBatchActivateProcessor.rejectCommand (:91-118) texts, as zbhip_job_batch_rejection_reason. */
  private static String rejection(final JobBatchRecord batch, final int reason) {
    final String f = "Expected to activate job batch with %s to be %s, but it was %s";
    return switch (reason) {
      case 1 -> String.format(f, "max jobs to activate", "greater than zero", "'" + batch.getMaxJobsToActivate() + "'");
      case 2 -> String.format(f, "timeout", "greater than zero", "'" + batch.getTimeout() + "'");
      case 3 -> String.format(f, "type", "present", "blank");
      default -> "";
    };
  }
}
