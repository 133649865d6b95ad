/*
 * One read-ahead window of the adapter: the zbhip_command rows and variable-document entries of
 * consecutive hot-path commands, their log positions, and after zbhip_run the drained records
 * (zbhip_record, ordered by source command then ordinal) rebuilt into the reference's record values
 * and metadata for ProcessingResultBuilder.appendRecord (ProcessingResultBuilder.java:30-54).
 *
 * Not compiled in this image (no JDK).  Record values follow ProcessInstanceRecord.java:61-72,
 * JobRecord.java, VariableRecord.java, ProcessEventRecord.java and
 * ProcessInstanceCreationRecord.java; the document entries follow the msgpack value mapping of
 * include/zbhip.h (int64, 6-digit scaled decimals, booleans, nil, value-dictionary strings).
 */
package io.camunda.zeebe.zbhip;

import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

import io.camunda.zeebe.msgpack.spec.MsgPackReader;
import io.camunda.zeebe.msgpack.spec.MsgPackToken;
import io.camunda.zeebe.msgpack.spec.MsgPackWriter;
import org.agrona.ExpandableArrayBuffer;
import io.camunda.zeebe.protocol.impl.record.RecordMetadata;
import io.camunda.zeebe.protocol.impl.record.UnifiedRecordValue;
import io.camunda.zeebe.protocol.impl.record.value.incident.IncidentRecord;
import io.camunda.zeebe.protocol.impl.record.value.job.JobBatchRecord;
import io.camunda.zeebe.protocol.impl.record.value.job.JobRecord;
import io.camunda.zeebe.protocol.impl.record.value.message.MessageRecord;
import io.camunda.zeebe.protocol.impl.record.value.message.MessageSubscriptionRecord;
import io.camunda.zeebe.protocol.impl.record.value.message.ProcessMessageSubscriptionRecord;
import io.camunda.zeebe.protocol.impl.record.value.processinstance.ProcessEventRecord;
import io.camunda.zeebe.protocol.impl.record.value.processinstance.ProcessInstanceCreationRecord;
import io.camunda.zeebe.protocol.impl.record.value.processinstance.ProcessInstanceBatchRecord;
import io.camunda.zeebe.protocol.impl.record.value.processinstance.ProcessInstanceRecord;
import io.camunda.zeebe.protocol.impl.record.value.timer.TimerRecord;
import io.camunda.zeebe.protocol.impl.record.value.variable.VariableRecord;
import io.camunda.zeebe.protocol.record.RecordType;
import io.camunda.zeebe.protocol.record.RejectionType;
import io.camunda.zeebe.protocol.record.ValueType;
import io.camunda.zeebe.protocol.record.intent.Intent;
import io.camunda.zeebe.protocol.record.intent.JobIntent;
import io.camunda.zeebe.protocol.record.intent.MessageSubscriptionIntent;
import io.camunda.zeebe.protocol.record.intent.ProcessEventIntent;
import io.camunda.zeebe.protocol.record.intent.ProcessInstanceCreationIntent;
import io.camunda.zeebe.protocol.record.intent.ProcessInstanceIntent;
import io.camunda.zeebe.protocol.record.intent.VariableIntent;
import io.camunda.zeebe.protocol.record.intent.TimerIntent;
import io.camunda.zeebe.protocol.record.value.BpmnElementType;
import io.camunda.zeebe.protocol.record.value.BpmnEventType;
import io.camunda.zeebe.protocol.record.value.ErrorType;
import io.camunda.zeebe.logstreams.log.LoggedEvent;
import io.camunda.zeebe.stream.api.ProcessingResultBuilder;
import io.camunda.zeebe.stream.api.records.TypedRecord;
import io.camunda.zeebe.stream.impl.records.RecordValues;
import io.camunda.zeebe.stream.impl.records.TypedRecordImpl;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.BitSet;
import java.util.List;
import org.agrona.DirectBuffer;
import org.agrona.concurrent.UnsafeBuffer;

final class Window {

  private static final String TENANT = "<default>"; // TenantOwned.DEFAULT_TENANT_IDENTIFIER
  private static final byte DOC_NIL = 0, DOC_BOOL = 1, DOC_INT = 2, DOC_DEC = 3, DOC_STR = 5; // zbhip_doc_type
  private static final int MAX = 1 << 16;
  private static final int MAX_DOCS = 16 * MAX;

  private MemorySegment handle;
  private MemorySegment cmds;
  private MemorySegment docs;
  private MemorySegment keyOffsets; // a document's key byte offsets (zbhip_doc_merge_order)
  private MemorySegment xparts; // received cross-partition commands of the window (config 5)
  private int nXparts;
  private Arena arena;
  private MemorySegment recs;
  private long recCap;
  private int n;
  private int nDocs;
  private long sourceBase; // zbhip_record.source_index of this window's first command (submission order)
  private final long[] positions = new long[MAX];
  private final int[] instances = new int[MAX];
  private final BitSet addressed = new BitSet(); // instance slots the window's commands address
  private static final RecordValues RECORD_VALUES = new RecordValues();
  // the command's msgpack variable document and each entry's msgpack value (VARIABLE records)
  private final DirectBuffer[] documents = new DirectBuffer[MAX];
  private final List<DirectBuffer> entryValues = new ArrayList<>();
  private final MsgPackReader msgpack = new MsgPackReader();

  void init(final Arena arena) {
    this.arena = arena;
    cmds = arena.allocate(ZbHip.COMMAND.byteSize() * MAX, 16);
    docs = arena.allocate(ZbHip.DOC_ENTRY.byteSize() * MAX_DOCS, 16);
    keyOffsets = arena.allocate(JAVA_INT.byteSize() * 256, 4);
    xparts = arena.allocate(ZbHip.XPART.byteSize() * MAX, 16);
  }

  /** Scratch for a read-ahead message command's xpart row (copied into the window by addMessageCommand). */
  Arena arena() {
    return arena;
  }

  void reset(final long firstPosition) {
    sourceBase += n;
    n = 0;
    addressed.clear();
    nDocs = 0;
    nXparts = 0;
    entryValues.clear();
    Arrays.fill(documents, null);
  }

  int size() {
    return n;
  }

  boolean covers(final long position) {
    return n > 0 && position >= positions[0] && position <= positions[n - 1];
  }

  int indexOf(final long position) {
    final int i = Arrays.binarySearch(positions, 0, n, position);
    return i >= 0 ? i : -1;
  }

  int instanceOf(final int i) {
    return instances[i];
  }

  boolean addresses(final int slot) {
    return addressed.get(slot);
  }

  /**
   * A log command read ahead, as the platform's TypedRecord: metadata copied, the value read into a
   * fresh object (RecordValues reuses its instances), so it stays valid while the reader moves on.
   */
  static TypedRecord typed(final LoggedEvent event, final RecordMetadata meta, final int partitionId) {
    final TypedRecordImpl r = new TypedRecordImpl(partitionId);
    final RecordMetadata copy = new RecordMetadata();
    copy.wrap(meta);
    final UnifiedRecordValue value =
        switch (meta.getValueType()) {
          case PROCESS_INSTANCE_CREATION -> new ProcessInstanceCreationRecord();
          case JOB -> new JobRecord();
          case TIMER -> new TimerRecord();
          case PROCESS_INSTANCE -> new ProcessInstanceRecord();
          case PROCESS_INSTANCE_BATCH -> new ProcessInstanceBatchRecord();
          default -> RECORD_VALUES.readRecordValue(event, meta.getValueType());
        };
    event.readValue(value);
    r.wrap(event, copy, value);
    return r;
  }

  /** PROCESS_INSTANCE_CREATION:CREATE -> ZBHIP_CMD_CREATE into instance slot {@code slot}. */
  boolean addCreate(
      final long position, final TypedRecord command, final int process, final int slot, final GpuBatchProcessor p) {
    final DirectBuffer variables = ((ProcessInstanceCreationRecord) command.getValue()).getVariablesBuffer();
    final int first = nDocs;
    final int count = decodeDocument(variables, p);
    if (count < 0) {
      return false;
    }
    put(position, command, slot, ZbHip.CMD_CREATE, count, process, first, variables);
    return true;
  }

  /** JOB:COMPLETE -> ZBHIP_CMD_JOB_COMPLETE; ref = zbhip_resolve_key's (slot << 16 | ordinal). */
  boolean addJobComplete(final long position, final TypedRecord command, final long ref, final GpuBatchProcessor p) {
    final DirectBuffer variables = ((JobRecord) command.getValue()).getVariablesBuffer();
    final int first = nDocs;
    final int count = decodeDocument(variables, p);
    if (count < 0) {
      return false;
    }
    put(position, command, (int) (ref >>> 16), ZbHip.CMD_JOB_COMPLETE, count, (int) (ref & 0xFFFF), first, variables);
    return true;
  }

  /**
   * TIMER:TRIGGER -> ZBHIP_CMD_TIMER_TRIGGER; ref = zbhip_resolve_key's (slot << 16 | ordinal) of the
   * timer key, the command's dueDate in doc_begin (low) and pad (high).
   */
  void addTimerTrigger(final long position, final TypedRecord command, final long ref, final long dueDate) {
    put(position, command, (int) (ref >>> 16), ZbHip.CMD_TIMER_TRIGGER, 0, (int) (ref & 0xFFFF), (int) dueDate, EMPTY);
    cmds.set(JAVA_INT, ZbHip.COMMAND.byteSize() * (n - 1) + 12, (int) (dueDate >>> 32)); // pad: dueDate high word
  }

  /**
   * A follow-up an earlier device batch wrote unprocessed, read back at its log position ->
   * ZBHIP_CMD_CONTINUE with its continuation id in doc_begin (low) and pad (high).
   */
  void addContinuation(final long position, final TypedRecord command, final int slot, final long id) {
    put(position, command, slot, ZbHip.CMD_CONTINUE, 0, 0, (int) id, EMPTY);
    cmds.set(JAVA_INT, ZbHip.COMMAND.byteSize() * (n - 1) + 12, (int) (id >>> 32));
  }

  /**
   * A message command (config 5, Messages.of): MESSAGE:PUBLISH -> ZBHIP_CMD_PUBLISH on its correlation
   * slot; a subscription command -> its xpart row appended to the window's, doc_begin = its index.
   */
  void addMessageCommand(final long position, final TypedRecord command, final Messages.DeviceCommand c) {
    int docBegin = 0;
    if (c.xpart() != null) {
      MemorySegment.copy(c.xpart(), 0, xparts, ZbHip.XPART.byteSize() * nXparts, ZbHip.XPART.byteSize());
      docBegin = nXparts++;
    }
    put(position, command, c.instance(), c.kind(), 0, c.ref(), docBegin, EMPTY);
  }

  private static final DirectBuffer EMPTY = new UnsafeBuffer(new byte[0]);

  private void put(
      final long position,
      final TypedRecord command,
      final int instance,
      final byte kind,
      final int docCount,
      final int ref,
      final int docBegin,
      final DirectBuffer variables) {
    final long o = ZbHip.COMMAND.byteSize() * n;
    cmds.set(JAVA_INT, o, instance);
    cmds.set(JAVA_BYTE, o + 4, kind);
    cmds.set(JAVA_BYTE, o + 5, (byte) docCount);
    cmds.set(JAVA_SHORT, o + 6, (short) ref);
    cmds.set(JAVA_INT, o + 8, docBegin);
    cmds.set(JAVA_INT, o + 12, 0);
    positions[n] = position;
    instances[n] = instance;
    addressed.set(instance);
    documents[n] = copy(variables, 0, variables.capacity());
    n++;
  }

  /**
   * The command's variable document as zbhip_doc_entry rows in document order, with the order
   * IndexedDocument (IndexedDocument.java:44-63) merges them in -- an agrona Int2IntHashMap over the keys'
   * byte offsets in these very bytes -- in their pad bytes (zbhip_doc_merge_order); -1 when an entry is
   * outside the device's value subset (the command stays on the CPU engine).
   */
  private int decodeDocument(final DirectBuffer doc, final GpuBatchProcessor p) {
    if (doc.capacity() == 0) {
      return 0;
    }
    msgpack.wrap(doc, 0, doc.capacity());
    final int size = msgpack.readMapHeader();
    if (size > 255 || nDocs + size > MAX_DOCS) {
      return -1;
    }
    final int first = nDocs;
    for (int e = 0; e < size; e++) {
      keyOffsets.setAtIndex(JAVA_INT, e, msgpack.getOffset());
      final MsgPackToken name = msgpack.readToken();
      final String nameStr = name.getValueBuffer().getStringWithoutLengthUtf8(0, name.getValueBuffer().capacity());
      final int valueStart = msgpack.getOffset();
      final MsgPackToken v = msgpack.readToken();
      final byte type;
      final long value;
      switch (v.getType()) {
        case NIL -> { type = DOC_NIL; value = 0; }
        case BOOLEAN -> { type = DOC_BOOL; value = v.getBooleanValue() ? 1 : 0; }
        case INTEGER -> { type = DOC_INT; value = v.getIntegerValue(); }
        case FLOAT -> {
          final double d = v.getFloatValue();
          final long scaled = Math.round(d * 1_000_000d);
          if ((double) scaled / 1_000_000d != d) {
            return -1; // not exactly a 6-digit decimal: FEEL over it is outside the subset
          }
          type = DOC_DEC;
          value = scaled;
        }
        case STRING -> {
          final DirectBuffer s = v.getValueBuffer();
          final byte[] b = new byte[s.capacity()];
          s.getBytes(0, b);
          type = DOC_STR;
          value = p.internString(b);
        }
        default -> { return -1; } // arrays, maps, binaries: outside the subset
      }
      final long o = ZbHip.DOC_ENTRY.byteSize() * nDocs;
      docs.set(JAVA_INT, o, p.internName(nameStr));
      docs.set(JAVA_BYTE, o + 4, type);
      docs.set(JAVA_LONG, o + 8, value);
      entryValues.add(copy(doc, valueStart, msgpack.getOffset() - valueStart));
      nDocs++;
    }
    if (size > 1) {
      final long row = ZbHip.DOC_ENTRY.byteSize();
      ZbHip.docMergeOrder(keyOffsets, size, docs.asSlice(row * first, row * size));
    }
    return size;
  }

  private static DirectBuffer copy(final DirectBuffer src, final int offset, final int length) {
    final byte[] b = new byte[length];
    src.getBytes(offset, b);
    return new UnsafeBuffer(b);
  }

  /**
   * zbhip_submit + zbhip_run.  The records are drained command by command when the platform reaches
   * each (zbhip_drain_command): the keys of commands after a fallback command are fixed only once the
   * CPU engine's keys for it are declared.
   */
  void submitRun(final MemorySegment handle) {
    this.handle = handle;
    if (nXparts > 0) {
      ZbHip.submitEx(handle, cmds, n, docs, nDocs, xparts, nXparts);
    } else {
      ZbHip.submit(handle, cmds, n, docs, nDocs);
    }
    ZbHip.run(handle, 0);
  }

  /**
   * Appends window command i's records to the builder, as the reference's processors would, and
   * returns how many follow-up commands the platform will feed back (the ones not written
   * unprocessed).  A rejection of the command itself carries the command's value
   * (TypedRejectionWriter.appendRejection: TimerRecord, JobRecord, ... as the log holds them);
   * every follow-up written unprocessed is expected back from the log as a continuation (its id in
   * the record's aux); a process instance that completed frees its slot once its continuations ran.
   */
  int emit(final int i, final TypedRecord command, final ProcessingResultBuilder out, final GpuBatchProcessor p) {
    final long nr = ZbHip.drainCommand(handle, i, this::ofAtLeast);
    final RecordMetadata meta = new RecordMetadata();
    commandTimestamp = command.getTimestamp(); // a MESSAGE record's deadline = timestamp + timeToLive
    int admitted = 0;
    final java.util.LinkedHashMap<Long, String> created = new java.util.LinkedHashMap<>(); // jobs not pushed (yet)
    for (long r = 0; r < nr; r++) {
      final MemorySegment rec = recs.asSlice(80L * r, 80);
      final long key = rec.get(JAVA_LONG, ZbHip.Rec.KEY);
      final byte recordType = rec.get(JAVA_BYTE, ZbHip.Rec.RECORD_TYPE);
      final byte valueType = rec.get(JAVA_BYTE, ZbHip.Rec.VALUE_TYPE);
      final byte intent = rec.get(JAVA_BYTE, ZbHip.Rec.INTENT);
      final int rejection = rec.get(JAVA_BYTE, ZbHip.Rec.REJECTION_TYPE) & 0xFF;
      final int ordinal = rec.get(JAVA_SHORT, ZbHip.Rec.ORDINAL) & 0xFFFF;
      meta.reset()
          .recordType(RecordType.values()[recordType])
          .valueType(ValueType.get((short) valueType))
          .intent(intent(valueType, intent));
      if (rejection != 0xFF) {
        meta.rejectionType(RejectionType.get((short) rejection)).rejectionReason(p.rejectionReason(rec));
      }
      final boolean ofCommand = recordType == RecordType.COMMAND_REJECTION.value() && ordinal == 0
          && valueType == command.getValueType().value() && intent == command.getIntent().value();
      final UnifiedRecordValue value = ofCommand ? (UnifiedRecordValue) command.getValue() : value(rec, i, p);
      out.appendRecord(key, value, meta);
      if (recordType == RecordType.COMMAND.value()) {
        if (rec.get(JAVA_BYTE, ZbHip.Rec.UNPROCESSED) != 0) { // zbhip_record.unprocessed: a continuation, its id in aux
          if (value instanceof final ProcessInstanceRecord v) {
            p.expectContinuation(new GpuBatchProcessor.Continuation(
                rec.get(JAVA_LONG, ZbHip.Rec.AUX), instances[i], key, valueType, intent, v.getElementId(), v.getFlowScopeKey(),
                -1, v.getProcessInstanceKey()));
          } else {
            final ProcessInstanceBatchRecord v = (ProcessInstanceBatchRecord) value;
            p.expectContinuation(new GpuBatchProcessor.Continuation(
                rec.get(JAVA_LONG, ZbHip.Rec.AUX), instances[i], key, valueType, intent, null, -1,
                v.getBatchElementInstanceKey(), v.getProcessInstanceKey()));
          }
        } else {
          admitted++;
        }
      } else if (valueType == ValueType.PROCESS_INSTANCE.value()
          && intent == ProcessInstanceIntent.ELEMENT_COMPLETED.value() && rec.get(JAVA_INT, ZbHip.Rec.ELEMENT_IDX) == 0) {
        p.instanceEnded(instances[i]); // the process element (index 0) completed
      } else if (valueType == ValueType.JOB.value() && recordType == RecordType.EVENT.value()
          && intent == JobIntent.CREATED.value()) {
        created.put(key, ((JobRecord) value).getType());
      } else if (valueType == ValueType.JOB_BATCH.value() && recordType == RecordType.EVENT.value()) {
        p.jobStreams().push(out, handle, (JobBatchRecord) value, p); // publishWork's push, post-commit
        created.remove(((JobBatchRecord) value).jobKeys().iterator().next().getValue());
      } else if (valueType == ValueType.TIMER.value() && recordType == RecordType.EVENT.value()
          && intent == TimerIntent.CREATED.value()) {
        p.timerCreated(out, ((TimerRecord) value).getDueDate()); // DueDateTimerChecker.scheduleTimer, post-commit
      } else if (valueType == ValueType.MESSAGE_SUBSCRIPTION.value() && recordType == RecordType.EVENT.value()) {
        p.messages().onSubscriptionEvent(meta.getIntent(), (MessageSubscriptionRecord) value, rec.get(JAVA_INT, ZbHip.Rec.CORRELATION_KEY));
      } else if (valueType == ValueType.PROCESS_MESSAGE_SUBSCRIPTION.value() && recordType == RecordType.EVENT.value()) {
        p.messages().onProcessSubscriptionEvent(meta.getIntent(), (ProcessMessageSubscriptionRecord) value, instances[i], p);
      }
    }
    // publishWork of a created job no stream took: notifyJobAvailable (BpmnJobActivationBehavior.java:97-111)
    for (final String type : created.values()) {
      p.jobStreams().notifyAvailable(out, type);
    }
    return admitted;
  }

  /** A record buffer of at least {@code n} rows (zbhip_drain_command's output). */
  private MemorySegment ofAtLeast(final long n) {
    if (n > recCap) {
      recCap = Math.max(n, 2 * recCap);
      recs = Arena.ofAuto().allocate(ZbHip.RECORD.byteSize() * recCap, 16);
    }
    return recs;
  }

  private static Intent intent(final byte valueType, final byte intent) {
    return Intent.fromProtocolValue(ValueType.get((short) valueType), (short) intent);
  }

  private long commandTimestamp; // the timestamp of the command emit() expands

  /** The record value of a zbhip_record row without a source document (the scheduled-task calls). */
  UnifiedRecordValue valueOf(final MemorySegment r, final GpuBatchProcessor p) {
    return value(r, -1, p);
  }

  private UnifiedRecordValue value(final MemorySegment r, final int i, final GpuBatchProcessor p) {
    final ZbHip.Deployed d = p.process(r.get(JAVA_INT, ZbHip.Rec.PROCESS_IDX) < 0 ? 0 : r.get(JAVA_INT, ZbHip.Rec.PROCESS_IDX));
    final int elem = r.get(JAVA_INT, ZbHip.Rec.ELEMENT_IDX);
    final long scope = r.get(JAVA_LONG, ZbHip.Rec.SCOPE_KEY);
    final long pik = r.get(JAVA_LONG, ZbHip.Rec.PROCESS_INSTANCE_KEY);
    final long aux = r.get(JAVA_LONG, ZbHip.Rec.AUX);
    final ValueType vt = ValueType.get((short) r.get(JAVA_BYTE, ZbHip.Rec.VALUE_TYPE));
    switch (vt) {
      case PROCESS_INSTANCE -> {
        final ProcessInstanceRecord v = new ProcessInstanceRecord();
        v.setBpmnElementType(BpmnElementType.values()[d.elementTypes()[elem]])
            .setBpmnEventType(BpmnEventType.values()[d.eventTypes()[elem]])
            .setElementId(d.elementIds()[elem])
            .setBpmnProcessId(d.bpmnProcessId())
            .setVersion(d.version())
            .setProcessDefinitionKey(d.definitionKey())
            .setProcessInstanceKey(pik)
            .setFlowScopeKey(scope)
            .setParentProcessInstanceKey(-1)
            .setParentElementInstanceKey(-1)
            .setTenantId(TENANT);
        return v;
      }
      case JOB -> {
        final JobRecord v = new JobRecord();
        if (elem >= 0) {
          v.setType(d.jobTypes()[elem])
              .setRetries(d.retries()[elem])
              .setElementId(d.elementIds()[elem])
              .setElementInstanceKey(scope)
              .setProcessInstanceKey(pik)
              .setBpmnProcessId(d.bpmnProcessId())
              .setProcessDefinitionVersion(d.version())
              .setProcessDefinitionKey(d.definitionKey());
          if (d.customHeaders()[elem] != null) {
            // BpmnJobBehavior.encodeHeaders: the task headers' msgpack map (the compiler's HashMap order)
            v.setCustomHeaders(new UnsafeBuffer(d.customHeaders()[elem]));
          }
        }
        if (aux >= 0) {
          v.setVariables(documents[i]); // JOB:COMPLETED / COMPLETE rejection: the command's variables
        }
        final long deadline = r.get(JAVA_LONG, ZbHip.Rec.MESSAGE_KEY); // message_key: an ACTIVATED job's deadline
        if (deadline != -1) {
          final int worker = r.get(JAVA_INT, ZbHip.Rec.CORRELATION_KEY); // correlation_key: its worker (value dictionary)
          v.setDeadline(deadline)
              .setWorker(new UnsafeBuffer(worker == Messages.NO_STRING ? new byte[0] : p.stringValue(worker)));
        }
        if (r.get(JAVA_BYTE, ZbHip.Rec.RECORD_TYPE) == RecordType.EVENT.value() && (r.get(JAVA_BYTE, ZbHip.Rec.REASON_ARG) & 1) != 0) {
          // a failed job's stored retries and errorMessage (JobFailProcessor.failJob): reason_arg bit 0,
          // retries in partition, the errorMessage's value-dictionary id in message_name | bpmn_process_id << 16
          final int eid = (r.get(JAVA_SHORT, ZbHip.Rec.MESSAGE_NAME) & 0xFFFF) | (r.get(JAVA_SHORT, ZbHip.Rec.BPMN_PROCESS_ID) & 0xFFFF) << 16;
          v.setRetries(r.get(JAVA_INT, ZbHip.Rec.PARTITION))
              .setErrorMessage(eid == Messages.NO_STRING ? "" : new String(p.stringValue(eid), java.nio.charset.StandardCharsets.UTF_8));
        }
        return v.setTenantId(TENANT);
      }
      case JOB_BATCH -> {
        // a job stream's push (BpmnJobActivationBehavior.publishWork :61-100): the job (its row read as
        // JOB:CREATED) in a fresh JobBatchRecord with the stream's type, worker and timeout
        final MemorySegment asJob = Arena.ofAuto().allocate(ZbHip.RECORD);
        asJob.copyFrom(r);
        asJob.set(JAVA_BYTE, 41, (byte) ValueType.JOB.value());
        asJob.set(JAVA_BYTE, 42, (byte) JobIntent.CREATED.value());
        asJob.set(JAVA_LONG, 48, -1L);
        final JobRecord job = (JobRecord) value(asJob, i, p);
        final JobBatchRecord v = new JobBatchRecord();
        v.setType(job.getTypeBuffer()).setWorker(job.getWorkerBuffer()).setTimeout(p.jobStreams().timeout(job.getType()));
        v.jobKeys().add().setValue(aux);
        v.jobs().add().wrapWithoutVariables(job);
        return v;
      }
      case VARIABLE -> {
        final VariableRecord v = new VariableRecord();
        // aux == ZBHIP_AUX_INLINE: a value the engine computed (a multi-instance loop variable), its
        // zbhip_doc_type in zbhip_record.partition and the value in message_key
        v.setName(new UnsafeBuffer(p.name(elem).getBytes()))
            .setValue(aux == -2 ? inline(r.get(JAVA_INT, ZbHip.Rec.PARTITION), r.get(JAVA_LONG, ZbHip.Rec.MESSAGE_KEY), p) : entryValues.get((int) aux))
            .setScopeKey(scope)
            .setProcessInstanceKey(pik)
            .setProcessDefinitionKey(d.definitionKey())
            .setBpmnProcessId(new UnsafeBuffer(d.bpmnProcessId().getBytes()));
        return v.setTenantId(TENANT);
      }
      case PROCESS_EVENT -> {
        final ProcessEventRecord v = new ProcessEventRecord();
        v.setScopeKey(scope)
            .setTargetElementIdBuffer(new UnsafeBuffer(d.elementIds()[elem].getBytes()));
        if (r.get(JAVA_BYTE, ZbHip.Rec.INTENT) == ProcessEventIntent.TRIGGERING.value()) {
          v.setVariablesBuffer(documents[i]); // TRIGGERED: processEventTriggered resets the record
        }
        v
            .setProcessDefinitionKey(d.definitionKey())
            .setProcessInstanceKey(pik);
        return v.setTenantId(TENANT);
      }
      case TIMER -> {
        // TimerRecord (CatchEventBehavior.java:311-319): CREATED / CANCELED / TRIGGERED carry the
        // timer's value, a rejected TRIGGER the command's key and dueDate
        final TimerRecord v = new TimerRecord();
        v.setElementInstanceKey(scope)
            .setProcessInstanceKey(pik)
            .setDueDate(aux)
            // zbhip_record.partition: the TimerRecord's repetitions (-1 infinite); a rejection: 1
            .setRepetitions(r.get(JAVA_BYTE, ZbHip.Rec.RECORD_TYPE) == RecordType.COMMAND_REJECTION.value() ? 1 : r.get(JAVA_INT, ZbHip.Rec.PARTITION))
            .setTargetElementId(new UnsafeBuffer(elem >= 0 ? d.elementIds()[elem].getBytes() : new byte[0]))
            .setProcessDefinitionKey(elem >= 0 ? d.definitionKey() : -1);
        return v.setTenantId(TENANT);
      }
      case INCIDENT -> {
        // BpmnIncidentBehavior.createIncident (:51-71) of an exclusive gateway: the ErrorType ordinal
        // in zbhip_record.partition, the message composed by the library (zbhip_incident_message)
        final IncidentRecord v = new IncidentRecord();
        final boolean job = r.get(JAVA_INT, ZbHip.Rec.PARTITION) == ErrorType.JOB_NO_RETRIES.ordinal();
        if (job) { // JobFailProcessor.raiseIncident (:139-162): the job's key and message
          final int mid = r.get(JAVA_INT, ZbHip.Rec.CORRELATION_KEY);
          v.setJobKey(aux).setErrorMessage(new String(p.stringValue(mid), java.nio.charset.StandardCharsets.UTF_8));
        } else {
          v.setErrorMessage(p.incidentMessage(r));
        }
        v.setErrorType(ErrorType.values()[r.get(JAVA_INT, ZbHip.Rec.PARTITION)])
            .setBpmnProcessId(new UnsafeBuffer(d.bpmnProcessId().getBytes()))
            .setProcessDefinitionKey(d.definitionKey())
            .setProcessInstanceKey(pik)
            .setElementId(new UnsafeBuffer(d.elementIds()[elem].getBytes()))
            .setElementInstanceKey(scope)
            .setVariableScopeKey(scope);
        return v.setTenantId(TENANT);
      }
      case PROCESS_INSTANCE_BATCH -> {
        // a multi-instance body's activateChildInstancesInBatches (index in zbhip_record.partition)
        final ProcessInstanceBatchRecord v = new ProcessInstanceBatchRecord();
        return v.setProcessInstanceKey(pik).setBatchElementInstanceKey(scope).setIndex(r.get(JAVA_INT, ZbHip.Rec.PARTITION));
      }
      case PROCESS_INSTANCE_CREATION -> {
        final ProcessInstanceCreationRecord v = new ProcessInstanceCreationRecord();
        v.setBpmnProcessId(d.bpmnProcessId())
            .setProcessDefinitionKey(d.definitionKey())
            .setVersion(d.version())
            .setProcessInstanceKey(scope)
            .setVariables(documents[i]);
        return v.setTenantId(TENANT);
      }
      case MESSAGE, MESSAGE_SUBSCRIPTION, PROCESS_MESSAGE_SUBSCRIPTION -> {
        return messageValue(r, vt, d, elem, scope, pik, p, commandTimestamp);
      }
      default -> throw new IllegalStateException("value type outside the device subset: " + vt);
    }
  }

  /**
   * A message record: the drained zbhip_record carries every property (the log writer's fields,
   * logwriter.cpp); message variables are empty in the subset, deadline = the PUBLISH command's
   * timestamp + timeToLive 0 (MessagePublishProcessor.java:110).
   */
  private static UnifiedRecordValue messageValue(final MemorySegment r, final ValueType vt, final ZbHip.Deployed d,
      final int elem, final long scope, final long pik, final GpuBatchProcessor p, final long timestamp) {
    final int nameId = r.get(JAVA_SHORT, ZbHip.Rec.MESSAGE_NAME) & 0xFFFF, bpmnId = r.get(JAVA_SHORT, ZbHip.Rec.BPMN_PROCESS_ID) & 0xFFFF;
    final int corrId = r.get(JAVA_INT, ZbHip.Rec.CORRELATION_KEY);
    final DirectBuffer name = new UnsafeBuffer((nameId == 0xFFFF ? "" : p.name(nameId)).getBytes());
    final DirectBuffer bpmn = new UnsafeBuffer((bpmnId == 0xFFFF ? "" : p.name(bpmnId)).getBytes());
    final DirectBuffer corr = new UnsafeBuffer(corrId == Messages.NO_STRING ? new byte[0] : p.stringValue(corrId));
    final boolean interrupting = r.get(JAVA_BYTE, ZbHip.Rec.INTERRUPTING) != 0;
    final long messageKey = r.get(JAVA_LONG, ZbHip.Rec.MESSAGE_KEY);
    if (vt == ValueType.MESSAGE) {
      return new MessageRecord().setName(name).setCorrelationKey(corr).setTimeToLive(0).setDeadline(timestamp)
          .setTenantId(TENANT);
    }
    if (vt == ValueType.MESSAGE_SUBSCRIPTION) {
      return new MessageSubscriptionRecord().setProcessInstanceKey(pik).setElementInstanceKey(scope)
          .setMessageKey(messageKey).setMessageName(name).setCorrelationKey(corr).setInterrupting(interrupting)
          .setBpmnProcessId(bpmn).setTenantId(TENANT);
    }
    return new ProcessMessageSubscriptionRecord().setSubscriptionPartitionId(r.get(JAVA_INT, ZbHip.Rec.PARTITION))
        .setProcessInstanceKey(pik).setElementInstanceKey(scope).setMessageKey(messageKey).setMessageName(name)
        .setInterrupting(interrupting).setBpmnProcessId(bpmn).setCorrelationKey(corr)
        .setElementId(new UnsafeBuffer((elem >= 0 && r.get(JAVA_INT, ZbHip.Rec.PROCESS_IDX) >= 0 ? d.elementIds()[elem] : "").getBytes()))
        .setTenantId(TENANT);
  }

  /** One msgpack value of a zbhip_doc_type (FeelToMessagePackTransformer's encoding of an item). */
  private static DirectBuffer inline(final int type, final long value, final GpuBatchProcessor p) {
    final ExpandableArrayBuffer buf = new ExpandableArrayBuffer(16);
    final MsgPackWriter w = new MsgPackWriter().wrap(buf, 0);
    switch (type) {
      case DOC_BOOL -> w.writeBoolean(value != 0);
      case DOC_INT -> w.writeInteger(value);
      case DOC_DEC -> w.writeFloat(value / 1_000_000d);
      case DOC_STR -> w.writeString(new UnsafeBuffer(p.stringValue(value)));
      default -> w.writeNil();
    }
    return new UnsafeBuffer(buf, 0, w.getOffset());
  }

  static {
    // record kinds the device emits for configs 1-4 (zbhip.h enums) map onto these reference intents
    assert JobIntent.CREATED.value() == 0 && VariableIntent.CREATED.value() == 0
        && ProcessEventIntent.TRIGGERING.value() == 0 && ProcessInstanceCreationIntent.CREATED.value() == 1;
  }
}
