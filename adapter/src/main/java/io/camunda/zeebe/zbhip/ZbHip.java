/*
 * Panama FFM binding of libzbhip.so (include/zbhip.h) for the broker's Java host.
 *
 * Written against Java 21 (the reference's toolchain, parent/pom.xml:28), where java.lang.foreign
 * is a preview API (JEP 442): compile and run with --enable-preview.  This image has no JDK, so the
 * file is not compiled here; the ABI it binds is exercised from Python (zeebe_amd/native.py) and C
 * (tests/test_abi.py) instead; every layout below mirrors the header byte for byte (COMMAND 16,
 * DOC_ENTRY 16, RECORD 80, XPART 48 bytes -- the sizes tests/test_abi.py checks for the Python
 * mirror).
 */
package io.camunda.zeebe.zbhip;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.StructLayout;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.lang.invoke.MethodHandles;
import java.lang.invoke.MethodType;
import java.nio.charset.StandardCharsets;

/** Downcalls and struct layouts of the zbhip C ABI; every method throws on a negative return code. */
public final class ZbHip {

  // ---- error codes (zbhip.h zbhip_status) ----
  public static final int OK = 0;
  public static final int EUNSUPP = -5;
  public static final int ENOMEM = -2;

  // ---- command kinds (zbhip_command_kind) ----
  public static final byte CMD_CREATE = 1; // PROCESS_INSTANCE_CREATION:CREATE
  public static final byte CMD_JOB_COMPLETE = 2; // JOB:COMPLETE
  public static final byte CMD_TIMER_TRIGGER = 8; // TIMER:TRIGGER (the due-date checker's command)
  public static final byte CMD_CONTINUE = 9; // a deferred continuation read back from the log
  public static final int OPEN_DEFER_CONTINUATIONS = 2; // zbhip_config.flags
  public static final byte CMD_PUBLISH = 3; // MESSAGE:PUBLISH (config 5)
  public static final byte CMD_MSG_SUB_CREATE = 4;
  public static final byte CMD_PMS_CREATE = 5;
  public static final byte CMD_PMS_CORRELATE = 6;
  public static final byte CMD_MSG_SUB_CORRELATE = 7;
  public static final byte CMD_MSG_SUB_DELETE = 10; // closeMessageSubscription
  public static final byte CMD_PMS_DELETE = 11; // closeProcessMessageSubscription (the acknowledgement)

  public static final int RUN_DEVICE_RECORDS = 8;

  // ---- struct layouts (little-endian, natural alignment) ----
  public static final StructLayout CONFIG =
      MemoryLayout.structLayout(
          JAVA_INT.withName("partition_id"),
          JAVA_INT.withName("partition_count"),
          JAVA_INT.withName("device"),
          JAVA_INT.withName("max_commands_in_batch"),
          JAVA_INT.withName("max_instances"),
          JAVA_INT.withName("max_commands"),
          JAVA_INT.withName("max_records_per_batch"),
          JAVA_INT.withName("max_doc_entries"),
          JAVA_LONG.withName("initial_key"),
          JAVA_INT.withName("max_correlation_keys"),
          JAVA_INT.withName("flags"),
          ADDRESS.withName("stream"));

  public static final StructLayout COMMAND =
      MemoryLayout.structLayout(
          JAVA_INT.withName("instance"),
          JAVA_BYTE.withName("kind"),
          JAVA_BYTE.withName("doc_count"),
          JAVA_SHORT.withName("ref"),
          JAVA_INT.withName("doc_begin"),
          JAVA_INT.withName("pad")); // 16 bytes

  public static final StructLayout DOC_ENTRY =
      MemoryLayout.structLayout(
          JAVA_INT.withName("name_id"),
          JAVA_BYTE.withName("type"),
          MemoryLayout.paddingLayout(3),
          JAVA_LONG.withName("value")); // 16 bytes

  public static final StructLayout RECORD =
      MemoryLayout.structLayout(
          JAVA_LONG.withName("key"),
          JAVA_LONG.withName("scope_key"),
          JAVA_LONG.withName("process_instance_key"),
          JAVA_LONG.withName("source_index"),
          JAVA_INT.withName("process_idx"),
          JAVA_INT.withName("element_idx"),
          JAVA_BYTE.withName("record_type"),
          JAVA_BYTE.withName("value_type"),
          JAVA_BYTE.withName("intent"),
          JAVA_BYTE.withName("rejection_type"),
          JAVA_SHORT.withName("ordinal"),
          JAVA_BYTE.withName("reason"),
          JAVA_BYTE.withName("reason_arg"),
          JAVA_LONG.withName("aux"),
          JAVA_LONG.withName("message_key"),
          JAVA_INT.withName("correlation_key"),
          JAVA_SHORT.withName("message_name"),
          JAVA_SHORT.withName("bpmn_process_id"),
          JAVA_INT.withName("partition"),
          JAVA_BYTE.withName("interrupting"),
          JAVA_BYTE.withName("unprocessed"),
          MemoryLayout.paddingLayout(2)); // 80 bytes

  /** Byte offsets of zbhip_record fields, taken from RECORD (one source for every reader of a row). */
  public static final class Rec {
    private static long off(final String f) {
      return RECORD.byteOffset(MemoryLayout.PathElement.groupElement(f));
    }

    public static final long KEY = off("key");
    public static final long SCOPE_KEY = off("scope_key");
    public static final long PROCESS_INSTANCE_KEY = off("process_instance_key");
    public static final long PROCESS_IDX = off("process_idx");
    public static final long ELEMENT_IDX = off("element_idx");
    public static final long RECORD_TYPE = off("record_type");
    public static final long VALUE_TYPE = off("value_type");
    public static final long INTENT = off("intent");
    public static final long REJECTION_TYPE = off("rejection_type");
    public static final long ORDINAL = off("ordinal");
    public static final long REASON_ARG = off("reason_arg");
    public static final long AUX = off("aux");
    public static final long MESSAGE_KEY = off("message_key");
    public static final long CORRELATION_KEY = off("correlation_key");
    public static final long MESSAGE_NAME = off("message_name");
    public static final long BPMN_PROCESS_ID = off("bpmn_process_id");
    public static final long PARTITION = off("partition");
    public static final long INTERRUPTING = off("interrupting");
    public static final long UNPROCESSED = off("unprocessed");

    private Rec() {}
  }

  public static final StructLayout XPART =
      MemoryLayout.structLayout(
          JAVA_LONG.withName("element_instance_key"),
          JAVA_LONG.withName("process_instance_key"),
          JAVA_LONG.withName("message_key"),
          JAVA_INT.withName("correlation_key"),
          JAVA_INT.withName("instance"),
          JAVA_SHORT.withName("element_ord"),
          JAVA_SHORT.withName("message_name"),
          JAVA_SHORT.withName("bpmn_process_id"),
          JAVA_BYTE.withName("kind"),
          JAVA_BYTE.withName("interrupting"),
          JAVA_SHORT.withName("source_partition"),
          JAVA_SHORT.withName("target_partition"),
          JAVA_INT.withName("pad")); // 48 bytes

  public static final StructLayout STATS =
      MemoryLayout.structLayout(
          JAVA_LONG.withName("commands"),
          JAVA_LONG.withName("records"),
          JAVA_LONG.withName("transitions"),
          JAVA_LONG.withName("completed_instances"),
          JAVA_LONG.withName("keys"),
          JAVA_LONG.withName("fallback"),
          JAVA_DOUBLE.withName("step_ms"),
          JAVA_DOUBLE.withName("compact_ms"),
          JAVA_INT.withName("rounds"),
          JAVA_INT.withName("launches"),
          JAVA_LONG.withName("template_batches"));

  private static final Linker LINKER = Linker.nativeLinker();
  private static final SymbolLookup LIB =
      SymbolLookup.libraryLookup(System.getProperty("zbhip.library", "libzbhip.so"), Arena.global());

  private static MethodHandle fn(final String name, final FunctionDescriptor d) {
    return LINKER.downcallHandle(LIB.find(name).orElseThrow(), d);
  }

  // int zbhip_compile_bpmn(const char*, size_t, int64_t, int32_t, zbhip_process_csr**, char*, size_t)
  private static final MethodHandle COMPILE =
      fn("zbhip_compile_bpmn", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, JAVA_LONG, JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG));
  private static final MethodHandle FREE_CSR = fn("zbhip_free_csr", FunctionDescriptor.ofVoid(ADDRESS));
  private static final MethodHandle OPEN = fn("zbhip_open", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
  private static final MethodHandle CLOSE = fn("zbhip_close", FunctionDescriptor.ofVoid(ADDRESS));
  private static final MethodHandle DEPLOY = fn("zbhip_deploy", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS));
  private static final MethodHandle INTERN = fn("zbhip_intern", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
  private static final MethodHandle INTERN_STRING =
      fn("zbhip_intern_string", FunctionDescriptor.of(JAVA_LONG, ADDRESS, ADDRESS, JAVA_LONG));
  private static final MethodHandle SUBMIT =
      fn("zbhip_submit", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG));
  private static final MethodHandle SUBMIT_EX =
      fn("zbhip_submit_ex", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG));
  private static final MethodHandle RUN = fn("zbhip_run", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
  private static final MethodHandle DOC_MERGE_ORDER =
      fn("zbhip_doc_merge_order", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle SET_CLOCK = fn("zbhip_set_clock", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG));
  private static final MethodHandle PENDING = fn("zbhip_pending_records", FunctionDescriptor.of(JAVA_LONG, ADDRESS));
  private static final MethodHandle DRAIN = fn("zbhip_drain", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle OUTBOX = fn("zbhip_outbox", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle OUTBOX_COMMAND =
      fn("zbhip_outbox_command", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle STATS_FN = fn("zbhip_get_stats", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
  private static final MethodHandle STATUS =
      fn("zbhip_command_status", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS, ADDRESS));
  private static final MethodHandle RESOLVE =
      fn("zbhip_resolve_key", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS, ADDRESS));
  private static final MethodHandle REASON =
      fn("zbhip_rejection_reason", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG));
  private static final MethodHandle INCIDENT_MESSAGE =
      fn("zbhip_incident_message", FunctionDescriptor.of(JAVA_LONG, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG));
  private static final MethodHandle EXPORT_INSTANCES_DB =
      fn("zbhip_export_instances_db", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, ADDRESS));
  private static final MethodHandle EVICT = fn("zbhip_evict_instances", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG));
  private static final MethodHandle EXPORT_SLOTS =
      fn("zbhip_export_correlation_slots", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, ADDRESS));
  private static final MethodHandle EXPORT_SLOTS_DB =
      fn("zbhip_export_correlation_slots_db", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, ADDRESS));
  private static final MethodHandle EVICT_SLOTS =
      fn("zbhip_evict_correlation_slots", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG));
  private static final MethodHandle KEY_BEFORE = fn("zbhip_key_before", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle CONTINUATIONS =
      fn("zbhip_continuations", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS));
  private static final MethodHandle PENDING_CONTINUATIONS =
      fn("zbhip_pending_continuations", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
  private static final MethodHandle CURRENT_KEY = fn("zbhip_current_key", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
  private static final MethodHandle SET_KEY_IF_HIGHER =
      fn("zbhip_set_key_if_higher", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG));
  private static final MethodHandle ACTIVATE_JOBS =
      fn("zbhip_activate_jobs", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle DRAIN_COMMAND =
      fn("zbhip_drain_command", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle STRING_VALUE =
      fn("zbhip_string_value", FunctionDescriptor.of(ADDRESS, ADDRESS, JAVA_INT, ADDRESS));
  private static final MethodHandle SELECT_INSTANCES_DB =
      fn("zbhip_select_instances_db",
          FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle EXTERNAL_KEYS =
      fn("zbhip_set_external_keys", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, JAVA_INT));
  private static final MethodHandle IMPORT_DB =
      fn("zbhip_import_state_db", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, JAVA_INT, ADDRESS));
  private static final MethodHandle STRING = fn("zbhip_string", FunctionDescriptor.of(ADDRESS, ADDRESS, JAVA_INT, JAVA_INT));
  private static final MethodHandle NAME = fn("zbhip_name", FunctionDescriptor.of(ADDRESS, ADDRESS, JAVA_INT));
  private static final MethodHandle DUE_TIMERS =
      fn("zbhip_due_timers", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS, ADDRESS));
  private static final MethodHandle TIMED_OUT_JOBS =
      fn("zbhip_timed_out_jobs", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS, ADDRESS));
  private static final MethodHandle TIME_OUT_JOB =
      fn("zbhip_time_out_job",
          FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle FAIL_JOB =
      fn("zbhip_fail_job", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle SET_JOB_STREAM =
      fn("zbhip_set_job_stream",
          FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, JAVA_LONG, JAVA_INT));
  private static final MethodHandle JOB_VARIABLES =
      fn("zbhip_job_variables",
          FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
  private static final MethodHandle JOB_STATE =
      fn("zbhip_job_state", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG));
  private static final MethodHandle ACTIVATABLE_JOBS =
      fn("zbhip_activatable_jobs", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));

  /** The zbhip_db_sink upcall: (ctx, column family, key, key length, value, value length). */
  @FunctionalInterface
  public interface DbSink {
    void entry(int columnFamily, byte[] key, byte[] value);
  }

  private static final FunctionDescriptor DB_SINK =
      FunctionDescriptor.ofVoid(ADDRESS, JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG);

  private ZbHip() {}

  static int check(final int rc, final String what) {
    if (rc < 0) {
      throw new ZbHipException(what, rc);
    }
    return rc;
  }

  private static Object call(final MethodHandle h, final Object... args) {
    try {
      return h.invokeWithArguments(args);
    } catch (final RuntimeException e) {
      throw e;
    } catch (final Throwable t) {
      throw new IllegalStateException(t);
    }
  }

  /** zbhip_open: one handle per partition, on the partition's GPU. */
  public static MemorySegment open(
      final Arena arena,
      final int partitionId,
      final int partitionCount,
      final int device,
      final int maxCommandsInBatch,
      final int maxInstances,
      final int maxCommands,
      final long initialKey,
      final int maxCorrelationKeys,
      final int flags) {
    final MemorySegment cfg = arena.allocate(CONFIG);
    cfg.set(JAVA_INT, 0, partitionId);
    cfg.set(JAVA_INT, 4, partitionCount);
    cfg.set(JAVA_INT, 8, device);
    cfg.set(JAVA_INT, 12, maxCommandsInBatch);
    cfg.set(JAVA_INT, 16, maxInstances);
    cfg.set(JAVA_INT, 20, maxCommands);
    cfg.set(JAVA_INT, 24, 0); // records per batch: derived from the deployed processes
    cfg.set(JAVA_INT, 28, 16 * maxCommands);
    cfg.set(JAVA_LONG, 32, initialKey);
    cfg.set(JAVA_INT, 40, maxCorrelationKeys);
    cfg.set(JAVA_INT, 44, flags);
    cfg.set(ADDRESS, 48, MemorySegment.NULL);
    final MemorySegment out = arena.allocate(ADDRESS);
    check((int) call(OPEN, cfg, out), "zbhip_open");
    return out.get(ADDRESS, 0);
  }

  public static void close(final MemorySegment h) {
    call(CLOSE, h);
  }

  /** What the adapter keeps of a deployed process to build record values (zbhip_process_csr). */
  public record Deployed(
      int index,
      String bpmnProcessId,
      long definitionKey,
      int version,
      String[] elementIds,
      byte[] elementTypes,
      byte[] eventTypes,
      String[] jobTypes,
      int[] retries,
      byte[][] customHeaders) {} // zeebe:taskHeaders per element (zbhip_process_csr.header_bytes), null: none

  /**
   * zbhip_compile_bpmn + zbhip_deploy: the deployment, or null when the process uses a construct
   * outside the GPU subset (ZBHIP_EUNSUPP: its commands stay on the CPU engine).  The element table
   * is read from the compiled CSR (zbhip_process_csr / zbhip_element, 36-byte elements).
   */
  public static Deployed deploy(final MemorySegment h, final byte[] bpmnXml, final long definitionKey, final int version) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment xml = a.allocateArray(JAVA_BYTE, bpmnXml);
      final MemorySegment csrOut = a.allocate(ADDRESS);
      final MemorySegment err = a.allocate(512);
      final int rc = (int) call(COMPILE, xml, (long) bpmnXml.length, definitionKey, version, csrOut, err, 512L);
      if (rc == EUNSUPP) {
        return null;
      }
      check(rc, "zbhip_compile_bpmn: " + err.getUtf8String(0));
      final MemorySegment c = csrOut.get(ADDRESS, 0).reinterpret(144);
      try {
        final MemorySegment idx = a.allocate(JAVA_INT);
        final int d = (int) call(DEPLOY, h, c, idx);
        if (d == EUNSUPP) {
          return null;
        }
        check(d, "zbhip_deploy");
        final int n = c.get(JAVA_INT, 0);
        final MemorySegment els = c.get(ADDRESS, 8).reinterpret(36L * n);
        final int nStrings = c.get(JAVA_INT, 64);
        final MemorySegment strs = c.get(ADDRESS, 72).reinterpret(8L * nStrings);
        final String[] strings = new String[nStrings];
        for (int i = 0; i < nStrings; i++) {
          strings[i] = strs.getAtIndex(ADDRESS, i).reinterpret(Long.MAX_VALUE).getUtf8String(0);
        }
        final String[] ids = new String[n];
        final String[] jobTypes = new String[n];
        final byte[] types = new byte[n];
        final byte[] events = new byte[n];
        final int[] retries = new int[n];
        for (int e = 0; e < n; e++) {
          final long o = 36L * e;
          types[e] = els.get(JAVA_BYTE, o);
          events[e] = els.get(JAVA_BYTE, o + 1);
          final int jt = els.get(JAVA_SHORT, o + 16) & 0xFFFF;
          jobTypes[e] = jt < nStrings ? strings[jt] : "";
          retries[e] = els.get(JAVA_SHORT, o + 18) & 0xFFFF;
          ids[e] = strings[els.get(JAVA_SHORT, o + 22) & 0xFFFF];
        }
        final String bpmnId = strings[c.get(JAVA_SHORT, 100) & 0xFFFF];
        // header_begin (offset 128: n + 1 offsets) and header_bytes (136), ABI 10
        final byte[][] headers = new byte[n][];
        final MemorySegment hb = c.get(ADDRESS, 128);
        if (hb.address() != 0) {
          final MemorySegment begin = hb.reinterpret(4L * (n + 1));
          final MemorySegment bytes = c.get(ADDRESS, 136).reinterpret(begin.getAtIndex(JAVA_INT, n));
          for (int e = 0; e < n; e++) {
            final int b = begin.getAtIndex(JAVA_INT, e), end = begin.getAtIndex(JAVA_INT, e + 1);
            if (end > b) {
              headers[e] = bytes.asSlice(b, end - b).toArray(JAVA_BYTE);
            }
          }
        }
        return new Deployed(
            idx.get(JAVA_INT, 0), bpmnId, definitionKey, version, ids, types, events, jobTypes, retries, headers);
      } finally {
        call(FREE_CSR, c);
      }
    }
  }

  public static int intern(final MemorySegment h, final String name) {
    try (Arena a = Arena.ofConfined()) {
      return check((int) call(INTERN, h, a.allocateUtf8String(name)), "zbhip_intern");
    }
  }

  public static long internString(final MemorySegment h, final byte[] value) {
    try (Arena a = Arena.ofConfined()) {
      final long id = (long) call(INTERN_STRING, h, a.allocateArray(JAVA_BYTE, value), (long) value.length);
      check((int) Math.min(id, 0), "zbhip_intern_string");
      return id;
    }
  }

  /** zbhip_submit: one window of commands (caller-owned, copied) and their document entries. */
  /**
   * zbhip_doc_merge_order: the merge order of a document's n entries (IndexedDocument's agrona map over
   * the keys' byte offsets) into the entries' pad bytes.
   */
  public static void docMergeOrder(final MemorySegment keyOffsets, final long n, final MemorySegment entries) {
    check((int) call(DOC_MERGE_ORDER, keyOffsets, n, entries), "zbhip_doc_merge_order");
  }

  public static void submit(
      final MemorySegment h, final MemorySegment cmds, final long n, final MemorySegment docs, final long nDocs) {
    check((int) call(SUBMIT, h, cmds, n, docs, nDocs), "zbhip_submit");
  }

  /** zbhip_submit_ex: a window with received cross-partition commands (config 5). */
  public static void submitEx(
      final MemorySegment h,
      final MemorySegment cmds,
      final long n,
      final MemorySegment docs,
      final long nDocs,
      final MemorySegment xparts,
      final long nXparts) {
    check((int) call(SUBMIT_EX, h, cmds, n, docs, nDocs, xparts, nXparts), "zbhip_submit_ex");
  }

  public static int run(final MemorySegment h, final int flags) {
    return check((int) call(RUN, h, flags), "zbhip_run");
  }

  /** ActorClock.currentTimeMillis() of the next window (timer dueDates: CatchEventBehavior.java:310). */
  public static void setClock(final MemorySegment h, final long nowMillis) {
    check((int) call(SET_CLOCK, h, nowMillis), "zbhip_set_clock");
  }

  public static long pendingRecords(final MemorySegment h) {
    return (long) call(PENDING, h);
  }

  /** zbhip_drain into {@code out} (RECORD rows); returns the number of records written. */
  public static long drain(final MemorySegment h, final MemorySegment out, final long cap) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_LONG);
      check((int) call(DRAIN, h, out, cap, n), "zbhip_drain");
      return n.get(JAVA_LONG, 0);
    }
  }

  public static long outbox(final MemorySegment h, final MemorySegment out, final long cap) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_LONG);
      check((int) call(OUTBOX, h, out, cap, n), "zbhip_outbox");
      return n.get(JAVA_LONG, 0);
    }
  }

  /**
   * zbhip_outbox_command: the cross-partition commands window command i sent (XPART rows, its batch's
   * post-commit side effects in batch order); returns a segment of exactly those rows.
   */
  public static MemorySegment outboxCommand(final MemorySegment h, final long i, final Arena arena) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_LONG);
      MemorySegment out = arena.allocate(XPART.byteSize() * 4, 16);
      int rc = (int) call(OUTBOX_COMMAND, h, i, out, 4L, n);
      if (rc == ENOMEM) {
        out = arena.allocate(XPART.byteSize() * n.get(JAVA_LONG, 0), 16);
        rc = (int) call(OUTBOX_COMMAND, h, i, out, n.get(JAVA_LONG, 0), n);
      }
      check(rc, "zbhip_outbox_command");
      return out.asSlice(0, XPART.byteSize() * n.get(JAVA_LONG, 0));
    }
  }

  /** Status of window command i: 0 processed on the device, else the fallback reason. */
  public static int commandStatus(final MemorySegment h, final long i) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment st = a.allocate(JAVA_INT);
      final MemorySegment why = a.allocate(JAVA_INT);
      check((int) call(STATUS, h, i, st, why), "zbhip_command_status");
      return st.get(JAVA_INT, 0) == 0 ? 0 : Math.max(1, why.get(JAVA_INT, 0));
    }
  }

  /** Key -> (instance slot, ordinal) packed as slot << 16 | ordinal; -1 when the key is unknown. */
  public static long resolveKey(final MemorySegment h, final long key) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment inst = a.allocate(JAVA_INT);
      final MemorySegment ord = a.allocate(JAVA_SHORT);
      final int rc = (int) call(RESOLVE, h, key, inst, ord);
      if (rc < 0) {
        return -1;
      }
      return ((long) inst.get(JAVA_INT, 0) << 16) | (ord.get(JAVA_SHORT, 0) & 0xFFFF);
    }
  }

  public static String rejectionReason(final MemorySegment h, final MemorySegment record) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment buf = a.allocate(1024);
      check((int) call(REASON, h, record, buf, 1024L), "zbhip_rejection_reason");
      return buf.getUtf8String(0);
    }
  }

  /** The errorMessage of a drained INCIDENT record (zbhip_incident_message). */
  public static String incidentMessage(final MemorySegment h, final MemorySegment record) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment buf = a.allocate(4096);
      final long n = (long) call(INCIDENT_MESSAGE, h, record, buf, 4096L);
      check(n < 0 ? (int) n : 0, "zbhip_incident_message");
      final byte[] b = buf.asSlice(0, Math.min(n, 4096L)).toArray(JAVA_BYTE);
      return new String(b, java.nio.charset.StandardCharsets.UTF_8);
    }
  }

  public static long stat(final MemorySegment h, final String field) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment s = a.allocate(STATS);
      check((int) call(STATS_FN, h, s), "zbhip_get_stats");
      return s.get(JAVA_LONG, STATS.byteOffset(MemoryLayout.PathElement.groupElement(field)));
    }
  }

  /** zbhip_export_instances_db + zbhip_evict_instances: the fallback hand-off of one instance. */
  public static void handOff(final MemorySegment h, final int instance, final DbSink sink) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment ids = a.allocateArray(JAVA_INT, instance);
      final MemorySegment stub = sinkStub(a, sink);
      check((int) call(EXPORT_INSTANCES_DB, h, ids, 1L, stub, MemorySegment.NULL), "zbhip_export_instances_db");
      check((int) call(EVICT, h, ids, 1L), "zbhip_evict_instances");
    }
  }

  /**
   * A correlation key's message state moves to the engine (one owner per key): the slot's
   * MESSAGE_SUBSCRIPTION zb-db entries into {@code sink} (RocksDB), then the rows leave the device.
   */
  public static void correlationSlotToEngine(final MemorySegment h, final int slot, final DbSink sink) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment ids = a.allocateArray(JAVA_INT, slot);
      final MemorySegment stub = sinkStub(a, sink);
      check((int) call(EXPORT_SLOTS_DB, h, ids, 1L, stub, MemorySegment.NULL), "zbhip_export_correlation_slots_db");
      check((int) call(EVICT_SLOTS, h, ids, 1L), "zbhip_evict_correlation_slots");
    }
  }

  /** zbhip_export_correlation_slots of one slot: its MESSAGE_SUBSCRIPTION rows as text (the state export format). */
  public static java.util.List<String> exportCorrelationSlotRows(final MemorySegment h, final int slot) {
    final java.util.List<String> rows = new java.util.ArrayList<>();
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment ids = a.allocateArray(JAVA_INT, slot);
      final MemorySegment stub = stateSinkStub(a, rows::add);
      check((int) call(EXPORT_SLOTS, h, ids, 1L, stub, MemorySegment.NULL), "zbhip_export_correlation_slots");
    }
    return rows;
  }

  /** DbKeyGenerator's value before window command i (the keys of everything before it are fixed). */
  public static long keyBefore(final MemorySegment h, final long i) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment k = a.allocate(JAVA_LONG);
      check((int) call(KEY_BEFORE, h, i, k), "zbhip_key_before");
      return k.get(JAVA_LONG, 0);
    }
  }

  /** zbhip_continuations: [first id, count] the last run deferred, in drain order of its unprocessed records. */
  public static long[] continuations(final MemorySegment h) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment first = a.allocate(JAVA_LONG);
      final MemorySegment n = a.allocate(JAVA_LONG);
      check((int) call(CONTINUATIONS, h, first, n), "zbhip_continuations");
      return new long[] {first.get(JAVA_LONG, 0), n.get(JAVA_LONG, 0)};
    }
  }

  public static int pendingContinuations(final MemorySegment h, final int instance) {
    return check((int) call(PENDING_CONTINUATIONS, h, instance), "zbhip_pending_continuations");
  }

  /** DbKeyGenerator's last key on the device (the last window's keys and the declared CPU-engine keys). */
  public static long currentKey(final MemorySegment h) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment k = a.allocate(JAVA_LONG);
      check((int) call(CURRENT_KEY, h, k), "zbhip_current_key");
      return k.get(JAVA_LONG, 0);
    }
  }

  /** KeyGeneratorControls.setKeyIfHigher on the device: keys the CPU engine generated between windows. */
  public static void setKeyIfHigher(final MemorySegment h, final long key) {
    check((int) call(SET_KEY_IF_HIGHER, h, key), "zbhip_set_key_if_higher");
  }

  /**
   * zbhip_activate_jobs (JOB_BATCH:ACTIVATE): {@code cmd} a zbhip_job_activation, {@code jobs} room
   * for {@code cap} zbhip_activated_job rows, {@code result} a zbhip_job_batch.
   */
  public static void activateJobs(
      final MemorySegment h, final MemorySegment cmd, final MemorySegment jobs, final long cap, final MemorySegment result) {
    check((int) call(ACTIVATE_JOBS, h, cmd, jobs, cap, result), "zbhip_activate_jobs");
  }

  /** zbhip_activatable_jobs: the first {@code cap} JOB_ACTIVATABLE keys of a job type on the device, key order. */
  public static long[] activatableJobs(final MemorySegment h, final byte[] type, final int cap) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment keys = a.allocate(JAVA_LONG.byteSize() * Math.max(cap, 1), 8);
      final MemorySegment n = a.allocate(JAVA_LONG);
      check((int) call(ACTIVATABLE_JOBS, h, a.allocateArray(JAVA_BYTE, type), (long) type.length, keys, (long) cap, n),
          "zbhip_activatable_jobs");
      final long[] out = new long[(int) n.get(JAVA_LONG, 0)];
      for (int i = 0; i < out.length; i++) {
        out[i] = keys.getAtIndex(JAVA_LONG, i);
      }
      return out;
    }
  }

  /**
   * zbhip_due_timers: the TIMER:TRIGGER commands of device timers with dueDate <= now (RECORD rows in
   * TIMER_DUE_DATES order) into {@code out}; returns their number, the first dueDate not returned in
   * {@code nextDue[0]} (-1 none).
   */
  public static long dueTimers(final MemorySegment h, final long now, final MemorySegment out, final long cap,
      final long[] nextDue) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_LONG);
      final MemorySegment next = a.allocate(JAVA_LONG);
      check((int) call(DUE_TIMERS, h, now, out, cap, n, next), "zbhip_due_timers");
      nextDue[0] = next.get(JAVA_LONG, 0);
      return n.get(JAVA_LONG, 0);
    }
  }

  /**
   * zbhip_timed_out_jobs: the JOB:TIME_OUT commands of activated device jobs with deadline < now;
   * {@code nextDeadline[0]} = the deadline of the first one left out (-1: none).
   */
  public static long timedOutJobs(final MemorySegment h, final long now, final MemorySegment out, final long cap,
      final long[] nextDeadline) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_LONG);
      final MemorySegment next = a.allocate(JAVA_LONG);
      check((int) call(TIMED_OUT_JOBS, h, now, out, cap, n, next), "zbhip_timed_out_jobs");
      nextDeadline[0] = next.get(JAVA_LONG, 0);
      return n.get(JAVA_LONG, 0);
    }
  }

  /**
   * zbhip_time_out_job: JOB:TIMED_OUT (then the push of a job stream's type, JOB_BATCH:ACTIVATED) or the
   * rejection of a device job into {@code out} (room for 2 RECORD rows); returns the number of rows.
   */
  public static long timeOutJob(final MemorySegment h, final long jobKey, final long now, final MemorySegment out) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_LONG);
      check((int) call(TIME_OUT_JOB, h, jobKey, now, out, out.byteSize() / RECORD.byteSize(), n),
          "zbhip_time_out_job");
      return n.get(JAVA_LONG, 0);
    }
  }

  /** zbhip_job_fail: the JOB:FAIL command's fields (JobRecord retries / retryBackoff / errorMessage). */
  public static final StructLayout JOB_FAIL =
      MemoryLayout.structLayout(
          JAVA_LONG.withName("job_key"),
          JAVA_LONG.withName("retry_backoff"),
          JAVA_LONG.withName("timestamp"),
          ADDRESS.withName("error_message"),
          JAVA_LONG.withName("error_message_len"),
          JAVA_INT.withName("retries"),
          JAVA_INT.withName("n_variables"));

  /**
   * zbhip_fail_job (JobFailProcessor): JOB:FAILED (+ the push, or INCIDENT:CREATED JOB_NO_RETRIES) or the
   * rejection into {@code out} (room for 2 rows); returns the number of rows, or -1 when the command is
   * outside the device subset (variables, a back-off with retries left) and the engine must process it.
   */
  public static long failJob(final MemorySegment h, final long jobKey, final int retries, final long retryBackoff,
      final byte[] errorMessage, final int nVariables, final long timestamp, final MemorySegment out) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment cmd = a.allocate(JOB_FAIL);
      final MemorySegment msg = a.allocate(Math.max(1, errorMessage.length));
      MemorySegment.copy(errorMessage, 0, msg, JAVA_BYTE, 0, errorMessage.length);
      cmd.set(JAVA_LONG, 0, jobKey);
      cmd.set(JAVA_LONG, 8, retryBackoff);
      cmd.set(JAVA_LONG, 16, timestamp);
      cmd.set(ADDRESS, 24, msg);
      cmd.set(JAVA_LONG, 32, errorMessage.length);
      cmd.set(JAVA_INT, 40, retries);
      cmd.set(JAVA_INT, 44, nVariables);
      final MemorySegment n = a.allocate(JAVA_LONG);
      final int rc = (int) call(FAIL_JOB, h, cmd, out, out.byteSize() / RECORD.byteSize(), n);
      if (rc == EUNSUPP) {
        return -1;
      }
      check(rc, "zbhip_fail_job");
      return n.get(JAVA_LONG, 0);
    }
  }

  /**
   * zbhip_set_job_stream (JobStreamer.streamFor): jobs of {@code type} the device creates are activated for
   * the stream's worker and timeout (JOB_BATCH:ACTIVATED after JOB:CREATED) while {@code on}.
   */
  public static void setJobStream(final MemorySegment h, final byte[] type, final byte[] worker, final long timeout,
      final boolean on) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment t = a.allocate(Math.max(1, type.length));
      final MemorySegment w = a.allocate(Math.max(1, worker.length));
      MemorySegment.copy(type, 0, t, JAVA_BYTE, 0, type.length);
      MemorySegment.copy(worker, 0, w, JAVA_BYTE, 0, worker.length);
      check((int) call(SET_JOB_STREAM, h, t, (long) type.length, w, (long) worker.length, timeout, on ? 1 : 0),
          "zbhip_set_job_stream");
    }
  }

  /**
   * zbhip_job_variables: the pushed jobs' zbhip_activated_job rows (their activation and the variables of
   * the stream's fetchVariables, {@code names}: name ids, none = all) into {@code out}.
   */
  public static void jobVariables(final MemorySegment h, final MemorySegment keys, final long n,
      final MemorySegment names, final long nNames, final MemorySegment out) {
    check((int) call(JOB_VARIABLES, h, keys, n, names, nNames, out), "zbhip_job_variables");
  }

  /** zbhip_job_state: 0 ACTIVATABLE, 1 ACTIVATED, 2 FAILED, 3 gone, -1 not a device job. */
  public static int jobState(final MemorySegment h, final long jobKey) {
    return (int) call(JOB_STATE, h, jobKey);
  }

  /** Room for the records of one command: returns a buffer of at least n RECORD rows. */
  public interface RecordBuffer {
    MemorySegment ofAtLeast(long n);
  }

  /** zbhip_drain_command: the records of window command i into {@code buffer}; returns their number. */
  public static long drainCommand(final MemorySegment h, final long i, final RecordBuffer buffer) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_LONG);
      MemorySegment out = buffer.ofAtLeast(256);
      int rc = (int) call(DRAIN_COMMAND, h, i, out, out.byteSize() / 80, n);
      if (rc == ENOMEM) { // more records than the buffer: n holds how many
        out = buffer.ofAtLeast(n.get(JAVA_LONG, 0));
        rc = (int) call(DRAIN_COMMAND, h, i, out, out.byteSize() / 80, n);
      }
      check(rc, "zbhip_drain_command");
      return n.get(JAVA_LONG, 0);
    }
  }

  /** zbhip_string_value: the bytes of value-dictionary string {@code id}. */
  public static byte[] stringValue(final MemorySegment h, final long id) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment len = a.allocate(JAVA_LONG);
      final MemorySegment p = (MemorySegment) call(STRING_VALUE, h, (int) id, len);
      return p.reinterpret(len.get(JAVA_LONG, 0)).toArray(JAVA_BYTE);
    }
  }

  /** zbhip_select_instances_db: marks in {@code take} the entries of the instances the device takes over. */
  public static int selectInstancesDb(
      final MemorySegment h,
      final MemorySegment entries,
      final long len,
      final MemorySegment exclude,
      final long nExclude,
      final MemorySegment take,
      final long nTake) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_LONG);
      return check((int) call(SELECT_INSTANCES_DB, h, entries, len, exclude, nExclude, take, nTake, n),
          "zbhip_select_instances_db");
    }
  }

  public static void setExternalKeys(final MemorySegment h, final long i, final int n) {
    check((int) call(EXTERNAL_KEYS, h, i, n), "zbhip_set_external_keys");
  }

  /** zb-db entries ({u32 cf, u32 key length, u32 value length, key, value}*) back into HBM. */
  public static int importStateDb(final MemorySegment h, final MemorySegment entries, final long len, final int firstSlot) {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment n = a.allocate(JAVA_INT);
      check((int) call(IMPORT_DB, h, entries, len, firstSlot, n), "zbhip_import_state_db");
      return n.get(JAVA_INT, 0);
    }
  }

  /** Deployment string-table entry (element ids, job types) of process p. */
  public static String string(final MemorySegment h, final int process, final int index) {
    return ((MemorySegment) call(STRING, h, process, index)).reinterpret(Long.MAX_VALUE).getUtf8String(0);
  }

  /** Partition name dictionary (variable names, message names, bpmnProcessIds of config 5). */
  public static String name(final MemorySegment h, final int id) {
    return ((MemorySegment) call(NAME, h, id)).reinterpret(Long.MAX_VALUE).getUtf8String(0);
  }

  private static MemorySegment sinkStub(final Arena a, final DbSink sink) {
    try {
      final MethodHandle target =
          MethodHandles.lookup()
              .findStatic(
                  ZbHip.class,
                  "sinkTrampoline",
                  MethodType.methodType(
                      void.class, DbSink.class, MemorySegment.class, int.class, MemorySegment.class, long.class,
                      MemorySegment.class, long.class))
              .bindTo(sink);
      return LINKER.upcallStub(target, DB_SINK, a);
    } catch (final ReflectiveOperationException e) {
      throw new IllegalStateException(e);
    }
  }

  /** The zbhip_state_sink upcall: (ctx, NUL-terminated row). */
  private static final FunctionDescriptor STATE_SINK = FunctionDescriptor.ofVoid(ADDRESS, ADDRESS);

  private static MemorySegment stateSinkStub(final Arena a, final java.util.function.Consumer<String> rows) {
    try {
      final MethodHandle target =
          MethodHandles.lookup()
              .findStatic(ZbHip.class, "stateSinkTrampoline",
                  MethodType.methodType(void.class, java.util.function.Consumer.class, MemorySegment.class,
                      MemorySegment.class))
              .bindTo(rows);
      return LINKER.upcallStub(target, STATE_SINK, a);
    } catch (final ReflectiveOperationException e) {
      throw new IllegalStateException(e);
    }
  }

  @SuppressWarnings({"unused", "unchecked"})
  private static void stateSinkTrampoline(
      final java.util.function.Consumer<String> rows, final MemorySegment ctx, final MemorySegment row) {
    rows.accept(row.reinterpret(Long.MAX_VALUE).getUtf8String(0));
  }

  @SuppressWarnings("unused")
  private static void sinkTrampoline(
      final DbSink sink,
      final MemorySegment ctx,
      final int cf,
      final MemorySegment key,
      final long keyLen,
      final MemorySegment value,
      final long valueLen) {
    sink.entry(
        cf,
        key.reinterpret(keyLen).toArray(JAVA_BYTE),
        value.reinterpret(valueLen).toArray(JAVA_BYTE));
  }

  static String utf8(final byte[] b) {
    return new String(b, StandardCharsets.UTF_8);
  }

  /** A negative zbhip status code. */
  public static final class ZbHipException extends RuntimeException {
    public final int code;

    ZbHipException(final String what, final int code) {
      super(what + " failed: " + code);
      this.code = code;
    }
  }
}
