"""Host-side mirror of the reference's processing interface for the BPMN element-lifecycle
hot path, driving libzbhip.so (gfx950).

* :class:`Partition` -- one partition handle (the C ABI in include/zbhip.h).
* :class:`GpuRecordProcessor` -- the stream-platform ``RecordProcessor`` contract
  (stream-platform/.../stream/api/RecordProcessor.java:17-108): ``accepts(value_type)``,
  ``process(window)`` returning the follow-up records grouped per source command.
* :class:`EngineRule` -- the test-client surface of the reference's ``EngineRule``
  (engine/src/test/java/io/camunda/zeebe/engine/util/EngineRule.java) so parity tests read
  like the reference's own tests: ``deployment().with_xml_resource(xml).deploy()``,
  ``process_instance().of_bpmn_process_id(id).with_variable(k, v).create()``,
  ``job().of_instance(pi).with_type(t).complete()``, and RecordingExporter-style queries.
"""
import ctypes as C

import numpy as np

from . import abi
from .native import STATE_SINK, ZbhipError, check, load


class ProcessDefinition:
    def __init__(self, idx, bpmn_process_id, element_ids, element_types, job_types, event_types=None, retries=None,
                 version=1, definition_key=-1, custom_headers=None):
        self.idx = idx
        self.bpmn_process_id = bpmn_process_id
        self.element_ids = element_ids
        self.element_types = element_types
        self.job_types = job_types
        self.event_types = event_types       # BpmnEventType names
        self.retries = retries               # job retries of job worker elements
        self.version = version
        self.definition_key = definition_key
        # zeebe:taskHeaders per element: (key, value) pairs in the order BpmnJobBehavior writes them
        self.custom_headers = custom_headers or [()] * len(element_ids)


class _Csr(C.Structure):  # zbhip_process_csr (include/zbhip.h, ABI 10)
    _fields_ = [("n_elements", C.c_uint32), ("elements", C.c_void_p), ("n_out", C.c_uint32),
                ("out_flow", C.c_void_p), ("n_conditions", C.c_uint32), ("cond_begin", C.c_void_p),
                ("n_code", C.c_uint32), ("code", C.c_void_p), ("n_strings", C.c_uint32),
                ("strings", C.POINTER(C.c_char_p)), ("none_start", C.c_uint16), ("n_join_slots", C.c_uint16),
                ("process_definition_key", C.c_int64), ("version", C.c_int32), ("bpmn_process_id", C.c_uint16),
                ("pad", C.c_uint16), ("cond_text", C.c_void_p), ("n_mappings", C.c_uint32), ("mappings", C.c_void_p),
                ("header_begin", C.POINTER(C.c_uint32)), ("header_bytes", C.c_void_p)]


def msgpack_string_map(b):
    """The (key, value) pairs of a msgpack map of strings (a job's customHeaders), in stored order."""
    def ln(i, fix, fixmask):
        t = b[i]
        if t & ~fixmask == fix:
            return t & fixmask, i + 1
        w = {0xD9: 1, 0xDA: 2, 0xDB: 4, 0xDE: 2, 0xDF: 4}[t]
        return int.from_bytes(b[i + 1:i + 1 + w], "big"), i + 1 + w
    n, i = ln(0, 0x80, 0x0F)
    out = []
    for _ in range(n):
        kv = []
        for _ in range(2):
            m, i = ln(i, 0xA0, 0x1F)
            kv.append(b[i:i + m].decode())
            i += m
        out.append(tuple(kv))
    return tuple(out)


ELEMENT_DTYPE = np.dtype([("element_type", "u1"), ("event_type", "u1"), ("out_begin", "<u2"), ("out_count", "<u2"),
                          ("in_count", "<u2"), ("flow_source", "<u2"), ("flow_target", "<u2"), ("condition", "<u2"),
                          ("default_flow", "<u2"), ("job_type", "<u2"), ("job_retries", "<u2"), ("join_slot", "<u2"),
                          ("id", "<u2"), ("message_name", "<u2"), ("correlation_var", "<u2"),
                          ("flow_scope", "<u2"), ("start_event", "<u2"), ("duration_ms", "<u4")])


class Partition:
    """One Zeebe partition executed on one MI355X (a libzbhip handle)."""

    def __init__(self, partition_id=1, partition_count=1, device=0, max_instances=1 << 16, max_commands=1 << 16,
                 max_records_per_batch=64, max_doc_entries=0, max_commands_in_batch=100, initial_key=0, stream=None,
                 max_correlation_keys=0, trusted_device_windows=False, defer_continuations=False):
        self.L = load()
        cfg = abi.Config(partition_id=partition_id, partition_count=partition_count, device=device,
                         max_commands_in_batch=max_commands_in_batch, max_instances=max_instances,
                         max_commands=max_commands, max_records_per_batch=max_records_per_batch,
                         max_doc_entries=max_doc_entries, initial_key=initial_key, stream=stream,
                         max_correlation_keys=max_correlation_keys,
                         flags=(abi.OPEN_TRUSTED_DEVICE_WINDOWS if trusted_device_windows else 0)
                         | (abi.OPEN_DEFER_CONTINUATIONS if defer_continuations else 0))
        h = C.c_void_p()
        check(self.L.zbhip_open(C.byref(cfg), C.byref(h)), "zbhip_open")
        self.h = h
        self.partition_id = partition_id
        self.partition_count = partition_count
        self.device = device
        self.processes = []
        self.max_commands = max_commands

    def close(self):
        if getattr(self, "h", None):
            self.L.zbhip_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    # ---- deployment (host compiler -> CSR -> LDS program arena) ----
    def deploy(self, xml, process_definition_key=2251799813685249, version=1):
        if isinstance(xml, str):
            xml = xml.encode()
        csr = C.c_void_p()
        err = C.create_string_buffer(512)
        check(self.L.zbhip_compile_bpmn(xml, len(xml), process_definition_key, version, C.byref(csr), err, 512),
              err.value.decode())
        try:
            c = C.cast(csr, C.POINTER(_Csr)).contents
            els = np.frombuffer(C.string_at(c.elements, c.n_elements * ELEMENT_DTYPE.itemsize), dtype=ELEMENT_DTYPE)
            strings = [c.strings[i].decode() for i in range(c.n_strings)]
            headers = [()] * c.n_elements
            if c.header_begin:
                hb = [c.header_begin[i] for i in range(c.n_elements + 1)]
                raw = C.string_at(c.header_bytes, hb[-1])
                headers = [msgpack_string_map(raw[hb[e]:hb[e + 1]]) if hb[e + 1] > hb[e] else ()
                           for e in range(c.n_elements)]
            idx = C.c_uint32()
            check(self.L.zbhip_deploy(self.h, csr, C.byref(idx)), "zbhip_deploy")
        finally:
            self.L.zbhip_free_csr(csr)
        pd = ProcessDefinition(idx.value, strings[els[0]["id"]], [strings[i] for i in els["id"]],
                               [abi.ELEMENT_TYPES[t] for t in els["element_type"]],
                               [strings[j] if j != 0xFFFF else None for j in els["job_type"]],
                               [abi.EVENT_TYPES[t] for t in els["event_type"]],
                               [int(r) if j != 0xFFFF else None for r, j in zip(els["job_retries"], els["job_type"])],
                               version, process_definition_key, headers)
        self.processes.append(pd)
        return idx.value

    def intern(self, name):
        return check(self.L.zbhip_intern(self.h, name.encode()))

    def state_db(self):
        """The partition state as zb-db entries (column family ordinal, key bytes, value bytes)."""
        from .logwriter import _db_collector
        out, cb = _db_collector()
        check(self.L.zbhip_export_state_db(self.h, cb, None), "zbhip_export_state_db")
        return sorted(out)

    def serialize_log_device(self, source_positions=None, first_position=1, timestamp=0, copy=True):
        """Log bytes of the last run's window written on the device (zbhip_serialize_log_device):
        the bytes `log_serializer().serialize(drain(), ...)` gives for the same window.  Returns the
        bytes (copy=True) or (device pointer, size) -- written in the handle's stream order
        (zbhip_stream), so a reader on another stream waits on that one first; raises
        ZbhipError(ZBHIP_EUNSUPP) when the window needs the host serialiser."""
        pos = np.ascontiguousarray(source_positions if source_positions is not None
                                   else np.arange(1, self._n_cmds + 1), dtype=np.int64)
        w = abi.LogWindow(None, self._n_cmds, 0, None, 0, 0, pos.ctypes.data, first_position, timestamp, None)
        ptr, used = C.c_void_p(), C.c_size_t()
        check(self.L.zbhip_serialize_log_device(self.h, C.byref(w), C.byref(ptr), C.byref(used)),
              "zbhip_serialize_log_device")
        if not copy:
            return ptr.value, used.value
        out = C.create_string_buffer(max(used.value, 1))
        check(self.L.zbhip_log_device_copy(self.h, out, used.value), "zbhip_log_device_copy")
        return out.raw[:used.value]

    def log_copy_async(self, used):
        """zbhip_log_copy_async: the last serialised window's `used` bytes on their way into the handle's
        pinned buffer; returns the host address (complete after log_copy_wait(address))."""
        ptr = C.c_void_p()
        check(self.L.zbhip_log_copy_async(self.h, used, C.byref(ptr)), "zbhip_log_copy_async")
        return ptr.value

    def log_copy_wait(self, address=None, used=None):
        """zbhip_log_copy_wait; with `used`, returns the bytes at `address`."""
        check(self.L.zbhip_log_copy_wait(self.h, address), "zbhip_log_copy_wait")
        return C.string_at(address, used) if used is not None else None

    def log_serializer(self):
        """The partition's log serialiser (follows its deployments and dictionaries)."""
        from .logwriter import LogSerializer
        return LogSerializer(self)

    def name(self, nid):
        return self.L.zbhip_name(self.h, nid).decode()

    def element_id(self, proc, elem):
        return self.processes[proc].element_ids[elem]

    # ---- commands ----
    def submit(self, cmds, docs=None, xparts=None):
        cmds = np.ascontiguousarray(cmds, dtype=abi.COMMAND_DTYPE)
        docs = np.ascontiguousarray(docs if docs is not None else abi.make_docs(0), dtype=abi.DOC_DTYPE)
        xp = np.ascontiguousarray(xparts if xparts is not None else abi.make_xparts(0), dtype=abi.XPART_DTYPE)
        check(self.L.zbhip_submit_ex(self.h, cmds.ctypes.data, len(cmds), docs.ctypes.data, len(docs),
                                     xp.ctypes.data if len(xp) else None, len(xp)), "zbhip_submit")
        self._n_cmds = len(cmds)

    def submit_device(self, cmd_ptr, n, doc_ptr=0, n_docs=0, xpart_ptr=0, n_xparts=0):
        """Commands already resident in HBM (e.g. a torch uint8 tensor's data_ptr())."""
        check(self.L.zbhip_submit_device_ex(self.h, cmd_ptr, n, doc_ptr or None, n_docs, xpart_ptr or None, n_xparts),
              "zbhip_submit_device")
        self._n_cmds = n

    # ---- value dictionary (correlation keys) ----
    def intern_string(self, value):
        b = value.encode() if isinstance(value, str) else value
        return check(self.L.zbhip_intern_string(self.h, b, len(b)), "zbhip_intern_string")

    def intern_strings(self, values):
        bs = [v.encode() if isinstance(v, str) else v for v in values]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs])
        blob = b"".join(bs)
        ids = np.zeros(len(bs), dtype=np.uint32)
        check(self.L.zbhip_intern_strings(self.h, blob, off.ctypes.data, len(bs), ids.ctypes.data), "intern_strings")
        return ids

    def string_value(self, sid):
        return self.L.zbhip_string_value(self.h, sid, None).decode()

    # ---- cross-partition outbox (SubscriptionCommandSender sends) ----
    def outbox(self):
        n = C.c_size_t()
        check(self.L.zbhip_outbox(self.h, None, 0, C.byref(n)), "zbhip_outbox")
        out = abi.make_xparts(n.value)
        if n.value:
            check(self.L.zbhip_outbox(self.h, out.ctypes.data, n.value, C.byref(n)), "zbhip_outbox")
        return out

    def outbox_command(self, i, cap=8):
        """The cross-partition commands window command i sent (zbhip_outbox_command)."""
        out = abi.make_xparts(cap)
        n = C.c_size_t()
        rc = self.L.zbhip_outbox_command(self.h, i, out.ctypes.data, cap, C.byref(n))
        if rc == -2 and n.value > cap:
            return self.outbox_command(i, n.value)
        check(rc, "zbhip_outbox_command")
        return out[: n.value]

    def outbox_copy(self, dev_dst, first, count):
        check(self.L.zbhip_outbox_copy(self.h, dev_dst, first, count), "zbhip_outbox_copy")

    def submit_xparts_device(self, dev_xparts, n):
        """The exchange's receiving side: a window of n received commands already in HBM."""
        check(self.L.zbhip_submit_xparts_device(self.h, dev_xparts or None, n), "zbhip_submit_xparts_device")

    def string_partitions(self, ids, partition_count):
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        out = np.zeros(len(ids), dtype=np.int32)
        check(self.L.zbhip_string_partitions(self.h, ids.ctypes.data, len(ids), partition_count, out.ctypes.data))
        return out

    def outbox_device(self):
        """(device pointer, per-target counts) of the outbox bucketed by target partition."""
        ptr = C.c_void_p()
        counts = np.zeros(max(1, self.partition_count), dtype=np.uint32)
        check(self.L.zbhip_outbox_device(self.h, C.byref(ptr), counts.ctypes.data), "zbhip_outbox_device")
        return ptr.value or 0, counts

    def torch_stream(self):
        """The partition's HIP stream as a torch stream: device work that must be ordered with the
        partition's launches (exchange buffers, collectives) is issued on it."""
        import torch
        if getattr(self, "_tstream", None) is None:
            self._tstream = torch.cuda.ExternalStream(self.L.zbhip_stream(self.h), device=torch.device("cuda", self.device))
        return self._tstream

    def outbox_device_async(self, dev_counts):
        """Device pointer of the bucketed outbox; the per-target counts (uint32) are copied to the
        device buffer dev_counts on the partition's stream (no host wait)."""
        ptr = C.c_void_p()
        check(self.L.zbhip_outbox_device_async(self.h, C.byref(ptr), dev_counts), "zbhip_outbox_device_async")
        return ptr.value or 0

    def run(self, flags=0):
        return check(self.L.zbhip_run(self.h, flags), "zbhip_run")

    def set_clock(self, now_ms):
        """ActorClock.currentTimeMillis() for the next runs (timer catch events' due dates)."""
        check(self.L.zbhip_set_clock(self.h, int(now_ms)), "zbhip_set_clock")

    def drain(self, out=None):
        """The window's records in log order; `out` (a RECORD_DTYPE array) is reused when it is
        large enough, so a host loop over windows does not fault in fresh pages every time.  The
        result is then a view of `out`: it is only valid until the next drain into the same buffer
        (callers that keep records, like EngineRule, copy them)."""
        n = self.L.zbhip_pending_records(self.h)
        # every field of a drained record is written by zbhip_drain: no zero fill (a window of
        # 10^6 linear-10 commands drains ~0.9 GB)
        if out is None or len(out) < n:
            out = np.empty(max(n, 0), dtype=abi.RECORD_DTYPE)
        got = C.c_size_t()
        check(self.L.zbhip_drain(self.h, out.ctypes.data if n else None, n, C.byref(got)), "zbhip_drain")
        return out[: got.value]

    def drain_command(self, i, cap=256):
        """The records of window command i (zbhip_drain_command)."""
        out = np.empty(cap, dtype=abi.RECORD_DTYPE)
        n = C.c_size_t()
        rc = self.L.zbhip_drain_command(self.h, i, out.ctypes.data, cap, C.byref(n))
        if rc == -2 and n.value > cap:
            return self.drain_command(i, n.value)
        check(rc, "zbhip_drain_command")
        return out[: n.value]

    def drain_chunks(self, chunk=1 << 22):
        """The window's records in log order, `chunk` at a time (bounded host memory for windows of
        10^7 commands); every yielded view is overwritten by the next one."""
        out = np.empty(chunk, dtype=abi.RECORD_DTYPE)
        got = C.c_size_t()
        while True:
            check(self.L.zbhip_drain(self.h, out.ctypes.data, chunk, C.byref(got)), "zbhip_drain")
            if got.value == 0:
                return
            yield out[: got.value]

    def reason(self, rec):
        r = abi.Record()
        for f, _ in abi.Record._fields_:
            if f != "pad":
                setattr(r, f, int(rec[f]))
        buf = C.create_string_buffer(512)
        self.L.zbhip_rejection_reason(self.h, C.byref(r), buf, 512)
        return buf.value.decode()

    def incident_message(self, rec):
        """errorMessage of a drained INCIDENT record (zbhip_incident_message)."""
        r = abi.Record()
        for f, _ in abi.Record._fields_:
            if f != "pad":
                setattr(r, f, int(rec[f]))
        cap = 1024
        while True:
            buf = C.create_string_buffer(cap)
            n = self.L.zbhip_incident_message(self.h, C.byref(r), buf, cap)
            if n < 0:
                raise ZbhipError(n, "zbhip_incident_message")
            if n <= cap:
                return buf.raw[:n].decode()
            cap = n  # the full length: call again with room for it

    def stats(self):
        s = abi.Stats()
        check(self.L.zbhip_get_stats(self.h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in abi.Stats._fields_}

    def state(self):
        rows = []
        cb = STATE_SINK(lambda ctx, row: rows.append(row.decode()))
        check(self.L.zbhip_export_state(self.h, cb, None), "zbhip_export_state")
        return sorted(rows)

    # ---- fallback hand-off to the CPU engine (include/zbhip.h) ----
    def export_instances(self, instances):
        rows = []
        cb = STATE_SINK(lambda ctx, row: rows.append(row.decode()))
        ids = np.ascontiguousarray(instances, dtype=np.uint32)
        check(self.L.zbhip_export_instances(self.h, ids.ctypes.data, len(ids), cb, None), "zbhip_export_instances")
        return sorted(rows)

    def export_instances_db(self, instances):
        from .logwriter import _db_collector
        out, cb = _db_collector()
        ids = np.ascontiguousarray(instances, dtype=np.uint32)
        check(self.L.zbhip_export_instances_db(self.h, ids.ctypes.data, len(ids), cb, None), "zbhip_export_instances_db")
        return sorted(out)

    # ---- one owner per correlation key (config 5, include/zbhip.h) ----
    def export_correlation_slots(self, slots):
        """The correlation slots' MESSAGE_SUBSCRIPTION rows (text, the export_state format)."""
        rows = []
        cb = STATE_SINK(lambda ctx, row: rows.append(row.decode()))
        ids = np.ascontiguousarray(slots, dtype=np.uint32)
        check(self.L.zbhip_export_correlation_slots(self.h, ids.ctypes.data, len(ids), cb, None),
              "zbhip_export_correlation_slots")
        return sorted(rows)

    def export_correlation_slots_db(self, slots):
        from .logwriter import _db_collector
        out, cb = _db_collector()
        ids = np.ascontiguousarray(slots, dtype=np.uint32)
        check(self.L.zbhip_export_correlation_slots_db(self.h, ids.ctypes.data, len(ids), cb, None),
              "zbhip_export_correlation_slots_db")
        return sorted(out)

    def evict_correlation_slots(self, slots):
        ids = np.ascontiguousarray(slots, dtype=np.uint32)
        check(self.L.zbhip_evict_correlation_slots(self.h, ids.ctypes.data, len(ids)), "zbhip_evict_correlation_slots")

    def evict_instances(self, instances):
        ids = np.ascontiguousarray(instances, dtype=np.uint32)
        check(self.L.zbhip_evict_instances(self.h, ids.ctypes.data, len(ids)), "zbhip_evict_instances")

    def import_state_db(self, entries, first_slot=0):
        """Loads process instances from zb-db entries [(column family, key, value)] into free slots
        first_slot, ... (process-instance-key order); returns the number of instances."""
        import struct
        blob = b"".join(struct.pack("<III", cf, len(k), len(v)) + bytes(k) + bytes(v) for cf, k, v in entries)
        n = C.c_uint32()
        check(self.L.zbhip_import_state_db(self.h, blob, len(blob), first_slot, C.byref(n)), "zbhip_import_state_db")
        return n.value

    def select_instances_db(self, entries, exclude=()):
        """zbhip_select_instances_db: which of the zb-db entries [(column family, key, value)] belong to
        process instances this partition can take over (recovery); returns (mask, instances)."""
        import struct
        blob = b"".join(struct.pack("<III", cf, len(k), len(v)) + bytes(k) + bytes(v) for cf, k, v in entries)
        ex = np.ascontiguousarray(list(exclude), dtype=np.int64)
        take = np.zeros(max(len(entries), 1), dtype=np.uint8)
        n = C.c_size_t()
        rc = check(self.L.zbhip_select_instances_db(self.h, blob, len(blob), ex.ctypes.data if len(ex) else None, len(ex),
                                                    take.ctypes.data, len(take), C.byref(n)), "zbhip_select_instances_db")
        return take[: n.value].astype(bool), rc

    def import_state(self, rows, first_slot=0):
        text = "\n".join(rows).encode()
        n = C.c_uint32()
        check(self.L.zbhip_import_state(self.h, text, len(text), first_slot, C.byref(n)), "zbhip_import_state")
        return n.value

    def activate_jobs(self, job_type, worker="worker", timeout=300000, max_jobs=10, timestamp=0, variables=(),
                      cap=None):
        """JOB_BATCH:ACTIVATE (JobBatchActivateProcessor): (batch key, activated jobs, rejection reason);
        the key is -1 and the reason 1/2/3 for an invalid command."""
        t, w = job_type.encode(), worker.encode()
        names = np.asarray([self.intern(v) for v in variables], dtype=np.uint32)
        cap = max_jobs if cap is None else cap
        out = np.zeros(max(cap, 1), dtype=abi.ACTIVATED_JOB_DTYPE)
        cmd = abi.JobActivation(type=t, type_len=len(t), worker=w, worker_len=len(w), timeout=timeout,
                                max_jobs=max_jobs, timestamp=timestamp,
                                variables=names.ctypes.data if len(names) else None, n_variables=len(names))
        res = abi.JobBatch()
        check(self.L.zbhip_activate_jobs(self.h, C.byref(cmd), out.ctypes.data, cap, C.byref(res)), "zbhip_activate_jobs")
        return res.key, out[: res.n_jobs], res.reason

    def activatable_jobs(self, job_type, cap=1 << 16):
        """The device's JOB_ACTIVATABLE keys of `job_type` in key order (zbhip_activatable_jobs)."""
        t = job_type.encode()
        keys = np.zeros(max(cap, 1), dtype=np.int64)
        n = C.c_size_t()
        check(self.L.zbhip_activatable_jobs(self.h, t, len(t), keys.ctypes.data, cap, C.byref(n)), "zbhip_activatable_jobs")
        return [int(k) for k in keys[: n.value]]

    def intern_list(self, items):
        """A list value [(zbhip_doc_type, value)] into the list dictionary (zbhip_intern_list): its id."""
        d = abi.make_docs(max(len(items), 1))
        for j, (t, v) in enumerate(items):
            d[j]["type"], d[j]["value"] = t, v
        return check(self.L.zbhip_intern_list(self.h, d.ctypes.data, len(items)), "zbhip_intern_list")

    def list_items(self, list_id):
        """The items [(zbhip_doc_type, value)] of list `list_id` (zbhip_list_items)."""
        n = C.c_size_t()
        check(self.L.zbhip_list_items(self.h, int(list_id), None, 0, C.byref(n)), "zbhip_list_items")
        out = abi.make_docs(max(n.value, 1))
        check(self.L.zbhip_list_items(self.h, int(list_id), out.ctypes.data, n.value, C.byref(n)), "zbhip_list_items")
        return [(int(x["type"]), int(x["value"])) for x in out[: n.value]]

    def job_variables(self, job_keys, variables=()):
        """The pushed jobs' ActivatedJob rows (zbhip_job_variables: activation + variables document)."""
        keys = np.asarray(job_keys, dtype=np.int64)
        names = np.asarray([self.intern(v) for v in variables], dtype=np.uint32)
        out = np.zeros(max(len(keys), 1), dtype=abi.ACTIVATED_JOB_DTYPE)
        check(self.L.zbhip_job_variables(self.h, keys.ctypes.data, len(keys), names.ctypes.data if len(names) else None,
                                         len(names), out.ctypes.data), "zbhip_job_variables")
        return out[: len(keys)]

    def key_before(self, i):
        k = C.c_int64()
        check(self.L.zbhip_key_before(self.h, i, C.byref(k)), "zbhip_key_before")
        return k.value

    def continuations(self):
        """Ids of the continuations the last run deferred, in drain order of the unprocessed records."""
        first, n = C.c_uint64(), C.c_uint64()
        check(self.L.zbhip_continuations(self.h, C.byref(first), C.byref(n)), "zbhip_continuations")
        return range(first.value, first.value + n.value)

    def pending_continuations(self, instance):
        return check(self.L.zbhip_pending_continuations(self.h, instance), "zbhip_pending_continuations")

    def current_key(self):
        k = C.c_int64()
        check(self.L.zbhip_current_key(self.h, C.byref(k)), "zbhip_current_key")
        return k.value

    def set_key_if_higher(self, key):
        check(self.L.zbhip_set_key_if_higher(self.h, key), "zbhip_set_key_if_higher")

    def set_external_keys(self, i, nkeys):
        check(self.L.zbhip_set_external_keys(self.h, i, nkeys), "zbhip_set_external_keys")

    def fallback(self):
        n = C.c_size_t()
        check(self.L.zbhip_fallback(self.h, None, 0, C.byref(n)))
        buf = (C.c_uint32 * max(n.value, 1))()
        check(self.L.zbhip_fallback(self.h, buf, n.value, C.byref(n)))
        return list(buf[: n.value])

    FALLBACK_REASONS = {1: "queue", 2: "table", 3: "records", 4: "keys", 5: "batch-limit", 6: "feel", 7: "vars",
                        8: "slot-in-use", 9: "no-condition", 10: "unsupported", 11: "doc", 12: "join",
                        13: "slots", 14: "bad-process", 15: "message", 16: "fenced", 17: "duplicate"}

    def command_status(self, i):
        st, rs = C.c_uint32(), C.c_uint32()
        check(self.L.zbhip_command_status(self.h, i, C.byref(st), C.byref(rs)))
        return st.value, self.FALLBACK_REASONS.get(rs.value, rs.value)

    # ---- the engine's scheduled tasks over device-held state ----
    def due_timers(self, now, cap=1 << 16):
        """DueDateTimerChecker over the device timers (zbhip_due_timers): (the TIMER:TRIGGER commands as
        RECORD_DTYPE rows in TIMER_DUE_DATES order, the first dueDate not returned or -1)."""
        out = np.zeros(max(cap, 1), dtype=abi.RECORD_DTYPE)
        n, nxt = C.c_size_t(), C.c_int64()
        check(self.L.zbhip_due_timers(self.h, int(now), out.ctypes.data, cap, C.byref(n), C.byref(nxt)),
              "zbhip_due_timers")
        return out[: n.value], nxt.value

    def timed_out_jobs(self, now, cap=1 << 16, with_next=False):
        """JobTimeoutTrigger over the device's activated jobs (zbhip_timed_out_jobs): the JOB:TIME_OUT
        commands (RECORD_DTYPE rows, the stored job) in JOB_DEADLINES order (with_next: and the deadline of
        the first timed-out job not returned, -1 none)."""
        out = np.zeros(max(cap, 1), dtype=abi.RECORD_DTYPE)
        n, nxt = C.c_size_t(), C.c_int64()
        check(self.L.zbhip_timed_out_jobs(self.h, int(now), out.ctypes.data, cap, C.byref(n), C.byref(nxt)),
              "zbhip_timed_out_jobs")
        return (out[: n.value], nxt.value) if with_next else out[: n.value]

    def time_out_job(self, job_key, now):
        """JOB:TIME_OUT of a device job (zbhip_time_out_job): JOB:TIMED_OUT (+ its push) or the rejection,
        RECORD_DTYPE rows."""
        out = np.zeros(2, dtype=abi.RECORD_DTYPE)
        n = C.c_size_t()
        check(self.L.zbhip_time_out_job(self.h, int(job_key), int(now), out.ctypes.data, 2, C.byref(n)),
              "zbhip_time_out_job")
        return out[: n.value]

    def set_job_stream(self, job_type, worker="", timeout=300000, on=True):
        """zbhip_set_job_stream: a job stream of `job_type` (jobs of it are pushed when created)."""
        t, w = job_type.encode(), worker.encode()
        check(self.L.zbhip_set_job_stream(self.h, t, len(t), w, len(w), int(timeout), 1 if on else 0),
              "zbhip_set_job_stream")

    def fail_job(self, job_key, retries, error_message="", retry_backoff=0, n_variables=0, timestamp=0):
        """JOB:FAIL of a device job (zbhip_fail_job): the JOB:FAILED (+ INCIDENT:CREATED) or rejection
        records, RECORD_DTYPE rows; None when the command is outside the device subset (the engine's)."""
        m = error_message.encode()
        cmd = abi.JobFail(job_key=int(job_key), retry_backoff=int(retry_backoff), timestamp=int(timestamp), error_message=m,
                          error_message_len=len(m), retries=int(retries), n_variables=int(n_variables))
        out = np.zeros(2, dtype=abi.RECORD_DTYPE)
        n = C.c_size_t()
        rc = self.L.zbhip_fail_job(self.h, C.byref(cmd), out.ctypes.data, 2, C.byref(n))
        if rc == -5:
            return None
        check(rc, "zbhip_fail_job")
        return out[: n.value]

    def job_state(self, job_key):
        """zbhip_job_state: 0 ACTIVATABLE, 1 ACTIVATED, 2 FAILED, 3 gone, -1 nothing stored."""
        return self.L.zbhip_job_state(self.h, int(job_key))

    def resolve_key(self, key):
        inst, ordv = C.c_uint32(), C.c_uint16()
        check(self.L.zbhip_resolve_key(self.h, key, C.byref(inst), C.byref(ordv)), "unknown key %d" % key)
        return inst.value, ordv.value


class GpuRecordProcessor:
    """The RecordProcessor contract for a window of hot-path commands (see module doc)."""

    ACCEPTED = (abi.VT_PROCESS_INSTANCE_CREATION, abi.VT_JOB)

    def __init__(self, partition):
        self.partition = partition

    def accepts(self, value_type):
        return value_type in self.ACCEPTED

    def process(self, cmds, docs=None):
        """Processes the window to quiescence; returns {source_index: [records]} in log order."""
        self.partition.submit(cmds, docs)
        self.partition.run()
        recs = self.partition.drain()
        out = {}
        for r in recs:
            out.setdefault(int(r["source_index"]), []).append(r)
        return out


# ---------------------------------------------------------------------------------------------
# EngineRule-style client
# ---------------------------------------------------------------------------------------------
class EngineRule:
    """Single-partition test engine on the GPU (EngineRule.singlePartition)."""

    def __init__(self, partition=None, **kw):
        self.partition = partition or Partition(**kw)
        self.records = []       # RecordingExporter: every drained record, in log order
        self.reasons = {}
        self._next_instance = 0
        self._pi_instance = {}  # process instance key -> instance slot
        self._by_id = {}

    @classmethod
    def single_partition(cls, **kw):
        return cls(**kw)

    # deployment().withXmlResource(xml).deploy()
    def deployment(self):
        rule = self

        class _D:
            def __init__(self):
                self.xml = None

            def with_xml_resource(self, xml):
                self.xml = xml
                return self

            def deploy(self):
                idx = rule.partition.deploy(self.xml)
                rule._by_id[rule.partition.processes[idx].bpmn_process_id] = idx
                return idx

        return _D()

    def _execute(self, cmds, docs=None):
        self.partition.submit(cmds, docs)
        self.partition.run()
        recs = self.partition.drain()
        base = len(self.records)
        for i, r in enumerate(recs):
            if r["record_type"] == abi.RT_REJECTION:
                self.reasons[base + i] = self.partition.reason(r)
        self.records.extend(recs)
        return recs

    def process_instance(self):
        rule = self

        class _P:
            def __init__(self):
                self.proc = None
                self.vars = []

            def of_bpmn_process_id(self, pid):
                self.proc = rule._by_id[pid]
                return self

            def with_variable(self, name, value):
                self.vars.append((name, value))
                return self

            def create(self):
                inst = rule._next_instance
                rule._next_instance += 1
                cmds = abi.make_commands(1)
                cmds["instance"] = inst
                cmds["kind"] = abi.CMD_CREATE
                cmds["ref"] = self.proc
                docs = abi.make_docs(len(self.vars))
                for j, (n, v) in enumerate(self.vars):
                    docs[j]["name_id"] = rule.partition.intern(n)
                    if isinstance(v, bool):
                        docs[j]["type"], docs[j]["value"] = abi.DOC_BOOL, int(v)
                    elif isinstance(v, int):
                        docs[j]["type"], docs[j]["value"] = abi.DOC_INT, v
                    else:
                        docs[j]["type"], docs[j]["value"] = abi.DOC_DEC, int(round(v * 10 ** abi.DEC_SCALE))
                cmds["doc_count"] = len(self.vars)
                recs = rule._execute(cmds, docs)
                created = [r for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE_CREATION]
                pi = int(created[0]["process_instance_key"])
                rule._pi_instance[pi] = inst
                return pi

        return _P()

    def job(self):
        rule = self

        class _J:
            def __init__(self):
                self.pi = None
                self.type = None
                self.key = None

            def of_instance(self, pi):
                self.pi = pi
                return self

            def with_type(self, t):
                self.type = t
                return self

            def with_key(self, k):
                self.key = k
                return self

            def complete(self):
                key = self.key
                if key is None:
                    created = [r for r in rule.records if r["value_type"] == abi.VT_JOB and r["intent"] == 0
                               and int(r["process_instance_key"]) == self.pi and
                               rule.partition.processes[int(r["process_idx"])].job_types[int(r["element_idx"])]
                               == self.type]
                    key = int(created[-1]["key"])
                inst, ordv = rule.partition.resolve_key(key)
                cmds = abi.make_commands(1)
                cmds["instance"] = inst
                cmds["kind"] = abi.CMD_JOB_COMPLETE
                cmds["ref"] = ordv
                return rule._execute(cmds)

        return _J()

    # RecordingExporter.processInstanceRecords() as (elementId, intent-name) pairs
    def process_instance_records(self, only_events=False):
        out = []
        for r in self.records:
            if r["value_type"] != abi.VT_PROCESS_INSTANCE:
                continue
            if only_events and r["record_type"] != abi.RT_EVENT:
                continue
            out.append((self.partition.element_id(int(r["process_idx"]), int(r["element_idx"])),
                        abi.PI_INTENTS[int(r["intent"])]))
        return out


__all__ = ["Partition", "GpuRecordProcessor", "EngineRule", "ZbhipError"]
