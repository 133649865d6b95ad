"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (oracle/zb_oracle.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product (zeebe_amd) never does.  Parity is pinned by the
golden vectors in tests/golden/ (the Java reference cannot run in this image).
"""
import ctypes as C
import os
import subprocess

import numpy as np

from zeebe_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB selects another build of the same sources (scripts/sanitize.sh: the ASan build)
LIB = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "zb_oracle.cpp")):
            build()
        L = C.CDLL(LIB)
        L.zbo_new.restype = C.c_void_p
        L.zbo_new.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int64]
        L.zbo_free.argtypes = [C.c_void_p]
        L.zbo_last_error.restype = C.c_char_p
        L.zbo_last_error.argtypes = [C.c_void_p]
        L.zbo_deploy_xml.argtypes = [C.c_void_p, C.c_char_p, C.c_int64, C.c_int]
        L.zbo_intern.argtypes = [C.c_void_p, C.c_char_p]
        L.zbo_name.restype = C.c_char_p
        L.zbo_element_job_type.restype = C.c_char_p
        L.zbo_element_job_type.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.zbo_element_headers.restype = C.c_int
        L.zbo_element_headers.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.c_int]
        L.zbo_element_cond_text.restype = C.c_char_p
        L.zbo_element_cond_text.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.zbo_process_info.restype = C.c_char_p
        L.zbo_process_info.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.zbo_element_info.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.zbo_n_names.argtypes = [C.c_void_p]
        L.zbo_n_strings.argtypes = [C.c_void_p]
        L.zbo_string_value.restype = C.c_void_p
        L.zbo_string_value.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_size_t)]
        L.zbo_n_processes.argtypes = [C.c_void_p]
        L.zbo_name.argtypes = [C.c_void_p, C.c_int]
        L.zbo_n_elements.argtypes = [C.c_void_p, C.c_int]
        L.zbo_element_id.restype = C.c_char_p
        L.zbo_element_id.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.zbo_submit.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.zbo_run.argtypes = [C.c_void_p]
        L.zbo_activate_jobs.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int64, C.c_int, C.c_int64, C.c_char_p,
                                        C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                        C.POINTER(C.c_int64)]
        L.zbo_set_job_stream.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int64, C.c_int]
        L.zbo_job_variables.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_void_p]
        L.zbo_set_job_stream.restype = None
        L.zbo_key_counter.restype = C.c_int64
        L.zbo_key_counter.argtypes = [C.c_void_p]
        L.zbo_set_key_counter.argtypes = [C.c_void_p, C.c_int64]
        L.zbo_process_one.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.c_int64, C.c_int]
        L.zbo_import_rows.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        L.zbo_ordinal_of.restype = C.c_int64
        L.zbo_ordinal_of.argtypes = [C.c_void_p, C.c_uint32, C.c_int64]
        L.zbo_n_records.restype = C.c_size_t
        L.zbo_n_records.argtypes = [C.c_void_p]
        L.zbo_records.restype = C.c_size_t
        L.zbo_records.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.zbo_reason.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t]
        L.zbo_set_clock.argtypes = [C.c_void_p, C.c_int64]
        L.zbo_set_clock.restype = None
        L.zbo_clear_records.argtypes = [C.c_void_p]
        L.zbo_resolve.restype = C.c_int64
        L.zbo_resolve.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.zbo_state.restype = C.c_size_t
        L.zbo_state.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        L.zbo_fallback.restype = C.c_size_t
        L.zbo_fallback.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.zbo_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint64)]
        L.zbo_submit_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p,
                                    C.c_size_t]
        L.zbo_intern_string.restype = C.c_int64
        L.zbo_intern_string.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        L.zbo_intern_list.restype = C.c_int64
        L.zbo_intern_list.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.zbo_list_items.restype = C.c_size_t
        L.zbo_list_items.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_size_t]
        L.zbo_outbox.restype = C.c_size_t
        L.zbo_outbox.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.zbo_clear_outbox.argtypes = [C.c_void_p]
        L.zbo_take_notified.restype = C.c_size_t
        L.zbo_take_notified.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        L.zbo_subscription_partition.argtypes = [C.c_char_p, C.c_size_t, C.c_int]
        L.zbo_java_hash.restype = C.c_int32
        L.zbo_java_hash.argtypes = [C.c_char_p, C.c_size_t]
        L.zbo_bench_msg.restype = C.c_double
        L.zbo_bench_msg.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.zbo_bench_jobs.restype = C.c_double
        L.zbo_bench_jobs.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_uint64,
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.zbo_bench.restype = C.c_double
        L.zbo_bench.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    pass


class Oracle:
    """One partition of the CPU restatement (EngineRule.singlePartition analogue)."""

    def __init__(self, partition_id=1, partition_count=1, max_commands_in_batch=100, initial_key=0):
        self.L = lib()
        self.h = self.L.zbo_new(partition_id, partition_count, max_commands_in_batch, initial_key)
        self.partition_id = partition_id

    def close(self):
        if self.h:
            self.L.zbo_free(self.h)
            self.h = None

    __del__ = close

    def deploy(self, xml, process_definition_key=2251799813685249, version=1):
        if isinstance(xml, str):
            xml = xml.encode()
        r = self.L.zbo_deploy_xml(self.h, xml, process_definition_key, version)
        if r < 0:
            raise OracleError(self.L.zbo_last_error(self.h).decode())
        return r

    def intern(self, name):
        return self.L.zbo_intern(self.h, name.encode())

    def name(self, nid):
        return self.L.zbo_name(self.h, nid).decode()

    def element_id(self, proc, elem):
        return self.L.zbo_element_id(self.h, proc, elem).decode()

    def set_clock(self, now_ms):
        """ActorClock.currentTimeMillis() for the next windows (timer due dates)."""
        self.L.zbo_set_clock(self.h, int(now_ms))

    def element_type(self, proc, elem):
        t, ev, r = C.c_int(), C.c_int(), C.c_int()
        self.L.zbo_element_info(self.h, proc, elem, C.byref(t), C.byref(ev), C.byref(r))
        return t.value

    def string_value(self, sid):
        n = C.c_size_t()
        p = self.L.zbo_string_value(self.h, sid, C.byref(n))
        return C.string_at(p, n.value)

    def strings(self):
        return [self.string_value(i) for i in range(self.L.zbo_n_strings(self.h))]

    def names(self):
        return [self.name(i) for i in range(self.L.zbo_n_names(self.h))]

    def element_headers(self, p, e):
        """The customHeaders msgpack map of element e's jobs (b"": NO_HEADERS)."""
        n = self.L.zbo_element_headers(self.h, p, e, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        self.L.zbo_element_headers(self.h, p, e, buf, n)
        return buf.raw[:n]

    def process_tables(self):
        """Deployment tables for oracle/logserial.py: per process bpmn_process_id, version, key and
        elements (type, event_type, id, job_type, retries)."""
        out = []
        for p in range(self.L.zbo_n_processes(self.h)):
            key, ver = C.c_int64(), C.c_int()
            bid = self.L.zbo_process_info(self.h, p, C.byref(key), C.byref(ver)).decode()
            els = []
            for e in range(self.L.zbo_n_elements(self.h, p)):
                t, ev, r = C.c_int(), C.c_int(), C.c_int()
                self.L.zbo_element_info(self.h, p, e, C.byref(t), C.byref(ev), C.byref(r))
                els.append((t.value, ev.value, self.element_id(p, e),
                            self.L.zbo_element_job_type(self.h, p, e).decode(), r.value))
            conds = [self.L.zbo_element_cond_text(self.h, p, e).decode() for e in range(len(els))]
            out.append({"bpmn_process_id": bid, "version": ver.value, "key": key.value, "elements": els,
                        "cond_text": conds, "headers": [self.element_headers(p, e) for e in range(len(els))]})
        return out

    def submit(self, cmds, docs=None, xparts=None):
        cmds = np.ascontiguousarray(cmds, dtype=abi.COMMAND_DTYPE)
        docs = np.ascontiguousarray(docs if docs is not None else abi.make_docs(0), dtype=abi.DOC_DTYPE)
        xp = np.ascontiguousarray(xparts if xparts is not None else abi.make_xparts(0), dtype=abi.XPART_DTYPE)
        self.L.zbo_submit_ex(self.h, cmds.ctypes.data, len(cmds), docs.ctypes.data, len(docs), xp.ctypes.data,
                             len(xp))

    def intern_string(self, value):
        b = value.encode() if isinstance(value, str) else value
        return self.L.zbo_intern_string(self.h, b, len(b))

    def intern_list(self, items):
        """A list value [(zbhip_doc_type, value)] into the list dictionary: its id."""
        d = abi_docs(items)
        return self.L.zbo_intern_list(self.h, d.ctypes.data, len(items))

    def list_items(self, list_id):
        """The items [(zbhip_doc_type, value)] of list `list_id`."""
        n = self.L.zbo_list_items(self.h, list_id, None, 0)
        out = abi.make_docs(max(n, 1))
        self.L.zbo_list_items(self.h, list_id, out.ctypes.data, n)
        return [(int(x["type"]), int(x["value"])) for x in out[:n]]

    def take_notified(self):
        """The job types publishWork notified (JobStreamer.notifyWorkAvailable, no stream) since the last
        call, in order."""
        n = self.L.zbo_take_notified(self.h, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        self.L.zbo_take_notified(self.h, buf, n)
        return buf.raw[:n].decode().split("\n")[:-1] if n else []

    def outbox(self, clear=True):
        n = self.L.zbo_outbox(self.h, None, 0)
        out = abi.make_xparts(n)
        self.L.zbo_outbox(self.h, out.ctypes.data, n)
        if clear:
            self.L.zbo_clear_outbox(self.h)
        return out

    def activate_jobs(self, job_type, worker="worker", timeout=300000, max_jobs=10, timestamp=0, variables=()):
        """JOB_BATCH:ACTIVATE on the oracle: (batch key, activated jobs, rejection reason)."""
        import numpy as np
        from zeebe_amd import abi
        out = np.zeros(max(max_jobs, 1) + 1, dtype=abi.ACTIVATED_JOB_DTYPE)
        n, key = C.c_size_t(), C.c_int64()
        blob = b"".join(v.encode() + b"\0" for v in variables)
        reason = self.L.zbo_activate_jobs(self.h, job_type.encode(), worker.encode(), timeout, max_jobs, timestamp, blob,
                                          len(variables), out.ctypes.data, len(out), C.byref(n), C.byref(key))
        return key.value, out[: n.value], reason

    def set_job_stream(self, job_type, worker="", timeout=300000, on=True):
        """A job stream of `job_type` (JobStreamer.streamFor): created jobs are pushed (publishWork)."""
        self.L.zbo_set_job_stream(self.h, job_type.encode(), worker.encode(), int(timeout), 1 if on else 0)

    def job_variables(self, job_keys, variables=()):
        """The pushed jobs as stored now, with the stream's fetchVariables (zbo_job_variables)."""
        import numpy as np
        from zeebe_amd import abi
        keys = np.asarray(job_keys, dtype=np.int64)
        out = np.zeros(max(len(keys), 1), dtype=abi.ACTIVATED_JOB_DTYPE)
        blob = b"".join(v.encode() + b"\0" for v in variables)
        self.L.zbo_job_variables(self.h, keys.ctypes.data, len(keys), blob, len(variables), out.ctypes.data)
        return out[: len(keys)]

    def key_counter(self):
        """DbKeyGenerator's current value (the counter, without the partition bits)."""
        return self.L.zbo_key_counter(self.h)

    def set_key_counter(self, v):
        self.L.zbo_set_key_counter(self.h, v)

    def run(self):
        r = self.L.zbo_run(self.h)
        if r < 0:
            raise OracleError(self.L.zbo_last_error(self.h).decode())
        return r

    def records(self):
        n = self.L.zbo_n_records(self.h)
        out = np.zeros(n, dtype=abi.RECORD_DTYPE)
        self.L.zbo_records(self.h, out.ctypes.data, n)
        return out

    def reason(self, idx):
        buf = C.create_string_buffer(1024)
        self.L.zbo_reason(self.h, idx, buf, 1024)
        return buf.value.decode()

    def clear_records(self):
        self.L.zbo_clear_records(self.h)

    def resolve(self, instance, ordinal):
        return self.L.zbo_resolve(self.h, instance, ordinal)

    def state(self):
        n = self.L.zbo_state(self.h, None, 0)
        buf = C.create_string_buffer(n)
        self.L.zbo_state(self.h, buf, n)
        return [r for r in buf.value.decode().split("\n") if r]

    def process_one(self, rec, instance, docs=None, source=0, first_ordinal=0):
        """Engine.process for exactly one command (a RECORD_DTYPE row, see zb_oracle.cpp
        process_one): its records are appended to records(); returns how many."""
        r = np.ascontiguousarray(np.asarray(rec, dtype=abi.RECORD_DTYPE).reshape(1))
        d = np.ascontiguousarray(docs if docs is not None else abi.make_docs(0), dtype=abi.DOC_DTYPE)
        n = self.L.zbo_process_one(self.h, r.ctypes.data, instance, d.ctypes.data, len(d), source, first_ordinal)
        if n < 0:
            raise OracleError(self.L.zbo_last_error(self.h).decode())
        return n

    def ordinal_of(self, instance, key):
        """The key's ordinal among the keys instance slot `instance` generated (-1 unknown)."""
        return self.L.zbo_ordinal_of(self.h, instance, key)

    def import_rows(self, rows):
        """Column-family rows (the dump_state / zbhip_export_instances text) into this engine's state."""
        text = "\n".join(rows).encode()
        n = self.L.zbo_import_rows(self.h, text, len(text))
        if n < 0:
            raise OracleError(self.L.zbo_last_error(self.h).decode())
        return n

    def counters(self):
        t, c, m = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self.L.zbo_counters(self.h, C.byref(t), C.byref(c), C.byref(m))
        return {"transitions": t.value, "completed_instances": c.value, "commands": m.value}


def subscription_partition(correlation_key, partition_count):
    b = correlation_key.encode() if isinstance(correlation_key, str) else correlation_key
    return lib().zbo_subscription_partition(b, len(b), partition_count)


def java_hash(value):
    b = value.encode() if isinstance(value, str) else value
    return lib().zbo_java_hash(b, len(b))


def bench(xml, threads, n_instances, phases, with_amount=False, seed=0x5EED03):
    """CPU baseline: `threads` partitions, one per core (returns seconds, transitions, completed)."""
    if isinstance(xml, str):
        xml = xml.encode()
    t, c = C.c_uint64(), C.c_uint64()
    sec = lib().zbo_bench(xml, threads, n_instances, phases, 1 if with_amount else 0, seed, C.byref(t), C.byref(c))
    if sec < 0:
        raise OracleError("bench deploy failed")
    return sec, t.value, c.value


def bench_jobs(xml, threads, n_instances, job_ords, seed=0x5EED04):
    """CPU baseline of variant 4b: each instance completes its jobs (key ordinals job_ords) in its
    own random order, one per phase; returns seconds, transitions, completed."""
    import numpy as np
    if isinstance(xml, str):
        xml = xml.encode()
    o = np.ascontiguousarray(job_ords, dtype=np.uint16)
    t, c = C.c_uint64(), C.c_uint64()
    sec = lib().zbo_bench_jobs(xml, threads, n_instances, o.ctypes.data, len(o), seed, C.byref(t), C.byref(c))
    if sec < 0:
        raise OracleError("bench deploy failed")
    return sec, t.value, c.value


def bench_msg(xml, partitions, n_instances):
    """CPU baseline of config 5: `partitions` partitions (one thread each), n instances each."""
    if isinstance(xml, str):
        xml = xml.encode()
    t, c = C.c_uint64(), C.c_uint64()
    sec = lib().zbo_bench_msg(xml, partitions, n_instances, C.byref(t), C.byref(c))
    if sec < 0:
        raise OracleError("bench deploy failed")
    return sec, t.value, c.value


def abi_docs(items):
    """[(zbhip_doc_type, value)] as zbhip_doc_entry rows (the list dictionary's item form; one spare row
    for an empty list, so the buffer is never null)."""
    d = abi.make_docs(max(len(items), 1))
    for j, (t, v) in enumerate(items):
        d[j]["type"], d[j]["value"] = t, v
    return d
