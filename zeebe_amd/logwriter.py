"""Host mirror of the log serialiser (zbhip_serializer in zeebe_amd/csrc/logwriter.cpp).

The reference writes every record of a processed batch into the partition's log as one
sequenced batch (stream-platform ProcessingStateMachine.writeRecords ->
logstreams SequencedBatchSerializer.java:33-67).  `LogSerializer.serialize` produces those bytes
for drained records, through the C ABI only; a Partition owns one that follows its deployments
and dictionaries (`Partition.log_serializer()`), a standalone one is built with the same
deploy / intern calls in the same order.
"""
import ctypes as C

import numpy as np

from . import abi
from .native import DB_SINK, check, load


def _db_collector():
    rows = []

    def sink(_ctx, cf, k, kn, v, vn):
        rows.append((cf, C.string_at(k, kn), C.string_at(v, vn)))

    return rows, DB_SINK(sink)


class LogSerializer:
    def __init__(self, partition=None):
        self.L = load()
        self._own = partition is None
        if partition is None:
            out = C.c_void_p()
            check(self.L.zbhip_serializer_new(C.byref(out)), "zbhip_serializer_new")
            self.s = out.value
        else:
            self.s = self.L.zbhip_handle_serializer(partition.h)
            self._partition = partition  # keeps the handle (and its serializer) alive

    def close(self):
        if self._own and self.s:
            self.L.zbhip_serializer_free(self.s)
        self.s = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    def deploy(self, xml, process_definition_key=2251799813685249, version=1):
        if isinstance(xml, str):
            xml = xml.encode()
        csr = C.c_void_p()
        err = C.create_string_buffer(512)
        check(self.L.zbhip_compile_bpmn(xml, len(xml), process_definition_key, version, C.byref(csr), err, 512),
              err.value.decode())
        try:
            idx = C.c_uint32()
            check(self.L.zbhip_serializer_deploy(self.s, csr, C.byref(idx)), "zbhip_serializer_deploy")
        finally:
            self.L.zbhip_free_csr(csr)
        return idx.value

    def intern(self, name):
        return check(self.L.zbhip_serializer_intern(self.s, name.encode()))

    def intern_string(self, value):
        b = value.encode() if isinstance(value, str) else bytes(value)
        return check(self.L.zbhip_serializer_intern_string(self.s, b, len(b)))

    def encode_state_rows(self, rows):
        """zb-db entries (column family ordinal, key bytes, value bytes) of canonical state rows."""
        out, cb = _db_collector()
        for r in rows:
            check(self.L.zbhip_serializer_encode_state_row(self.s, r.encode(), cb, None), "encode_state_row")
        return sorted(out)

    def decode_state_entries(self, entries, intern=None):
        """zb-db entries -> canonical state rows (the inverse of encode_state_rows); intern(bytes) -> id
        maps string variable values to value-dictionary ids."""
        import ctypes as C

        from .native import INTERNER
        cb = INTERNER((lambda ctx, b, n: intern(C.string_at(b, n))) if intern else (lambda ctx, b, n: -5))
        cap = 8192
        buf = C.create_string_buffer(cap)
        rows = []
        for cf, k, v in entries:
            n = self.L.zbhip_serializer_decode_state_entry(self.s, cf, k, len(k), v, len(v), cb, None, buf, cap)
            while n == -2 and cap < 1 << 26:  # ZBHIP_ENOMEM: a long value (an errorMessage of 10 000 chars)
                cap *= 8
                buf = C.create_string_buffer(cap)
                n = self.L.zbhip_serializer_decode_state_entry(self.s, cf, k, len(k), v, len(v), cb, None, buf, cap)
            n = check(n, "decode_state_entry")
            if n:
                rows.append(buf.value.decode())
        return sorted(rows)

    def set_broker_version(self, major, minor, patch):
        check(self.L.zbhip_serializer_set_broker_version(self.s, major, minor, patch))

    def serialize(self, records, cmds, docs=None, source_base=0, doc_base=0, source_positions=None,
                  first_position=1, timestamp=0, source_timestamps=None, timer_values=None):
        """Log bytes of `records` (drain order) drained from the window (cmds, docs).
        source_positions[i] = log position of cmds[i] (default: 1 + i); source_timestamps[i] = its
        timestamp (default: timestamp); timer_values[i] = the TimerRecord of a TIMER:TRIGGER cmds[i]
        (abi.TIMER_VALUE_DTYPE, written for its rejection)."""
        recs = np.ascontiguousarray(records, dtype=abi.RECORD_DTYPE)
        cmds = np.ascontiguousarray(cmds, dtype=abi.COMMAND_DTYPE)
        docs = np.ascontiguousarray(docs if docs is not None else abi.make_docs(0), dtype=abi.DOC_DTYPE)
        pos = np.ascontiguousarray(source_positions if source_positions is not None
                                   else np.arange(1, len(cmds) + 1), dtype=np.int64)
        ts = (np.ascontiguousarray(source_timestamps, dtype=np.int64) if source_timestamps is not None else None)
        tv = (np.ascontiguousarray(timer_values, dtype=abi.TIMER_VALUE_DTYPE) if timer_values is not None else None)
        if tv is not None and len(tv) != len(cmds):
            raise ValueError("timer_values: one per window command")
        w = abi.LogWindow(cmds.ctypes.data, len(cmds), source_base, docs.ctypes.data if len(docs) else None, len(docs),
                          doc_base, pos.ctypes.data, first_position, timestamp,
                          ts.ctypes.data if ts is not None else None, tv.ctypes.data if tv is not None else None)
        used = C.c_size_t()
        check(self.L.zbhip_serialize_log(self.s, recs.ctypes.data, len(recs), C.byref(w), None, 0, C.byref(used)),
              "zbhip_serialize_log")
        out = C.create_string_buffer(max(used.value, 1))
        check(self.L.zbhip_serialize_log(self.s, recs.ctypes.data, len(recs), C.byref(w), out, used.value,
                                         C.byref(used)), "zbhip_serialize_log")
        return out.raw[:used.value]


def split_entries(buf):
    """Walks serialised log bytes: yields (offset, framed_length) per entry (8-aligned frames)."""
    off = 0
    while off < len(buf):
        n = int.from_bytes(buf[off:off + 4], "little")
        if n < 52:
            raise ValueError("corrupt frame at %d" % off)
        yield off, n
        off += (n + 7) & ~7
