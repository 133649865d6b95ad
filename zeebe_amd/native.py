"""Loads the in-tree libzbhip.so (gfx950) and declares its C ABI.

There is no fallback: if the library is missing or cannot be loaded, every entry
point raises.  The CPU oracle is test infrastructure and is never used here.
"""
import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
# ZBHIP_LIB selects an alternative in-tree build (e.g. the instrumented libzbhip_stamps.so)
LIB_PATH = os.path.join(HERE, os.environ.get("ZBHIP_LIB", "libzbhip.so"))

ERRORS = {-1: "ZBHIP_EINVAL", -2: "ZBHIP_ENOMEM", -3: "ZBHIP_EDEVICE", -4: "ZBHIP_EPARSE",
          -5: "ZBHIP_EUNSUPP", -6: "ZBHIP_ESTATE", -7: "ZBHIP_ENODEV"}

# every symbol include/zbhip.h declares (tests/test_abi.py checks the export table)
SYMBOLS = ["zbhip_compile_bpmn", "zbhip_free_csr", "zbhip_open", "zbhip_close", "zbhip_deploy", "zbhip_intern",
           "zbhip_string", "zbhip_name", "zbhip_submit", "zbhip_submit_device", "zbhip_run", "zbhip_set_clock", "zbhip_drain",
           "zbhip_pending_records", "zbhip_get_stats", "zbhip_export_state", "zbhip_fallback",
           "zbhip_resolve_key", "zbhip_rejection_reason", "zbhip_incident_message", "zbhip_build_info", "zbhip_command_status",
           "zbhip_submit_ex", "zbhip_submit_device_ex", "zbhip_intern_string", "zbhip_intern_strings",
           "zbhip_string_value", "zbhip_subscription_partition", "zbhip_outbox", "zbhip_outbox_device",
           "zbhip_outbox_copy", "zbhip_exchange_gather", "zbhip_submit_xparts_device", "zbhip_string_partitions",
           "zbhip_serializer_new", "zbhip_serializer_free", "zbhip_serializer_deploy", "zbhip_serializer_intern",
           "zbhip_serializer_intern_string", "zbhip_serializer_set_broker_version",
           "zbhip_serializer_rejection_reason", "zbhip_serializer_incident_message", "zbhip_handle_serializer", "zbhip_serialize_log",
           "zbhip_export_state_db", "zbhip_serializer_encode_state_row", "zbhip_outbox_device_async", "zbhip_stream",
           "zbhip_export_instances", "zbhip_export_instances_db", "zbhip_evict_instances", "zbhip_key_before",
           "zbhip_set_external_keys", "zbhip_export_correlation_slots", "zbhip_export_correlation_slots_db",
           "zbhip_evict_correlation_slots", "zbhip_log_copy_async", "zbhip_log_copy_wait", "zbhip_serializer_decode_state_entry", "zbhip_import_state_db",
           "zbhip_import_state", "zbhip_activate_jobs", "zbhip_activatable_jobs", "zbhip_job_batch_rejection_reason",
           "zbhip_serialize_log_device", "zbhip_log_device_copy", "zbhip_continuations",
           "zbhip_pending_continuations", "zbhip_current_key", "zbhip_set_key_if_higher",
           "zbhip_select_instances_db", "zbhip_drain_command", "zbhip_outbox_command", "zbhip_due_timers",
           "zbhip_timed_out_jobs", "zbhip_time_out_job", "zbhip_fail_job", "zbhip_job_state", "zbhip_set_job_stream",
           "zbhip_job_variables", "zbhip_intern_list", "zbhip_list_items", "zbhip_serializer_intern_list",
           "zbhip_doc_merge_order"]


class ZbhipError(RuntimeError):
    def __init__(self, code, what=""):
        super().__init__("%s (%d)%s" % (ERRORS.get(code, "?"), code, (": " + what) if what else ""))
        self.code = code


STATE_SINK = C.CFUNCTYPE(None, C.c_void_p, C.c_char_p)
DB_SINK = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_uint8),
                      C.c_size_t)
INTERNER = C.CFUNCTYPE(C.c_int64, C.c_void_p, C.c_void_p, C.c_size_t)

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ZbhipError(-7, "libzbhip.so not built (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, sz, i64, u32 = C.c_void_p, C.c_size_t, C.c_int64, C.c_uint32
    L.zbhip_compile_bpmn.argtypes = [C.c_char_p, sz, i64, C.c_int32, C.POINTER(vp), C.c_char_p, sz]
    L.zbhip_free_csr.argtypes = [vp]
    L.zbhip_free_csr.restype = None
    L.zbhip_open.argtypes = [C.POINTER(abi.Config), C.POINTER(vp)]
    L.zbhip_close.argtypes = [vp]
    L.zbhip_close.restype = None
    L.zbhip_deploy.argtypes = [vp, vp, C.POINTER(u32)]
    L.zbhip_intern.argtypes = [vp, C.c_char_p]
    L.zbhip_string.argtypes = [vp, u32, u32]
    L.zbhip_string.restype = C.c_char_p
    L.zbhip_name.argtypes = [vp, u32]
    L.zbhip_name.restype = C.c_char_p
    L.zbhip_submit.argtypes = [vp, vp, sz, vp, sz]
    L.zbhip_submit_device.argtypes = [vp, vp, sz, vp, sz]
    L.zbhip_run.argtypes = [vp, u32]
    L.zbhip_set_clock.argtypes = [vp, C.c_int64]
    L.zbhip_drain.argtypes = [vp, vp, sz, C.POINTER(sz)]
    L.zbhip_pending_records.argtypes = [vp]
    L.zbhip_pending_records.restype = i64
    L.zbhip_get_stats.argtypes = [vp, C.POINTER(abi.Stats)]
    L.zbhip_export_state.argtypes = [vp, STATE_SINK, vp]
    L.zbhip_fallback.argtypes = [vp, C.POINTER(u32), sz, C.POINTER(sz)]
    L.zbhip_resolve_key.argtypes = [vp, i64, C.POINTER(u32), C.POINTER(C.c_uint16)]
    L.zbhip_rejection_reason.argtypes = [vp, C.POINTER(abi.Record), C.c_char_p, sz]
    L.zbhip_incident_message.argtypes = [vp, C.POINTER(abi.Record), C.c_char_p, sz]
    L.zbhip_incident_message.restype = i64
    L.zbhip_command_status.argtypes = [vp, sz, C.POINTER(u32), C.POINTER(u32)]
    L.zbhip_submit_ex.argtypes = [vp, vp, sz, vp, sz, vp, sz]
    L.zbhip_submit_device_ex.argtypes = [vp, vp, sz, vp, sz, vp, sz]
    L.zbhip_intern_string.argtypes = [vp, C.c_char_p, sz]
    L.zbhip_intern_string.restype = i64
    L.zbhip_intern_strings.argtypes = [vp, C.c_char_p, vp, sz, vp]
    L.zbhip_string_value.argtypes = [vp, u32, C.POINTER(sz)]
    L.zbhip_string_value.restype = C.c_char_p
    L.zbhip_subscription_partition.argtypes = [C.c_char_p, sz, C.c_int32]
    L.zbhip_subscription_partition.restype = C.c_int32
    L.zbhip_outbox.argtypes = [vp, vp, sz, C.POINTER(sz)]
    L.zbhip_outbox_device.argtypes = [vp, C.POINTER(vp), vp]
    L.zbhip_outbox_copy.argtypes = [vp, vp, sz, sz]
    L.zbhip_exchange_gather.argtypes = [C.POINTER(vp), u32, vp, C.POINTER(vp), u32, vp]
    L.zbhip_outbox_device_async.argtypes = [vp, C.POINTER(vp), vp]
    L.zbhip_export_instances.argtypes = [vp, vp, sz, STATE_SINK, vp]
    L.zbhip_export_instances_db.argtypes = [vp, vp, sz, DB_SINK, vp]
    L.zbhip_export_correlation_slots.argtypes = [vp, vp, sz, STATE_SINK, vp]
    L.zbhip_export_correlation_slots_db.argtypes = [vp, vp, sz, DB_SINK, vp]
    L.zbhip_evict_correlation_slots.argtypes = [vp, vp, sz]
    L.zbhip_log_copy_async.argtypes = [vp, sz, C.POINTER(vp)]
    L.zbhip_log_copy_wait.argtypes = [vp, vp]
    L.zbhip_evict_instances.argtypes = [vp, vp, sz]
    L.zbhip_key_before.argtypes = [vp, sz, C.POINTER(i64)]
    L.zbhip_continuations.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.zbhip_pending_continuations.argtypes = [vp, u32]
    L.zbhip_current_key.argtypes = [vp, C.POINTER(i64)]
    L.zbhip_set_key_if_higher.argtypes = [vp, i64]
    L.zbhip_drain_command.argtypes = [vp, sz, vp, sz, C.POINTER(sz)]
    L.zbhip_outbox_command.argtypes = [vp, sz, vp, sz, C.POINTER(sz)]
    L.zbhip_select_instances_db.argtypes = [vp, vp, sz, vp, sz, vp, sz, C.POINTER(sz)]
    L.zbhip_set_external_keys.argtypes = [vp, sz, u32]
    L.zbhip_serializer_decode_state_entry.argtypes = [vp, u32, C.c_char_p, sz, C.c_char_p, sz, INTERNER, vp,
                                                      C.c_char_p, sz]
    L.zbhip_import_state_db.argtypes = [vp, C.c_char_p, sz, u32, C.POINTER(u32)]
    L.zbhip_import_state.argtypes = [vp, C.c_char_p, sz, u32, C.POINTER(u32)]
    L.zbhip_activate_jobs.argtypes = [vp, C.POINTER(abi.JobActivation), vp, sz, C.POINTER(abi.JobBatch)]
    L.zbhip_activatable_jobs.argtypes = [vp, C.c_char_p, sz, vp, sz, C.POINTER(sz)]
    L.zbhip_job_batch_rejection_reason.argtypes = [C.POINTER(abi.JobActivation), C.POINTER(abi.JobBatch), C.c_char_p, sz]
    L.zbhip_due_timers.argtypes = [vp, i64, vp, sz, C.POINTER(sz), C.POINTER(i64)]
    L.zbhip_timed_out_jobs.argtypes = [vp, i64, vp, sz, C.POINTER(sz), C.POINTER(i64)]
    L.zbhip_time_out_job.argtypes = [vp, i64, i64, vp, sz, C.POINTER(sz)]
    L.zbhip_set_job_stream.argtypes = [vp, C.c_char_p, sz, C.c_char_p, sz, i64, C.c_int]
    L.zbhip_fail_job.argtypes = [vp, C.POINTER(abi.JobFail), vp, sz, C.POINTER(sz)]
    L.zbhip_job_state.argtypes = [vp, i64]
    L.zbhip_job_variables.argtypes = [vp, vp, sz, vp, sz, vp]
    L.zbhip_intern_list.restype = i64
    L.zbhip_intern_list.argtypes = [vp, vp, sz]
    L.zbhip_list_items.argtypes = [vp, i64, vp, sz, C.POINTER(sz)]
    L.zbhip_doc_merge_order.argtypes = [vp, sz, vp]
    L.zbhip_stream.argtypes = [vp]
    L.zbhip_stream.restype = vp
    L.zbhip_submit_xparts_device.argtypes = [vp, vp, sz]
    L.zbhip_string_partitions.argtypes = [vp, vp, sz, C.c_int32, vp]
    L.zbhip_serializer_new.argtypes = [C.POINTER(vp)]
    L.zbhip_serializer_free.argtypes = [vp]
    L.zbhip_serializer_free.restype = None
    L.zbhip_serializer_deploy.argtypes = [vp, vp, C.POINTER(u32)]
    L.zbhip_serializer_intern.argtypes = [vp, C.c_char_p]
    L.zbhip_serializer_intern_string.argtypes = [vp, C.c_char_p, sz]
    L.zbhip_serializer_intern_string.restype = i64
    L.zbhip_serializer_set_broker_version.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32]
    L.zbhip_serializer_rejection_reason.argtypes = [vp, C.POINTER(abi.Record), C.c_char_p, sz]
    L.zbhip_handle_serializer.argtypes = [vp]
    L.zbhip_handle_serializer.restype = vp
    L.zbhip_serialize_log.argtypes = [vp, vp, sz, C.POINTER(abi.LogWindow), vp, sz, C.POINTER(sz)]
    L.zbhip_serialize_log_device.argtypes = [vp, C.POINTER(abi.LogWindow), C.POINTER(vp), C.POINTER(sz)]
    L.zbhip_log_device_copy.argtypes = [vp, vp, sz]
    L.zbhip_export_state_db.argtypes = [vp, DB_SINK, vp]
    L.zbhip_serializer_encode_state_row.argtypes = [vp, C.c_char_p, DB_SINK, vp]
    L.zbhip_build_info.argtypes = []
    L.zbhip_build_info.restype = C.c_char_p
    _lib = L
    return L


def check(rc, what=""):
    if rc < 0:
        raise ZbhipError(rc, what)
    return rc
