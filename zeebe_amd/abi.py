"""ctypes / numpy mirror of ``include/zbhip.h`` (the libzbhip.so C ABI).

The layouts here must match the header byte for byte; ``tests/test_abi.py``
checks the sizes against the compiled library.
"""
import ctypes as C

import numpy as np

# ---- protocol enums (protocol/src/main/resources/protocol.xml:23-72) ----
RT_EVENT, RT_COMMAND, RT_REJECTION = 0, 1, 2
VT_JOB_BATCH = 14  # ValueType.JOB_BATCH (protocol.xml:31)
JOB_BATCH_ACTIVATE, JOB_BATCH_ACTIVATED = 0, 1
VT_JOB = 0
VT_PROCESS_INSTANCE = 5
VT_MESSAGE = 10
VT_MESSAGE_SUBSCRIPTION = 11
VT_PROCESS_MESSAGE_SUBSCRIPTION = 12
VT_MESSAGE_START_EVENT_SUBSCRIPTION = 16  # engine-only (message start events stay with the CPU engine)
VT_VARIABLE = 17
VT_PROCESS_INSTANCE_CREATION = 19
VT_PROCESS_EVENT = 24
VT_TIMER = 15
VT_PROCESS_INSTANCE_BATCH = 34
VT_INCIDENT = 6
INCIDENT_CREATED = 0
ERR_JOB_NO_RETRIES, ERR_CONDITION_ERROR, ERR_EXTRACT_VALUE_ERROR = 2, 3, 4  # ErrorType ordinals
ERR_UNHANDLED_ERROR_EVENT = 6
ERROR_TYPES = {2: "JOB_NO_RETRIES", 3: "CONDITION_ERROR", 4: "EXTRACT_VALUE_ERROR", 6: "UNHANDLED_ERROR_EVENT"}
FEEL_NULL, FEEL_NUMBER, FEEL_STRING = 0, 1, 2       # zbhip_record.reason_arg of an INCIDENT

REJ_INVALID_ARGUMENT, REJ_NOT_FOUND, REJ_ALREADY_EXISTS, REJ_INVALID_STATE = 0, 1, 2, 3
REJ_PROCESSING_ERROR, REJ_NONE = 4, 255

# ProcessInstanceIntent (protocol/.../intent/ProcessInstanceIntent.java:22-35)
PI_INTENTS = {
    1: "SEQUENCE_FLOW_TAKEN", 2: "ELEMENT_ACTIVATING", 3: "ELEMENT_ACTIVATED",
    4: "ELEMENT_COMPLETING", 5: "ELEMENT_COMPLETED", 6: "ELEMENT_TERMINATING",
    7: "ELEMENT_TERMINATED", 8: "ACTIVATE_ELEMENT", 9: "COMPLETE_ELEMENT", 10: "TERMINATE_ELEMENT",
}
PI_INTENT_IDS = {v: k for k, v in PI_INTENTS.items()}
PI_SEQUENCE_FLOW_TAKEN, PI_ELEMENT_ACTIVATING, PI_ELEMENT_ACTIVATED = 1, 2, 3
PI_ELEMENT_COMPLETING, PI_ELEMENT_COMPLETED, PI_ELEMENT_TERMINATED = 4, 5, 7
JOB_INTENTS = {0: "CREATED", 1: "COMPLETE", 2: "COMPLETED", 3: "TIME_OUT", 4: "TIMED_OUT", 5: "FAIL", 6: "FAILED",
               10: "CANCELED", 11: "THROW_ERROR", 12: "ERROR_THROWN"}
JOB_THROW_ERROR, JOB_ERROR_THROWN = 11, 12
JOB_CREATED, JOB_COMPLETE, JOB_COMPLETED, JOB_CANCELED = 0, 1, 2, 10
JOB_TIME_OUT, JOB_TIMED_OUT, JOB_FAIL, JOB_FAILED = 3, 4, 5, 6
VAR_INTENTS = {0: "CREATED", 1: "UPDATED"}
VAR_CREATED, VAR_UPDATED = 0, 1
PE_INTENTS = {0: "TRIGGERING", 1: "TRIGGERED"}
PIC_INTENTS = {0: "CREATE", 1: "CREATED"}
TIMER_INTENTS = {0: "CREATED", 1: "TRIGGER", 2: "TRIGGERED", 3: "CANCEL", 4: "CANCELED"}
PIB_INTENTS = {0: "TERMINATE", 1: "ACTIVATE"}
PIB_TERMINATE, PIB_ACTIVATE = 0, 1
AUX_INLINE = -2  # VARIABLE record with its value inline (message_key, doc type in partition)
TIMER_CREATED, TIMER_TRIGGER, TIMER_TRIGGERED, TIMER_CANCELED = 0, 1, 2, 4
PE_TRIGGERING, PE_TRIGGERED = 0, 1
# MessageIntent / MessageSubscriptionIntent / ProcessMessageSubscriptionIntent
MSG_INTENTS = {0: "PUBLISH", 1: "PUBLISHED", 2: "EXPIRE", 3: "EXPIRED"}
MS_INTENTS = {0: "CREATE", 1: "CREATED", 2: "CORRELATE", 3: "CORRELATED", 4: "REJECT", 5: "REJECTED",
              6: "DELETE", 7: "DELETED", 8: "CORRELATING"}
PMS_INTENTS = {0: "CREATING", 1: "CREATE", 2: "CREATED", 3: "CORRELATE", 4: "CORRELATED", 5: "DELETING",
               6: "DELETE", 7: "DELETED"}
MSG_PUBLISH, MSG_PUBLISHED, MSG_EXPIRE, MSG_EXPIRED = 0, 1, 2, 3
VT_MESSAGE_BATCH, MESSAGE_BATCH_EXPIRE = 35, 0  # ValueType.MESSAGE_BATCH (protocol.xml:52), MessageBatchIntent
MS_CREATE, MS_CREATED, MS_CORRELATE, MS_CORRELATED, MS_CORRELATING = 0, 1, 2, 3, 8
MS_DELETE, MS_DELETED = 6, 7
PMS_CREATING, PMS_CREATE, PMS_CREATED, PMS_CORRELATE, PMS_CORRELATED = 0, 1, 2, 3, 4
PMS_DELETING, PMS_DELETE, PMS_DELETED = 5, 6, 7
MSES_INTENTS = {0: "CREATED", 1: "CORRELATED", 2: "DELETED"}  # MessageStartEventSubscriptionIntent
MSES_CREATED, MSES_CORRELATED, MSES_DELETED = 0, 1, 2
VALUE_TYPES = {0: "JOB", 5: "PROCESS_INSTANCE", 10: "MESSAGE", 11: "MESSAGE_SUBSCRIPTION",
               12: "PROCESS_MESSAGE_SUBSCRIPTION", 17: "VARIABLE", 19: "PROCESS_INSTANCE_CREATION",
               24: "PROCESS_EVENT", 15: "TIMER", 34: "PROCESS_INSTANCE_BATCH",
               16: "MESSAGE_START_EVENT_SUBSCRIPTION"}
RECORD_TYPES = {0: "EVENT", 1: "COMMAND", 2: "COMMAND_REJECTION"}
REJECTION_TYPES = {0: "INVALID_ARGUMENT", 1: "NOT_FOUND", 2: "ALREADY_EXISTS", 3: "INVALID_STATE",
                   4: "PROCESSING_ERROR", 255: "NULL_VAL"}
ELEMENT_TYPES = ["UNSPECIFIED", "PROCESS", "SUB_PROCESS", "EVENT_SUB_PROCESS", "START_EVENT",
                 "INTERMEDIATE_CATCH_EVENT", "INTERMEDIATE_THROW_EVENT", "BOUNDARY_EVENT", "END_EVENT",
                 "SERVICE_TASK", "RECEIVE_TASK", "USER_TASK", "MANUAL_TASK", "TASK", "EXCLUSIVE_GATEWAY",
                 "PARALLEL_GATEWAY", "EVENT_BASED_GATEWAY", "INCLUSIVE_GATEWAY", "SEQUENCE_FLOW",
                 "MULTI_INSTANCE_BODY", "CALL_ACTIVITY", "BUSINESS_RULE_TASK", "SCRIPT_TASK", "SEND_TASK"]
EVENT_TYPES = ["UNSPECIFIED", "CONDITIONAL", "ERROR", "ESCALATION", "LINK", "MESSAGE", "NONE",
               "SIGNAL", "TERMINATE", "TIMER"]


def intent_name(value_type, intent):
    table = {VT_PROCESS_INSTANCE: PI_INTENTS, VT_JOB: JOB_INTENTS, VT_VARIABLE: VAR_INTENTS,
             VT_PROCESS_EVENT: PE_INTENTS, VT_PROCESS_INSTANCE_CREATION: PIC_INTENTS, VT_MESSAGE: MSG_INTENTS,
             VT_MESSAGE_SUBSCRIPTION: MS_INTENTS, VT_PROCESS_MESSAGE_SUBSCRIPTION: PMS_INTENTS,
             VT_TIMER: TIMER_INTENTS, VT_PROCESS_INSTANCE_BATCH: PIB_INTENTS,
             VT_MESSAGE_START_EVENT_SUBSCRIPTION: MSES_INTENTS}.get(value_type, {})
    return table.get(intent, str(intent))


CMD_CREATE = 1
CMD_JOB_COMPLETE = 2
CMD_PUBLISH = 3
CMD_MSG_SUB_CREATE, CMD_PMS_CREATE, CMD_PMS_CORRELATE, CMD_MSG_SUB_CORRELATE = 4, 5, 6, 7
CMD_TIMER_TRIGGER = 8  # ref = timer key ordinal, doc_begin | pad << 32 = the timer's dueDate
CMD_CONTINUE = 9  # a deferred continuation read back from the log: doc_begin | pad << 32 = its id
CMD_MSG_SUB_DELETE, CMD_PMS_DELETE = 10, 11  # closing a subscription and its acknowledgement
XPART_KINDS = (CMD_MSG_SUB_CREATE, CMD_PMS_CREATE, CMD_PMS_CORRELATE, CMD_MSG_SUB_CORRELATE, CMD_MSG_SUB_DELETE,
               CMD_PMS_DELETE)
SLOT_KINDS = (CMD_PUBLISH, CMD_MSG_SUB_CREATE, CMD_MSG_SUB_CORRELATE, CMD_MSG_SUB_DELETE)
PMS_KINDS = (CMD_PMS_CREATE, CMD_PMS_CORRELATE, CMD_PMS_DELETE)
DOC_NIL, DOC_BOOL, DOC_INT, DOC_DEC, DOC_OTHER, DOC_STR, DOC_LIST = 0, 1, 2, 3, 4, 5, 6
NO_STRING = 0xFFFFFFFF
DEC_SCALE = 6

RUN_NO_RESULTS = 1
RUN_TIMED = 2
RUN_ACCUMULATE = 4
RUN_DEVICE_RECORDS = 8


class DocEntry(C.Structure):
    _fields_ = [("name_id", C.c_uint32), ("type", C.c_uint8), ("pad", C.c_uint8 * 3), ("value", C.c_int64)]


class Command(C.Structure):
    _fields_ = [("instance", C.c_uint32), ("kind", C.c_uint8), ("doc_count", C.c_uint8),
                ("ref", C.c_uint16), ("doc_begin", C.c_uint32), ("pad", C.c_uint32)]


class Record(C.Structure):
    _fields_ = [("key", C.c_int64), ("scope_key", C.c_int64), ("process_instance_key", C.c_int64),
                ("source_index", C.c_int64), ("process_idx", C.c_int32), ("element_idx", C.c_int32),
                ("record_type", C.c_uint8), ("value_type", C.c_uint8), ("intent", C.c_uint8),
                ("rejection_type", C.c_uint8), ("ordinal", C.c_uint16), ("reason", C.c_uint8),
                ("reason_arg", C.c_uint8), ("aux", C.c_int64), ("message_key", C.c_int64),
                ("correlation_key", C.c_uint32), ("message_name", C.c_uint16), ("bpmn_process_id", C.c_uint16),
                ("partition", C.c_int32), ("interrupting", C.c_uint8), ("unprocessed", C.c_uint8),
                ("pad", C.c_uint8 * 2)]


class XpartCmd(C.Structure):
    _fields_ = [("element_instance_key", C.c_int64), ("process_instance_key", C.c_int64),
                ("message_key", C.c_int64), ("correlation_key", C.c_uint32), ("instance", C.c_uint32),
                ("element_ord", C.c_uint16), ("message_name", C.c_uint16), ("bpmn_process_id", C.c_uint16),
                ("kind", C.c_uint8), ("interrupting", C.c_uint8), ("source_partition", C.c_int16),
                ("target_partition", C.c_int16), ("pad", C.c_uint32)]


class LogWindow(C.Structure):  # zbhip_log_window
    _fields_ = [("cmds", C.c_void_p), ("n_cmds", C.c_size_t), ("source_base", C.c_int64), ("docs", C.c_void_p),
                ("n_docs", C.c_size_t), ("doc_base", C.c_int64), ("source_positions", C.c_void_p),
                ("first_position", C.c_int64), ("timestamp", C.c_int64), ("source_timestamps", C.c_void_p),
                ("timer_values", C.c_void_p)]


# zbhip_timer_value: a TIMER:TRIGGER command's TimerRecord (DueDateTimerChecker.java:118-125)
TIMER_VALUE_DTYPE = np.dtype([("element_instance_key", "<i8"), ("process_instance_key", "<i8"),
                              ("process_definition_key", "<i8"), ("repetitions", "<i4"), ("process_idx", "<i4"),
                              ("element_idx", "<i4"), ("pad", "<i4")])


OPEN_TRUSTED_DEVICE_WINDOWS = 1
OPEN_DEFER_CONTINUATIONS = 2


class JobActivation(C.Structure):  # zbhip_job_activation (JOB_BATCH:ACTIVATE)
    _fields_ = [("type", C.c_char_p), ("type_len", C.c_size_t), ("worker", C.c_char_p), ("worker_len", C.c_size_t),
                ("timeout", C.c_int64), ("max_jobs", C.c_int32), ("pad", C.c_int32), ("timestamp", C.c_int64),
                ("variables", C.c_void_p), ("n_variables", C.c_size_t)]


class JobBatch(C.Structure):  # zbhip_job_batch
    _fields_ = [("key", C.c_int64), ("n_jobs", C.c_uint32), ("rejection_type", C.c_uint8), ("reason", C.c_uint8),
                ("truncated", C.c_uint8), ("pad", C.c_uint8)]


class Config(C.Structure):
    _fields_ = [("partition_id", C.c_int32), ("partition_count", C.c_int32), ("device", C.c_int32),
                ("max_commands_in_batch", C.c_int32), ("max_instances", C.c_uint32),
                ("max_commands", C.c_uint32), ("max_records_per_batch", C.c_uint32),
                ("max_doc_entries", C.c_uint32), ("initial_key", C.c_int64), ("max_correlation_keys", C.c_uint32),
                ("flags", C.c_uint32), ("stream", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("commands", C.c_uint64), ("records", C.c_uint64), ("transitions", C.c_uint64),
                ("completed_instances", C.c_uint64), ("keys", C.c_uint64), ("fallback", C.c_uint64),
                ("step_ms", C.c_double), ("compact_ms", C.c_double), ("rounds", C.c_uint32),
                ("launches", C.c_uint32), ("template_batches", C.c_uint64)]


COMMAND_DTYPE = np.dtype([("instance", "<u4"), ("kind", "u1"), ("doc_count", "u1"), ("ref", "<u2"),
                          ("doc_begin", "<u4"), ("pad", "<u4")])
DOC_DTYPE = np.dtype([("name_id", "<u4"), ("type", "u1"), ("pad", "u1", (3,)), ("value", "<i8")])
# zbhip_activated_job
ACTIVATED_JOB_DTYPE = np.dtype([("key", "<i8"), ("element_instance_key", "<i8"), ("process_instance_key", "<i8"),
                                ("deadline", "<i8"), ("instance", "<u4"), ("process_idx", "<i4"),
                                ("element_idx", "<i4"), ("retries", "<u2"), ("n_variables", "<u2"),
                                ("variables", DOC_DTYPE, (6,))])
RECORD_DTYPE = np.dtype([("key", "<i8"), ("scope_key", "<i8"), ("process_instance_key", "<i8"),
                         ("source_index", "<i8"), ("process_idx", "<i4"), ("element_idx", "<i4"),
                         ("record_type", "u1"), ("value_type", "u1"), ("intent", "u1"),
                         ("rejection_type", "u1"), ("ordinal", "<u2"), ("reason", "u1"), ("reason_arg", "u1"),
                         ("aux", "<i8"), ("message_key", "<i8"), ("correlation_key", "<u4"),
                         ("message_name", "<u2"), ("bpmn_process_id", "<u2"), ("partition", "<i4"),
                         ("interrupting", "u1"), ("unprocessed", "u1"), ("pad", "u1", (2,))])
XPART_DTYPE = np.dtype([("element_instance_key", "<i8"), ("process_instance_key", "<i8"), ("message_key", "<i8"),
                        ("correlation_key", "<u4"), ("instance", "<u4"), ("element_ord", "<u2"),
                        ("message_name", "<u2"), ("bpmn_process_id", "<u2"), ("kind", "u1"),
                        ("interrupting", "u1"), ("source_partition", "<i2"), ("target_partition", "<i2"),
                        ("pad", "<u4")])

assert COMMAND_DTYPE.itemsize == C.sizeof(Command) == 16
assert DOC_DTYPE.itemsize == C.sizeof(DocEntry) == 16
assert RECORD_DTYPE.itemsize == C.sizeof(Record) == 80
assert XPART_DTYPE.itemsize == C.sizeof(XpartCmd) == 48

# fields compared between the GPU path and the oracle (the rejection reason is compared as text)
PARITY_FIELDS = [f for f in RECORD_DTYPE.names if f not in ("reason", "reason_arg", "pad")]


def make_commands(n):
    return np.zeros(n, dtype=COMMAND_DTYPE)


def make_docs(n):
    return np.zeros(n, dtype=DOC_DTYPE)


def make_xparts(n):
    return np.zeros(n, dtype=XPART_DTYPE)


def record_tuple(r, element_id=None, name=None):
    """Canonical comparable tuple of one drained record (numpy row or ctypes Record)."""
    return (int(r["source_index"]), int(r["ordinal"]), int(r["record_type"]), int(r["value_type"]),
            int(r["intent"]), int(r["rejection_type"]), int(r["key"]), int(r["scope_key"]),
            int(r["process_instance_key"]), int(r["process_idx"]), int(r["element_idx"]), int(r["aux"]),
            int(r["message_key"]), int(r["correlation_key"]), int(r["message_name"]), int(r["bpmn_process_id"]),
            int(r["partition"]), int(r["interrupting"]))


class JobFail(C.Structure):
    """zbhip_job_fail (JOB:FAIL of a device job)."""
    _fields_ = [("job_key", C.c_int64), ("retry_backoff", C.c_int64), ("timestamp", C.c_int64), ("error_message", C.c_char_p),
                ("error_message_len", C.c_size_t), ("retries", C.c_int32), ("n_variables", C.c_uint32)]
