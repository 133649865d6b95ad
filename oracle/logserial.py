"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's log serialisation of the hot
path's records, the checker of zeebe_amd/csrc/logwriter.cpp.

Only tests/ may import this module.  It restates, in plain Python:
  * msgpack-core MsgPackWriter (msgpack-core/.../spec/MsgPackWriter.java:62-316);
  * msgpack-value ObjectValue.write (msgpack-value/.../value/ObjectValue.java:78-84,152-158):
    every declared property in declaration order, the default when unset; StringValue -> str,
    EnumValue -> its name as str (EnumValue.java:33-35), Long/IntegerValue -> writeInteger,
    BinaryValue / DocumentValue -> bin (BinaryValue.java:40-42), PackedValue -> raw bytes
    (PackedValue.java:28-30), ArrayValue -> array header + items (ArrayValue.java:31-35);
  * the record values the engine writes for the path (protocol-impl/.../record/value/...):
    ProcessInstanceRecord.java:62-74, JobRecord.java:39-83, VariableRecord.java:25-41,
    ProcessEventRecord.java:25-42, ProcessInstanceCreationRecord.java:32-55, MessageRecord.java:37-43,
    MessageSubscriptionRecord.java:40-48, ProcessMessageSubscriptionRecord.java:44-54, with the field values
    of BpmnStateTransitionBehavior.java:243-339, CreateProcessInstanceProcessor.java:129-158,319-330,
    BpmnJobBehavior.java:194-218,359-400 (jobRecord reused, variables EMPTY_DOCUMENT, NO_HEADERS),
    JobCompleteProcessor.java:75-92, EventTriggerBehavior.java:148-166, EventHandle.java:151-158,
    VariableBehavior.java:60-200, ResultBuilderBackedRejectionWriter.java:25-38 (command value);
  * RecordMetadata's SBE encoding (protocol/src/main/resources/protocol.xml:137-152,
    common-types.xml; RecordMetadata.java write/reset, schema version 4 = protocol/pom.xml:28)
    with the writers' metadata (ResultBuilderBackedTypedCommandWriter.java:43-47,
    ResultBuilderBackedEventApplyingStateWriter.java:40-56 recordVersion = latest applier
    version = 1 for every intent of the path, EventAppliers.java:311-325);
  * the log entry (LogEntryDescriptor.java static block: 40-byte header), dispatcher framing
    (DataFrameDescriptor.java: 12-byte header, 8-byte alignment) and batch sequencing
    (SequencedBatchSerializer.java:33-67: consecutive positions, sourcePosition = the batch's
    command, one timestamp), processed follow-up commands flagged (ProcessingStateMachine.java:
    388-417 LogAppendEntry.ofProcessed).
Pinned by tests/golden/msgpack_writer.json (MsgPackWriterTest.java vectors) and
tests/golden/record_json.json (JsonSerializableToJsonTest.java record values).
"""
import struct

# ---- MsgPackWriter ------------------------------------------------------------------------------


class MsgPackWriter:
    def __init__(self):
        self.b = bytearray()

    def map_header(self, n):  # :85-102
        if n < 16:
            self.b.append(0x80 | n)
        elif n < 1 << 16:
            self.b += b"\xde" + struct.pack(">H", n)
        else:
            self.b += b"\xdf" + struct.pack(">I", n)

    def array_header(self, n):  # :62-83
        if n < 16:
            self.b.append(0x90 | n)
        elif n < 1 << 16:
            self.b += b"\xdc" + struct.pack(">H", n)
        else:
            self.b += b"\xdd" + struct.pack(">I", n)

    def integer(self, v):  # :154-212, signed semantics
        if v < -(1 << 5):
            if v < -(1 << 15):
                if v < -(1 << 31):
                    self.b += b"\xd3" + struct.pack(">q", v)
                else:
                    self.b += b"\xd2" + struct.pack(">i", v)
            elif v < -(1 << 7):
                self.b += b"\xd1" + struct.pack(">h", v)
            else:
                self.b += b"\xd0" + struct.pack(">b", v)
        elif v < (1 << 7):
            self.b += struct.pack(">b", v)
        elif v < (1 << 16):
            if v < (1 << 8):
                self.b += b"\xcc" + struct.pack(">B", v)
            else:
                self.b += b"\xcd" + struct.pack(">H", v)
        elif v < (1 << 32):
            self.b += b"\xce" + struct.pack(">I", v)
        else:
            self.b += b"\xcf" + struct.pack(">q", v)

    def string_header(self, n):  # :214-240
        if n < 32:
            self.b.append(0xA0 | n)
        elif n < 1 << 8:
            self.b += b"\xd9" + struct.pack(">B", n)
        elif n < 1 << 16:
            self.b += b"\xda" + struct.pack(">H", n)
        else:
            self.b += b"\xdb" + struct.pack(">I", n)

    def string(self, s):
        raw = s.encode() if isinstance(s, str) else bytes(s)
        self.string_header(len(raw))
        self.b += raw

    def binary_header(self, n):  # :252-275
        if n < 1 << 8:
            self.b += b"\xc4" + struct.pack(">B", n)
        elif n < 1 << 16:
            self.b += b"\xc5" + struct.pack(">H", n)
        else:
            self.b += b"\xc6" + struct.pack(">I", n)

    def binary(self, raw):
        self.binary_header(len(raw))
        self.b += raw

    def boolean(self, v):
        self.b.append(0xC3 if v else 0xC2)

    def nil(self):
        self.b.append(0xC0)

    def float_(self, v):  # :297-316: float32 when exact
        f = struct.unpack(">f", struct.pack(">f", v))[0] if abs(v) <= 3.4028234663852886e38 else None
        if f is not None and f == v:
            self.b += b"\xca" + struct.pack(">f", v)
        else:
            self.b += b"\xcb" + struct.pack(">d", v)


# ---- ObjectValue with declared properties ---------------------------------------------------------
# property kinds: "str", "enum", "long", "int", "bin" (BinaryValue / DocumentValue), "raw"
# (PackedValue), "array" (items: raw msgpack of each element)
NO_DEFAULT = object()
EMPTY_DOCUMENT = b"\x80"  # MsgPackHelper.EMTPY_OBJECT


def write_object(schema, values, w=None):
    w = w or MsgPackWriter()
    w.map_header(len(schema))
    for name, kind, default in schema:
        v = values.get(name, default)
        if v is NO_DEFAULT:
            raise ValueError("property %s has no value" % name)
        w.string(name)
        if kind in ("str", "enum"):
            w.string(v)
        elif kind in ("long", "int"):
            w.integer(v)
        elif kind == "bin":
            w.binary(v)
        elif kind == "bool":
            w.boolean(v)
        elif kind == "raw":
            w.b += v
        elif kind == "array":
            w.array_header(len(v))
            for item in v:
                w.b += item
        else:
            raise ValueError(kind)
    return bytes(w.b)


# ProcessInstanceRecord.java:37-73 (declaration order :63-73)
PROCESS_INSTANCE = [
    ("bpmnElementType", "enum", "UNSPECIFIED"), ("elementId", "str", ""), ("bpmnProcessId", "str", ""),
    ("version", "int", -1), ("processDefinitionKey", "long", -1), ("processInstanceKey", "long", -1),
    ("flowScopeKey", "long", -1), ("bpmnEventType", "enum", "UNSPECIFIED"),
    ("parentProcessInstanceKey", "long", -1), ("parentElementInstanceKey", "long", -1),
    ("tenantId", "str", "<default>")]
# JobRecord.java:39-83
JOB = [
    ("deadline", "long", -1), ("worker", "str", ""), ("retries", "int", -1), ("retryBackoff", "long", 0),
    ("recurringTime", "long", -1), ("type", "str", ""), ("customHeaders", "raw", EMPTY_DOCUMENT),
    ("variables", "bin", EMPTY_DOCUMENT), ("errorMessage", "str", ""), ("errorCode", "str", ""),
    ("bpmnProcessId", "str", ""), ("processDefinitionVersion", "int", -1), ("processDefinitionKey", "long", -1),
    ("processInstanceKey", "long", -1), ("elementId", "str", ""), ("elementInstanceKey", "long", -1),
    ("tenantId", "str", "<default>")]
# VariableRecord.java:25-41
VARIABLE = [
    ("name", "str", NO_DEFAULT), ("value", "bin", NO_DEFAULT), ("scopeKey", "long", NO_DEFAULT),
    ("processInstanceKey", "long", NO_DEFAULT), ("processDefinitionKey", "long", NO_DEFAULT),
    ("bpmnProcessId", "str", ""), ("tenantId", "str", "<default>")]
# ProcessEventRecord.java:25-42
PROCESS_EVENT = [
    ("scopeKey", "long", NO_DEFAULT), ("targetElementId", "str", NO_DEFAULT), ("variables", "bin", EMPTY_DOCUMENT),
    ("processDefinitionKey", "long", -1), ("processInstanceKey", "long", -1), ("tenantId", "str", "<default>")]
# TimerRecord.java:24-40 (every property written by CatchEventBehavior.subscribeToTimerEvent)
TIMER = [
    ("elementInstanceKey", "long", NO_DEFAULT), ("processInstanceKey", "long", NO_DEFAULT),
    ("dueDate", "long", NO_DEFAULT), ("targetElementId", "str", NO_DEFAULT), ("repetitions", "int", NO_DEFAULT),
    ("processDefinitionKey", "long", NO_DEFAULT), ("tenantId", "str", "<default>")]
# IncidentRecord.java:20-47
INCIDENT = [
    ("errorType", "enum", "UNKNOWN"), ("errorMessage", "str", ""), ("bpmnProcessId", "str", ""),
    ("processDefinitionKey", "long", -1), ("processInstanceKey", "long", -1), ("elementId", "str", ""),
    ("elementInstanceKey", "long", -1), ("jobKey", "long", -1), ("variableScopeKey", "long", -1),
    ("tenantId", "str", "<default>")]
ERROR_TYPE = {2: "JOB_NO_RETRIES", 3: "CONDITION_ERROR", 4: "EXTRACT_VALUE_ERROR"}  # ErrorType.java ordinals
FEEL_RESULT = {0: "NULL", 1: "NUMBER", 2: "STRING"}


def incident_message(p, error_type, flow, result):
    """errorMessage of an exclusive gateway's incident: ExclusiveGatewayProcessor.java:121-125
    (CONDITION_ERROR) or ExpressionProcessor.typeCheck (:356-368, EXTRACT_VALUE_ERROR)."""
    if error_type == 3:
        return "Expected at least one condition to evaluate to true, or to have a default flow"
    return "Expected result of the expression '%s' to be 'BOOLEAN', but was '%s'." % (
        p["cond_text"][flow], FEEL_RESULT[result])


# ProcessInstanceBatchRecord.java:18-40 (no tenantId)
PROCESS_INSTANCE_BATCH = [
    ("processInstanceKey", "long", NO_DEFAULT), ("batchElementInstanceKey", "long", NO_DEFAULT),
    ("index", "long", -1)]
# ProcessInstanceCreationRecord.java:32-55 (ArrayProperty is always set, ArrayProperty.java)
PROCESS_INSTANCE_CREATION = [
    ("bpmnProcessId", "str", ""), ("processDefinitionKey", "long", -1), ("processInstanceKey", "long", -1),
    ("version", "int", -1), ("variables", "bin", EMPTY_DOCUMENT), ("fetchVariables", "array", []),
    ("startInstructions", "array", []), ("tenantId", "str", "<default>")]
# MessageRecord.java:37-43 (name, correlationKey, timeToLive have no default)
MESSAGE = [
    ("name", "str", NO_DEFAULT), ("correlationKey", "str", NO_DEFAULT), ("timeToLive", "long", NO_DEFAULT),
    ("variables", "bin", EMPTY_DOCUMENT), ("messageId", "str", ""), ("deadline", "long", -1),
    ("tenantId", "str", "<default>")]
# MessageSubscriptionRecord.java:40-48
MESSAGE_SUBSCRIPTION = [
    ("processInstanceKey", "long", NO_DEFAULT), ("elementInstanceKey", "long", NO_DEFAULT), ("messageKey", "long", -1),
    ("messageName", "str", ""), ("correlationKey", "str", ""), ("interrupting", "bool", True),
    ("bpmnProcessId", "str", ""), ("variables", "bin", EMPTY_DOCUMENT), ("tenantId", "str", "<default>")]
# ProcessMessageSubscriptionRecord.java:44-54
PROCESS_MESSAGE_SUBSCRIPTION = [
    ("subscriptionPartitionId", "int", NO_DEFAULT), ("processInstanceKey", "long", NO_DEFAULT),
    ("elementInstanceKey", "long", NO_DEFAULT), ("messageKey", "long", -1), ("messageName", "str", ""),
    ("variables", "bin", EMPTY_DOCUMENT), ("interrupting", "bool", True), ("bpmnProcessId", "str", ""),
    ("correlationKey", "str", ""), ("elementId", "str", ""), ("tenantId", "str", "<default>")]
# AuthInfo.java: format (enum, UNKNOWN), authData ("")
AUTH_INFO = [("format", "enum", "UNKNOWN"), ("authData", "str", "")]

ELEMENT_TYPE = {0: "UNSPECIFIED", 1: "PROCESS", 2: "SUB_PROCESS", 3: "EVENT_SUB_PROCESS", 4: "START_EVENT",
                5: "INTERMEDIATE_CATCH_EVENT", 6: "INTERMEDIATE_THROW_EVENT", 7: "BOUNDARY_EVENT", 8: "END_EVENT",
                9: "SERVICE_TASK", 10: "RECEIVE_TASK", 11: "USER_TASK", 12: "MANUAL_TASK", 13: "TASK",
                14: "EXCLUSIVE_GATEWAY", 15: "PARALLEL_GATEWAY", 16: "EVENT_BASED_GATEWAY", 17: "INCLUSIVE_GATEWAY",
                18: "SEQUENCE_FLOW", 19: "MULTI_INSTANCE_BODY", 20: "CALL_ACTIVITY", 21: "BUSINESS_RULE_TASK",
                22: "SCRIPT_TASK", 23: "SEND_TASK"}
EVENT_TYPE = {0: "UNSPECIFIED", 1: "CONDITIONAL", 2: "ERROR", 3: "ESCALATION", 4: "LINK", 5: "MESSAGE", 6: "NONE",
              7: "SIGNAL", 8: "TERMINATE", 9: "TIMER"}

# ---- documents (variables) -------------------------------------------------------------------------
DOC_NIL, DOC_BOOL, DOC_INT, DOC_DEC, DOC_OTHER, DOC_STR, DOC_LIST = 0, 1, 2, 3, 4, 5, 6


def value_bytes(entry, string_value, list_items=None):
    """msgpack of one document value in the canonical encoding a client writes (compact ints,
    float64 for decimals -- exact value v / 10^6 --, shortest str header); a list (`list_items(id)` ->
    [(type, value)]): an array header and its items (MultiInstanceOutputCollectionBehavior.java:43-55,
    writeArrayHeader + the items' own msgpack)."""
    w = MsgPackWriter()
    t, v = entry["type"], int(entry["value"])
    if t == DOC_LIST:
        if list_items is None:
            raise ValueError("a list value without the list dictionary")
        items = list_items(v)
        w.array_header(len(items))
        for it, iv in items:
            w.b += value_bytes({"type": it, "value": iv}, string_value)
        return bytes(w.b)
    if t == DOC_NIL:
        w.nil()
    elif t == DOC_BOOL:
        w.boolean(v != 0)
    elif t == DOC_INT:
        w.integer(v)
    elif t == DOC_DEC:
        w.b += b"\xcb" + struct.pack(">d", v / 1e6)
    elif t == DOC_STR:
        w.string(string_value(v))
    else:
        raise ValueError("document value outside the serialisable subset")
    return bytes(w.b)


def document_bytes(entries, name, string_value, list_items=None):
    if len(entries) == 0:
        return EMPTY_DOCUMENT  # DocumentValue.wrap: empty / nil document -> EMPTY_DOCUMENT
    w = MsgPackWriter()
    w.map_header(len(entries))
    for e in entries:
        w.string(name(int(e["name_id"])))
        w.b += value_bytes(e, string_value, list_items)
    return bytes(w.b)


# ---- SBE RecordMetadata -----------------------------------------------------------------------------
SCHEMA_VERSION = 4            # protocol/pom.xml:28 protocol.version
TEMPLATE_ID = 200             # protocol.xml:137
BLOCK_LENGTH = 32             # recordType 1 + requestStreamId 4 + requestId 8 + protocolVersion 2 + valueType 1
                              # + intent 1 + brokerVersion 12 + recordVersion 2 + rejectionType 1
INT32_NULL = -(1 << 31)       # SBE int32 null (requestStreamIdNullValue)
UINT64_NULL = (1 << 64) - 1   # SBE uint64 null (requestIdNullValue)
REJECTION_NULL = 255          # RejectionType.NULL_VAL


def record_metadata(record_type, value_type, intent, rejection_type=REJECTION_NULL, reason=b"",
                    broker_version=(8, 4, 0), record_version=1):
    auth = write_object(AUTH_INFO, {})
    out = struct.pack("<HHHH", BLOCK_LENGTH, TEMPLATE_ID, 0, SCHEMA_VERSION)
    out += struct.pack("<BiQHBB", record_type, INT32_NULL, UINT64_NULL, SCHEMA_VERSION, value_type, intent)
    out += struct.pack("<iiiHB", broker_version[0], broker_version[1], broker_version[2], record_version,
                       rejection_type)
    out += struct.pack("<I", len(reason)) + reason
    out += struct.pack("<I", len(auth)) + auth
    return out


# ---- log entries ------------------------------------------------------------------------------------
ENTRY_HEADER = 40  # LogEntryDescriptor: version 2, flags 1, reserved 1, position 8, sourcePosition 8,
                   # key 8, timestamp 8, metadataLength 2, unused 2
FRAME_HEADER = 12  # DataFrameDescriptor.HEADER_LENGTH


def log_entry(key, metadata, value, position, source_position, timestamp, processed):
    body = struct.pack("<HBBqqqqHH", 0, 1 if processed else 0, 0, position, source_position, key, timestamp,
                       len(metadata), 0)
    body += metadata + value
    framed = FRAME_HEADER + len(body)
    out = struct.pack("<i", framed) + bytes(8) + body
    return out + bytes((-len(out)) % 8)


# ---- the path's records -----------------------------------------------------------------------------
RT_EVENT, RT_COMMAND, RT_REJECTION = 0, 1, 2
VT_JOB, VT_PI, VT_VARIABLE, VT_PIC, VT_PE = 0, 5, 17, 19, 24
VT_MESSAGE, VT_MS, VT_PMS = 10, 11, 12
VT_TIMER = 15
VT_PIB = 34
VT_INCIDENT = 6
AUX_INLINE = -2
NO_STRING, NO_NAME = 0xFFFFFFFF, 0xFFFF


class Tables:
    """What the serialiser needs from the deployment and the dictionaries: per process a dict
    {bpmn_process_id, version, key, elements: [(type, event_type, id, job_type, retries)]},
    name(id) for variable names, string_value(id) for STR values."""

    def __init__(self, processes, name, string_value, list_items=None):
        self.processes, self.name, self.string_value = processes, name, string_value
        self.list_items = list_items  # list-dictionary id -> [(type, value)] (LIST values)


def _message_value(r, vt, tables, timestamp):
    """Values of the message-correlation records (the drained record carries every field the
    reference record holds: MessagePublishProcessor.java:100-125 deadline = the PUBLISH command's
    timestamp + timeToLive (0 in the subset), SubscriptionCommandSender / the subscription
    processors for the others; message variables are empty in the subset)."""
    name = lambda i: tables.name(i) if i != NO_NAME else ""  # noqa: E731
    corr = int(r["correlation_key"])
    corr_s = tables.string_value(corr) if corr != NO_STRING else b""
    if vt == VT_MESSAGE:
        return write_object(MESSAGE, dict(name=name(int(r["message_name"])), correlationKey=corr_s, timeToLive=0,
                                          deadline=timestamp))
    common = dict(processInstanceKey=int(r["process_instance_key"]), elementInstanceKey=int(r["scope_key"]),
                  messageKey=int(r["message_key"]), messageName=name(int(r["message_name"])), correlationKey=corr_s,
                  interrupting=bool(r["interrupting"]), bpmnProcessId=name(int(r["bpmn_process_id"])))
    if vt == VT_MS:
        return write_object(MESSAGE_SUBSCRIPTION, common)
    p, e = int(r["process_idx"]), int(r["element_idx"])
    elem = tables.processes[p]["elements"][e][2] if p >= 0 and e >= 0 else ""
    return write_object(PROCESS_MESSAGE_SUBSCRIPTION, dict(common, subscriptionPartitionId=int(r["partition"]),
                                                           elementId=elem))


def record_value(r, tables, docs_of_source, doc_entry, timestamp=0, timer_value=None):
    """msgpack record value of one drained record (fields of zbhip_record)."""
    vt, rt = int(r["value_type"]), int(r["record_type"])
    if vt in (VT_MESSAGE, VT_MS, VT_PMS):
        return _message_value(r, vt, tables, timestamp)
    p = tables.processes[int(r["process_idx"])] if int(r["process_idx"]) >= 0 else None
    el = p["elements"][int(r["element_idx"])] if p is not None and int(r["element_idx"]) >= 0 else None
    src_doc = document_bytes(docs_of_source(int(r["source_index"])), tables.name, tables.string_value,
                             getattr(tables, "list_items", None))
    if vt == VT_PI:
        fields = dict(bpmnElementType=ELEMENT_TYPE[el[0]], elementId=el[2], bpmnProcessId=p["bpmn_process_id"],
                      version=p["version"], processDefinitionKey=p["key"],
                      processInstanceKey=int(r["process_instance_key"]), flowScopeKey=int(r["scope_key"]),
                      bpmnEventType=EVENT_TYPE[el[1]] if el[0] != 1 else "UNSPECIFIED")
        return write_object(PROCESS_INSTANCE, fields)
    if vt == VT_JOB:
        if rt == RT_REJECTION:  # the JOB:COMPLETE command's value: defaults + the command's variables
            return write_object(JOB, dict(variables=src_doc))
        fields = dict(retries=el[4], type=el[3], bpmnProcessId=p["bpmn_process_id"],
                      processDefinitionVersion=p["version"], processDefinitionKey=p["key"],
                      processInstanceKey=int(r["process_instance_key"]), elementId=el[2],
                      elementInstanceKey=int(r["scope_key"]))
        hs = p.get("headers")
        if hs and hs[int(r["element_idx"])]:  # zeebe:taskHeaders (BpmnJobBehavior.encodeHeaders)
            fields["customHeaders"] = hs[int(r["element_idx"])]
        if int(r["intent"]) == 2:  # COMPLETED: the stored job + the command's variables
            fields["variables"] = src_doc
        if int(r["message_key"]) != -1:  # an ACTIVATED job (DbJobState.activate): its deadline and worker
            fields["deadline"] = int(r["message_key"])
            cid = int(r["correlation_key"])
            fields["worker"] = tables.string_value(cid) if cid != NO_STRING else ""
        return write_object(JOB, fields)
    if vt == VT_VARIABLE:
        if int(r["aux"]) == AUX_INLINE:  # a value the engine computed (multi-instance loop variables)
            e = {"name_id": int(r["element_idx"]), "type": int(r["partition"]), "value": int(r["message_key"])}
        else:
            e = doc_entry(int(r["aux"]))
        return write_object(VARIABLE, dict(name=tables.name(int(r["element_idx"])),
                                           value=value_bytes(e, tables.string_value, getattr(tables, "list_items", None)),
                                           scopeKey=int(r["scope_key"]),
                                           processInstanceKey=int(r["process_instance_key"]),
                                           processDefinitionKey=p["key"], bpmnProcessId=p["bpmn_process_id"]))
    if vt == VT_PE:
        # TRIGGERED: EventTriggerBehavior.processEventTriggered resets the record (no variables)
        pe_vars = EMPTY_DOCUMENT if int(r["intent"]) == 1 else src_doc
        return write_object(PROCESS_EVENT, dict(scopeKey=int(r["scope_key"]), targetElementId=el[2], variables=pe_vars,
                                                processDefinitionKey=p["key"],
                                                processInstanceKey=int(r["process_instance_key"])))
    if vt == VT_TIMER and rt == RT_REJECTION and timer_value is not None:
        # the TIMER:TRIGGER command's TimerRecord (DueDateTimerChecker.java:118-125), as the rejection
        # writer copies it (TypedRejectionWriter.appendRejection)
        tv = timer_value
        tp = tables.processes[int(tv["process_idx"])] if int(tv["process_idx"]) >= 0 else None
        return write_object(TIMER, dict(elementInstanceKey=int(tv["element_instance_key"]),
                                        processInstanceKey=int(tv["process_instance_key"]), dueDate=int(r["aux"]),
                                        targetElementId=tp["elements"][int(tv["element_idx"])][2] if tp else "",
                                        repetitions=int(tv["repetitions"]),
                                        processDefinitionKey=int(tv["process_definition_key"])))
    if vt == VT_TIMER:  # events: the timer's value (repetitions in `partition`); a rejected TIMER:TRIGGER:
        # the command's key and dueDate (the window's view of it)
        reps = 1 if rt == RT_REJECTION else int(r["partition"])
        return write_object(TIMER, dict(elementInstanceKey=int(r["scope_key"]),
                                        processInstanceKey=int(r["process_instance_key"]), dueDate=int(r["aux"]),
                                        targetElementId=el[2] if el is not None else "", repetitions=reps,
                                        processDefinitionKey=p["key"] if p is not None else -1))
    if vt == VT_INCIDENT:  # BpmnIncidentBehavior.createIncident (:51-71)
        et = int(r["partition"])
        return write_object(INCIDENT, dict(
            errorType=ERROR_TYPE[et], errorMessage=incident_message(p, et, int(r["aux"]), int(r["reason_arg"])),
            bpmnProcessId=p["bpmn_process_id"], processDefinitionKey=p["key"],
            processInstanceKey=int(r["process_instance_key"]), elementId=el[2],
            elementInstanceKey=int(r["scope_key"]), variableScopeKey=int(r["scope_key"])))
    if vt == VT_PIB:
        return write_object(PROCESS_INSTANCE_BATCH, dict(processInstanceKey=int(r["process_instance_key"]),
                                                         batchElementInstanceKey=int(r["scope_key"]),
                                                         index=int(r["partition"])))
    if vt == VT_PIC:
        return write_object(PROCESS_INSTANCE_CREATION, dict(
            bpmnProcessId=p["bpmn_process_id"], processDefinitionKey=p["key"],
            processInstanceKey=int(r["scope_key"]), version=p["version"], variables=src_doc))
    raise ValueError("value type %d outside the serialiser's subset" % vt)


def serialize(records, tables, docs_of_source, doc_entry, reason_text, first_position, source_position, timestamp,
              broker_version=(8, 4, 0), source_timestamp=None, timer_value_of=None):
    """The log bytes of the records' batches: records of one source command form one sequenced
    batch (sourcePosition = that command's position), positions consecutive from first_position."""
    out = bytearray()
    for i, r in enumerate(records):
        rt = int(r["record_type"])
        rej = int(r["rejection_type"]) if rt == RT_REJECTION else REJECTION_NULL
        reason = reason_text(i).encode() if rt == RT_REJECTION else b""
        md = record_metadata(rt, int(r["value_type"]), int(r["intent"]), rej, reason, broker_version)
        si = int(r["source_index"])
        value = record_value(r, tables, docs_of_source, doc_entry,
                             source_timestamp(si) if source_timestamp else timestamp,
                             timer_value_of(si) if timer_value_of else None)
        out += log_entry(int(r["key"]), md, value, first_position + i, source_position(int(r["source_index"])),
                         timestamp, rt == RT_COMMAND and not int(r["unprocessed"]))
    return bytes(out)
