"""TEST INFRASTRUCTURE ONLY -- CPU restatement of zb-db's byte encoding of the hot path's state
(SURVEY.md §8(f) row 2), the checker of zbhip_export_state_db (zeebe_amd/csrc/statedb.cpp).

Input: the canonical state rows both engines export ("CF|key parts|value fields", compared for
equality by the parity tests) plus the deployment tables.  Output: (column family ordinal, key
bytes, value bytes) as RocksDB holds them:
  * key = 8-byte big-endian column-family ordinal (ColumnFamilyContext.writeKey, ZeebeDbConstants
    ZB_DB_BYTE_ORDER = BIG_ENDIAN; ordinals = positions in protocol/.../ZbColumnFamilies.java)
    + the key parts: DbLong 8 bytes BE, DbInt 4 bytes BE, DbString 4-byte BE length + bytes
    (zb-db/.../impl/DbLong.java, DbInt.java, DbString.java), DbCompositeKey first ++ second,
    DbForeignKey = its inner key, DbTenantAwareKey SUFFIX = wrapped ++ tenant (DbTenantAwareKey.java);
  * value = DbNil one 0xFF byte (DbNil.java), DbLong / DbInt as above, or an UnpackedObject's
    msgpack (ObjectValue.write, oracle/logserial.py):
      ELEMENT_INSTANCE_KEY  DbLong -> ElementInstance (state/instance/ElementInstance.java:23-55)
                            with IndexedRecord (IndexedRecord.java:22-29) around the element's
                            ProcessInstanceRecord;
      ELEMENT_INSTANCE_PARENT_CHILD  [parent, child] -> DbNil (DbElementInstanceState.java:80-97);
      ELEMENT_INSTANCE_CHILD_PARENT  child -> DbLong parent (DbVariableState.java:57-63);
      NUMBER_OF_TAKEN_SEQUENCE_FLOWS [[flowScopeKey, gatewayId], flowId] -> DbInt (:114-121);
      PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY [definitionKey, piKey] -> DbNil (:124-131);
      VARIABLES [scopeKey, name] -> VariableInstance{key, value} (DbVariableState.java:66-73,
                            VariableInstance.java:18-22);
      EVENT_SCOPE key -> EventScopeInstance{accepting, interrupting [], boundaryElementIds [],
                            interrupted} (DbEventScopeInstanceState.java:35-39, EventScopeInstance.java);
      JOBS key -> JobRecordValue{jobRecord} stored without variables (DbJobState.java:77-81);
      JOB_STATES key -> JobStateValue{jobState: ACTIVATABLE} (:84-85);
      JOB_ACTIVATABLE [[type, jobKey], tenant] -> DbNil (:87-95, PlacementType.SUFFIX);
      JOB_DEADLINES [deadline, jobKey] -> DbNil (:100-102; activated jobs);
      KEY "latestKey" -> NextValue{nextValue} (stream-platform/.../state/NextValueManager.java:32-34,
                            DbKeyGenerator.java:21).
      MESSAGE_SUBSCRIPTION_BY_KEY [eik, name] -> MessageSubscription{record, key, correlating};
      MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY [[tenant, [name, correlationKey]], eik] -> DbNil;
      PROCESS_SUBSCRIPTION_BY_KEY [eik, [tenant, name]] -> ProcessMessageSubscription{record, state, key};
      MESSAGE_STATS "deadline_message_count" -> DbLong (DbMessageState.java:165-175).
Parity of the values is
restated from the code (no reference fixture holds zb-db bytes): "parity unpinned" beyond the
msgpack primitives oracle/logserial.py is pinned on.
"""
import struct

from oracle import logserial as LS

CF = {"KEY": 1, "ELEMENT_INSTANCE_PARENT_CHILD": 6, "ELEMENT_INSTANCE_KEY": 7, "NUMBER_OF_TAKEN_SEQUENCE_FLOWS": 8,
      "ELEMENT_INSTANCE_CHILD_PARENT": 9, "VARIABLES": 10, "JOBS": 16, "JOB_STATES": 17, "EVENT_SCOPE": 37,
      "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY": 55, "JOB_ACTIVATABLE": 76, "MESSAGE_SUBSCRIPTION_BY_KEY": 27,
      "MESSAGE_STATS": 54, "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY": 74, "PROCESS_SUBSCRIPTION_BY_KEY": 75,
      "JOB_DEADLINES": 18, "TIMERS": 12, "TIMER_DUE_DATES": 13, "INCIDENTS": 34, "INCIDENT_PROCESS_INSTANCES": 35,
      "INCIDENT_JOBS": 36, "JOB_BACKOFF": 42}
# TimerInstance.java:25-43 (declaration order)
TIMER_INSTANCE = [
    ("handlerNodeId", "str", ""), ("processDefinitionKey", "long", 0), ("key", "long", 0),
    ("elementInstanceKey", "long", 0), ("processInstanceKey", "long", 0), ("dueDate", "long", 0),
    ("repetitions", "int", 0), ("tenantId", "str", "<default>")]
NIL = b"\xff"
PI_INTENT = {1: "SEQUENCE_FLOW_TAKEN", 2: "ELEMENT_ACTIVATING", 3: "ELEMENT_ACTIVATED", 4: "ELEMENT_COMPLETING",
             5: "ELEMENT_COMPLETED", 6: "ELEMENT_TERMINATING", 7: "ELEMENT_TERMINATED"}

ELEMENT_INSTANCE = [
    ("parentKey", "long", -1), ("childCount", "int", 0), ("childActivatedCount", "int", 0),
    ("childCompletedCount", "int", 0), ("childTerminatedCount", "int", 0), ("jobKey", "long", 0),
    ("multiInstanceLoopCounter", "int", 0), ("interruptingElementId", "str", ""),
    ("calledChildInstanceKey", "long", -1), ("elementRecord", "raw", None), ("activeSequenceFlows", "int", 0)]
INDEXED_RECORD = [("key", "long", 0), ("state", "enum", LS.NO_DEFAULT), ("processInstanceRecord", "raw", None)]
VARIABLE_INSTANCE = [("key", "long", LS.NO_DEFAULT), ("value", "bin", LS.NO_DEFAULT)]
EVENT_SCOPE_INSTANCE = [("accepting", "bool", LS.NO_DEFAULT), ("interrupting", "array", []),
                        ("boundaryElementIds", "array", []), ("interrupted", "bool", False)]
NEXT_VALUE = [("nextValue", "long", -1)]


def dblong(v):
    return struct.pack(">q", v)


def dbint(v):
    return struct.pack(">i", v)


def dbstr(s):
    b = s.encode() if isinstance(s, str) else s
    return struct.pack(">i", len(b)) + b


def fields(text):
    out = {}
    for kv in text.split(","):
        k, _, v = kv.partition("=")
        out[k] = v
    return out


def encode_rows(rows, processes, string_value):
    """rows: canonical state rows; processes: oracle process tables (Oracle.process_tables());
    string_value(id) -> bytes.  Returns sorted [(cf, key, value)]."""
    by_def = {p["key"]: p for p in processes}
    out = []
    for row in rows:
        parts = row.split("|")
        name = parts[0]
        if name not in CF:
            continue  # not a column family of the path
        prefix = struct.pack(">q", CF[name])
        if name == "KEY":
            out.append((CF[name], prefix + dbstr(parts[1]), LS.write_object(NEXT_VALUE, {"nextValue": int(parts[2])})))
        elif name == "ELEMENT_INSTANCE_KEY":
            key, f = int(parts[1]), fields(parts[2])
            proc = by_def[int(f["processDefinitionKey"])]
            etype, ev = int(f["bpmnElementType"]), int(f["bpmnEventType"])
            pir = LS.write_object(LS.PROCESS_INSTANCE, dict(
                bpmnElementType=LS.ELEMENT_TYPE[etype], elementId=f["elementId"], bpmnProcessId=proc["bpmn_process_id"],
                version=proc["version"], processDefinitionKey=proc["key"],
                processInstanceKey=int(f["processInstanceKey"]), flowScopeKey=int(f["flowScopeKey"]),
                bpmnEventType=LS.EVENT_TYPE[ev]))
            rec = LS.write_object(INDEXED_RECORD, {"key": key, "state": PI_INTENT[int(f["state"])],
                                                   "processInstanceRecord": pir})
            val = LS.write_object(ELEMENT_INSTANCE, dict(
                parentKey=int(f["parentKey"]), childCount=int(f["childCount"]), jobKey=int(f["jobKey"]),
                childActivatedCount=int(f["childActivatedCount"]), childCompletedCount=int(f["childCompletedCount"]),
                childTerminatedCount=int(f["childTerminatedCount"]),
                multiInstanceLoopCounter=int(f["multiInstanceLoopCounter"]),
                interruptingElementId=f["interruptingElementId"], calledChildInstanceKey=int(f["calledChildInstanceKey"]),
                elementRecord=rec, activeSequenceFlows=int(f["activeSequenceFlows"])))
            out.append((CF[name], prefix + dblong(key), val))
        elif name == "ELEMENT_INSTANCE_PARENT_CHILD":
            out.append((CF[name], prefix + dblong(int(parts[1])) + dblong(int(parts[2])), NIL))
        elif name == "ELEMENT_INSTANCE_CHILD_PARENT":
            out.append((CF[name], prefix + dblong(int(parts[1])), dblong(int(parts[2]))))
        elif name == "NUMBER_OF_TAKEN_SEQUENCE_FLOWS":
            out.append((CF[name], prefix + dblong(int(parts[1])) + dbstr(parts[2]) + dbstr(parts[3]), dbint(int(parts[4]))))
        elif name == "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY":
            out.append((CF[name], prefix + dblong(int(parts[1])) + dblong(int(parts[2])), NIL))
        elif name == "VARIABLES":
            f = fields(parts[3])
            if int(f["type"]) == LS.DOC_LIST:  # a list: its items in the row ("type:value;...")
                items = [tuple(int(x) for x in it.split(":")) for it in f["value"].split(";") if it]
                entry = {"type": LS.DOC_LIST, "value": 0}
                vb = LS.value_bytes(entry, string_value, lambda _: items)
            else:
                entry = {"type": int(f["type"]), "value": int(f["value"])}
                vb = LS.value_bytes(entry, string_value)
            val = LS.write_object(VARIABLE_INSTANCE, {"key": int(f["key"]), "value": vb})
            out.append((CF[name], prefix + dblong(int(parts[1])) + dbstr(parts[2]), val))
        elif name == "EVENT_SCOPE":
            f = fields(parts[2])
            def ids(v):  # ';'-separated element ids -> ArrayProperty<StringValue> items
                out = []
                for x in (v.split(";") if v else []):
                    w = LS.MsgPackWriter()
                    w.string(x)
                    out.append(bytes(w.b))
                return out
            val = LS.write_object(EVENT_SCOPE_INSTANCE, {"accepting": f["accepting"] == "1",
                                                      "interrupted": f["interrupted"] == "1",
                                                      "interrupting": ids(f.get("interrupting", "")),
                                                      "boundaryElementIds": ids(f.get("boundaryElementIds", ""))})
            out.append((CF[name], prefix + dblong(int(parts[1])), val))
        elif name == "JOBS":
            key, f = int(parts[1]), fields(parts[2])
            failed = {}
            if "errorMessageHex" in f:  # a failed job's stored fields (JobFailProcessor.failJob)
                failed = dict(errorMessage=bytes.fromhex(f["errorMessageHex"]).decode(),
                              retryBackoff=int(f["retryBackoff"]), recurringTime=int(f["recurringTime"]))
            # the stored job's customHeaders: its element's task headers (BpmnJobBehavior.encodeHeaders)
            proc = by_def.get(int(f["processDefinitionKey"]))
            hdr = {}
            if proc is not None and proc.get("headers"):
                for e, el in enumerate(proc["elements"]):
                    if el[2] == f["elementId"] and proc["headers"][e]:
                        hdr = {"customHeaders": proc["headers"][e]}
            job = LS.write_object(LS.JOB, dict(
                deadline=int(f.get("deadline", -1)), worker=f.get("worker", ""), **failed, **hdr,
                retries=int(f["retries"]), type=f["type"], bpmnProcessId=f["bpmnProcessId"],
                processDefinitionVersion=int(f["processDefinitionVersion"]),
                processDefinitionKey=int(f["processDefinitionKey"]), processInstanceKey=int(f["processInstanceKey"]),
                elementId=f["elementId"], elementInstanceKey=int(f["elementInstanceKey"]), tenantId=f["tenantId"]))
            out.append((CF[name], prefix + dblong(key), LS.write_object([("jobRecord", "raw", None)], {"jobRecord": job})))
        elif name == "JOB_STATES":
            out.append((CF[name], prefix + dblong(int(parts[1])),
                        LS.write_object([("jobState", "enum", LS.NO_DEFAULT)], {"jobState": parts[2]})))
        elif name == "MESSAGE_SUBSCRIPTION_BY_KEY":  # DbMessageSubscriptionState.java:64-73, MessageSubscription.java
            f = fields(parts[3])
            rec = LS.write_object(LS.MESSAGE_SUBSCRIPTION, dict(
                processInstanceKey=int(f["processInstanceKey"]), elementInstanceKey=int(parts[1]),
                messageKey=int(f["messageKey"]), messageName=parts[2], correlationKey=f["correlationKey"],
                interrupting=f["interrupting"] == "1", bpmnProcessId=f["bpmnProcessId"]))
            val = LS.write_object([("record", "raw", None), ("key", "long", LS.NO_DEFAULT), ("correlating", "bool", False)],
                                  {"record": rec, "key": int(f["key"]), "correlating": f["correlating"] == "1"})
            out.append((CF[name], prefix + dblong(int(parts[1])) + dbstr(parts[2]), val))
        elif name == "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY":  # :75-86, tenant PREFIX
            out.append((CF[name], prefix + dbstr(parts[1]) + dbstr(parts[2]) + dbstr(parts[3]) + dblong(int(parts[4])),
                        NIL))
        elif name == "PROCESS_SUBSCRIPTION_BY_KEY":  # DbProcessMessageSubscriptionState.java:53-66
            f = fields(parts[3])
            rec = LS.write_object(LS.PROCESS_MESSAGE_SUBSCRIPTION, dict(
                subscriptionPartitionId=int(f["subscriptionPartitionId"]), processInstanceKey=int(f["processInstanceKey"]),
                elementInstanceKey=int(parts[1]), messageKey=int(f["messageKey"]), messageName=parts[2],
                interrupting=f["interrupting"] == "1", bpmnProcessId=f["bpmnProcessId"],
                correlationKey=f["correlationKey"], elementId=f["elementId"]))
            val = LS.write_object([("record", "raw", None), ("state", "enum", "STATE_OPENING"), ("key", "long", LS.NO_DEFAULT)],
                                  {"record": rec, "state": "STATE_" + f["state"], "key": int(f["key"])})
            out.append((CF[name], prefix + dblong(int(parts[1])) + dbstr("<default>") + dbstr(parts[2]), val))
        elif name == "MESSAGE_STATS":  # DbMessageState.java:165-175
            out.append((CF[name], prefix + dbstr("deadline_message_count"), dblong(int(parts[2]))))
        elif name == "TIMERS":  # DbTimerInstanceState: [elementInstanceKey, timerKey] -> TimerInstance
            f = fields(parts[3])
            val = LS.write_object(TIMER_INSTANCE, dict(
                handlerNodeId=f["handlerNodeId"], processDefinitionKey=int(f["processDefinitionKey"]), key=int(f["key"]),
                elementInstanceKey=int(f["elementInstanceKey"]), processInstanceKey=int(f["processInstanceKey"]),
                dueDate=int(f["dueDate"]), repetitions=int(f["repetitions"]), tenantId=f["tenantId"]))
            out.append((CF[name], prefix + dblong(int(parts[1])) + dblong(int(parts[2])), val))
        elif name == "INCIDENTS":  # DbIncidentState: incidentKey -> Incident{incidentRecord} (Incident.java)
            f = fields(parts[2])
            proc = by_def[int(f["processDefinitionKey"])]
            et, eik = int(f["errorType"]), int(f["elementInstanceKey"])
            job = int(f.get("jobKey", -1))  # a job's incident (JOB_NO_RETRIES): its key and message
            msg = bytes.fromhex(f["messageHex"]).decode() if job >= 0 else \
                LS.incident_message(proc, et, int(f["flow"]), int(f["result"]))
            rec = LS.write_object(LS.INCIDENT, dict(
                errorType=LS.ERROR_TYPE[et], errorMessage=msg,
                bpmnProcessId=proc["bpmn_process_id"], processDefinitionKey=proc["key"],
                processInstanceKey=int(f["processInstanceKey"]), elementId=f["elementId"], elementInstanceKey=eik,
                jobKey=job, variableScopeKey=eik))
            out.append((CF[name], prefix + dblong(int(parts[1])), LS.write_object([("incidentRecord", "raw", None)],
                                                                                  {"incidentRecord": rec})))
        elif name == "INCIDENT_PROCESS_INSTANCES":  # DbForeignKey<DbLong> eik -> IncidentKey{key}
            out.append((CF[name], prefix + dblong(int(parts[1])),
                        LS.write_object([("key", "long", LS.NO_DEFAULT)], {"key": int(parts[2])})))
        elif name == "INCIDENT_JOBS":  # DbForeignKey<DbLong> jobKey -> IncidentKey{key}
            out.append((CF[name], prefix + dblong(int(parts[1])),
                        LS.write_object([("key", "long", LS.NO_DEFAULT)], {"key": int(parts[2])})))
        elif name == "JOB_BACKOFF":  # [recurringTime, jobKey] -> DbNil (DbJobState.java:103-108)
            out.append((CF[name], prefix + dblong(int(parts[1])) + dblong(int(parts[2])), NIL))
        elif name == "TIMER_DUE_DATES":  # [dueDate, [elementInstanceKey, timerKey]] -> DbNil
            out.append((CF[name], prefix + dblong(int(parts[1])) + dblong(int(parts[2])) + dblong(int(parts[3])), NIL))
        elif name == "JOB_DEADLINES":  # DbJobState.java:100-102: [deadline, jobKey] -> DbNil
            out.append((CF[name], prefix + dblong(int(parts[1])) + dblong(int(parts[2])), NIL))
        elif name == "JOB_ACTIVATABLE":
            out.append((CF[name], prefix + dbstr(parts[1]) + dblong(int(parts[3])) + dbstr(parts[2]), NIL))
    return sorted(out)
