"""Python mirror of the reference-side host adapter (adapter/src/main/java/io/camunda/zeebe/zbhip/
GpuBatchProcessor.java + Window.java), line for line in behaviour: a stream-platform
``RecordProcessor`` (stream-platform/.../stream/api/RecordProcessor.java:17-108) placed before the
engine (StreamProcessorTransitionStep.java:135-147: ``List.of(gpu, engine, checkpointProcessor)``) that
answers the hot-path commands from libzbhip.so and hands everything else to the engine.  It behaves
inside ``ProcessingStateMachine.batchProcessing`` / ``collectBatchProcessingStepResult``
(stream-platform/.../stream/impl/ProcessingStateMachine.java:328-417) as the engine would:

* A device batch is emitted whole when the platform processes its initial command.  The follow-up
  commands the platform then feeds back (``UnwrittenRecord``) were already processed on the device,
  so they return the builder unchanged -- ``out.build()``, not an empty result: the platform skips
  the builder's entries it has seen by their count (``lastProcessingResultSize``).
* Follow-ups the platform writes to the log unprocessed (past ``maxCommandsInBatch``) are device
  continuations (``ZBHIP_OPEN_DEFER_CONTINUATIONS``): they run when the platform reads them back,
  at their own log position (``ZBHIP_CMD_CONTINUE``), after whatever the log holds before them.
* The partition has one key generator (``DbKeyGenerator``): after every device command the engine's
  generator is moved past the device's keys (``KeyGeneratorControls.setKeyIfHigher``), before every
  window the device's past the engine's (``zbhip_set_key_if_higher``).
* A command the device falls back on hands its instance to the engine (zb-db rows through the
  platform's transaction, then evicted) and the engine's keys are declared once its batch is done.
* ``JOB_BATCH:ACTIVATE`` of a job type only device instances hold goes to ``zbhip_activate_jobs``
  (JobBatchActivateProcessor.java:60-143).
* After recovery, instances of device processes move from the engine's state into HBM
  (``on_recovered`` -> ``zbhip_import_state``), as StreamProcessorLifecycleAware.onRecovered would.
* Config 5 (``correlation_keys`` > 0): MESSAGE:PUBLISH (time-to-live 0, no message id, no
  variables), MESSAGE_SUBSCRIPTION:CREATE / CORRELATE and PROCESS_MESSAGE_SUBSCRIPTION:CREATE /
  CORRELATE go to the device.  The cross-partition commands a device batch sends
  (``zbhip_outbox_command``) are handed to ``InterPartitionCommandSender.sendCommand`` in a post-commit
  task of that batch, as SubscriptionCommandSender.handleFollowUpCommandBasedOnPartition (:320-338)
  does; received ones become device commands again (``xpart_of``).

Record values are dicts keyed by the reference's property names (ProcessInstanceRecord.java:61-72,
JobRecord, VariableRecord, ProcessEventRecord, TimerRecord, ProcessInstanceCreationRecord,
JobBatchRecord); variable documents are tuples of (name, value) in document order.

Platform objects used (duck-typed like the Java interfaces):
  record  -- TypedRecord: record_type, value_type, intent, key, value, position (None for an
             UnwrittenRecord), timestamp
  out     -- ProcessingResultBuilder: append_record(key, record_type, value_type, intent,
             rejection_type, rejection_reason, value); build()
  reader  -- LogStreamReader: seek(position), has_next(), next() (records with .processed)
  engine  -- the engine's RecordProcessor (accepts / process / replay / on_processing_error)
  zeebe_db-- RawDbWriter: upsert(rows) of a hand-off (the zb-db rows of the instance)
  key_generator -- DbKeyGenerator: current_key(), set_key_if_higher(key)
"""
import copy
import types

import numpy as np

from . import abi
from .engine import Partition

VT_JOB_BATCH = abi.VT_JOB_BATCH
JOB_BATCH_ACTIVATE, JOB_BATCH_ACTIVATED = abi.JOB_BATCH_ACTIVATE, abi.JOB_BATCH_ACTIVATED
MESSAGE_VALUE_TYPES = (abi.VT_MESSAGE, abi.VT_MESSAGE_SUBSCRIPTION, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION)
# zbhip_xpart_cmd kind <-> (value type, intent) of the command SubscriptionCommandSender sends
XPART_COMMAND = {abi.CMD_MSG_SUB_CREATE: (abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_CREATE),
                 abi.CMD_MSG_SUB_CORRELATE: (abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_CORRELATE),
                 abi.CMD_PMS_CREATE: (abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CREATE),
                 abi.CMD_PMS_CORRELATE: (abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CORRELATE),
                 abi.CMD_MSG_SUB_DELETE: (abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_DELETE),
                 abi.CMD_PMS_DELETE: (abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_DELETE)}
XPART_KIND = {v: k for k, v in XPART_COMMAND.items()}
KEY_BITS = 51  # Protocol.KEY_BITS


def partition_of_key(key):
    """Protocol.decodePartitionId (protocol/.../Protocol.java:102-104)."""
    return key >> KEY_BITS


def xpart_value(x, name, string_value):
    """The record value of a sent cross-partition command (a zbhip_xpart_cmd row), exactly as the
    SubscriptionCommandSender method that sends it sets it (SubscriptionCommandSender.java:54-218);
    properties it does not set keep their declared defaults (MessageSubscriptionRecord.java:33-48,
    ProcessMessageSubscriptionRecord.java:37-54: interrupting true, messageKey -1, strings empty)."""
    kind = int(x["kind"])
    nm = name(int(x["message_name"]))
    bpmn = name(int(x["bpmn_process_id"])) if int(x["bpmn_process_id"]) != 0xFFFF else ""
    corr = string_value(int(x["correlation_key"])) if int(x["correlation_key"]) != abi.NO_STRING else ""
    pik, eik = int(x["process_instance_key"]), int(x["element_instance_key"])
    if kind == abi.CMD_MSG_SUB_CREATE:  # openMessageSubscription (:54-76)
        return {"processInstanceKey": pik, "elementInstanceKey": eik, "messageKey": -1, "messageName": nm,
                "correlationKey": corr, "interrupting": bool(x["interrupting"]), "bpmnProcessId": bpmn,
                "variables": (), "tenantId": TENANT}
    if kind == abi.CMD_MSG_SUB_CORRELATE:  # correlateMessageSubscription (:200-218)
        return {"processInstanceKey": pik, "elementInstanceKey": eik, "messageKey": -1, "messageName": nm,
                "correlationKey": "", "interrupting": True, "bpmnProcessId": bpmn, "variables": (),
                "tenantId": TENANT}
    if kind == abi.CMD_MSG_SUB_DELETE:  # closeMessageSubscription (:220-236)
        return {"processInstanceKey": pik, "elementInstanceKey": eik, "messageKey": -1, "messageName": nm,
                "correlationKey": "", "interrupting": True, "bpmnProcessId": "", "variables": (),
                "tenantId": TENANT}
    sender = int(x["source_partition"])
    if kind == abi.CMD_PMS_DELETE:  # closeProcessMessageSubscription (:267-283)
        return {"subscriptionPartitionId": sender, "processInstanceKey": pik, "elementInstanceKey": eik,
                "messageKey": -1, "messageName": nm, "variables": (), "interrupting": True,
                "bpmnProcessId": "", "correlationKey": "", "elementId": "", "tenantId": TENANT}
    if kind == abi.CMD_PMS_CREATE:  # openProcessMessageSubscription (:116-134)
        return {"subscriptionPartitionId": sender, "processInstanceKey": pik, "elementInstanceKey": eik,
                "messageKey": -1, "messageName": nm, "variables": (), "interrupting": bool(x["interrupting"]),
                "bpmnProcessId": "", "correlationKey": "", "elementId": "", "tenantId": TENANT}
    # correlateProcessMessageSubscription (:136-159)
    return {"subscriptionPartitionId": sender, "processInstanceKey": pik, "elementInstanceKey": eik,
            "messageKey": int(x["message_key"]), "messageName": nm, "variables": (), "interrupting": True,
            "bpmnProcessId": bpmn, "correlationKey": corr, "elementId": "", "tenantId": TENANT}
PI_COMMAND_INTENTS = (8, 9, 10)  # ACTIVATE_ELEMENT, COMPLETE_ELEMENT, TERMINATE_ELEMENT
TENANT = "<default>"  # TenantOwned.DEFAULT_TENANT_IDENTIFIER


def scalar_entry(v, intern_string):
    """A scalar client value as (zbhip_doc_type, value), or None outside the subset (maps, nested
    arrays, inexact decimals)."""
    if v is None:
        return abi.DOC_NIL, 0
    if isinstance(v, bool):
        return abi.DOC_BOOL, int(v)
    if isinstance(v, int):
        return abi.DOC_INT, v
    if isinstance(v, float):
        scaled = round(v * 10 ** abi.DEC_SCALE)
        return (abi.DOC_DEC, scaled) if scaled / 10 ** abi.DEC_SCALE == v else None
    if isinstance(v, str):
        return abi.DOC_STR, intern_string(v)
    return None


def _mp_str_len(n):
    return 1 + n if n < 32 else 2 + n if n < 256 else 3 + n if n < 65536 else 5 + n


def _mp_value_len(v):
    if v is None or isinstance(v, bool):
        return 1
    if isinstance(v, int):
        if v < -(1 << 5):
            return 9 if v < -(1 << 31) else 5 if v < -(1 << 15) else 3 if v < -(1 << 7) else 2
        return 1 if v < (1 << 7) else 2 if v < (1 << 8) else 3 if v < (1 << 16) else 5 if v < (1 << 32) else 9
    if isinstance(v, float):
        return 9
    if isinstance(v, str):
        return _mp_str_len(len(v.encode()))
    if isinstance(v, (list, tuple)):
        n = len(v)
        return (1 if n < 16 else 3 if n < 65536 else 5) + sum(_mp_value_len(x) for x in v)
    raise ValueError("no msgpack size for %r" % (v,))


def msgpack_key_offsets(variables):
    """The byte offsets of a document's keys as the log writes it (MsgPackWriter: fixmap / map16 header,
    the smallest integer form, float64 decimals, fixstr / str8 / str16 / str32 strings)."""
    n = len(variables)
    at = 1 if n < 16 else 3 if n < 65536 else 5
    out = []
    for name, v in variables:
        out.append(at)
        at += _mp_str_len(len(name.encode())) + _mp_value_len(v)
    return out


def set_merge_order(d, variables):
    """The reference's merge order of a multi-entry document into its rows' pad bytes
    (zbhip_doc_merge_order over the keys' byte offsets; IndexedDocument.java:44-63)."""
    if len(d) < 2:
        return d
    import ctypes as C
    from .native import check, load
    offs = np.asarray(msgpack_key_offsets(variables), dtype=np.uint32)
    check(load().zbhip_doc_merge_order(offs.ctypes.data_as(C.c_void_p), len(d), d.ctypes.data_as(C.c_void_p)),
          "zbhip_doc_merge_order")
    return d


def doc_entries(variables, intern_name, intern_string, intern_list=None):
    """A client's variable document [(name, value)] as zbhip_doc_entry rows (a multi-entry one with its
    merge order), or None when a value is outside the device subset (Window.decodeDocument: maps, nested
    arrays, inexact decimals; arrays of scalars only where the side has a list dictionary, `intern_list`)."""
    d = abi.make_docs(len(variables))
    for j, (name, v) in enumerate(variables):
        d[j]["name_id"] = intern_name(name)
        if isinstance(v, (list, tuple)):
            items = [scalar_entry(x, intern_string) for x in v]
            if intern_list is None or any(x is None for x in items):
                return None
            d[j]["type"], d[j]["value"] = abi.DOC_LIST, intern_list(items)
            continue
        e = scalar_entry(v, intern_string)
        if e is None:
            return None
        d[j]["type"], d[j]["value"] = e
    return set_merge_order(d, variables)


def typed_value(t, v, string_value, list_items=None):
    """A stored variable (zbhip_doc_type, value) as the client's value (a list: a tuple of its items,
    `list_items(id)` -> [(type, value)])."""
    if t == abi.DOC_LIST and list_items is not None:
        return tuple(typed_value(it, iv, string_value) for it, iv in list_items(int(v)))
    return (None if t == abi.DOC_NIL else bool(v) if t == abi.DOC_BOOL else int(v) if t == abi.DOC_INT
            else int(v) / 10 ** abi.DEC_SCALE if t == abi.DOC_DEC else string_value(int(v)) if t == abi.DOC_STR
            else ("other", int(v)))


def _as_job(r):
    """A push's JOB_BATCH row read as the JOB record of its job (the same fields)."""
    j = r.copy()
    j["value_type"] = abi.VT_JOB
    j["intent"] = abi.JOB_CREATED
    j["aux"] = -1
    return j


class RecordValues:
    """zbhip_record rows -> the reference's record values (Window.value).  `procs` are the
    deployment's ProcessDefinitions (by process index), `name` the variable-name dictionary."""

    def __init__(self, procs, name, string_value=None, incident_message=None, streams=None, list_items=None):
        self.procs = procs
        self.name = name
        self.string_value = string_value  # value-dictionary id -> str (inline STR values)
        self.list_items = list_items  # list-dictionary id -> [(type, value)] (inline LIST values)
        self.incident_message = incident_message  # a gateway incident's errorMessage (zbhip_incident_message)
        self.streams = streams if streams is not None else {}  # job streams: type -> (worker, timeout)

    def value(self, r, command_doc=(), entry_value=None, timestamp=0):
        """`timestamp`: the source command's (a MESSAGE record's deadline = timestamp + timeToLive)."""
        vt = int(r["value_type"])
        p = self.procs[max(int(r["process_idx"]), 0)] if self.procs else None
        elem = int(r["element_idx"])
        scope, pik, aux = int(r["scope_key"]), int(r["process_instance_key"]), int(r["aux"])
        if vt == abi.VT_PROCESS_INSTANCE:
            return {"bpmnElementType": p.element_types[elem], "elementId": p.element_ids[elem],
                    "bpmnProcessId": p.bpmn_process_id, "version": p.version,
                    "processDefinitionKey": p.definition_key, "processInstanceKey": pik, "flowScopeKey": scope,
                    "bpmnEventType": p.event_types[elem], "parentProcessInstanceKey": -1,
                    "parentElementInstanceKey": -1, "tenantId": TENANT}
        if vt == abi.VT_JOB:
            v = {"tenantId": TENANT, "variables": tuple(command_doc) if aux >= 0 else ()}
            if elem >= 0:
                v.update({"type": p.job_types[elem], "retries": p.retries[elem], "elementId": p.element_ids[elem],
                          "elementInstanceKey": scope, "processInstanceKey": pik, "bpmnProcessId": p.bpmn_process_id,
                          "processDefinitionVersion": p.version, "processDefinitionKey": p.definition_key})
                if p.custom_headers[elem]:  # zeebe:taskHeaders (BpmnJobBehavior.encodeHeaders)
                    v["customHeaders"] = p.custom_headers[elem]
            if int(r["message_key"]) != -1:  # an ACTIVATED job: the deadline and worker it holds
                cid = int(r["correlation_key"])
                v.update({"deadline": int(r["message_key"]),
                          "worker": self.string_value(cid) if cid != abi.NO_STRING else ""})
            if int(r["record_type"]) in (abi.RT_EVENT, abi.RT_COMMAND) and int(r["reason_arg"]) & 1:
                # a failed job's stored retries and errorMessage (JobFailProcessor.failJob), in its events
                # and in the TIME_OUT command JobTimeoutTrigger writes from the stored record
                eid = int(r["message_name"]) | int(r["bpmn_process_id"]) << 16
                v.update({"retries": int(r["partition"]),
                          "errorMessage": self.string_value(eid) if eid != abi.NO_STRING else ""})
            if int(r["record_type"]) == abi.RT_EVENT and int(r["reason_arg"]) & 4:
                # JOB:ERROR_THROWN (JobThrowErrorProcessor): the errorCode (bit 2) and, no catch event, the
                # NO_CATCH_EVENT_FOUND elementId (bit 3)
                cid = int(r["interrupting"]) | int(r["pad"][0]) << 8 | int(r["pad"][1]) << 16
                v["errorCode"] = self.string_value(cid)
                if int(r["reason_arg"]) & 8:
                    v["elementId"] = "NO_CATCH_EVENT_FOUND"
            return v
        if vt == VT_JOB_BATCH:
            # a job stream's push (BpmnJobActivationBehavior.publishWork :61-100): a fresh JobBatchRecord
            # (type, worker, timeout of the stream) with the one job, its variables left out
            j = self.value(_as_job(r))
            jt = j["type"]
            return {"type": jt, "worker": j.get("worker", ""), "timeout": self.streams.get(jt, ("", -1))[1],
                    "maxJobsToActivate": -1, "jobKeys": (aux,), "jobs": (j,), "variables": (), "truncated": False,
                    "tenantIds": ()}
        if vt == abi.VT_INCIDENT:  # IncidentRecord.java:36-47
            et = int(r["partition"])
            job = et in (abi.ERR_JOB_NO_RETRIES, abi.ERR_UNHANDLED_ERROR_EVENT)
            msg = self.string_value(int(r["correlation_key"])) if job else \
                (self.incident_message(r) if self.incident_message else "")
            no_catch = et == abi.ERR_UNHANDLED_ERROR_EVENT and int(r["reason_arg"]) & 8
            return {"errorType": abi.ERROR_TYPES.get(et, str(et)), "errorMessage": msg,
                    "bpmnProcessId": p.bpmn_process_id, "processDefinitionKey": p.definition_key,
                    "processInstanceKey": pik, "elementId": "NO_CATCH_EVENT_FOUND" if no_catch else p.element_ids[elem],
                    "elementInstanceKey": scope, "jobKey": aux if job else -1, "variableScopeKey": scope,
                    "tenantId": TENANT}
        if vt == abi.VT_VARIABLE:
            # ZBHIP_AUX_INLINE: a value the engine computed (multi-instance loop variables)
            val = typed_value(int(r["partition"]), int(r["message_key"]), self.string_value, self.list_items) \
                if aux == abi.AUX_INLINE else entry_value(aux)
            return {"name": self.name(elem), "value": val, "scopeKey": scope, "processInstanceKey": pik,
                    "processDefinitionKey": p.definition_key, "bpmnProcessId": p.bpmn_process_id, "tenantId": TENANT}
        if vt == abi.VT_PROCESS_EVENT:
            return {"scopeKey": scope, "targetElementId": p.element_ids[elem],
                    "variables": tuple(command_doc) if int(r["intent"]) == abi.PE_TRIGGERING else (),
                    "processDefinitionKey": p.definition_key, "processInstanceKey": pik, "tenantId": TENANT}
        if vt == abi.VT_TIMER:
            return {"elementInstanceKey": scope, "processInstanceKey": pik, "dueDate": aux,
                    "repetitions": int(r["partition"]), "targetElementId": p.element_ids[elem] if elem >= 0 else "",
                    "processDefinitionKey": p.definition_key if elem >= 0 else -1, "tenantId": TENANT}
        if vt == abi.VT_PROCESS_INSTANCE_BATCH:  # ProcessInstanceBatchRecord.java:18-40
            return {"processInstanceKey": pik, "batchElementInstanceKey": scope, "index": int(r["partition"])}
        if vt == abi.VT_PROCESS_INSTANCE_CREATION:
            return {"bpmnProcessId": p.bpmn_process_id, "processDefinitionKey": p.definition_key,
                    "version": p.version, "processInstanceKey": scope, "variables": tuple(command_doc),
                    "tenantId": TENANT}
        if vt == abi.VT_MESSAGE_START_EVENT_SUBSCRIPTION:
            # MessageStartEventSubscriptionRecord.java:26-48 (the engine's records: message start events are
            # outside the device subset)
            nid, cid = int(r["message_name"]), int(r["correlation_key"])
            return {"processDefinitionKey": p.definition_key, "messageName": self.name(nid) if nid != 0xFFFF else "",
                    "startEventId": p.element_ids[elem], "bpmnProcessId": p.bpmn_process_id,
                    "processInstanceKey": pik, "messageKey": int(r["message_key"]),
                    "correlationKey": self.string_value(cid) if cid != abi.NO_STRING else "", "variables": (),
                    "tenantId": TENANT}
        if vt in MESSAGE_VALUE_TYPES:
            # the drained record carries every property of the reference value (logwriter.cpp: the
            # same fields); message variables are empty in the subset, deadline = the PUBLISH
            # command's timestamp + timeToLive 0 (MessagePublishProcessor.java:110)
            nid, bid, cid = int(r["message_name"]), int(r["bpmn_process_id"]), int(r["correlation_key"])
            nm = self.name(nid) if nid != 0xFFFF else ""
            corr = self.string_value(cid) if cid != abi.NO_STRING else ""
            if vt == abi.VT_MESSAGE:  # MessageRecord.java:37-43
                if int(r["reason_arg"]) & 2:  # the fields set (a buffered message, an EXPIRED of the TTL checker)
                    mid = int(r["partition"])
                    return {"name": nm, "correlationKey": corr, "timeToLive": aux, "variables": (),
                            "messageId": self.string_value(mid) if mid >= 0 else "", "deadline": scope,
                            "tenantId": TENANT}
                return {"name": nm, "correlationKey": corr, "timeToLive": 0, "variables": (), "messageId": "",
                        "deadline": timestamp, "tenantId": TENANT}
            bpmn = self.name(bid) if bid != 0xFFFF else ""
            common = {"processInstanceKey": pik, "elementInstanceKey": scope, "messageKey": int(r["message_key"]),
                      "messageName": nm, "correlationKey": corr, "interrupting": bool(r["interrupting"]),
                      "bpmnProcessId": bpmn, "variables": (), "tenantId": TENANT}
            if vt == abi.VT_MESSAGE_SUBSCRIPTION:  # MessageSubscriptionRecord.java:40-48
                return common
            # ProcessMessageSubscriptionRecord.java:44-54
            common.update({"subscriptionPartitionId": int(r["partition"]),
                           "elementId": p.element_ids[elem] if elem >= 0 and int(r["process_idx"]) >= 0 else ""})
            return common
        raise ValueError("value type outside the adapter's subset: %d" % vt)

    def job_batch(self, command, key, jobs, name, string_value):
        """JobBatchRecord of an accepted JOB_BATCH:ACTIVATE (JobBatchActivateProcessor.java:120-143)."""
        v = dict(command)
        out = []
        for j in jobs:
            p = self.procs[int(j["process_idx"])]
            e = int(j["element_idx"])
            out.append({"type": command["type"], "worker": command["worker"], "deadline": int(j["deadline"]),
                        **({"customHeaders": p.custom_headers[e]} if p.custom_headers[e] else {}),
                        "retries": int(j["retries"]), "elementId": p.element_ids[e],
                        "elementInstanceKey": int(j["element_instance_key"]),
                        "processInstanceKey": int(j["process_instance_key"]), "bpmnProcessId": p.bpmn_process_id,
                        "processDefinitionKey": p.definition_key, "processDefinitionVersion": p.version,
                        "variables": tuple((name(int(x["name_id"])),
                                            typed_value(int(x["type"]), x["value"], string_value, self.list_items))
                                           for x in j["variables"][:int(j["n_variables"])]),
                        "tenantId": TENANT})
        v.update({"jobKeys": tuple(int(j["key"]) for j in jobs), "jobs": tuple(out), "truncated": False})
        return v

    def pushed_job(self, push_value, row, name, string_value):
        """The ActivatedJob a job stream receives (BpmnJobActivationBehavior.publishWork :83-97): the
        JOB_BATCH:ACTIVATED record's job with the variables JobVariablesCollector gathered (`row`: a
        zbhip_job_variables / zbo_job_variables row)."""
        j = dict(push_value["jobs"][0])
        j["variables"] = tuple((name(int(x["name_id"])),
                                typed_value(int(x["type"]), x["value"], string_value, self.list_items))
                               for x in row["variables"][:int(row["n_variables"])])
        return j


def push_side_effects(out, pushes, sinks, gather, values, name, string_value):
    """publishWork's side effect for the JOB_BATCH:ACTIVATED records of one command (`pushes`: (job key,
    record value)): the jobs' variables collected now, the stream's push(jobKey, job) after the commit.
    `sinks`: job type -> (fetchVariables, push); `gather(keys, fetch)` -> job-variable rows."""
    by_type = {}
    for key, value in pushes:
        if value["type"] in sinks:
            by_type.setdefault(value["type"], []).append((key, value))
    for jt, items in by_type.items():
        fetch, push = sinks[jt]
        rows = gather([k for k, _ in items], fetch)
        jobs = [(k, values.pushed_job(v, r, name, string_value)) for (k, v), r in zip(items, rows)]

        def task(jobs=jobs, push=push):
            for k, j in jobs:
                push(k, j)
            return True
        out.append_post_commit_task(task)


class DeviceTimerInstanceState:
    """The TimerInstanceState the platform's DueDateTimerChecker reads behind the adapter: the engine's
    timers (RocksDB) and the device's (zbhip_due_timers), merged in TIMER_DUE_DATES order [dueDate,
    [elementInstanceKey, timerKey]] -- DbTimerInstanceState.processTimersWithDueDateBefore (:87-116) over
    both.  `engine` provides due(now) -> [(dueDate, elementInstanceKey, key, TimerRecord)] and
    next_after(now) (the Java adapter wraps the engine's DbTimerInstanceState the same way)."""

    def __init__(self, adapter, engine):
        self.adapter, self.engine = adapter, engine

    def process_timers_with_due_date_before(self, now, visitor):
        if not self.adapter.scheduled_ready():
            return now  # mid-window: look again after the timer resolution
        dev, dev_next = self.adapter.due_timers(now)
        dev_rows = [(v["dueDate"], v["elementInstanceKey"], k, v) for k, v in dev]
        both = sorted(dev_rows + list(self.engine.due(now)), key=lambda t: t[:3])
        # a truncated device scan (due rows left out): the first row left out may precede engine timers
        # ordered after the last row returned, so the merge stops there; the checker runs again at the
        # date returned (processTimersWithDueDateBefore stops at any timer its visitor refuses, :87-116)
        bound = dev_rows[-1][:3] if dev_rows and 0 <= dev_next <= now else None
        for due, eik, key, value in both:
            if bound is not None and (due, eik, key) > bound:
                return min(due, dev_next)
            if not visitor(key, value):
                return due
        later = [d for d in (dev_next, self.engine.next_after(now)) if d >= 0]
        return min(later) if later else -1


class DeviceJobState:
    """The JobState JobTimeoutTrigger reads behind the adapter: the engine's JOB_DEADLINES and the
    device's activated jobs (zbhip_timed_out_jobs), merged in [deadline, jobKey] order --
    DbJobState.forEachTimedOutEntry (:286-298) over both.  `engine` provides timed_out(now) ->
    [(deadline, jobKey, JobRecord)]."""

    def __init__(self, adapter, engine):
        self.adapter, self.engine = adapter, engine

    def for_each_timed_out_entry(self, now, callback):
        dev, dev_next = self.adapter.timed_out_jobs(now, with_next=True) if self.adapter.scheduled_ready() else ([], -1)
        # a truncated device list: engine entries past its last row wait for the trigger's next run
        bound = dev[-1][:2] if dev and dev_next >= 0 else None
        for deadline, key, value in sorted(dev + list(self.engine.timed_out(now)), key=lambda t: t[:2]):
            if bound is not None and (deadline, key) > bound:
                return
            if not callback(key, value):
                return


class DevicePendingSubscriptionState:
    """The pending-subscription states the platform's PendingProcessMessageSubscriptionChecker and
    PendingMessageSubscriptionChecker (MessageObserver) read behind the adapter: the engine's transient
    states and the device's (kept by the adapter from the device's records), visited by last sent time
    (TransientPendingSubscriptionState.entriesBefore): the engine's entries, then the device's, each
    group by last sent time (DeviceScheduledState.java: the engine's visitPending exposes no times).
    `engine` provides the same four calls."""

    def __init__(self, adapter, engine):
        self.adapter, self.engine = adapter, engine
        adapter.engine_pending = engine  # entries moved to the engine go there at once

    def pending_process_message_subscriptions(self, deadline):
        for sub, entry in self.adapter.moved_pending:  # handed-off instances: the engine's now
            self.engine.add_pms(sub, *entry)
        self.adapter.moved_pending.clear()
        dev = self.adapter.pending_process_message_subscriptions(deadline) if self.adapter.scheduled_ready() else []
        return self.engine.pending_process_message_subscriptions(deadline) + dev

    def pending_message_subscriptions(self, deadline):
        for sub, entry in self.adapter.moved_pending_ms:  # subscriptions moved with their key: the engine's now
            self.engine.add_ms(sub, *entry)
        self.adapter.moved_pending_ms.clear()
        dev = self.adapter.pending_message_subscriptions(deadline) if self.adapter.scheduled_ready() else []
        return self.engine.pending_message_subscriptions(deadline) + dev

    def on_sent_pms(self, sub, when):
        self.adapter.on_sent_pms(sub, when)
        self.engine.on_sent_pms(sub, when)

    def on_sent_ms(self, sub, when):
        self.adapter.on_sent_ms(sub, when)
        self.engine.on_sent_ms(sub, when)


class Window:
    """One read-ahead window (Window.java): the zbhip_command rows and documents of consecutive
    hot-path commands and their log positions."""

    def __init__(self):
        self.cmds = []       # zbhip_command rows (dicts)
        self.docs = []       # zbhip_doc_entry rows
        self.doc_values = []  # the client value of each entry (VARIABLE records)
        self.positions = []
        self.instances = []
        self.xparts = []     # received cross-partition commands (zbhip_xpart_cmd rows)
        self.doc_base = 0    # zbhip doc index of this window's first entry

    def reset(self, doc_base):
        self.__init__()
        self.doc_base = doc_base

    def size(self):
        return len(self.cmds)

    def covers(self, position):
        return bool(self.positions) and self.positions[0] <= position <= self.positions[-1]

    def index_of(self, position):
        try:
            return self.positions.index(position)
        except ValueError:
            return -1

    def put(self, record, instance, kind, ref, docs=None, values=(), doc_begin=None, pad=0):
        c = {"instance": instance, "kind": kind, "ref": ref, "doc_count": 0, "doc_begin": 0, "pad": pad}
        if docs is not None and len(docs):
            c["doc_count"], c["doc_begin"] = len(docs), len(self.docs)
            self.docs.extend(docs)
            self.doc_values.extend(values)
        if doc_begin is not None:
            c["doc_begin"] = doc_begin
        self.cmds.append(c)
        self.positions.append(record.position)
        self.instances.append(instance)

    def arrays(self):
        cmds = abi.make_commands(len(self.cmds))
        for i, c in enumerate(self.cmds):
            for f, v in c.items():
                cmds[i][f] = v
        docs = abi.make_docs(len(self.docs))
        for j, d in enumerate(self.docs):
            docs[j] = d
        return cmds, docs


class _Scratch:
    """A result builder for one side's share of a merged command (the records are combined afterwards)."""

    def __init__(self):
        self.entries, self.post_commit = [], []

    def append_record(self, key, record_type, value_type, intent, rejection_type, rejection_reason, value):
        self.entries.append(types.SimpleNamespace(key=key, record_type=record_type, value_type=value_type, intent=intent,
                                                  rejection_type=rejection_type, rejection_reason=rejection_reason,
                                                  value=value))

    def append_post_commit_task(self, task):
        self.post_commit.append(task)

    def build(self):
        return self


class GpuBatchProcessor:
    """The adapter (GpuBatchProcessor.java).  `deployments`: [(bpmn xml, definition key, version)]
    in deployment order; processes the device compiler refuses stay with the engine, as do
    `engine_deployments` (processes the host keeps on the engine, e.g. deployed after start-up).
    JOB_BATCH:ACTIVATE goes to the device only for job types no engine process declares: the
    reference activates jobs of a type across all instances in key order, and the engine's
    JOB_ACTIVATABLE rows are not visible here."""

    WINDOW = 1 << 16

    def __init__(self, engine, reader, deployments, zeebe_db, key_generator, partition_id=1, partition_count=1,
                 device=0, instances=1 << 16, window=None, max_commands_in_batch=100, max_records_per_batch=256,
                 clock=None, engine_deployments=(), correlation_keys=0, command_sender=None):
        self.engine = engine
        self.reader = reader
        self.deployments = deployments
        self.zeebe_db = zeebe_db
        self.key_generator = key_generator
        self.partition_id = partition_id
        self.partition_count = partition_count
        self.device = device
        self.instances = instances
        self.window_size = window or self.WINDOW
        self.limit = max_commands_in_batch
        self.max_records = max_records_per_batch
        self.clock = clock or (lambda: 0)  # ActorClock.currentTimeMillis
        # config 5: correlation slots in HBM (0: message commands stay with the engine) and the
        # platform's InterPartitionCommandSender (RecordProcessorContext.getPartitionCommandSender)
        self.correlation_keys = correlation_keys
        self.command_sender = command_sender
        self.message_names = set()     # message names of the device's catch events (PUBLISH subset)
        # message names of any deployed process's message start events: a publish of such a name is the
        # engine's (MessagePublishProcessor.correlateToMessageStartEvents, :157-180), and so its key
        self.start_message_names = set()
        self.subscriptions = {}        # (elementInstanceKey, messageName) -> correlation slot of an open
                                       # MESSAGE_SUBSCRIPTION (MESSAGE_SUBSCRIPTION_BY_KEY): a CORRELATE's
                                       # value carries no correlation key
        self.engine_owned = set()      # correlation keys whose message state the engine holds (one owner
                                       # per key: _message_state_to_engine)
        self.moved_pending_ms = []     # CORRELATING entries of subscriptions moved with their key
        self.engine_pending = None     # the engine's transient pending states (DevicePendingSubscriptionState)
        self.part = None
        self.by_key, self.latest_by_id, self.by_index = {}, {}, []
        self.engine_job_types = set()  # job types the engine's processes (or handed-off instances) hold
        self.device_job_types = set()  # job types of the device's processes
        from .bpmn import job_types_of
        for xml, _, _ in engine_deployments:
            self.engine_job_types.update(job_types_of(xml))
            self.on_engine_deployment(xml)
        self.used_slots = set()
        self.ended = set()             # ended instances whose slot waits for their continuations
        self.closing = set()           # instance slots with a closing process message subscription
        self.pms_handles = {}          # (elementInstanceKey, messageName) -> (slot, ordinal) of a device
                                       # subscription (its PROCESS_MESSAGE_SUBSCRIPTION:DELETE may come late)
        self.next_free = 0
        self.window = Window()
        self._window_done = True       # every command of the current window was emitted
        self.due_date_checker = None   # DueDateTimerChecker.scheduleTimer of the platform (side effects)
        self.scheduled_cap = 1 << 16   # rows per device scan of the scheduled tasks (the rest: the next run)
        self.pending_pms = {}          # (elementInstanceKey, messageName) -> [sent time, record, opening]
        self.pending_ms = {}           # (elementInstanceKey, messageName) -> [sent time, record]
        self.moved_pending = []        # pending entries of handed-off instances, for the engine's state
        self.handed_off = set()
        self.followups = 0             # follow-ups of the current device batch the platform feeds back
        self.engine_batch = False      # the current batch's initial command went to the engine
        self.pending_declaration = None  # (window index, key before) of a fallback command
        self.continuations = []        # expected continuations, in log order: (id, slot, match key)
        self.doc_total = 0             # document entries submitted so far (zbhip doc indices)
        self.values = None
        self.stream_sinks = {}  # job type -> (fetchVariables, push): the job streams' push side effects
        self.job_streamer = None  # JobStreamer: notifyWorkAvailable(type) of publishWork without a stream
        # what went where (tests read these)
        self.fallback_reasons = []
        self.counts = {"windows": 0, "device_commands": 0, "continuations": 0, "fallbacks": 0, "activations": 0,
                       "engine_commands": 0, "followups_answered": 0, "time_outs": 0, "job_failures": 0,
                       "keys_to_engine": 0}

    # ---- RecordProcessor ----------------------------------------------------------------------
    def init(self):
        pbits = self.partition_id << 51
        self.part = Partition(partition_id=self.partition_id, partition_count=self.partition_count,
                              device=self.device, max_instances=self.instances, max_commands=self.window_size,
                              max_records_per_batch=self.max_records, max_doc_entries=16 * self.window_size,
                              max_commands_in_batch=self.limit, max_correlation_keys=self.correlation_keys,
                              initial_key=self.key_generator.current_key() - pbits, defer_continuations=True)
        for xml, key, version in self.deployments:
            self.deploy(xml, key, version)
        self.values = RecordValues(self.part.processes, self.part.name, self.part.string_value, self.part.incident_message,
                                   list_items=self.part.list_items)

    def deploy(self, xml, key, version):
        from .native import ZbhipError
        try:
            idx = self.part.deploy(xml, key, version)
        except ZbhipError:
            # outside the device subset: its instances (and job types) run on the CPU engine
            from .bpmn import job_types_of
            self.engine_job_types.update(job_types_of(xml))
            self.on_engine_deployment(xml)
            self.by_index.append(None)
            return None
        p = self.part.processes[idx]
        from .bpmn import job_types_of, message_names_of, message_start_names_of
        self.device_job_types.update(job_types_of(xml))
        self.message_names.update(message_names_of(xml))
        self.start_message_names.update(message_start_names_of(xml))
        self.by_key[key] = p
        self.by_index.append(p)
        prev = self.latest_by_id.get(p.bpmn_process_id)
        if prev is None or prev.version < version:
            self.latest_by_id[p.bpmn_process_id] = p
        return p

    def on_engine_deployment(self, xml):
        """A process the engine holds (the device refused it, or the host deployed it there): its message
        start events' names go to the engine from now on."""
        from .bpmn import message_start_names_of
        self.start_message_names.update(message_start_names_of(xml))

    def accepts(self, value_type):
        return value_type in (abi.VT_PROCESS_INSTANCE_CREATION, abi.VT_JOB, abi.VT_TIMER, VT_JOB_BATCH) \
            or (self.correlation_keys > 0 and value_type in MESSAGE_VALUE_TYPES) or self.engine.accepts(value_type)

    def replay(self, record):
        # events only; the appliers write the engine's state.  Instances restored this way move
        # into HBM after recovery (on_recovered)
        self.engine.replay(record)

    def on_recovered(self, entries, resume_position=None):
        """StreamProcessorLifecycleAware.onRecovered: instances of device processes move from the
        engine's state (its zb-db entries [(column family, key, value)], RocksDB after replay) into HBM
        (zbhip_select_instances_db + zbhip_import_state_db).  Instances that a command still waiting in
        the log addresses by its own record (a follow-up written unprocessed before the restart) stay
        with the engine.  Returns the mask of the entries moved (the caller deletes them)."""
        waiting = set()
        if resume_position is not None:
            self.reader.seek(resume_position)
            while self.reader.has_next():
                rec = self.reader.next()
                if rec.record_type == abi.RT_COMMAND and not rec.processed and \
                        rec.value_type in (abi.VT_PROCESS_INSTANCE, abi.VT_PROCESS_INSTANCE_BATCH):
                    waiting.add(rec.value.get("processInstanceKey"))
        take, n = self.part.select_instances_db(entries, sorted(waiting))
        if n:
            first = self.next_free
            got = self.part.import_state_db([e for e, t in zip(entries, take) if t], first_slot=first)
            self.used_slots.update(range(first, first + got))
            self.next_free = first + got
        self.part.set_key_if_higher(self.key_generator.current_key())
        return take

    def process(self, record, out):
        if record.position is None:
            # a follow-up command the platform feeds back within the current batch
            if self.followups > 0:
                self.followups -= 1
                self.counts["followups_answered"] += 1
                return out.build()  # already processed on the device, its records are in the builder
            return self.engine.process(record, out)
        self._batch_done()
        self.followups = 0
        self.engine_batch = False
        if record.value_type == VT_JOB_BATCH and record.intent == JOB_BATCH_ACTIVATE:
            if record.value["type"] not in self.engine_job_types:
                return self._activate_jobs(record, out)
            if record.value["type"] in self.device_job_types:
                return self._activate_jobs_merged(record, out)
        if record.value_type == abi.VT_JOB and record.intent == abi.JOB_TIME_OUT and self._resolve(record.key) is not None:
            return self._time_out_job(record, out)
        if record.value_type == abi.VT_JOB and record.intent == abi.JOB_FAIL and self._resolve(record.key) is not None:
            return self._fail_job(record, out)
        i = self.window.index_of(record.position) if self.window.covers(record.position) else -1
        if i < 0:
            if not self._hot(record, 0):
                if self.correlation_keys > 0 and record.value_type == abi.VT_MESSAGE and \
                        record.intent == abi.MSG_PUBLISH:
                    # a publish the engine processes: its correlation key's message state goes there first
                    self._message_state_to_engine(record.value.get("correlationKey"))
                # a command the device does not run for an instance it holds (INCIDENT:RESOLVE of a
                # gateway's incident, PROCESS_INSTANCE:CANCEL, ...): the instance moves to the engine first
                held = self._held_instance(record)
                if held is not None:
                    self._hand_off(held)
                    self.key_generator.set_key_if_higher(self.part.current_key())
                self.engine_batch = True
                self.counts["engine_commands"] += 1
                return self.engine.process(record, out)
            self._fill_window(record)
            i = self.window.index_of(record.position)
        if i < 0:
            self.engine_batch = True
            return self.engine.process(record, out)
        self._window_done = i == self.window.size() - 1
        st, why = self.part.command_status(i)
        if st != 0:
            self.counts["fallbacks"] += 1
            self.fallback_reasons.append(why)
            return self._fall_back(i, record, out)
        self.counts["device_commands"] += 1
        self.counts["continuations"] += self.window.cmds[i]["kind"] == abi.CMD_CONTINUE
        self._emit(i, record, out)
        # DbKeyGenerator after this command: the device's keys so far (the engine's next command, a
        # fallback in this window or whatever follows the window, continues after them)
        self.key_generator.set_key_if_higher(self.part.key_before(i + 1))
        return out.build()

    def on_processing_error(self, error, record, out):
        return self.engine.on_processing_error(error, record, out)

    # ---- the window -----------------------------------------------------------------------------
    def _create_target(self, v):
        pdk = v.get("processDefinitionKey", -1)
        return self.by_key.get(pdk) if pdk is not None and pdk > 0 else self.latest_by_id.get(v.get("bpmnProcessId"))

    def _resolve(self, key):
        from .native import ZbhipError
        try:
            return self.part.resolve_key(key)
        except ZbhipError:
            return None

    @staticmethod
    def _match(key, vt, it, v):
        """What identifies a follow-up command written unprocessed when it comes back from the log."""
        return (key, vt, it, v.get("elementId"), v.get("flowScopeKey"), v.get("batchElementInstanceKey"),
                v.get("processInstanceKey"))

    def _continuation_match(self, record):
        return self._match(record.key, record.value_type, record.intent, record.value)

    def _hot(self, record, k):
        """Would the device take this log command?  k: continuations already claimed by the read-ahead."""
        if record.record_type != abi.RT_COMMAND:
            return False
        vt, it = record.value_type, record.intent
        if vt == abi.VT_PROCESS_INSTANCE_CREATION:
            return it == 0 and self._create_target(record.value) is not None
        if vt == abi.VT_JOB and it == abi.JOB_COMPLETE or vt == abi.VT_TIMER and it == abi.TIMER_TRIGGER:
            return self._resolve(record.key) is not None
        if (vt == abi.VT_PROCESS_INSTANCE and it in PI_COMMAND_INTENTS) or \
                (vt == abi.VT_PROCESS_INSTANCE_BATCH and it == abi.PIB_ACTIVATE):
            # a follow-up a device batch wrote unprocessed, read back in the order written
            return k < len(self.continuations) and self.continuations[k][2] == self._continuation_match(record)
        if self.correlation_keys > 0 and vt in MESSAGE_VALUE_TYPES:
            return self._message_command(record) is not None
        return False

    # ---- config 5: message commands <-> device commands ------------------------------------------
    def _message_command(self, record):
        """A message command of the log as (zbhip_command row, zbhip_xpart_cmd row or None), or None
        when the device does not take it: PUBLISH outside the subset (a time-to-live, a message id,
        variables, a name no device catch event waits for, a name of a message start event: the engine
        starts those instances), PROCESS_MESSAGE_SUBSCRIPTION commands of an
        instance the device does not hold, MESSAGE_SUBSCRIPTION commands of a local instance the
        device does not hold."""
        v, vt, it = record.value, record.value_type, record.intent
        if vt == abi.VT_MESSAGE:
            if it != abi.MSG_PUBLISH or v.get("timeToLive", 0) != 0 or v.get("messageId") or v.get("variables") \
                    or v.get("name") not in self.message_names or v.get("name") in self.start_message_names \
                    or not isinstance(v.get("correlationKey"), str) or v["correlationKey"] in self.engine_owned:
                return None
            corr = self.part.intern_string(v["correlationKey"])
            if corr >= self.correlation_keys:
                return None
            return {"instance": corr, "kind": abi.CMD_PUBLISH, "ref": self.part.intern(v["name"])}, None
        kind = XPART_KIND.get((vt, it))
        if kind is None or v.get("variables"):
            return None
        pik, eik = v["processInstanceKey"], v["elementInstanceKey"]
        # the message partition's commands of a correlation key the engine owns stay with the engine: a
        # CREATE by its key, a CORRELATE / DELETE (no key in the value) when the device holds no such
        # subscription
        if kind == abi.CMD_MSG_SUB_CREATE and v.get("correlationKey") in self.engine_owned:
            return None
        if kind in (abi.CMD_MSG_SUB_CORRELATE, abi.CMD_MSG_SUB_DELETE) and \
                (eik, v["messageName"]) not in self.subscriptions:
            return None
        x = abi.make_xparts(1)[0]
        x["element_instance_key"], x["process_instance_key"] = eik, pik
        x["message_key"] = v.get("messageKey", -1)
        x["message_name"] = self.part.intern(v["messageName"])
        x["bpmn_process_id"] = self.part.intern(v["bpmnProcessId"]) if v.get("bpmnProcessId") else 0xFFFF
        x["correlation_key"] = self.part.intern_string(v["correlationKey"]) if v.get("correlationKey") else abi.NO_STRING
        x["kind"] = kind
        x["interrupting"] = int(bool(v.get("interrupting", True)))
        x["target_partition"] = self.partition_id
        if vt == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION:
            # the PI partition's side: the subscribing element instance of a device instance (a closing
            # subscription's DELETE may arrive after its instance ended: the handle kept at CREATING)
            pi, el = self._resolve(pik), self._resolve(eik)
            if (pi is None or el is None) and kind == abi.CMD_PMS_DELETE:
                pi = el = self.pms_handles.get((eik, v["messageName"]))
            if pi is None or el is None or pi[0] != el[0]:
                return None
            x["instance"], x["element_ord"] = el
            x["source_partition"] = v["subscriptionPartitionId"]
            return {"instance": el[0], "kind": kind, "ref": 0}, x
        # the message partition's side: the routing handle of the subscribing element instance --
        # its slot and key ordinal when the instance lives here (a local correlation enters it in the
        # same batch), else an id derived from the element instance key, unique per subscription like
        # the reference's [elementInstanceKey, messageName] (the PI partition resolves the keys itself)
        src = partition_of_key(pik)
        if src == self.partition_id:
            el = self._resolve(eik)
            if el is None:
                return None
            x["instance"], x["element_ord"] = el
        else:
            n = eik - (partition_of_key(eik) << KEY_BITS)
            x["instance"], x["element_ord"] = n & 0xFFFFFFFF, (n >> 32) & 0xFFFF
        x["source_partition"] = src
        if kind in (abi.CMD_MSG_SUB_CORRELATE, abi.CMD_MSG_SUB_DELETE):
            # no correlation key in the value: the slot of the subscription it names
            x["correlation_key"] = self.subscriptions[(eik, v["messageName"])]
        if int(x["correlation_key"]) >= self.correlation_keys:
            return None
        return {"instance": int(x["correlation_key"]), "kind": kind, "ref": 0}, x

    def _send(self, i, out):
        """Window command i's cross-partition commands, sent once its batch is committed
        (SubscriptionCommandSender.handleFollowUpCommandBasedOnPartition :320-338: a side effect)."""
        sends = self.part.outbox_command(i)
        if not len(sends):
            return
        if self.command_sender is None:
            raise RuntimeError("a device batch sent cross-partition commands but no InterPartitionCommandSender is set")
        cmds = [(int(x["target_partition"]),) + XPART_COMMAND[int(x["kind"])] +
                (xpart_value(x, self.part.name, self.part.string_value),) for x in sends]

        def task():
            for target, vt, it, value in cmds:
                self.command_sender.send_command(target, vt, it, value)
            return True
        out.append_post_commit_task(task)

    def _fill_window(self, first):
        """Reads consecutive hot-path commands from the log starting at `first` (GpuBatchProcessor
        .fillWindow) and submits and runs them once."""
        self._free_ended()
        self.window.reset(self.doc_total)
        self.reader.seek(first.position)
        claimed = 0
        while self.reader.has_next() and self.window.size() < self.window_size:
            rec = self.reader.next()
            if rec.record_type != abi.RT_COMMAND or rec.processed:
                continue  # events and processed follow-ups of earlier batches between the commands
            if not self._hot(rec, claimed):
                break  # the engine's: the window ends before it (log order is kept)
            if self._push_fenced(rec, claimed):
                break  # the next window takes it (see _push_fenced)
            vt = rec.value_type
            if vt == abi.VT_PROCESS_INSTANCE_CREATION:
                v = rec.value
                docs = doc_entries(v.get("variables", ()), self.part.intern, self.part.intern_string, self.part.intern_list)
                if docs is None:
                    break  # a document outside the subset: the engine takes this CREATE
                slot = self._take_slot()
                if slot is None:
                    break
                self.window.put(rec, slot, abi.CMD_CREATE, self._create_target(v).idx, docs,
                                [val for _, val in v.get("variables", ())])
            elif vt == abi.VT_JOB:
                docs = doc_entries(rec.value.get("variables", ()), self.part.intern, self.part.intern_string,
                                   self.part.intern_list)
                if docs is None:
                    break
                inst, ordv = self._resolve(rec.key)
                self.window.put(rec, inst, abi.CMD_JOB_COMPLETE, ordv, docs,
                                [val for _, val in rec.value.get("variables", ())])
            elif vt == abi.VT_TIMER:
                inst, ordv = self._resolve(rec.key)
                due = rec.value["dueDate"]
                self.window.put(rec, inst, abi.CMD_TIMER_TRIGGER, ordv, doc_begin=due & 0xFFFFFFFF, pad=due >> 32)
            elif vt in MESSAGE_VALUE_TYPES:
                c, x = self._message_command(rec)
                if x is not None:
                    c["doc_begin"] = len(self.window.xparts)
                    self.window.xparts.append(x)
                    if c["kind"] == abi.CMD_MSG_SUB_CREATE:
                        # a DELETE read into the same window finds the slot (its CREATED is emitted later)
                        self.subscriptions.setdefault((rec.value["elementInstanceKey"], rec.value["messageName"]),
                                                      c["instance"])
                self.window.put(rec, c["instance"], c["kind"], c["ref"], doc_begin=c.get("doc_begin", 0))
            else:
                cid, slot, _ = self.continuations[claimed]
                claimed += 1
                self.window.put(rec, slot, abi.CMD_CONTINUE, 0, doc_begin=cid & 0xFFFFFFFF, pad=cid >> 32)
            if self.engine_owned and self.window.cmds[-1]["kind"] not in abi.SLOT_KINDS:
                # a correlation key of this partition is the engine's: a process-instance command may subscribe
                # to it locally and fall back with engine keys, which a message window takes only after its
                # last device key (zbhip_set_external_keys) -- such a command ends its window
                break
        del self.continuations[:claimed]
        # keys the engine generated since the last window come first (setKeyIfHigher)
        self.part.set_key_if_higher(self.key_generator.current_key())
        # the window's clock: TIMER:CREATED dueDates (CatchEventBehavior.java:310, ActorClock)
        self.part.set_clock(self.clock())
        cmds, docs = self.window.arrays()
        self.counts["windows"] += 1
        xparts = None
        if self.window.xparts:
            xparts = abi.make_xparts(len(self.window.xparts))
            for j, x in enumerate(self.window.xparts):
                xparts[j] = x
        self.part.submit(cmds, docs, xparts)
        self.doc_total += len(docs)
        self._window_done = False
        self.part.run()
        # the records are drained command by command as the platform reaches them
        # (zbhip_drain_command): a fallback command's CPU-engine keys come before the later ones

    def _push_fenced(self, rec, claimed):
        """A job stream's push gathers the job's variables when the push record is emitted
        (zbhip_job_variables), after the whole window ran; the reference gathers them in publishWork, at
        JOB:CREATED (BpmnJobActivationBehavior.java:83).  While a stream pushes, a window therefore holds
        at most one command per process instance: no later command of the window changes the variables a
        push reads, or ends its job.  (CREATEs take fresh slots; message-partition commands address
        correlation slots, not instances.)"""
        if not self.stream_sinks:
            return False
        vt = rec.value_type
        if vt in (abi.VT_JOB, abi.VT_TIMER):
            inst = self._resolve(rec.key)[0]
        elif vt in (abi.VT_PROCESS_INSTANCE, abi.VT_PROCESS_INSTANCE_BATCH):
            inst = self.continuations[claimed][1]
        elif vt == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION:
            inst = self._message_command(rec)[0]["instance"]
        else:
            return False
        return inst in self.window.instances

    def _free_ended(self):
        for s in list(self.ended):
            if self.part.pending_continuations(s) == 0 and s not in self.closing:
                self.ended.discard(s)
                self.used_slots.discard(s)

    def _take_slot(self):
        for _ in range(self.instances):
            s = self.next_free % self.instances
            self.next_free = s + 1
            if s not in self.used_slots and s not in self.window.instances:
                self.used_slots.add(s)
                return s
        return None

    def _emit(self, i, record, out):
        """Window command i's records into the builder as the reference's processors write them
        (Window.emit).  A rejection of the command itself carries the command's value
        (TypedRejectionWriter.appendRejection)."""
        cmd_doc = tuple(record.value.get("variables", ())) if isinstance(record.value, dict) else ()
        win = self.window
        admitted = 0
        pushes = []
        created = {}  # jobs created in the batch -> type (publishWork: pushed, or notified)
        for r in self.part.drain_command(i):
            rt, vt, it = int(r["record_type"]), int(r["value_type"]), int(r["intent"])
            if rt == abi.RT_REJECTION and int(r["ordinal"]) == 0 and vt == record.value_type and it == record.intent:
                value = dict(record.value)
            else:
                value = self.values.value(r, cmd_doc, lambda aux: win.doc_values[aux - win.doc_base],
                                          getattr(record, "timestamp", 0))
            reason = self.part.reason(r) if rt == abi.RT_REJECTION else ""
            out.append_record(int(r["key"]), rt, vt, it, int(r["rejection_type"]), reason, value)
            if vt == VT_JOB_BATCH and rt == abi.RT_EVENT:
                pushes.append((int(r["aux"]), value))
                created.pop(int(r["aux"]), None)
            elif vt == abi.VT_JOB and rt == abi.RT_EVENT and it == abi.JOB_CREATED:
                created[int(r["key"])] = value["type"]
            if self.correlation_keys > 0:
                self._track_pending(rt, vt, it, value)
            if rt == abi.RT_EVENT and vt == abi.VT_TIMER and it == abi.TIMER_CREATED and self.due_date_checker:
                due = value["dueDate"]
                # CatchEventBehavior.subscribeToTimerEvent's side effect: timerChecker.scheduleTimer(dueDate)
                out.append_post_commit_task(lambda d=due: self.due_date_checker.schedule_timer(d) or True)
            if rt == abi.RT_COMMAND:
                if r["unprocessed"]:
                    # a continuation (its id in aux): expected back from the log in the order written
                    self.continuations.append((int(r["aux"]), win.instances[i], self._match(int(r["key"]), vt, it, value)))
                else:
                    admitted += 1
            elif vt == abi.VT_PROCESS_INSTANCE and it == 5 and value.get("bpmnElementType") == "PROCESS":
                self.ended.add(win.instances[i])  # its slot is free once its continuations ran
            elif vt == abi.VT_MESSAGE_SUBSCRIPTION and rt == abi.RT_EVENT:
                sub = (value["elementInstanceKey"], value["messageName"])
                if it == abi.MS_CREATED:
                    self.subscriptions[sub] = int(r["correlation_key"])
                elif it == abi.MS_DELETED or (it == abi.MS_CORRELATED and value.get("interrupting", True)):
                    # (a non-interrupting subscription stays open after its correlation)
                    self.subscriptions.pop(sub, None)
            elif vt == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION and rt == abi.RT_EVENT:
                # a closing subscription keeps its instance slot until PROCESS_MESSAGE_SUBSCRIPTION:DELETED
                # (the device row outlives the instance: a CREATE into the slot would fall back)
                sub = (value["elementInstanceKey"], value["messageName"])
                if it == abi.PMS_CREATING:
                    self.pms_handles[sub] = self._resolve(value["elementInstanceKey"])
                elif it == abi.PMS_DELETING:
                    self.closing.add(win.instances[i])
                elif it == abi.PMS_DELETED or (it == abi.PMS_CORRELATED and value.get("interrupting", True)):
                    # (a non-interrupting subscription stays open after its correlation)
                    self.pms_handles.pop(sub, None)
                    if it == abi.PMS_DELETED:
                        self.closing.discard(win.instances[i])
        self.followups = admitted
        if pushes:
            self._push(out, pushes)
        self._notify(out, created.values())
        if self.correlation_keys > 0:
            self._send(i, out)

    # ---- the engine's scheduled tasks over device-held state -------------------
    def scheduled_ready(self):
        """The device state equals the log's: every command of the current window was emitted (the
        platform runs scheduled tasks between batches; mid-window the device is ahead of the log, so a
        check waits for the window's end -- a later run of the checker, which the reference's actor
        scheduling allows)."""
        return self._window_done

    def due_timers(self, now):
        """TimerInstanceState.processTimersWithDueDateBefore over the device: [(timer key, TimerRecord)]
        in TIMER_DUE_DATES order (at most `scheduled_cap`), and the first dueDate not returned (-1 none)."""
        rows, nxt = self.part.due_timers(now, cap=self.scheduled_cap)
        return [(int(r["key"]), self.values.value(r)) for r in rows], nxt

    def timed_out_jobs(self, now, with_next=False):
        """JobState.forEachTimedOutEntry over the device's activated jobs: [(deadline, job key, JobRecord)] in
        JOB_DEADLINES order (at most `scheduled_cap`; with_next: and the deadline of the first one left out)."""
        rows, nxt = self.part.timed_out_jobs(now, cap=self.scheduled_cap, with_next=True)
        out = [(int(r["message_key"]), int(r["key"]), self.values.value(r)) for r in rows]
        return (out, nxt) if with_next else out

    def _track_pending(self, rt, vt, it, value):
        """The transient pending-subscription states the appliers of the device's records keep in the
        reference (DbProcessMessageSubscriptionState.java:82-124,180-222, DbMessageSubscriptionState.java
        :157-222, TransientPendingSubscriptionState): the PI side's OPENING / CLOSING subscriptions and the
        message side's CORRELATING ones, with the time they were last sent."""
        if rt != abi.RT_EVENT:
            return
        now = self.clock()
        if vt == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION:
            sub = (value["elementInstanceKey"], value["messageName"])
            if it == abi.PMS_CREATING:  # put: OPENING
                self.pending_pms[sub] = [now, dict(value), True]
            elif it == abi.PMS_DELETING:
                self.pending_pms[sub] = [now, dict(value), False]  # updateToClosingState
            elif it in (abi.PMS_CREATED, abi.PMS_DELETED, abi.PMS_CORRELATED):
                self.pending_pms.pop(sub, None)
        elif vt == abi.VT_MESSAGE_SUBSCRIPTION:
            sub = (value["elementInstanceKey"], value["messageName"])
            if it == abi.MS_CORRELATING:  # updateToCorrelatingState
                self.pending_ms[sub] = [now, dict(value)]
            elif it in (abi.MS_CORRELATED, abi.MS_DELETED):
                self.pending_ms.pop(sub, None)

    def pending_process_message_subscriptions(self, deadline):
        """PendingProcessMessageSubscriptionState.visitPending: the device's OPENING / CLOSING
        subscriptions last sent before `deadline`, ordered by that time: [(time, sub, record, opening)]."""
        due = sorted(((t, sub) for sub, (t, _, _) in self.pending_pms.items() if t < deadline), key=lambda x: x[0])
        return [(t, sub, self.pending_pms[sub][1], self.pending_pms[sub][2]) for t, sub in due]

    def pending_message_subscriptions(self, deadline):
        """PendingMessageSubscriptionState.visitPending: the CORRELATING subscriptions of the device's
        correlation slots last sent before `deadline`: [(time, sub, record)]."""
        due = sorted(((t, sub) for sub, (t, _) in self.pending_ms.items() if t < deadline), key=lambda x: x[0])
        return [(t, sub, self.pending_ms[sub][1]) for t, sub in due]

    def on_sent_pms(self, sub, when):
        if sub in self.pending_pms:
            self.pending_pms[sub][0] = when

    def on_sent_ms(self, sub, when):
        if sub in self.pending_ms:
            self.pending_ms[sub][0] = when

    # ---- keys ------------------------------------------------------------------------------------
    def _batch_done(self):
        """The previous batch ended: the keys a fallback command's engine batch generated are declared
        (zbhip_set_external_keys) before the window's later commands fix theirs."""
        if self.pending_declaration is not None:
            i, before = self.pending_declaration
            self.pending_declaration = None
            self.part.set_external_keys(i, self.key_generator.current_key() - before)

    # ---- fallback hand-off (Engine.java:134, ProcessingStateMachine.java:276-310) ----
    def _held_instance(self, record):
        """the device instance slot a non-hot-path command addresses by its key or its value's
        processInstanceKey, or None"""
        for k in (record.key, (record.value or {}).get("processInstanceKey", -1)):
            if k is not None and k >= 0:
                ref = self._resolve(k)
                if ref is not None:
                    return ref[0]
        return None

    def _message_state_to_engine(self, correlation_key):
        """One owner per correlation key (include/zbhip.h).  The reference correlates a
        publish to every open subscription of [name, correlationKey] (MessagePublishProcessor.java:127-185)
        and buffers a message with a time-to-live for later subscriptions (MessageCorrelator.java:41-96);
        the device holds subscriptions only.  Before the engine processes a publish of a key, the key's
        subscriptions move from its correlation slot into the engine's state (zb-db rows through the
        platform's transaction, then evicted) with their pending CORRELATING entries, and every later
        message command of the key goes to the engine."""
        if not isinstance(correlation_key, str) or correlation_key in self.engine_owned:
            return
        self.engine_owned.add(correlation_key)
        slot = self.part.intern_string(correlation_key)
        if slot >= self.correlation_keys:
            return  # (never a device slot)
        rows = self.part.export_correlation_slots([slot])
        if rows:
            self.zeebe_db.upsert(rows, self.part.string_value)
        self.part.evict_correlation_slots([slot])  # (and the device declines the key's commands from now on)
        for sub in [k for k, s in self.subscriptions.items() if s == slot]:
            del self.subscriptions[sub]
            if sub in self.pending_ms:
                if self.engine_pending is not None:  # the engine's transient state now (its appliers clear it)
                    self.engine_pending.add_ms(sub, *self.pending_ms.pop(sub))
                else:
                    self.moved_pending_ms.append((sub, self.pending_ms.pop(sub)))
        # subscribers on this partition: the engine's correlations reach them as follow-ups of its own
        # batches (SubscriptionCommandSender: the own partition is a follow-up command), so their instances
        # go with the key (a later local subscription to the key falls back and goes the same way)
        if self._window_done:
            for r in rows:
                if r.startswith("MESSAGE_SUBSCRIPTION_BY_KEY|"):
                    pik = int(r.split("processInstanceKey=", 1)[1].split(",", 1)[0])
                    held = self._resolve(pik) if partition_of_key(pik) == self.partition_id else None
                    if held is not None:
                        self._hand_off(held[0])
                        self.key_generator.set_key_if_higher(self.part.current_key())
        self.counts["keys_to_engine"] += 1

    def _fall_back(self, i, record, out):
        inst = self.window.instances[i]
        if self.window.cmds[i]["kind"] in abi.SLOT_KINDS:
            # a message-partition command the device declined: its correlation key's state moves to the engine
            self._message_state_to_engine(self.part.string_value(inst))
        else:
            self._hand_off(inst)
        before = self.part.key_before(i)
        self.key_generator.set_key_if_higher(before)
        self.engine_batch = True
        self.pending_declaration = (i, before)
        # the engine's keys are declared when its batch (follow-ups included) is done
        out.append_post_commit_task(self._batch_done)
        return self.engine.process(record, out)

    def _hand_off(self, inst):
        if inst not in self.handed_off:
            # the instance's zb-db rows into the engine's state (the platform's transaction), then off
            # the device with its waiting continuations (the engine reads them back from the log)
            self.handed_off.add(inst)
            rows = self.part.export_instances([inst])
            # its jobs are the engine's now: activations of their types go there too
            self.engine_job_types.update(r.split("|")[2].split(",")[0][len("type="):] for r in rows
                                         if r.startswith("JOBS|"))
            self.zeebe_db.upsert(rows, self.part.string_value)
            self.part.evict_instances([inst])
            self.continuations = [c for c in self.continuations if c[1] != inst]
            self.used_slots.discard(inst)
            self.ended.discard(inst)
            # its subscriptions are the engine's now: no closing row holds the slot, no routing handle
            # points into it, and their pending entries move to the engine's transient state
            self.closing.discard(inst)
            for sub in [k for k, v in self.pms_handles.items() if v is not None and v[0] == inst]:
                del self.pms_handles[sub]
                if sub in self.pending_pms:
                    if self.engine_pending is not None:
                        self.engine_pending.add_pms(sub, *self.pending_pms.pop(sub))
                    else:
                        self.moved_pending.append((sub, self.pending_pms.pop(sub)))

    # ---- JOB:FAIL of a device job (JobFailProcessor.java:79-162) -------------------------------------
    def _fail_job(self, record, out):
        v = record.value
        self.part.set_key_if_higher(self.key_generator.current_key())
        recs = self.part.fail_job(record.key, v.get("retries", 0), v.get("errorMessage", ""), v.get("retryBackoff", 0),
                                  len(v.get("variables", ())), timestamp=self.clock())
        if recs is None:  # outside the device subset (variables, a back-off): the engine's, with the instance
            self._hand_off(self._resolve(record.key)[0])
            self.key_generator.set_key_if_higher(self.part.current_key())
            self.engine_batch = True
            return self.engine.process(record, out)
        self.counts["job_failures"] += 1
        incident = False
        for r in recs:
            rt, vt, it = int(r["record_type"]), int(r["value_type"]), int(r["intent"])
            if rt == abi.RT_REJECTION:
                out.append_record(record.key, rt, vt, it, int(r["rejection_type"]), self.part.reason(r), dict(v))
                continue
            value = self.values.value(r)
            out.append_record(int(r["key"]), rt, vt, it, abi.REJ_NONE, "", value)
            incident |= vt == abi.VT_INCIDENT
            if vt == VT_JOB_BATCH:
                self._push(out, [(int(r["aux"]), value)])
            elif vt == abi.VT_JOB and it == abi.JOB_FAILED and value["retries"] > 0 and len(recs) == 1:
                self._notify(out, [value["type"]])  # retryImmediately -> publishWork, no stream
        self.key_generator.set_key_if_higher(self.part.current_key())
        if incident:
            # the instance waits for the incident's resolution (JOB:UPDATE_RETRIES, INCIDENT:RESOLVE): the
            # engine's, with the job's FAILED state and the incident rows
            self._hand_off(self._resolve(record.key)[0])
        return out.build()

    # ---- JOB:TIME_OUT of a device job (JobTimeOutProcessor.java:46-73) ------------------------------
    def _time_out_job(self, record, out):
        self.counts["time_outs"] += 1
        self.part.set_key_if_higher(self.key_generator.current_key())
        recs = self.part.time_out_job(record.key, self.clock())
        r = recs[0]
        if int(r["record_type"]) == abi.RT_REJECTION:
            out.append_record(record.key, abi.RT_REJECTION, abi.VT_JOB, abi.JOB_TIME_OUT, int(r["rejection_type"]),
                              self.part.reason(r), dict(record.value))
            return out.build()
        value = self.values.value(r)
        out.append_record(record.key, abi.RT_EVENT, abi.VT_JOB, abi.JOB_TIMED_OUT, abi.REJ_NONE, "", value)
        # publishWork: a job stream of the type -> the push (JOB_BATCH:ACTIVATED); none -> a notification
        if len(recs) == 1:
            self._notify(out, [value["type"]])
        for p in recs[1:]:
            value = self.values.value(p)
            out.append_record(int(p["key"]), abi.RT_EVENT, VT_JOB_BATCH, JOB_BATCH_ACTIVATED, abi.REJ_NONE, "", value)
            self._push(out, [(int(p["aux"]), value)])
        self.key_generator.set_key_if_higher(self.part.current_key())
        return out.build()

    def set_job_stream(self, job_type, worker, timeout, on=True, fetch_variables=(), push=None):
        """A job stream opened / closed for `job_type` (JobStreamer: the gateway's StreamActivatedJobs): jobs
        the device creates of that type are pushed from the next window on -- JOB_BATCH:ACTIVATED in the log,
        and after the commit push(jobKey, job) with the job's `fetch_variables` (all when empty)."""
        self.part.set_job_stream(job_type, worker, timeout, on)
        if on:
            self.values.streams[job_type] = (worker, timeout)
            if push is not None:
                self.stream_sinks[job_type] = (tuple(fetch_variables), push)
        else:
            self.values.streams.pop(job_type, None)
            self.stream_sinks.pop(job_type, None)

    def _notify(self, out, types):
        """publishWork without a stream: notifyJobAvailable's side effect (BpmnJobActivationBehavior.java
        :97-111), JobStreamer.notifyWorkAvailable(type) after the commit -- long-polling workers wake up."""
        types = list(types)
        if types and self.job_streamer is not None:
            out.append_post_commit_task(lambda: [self.job_streamer.notify_work_available(t) for t in types] and True)

    def _push(self, out, pushes):
        push_side_effects(out, pushes, self.stream_sinks, self.part.job_variables, self.values, self.part.name,
                          self.part.string_value)

    # ---- job activation (JobBatchActivateProcessor.java:60-143) ------------------------------------
    def _activate_jobs_merged(self, record, out):
        """JOB_BATCH:ACTIVATE of a job type both the engine and the device hold jobs of (handed-off instances,
        engine-only processes of a device type): JobBatchCollector.collectJobs (:67-123) walks
        JOB_ACTIVATABLE [type, jobKey] in key order over both.  The first maxJobsToActivate keys of the two
        lists (the engine's JobState.forEachActivatableJobs, zbhip_activatable_jobs) split into each side's
        share; the engine activates its share first (its nextKey is the batch key), the device its own with
        the same key (its key counter is one behind), and the one JOB_BATCH:ACTIVATED record lists both in
        key order."""
        v = record.value
        mx = v["maxJobsToActivate"]
        if mx < 1 or v["timeout"] < 1 or not v["type"]:
            return self.engine.process(record, out)  # the rejection
        self.part.set_key_if_higher(self.key_generator.current_key())
        dev = self.part.activatable_jobs(v["type"], mx)
        if not dev:
            return self.engine.process(record, out)
        eng = self.engine.activatable_jobs(v["type"])
        picked = sorted(dev + eng[:mx])[:mx]
        ndev = len(set(picked) & set(dev))
        if ndev == len(picked):
            return self._activate_jobs(record, out)
        self.counts["activations"] += 1
        share = _Scratch()
        cmd = copy.copy(record)
        cmd.value = dict(v, maxJobsToActivate=len(picked) - ndev)
        self.engine.process(cmd, share)
        ev = share.entries[-1]
        key, jobs, _ = self.part.activate_jobs(v["type"], v["worker"], v["timeout"], ndev, v.get("timestamp", 0))
        if key != ev.key:
            raise RuntimeError("merged activation: batch keys %d / %d" % (ev.key, key))
        value = dict(ev.value)
        mine = self.values.job_batch(v, key, jobs, self.part.name, self.part.string_value)
        both = sorted(zip(value["jobKeys"] + mine["jobKeys"], value["jobs"] + mine["jobs"]), key=lambda t: t[0])
        value["jobKeys"] = tuple(k for k, _ in both) if isinstance(value["jobKeys"], tuple) else [k for k, _ in both]
        value["jobs"] = tuple(j for _, j in both) if isinstance(value["jobs"], tuple) else [j for _, j in both]
        value["maxJobsToActivate"] = mx
        value["truncated"] = bool(value.get("truncated")) or bool(mine.get("truncated"))
        self.key_generator.set_key_if_higher(key)
        out.append_record(key, abi.RT_EVENT, VT_JOB_BATCH, JOB_BATCH_ACTIVATED, abi.REJ_NONE, "", value)
        for task in share.post_commit:
            out.append_post_commit_task(task)
        return out.build()

    def _activate_jobs(self, record, out):
        v = record.value
        self.part.set_key_if_higher(self.key_generator.current_key())
        self.counts["activations"] += 1
        key, jobs, reason = self.part.activate_jobs(v["type"], v["worker"], v["timeout"], v["maxJobsToActivate"],
                                                    v.get("timestamp", 0))
        if key < 0:
            out.append_record(record.key, abi.RT_REJECTION, VT_JOB_BATCH, JOB_BATCH_ACTIVATE,
                              abi.REJ_INVALID_ARGUMENT, "reason %d" % reason, dict(v))
            return out.build()
        self.key_generator.set_key_if_higher(key)
        out.append_record(key, abi.RT_EVENT, VT_JOB_BATCH, JOB_BATCH_ACTIVATED, abi.REJ_NONE, "",
                          self.values.job_batch(v, key, jobs, self.part.name, self.part.string_value))
        return out.build()
