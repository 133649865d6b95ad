// Log serialiser of libzbhip.so: drained records -> the bytes the reference's log stream holds
// for them.  Host code, no device work: it turns the compact records of a
// window into sequenced batches of log entries -- dispatcher framing, the LogEntryDescriptor
// header, the SBE RecordMetadata and the msgpack record value -- exactly as
//   SequencedBatchSerializer.java:33-67, LogAppendEntrySerializer.java:40-111,
//   LogEntryDescriptor.java (static block), DataFrameDescriptor.java,
//   RecordMetadata.java write/reset + protocol.xml:137-152 (schema version 4, protocol/pom.xml:28),
//   ObjectValue.java:78-84 + MsgPackWriter.java:62-316
// write them.  Record values follow the engine's writers: ProcessInstanceRecord.java:62-74 with
// BpmnStateTransitionBehavior.java:243-339 / CreateProcessInstanceProcessor.java:319-330,
// JobRecord.java:39-83 with BpmnJobBehavior.java:194-218 and JobCompleteProcessor.java:75-92,
// VariableRecord.java:25-41, ProcessEventRecord.java:25-42 with EventTriggerBehavior.java:148-166,
// ProcessInstanceCreationRecord.java:32-55 with CreateProcessInstanceProcessor.java:129-158, and a
// rejection carries its command's value (ResultBuilderBackedRejectionWriter.java:25-38).
//
// Deploy time compiles, per element, the constant msgpack runs of its records (everything but
// the keys), so a record costs a few memcpys and the variable-length key integers.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/zbhip.h"

namespace {

using Bytes = std::string;

// ---- MsgPackWriter (MsgPackWriter.java:62-316) ------------------------------------------------
void be16(Bytes& b, uint16_t v) { b.push_back((char)(v >> 8)); b.push_back((char)v); }
void be32(Bytes& b, uint32_t v) { be16(b, (uint16_t)(v >> 16)); be16(b, (uint16_t)v); }
void be64(Bytes& b, uint64_t v) { be32(b, (uint32_t)(v >> 32)); be32(b, (uint32_t)v); }

void mp_map(Bytes& b, uint32_t n) {
  if (n < 16) b.push_back((char)(0x80 | n));
  else if (n < 65536) { b.push_back((char)0xde); be16(b, (uint16_t)n); }
  else { b.push_back((char)0xdf); be32(b, n); }
}
void mp_array(Bytes& b, uint32_t n) {
  if (n < 16) b.push_back((char)(0x90 | n));
  else if (n < 65536) { b.push_back((char)0xdc); be16(b, (uint16_t)n); }
  else { b.push_back((char)0xdd); be32(b, n); }
}
void mp_int(Bytes& b, int64_t v) {
  if (v < -(1LL << 5)) {
    if (v < -(1LL << 15)) {
      if (v < -(1LL << 31)) { b.push_back((char)0xd3); be64(b, (uint64_t)v); }
      else { b.push_back((char)0xd2); be32(b, (uint32_t)v); }
    } else if (v < -(1LL << 7)) { b.push_back((char)0xd1); be16(b, (uint16_t)v); }
    else { b.push_back((char)0xd0); b.push_back((char)v); }
  } else if (v < (1LL << 7)) {
    b.push_back((char)v);
  } else if (v < (1LL << 16)) {
    if (v < (1LL << 8)) { b.push_back((char)0xcc); b.push_back((char)v); }
    else { b.push_back((char)0xcd); be16(b, (uint16_t)v); }
  } else if (v < (1LL << 32)) { b.push_back((char)0xce); be32(b, (uint32_t)v); }
  else { b.push_back((char)0xcf); be64(b, (uint64_t)v); }
}
void mp_str(Bytes& b, const char* s, size_t n) {
  if (n < 32) b.push_back((char)(0xa0 | n));
  else if (n < 256) { b.push_back((char)0xd9); b.push_back((char)n); }
  else if (n < 65536) { b.push_back((char)0xda); be16(b, (uint16_t)n); }
  else { b.push_back((char)0xdb); be32(b, (uint32_t)n); }
  b.append(s, n);
}
void mp_str(Bytes& b, const std::string& s) { mp_str(b, s.data(), s.size()); }
void mp_bin(Bytes& b, const Bytes& v) {
  const size_t n = v.size();
  if (n < 256) { b.push_back((char)0xc4); b.push_back((char)n); }
  else if (n < 65536) { b.push_back((char)0xc5); be16(b, (uint16_t)n); }
  else { b.push_back((char)0xc6); be32(b, (uint32_t)n); }
  b.append(v);
}
void key(Bytes& b, const char* k) { mp_str(b, k, strlen(k)); }

const char* element_type_name(uint32_t t) {
  static const char* n[] = {"UNSPECIFIED", "PROCESS", "SUB_PROCESS", "EVENT_SUB_PROCESS", "START_EVENT",
                            "INTERMEDIATE_CATCH_EVENT", "INTERMEDIATE_THROW_EVENT", "BOUNDARY_EVENT", "END_EVENT",
                            "SERVICE_TASK", "RECEIVE_TASK", "USER_TASK", "MANUAL_TASK", "TASK", "EXCLUSIVE_GATEWAY",
                            "PARALLEL_GATEWAY", "EVENT_BASED_GATEWAY", "INCLUSIVE_GATEWAY", "SEQUENCE_FLOW",
                            "MULTI_INSTANCE_BODY", "CALL_ACTIVITY", "BUSINESS_RULE_TASK", "SCRIPT_TASK", "SEND_TASK"};
  return t < sizeof(n) / sizeof(n[0]) ? n[t] : "UNSPECIFIED";
}
const char* event_type_name(uint32_t t) {
  static const char* n[] = {"UNSPECIFIED", "CONDITIONAL", "ERROR", "ESCALATION", "LINK", "MESSAGE", "NONE",
                            "SIGNAL", "TERMINATE", "TIMER"};
  return t < sizeof(n) / sizeof(n[0]) ? n[t] : "UNSPECIFIED";
}
const char* state_text(int s) {
  switch (s) {
    case ZBHIP_PI_ELEMENT_ACTIVATING: return "ELEMENT_ACTIVATING";
    case ZBHIP_PI_ELEMENT_ACTIVATED: return "ELEMENT_ACTIVATED";
    case ZBHIP_PI_ELEMENT_COMPLETING: return "ELEMENT_COMPLETING";
    case ZBHIP_PI_ELEMENT_COMPLETED: return "ELEMENT_COMPLETED";
    case ZBHIP_PI_ELEMENT_TERMINATING: return "ELEMENT_TERMINATING";
    case ZBHIP_PI_ELEMENT_TERMINATED: return "ELEMENT_TERMINATED";
    default: return "?";
  }
}

const char* kTenant = "<default>";  // TenantOwned.DEFAULT_TENANT_IDENTIFIER
const Bytes kEmptyDoc("\x80", 1);   // MsgPackHelper.EMTPY_OBJECT (DocumentValue.EMPTY_DOCUMENT, JobRecord.NO_HEADERS)

// deploy-time constant runs of one element's records
struct SerElement {
  uint8_t type = 0, event = 0;
  std::string id;
  uint32_t duration_ms = 0;  // timer catch / boundary event (the device log path's TIMER dueDates)
  uint32_t interrupting_cycle = 0;  // an interrupting boundary event's timeCycle (its next timer, E_DUR .y)
  std::string cond_text;     // sequence flow: its condition's FEEL text (incident messages)
  // ProcessInstanceRecord: [map, bpmnElementType .. processDefinitionKey, "processInstanceKey"] key
  // ["flowScopeKey"] key [bpmnEventType .. tenantId]
  Bytes pi_head, pi_tail;
  // JobRecord of a service task: [map .. customHeaders, "variables"] bin(doc) [errorMessage ..
  // processDefinitionKey, "processInstanceKey"] key ["elementId" .. "elementInstanceKey"] key [tenantId]
  Bytes job_head, job_mid, job_tail;
  size_t job_rest = 0;  // job_head after its deadline and worker entries
  Bytes headers;        // customHeaders: the task headers' msgpack map (zbhip_process_csr.header_bytes)
};
struct SerProcess {
  std::string bpmn_id;
  int32_t version = 1;
  int64_t def_key = 0;
  std::vector<SerElement> els;
};

}  // namespace

struct zbhip_serializer {
  std::vector<SerProcess> procs;
  std::vector<std::string> names;
  std::unordered_map<std::string, uint32_t> name_ids;
  std::vector<std::string> strs;
  std::unordered_map<std::string, uint32_t> str_ids;
  // the list dictionary (ZBHIP_DOC_LIST values), mirrored from the handle's (zbhip_intern_list)
  std::vector<std::vector<std::pair<uint8_t, int64_t>>> lists;
  int32_t broker[3] = {8, 4, 0};  // RecordMetadata.CURRENT_BROKER_VERSION of the reference build (8.4.0-SNAPSHOT)
  Bytes auth;                     // empty AuthInfo (format UNKNOWN, authData "")
};

extern "C" {

int zbhip_serializer_new(zbhip_serializer** out) {
  if (!out) return ZBHIP_EINVAL;
  auto* s = new zbhip_serializer();
  mp_map(s->auth, 2);  // AuthInfo.java: declareProperty(formatProp).declareProperty(authDataProp)
  key(s->auth, "format");
  key(s->auth, "UNKNOWN");
  key(s->auth, "authData");
  key(s->auth, "");
  *out = s;
  return ZBHIP_OK;
}

void zbhip_serializer_free(zbhip_serializer* s) { delete s; }

int zbhip_serializer_set_broker_version(zbhip_serializer* s, int32_t major, int32_t minor, int32_t patch) {
  if (!s) return ZBHIP_EINVAL;
  s->broker[0] = major;
  s->broker[1] = minor;
  s->broker[2] = patch;
  return ZBHIP_OK;
}

int zbhip_serializer_intern(zbhip_serializer* s, const char* name) {
  if (!s || !name) return ZBHIP_EINVAL;
  auto it = s->name_ids.find(name);
  if (it != s->name_ids.end()) return (int)it->second;
  const uint32_t id = (uint32_t)s->names.size();
  s->names.emplace_back(name);
  s->name_ids.emplace(name, id);
  return (int)id;
}

int64_t zbhip_serializer_intern_string(zbhip_serializer* s, const char* bytes, size_t len) {
  if (!s || (len && !bytes)) return ZBHIP_EINVAL;
  std::string v(bytes ? bytes : "", len);
  auto it = s->str_ids.find(v);
  if (it != s->str_ids.end()) return it->second;
  const uint32_t id = (uint32_t)s->strs.size();
  s->strs.push_back(v);
  s->str_ids.emplace(std::move(v), id);
  return id;
}

int64_t zbhip_serializer_intern_list(zbhip_serializer* s, const zbhip_doc_entry* items, size_t n) {
  if (!s || (n && !items)) return ZBHIP_EINVAL;
  std::vector<std::pair<uint8_t, int64_t>> v;
  for (size_t i = 0; i < n; ++i) v.push_back({items[i].type, items[i].value});
  s->lists.push_back(std::move(v));
  return (int64_t)s->lists.size() - 1;
}

int zbhip_serializer_deploy(zbhip_serializer* s, const zbhip_process_csr* csr, uint32_t* idx_out) {
  if (!s || !csr || csr->n_elements == 0) return ZBHIP_EINVAL;
  SerProcess P;
  auto str = [&](uint16_t i) -> std::string { return i < csr->n_strings ? csr->strings[i] : ""; };
  P.bpmn_id = str(csr->bpmn_process_id);
  P.version = csr->version;
  P.def_key = csr->process_definition_key;
  P.els.resize(csr->n_elements);
  for (uint32_t e = 0; e < csr->n_elements; ++e) {
    const zbhip_element& E = csr->elements[e];
    SerElement& S = P.els[e];
    S.type = E.element_type;
    S.event = E.element_type == ZBHIP_EL_PROCESS ? ZBHIP_EV_UNSPECIFIED : E.event_type;
    S.id = str(E.id);
    S.duration_ms = E.duration_ms;
    S.interrupting_cycle = E.element_type == ZBHIP_EL_BOUNDARY_EVENT && E.event_type == ZBHIP_EV_TIMER &&
                           (E.job_retries & 1) && (E.job_retries >> 8) != 1;
    if (E.element_type == ZBHIP_EL_SEQUENCE_FLOW && E.condition != ZBHIP_NONE16 && csr->cond_text &&
        E.condition < csr->n_conditions && csr->cond_text[E.condition])
      S.cond_text = csr->cond_text[E.condition];
    // ProcessInstanceRecord (declaration order ProcessInstanceRecord.java:63-73)
    mp_map(S.pi_head, 11);
    key(S.pi_head, "bpmnElementType");
    key(S.pi_head, element_type_name(S.type));
    key(S.pi_head, "elementId");
    mp_str(S.pi_head, S.id);
    key(S.pi_head, "bpmnProcessId");
    mp_str(S.pi_head, P.bpmn_id);
    key(S.pi_head, "version");
    mp_int(S.pi_head, P.version);
    key(S.pi_head, "processDefinitionKey");
    mp_int(S.pi_head, P.def_key);
    key(S.pi_head, "processInstanceKey");
    key(S.pi_tail, "bpmnEventType");
    key(S.pi_tail, event_type_name(S.event));
    key(S.pi_tail, "parentProcessInstanceKey");
    mp_int(S.pi_tail, -1);
    key(S.pi_tail, "parentElementInstanceKey");
    mp_int(S.pi_tail, -1);
    key(S.pi_tail, "tenantId");
    key(S.pi_tail, kTenant);
    if (ZBHIP_IS_JOB_WORKER(E.element_type)) {
      // JobRecord (JobRecord.java:67-83) as BpmnJobBehavior.writeJobCreatedEvent fills it
      mp_map(S.job_head, 17);
      key(S.job_head, "deadline");
      mp_int(S.job_head, -1);
      key(S.job_head, "worker");
      key(S.job_head, "");
      S.job_rest = S.job_head.size();
      key(S.job_head, "retries");
      mp_int(S.job_head, (int32_t)E.job_retries);
      key(S.job_head, "retryBackoff");
      mp_int(S.job_head, 0);
      key(S.job_head, "recurringTime");
      mp_int(S.job_head, -1);
      key(S.job_head, "type");
      mp_str(S.job_head, str(E.job_type));
      key(S.job_head, "customHeaders");
      // BpmnJobBehavior.encodeHeaders (:219-248,365-399): the compiled task headers, or NO_HEADERS
      if (csr->header_begin && csr->header_begin[e + 1] > csr->header_begin[e])
        S.headers.assign(reinterpret_cast<const char*>(csr->header_bytes) + csr->header_begin[e],
                         csr->header_begin[e + 1] - csr->header_begin[e]);
      S.job_head += S.headers.empty() ? kEmptyDoc : S.headers;
      key(S.job_head, "variables");
      key(S.job_mid, "errorMessage");
      key(S.job_mid, "");
      key(S.job_mid, "errorCode");
      key(S.job_mid, "");
      key(S.job_mid, "bpmnProcessId");
      mp_str(S.job_mid, P.bpmn_id);
      key(S.job_mid, "processDefinitionVersion");
      mp_int(S.job_mid, P.version);
      key(S.job_mid, "processDefinitionKey");
      mp_int(S.job_mid, P.def_key);
      key(S.job_mid, "processInstanceKey");
      key(S.job_tail, "elementId");
      mp_str(S.job_tail, S.id);
      key(S.job_tail, "elementInstanceKey");
    }
  }
  if (idx_out) *idx_out = (uint32_t)s->procs.size();
  s->procs.push_back(std::move(P));
  return ZBHIP_OK;
}

// the stored customHeaders of a job of element `id` (its process by definition key): the element's task headers
static const Bytes& job_headers(const zbhip_serializer* s, int64_t def_key, const std::string& id) {
  for (const SerProcess& P : s->procs)
    if (P.def_key == def_key)
      for (const SerElement& E : P.els)
        if (E.id == id && ZBHIP_IS_JOB_WORKER(E.type)) return E.headers.empty() ? kEmptyDoc : E.headers;
  return kEmptyDoc;
}

// The errorMessage of an exclusive gateway's incident (BpmnIncidentBehavior.createIncident with the
// Failure of ExclusiveGatewayProcessor.findSequenceFlowToTake, :86-126): CONDITION_ERROR
// NO_OUTGOING_FLOW_CHOSEN_ERROR (:121-125), or ExpressionProcessor.typeCheck's EXTRACT_VALUE_ERROR
// (ExpressionProcessor.java:356-368) for the flow whose condition was not a boolean.
static bool incident_message(const zbhip_serializer* s, int32_t proc, int32_t error_type, int64_t flow,
                             uint32_t result, std::string& out) {
  if (error_type == ZBHIP_ERR_CONDITION_ERROR) {
    out = "Expected at least one condition to evaluate to true, or to have a default flow";
    return true;
  }
  if (error_type != ZBHIP_ERR_EXTRACT_VALUE_ERROR || proc < 0 || (size_t)proc >= s->procs.size() || flow < 0 ||
      (uint64_t)flow >= s->procs[proc].els.size() || result > ZBHIP_FEEL_STRING)
    return false;
  static const char* const kType[] = {"NULL", "NUMBER", "STRING"};
  out = "Expected result of the expression '" + s->procs[proc].els[flow].cond_text + "' to be 'BOOLEAN', but was '" +
        kType[result] + "'.";
  return true;
}

int64_t zbhip_serializer_incident_message(zbhip_serializer* s, const zbhip_record* r, char* buf, size_t cap) {
  if (!s || !r || (cap && !buf) || r->value_type != ZBHIP_VT_INCIDENT) return ZBHIP_EINVAL;
  std::string m;
  if (!incident_message(s, r->process_idx, r->partition, r->aux, r->reason_arg, m)) return ZBHIP_EINVAL;
  if (cap) memcpy(buf, m.data(), std::min(cap, m.size()));
  return (int64_t)m.size();
}

const char* zbhip_serializer_name(zbhip_serializer* s, uint32_t id) {
  return s && id < s->names.size() ? s->names[id].c_str() : "";
}

// Rejection reason text exactly as the reference writes it (ProcessInstanceStateTransitionGuard.java
// :74-186, JobCommandPreconditionChecker, processing/message/*Processor.java).
int zbhip_serializer_rejection_reason(zbhip_serializer* s, const zbhip_record* r, char* buf, size_t cap) {
  if (!s || !r || !buf) return ZBHIP_EINVAL;
  std::string id;
  if (r->process_idx >= 0 && (size_t)r->process_idx < s->procs.size() && r->element_idx >= 0 &&
      (size_t)r->element_idx < s->procs[r->process_idx].els.size())
    id = s->procs[r->process_idx].els[r->element_idx].id;
  const char* mname = zbhip_serializer_name(s, r->message_name);
  switch (r->reason) {
    case ZBHIP_REASON_PGW_NOT_ALL_TAKEN:
      return snprintf(buf, cap, "Expected to be able to activate parallel gateway '%s', but not all sequence flows have been taken.", id.c_str());
    case ZBHIP_REASON_FS_NOT_FOUND:
      return snprintf(buf, cap, "Expected flow scope instance with key '%lld' to be present in state but not found.", (long long)r->scope_key);
    case ZBHIP_REASON_FS_STATE:
      return snprintf(buf, cap, "Expected flow scope instance to be in state 'ELEMENT_ACTIVATED' but was '%s'.", state_text(r->reason_arg));
    case ZBHIP_REASON_EI_NOT_FOUND:
      return snprintf(buf, cap, "Expected element instance with key '%lld' to be present in state but not found.", (long long)r->key);
    case ZBHIP_REASON_EI_STATE:
      return snprintf(buf, cap, "Expected element instance to be in state 'ELEMENT_ACTIVATED' or one of '[ELEMENT_COMPLETING]' but was '%s'.", state_text(r->reason_arg));
    case ZBHIP_REASON_JOB_NOT_FOUND:
      return snprintf(buf, cap, "Expected to complete job with key '%lld', but no such job was found", (long long)r->key);
    case ZBHIP_REASON_MS_ALREADY_OPEN:
      return snprintf(buf, cap, "Expected to open a new message subscription for element with key '%lld' and message "
                      "name '%s', but there is already a message subscription for that element key and message name opened",
                      (long long)r->scope_key, mname);
    case ZBHIP_REASON_PMS_CREATE_NOT_FOUND:
      return snprintf(buf, cap, "Expected to create process message subscription with element key '%lld' and message "
                      "name '%s', but no such subscription was found", (long long)r->scope_key, mname);
    case ZBHIP_REASON_PMS_CREATE_NOT_OPENING:
      return snprintf(buf, cap, "Expected to create process message subscription with element key '%lld' and message "
                      "name '%s', but it is already %s", (long long)r->scope_key, mname, r->reason_arg ? "opened" : "closing");
    case ZBHIP_REASON_MS_CORR_NOT_FOUND:
      return snprintf(buf, cap, "Expected to correlate subscription for element with key '%lld' and message name '%s', "
                      "but no such message subscription exists", (long long)r->scope_key, mname);
    case ZBHIP_REASON_TIMER_NOT_FOUND:  // TriggerTimerProcessor.java:40-41
      return snprintf(buf, cap, "Expected to trigger timer with key '%lld', but no such timer was found", (long long)r->key);
    case ZBHIP_REASON_TIMER_NOT_ACTIVE:  // TriggerTimerProcessor.java:42-43
      return snprintf(buf, cap, "Expected to trigger a timer with key '%lld', but the timer is not active anymore",
                      (long long)r->key);
    case ZBHIP_REASON_JOB_STATE: {  // JobCommandPreconditionChecker.java:19-49
      const char* verb = r->intent == ZBHIP_JOB_FAIL ? "fail" : r->intent == ZBHIP_JOB_COMPLETE ? "complete" : "update";
      if (r->reason_arg == 3)
        return snprintf(buf, cap, "Expected to %s job with key '%lld', but no such job was found", verb, (long long)r->key);
      return snprintf(buf, cap, "Expected to %s job with key '%lld', but it is in state '%s'", verb, (long long)r->key,
                      r->reason_arg == 2 ? "FAILED" : r->reason_arg == 1 ? "ACTIVATED" : "ACTIVATABLE");
    }
    case ZBHIP_REASON_JOB_TIME_OUT:  // JobTimeOutProcessor.java:26-27,57-66
      return snprintf(buf, cap, "Expected to time out activated job with key '%lld', but %s", (long long)r->key,
                      r->reason_arg == 0 ? "no such job was found" : r->reason_arg == 1 ? "it must be activated first"
                      : r->reason_arg == 3 ? "it is marked as failed and is not activated" : "it has not timed out");
    default:
      if (cap) buf[0] = 0;
      return 0;
  }
}

}  // extern "C"

namespace {

// msgpack of one document value, canonical client encoding (compact ints, float64 decimals = v / 10^6)
bool doc_value(const zbhip_serializer* s, const zbhip_doc_entry& d, Bytes& b) {
  switch (d.type) {
    case ZBHIP_DOC_NIL: b.push_back((char)0xc0); return true;
    case ZBHIP_DOC_BOOL: b.push_back((char)(d.value ? 0xc3 : 0xc2)); return true;
    case ZBHIP_DOC_INT: mp_int(b, d.value); return true;
    case ZBHIP_DOC_DEC: {
      const double v = (double)d.value / 1e6;
      uint64_t u;
      memcpy(&u, &v, 8);
      b.push_back((char)0xcb);
      be64(b, u);
      return true;
    }
    case ZBHIP_DOC_STR:
      if ((uint64_t)d.value >= s->strs.size()) return false;
      mp_str(b, s->strs[(size_t)d.value]);
      return true;
    case ZBHIP_DOC_LIST: {  // an array of its items (MultiInstanceOutputCollectionBehavior: header + items)
      if ((uint64_t)d.value >= s->lists.size()) return false;
      const auto& items = s->lists[(size_t)d.value];
      mp_array(b, (uint32_t)items.size());
      for (const auto& it : items) {
        zbhip_doc_entry e{};
        e.type = it.first;
        e.value = it.second;
        if (e.type == ZBHIP_DOC_LIST || !doc_value(s, e, b)) return false;
      }
      return true;
    }
    default: return false;
  }
}

// a list value's items in a state row: "type:value;..." (the oracle's format, zb_oracle.cpp list_text)
std::vector<std::pair<uint8_t, int64_t>> parse_list_text(const std::string& t) {
  std::vector<std::pair<uint8_t, int64_t>> items;
  size_t a = 0;
  while (a < t.size()) {
    size_t e = t.find(';', a);
    if (e == std::string::npos) e = t.size();
    const std::string it = t.substr(a, e - a);
    const size_t c = it.find(':');
    if (c != std::string::npos)
      items.push_back({(uint8_t)strtol(it.substr(0, c).c_str(), nullptr, 10), (int64_t)strtoll(it.c_str() + c + 1, nullptr, 10)});
    a = e + 1;
  }
  return items;
}

bool document(const zbhip_serializer* s, const zbhip_doc_entry* e, size_t n, Bytes& b) {
  if (n == 0) { b = kEmptyDoc; return true; }  // DocumentValue.wrap: empty / nil -> EMPTY_DOCUMENT
  b.clear();
  mp_map(b, (uint32_t)n);
  for (size_t i = 0; i < n; ++i) {
    if (e[i].name_id >= s->names.size()) return false;
    mp_str(b, s->names[e[i].name_id]);
    if (!doc_value(s, e[i], b)) return false;
  }
  return true;
}

void le16(Bytes& b, uint16_t v) { b.push_back((char)v); b.push_back((char)(v >> 8)); }
void le32(Bytes& b, uint32_t v) { le16(b, (uint16_t)v); le16(b, (uint16_t)(v >> 16)); }
void le64(Bytes& b, uint64_t v) { le32(b, (uint32_t)v); le32(b, (uint32_t)(v >> 32)); }

}  // namespace

extern "C" int zbhip_serialize_log(zbhip_serializer* s, const zbhip_record* recs, size_t n, const zbhip_log_window* w,
                                   uint8_t* out, size_t cap, size_t* used) {
  if (!s || !w || (n && !recs) || !used) return ZBHIP_EINVAL;
  *used = 0;
  Bytes value, md, doc, entry;
  char reason[512];
  size_t off = 0;
  int64_t last_src = -1;
  Bytes src_doc;
  for (size_t i = 0; i < n; ++i) {
    const zbhip_record& r = recs[i];
    const int64_t ci = r.source_index - w->source_base;
    if (ci < 0 || (size_t)ci >= w->n_cmds) return ZBHIP_EINVAL;
    const zbhip_command& cm = w->cmds[ci];
    if (r.source_index != last_src) {  // the source command's variable document
      if (cm.doc_count && ((uint64_t)cm.doc_begin + cm.doc_count > w->n_docs || !w->docs)) return ZBHIP_EINVAL;
      if (!document(s, cm.doc_count ? w->docs + cm.doc_begin : nullptr, cm.doc_count, src_doc)) return ZBHIP_EUNSUPP;
      last_src = r.source_index;
    }
    const SerProcess* P = r.process_idx >= 0 && (size_t)r.process_idx < s->procs.size() ? &s->procs[r.process_idx] : nullptr;
    const SerElement* E = P && r.element_idx >= 0 && (size_t)r.element_idx < P->els.size() ? &P->els[r.element_idx] : nullptr;
    value.clear();
    switch (r.value_type) {
      case ZBHIP_VT_PROCESS_INSTANCE:
        if (!E) return ZBHIP_EINVAL;
        value += E->pi_head;
        mp_int(value, r.process_instance_key);
        key(value, "flowScopeKey");
        mp_int(value, r.scope_key);
        value += E->pi_tail;
        break;
      case ZBHIP_VT_JOB:
        if (r.record_type == ZBHIP_RT_REJECTION) {  // the JOB:COMPLETE command's value
          mp_map(value, 17);
          key(value, "deadline"); mp_int(value, -1);
          key(value, "worker"); key(value, "");
          key(value, "retries"); mp_int(value, -1);
          key(value, "retryBackoff"); mp_int(value, 0);
          key(value, "recurringTime"); mp_int(value, -1);
          key(value, "type"); key(value, "");
          key(value, "customHeaders"); value += kEmptyDoc;
          key(value, "variables"); mp_bin(value, src_doc);
          key(value, "errorMessage"); key(value, "");
          key(value, "errorCode"); key(value, "");
          key(value, "bpmnProcessId"); key(value, "");
          key(value, "processDefinitionVersion"); mp_int(value, -1);
          key(value, "processDefinitionKey"); mp_int(value, -1);
          key(value, "processInstanceKey"); mp_int(value, -1);
          key(value, "elementId"); key(value, "");
          key(value, "elementInstanceKey"); mp_int(value, -1);
          key(value, "tenantId"); key(value, kTenant);
        } else {
          if (!E || E->job_head.empty()) return ZBHIP_EINVAL;
          if (r.message_key != -1) {  // an ACTIVATED job: the deadline and worker it was activated with
            if (r.correlation_key != ZBHIP_NO_STRING && r.correlation_key >= s->strs.size()) return ZBHIP_EINVAL;
            mp_map(value, 17);
            key(value, "deadline");
            mp_int(value, r.message_key);
            key(value, "worker");
            mp_str(value, r.correlation_key == ZBHIP_NO_STRING ? std::string() : s->strs[r.correlation_key]);
            value.append(E->job_head, E->job_rest, std::string::npos);
          } else {
            value += E->job_head;
          }
          mp_bin(value, r.intent == ZBHIP_JOB_COMPLETED ? src_doc : kEmptyDoc);
          value += E->job_mid;
          mp_int(value, r.process_instance_key);
          value += E->job_tail;
          mp_int(value, r.scope_key);
          key(value, "tenantId");
          key(value, kTenant);
        }
        break;
      case ZBHIP_VT_VARIABLE: {
        if (!P || r.element_idx < 0 || (size_t)r.element_idx >= s->names.size()) return ZBHIP_EINVAL;
        doc.clear();
        if (r.aux == ZBHIP_AUX_INLINE) {  // a value the engine computed (multi-instance loop variables)
          zbhip_doc_entry d{};
          d.name_id = (uint32_t)r.element_idx;
          d.type = (uint8_t)r.partition;
          d.value = r.message_key;
          if (!doc_value(s, d, doc)) return ZBHIP_EUNSUPP;
        } else {
          const int64_t di = r.aux - w->doc_base;
          if (!w->docs || di < 0 || (size_t)di >= w->n_docs) return ZBHIP_EINVAL;
          if (!doc_value(s, w->docs[di], doc)) return ZBHIP_EUNSUPP;
        }
        mp_map(value, 7);  // VariableRecord.java:35-41
        key(value, "name"); mp_str(value, s->names[r.element_idx]);
        key(value, "value"); mp_bin(value, doc);
        key(value, "scopeKey"); mp_int(value, r.scope_key);
        key(value, "processInstanceKey"); mp_int(value, r.process_instance_key);
        key(value, "processDefinitionKey"); mp_int(value, P->def_key);
        key(value, "bpmnProcessId"); mp_str(value, P->bpmn_id);
        key(value, "tenantId"); key(value, kTenant);
        break;
      }
      case ZBHIP_VT_PROCESS_EVENT:
        if (!E || !P) return ZBHIP_EINVAL;
        mp_map(value, 6);  // ProcessEventRecord.java:37-42
        key(value, "scopeKey"); mp_int(value, r.scope_key);
        key(value, "targetElementId"); mp_str(value, E->id);
        // TRIGGERED: EventTriggerBehavior.processEventTriggered resets the record (no variables)
        key(value, "variables"); mp_bin(value, r.intent == ZBHIP_PE_TRIGGERED ? kEmptyDoc : src_doc);
        key(value, "processDefinitionKey"); mp_int(value, P->def_key);
        key(value, "processInstanceKey"); mp_int(value, r.process_instance_key);
        key(value, "tenantId"); key(value, kTenant);
        break;
      case ZBHIP_VT_TIMER:
        // TimerRecord.java:24-40 (CREATED / TRIGGERED: CatchEventBehavior.java:311-319; a rejected
        // TIMER:TRIGGER: the command's value -- DueDateTimerChecker.java:118-125 from the window's
        // timer_values, else as far as the window holds it: its key and dueDate)
        if (r.record_type == ZBHIP_RT_REJECTION && w->timer_values) {
          const zbhip_timer_value& tv = w->timer_values[ci];
          const SerProcess* TP = tv.process_idx >= 0 && (size_t)tv.process_idx < s->procs.size() ? &s->procs[tv.process_idx] : nullptr;
          const SerElement* TE = TP && tv.element_idx >= 0 && (size_t)tv.element_idx < TP->els.size() ? &TP->els[tv.element_idx] : nullptr;
          mp_map(value, 7);
          key(value, "elementInstanceKey"); mp_int(value, tv.element_instance_key);
          key(value, "processInstanceKey"); mp_int(value, tv.process_instance_key);
          key(value, "dueDate"); mp_int(value, r.aux);
          key(value, "targetElementId"); mp_str(value, TE ? TE->id : std::string());
          key(value, "repetitions"); mp_int(value, tv.repetitions);
          key(value, "processDefinitionKey"); mp_int(value, tv.process_definition_key);
          key(value, "tenantId"); key(value, kTenant);
          break;
        }
        mp_map(value, 7);
        key(value, "elementInstanceKey"); mp_int(value, r.scope_key);
        key(value, "processInstanceKey"); mp_int(value, r.process_instance_key);
        key(value, "dueDate"); mp_int(value, r.aux);
        key(value, "targetElementId"); mp_str(value, E ? E->id : std::string());
        key(value, "repetitions"); mp_int(value, r.record_type == ZBHIP_RT_REJECTION ? 1 : r.partition);
        key(value, "processDefinitionKey"); mp_int(value, P ? P->def_key : -1);
        key(value, "tenantId"); key(value, kTenant);
        break;
      case ZBHIP_VT_INCIDENT: {
        // IncidentRecord (protocol-impl/.../incident/IncidentRecord.java:36-47, declaration order)
        std::string msg;
        if (!E || !incident_message(s, r.process_idx, r.partition, r.aux, r.reason_arg, msg)) return ZBHIP_EINVAL;
        mp_map(value, 10);
        key(value, "errorType");
        key(value, r.partition == ZBHIP_ERR_CONDITION_ERROR ? "CONDITION_ERROR" : "EXTRACT_VALUE_ERROR");
        key(value, "errorMessage"); mp_str(value, msg);
        key(value, "bpmnProcessId"); mp_str(value, P->bpmn_id);
        key(value, "processDefinitionKey"); mp_int(value, P->def_key);
        key(value, "processInstanceKey"); mp_int(value, r.process_instance_key);
        key(value, "elementId"); mp_str(value, E->id);
        key(value, "elementInstanceKey"); mp_int(value, r.scope_key);
        key(value, "jobKey"); mp_int(value, -1);
        key(value, "variableScopeKey"); mp_int(value, r.scope_key);
        key(value, "tenantId"); key(value, kTenant);
        break;
      }
      case ZBHIP_VT_PROCESS_INSTANCE_BATCH:
        mp_map(value, 3);  // ProcessInstanceBatchRecord.java:38-40
        key(value, "processInstanceKey"); mp_int(value, r.process_instance_key);
        key(value, "batchElementInstanceKey"); mp_int(value, r.scope_key);
        key(value, "index"); mp_int(value, r.partition);
        break;
      case ZBHIP_VT_PROCESS_INSTANCE_CREATION:
        if (!P) return ZBHIP_EINVAL;
        mp_map(value, 8);  // ProcessInstanceCreationRecord.java:48-55
        key(value, "bpmnProcessId"); mp_str(value, P->bpmn_id);
        key(value, "processDefinitionKey"); mp_int(value, P->def_key);
        key(value, "processInstanceKey"); mp_int(value, r.scope_key);
        key(value, "version"); mp_int(value, P->version);
        key(value, "variables"); mp_bin(value, src_doc);
        key(value, "fetchVariables"); mp_array(value, 0);
        key(value, "startInstructions"); mp_array(value, 0);
        key(value, "tenantId"); key(value, kTenant);
        break;
      case ZBHIP_VT_MESSAGE:
      case ZBHIP_VT_MESSAGE_SUBSCRIPTION:
      case ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION: {
        // the drained record carries every field of the reference record; message variables are
        // empty in the subset; MESSAGE deadline = the PUBLISH command's timestamp + timeToLive (0)
        // (MessagePublishProcessor.java:100-125)
        auto name = [&](uint32_t id) -> const std::string& {
          static const std::string empty;
          return id != 0xFFFF && id < s->names.size() ? s->names[id] : empty;
        };
        static const std::string empty_s;
        const std::string& corr =
            r.correlation_key != ZBHIP_NO_STRING && r.correlation_key < s->strs.size() ? s->strs[r.correlation_key] : empty_s;
        if (r.value_type == ZBHIP_VT_MESSAGE) {
          const int64_t ts = w->source_timestamps ? w->source_timestamps[ci] : w->timestamp;
          mp_map(value, 7);  // MessageRecord.java:37-43
          key(value, "name"); mp_str(value, name(r.message_name));
          key(value, "correlationKey"); mp_str(value, corr);
          key(value, "timeToLive"); mp_int(value, 0);
          key(value, "variables"); mp_bin(value, kEmptyDoc);
          key(value, "messageId"); key(value, "");
          key(value, "deadline"); mp_int(value, ts);
          key(value, "tenantId"); key(value, kTenant);
        } else if (r.value_type == ZBHIP_VT_MESSAGE_SUBSCRIPTION) {
          mp_map(value, 9);  // MessageSubscriptionRecord.java:40-48
          key(value, "processInstanceKey"); mp_int(value, r.process_instance_key);
          key(value, "elementInstanceKey"); mp_int(value, r.scope_key);
          key(value, "messageKey"); mp_int(value, r.message_key);
          key(value, "messageName"); mp_str(value, name(r.message_name));
          key(value, "correlationKey"); mp_str(value, corr);
          key(value, "interrupting"); value.push_back((char)(r.interrupting ? 0xc3 : 0xc2));
          key(value, "bpmnProcessId"); mp_str(value, name(r.bpmn_process_id));
          key(value, "variables"); mp_bin(value, kEmptyDoc);
          key(value, "tenantId"); key(value, kTenant);
        } else {
          mp_map(value, 11);  // ProcessMessageSubscriptionRecord.java:44-54
          key(value, "subscriptionPartitionId"); mp_int(value, r.partition);
          key(value, "processInstanceKey"); mp_int(value, r.process_instance_key);
          key(value, "elementInstanceKey"); mp_int(value, r.scope_key);
          key(value, "messageKey"); mp_int(value, r.message_key);
          key(value, "messageName"); mp_str(value, name(r.message_name));
          key(value, "variables"); mp_bin(value, kEmptyDoc);
          key(value, "interrupting"); value.push_back((char)(r.interrupting ? 0xc3 : 0xc2));
          key(value, "bpmnProcessId"); mp_str(value, name(r.bpmn_process_id));
          key(value, "correlationKey"); mp_str(value, corr);
          key(value, "elementId"); mp_str(value, E ? E->id : empty_s);
          key(value, "tenantId"); key(value, kTenant);
        }
        break;
      }
      default:
        return ZBHIP_EUNSUPP;
    }
    // ---- SBE RecordMetadata (messageHeader + 32-byte block + 2 var-data fields) ----
    md.clear();
    le16(md, 32); le16(md, 200); le16(md, 0); le16(md, 4);   // blockLength, templateId, schemaId, version
    md.push_back((char)r.record_type);
    le32(md, 0x80000000u);                                   // requestStreamId: int32 null
    le64(md, ~0ull);                                         // requestId: uint64 null
    le16(md, 4);                                             // protocolVersion = Protocol.PROTOCOL_VERSION
    md.push_back((char)r.value_type);
    md.push_back((char)r.intent);
    le32(md, (uint32_t)s->broker[0]); le32(md, (uint32_t)s->broker[1]); le32(md, (uint32_t)s->broker[2]);
    le16(md, 1);                                             // recordVersion: latest applier version / default
    const bool rej = r.record_type == ZBHIP_RT_REJECTION;
    md.push_back((char)(rej ? r.rejection_type : 255));     // RejectionType.NULL_VAL
    size_t rl = 0;
    if (rej) {
      const int k = zbhip_serializer_rejection_reason(s, &r, reason, sizeof reason);
      rl = k > 0 ? std::min((size_t)k, sizeof reason - 1) : 0;
    }
    le32(md, (uint32_t)rl);
    md.append(reason, rl);
    le32(md, (uint32_t)s->auth.size());
    md += s->auth;
    // ---- dispatcher frame + LogEntryDescriptor header + metadata + value, 8-aligned ----
    const size_t body = 40 + md.size() + value.size();
    const size_t framed = 12 + body;
    const size_t aligned = (framed + 7) & ~(size_t)7;
    const size_t ci_pos = (size_t)ci;
    const int64_t src_pos = w->source_positions ? w->source_positions[ci_pos] : -1;
    if (out && off + aligned <= cap) {
      uint8_t* p = out + off;
      memset(p, 0, aligned);
      const uint32_t fl = (uint32_t)framed;
      memcpy(p, &fl, 4);
      uint8_t* e = p + 12;
      // skipProcessing: a follow-up command processed in its batch (not one written unprocessed)
      e[2] = r.record_type == ZBHIP_RT_COMMAND && !r.unprocessed ? 1 : 0;
      const int64_t pos = w->first_position + (int64_t)i;
      memcpy(e + 4, &pos, 8);
      memcpy(e + 12, &src_pos, 8);
      memcpy(e + 20, &r.key, 8);
      memcpy(e + 28, &w->timestamp, 8);
      const uint16_t ml = (uint16_t)md.size();
      memcpy(e + 36, &ml, 2);
      memcpy(e + 40, md.data(), md.size());
      memcpy(e + 40 + md.size(), value.data(), value.size());
    }
    off += aligned;
  }
  *used = off;
  return off <= cap || !out ? ZBHIP_OK : ZBHIP_ENOMEM;
}

// ---- zb-db byte encoding of the exported state ----------------------------
// One canonical state row of zbhip_export_state -> its RocksDB entry: key = 8-byte big-endian
// column-family ordinal (ColumnFamilyContext.writeKey; ordinals = ZbColumnFamilies.java positions)
// + DbLong / DbString / DbInt parts (zb-db/.../impl/DbLong.java, DbString.java, DbInt.java: big
// endian, strings with a 4-byte length), value = DbNil (0xFF), DbLong / DbInt or the msgpack of the
// state's UnpackedObject (ElementInstance.java:23-55 + IndexedRecord.java:22-29, VariableInstance,
// EventScopeInstance, JobRecordValue, JobStateValue, NextValue, MessageSubscription,
// ProcessMessageSubscription).  Rows are split at '|' and ',': correlation keys / names holding
// those characters are outside what this encoder reads back.
namespace {

void dbl(Bytes& b, int64_t v) { be64(b, (uint64_t)v); }
void dbs(Bytes& b, const std::string& s) { be32(b, (uint32_t)s.size()); b.append(s); }
void cf_prefix(Bytes& b, uint32_t cf) { be64(b, cf); }
// a string a state row holds in hex (error messages may contain ',' and '|')
std::string unhex(const std::string& h) {
  std::string o;
  for (size_t i = 0; i + 1 < h.size(); i += 2) o += (char)std::stoi(h.substr(i, 2), nullptr, 16);
  return o;
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t a = 0;
  for (;;) {
    const size_t p = s.find(sep, a);
    out.push_back(s.substr(a, p == std::string::npos ? std::string::npos : p - a));
    if (p == std::string::npos) return out;
    a = p + 1;
  }
}
std::unordered_map<std::string, std::string> fields_of(const std::string& s) {
  std::unordered_map<std::string, std::string> m;
  for (auto& kv : split(s, ',')) {
    const size_t e = kv.find('=');
    m[kv.substr(0, e)] = e == std::string::npos ? "" : kv.substr(e + 1);
  }
  return m;
}
int64_t ll(const std::string& s) { return strtoll(s.c_str(), nullptr, 10); }

const char* pi_intent_name(int s) {
  switch (s) {
    case ZBHIP_PI_SEQUENCE_FLOW_TAKEN: return "SEQUENCE_FLOW_TAKEN";
    default: return state_text(s);
  }
}

}  // namespace

extern "C" int zbhip_serializer_encode_state_row(zbhip_serializer* s, const char* row, zbhip_db_sink sink, void* ctx) {
  if (!s || !row || !sink) return ZBHIP_EINVAL;
  const std::vector<std::string> p = split(row, '|');
  const std::string& cf = p[0];
  Bytes k, v;
  uint32_t ord = 0;
  auto need = [&](size_t n) { return p.size() >= n; };
  if (cf == "KEY" && need(3)) {  // NextValueManager: DbString "latestKey" -> NextValue
    ord = 1;
    cf_prefix(k, ord); dbs(k, p[1]);
    mp_map(v, 1); key(v, "nextValue"); mp_int(v, ll(p[2]));
  } else if (cf == "ELEMENT_INSTANCE_KEY" && need(3)) {
    ord = 7;
    auto f = fields_of(p[2]);
    const int64_t def = ll(f["processDefinitionKey"]);
    const SerProcess* P = nullptr;
    for (auto& q : s->procs)
      if (q.def_key == def) { P = &q; break; }
    if (!P) return ZBHIP_EINVAL;
    const int64_t ek = ll(p[1]);
    cf_prefix(k, ord); dbl(k, ek);
    mp_map(v, 11);  // ElementInstance.java:44-54
    key(v, "parentKey"); mp_int(v, ll(f["parentKey"]));
    key(v, "childCount"); mp_int(v, ll(f["childCount"]));
    key(v, "childActivatedCount"); mp_int(v, ll(f["childActivatedCount"]));
    key(v, "childCompletedCount"); mp_int(v, ll(f["childCompletedCount"]));
    key(v, "childTerminatedCount"); mp_int(v, ll(f["childTerminatedCount"]));
    key(v, "jobKey"); mp_int(v, ll(f["jobKey"]));
    key(v, "multiInstanceLoopCounter"); mp_int(v, ll(f["multiInstanceLoopCounter"]));
    key(v, "interruptingElementId"); mp_str(v, f["interruptingElementId"]);
    key(v, "calledChildInstanceKey"); mp_int(v, ll(f["calledChildInstanceKey"]));
    key(v, "elementRecord");
    mp_map(v, 3);  // IndexedRecord.java:29
    key(v, "key"); mp_int(v, ek);
    key(v, "state"); key(v, pi_intent_name((int)ll(f["state"])));
    key(v, "processInstanceRecord");
    mp_map(v, 11);  // ProcessInstanceRecord.java:63-73
    key(v, "bpmnElementType"); key(v, element_type_name((uint32_t)ll(f["bpmnElementType"])));
    key(v, "elementId"); mp_str(v, f["elementId"]);
    key(v, "bpmnProcessId"); mp_str(v, P->bpmn_id);
    key(v, "version"); mp_int(v, P->version);
    key(v, "processDefinitionKey"); mp_int(v, P->def_key);
    key(v, "processInstanceKey"); mp_int(v, ll(f["processInstanceKey"]));
    key(v, "flowScopeKey"); mp_int(v, ll(f["flowScopeKey"]));
    key(v, "bpmnEventType"); key(v, event_type_name((uint32_t)ll(f["bpmnEventType"])));
    key(v, "parentProcessInstanceKey"); mp_int(v, -1);
    key(v, "parentElementInstanceKey"); mp_int(v, -1);
    key(v, "tenantId"); key(v, kTenant);
    key(v, "activeSequenceFlows"); mp_int(v, ll(f["activeSequenceFlows"]));
  } else if (cf == "ELEMENT_INSTANCE_PARENT_CHILD" && need(3)) {
    ord = 6;
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbl(k, ll(p[2]));
    v.push_back((char)0xff);
  } else if (cf == "ELEMENT_INSTANCE_CHILD_PARENT" && need(3)) {
    ord = 9;
    cf_prefix(k, ord); dbl(k, ll(p[1]));
    dbl(v, ll(p[2]));
  } else if (cf == "NUMBER_OF_TAKEN_SEQUENCE_FLOWS" && need(5)) {
    ord = 8;
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbs(k, p[2]); dbs(k, p[3]);
    be32(v, (uint32_t)ll(p[4]));
  } else if (cf == "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY" && need(3)) {
    ord = 55;
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbl(k, ll(p[2]));
    v.push_back((char)0xff);
  } else if (cf == "VARIABLES" && need(4)) {
    ord = 10;
    auto f = fields_of(p[3]);
    zbhip_doc_entry d{};
    d.type = (uint8_t)ll(f["type"]);
    Bytes val;
    if (d.type == ZBHIP_DOC_LIST) {  // the row holds the items
      const auto items = parse_list_text(f["value"]);
      mp_array(val, (uint32_t)items.size());
      for (const auto& it : items) {
        zbhip_doc_entry e{};
        e.type = it.first;
        e.value = it.second;
        if (e.type == ZBHIP_DOC_LIST || !doc_value(s, e, val)) return ZBHIP_EUNSUPP;
      }
    } else {
      d.value = ll(f["value"]);
      if (!doc_value(s, d, val)) return ZBHIP_EUNSUPP;
    }
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbs(k, p[2]);
    mp_map(v, 2);  // VariableInstance.java:22
    key(v, "key"); mp_int(v, ll(f["key"]));
    key(v, "value"); mp_bin(v, val);
  } else if (cf == "EVENT_SCOPE" && need(3)) {
    ord = 37;
    auto f = fields_of(p[2]);
    cf_prefix(k, ord); dbl(k, ll(p[1]));
    mp_map(v, 4);  // EventScopeInstance.java:32-35
    auto ids = [&](const std::string& list) {  // ';'-separated element ids -> ArrayProperty<StringValue>
      std::vector<std::string> out;
      if (!list.empty()) out = split(list, ';');
      mp_array(v, (uint32_t)out.size());
      for (auto& id : out) mp_str(v, id);
    };
    key(v, "accepting"); v.push_back((char)(f["accepting"] == "1" ? 0xc3 : 0xc2));
    key(v, "interrupting"); ids(f["interrupting"]);
    key(v, "boundaryElementIds"); ids(f["boundaryElementIds"]);
    key(v, "interrupted"); v.push_back((char)(f["interrupted"] == "1" ? 0xc3 : 0xc2));
  } else if (cf == "JOBS" && need(3)) {
    ord = 16;
    auto f = fields_of(p[2]);
    cf_prefix(k, ord); dbl(k, ll(p[1]));
    mp_map(v, 1);  // JobRecordValue.java:21 -> JobRecord stored without variables (DbJobState.create)
    key(v, "jobRecord");
    mp_map(v, 17);
    const bool failed = f.count("errorMessageHex") != 0;  // a failed job's stored fields (JobFailProcessor)
    key(v, "deadline"); mp_int(v, f.count("deadline") ? ll(f["deadline"]) : -1);
    key(v, "worker"); mp_str(v, f["worker"]);
    key(v, "retries"); mp_int(v, ll(f["retries"]));
    key(v, "retryBackoff"); mp_int(v, failed ? ll(f["retryBackoff"]) : 0);
    key(v, "recurringTime"); mp_int(v, failed ? ll(f["recurringTime"]) : -1);
    key(v, "type"); mp_str(v, f["type"]);
    key(v, "customHeaders"); v += job_headers(s, ll(f["processDefinitionKey"]), f["elementId"]);
    key(v, "variables"); mp_bin(v, kEmptyDoc);
    key(v, "errorMessage"); mp_str(v, failed ? unhex(f["errorMessageHex"]) : std::string());
    key(v, "errorCode"); key(v, "");
    key(v, "bpmnProcessId"); mp_str(v, f["bpmnProcessId"]);
    key(v, "processDefinitionVersion"); mp_int(v, ll(f["processDefinitionVersion"]));
    key(v, "processDefinitionKey"); mp_int(v, ll(f["processDefinitionKey"]));
    key(v, "processInstanceKey"); mp_int(v, ll(f["processInstanceKey"]));
    key(v, "elementId"); mp_str(v, f["elementId"]);
    key(v, "elementInstanceKey"); mp_int(v, ll(f["elementInstanceKey"]));
    key(v, "tenantId"); mp_str(v, f["tenantId"]);
  } else if (cf == "TIMERS" && need(4)) {
    ord = 12;  // DbTimerInstanceState: [elementInstanceKey, timerKey] -> TimerInstance (TimerInstance.java:36-43)
    auto f = fields_of(p[3]);
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbl(k, ll(p[2]));
    mp_map(v, 8);
    key(v, "handlerNodeId"); mp_str(v, f["handlerNodeId"]);
    key(v, "processDefinitionKey"); mp_int(v, ll(f["processDefinitionKey"]));
    key(v, "key"); mp_int(v, ll(f["key"]));
    key(v, "elementInstanceKey"); mp_int(v, ll(f["elementInstanceKey"]));
    key(v, "processInstanceKey"); mp_int(v, ll(f["processInstanceKey"]));
    key(v, "dueDate"); mp_int(v, ll(f["dueDate"]));
    key(v, "repetitions"); mp_int(v, ll(f["repetitions"]));
    key(v, "tenantId"); mp_str(v, f["tenantId"]);
  } else if (cf == "INCIDENTS" && need(3)) {
    ord = 34;  // DbIncidentState: DbLong incidentKey -> Incident{incidentRecord} (Incident.java:17-22)
    auto f = fields_of(p[2]);
    const int64_t def = ll(f["processDefinitionKey"]);
    int32_t pi = -1;
    for (size_t q = 0; q < s->procs.size(); ++q)
      if (s->procs[q].def_key == def) { pi = (int32_t)q; break; }
    std::string msg;
    const bool job = f.count("jobKey") != 0;  // a job's incident (JOB_NO_RETRIES): its key and message
    if (job) msg = unhex(f["messageHex"]);
    if (pi < 0 ||
        (!job && !incident_message(s, pi, (int32_t)ll(f["errorType"]), ll(f["flow"]), (uint32_t)ll(f["result"]), msg)))
      return ZBHIP_EINVAL;
    const SerProcess& P = s->procs[pi];
    cf_prefix(k, ord); dbl(k, ll(p[1]));
    mp_map(v, 1);
    key(v, "incidentRecord");
    mp_map(v, 10);  // IncidentRecord.java:36-47
    const int64_t et = ll(f["errorType"]);
    key(v, "errorType");
    key(v, et == ZBHIP_ERR_JOB_NO_RETRIES ? "JOB_NO_RETRIES" : et == ZBHIP_ERR_CONDITION_ERROR ? "CONDITION_ERROR" : "EXTRACT_VALUE_ERROR");
    key(v, "errorMessage"); mp_str(v, msg);
    key(v, "bpmnProcessId"); mp_str(v, P.bpmn_id);
    key(v, "processDefinitionKey"); mp_int(v, def);
    key(v, "processInstanceKey"); mp_int(v, ll(f["processInstanceKey"]));
    key(v, "elementId"); mp_str(v, f["elementId"]);
    key(v, "elementInstanceKey"); mp_int(v, ll(f["elementInstanceKey"]));
    key(v, "jobKey"); mp_int(v, job ? ll(f["jobKey"]) : -1);
    key(v, "variableScopeKey"); mp_int(v, ll(f["elementInstanceKey"]));
    key(v, "tenantId"); key(v, kTenant);
  } else if (cf == "INCIDENT_JOBS" && need(3)) {
    ord = 36;  // DbForeignKey<DbLong> jobKey -> IncidentKey{key} (DbIncidentState.java:68-71)
    cf_prefix(k, ord); dbl(k, ll(p[1]));
    mp_map(v, 1); key(v, "key"); mp_int(v, ll(p[2]));
  } else if (cf == "JOB_BACKOFF" && need(3)) {
    ord = 42;  // [recurringTime, jobKey] -> DbNil (DbJobState.java:103-108)
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbl(k, ll(p[2]));
    v.push_back((char)0xff);
  } else if (cf == "INCIDENT_PROCESS_INSTANCES" && need(3)) {
    ord = 35;  // DbForeignKey<DbLong> elementInstanceKey -> IncidentKey{key} (IncidentKey.java)
    cf_prefix(k, ord); dbl(k, ll(p[1]));
    mp_map(v, 1); key(v, "key"); mp_int(v, ll(p[2]));
  } else if (cf == "TIMER_DUE_DATES" && need(4)) {
    ord = 13;  // [dueDate, [elementInstanceKey, timerKey]] -> DbNil
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbl(k, ll(p[2])); dbl(k, ll(p[3]));
    v.push_back((char)0xff);
  } else if (cf == "JOB_STATES" && need(3)) {
    ord = 17;
    cf_prefix(k, ord); dbl(k, ll(p[1]));
    mp_map(v, 1);  // JobStateValue.java:21
    key(v, "jobState"); mp_str(v, p[2]);
  } else if (cf == "JOB_DEADLINES" && need(3)) {
    ord = 18;  // DbJobState.java:100-102: [deadline, jobKey] -> DbNil
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbl(k, ll(p[2]));
    v.push_back((char)0xff);
  } else if (cf == "JOB_ACTIVATABLE" && need(4)) {
    ord = 76;  // DbTenantAwareKey(tenant, [type, jobKey], SUFFIX)
    cf_prefix(k, ord); dbs(k, p[1]); dbl(k, ll(p[3])); dbs(k, p[2]);
    v.push_back((char)0xff);
  } else if (cf == "MESSAGE_SUBSCRIPTION_BY_KEY" && need(4)) {
    ord = 27;  // [eik, messageName] -> MessageSubscription{record, key, correlating} (DbMessageSubscriptionState.java:64-73)
    auto f = fields_of(p[3]);
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbs(k, p[2]);
    mp_map(v, 3);
    key(v, "record");
    mp_map(v, 9);  // MessageSubscriptionRecord.java:40-48
    key(v, "processInstanceKey"); mp_int(v, ll(f["processInstanceKey"]));
    key(v, "elementInstanceKey"); mp_int(v, ll(p[1]));
    key(v, "messageKey"); mp_int(v, ll(f["messageKey"]));
    key(v, "messageName"); mp_str(v, p[2]);
    key(v, "correlationKey"); mp_str(v, f["correlationKey"]);
    key(v, "interrupting"); v.push_back((char)(f["interrupting"] == "1" ? 0xc3 : 0xc2));
    key(v, "bpmnProcessId"); mp_str(v, f["bpmnProcessId"]);
    key(v, "variables"); mp_bin(v, kEmptyDoc);
    key(v, "tenantId"); key(v, kTenant);
    key(v, "key"); mp_int(v, ll(f["key"]));
    key(v, "correlating"); v.push_back((char)(f["correlating"] == "1" ? 0xc3 : 0xc2));
  } else if (cf == "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY" && need(5)) {
    ord = 74;  // [[tenant, [name, correlationKey]] PREFIX, eik] -> DbNil (:75-86)
    cf_prefix(k, ord); dbs(k, p[1]); dbs(k, p[2]); dbs(k, p[3]); dbl(k, ll(p[4]));
    v.push_back((char)0xff);
  } else if (cf == "PROCESS_SUBSCRIPTION_BY_KEY" && need(4)) {
    ord = 75;  // [eik, [tenant, messageName] PREFIX] -> ProcessMessageSubscription{record, state, key}
    auto f = fields_of(p[3]);  // (DbProcessMessageSubscriptionState.java:53-66, ProcessMessageSubscription.java:19-26)
    cf_prefix(k, ord); dbl(k, ll(p[1])); dbs(k, kTenant); dbs(k, p[2]);
    mp_map(v, 3);
    key(v, "record");
    mp_map(v, 11);  // ProcessMessageSubscriptionRecord.java:44-54
    key(v, "subscriptionPartitionId"); mp_int(v, ll(f["subscriptionPartitionId"]));
    key(v, "processInstanceKey"); mp_int(v, ll(f["processInstanceKey"]));
    key(v, "elementInstanceKey"); mp_int(v, ll(p[1]));
    key(v, "messageKey"); mp_int(v, ll(f["messageKey"]));
    key(v, "messageName"); mp_str(v, p[2]);
    key(v, "variables"); mp_bin(v, kEmptyDoc);
    key(v, "interrupting"); v.push_back((char)(f["interrupting"] == "1" ? 0xc3 : 0xc2));
    key(v, "bpmnProcessId"); mp_str(v, f["bpmnProcessId"]);
    key(v, "correlationKey"); mp_str(v, f["correlationKey"]);
    key(v, "elementId"); mp_str(v, f["elementId"]);
    key(v, "tenantId"); key(v, kTenant);
    key(v, "state"); mp_str(v, "STATE_" + f["state"]);
    key(v, "key"); mp_int(v, ll(f["key"]));
  } else if (cf == "MESSAGE_STATS" && need(3)) {
    ord = 54;  // DbMessageState.java:165-175: DbString "deadline_message_count" -> DbLong
    cf_prefix(k, ord); dbs(k, "deadline_message_count");
    dbl(v, ll(p[2]));
  } else {
    return 0;  // not a column family of the path
  }
  sink(ctx, ord, reinterpret_cast<const uint8_t*>(k.data()), k.size(), reinterpret_cast<const uint8_t*>(v.data()),
       v.size());
  return 1;
}

// ---- zb-db entry -> canonical state row (the inverse of zbhip_serializer_encode_state_row) ------
// The importer's front end (zbhip_import_state_db): RocksDB keys and the msgpack of the state
// objects read back exactly as the encoder above writes them (MsgPackReader.java semantics for the
// value types the path stores).
namespace {

struct MpNode {
  enum Kind { NIL, BOOL, INT, FLOAT, STR, BIN, MAP, ARR } k = NIL;
  int64_t i = 0;
  double f = 0;
  std::string s;                                   // STR / BIN bytes
  std::vector<std::pair<std::string, MpNode>> kv;  // MAP (string keys)
  std::vector<MpNode> arr;
  const MpNode* get(const char* name) const {
    for (auto& e : kv)
      if (e.first == name) return &e.second;
    return nullptr;
  }
};

struct MpReader {
  const uint8_t* p;
  const uint8_t* e;
  bool need(size_t n) const { return (size_t)(e - p) >= n; }
  uint64_t be(int n) {
    uint64_t v = 0;
    for (int k = 0; k < n; ++k) v = (v << 8) | *p++;
    return v;
  }
  bool parse(MpNode& o, int depth = 0) {
    if (depth > 8 || !need(1)) return false;
    const uint8_t t = *p++;
    auto bytes = [&](uint32_t n, MpNode::Kind k) {
      if (!need(n)) return false;
      o.k = k;
      o.s.assign(reinterpret_cast<const char*>(p), n);
      p += n;
      return true;
    };
    auto map = [&](uint32_t n) {
      o.k = MpNode::MAP;
      for (uint32_t j = 0; j < n; ++j) {
        MpNode key, v;
        if (!parse(key, depth + 1) || key.k != MpNode::STR || !parse(v, depth + 1)) return false;
        o.kv.emplace_back(std::move(key.s), std::move(v));
      }
      return true;
    };
    auto arr = [&](uint32_t n) {
      o.k = MpNode::ARR;
      o.arr.resize(n);
      for (uint32_t j = 0; j < n; ++j)
        if (!parse(o.arr[j], depth + 1)) return false;
      return true;
    };
    if (t <= 0x7f) { o.k = MpNode::INT; o.i = t; return true; }
    if (t >= 0xe0) { o.k = MpNode::INT; o.i = (int8_t)t; return true; }
    if ((t & 0xf0) == 0x80) return map(t & 0x0f);
    if ((t & 0xf0) == 0x90) return arr(t & 0x0f);
    if ((t & 0xe0) == 0xa0) return bytes(t & 0x1f, MpNode::STR);
    switch (t) {
      case 0xc0: o.k = MpNode::NIL; return true;
      case 0xc2: case 0xc3: o.k = MpNode::BOOL; o.i = t == 0xc3; return true;
      case 0xc4: return need(1) && bytes((uint32_t)be(1), MpNode::BIN);
      case 0xc5: return need(2) && bytes((uint32_t)be(2), MpNode::BIN);
      case 0xc6: return need(4) && bytes((uint32_t)be(4), MpNode::BIN);
      case 0xcb: {
        if (!need(8)) return false;
        const uint64_t u = be(8);
        o.k = MpNode::FLOAT;
        memcpy(&o.f, &u, 8);
        return true;
      }
      case 0xcc: if (!need(1)) return false; o.k = MpNode::INT; o.i = (int64_t)be(1); return true;
      case 0xcd: if (!need(2)) return false; o.k = MpNode::INT; o.i = (int64_t)be(2); return true;
      case 0xce: if (!need(4)) return false; o.k = MpNode::INT; o.i = (int64_t)be(4); return true;
      case 0xcf: if (!need(8)) return false; o.k = MpNode::INT; o.i = (int64_t)be(8); return true;
      case 0xd0: if (!need(1)) return false; o.k = MpNode::INT; o.i = (int8_t)be(1); return true;
      case 0xd1: if (!need(2)) return false; o.k = MpNode::INT; o.i = (int16_t)be(2); return true;
      case 0xd2: if (!need(4)) return false; o.k = MpNode::INT; o.i = (int32_t)be(4); return true;
      case 0xd3: if (!need(8)) return false; o.k = MpNode::INT; o.i = (int64_t)be(8); return true;
      case 0xd9: return need(1) && bytes((uint32_t)be(1), MpNode::STR);
      case 0xda: return need(2) && bytes((uint32_t)be(2), MpNode::STR);
      case 0xdb: return need(4) && bytes((uint32_t)be(4), MpNode::STR);
      case 0xdc: return need(2) && arr((uint32_t)be(2));
      case 0xdd: return need(4) && arr((uint32_t)be(4));
      case 0xde: return need(2) && map((uint32_t)be(2));
      case 0xdf: return need(4) && map((uint32_t)be(4));
      default: return false;
    }
  }
};

bool mp_read(const uint8_t* v, size_t n, MpNode& out) {
  MpReader r{v, v + n};
  return r.parse(out) && r.p == r.e;
}

// key parts: DbLong / DbInt / DbString (big-endian, DbString 4-byte length)
struct KeyReader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  int64_t dblong() {
    if (e - p < 8) { ok = false; return 0; }
    uint64_t v = 0;
    for (int k = 0; k < 8; ++k) v = (v << 8) | *p++;
    return (int64_t)v;
  }
  int32_t dbint() {
    if (e - p < 4) { ok = false; return 0; }
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) v = (v << 8) | *p++;
    return (int32_t)v;
  }
  std::string dbstr() {
    const int32_t n = dbint();
    if (!ok || n < 0 || e - p < n) { ok = false; return std::string(); }
    std::string s(reinterpret_cast<const char*>(p), (size_t)n);
    p += n;
    return s;
  }
};

int enum_index(const char* (*name)(uint32_t), uint32_t count, const std::string& s) {
  for (uint32_t t = 0; t < count; ++t)
    if (s == name(t)) return (int)t;
  return -1;
}
int state_index(const std::string& s) {
  for (int t = ZBHIP_PI_ELEMENT_ACTIVATING; t <= ZBHIP_PI_ELEMENT_TERMINATED; ++t)
    if (s == state_text(t)) return t;
  return -1;
}
int64_t mi(const MpNode* n) { return n && n->k == MpNode::INT ? n->i : 0; }
std::string ms(const MpNode* n) { return n && n->k == MpNode::STR ? n->s : std::string(); }
int mb(const MpNode* n) { return n && n->k == MpNode::BOOL && n->i ? 1 : 0; }

}  // namespace

extern "C" int zbhip_serializer_decode_state_entry(zbhip_serializer* s, uint32_t cf, const uint8_t* key, size_t klen,
                                                   const uint8_t* val, size_t vlen, zbhip_string_interner intern,
                                                   void* ictx, char* row, size_t cap) {
  if (!s || (!key && klen) || (!val && vlen) || !row || cap == 0) return ZBHIP_EINVAL;
  KeyReader K{key, key + klen};
  if (K.dblong() != (int64_t)cf || !K.ok) return ZBHIP_EINVAL;
  std::string out;
  char b[512];
  MpNode v;
  auto value = [&]() { return mp_read(val, vlen, v) && v.k == MpNode::MAP; };
  auto be_long = [&](const uint8_t* p, size_t n, int64_t& o) {
    if (n != 8) return false;
    uint64_t x = 0;
    for (int k = 0; k < 8; ++k) x = (x << 8) | p[k];
    o = (int64_t)x;
    return true;
  };
  switch (cf) {
    case 1: {  // KEY
      const std::string name = K.dbstr();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "KEY|%s|%lld", name.c_str(), (long long)mi(v.get("nextValue")));
      out = b;
      break;
    }
    case 7: {  // ELEMENT_INSTANCE_KEY
      const int64_t ek = K.dblong();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      const MpNode* rec = v.get("elementRecord");
      const MpNode* pir = rec ? rec->get("processInstanceRecord") : nullptr;
      if (!rec || !pir) return ZBHIP_EINVAL;
      const int state = state_index(ms(rec->get("state")));
      const int et = enum_index(element_type_name, 24, ms(pir->get("bpmnElementType")));
      const int ev = enum_index(event_type_name, 10, ms(pir->get("bpmnEventType")));
      if (state < 0 || et < 0 || ev < 0) return ZBHIP_EINVAL;
      snprintf(b, sizeof b,
               "ELEMENT_INSTANCE_KEY|%lld|parentKey=%lld,childCount=%lld,childActivatedCount=%lld,childCompletedCount=%lld,"
               "childTerminatedCount=%lld,jobKey=%lld,multiInstanceLoopCounter=%lld,interruptingElementId=%s,"
               "calledChildInstanceKey=%lld,state=%d,elementId=%s,bpmnElementType=%d,bpmnEventType=%d,flowScopeKey=%lld,"
               "processInstanceKey=%lld,processDefinitionKey=%lld,activeSequenceFlows=%lld",
               (long long)ek, (long long)mi(v.get("parentKey")), (long long)mi(v.get("childCount")),
               (long long)mi(v.get("childActivatedCount")), (long long)mi(v.get("childCompletedCount")),
               (long long)mi(v.get("childTerminatedCount")), (long long)mi(v.get("jobKey")),
               (long long)mi(v.get("multiInstanceLoopCounter")), ms(v.get("interruptingElementId")).c_str(),
               (long long)mi(v.get("calledChildInstanceKey")), state, ms(pir->get("elementId")).c_str(), et, ev,
               (long long)mi(pir->get("flowScopeKey")), (long long)mi(pir->get("processInstanceKey")),
               (long long)mi(pir->get("processDefinitionKey")), (long long)mi(v.get("activeSequenceFlows")));
      out = b;
      break;
    }
    case 6: case 55: {  // ELEMENT_INSTANCE_PARENT_CHILD, PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY -> DbNil
      const int64_t a = K.dblong(), c = K.dblong();
      if (!K.ok) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "%s|%lld|%lld", cf == 6 ? "ELEMENT_INSTANCE_PARENT_CHILD" : "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY",
               (long long)a, (long long)c);
      out = b;
      break;
    }
    case 9: {  // ELEMENT_INSTANCE_CHILD_PARENT -> DbLong
      const int64_t c = K.dblong();
      int64_t parent = 0;
      if (!K.ok || !be_long(val, vlen, parent)) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "ELEMENT_INSTANCE_CHILD_PARENT|%lld|%lld", (long long)c, (long long)parent);
      out = b;
      break;
    }
    case 8: {  // NUMBER_OF_TAKEN_SEQUENCE_FLOWS -> DbInt
      const int64_t scope = K.dblong();
      const std::string gw = K.dbstr(), flow = K.dbstr();
      if (!K.ok || vlen != 4) return ZBHIP_EINVAL;
      const int32_t n = (int32_t)(((uint32_t)val[0] << 24) | ((uint32_t)val[1] << 16) | ((uint32_t)val[2] << 8) | val[3]);
      snprintf(b, sizeof b, "NUMBER_OF_TAKEN_SEQUENCE_FLOWS|%lld|%s|%s|%d", (long long)scope, gw.c_str(), flow.c_str(), n);
      out = b;
      break;
    }
    case 10: {  // VARIABLES
      const int64_t scope = K.dblong();
      const std::string name = K.dbstr();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      const MpNode* bin = v.get("value");
      MpNode x;
      if (!bin || bin->k != MpNode::BIN ||
          !mp_read(reinterpret_cast<const uint8_t*>(bin->s.data()), bin->s.size(), x))
        return ZBHIP_EINVAL;
      int type;
      long long dv = 0;
      switch (x.k) {
        case MpNode::NIL: type = ZBHIP_DOC_NIL; break;
        case MpNode::BOOL: type = ZBHIP_DOC_BOOL; dv = x.i; break;
        case MpNode::INT: type = ZBHIP_DOC_INT; dv = x.i; break;
        case MpNode::FLOAT: {  // exact 6-digit scaled decimals only (the device's DEC)
          type = ZBHIP_DOC_DEC;
          const double sc = x.f * 1e6;
          if (!(sc > -9.2e18 && sc < 9.2e18)) return ZBHIP_EUNSUPP;
          dv = llround(sc);
          if ((double)dv / 1e6 != x.f) return ZBHIP_EUNSUPP;
          break;
        }
        case MpNode::STR: {
          if (!intern) return ZBHIP_EUNSUPP;
          const int64_t id = intern(ictx, x.s.data(), x.s.size());
          if (id < 0) return (int)id;
          type = ZBHIP_DOC_STR;
          dv = id;
          break;
        }
        case MpNode::ARR: {  // a list of scalars: its items in the row (ZBHIP_DOC_LIST)
          std::string items;
          for (const auto& it : x.arr) {
            long long iv = 0;
            int ity;
            if (it.k == MpNode::NIL) ity = ZBHIP_DOC_NIL;
            else if (it.k == MpNode::BOOL) { ity = ZBHIP_DOC_BOOL; iv = it.i; }
            else if (it.k == MpNode::INT) { ity = ZBHIP_DOC_INT; iv = it.i; }
            else if (it.k == MpNode::FLOAT) {
              ity = ZBHIP_DOC_DEC;
              const double sc = it.f * 1e6;
              if (!(sc > -9.2e18 && sc < 9.2e18)) return ZBHIP_EUNSUPP;
              iv = llround(sc);
              if ((double)iv / 1e6 != it.f) return ZBHIP_EUNSUPP;
            } else if (it.k == MpNode::STR) {
              if (!intern) return ZBHIP_EUNSUPP;
              const int64_t id = intern(ictx, it.s.data(), it.s.size());
              if (id < 0) return (int)id;
              ity = ZBHIP_DOC_STR;
              iv = id;
            } else {
              return ZBHIP_EUNSUPP;  // nested documents / arrays
            }
            items += (items.empty() ? "" : ";") + std::to_string(ity) + ":" + std::to_string(iv);
          }
          snprintf(b, sizeof b, "VARIABLES|%lld|%s|key=%lld,type=%d,value=", (long long)scope, name.c_str(),
                   (long long)mi(v.get("key")), (int)ZBHIP_DOC_LIST);
          out = std::string(b) + items;
          break;
        }
        default: return ZBHIP_EUNSUPP;  // documents: outside the device's variables
      }
      if (x.k == MpNode::ARR) break;
      snprintf(b, sizeof b, "VARIABLES|%lld|%s|key=%lld,type=%d,value=%lld", (long long)scope, name.c_str(),
               (long long)mi(v.get("key")), type, dv);
      out = b;
      break;
    }
    case 37: {  // EVENT_SCOPE
      const int64_t k = K.dblong();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      auto ids = [&](const char* name) {
        std::string out;
        if (const MpNode* a = v.get(name))
          for (const auto& it : a->arr) out += (out.empty() ? "" : ";") + ms(&it);
        return out;
      };
      snprintf(b, sizeof b, "EVENT_SCOPE|%lld|accepting=%d,interrupted=%d,interrupting=%s,boundaryElementIds=%s",
               (long long)k, mb(v.get("accepting")), mb(v.get("interrupted")), ids("interrupting").c_str(),
               ids("boundaryElementIds").c_str());
      out = b;
      break;
    }
    case 16: {  // JOBS
      const int64_t k = K.dblong();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      const MpNode* j = v.get("jobRecord");
      if (!j) return ZBHIP_EINVAL;
      snprintf(b, sizeof b,
               "JOBS|%lld|type=%s,retries=%lld,elementId=%s,elementInstanceKey=%lld,processInstanceKey=%lld,"
               "bpmnProcessId=%s,processDefinitionKey=%lld,processDefinitionVersion=%lld,tenantId=%s,deadline=%lld,"
               "worker=%s",
               (long long)k, ms(j->get("type")).c_str(), (long long)mi(j->get("retries")), ms(j->get("elementId")).c_str(),
               (long long)mi(j->get("elementInstanceKey")), (long long)mi(j->get("processInstanceKey")),
               ms(j->get("bpmnProcessId")).c_str(), (long long)mi(j->get("processDefinitionKey")),
               (long long)mi(j->get("processDefinitionVersion")), ms(j->get("tenantId")).c_str(),
               (long long)mi(j->get("deadline")), ms(j->get("worker")).c_str());
      out = b;
      // a failed job's stored fields (JobFailProcessor): errorMessage in hex, retryBackoff, recurringTime
      // (a failure that left all three at their defaults reads back through its retries alone)
      const std::string em = ms(j->get("errorMessage"));
      const long long rb = mi(j->get("retryBackoff")), rt = j->get("recurringTime") ? mi(j->get("recurringTime")) : -1;
      if (!em.empty() || rb != 0 || rt != -1) {
        static const char* hx = "0123456789abcdef";
        out += ",errorMessageHex=";
        for (unsigned char c : em) {
          out += hx[c >> 4];
          out += hx[c & 15];
        }
        out += ",retryBackoff=" + std::to_string(rb) + ",recurringTime=" + std::to_string(rt);
      }
      break;
    }
    case 17: {  // JOB_STATES
      const int64_t k = K.dblong();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "JOB_STATES|%lld|%s", (long long)k, ms(v.get("jobState")).c_str());
      out = b;
      break;
    }
    case 12: {  // TIMERS [eik, timerKey] -> TimerInstance
      const int64_t e = K.dblong(), t = K.dblong();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      snprintf(b, sizeof b,
               "TIMERS|%lld|%lld|handlerNodeId=%s,processDefinitionKey=%lld,key=%lld,elementInstanceKey=%lld,"
               "processInstanceKey=%lld,dueDate=%lld,repetitions=%lld,tenantId=%s",
               (long long)e, (long long)t, ms(v.get("handlerNodeId")).c_str(), (long long)mi(v.get("processDefinitionKey")),
               (long long)mi(v.get("key")), (long long)mi(v.get("elementInstanceKey")),
               (long long)mi(v.get("processInstanceKey")), (long long)mi(v.get("dueDate")),
               (long long)mi(v.get("repetitions")), ms(v.get("tenantId")).c_str());
      out = b;
      break;
    }
    case 13: {  // TIMER_DUE_DATES [dueDate, eik, timerKey] -> DbNil
      const int64_t d = K.dblong(), e = K.dblong(), t = K.dblong();
      if (!K.ok) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "TIMER_DUE_DATES|%lld|%lld|%lld", (long long)d, (long long)e, (long long)t);
      out = b;
      break;
    }
    case 18: {  // JOB_DEADLINES [deadline, jobKey] -> DbNil
      const int64_t d = K.dblong(), k = K.dblong();
      if (!K.ok) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "JOB_DEADLINES|%lld|%lld", (long long)d, (long long)k);
      out = b;
      break;
    }
    case 76: {  // JOB_ACTIVATABLE [[type, jobKey], tenant]
      const std::string type = K.dbstr();
      const int64_t k = K.dblong();
      const std::string tenant = K.dbstr();
      if (!K.ok) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "JOB_ACTIVATABLE|%s|%s|%lld", type.c_str(), tenant.c_str(), (long long)k);
      out = b;
      break;
    }
    case 75: {  // PROCESS_SUBSCRIPTION_BY_KEY [eik, [tenant, name]]
      const int64_t eik = K.dblong();
      const std::string tenant = K.dbstr(), name = K.dbstr();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      const MpNode* r = v.get("record");
      if (!r) return ZBHIP_EINVAL;
      std::string st = ms(v.get("state"));
      if (st.rfind("STATE_", 0) == 0) st = st.substr(6);
      snprintf(b, sizeof b,
               "PROCESS_SUBSCRIPTION_BY_KEY|%lld|%s|key=%lld,state=%s,subscriptionPartitionId=%lld,processInstanceKey=%lld,"
               "bpmnProcessId=%s,messageKey=%lld,correlationKey=%s,elementId=%s,interrupting=%d",
               (long long)eik, name.c_str(), (long long)mi(v.get("key")), st.c_str(),
               (long long)mi(r->get("subscriptionPartitionId")), (long long)mi(r->get("processInstanceKey")),
               ms(r->get("bpmnProcessId")).c_str(), (long long)mi(r->get("messageKey")),
               ms(r->get("correlationKey")).c_str(), ms(r->get("elementId")).c_str(), mb(r->get("interrupting")));
      out = b;
      break;
    }
    case 27: {  // MESSAGE_SUBSCRIPTION_BY_KEY [eik, name]
      const int64_t eik = K.dblong();
      const std::string name = K.dbstr();
      if (!K.ok || !value()) return ZBHIP_EINVAL;
      const MpNode* r = v.get("record");
      if (!r) return ZBHIP_EINVAL;
      snprintf(b, sizeof b,
               "MESSAGE_SUBSCRIPTION_BY_KEY|%lld|%s|key=%lld,correlating=%d,processInstanceKey=%lld,bpmnProcessId=%s,"
               "messageKey=%lld,correlationKey=%s,interrupting=%d",
               (long long)eik, name.c_str(), (long long)mi(v.get("key")), mb(v.get("correlating")),
               (long long)mi(r->get("processInstanceKey")), ms(r->get("bpmnProcessId")).c_str(),
               (long long)mi(r->get("messageKey")), ms(r->get("correlationKey")).c_str(), mb(r->get("interrupting")));
      out = b;
      break;
    }
    case 74: {  // MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY
      const std::string tenant = K.dbstr(), name = K.dbstr(), corr = K.dbstr();
      const int64_t eik = K.dblong();
      if (!K.ok) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY|%s|%s|%s|%lld", tenant.c_str(), name.c_str(),
               corr.c_str(), (long long)eik);
      out = b;
      break;
    }
    case 54: {  // MESSAGE_STATS
      const std::string name = K.dbstr();
      int64_t n = 0;
      if (!K.ok || !be_long(val, vlen, n)) return ZBHIP_EINVAL;
      snprintf(b, sizeof b, "MESSAGE_STATS|messagesDeadlineCount|%lld", (long long)n);
      out = b;
      break;
    }
    default:
      return 0;  // not a column family of the path
  }
  if (K.p != K.e) return ZBHIP_EINVAL;  // trailing key bytes
  if (out.size() + 1 > cap) return ZBHIP_ENOMEM;
  memcpy(row, out.c_str(), out.size() + 1);
  return (int)out.size();
}

// ---- device tables of the serialiser (logdev.hip) ------------------------------------------------
// The constant byte runs of zbhip_serialize_log, laid out for the device writer: a byte arena (runs
// 4-aligned) and a u32 table -- the global runs in logdev.hip's LogRun order (offset, length), the
// names (msgpack strings), then per process: bpmnProcessId (msgpack string), definition key (lo,
// hi), version, element count, and per element its ProcessInstanceRecord / JobRecord runs, its id as
// a msgpack string and raw (the reason texts).
namespace zb {
void serializer_broker(const zbhip_serializer* s, int32_t out[3]) {
  for (int i = 0; i < 3; ++i) out[i] = s ? s->broker[i] : 0;
}
// Entry templates for the device writer (logdev.hip k_log_write): every record kind whose log entry
// has a fixed layout once its keys are fixed-width -- PROCESS_INSTANCE events and commands,
// JOB:CREATED, JOB:COMPLETED / PROCESS_EVENT / PROCESS_INSTANCE_CREATION:CREATED without a document --
// serialised here once per (process, element, kind) with sentinel keys, positions and timestamp.
// The device copies a template and patches the header's position / sourcePosition / key / timestamp
// (8-byte little-endian at 16 / 24 / 32 / 40) and the value's processInstanceKey and scope key
// (msgpack uint64, big-endian, at the offsets found here).  Keys >= 2^32 always take the 9-byte msgpack
// form, and every key of the path is >= 2^51; a process element's flowScopeKey is -1 (its own template).
// desc (uint4 per template): x = byte offset (16-aligned), y = size | (pik value offset << 16), z =
// scope value offset (value offsets: the first byte after 0xcf, 0 = none); idx: [0] process count,
// [1 + p] the base of process p's [element][kLogTplKinds] table of template id + 1 (0: none).
constexpr uint32_t kLogTplKinds = 18;  // = zb_internal.h
int log_device_templates(zbhip_serializer* s, std::vector<uint8_t>& bytes, std::vector<uint32_t>& desc,
                         std::vector<uint32_t>& idx) {
  if (!s) return ZBHIP_EINVAL;
  bytes.clear();
  desc.clear();
  idx.clear();
  const int64_t KEY = 0x0F1E2D3C4B5A6978LL, PIK = 0x1A2B3C4D5E6F7081LL, SCOPE = 0x2B3C4D5E6F708192LL;
  const int64_t POS = 0x3C4D5E6F708192A3LL, SRC = 0x4D5E6F708192A3B4LL, TS = 0x5E6F708192A3B4C5LL;
  zbhip_command cmd{};
  const int64_t src = SRC;
  zbhip_log_window w{};
  w.cmds = &cmd;
  w.n_cmds = 1;
  w.source_positions = &src;
  w.first_position = POS;
  w.timestamp = TS;
  std::vector<uint8_t> out(4096);
  auto be_bytes = [](int64_t v) {
    std::string b(9, '\0');
    b[0] = (char)0xcf;
    for (int i = 0; i < 8; ++i) b[1 + i] = (char)((uint64_t)v >> (56 - 8 * i));
    return b;
  };
  const std::string pik_be = be_bytes(PIK), scope_be = be_bytes(SCOPE);
  idx.push_back((uint32_t)s->procs.size());
  idx.resize(1 + s->procs.size(), 0);
  for (size_t p = 0; p < s->procs.size(); ++p) {
    idx[1 + p] = (uint32_t)idx.size();
    const size_t ne = s->procs[p].els.size();
    const size_t base = idx.size();
    idx.resize(base + ne * kLogTplKinds, 0);
    for (size_t e = 0; e < ne; ++e) {
      for (uint32_t k = 0; k < kLogTplKinds; ++k) {
        zbhip_record r{};
        r.key = KEY;
        r.process_instance_key = PIK;
        r.scope_key = SCOPE;
        r.process_idx = (int32_t)p;
        r.element_idx = (int32_t)e;
        r.rejection_type = ZBHIP_REJ_NONE;
        r.aux = -1;
        r.message_key = -1;
        r.correlation_key = ZBHIP_NO_STRING;
        r.message_name = r.bpmn_process_id = 0xFFFF;
        // only the kinds an element of its type has on the path (a sequence flow is only taken; every
        // other element never is; unprocessed commands -- past the batch limit -- are composed): the
        // table then fits LDS next to the device writer's stages (logdev.hip k_log_stream)
        const bool flow = s->procs[p].els[e].type == ZBHIP_EL_SEQUENCE_FLOW;
        if (flow ? k != 0 : (k == 0 || (k >= 7 && k <= 9))) continue;
        if (k < 13) {  // PROCESS_INSTANCE: events 1..7, unprocessed commands 8..10, processed ones (10 + ...)
          const uint32_t intent = k < 10 ? k + 1 : k - 2;
          r.value_type = ZBHIP_VT_PROCESS_INSTANCE;
          r.intent = (uint8_t)intent;
          r.record_type = intent >= 8 ? ZBHIP_RT_COMMAND : ZBHIP_RT_EVENT;
          r.unprocessed = intent >= 8 && k < 10 ? 1 : 0;
          if (e == 0) r.scope_key = -1;  // the process: flowScopeKey -1
        } else if (k == 13 || k == 17) {
          if (!ZBHIP_IS_JOB_WORKER(s->procs[p].els[e].type)) continue;
          r.value_type = ZBHIP_VT_JOB;
          r.intent = k == 13 ? ZBHIP_JOB_CREATED : ZBHIP_JOB_COMPLETED;
          r.record_type = ZBHIP_RT_EVENT;
        } else if (k == 14 || k == 15) {
          r.value_type = ZBHIP_VT_PROCESS_EVENT;
          r.intent = k == 14 ? ZBHIP_PE_TRIGGERING : ZBHIP_PE_TRIGGERED;
          r.record_type = ZBHIP_RT_EVENT;
        } else {  // 16
          if (e != 0) continue;
          r.value_type = ZBHIP_VT_PROCESS_INSTANCE_CREATION;
          r.intent = ZBHIP_PIC_CREATED;
          r.record_type = ZBHIP_RT_EVENT;
        }
        size_t used = 0;
        if (zbhip_serialize_log(s, &r, 1, &w, out.data(), out.size(), &used) != ZBHIP_OK || used > 512 || used % 8)
          continue;
        const std::string b(reinterpret_cast<const char*>(out.data()), used);
        auto le_at = [&b](size_t o) {
          uint64_t v = 0;
          for (int i = 7; i >= 0; --i) v = (v << 8) | (uint8_t)b[o + i];
          return (int64_t)v;
        };
        if (le_at(16) != POS || le_at(24) != SRC || le_at(32) != KEY || le_at(40) != TS) continue;
        if (b.find(be_bytes(KEY)) != std::string::npos) continue;  // the record key inside the value
        const size_t a = b.find(pik_be), c = b.find(scope_be);
        if ((a != std::string::npos && b.find(pik_be, a + 1) != std::string::npos) ||
            (c != std::string::npos && b.find(scope_be, c + 1) != std::string::npos))
          continue;  // a sentinel twice: not a fixed layout
        const size_t off = bytes.size();
        bytes.insert(bytes.end(), b.begin(), b.end());
        bytes.resize((bytes.size() + 15) & ~(size_t)15, 0);
        const uint32_t id = (uint32_t)(desc.size() / 4);
        desc.push_back((uint32_t)off);
        desc.push_back((uint32_t)used | ((a == std::string::npos ? 0u : (uint32_t)a + 1) << 16));
        desc.push_back(c == std::string::npos ? 0u : (uint32_t)c + 1);
        desc.push_back(0);
        idx[base + e * kLogTplKinds + k] = id + 1;
      }
    }
  }
  return ZBHIP_OK;
}

int log_device_tables(const zbhip_serializer* s, std::vector<uint8_t>& arena, std::vector<uint32_t>& idx) {
  if (!s) return ZBHIP_EINVAL;
  arena.clear();
  idx.clear();
  auto push = [&](const Bytes& b) {
    while (arena.size() % 4) arena.push_back(0);
    idx.push_back((uint32_t)arena.size());
    idx.push_back((uint32_t)b.size());
    arena.insert(arena.end(), b.begin(), b.end());
  };
  auto k = [](std::initializer_list<const char*> keys) {
    Bytes b;
    for (const char* x : keys) key(b, x);
    return b;
  };
  Bytes b;
  le32(b, (uint32_t)s->auth.size());  // G_AUTH: the metadata's authorization var-data
  b += s->auth;
  push(b);
  b.clear(); key(b, "tenantId"); key(b, kTenant); push(b);           // G_TENANT
  push(k({"flowScopeKey"}));                                          // G_FLOWSCOPE
  b.clear(); mp_bin(b, kEmptyDoc); push(b);                           // G_EMPTY_BIN
  b.clear();                                                          // G_JREJ_HEAD (JOB:COMPLETE value)
  mp_map(b, 17);
  key(b, "deadline"); mp_int(b, -1);
  key(b, "worker"); key(b, "");
  key(b, "retries"); mp_int(b, -1);
  key(b, "retryBackoff"); mp_int(b, 0);
  key(b, "recurringTime"); mp_int(b, -1);
  key(b, "type"); key(b, "");
  key(b, "customHeaders"); b += kEmptyDoc;
  key(b, "variables");
  push(b);
  b.clear();                                                          // G_JREJ_TAIL
  key(b, "errorMessage"); key(b, "");
  key(b, "errorCode"); key(b, "");
  key(b, "bpmnProcessId"); key(b, "");
  key(b, "processDefinitionVersion"); mp_int(b, -1);
  key(b, "processDefinitionKey"); mp_int(b, -1);
  key(b, "processInstanceKey"); mp_int(b, -1);
  key(b, "elementId"); key(b, "");
  key(b, "elementInstanceKey"); mp_int(b, -1);
  key(b, "tenantId"); key(b, kTenant);
  push(b);
  b.clear(); mp_map(b, 7); key(b, "name"); push(b);                   // G_VAR_A
  push(k({"value"}));                                                 // G_VAR_VALUE
  push(k({"scopeKey"}));                                              // G_VAR_SCOPE
  push(k({"processInstanceKey"}));                                    // G_K_PIK
  push(k({"processDefinitionKey"}));                                  // G_K_DEF
  push(k({"bpmnProcessId"}));                                         // G_K_BPMN
  b.clear(); mp_map(b, 6); key(b, "scopeKey"); push(b);               // G_PE_A
  push(k({"targetElementId"}));                                       // G_PE_TARGET
  push(k({"variables"}));                                             // G_K_VARS
  b.clear(); mp_map(b, 8); key(b, "bpmnProcessId"); push(b);          // G_PIC_A
  push(k({"version"}));                                               // G_K_VERSION
  b.clear(); key(b, "fetchVariables"); mp_array(b, 0); key(b, "startInstructions"); mp_array(b, 0); push(b);  // G_PIC_TAIL
  for (const char* t : {"Expected to be able to activate parallel gateway '", "', but not all sequence flows have been taken.",
                        "Expected flow scope instance with key '", "' to be present in state but not found.",
                        "Expected flow scope instance to be in state 'ELEMENT_ACTIVATED' but was '", "'.",
                        "Expected element instance with key '",
                        "Expected element instance to be in state 'ELEMENT_ACTIVATED' or one of '[ELEMENT_COMPLETING]' but was '",
                        "Expected to complete job with key '", "', but no such job was found",
                        "Expected to trigger timer with key '", "', but no such timer was found",
                        "Expected to trigger a timer with key '", "', but the timer is not active anymore"})
    push(Bytes(t));                                                   // G_RS_*
  b.clear(); mp_map(b, 7); key(b, "elementInstanceKey"); push(b);     // G_TIMER_A (TimerRecord.java:24-40)
  push(k({"dueDate"}));                                               // G_TIMER_DUE
  push(k({"repetitions"}));                                           // G_TIMER_REPS
  b.clear(); mp_map(b, 17); key(b, "deadline"); push(b);              // G_JACT_A (an ACTIVATED job's head)
  push(k({"worker"}));                                                // G_JACT_W
  for (int st = 0; st < 16; ++st) push(Bytes(state_text(st)));       // G_ST0 ..
  idx.push_back((uint32_t)s->names.size());
  for (const std::string& nm : s->names) {
    b.clear();
    mp_str(b, nm);
    push(b);
  }
  const size_t p0 = idx.size();
  idx.push_back((uint32_t)s->procs.size());
  idx.resize(idx.size() + s->procs.size(), 0);
  for (size_t p = 0; p < s->procs.size(); ++p) {
    const SerProcess& P = s->procs[p];
    idx[p0 + 1 + p] = (uint32_t)idx.size();
    b.clear();
    mp_str(b, P.bpmn_id);
    push(b);
    idx.push_back((uint32_t)((uint64_t)P.def_key & 0xFFFFFFFFu));
    idx.push_back((uint32_t)((uint64_t)P.def_key >> 32));
    idx.push_back((uint32_t)P.version);
    idx.push_back((uint32_t)P.els.size());
    for (const SerElement& E : P.els) {
      push(E.pi_head);
      push(E.pi_tail);
      push(E.job_head);
      push(E.job_mid);
      push(E.job_tail);
      b.clear();
      mp_str(b, E.id);
      push(b);
      push(E.id);
      push(E.job_head.empty() ? Bytes() : E.job_head.substr(E.job_rest));  // E_JOB_REST
      idx.push_back(E.duration_ms);  // E_DUR: not a byte run, the element's timer duration
      idx.push_back(E.interrupting_cycle);  // (and whether it is an interrupting boundary event's cycle)
    }
  }
  while (arena.size() % 4) arena.push_back(0);
  return ZBHIP_OK;
}
}  // namespace zb
