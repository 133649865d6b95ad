// Internal layouts shared by the gfx950 kernels (engine.hip) and the host runtime.
#pragma once
#include <stdint.h>

#include "../../include/zbhip.h"

namespace zb {

// workgroup size and per-lane LDS capacities are per kernel variant (KCfg in kernels.hip);
// every workgroup owns one output region of (workgroup size) * rec_cap records
constexpr int kSlots = 8;          // persistent element-instance slots per process instance (HBM)
constexpr int kVars = 4;           // variables per process instance (HBM)
constexpr int kJoinWords = 4;      // 16 x u8 taken-sequence-flow counters per instance (HBM)
constexpr int kMaxJoinSlots = 4 * kJoinWords;
constexpr uint32_t kMaxProgWords = 6144;  // program arena staged in LDS (24 KiB; total LDS <= 64 KiB)
constexpr int kMaxElements = 4095;        // 12-bit element index in queue entries

constexpr uint16_t NONE = 0xFFFF;
constexpr int kMaxScopeDepth = 8;         // container scopes an io-mapped scope chain walk visits (KScopeIO)

// ---- message correlation (config 5; kernel variant KMsg) ----
constexpr int kSubs = 4;           // message-subscription rows per correlation slot (HBM)
// CREATE batch templates (kernels.hip tpl_create): per process kTplVar variants (the outcome of
// its one exclusive gateway), each a header (2 uint2) and up to kTplRec compact records
constexpr int kTplVar = 4;
constexpr int kTplRec = 126;
constexpr uint32_t kTplWords = kTplRec + 2;  // uint2 per variant
// the templates of processes 0 .. kTplLdsProcs-1 (their first kTplLdsWords words) are staged in LDS
// by every workgroup at kernel start
constexpr int kTplLdsProcs = 2;
constexpr uint32_t kTplLdsWords = 64;
constexpr uint32_t TPL_OK = 1u << 31;        // program header word 7: bit 31 eligible, bits 0..11 gateway
// row r of correlation slot s in sub_a / sub_b / sub_k: slot-major, so a slot's kSubs rows share
// one cache line per array (a lookup reads 3 lines, not 3 * kSubs)
__host__ __device__ inline size_t sub_ri(uint32_t r, size_t slot) { return slot * kSubs + r; }
// command kinds whose subject is a correlation slot (MESSAGE / MESSAGE_SUBSCRIPTION commands), and
// the PROCESS_MESSAGE_SUBSCRIPTION commands (subject: an instance slot)
__host__ __device__ inline bool zb_slot_kind(uint32_t k) {
  return k == ZBHIP_CMD_PUBLISH || k == ZBHIP_CMD_MSG_SUB_CREATE || k == ZBHIP_CMD_MSG_SUB_CORRELATE ||
         k == ZBHIP_CMD_MSG_SUB_DELETE;
}
__host__ __device__ inline bool zb_pms_kind(uint32_t k) {
  return k == ZBHIP_CMD_PMS_CREATE || k == ZBHIP_CMD_PMS_CORRELATE || k == ZBHIP_CMD_PMS_DELETE;
}
constexpr int kOut = 6;            // outbox entries per command (sends + local-row key patches)
constexpr uint8_t XK_PATCH = 0xFF; // outbox entry kind: patch the real keys of a locally inserted row
constexpr uint32_t kNoElem = 0xFFF;       // element field of records without an element
constexpr uint32_t kPayloadBit = 1u << 14; // record followed by kPayloadRows payload rows
constexpr int kPayloadRows = 6;
// 64-bit key references inside payload rows and outbox entries: >= 0 a real key, -1 none,
// <= -2 an ordinal: v = -2 - ref, space = v >> 16 (0: the lane's instance, 1: the lane's
// correlation slot), ord = v & 0xFFFF.  The device key scan / the host drain resolve them.
enum : uint32_t { KS_INST = 0, KS_SLOT = 1 };

// The dueDate of a timer cycle's next timer (TriggerTimerProcessor.refreshTimer, :161-175):
// Interval.withStart(the TRIGGER command's dueDate) starts at dueDate + interval, and
// Interval.toEpochMilli(now) (Interval.java:77-93) returns that start unless it is not after now,
// then now + interval (a trigger processed a period or more late does not schedule a past dueDate).
__host__ __device__ inline long long next_cycle_due(long long due, long long interval, long long now) {
  return due + interval <= now ? now + interval : due + interval;
}

// ElementInstance.jobKey encodings in a slot (ElementInstance.java:23-54: default 0,
// JobCreatedApplier sets the job key, JobCompletedApplier sets -1)
constexpr uint16_t JOB_ZERO = 0xFFFF;
constexpr uint16_t JOB_MINUS1 = 0xFFFE;

// Compact device record: 8 bytes
//   x = key_ord | aux_ord << 16        (0xFFFF = -1)
//   y = elem | code << 16 | flags << 24
// code: PI events/commands = ProcessInstanceIntent value (1..10), others below,
//       | kRejectBit for COMMAND_REJECTION.  flags: rejection reason | arg << 4.
enum : uint8_t {
  C_JOB_CREATED = 16,
  C_JOB_COMPLETED = 17,
  C_JOB_COMPLETE = 18,
  C_JOB_CANCELED = 19,    // BpmnJobBehavior.cancelJob (JOB:CANCELED, the stored job)
  C_VAR_CREATED = 20,
  C_VAR_UPDATED = 21,
  C_MI_ITEM = 22,         // VARIABLE:CREATED of a multi-instance inner instance's inputElement / its
  C_MI_LOOP = 23,         // loopCounter (MultiInstanceBodyProcessor.setLoopVariables): key = the variable,
                          // aux = the inner instance, elem = the body, flags = the loop counter
  C_PIB_ACTIVATE = 26,    // PROCESS_INSTANCE_BATCH:ACTIVATE (command): aux = the body, elem = the body,
                          // flags = the collection's size (the record's index) | F_UNPROCESSED
  C_PIB_TERMINATE = 27,   // PROCESS_INSTANCE_BATCH:TERMINATE (terminateChildInstances, command): aux = the
                          // container instance, elem = the container (index -1: from the first child)
  C_PE_TRIGGERING = 24,
  C_PE_TRIGGERED = 25,    // EventTriggerBehavior.processEventTriggered
  C_PIC_CREATED = 28,
  C_PMS_CREATING = 32,
  C_PMS_CREATE = 33,
  C_PMS_CREATED = 34,
  C_PMS_CORRELATE = 35,
  C_PMS_CORRELATED = 36,
  C_PMS_DELETING = 37,    // CatchEventBehavior.unsubscribeFromMessageEvent (the stored subscription)
  C_PMS_DELETE = 38,      // the acknowledgement command (closeProcessMessageSubscription)
  C_PMS_DELETED = 39,
  C_MS_CREATE = 40,
  C_MS_CREATED = 41,
  C_MS_CORRELATING = 42,
  C_MS_CORRELATE = 43,
  C_MS_CORRELATED = 44,
  C_MS_DELETE = 45,       // closeMessageSubscription (command)
  C_MS_DELETED = 46,
  C_MSG_PUBLISHED = 49,
  C_MSG_EXPIRED = 50,
  C_TIMER_CREATED = 52,   // key = timer, aux = element instance, flags = repetitions (255 infinite)
                          // (TimerRecord, CatchEventBehavior.java:303-330)
  C_TIMER_TRIGGER = 53,   // (rejections of TIMER:TRIGGER)
  C_TIMER_TRIGGERED = 54,
  C_TIMER_CANCELED = 55,  // CatchEventBehavior.unsubscribeFromTimerEvent; dueDate in StepParams.cmd_due
  C_TIMER_NEXT = 56,
  C_JOB_PUSHED = 59,      // JOB_BATCH:ACTIVATED of a job stream's push (BpmnJobActivationBehavior.publishWork):
                          // key = the batch, aux = the job, elem = the task
  // multi-instance collections (MultiInstanceBodyProcessor / MultiInstanceOutputCollectionBehavior); the
  // host completes their values from the drained rows in log order (runtime.cpp track_mi)
  C_MI_LIST_ITEM = 60,    // VARIABLE:CREATED of the inputElement from a list variable: key = the variable,
                          // aux / elem = the list id's low / high half (scope, body and loop counter: the
                          // C_MI_LOOP row that follows)
  C_MI_OUTEL = 61,        // VARIABLE:CREATED nil of the outputElement variable (setLoopVariables): key = the
                          // variable, aux = the inner instance, elem = the body
  C_MI_OUT = 62,          // the body's outputCollection: aux = the body instance, elem = the body; flags bit 7
                          // set: CREATED [nil] * (flags & 0x7F), key = the variable; else UPDATED at index
                          // key of the item (zbhip_doc_type flags & 7, value in map_val slot flags >> 4 & 3)
  C_MI_PROP = 63,         // propagateVariable of the outputCollection: VARIABLE:CREATED in the process scope,
                          // key = the variable, aux = the body instance, elem = the body
  C_VAR_MAPPED = 58,       // VARIABLE:CREATED / UPDATED of an io mapping (BpmnVariableMappingBehavior): key =
                           // the variable, aux = its scope, elem = its name, flags = zbhip_doc_type | updated
                           // << 3 | value slot << 4 (the value in StepParams.map_val)
  C_INCIDENT_CREATED = 57,  // INCIDENT:CREATED of an exclusive gateway: key = incident, aux = the gateway's
                            // element instance, elem = the gateway, flags = the incident info (kernels.hip
                            // find_sequence_flow: flow position 0..14 / 15 none chosen | FEEL type << 4)      // TIMER:CREATED of a cycle's next timer (rescheduleTimer): dueDate from the
                          // TRIGGER command's, not the run's clock
  kRejectBit = 0x40,
};

// zbhip_exchange_gather's launch arguments (kernels.hip k_xgather)
constexpr uint32_t kMaxGatherParts = 16;
struct XGather {
  const zbhip_xpart_cmd* src[kMaxGatherParts];
  zbhip_xpart_cmd* dst[kMaxGatherParts];
  const uint32_t* counts;
  uint32_t P;
};

// per-command header written by k_step: x = nrec | nkeys << 16, y = first_ord | status << 16 | fb << 24
enum : uint8_t { ST_OK = 0, ST_FALLBACK = 1 };
enum : uint8_t {
  FB_NONE = 0,
  FB_QUEUE = 1,        // more pending commands than the LDS ring holds
  FB_TABLE = 2,        // more live element instances than the LDS table holds
  FB_RECORDS = 3,      // more records than the per-command record slot holds
  FB_KEYS = 4,         // more than 65 520 keys in one instance
  FB_BATCH_LIMIT = 5,  // follow-up command beyond maxCommandsInBatch (written to the log by the PSM)
  FB_FEEL = 6,         // condition result not a boolean (incident) / value outside the subset
  FB_VARS = 7,         // more variables than the per-instance slots
  FB_SLOT_IN_USE = 8,  // CREATE into an occupied instance slot
  FB_NO_CONDITION = 9, // no flow chosen and no default flow (incident CONDITION_ERROR)
  FB_UNSUPPORTED = 10, // element/transition outside the subset
  FB_DOC = 11,         // multi-entry variable document (agrona iteration order unpinned)
  FB_JOIN = 12,        // taken-sequence-flow counter overflow
  FB_SLOTS = 13,       // more persistent element instances than kSlots
  FB_BAD_PROCESS = 14, // unknown process / no none start event
  FB_MESSAGE = 15,     // message path outside the subset (NUMBER correlation key, second open
                       // subscription, rejected correlation, full correlation slot, outbox overflow)
  FB_FENCED = 16,      // an earlier command of the same subject in this window fell back: the CPU
                       // engine must process this one after it (log order), so it is not run here
  FB_DUPLICATE = 17,   // (device windows) a second command for one subject in one launch
};
// cmd_hdr.y bit 31: the batch ended its process instance (completed; the slot is free)
constexpr uint32_t HDR_ENDED = 1u << 31;
// compact record flags (bits 24..31 of y) of a follow-up command the PSM wrote to the log
// unprocessed (past maxCommandsInBatch, ProcessingStateMachine.java:388-417)
constexpr uint32_t F_UNPROCESSED = 0x80;
// internal command kind: such a follow-up command read back from the log as a batch of its own
// (instance = its instance slot, ref = its process, doc_begin = its queue entry)
constexpr uint8_t CMD_FOLLOWUP = 0x20;

// Program arena (u32 words), LDS-staged by every workgroup:
//   [0] n_procs, [1 .. n_procs] word offset of each process block (multiple of 4)
// process block p:
//   p[0] = n_elements | none_start << 16
//   p[1] = n_join_slots | n_conditions << 16
//   p[2] = out_off, p[3] = cond_off, p[4] = code_off (words, relative to p), p[5] = bpmnProcessId
//   name id | has timer catch events << 16, p[6] = seg_off, p[7] = CREATE template word (TPL_OK |
//   exclusive gateway or 0xFFF; 0 = none)
//   p[8 + 4e .. ] element e: w0 = type | event << 8 | in_count << 16
//                            w1 = out_begin | out_count << 16
//                            w2 = flow: target | condition << 16; xgw: default_flow; task: job_type | retries << 16;
//                                 message catch: name | correlation variable << 16; timer catch / boundary
//                                 event: duration ms; sub-process: none start event | join slots of its
//                                 gateways << 16
//                            w3 = join_slot (job worker: its boundary event or 0xFFFF; boundary event:
//                                 interrupting | repetitions << 8) | container
//                                 (flow scope element; 0 = the process) << 16
//                            multi-instance body: w0 high half = its inputElement's name id (0xFFFF
//                                 none), w2 = inner activity | items << 12 | isSequential << 20, w3 low
//                                 half = the loopCounter name id
//   p[out_off]  u16 outgoing flows (two per word)
//   p[cond_off] u32 first instruction of each condition
//   p[code_off] instructions (16-byte aligned): op, arg, literal_lo, literal_hi
//   p[seg_off]  u32 straight-line segment word per element (kernels.hip fast_command):
//               valid << 31 | from_task << 30 | to_end << 24 | target << 12 | flow, or 0
struct DevState {
  uint4* hdr;        // [n] x = proc | next_ord << 16; y = pi_state | nslots << 8 | nvars << 16 | pi_live << 24
                     //     z = pi_child | pi_asf << 16; w = fence: the window stamp of a fallen-back command
  uint2* slots;      // [kSlots][n] x = elem | key << 16; y = job | state << 16 | flags << 24 (bit0: job row
                     // exists, bit1: its job ACTIVATED, bits 2..7: a multi-instance inner instance's loop
                     // counter).  Containers use the job field for childCount | activeSequenceFlows << 8
                     // (sub-process) or childCount | multiInstanceLoopCounter << 8 (multi-instance body:
                     // childActivatedCount = the loop counter, childCompletedCount = loop - childCount);
                     // an undefined-task inner instance for its loopCounter variable's key ordinal
  uint2* var_meta;   // [kVars][n]  x = name | scope << 16; y = key | type << 16
  long long* var_val;// [kVars][n]
  uint32_t* join;    // [kJoinWords][n]
  uint32_t n;
  // message correlation (allocated when max_correlation_keys > 0)
  uint4* pms;        // [n] PROCESS_SUBSCRIPTION row of the instance's waiting catch event:
                     //     x = elem | state << 12 (0 none, 1 opening, 2 opened) | interrupting << 14 | subpart << 16
                     //     y = eik ord | subscription key ord << 16; z = correlation key id; w = 0
  long long* pms_eik; // [n] real element-instance key of the instance's subscription once its
                      //     PROCESS_MESSAGE_SUBSCRIPTION:CREATE arrived from another partition (-1: none) --
                      //     the MESSAGE_SUBSCRIPTION:DELETE a later window sends carries it
  long long* pms_msg; // [n] the message key of the subscription's record: its last correlation's for a
                      //     non-interrupting one (updateToOpenedState), -1 before (a key reference or real key)
  long long* pi_key; // [n] real process-instance key (written by the device key scan)
  uint2* slot_hdr;   // [S] x = next key ordinal of the correlation slot; y = fence stamp (as hdr.w)
  uint4* sub_a;      // [kSubs][S] MESSAGE_SUBSCRIPTION rows: x = state (0 free, 1 open, 2 correlating)
                     //   | interrupting << 8 | key-in-instance-space << 9 | PI partition << 16;
                     //   y = message name | bpmnProcessId << 16; z = PI instance slot; w = eik ord | key ord << 16
  longlong2* sub_b;  // [kSubs][S] x = element instance key, y = process instance key (real)
  longlong2* sub_k;  // [kSubs][S] x = subscription key, y = message key while correlating (-1 else)
  uint32_t n_slots;
  uint4* tmr;        // [n] the instance's timer (KScope; one per instance): x = catch / boundary element |
                     //     timer key ordinal << 16, y = element-instance ordinal (the catch event's, or the
                     //     activity's a boundary event is attached to) | repetitions << 16 (255 infinite)
                     //     | live << 31, z/w = dueDate lo/hi
  uint4* act;        // [kSlots][n] activations of the instance's jobs (zbhip_activate_jobs; NULL until the
                     //     first): x = job key ordinal | valid << 31, y = worker (value-dictionary id),
                     //     z/w = deadline lo/hi -- the stored job's fields its later records carry
};

// a due timer found by k_due_timers (zbhip_due_timers): its DevState.tmr row, instance slot, process
struct DueTimer {
  uint4 tmr;
  uint32_t inst, proc;
};

// elements without behaviour: ACTIVATING, ACTIVATED, COMPLETE_ELEMENT, COMPLETING, COMPLETED, then
// the outgoing flows (UndefinedTaskProcessor / ManualTaskProcessor, NoneIntermediateThrowEventBehavior)
__host__ __device__ inline bool pass_through(uint32_t type) {
  return type == ZBHIP_EL_TASK || type == ZBHIP_EL_MANUAL_TASK || type == ZBHIP_EL_INTERMEDIATE_THROW_EVENT;
}

struct StepParams {
  const uint4* cmds;          // zbhip_command[n_cmds] (window, log order)
  const uint32_t* order;      // command indices processed by this launch (round); null = identity
  uint32_t n_launch;          // lanes in this launch
  const zbhip_doc_entry* docs;
  uint32_t n_docs;
  const uint32_t* prog;
  uint32_t prog_words;
  uint32_t n_procs;
  DevState st;
  uint32_t rec_cap;           // max records per batch
  uint32_t region_stride;     // records from one output region to the next (>= B * rec_cap)
  uint2* out;                 // workgroup regions: region g holds its block's records contiguously
  uint32_t region_base;       // region of this launch's workgroup 0
  uint32_t* region_total;     // [regions] records in each region (bit 31: holds rows j >= R)
  uint16_t* region_lanes;     // [regions][B] record counts of the lanes of a region with rows j >= R
  uint2* cmd_hdr;             // [n_cmds]
  unsigned long long* stats;  // [64][8] spread accumulators: records, transitions, completed, keys,
                              // fallback, commands
  int32_t max_cmds_in_batch;
  // message correlation (KMsg)
  const zbhip_xpart_cmd* xparts;
  uint32_t n_xparts;
  const uint32_t* str_hash;   // [n_strs] Java hashCode of each value-dictionary string
  uint32_t n_strs;
  uint4* cmd_hdr2;            // [n_cmds] x = secondary instance, y = first ord | nkeys << 16 (secondary
                              // space), z = outbox entries, w = payload rows
  zbhip_xpart_cmd* xout;      // [kOut][xcap]: entry j of command c at j * xcap + c (entry 0 of
                              // consecutive commands contiguous: coalesced writes and reads)
  uint32_t xcap;              // the outbox's command capacity (config.max_commands)
  int32_t partition_id, partition_count;
  uint32_t stamp;             // window stamp: hdr.w / slot_hdr.y of a subject whose command fell back
  uint32_t cmd_base;          // window index of cmds[0] (continuation launches of follow-up batches)
  // batch FIFO entries beyond the LDS ring (large fan-outs): per resident lane, qspill_cap entries
  // strided by gridDim.x * B
  uint32_t* qspill;
  uint32_t qspill_cap;
  // follow-up commands past maxCommandsInBatch: {window index, queue entry, record ordinal |
  // process << 16, instance slot}
  uint4* ovf;
  uint32_t* ovf_count;
  uint32_t ovf_cap;
  // CREATE batch templates [n_procs][kTplVar][kTplWords] (null: off) and this launch's sequence
  // number (a template recorded in the running launch is not used before the next one)
  uint2* tpl;
  uint32_t launch_seq;
  uint32_t no_fast_scope;     // ZBHIP_NO_FAST_SCOPE: KScope's straight-line JOB:COMPLETE batches off (A/B)
  long long now_ms;           // zbhip_set_clock: ActorClock.currentTimeMillis() of this window
  long long* cmd_due;         // [n_cmds] (KScope) dueDate of the timer a batch canceled (at most one)
  long long* map_val;         // [kMapVals][map_cap] (KScope) values of the variables a batch's io mappings
                              // wrote: value j of window command c at j * map_cap + c (C_VAR_MAPPED)
  uint32_t map_cap;
  uint4* cmd_act;             // [n_cmds] the ACTIVATED job a batch completed or canceled: its DevState.act
                              // entry (x bit 31 clear: none found)
  const uint32_t* guard;      // an untrusted device window's subject-check word (k_subject_check): stamp << 2 |
                              // flags; flags of this window's stamp -> the launch does nothing (the host
                              // replans the window); null: no guard
  uint32_t guard_stamp;       // the window's check stamp
  uint32_t* guard_host;       // host-mapped: the verdict, stamp << 2 | flags (block 0 writes it)
  // the list dictionary (ZBHIP_DOC_LIST values): per list its first item and count, the items' values
  // and zbhip_doc_types
  const uint2* list_hdr;
  const long long* list_val;
  const uint8_t* list_type;
  uint32_t n_lists;
};
constexpr int kMapVals = 2;   // io-mapped VARIABLE records per batch (more: FB_VARS)
// a variable holding a propagated multi-instance outputCollection: its items on the host
// (zbhip_handle::outlist_var, by the variable's key); never a document entry's type
constexpr uint8_t kDocOutList = 7;

// ---- log bytes on the device (logdev.hip) ----
// entry templates of the device log writer (logwriter.cpp log_device_templates): PROCESS_INSTANCE
// intents 1..10 (commands unprocessed), 10..12 the commands processed in their batch, 13 JOB:CREATED,
// 14 / 15 PROCESS_EVENT TRIGGERING / TRIGGERED, 16 PROCESS_INSTANCE_CREATION:CREATED, 17
// JOB:COMPLETED (the last four without a document)
constexpr uint32_t kLogTplKinds = 18;

struct LogCmd {
  unsigned long long rec_off;  // first gathered row of the command
  unsigned long long out_rec;  // log-order index of its first record in the window
  unsigned long long key0;     // key counter of its first new key: key = pbits + key0 + (ord - first_ord)
  long long src_pos;           // sourcePosition of its records
  uint32_t instance;
  uint32_t prev;               // previous command of the same instance in the window, or ~0
  uint16_t first_ord, nkeys, nrec, doc_count;
  uint32_t doc_begin;
  uint32_t pad;                // the command's pad (TIMER:TRIGGER: dueDate high word)
};
// the keys older than its own batch that a command's records name, found by the size pass for the
// write pass: the process instance's (ordinal 0) and the last three others it looked up
struct LogKeys {
  long long pik, k0, k1, k2;
  uint32_t o0, o1, o2, pad;    // ordinals of k0 / k1 / k2 (NONE: empty)
};
struct LogLaunch {
  int phase;                   // 0 sizes + offsets, 1 write, 2 key ring, 3 command table
  const uint2* rows;
  const LogCmd* cmds;
  uint32_t n;
  const uint8_t* arena;
  const uint32_t* idx;
  uint32_t arena_words, idx_words;
  const zbhip_doc_entry* docs;
  uint32_t n_docs;
  const uint16_t* inst_proc;
  unsigned long long* ring;
  unsigned long long* kpi;
  uint32_t n_inst;
  long long pbits;
  long long first_position, timestamp;
  int32_t broker[3];
  unsigned long long* bytes;   // [n + 1]
  unsigned long long* block_sums;
  uint64_t* out;
  uint32_t* flag;
  long long now_ms;            // the run's clock (TIMER:CREATED dueDates)
  const long long* cmd_due;    // [n] dueDate of the timer each batch canceled (KScope)
  // phase 3: the command table built on the device (a one-round window gathered in log order)
  const uint2* hdr;            // [n] per-command headers of the run (nrec | nkeys << 16, first_ord)
  const zbhip_command* wcmds;  // [n] the window's commands
  const long long* src_pos;    // [n] sourcePosition of each command (NULL: -1)
  unsigned long long key_base; // key counter before the window's first key
  LogCmd* table;               // [n] out
  unsigned long long* table_sums;  // scan blocks + 1
  uint16_t* inst_proc_w;       // the window's CREATEs set their slot's process here
  const uint8_t* tpl;          // entry templates (16-aligned)
  const uint4* tpl_desc;       // per template: offset, size | pik offset + 1 << 16, scope offset + 1
  const uint32_t* tpl_idx;     // [0] n procs, [1 + p] base of process p's [element][kLogTplKinds] ids + 1
  uint32_t* rinfo;             // [rows] per record: its template or composed, and its entry bytes
  int compose;                 // phase 1: entries without a template exist (the size pass's flag bit 1);
                               // 2: k_log_compose only (the write ran speculatively)
  unsigned long long out_cap;  // phase 1: bytes at `out` (0: unchecked); k_log_write does nothing when the
                               // window's total (bytes[n], from the scan) exceeds it
  LogKeys* wkeys;              // [n] (phase 0 writes, phase 1 reads)
  uint4* jrn;                  // phase 3: [n] the window's key bookkeeping journal (NULL: the host books it)
  const uint4* cmd_act;        // [n] StepParams.cmd_act (NULL: no job was ever activated)
  const uint8_t* strs;         // the value dictionary on the device (activated jobs' workers)
  const unsigned long long* str_off;
  uint32_t n_strs;
  uint32_t tpl_lds;            // bytes of the templates and their descriptors (the `tpl` block up to tpl_idx)
};

}  // namespace zb
