// gfx950 kernels of the BPMN element-lifecycle batch executor.
//
// k_step: one lane owns one command of the window (CREATE / JOB:COMPLETE) and runs that
// command's whole batch -- the ProcessingStateMachine follow-up FIFO
// (stream-platform/.../stream/impl/ProcessingStateMachine.java:328-417) -- over the
// instance it addresses.  Instances are independent inside a partition, so a lane never
// shares state with another lane (the host serialises commands of one instance into
// rounds): the join counters, the element-instance table and the variables of an instance
// are private to its lane, read once from HBM at batch start (coalesced SoA rows) and
// written back once at the end.  Transient element instances (start events, gateways, end
// events) live only in the lane's LDS table and never touch HBM.  The deployed processes'
// CSR transition tables are staged in LDS by every workgroup.
//
// Element processors and appliers restated here (paths relative to
// engine/src/main/java/io/camunda/zeebe/engine/):
//   processing/bpmn/BpmnStreamProcessor.java:74-162, ProcessInstanceStateTransitionGuard.java:47-186,
//   processing/bpmn/behavior/BpmnStateTransitionBehavior.java:72-417,
//   processing/bpmn/container/ProcessProcessor.java:55-140, event/StartEventProcessor.java:45-67,
//   event/EndEventProcessor.java:110-134, task/JobWorkerTaskProcessor.java:49-75,
//   gateway/ExclusiveGatewayProcessor.java:47-126, gateway/ParallelGatewayProcessor.java:34-50,
//   processing/processinstance/CreateProcessInstanceProcessor.java:129-158,
//   processing/job/JobCompleteProcessor.java:47-92, processing/common/EventTriggerBehavior.java:148-166,
//   processing/variable/VariableBehavior.java:60-200,
//   state/appliers/ProcessInstanceElement{Activating,Activated,Completing,Completed}Applier.java,
//   state/appliers/ProcessInstanceSequenceFlowTakenApplier.java:32-69, JobCreatedApplier.java:28-41,
//   JobCompletedApplier.java:28-45, state/instance/DbElementInstanceState.java:135-344.
//
// k_scan_regions / k_gather (drain path only): exclusive scan of the per-chunk record totals and
// an ordered copy of every chunk's records into one contiguous append buffer.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "zb_internal.h"

namespace zb {

// ---------------------------------------------------------------------------------------------
// per-lane batch context
// ---------------------------------------------------------------------------------------------
// Kernel configuration: workgroup size B, LDS element-instance table entries T, LDS queue
// entries Q, records staged in LDS per lane R (rows j >= R are written straight into the chunk's
// output region, above its packed run, and interleaved into order by the drain gather).
// After the chunk's wavefront scan an owner map in LDS lets the workgroup store the chunk's
// records contiguously with coalesced 16-byte writes.  (Measured alternatives, linear-10: every
// lane storing its own records at its prefix scatters each store over ~40 cache lines; a
// binary search of the lane prefix per record was slower still; B = 64 / 256 and R = 8 / 32
// were 2-10 % slower; for the single-wave KLinear, compacting through registers (each lane reads
// its column, then writes it at its prefix) spilled and was ~2 % slower, and an owner map of stage
// indices (one dependent LDS level fewer) ~4 % slower.)
template <int B_, int T_, int Q_, int R_, bool M_ = false, bool J_ = true, bool X_ = true, int W_ = 0,
          bool REG_ = false, bool S_ = false, bool IO_ = false>
struct KCfg {
  static constexpr int B = B_, T = T_, Q = Q_, R = R_;
  static constexpr int W = W_;   // waves per SIMD the register allocation targets (0 = compiler default)
  static constexpr bool REG = REG_;  // element table and FIFO in registers (T == Q == 2), not LDS
  static constexpr bool M = M_;  // message correlation (catch events, subscription commands)
  static constexpr bool J = J_;  // parallel-gateway join counters
  static constexpr bool X = X_;  // exclusive gateways (FEEL condition evaluation)
  static constexpr bool S = S_;  // flow scopes below the process (embedded sub-processes)
  static constexpr bool IO = IO_;  // io mappings: variables in the scopes of element instances (K::S only)
};
// One token per instance (exclusive gateways, no parallel gateways / multi-outgoing nodes: no join
// counters).  Only R = 4 stage rows: rows j >= R go straight to the output region (one coalesced
// wave store per row), so LDS no longer limits residency (5 KiB per workgroup) and the register
// file does (3 waves per SIMD).  Measured on config 3 (exclusive gateway, 26-record CREATE
// batches): R = 28 (the whole batch in LDS, 9 workgroups per CU) 1.57, R = 8 2.11, R = 4
// 2.22 x 10^11 transitions/s.
#ifndef ZB_KSIMPLE_B
#define ZB_KSIMPLE_B 64
#define ZB_KSIMPLE_R 4
#endif
#ifndef ZB_KSIMPLE_W
#define ZB_KSIMPLE_W 3  // 168 VGPRs, no spill: the register allocator is held to 3 waves per SIMD
#endif
using KSimple = KCfg<ZB_KSIMPLE_B, 4, 4, ZB_KSIMPLE_R, false, false, true, ZB_KSIMPLE_W>;
// Linear chains (every node <= 1 outgoing flow, no gateways, no catch events): at most two element
// instances are alive in a batch, no FEEL evaluator, no join counters.  T = 2 and R = 15 keep the
// workgroup at <= 20 KiB of LDS and the register target at 128 VGPRs, so 4 waves per SIMD are
// resident (KSimple: 3).  The FIFO never holds more than one entry there and the table two, so both
// live in registers: the batch logic issues no dependent LDS round trips, only the record stage.
// R = 15 holds every straight-line segment's fixed record sequence (fast_command's static rows).
#ifndef ZB_KLINEAR_W
#define ZB_KLINEAR_W 4
#endif
using KLinear = KCfg<64, 2, 2, 15, false, false, false, ZB_KLINEAR_W, true>;
// Everything else in the subset (parallel gateways: join counters).  R = 4 as for KSimple: config
// 4 (fork/join 8, ~60-record CREATE batches) R = 16 1.44, R = 8 1.63, R = 4 1.93 x 10^11.
#ifndef ZB_KGENERIC_B
#define ZB_KGENERIC_B 128
#define ZB_KGENERIC_R 4
#endif
#ifndef ZB_KGENERIC_W
#define ZB_KGENERIC_W 3
#endif
using KGeneric = KCfg<ZB_KGENERIC_B, 12, 16, ZB_KGENERIC_R, false, true, true, ZB_KGENERIC_W>;
#ifndef ZB_KMSG_R
#define ZB_KMSG_R 4
#endif
#ifndef ZB_KMSG_W
#define ZB_KMSG_W 2  // 256 VGPRs, no AGPR or scratch spill: 2 waves per SIMD (compiler default: 260 -> 1)
#endif
using KMsg = KCfg<128, 12, 16, ZB_KMSG_R, true, true, true, ZB_KMSG_W>;  // message catch events (config 5)
// Embedded sub-processes: KGeneric plus flow scopes (a sub-process instance is an element-table
// entry whose job field counts its children and active sequence flows)
#ifndef ZB_KSCOPE_W
#define ZB_KSCOPE_W ZB_KGENERIC_W
#endif
using KScope = KCfg<ZB_KGENERIC_B, 12, 16, ZB_KGENERIC_R, false, true, true, ZB_KSCOPE_W, false, true>;
// KScope plus zeebe:ioMapping (element-instance variable scopes, their lookups through the scope chain
// and removal with the instance): a variant of its own so processes without mappings keep KScope's
// register allocation
using KScopeIO = KCfg<ZB_KGENERIC_B, 12, 16, ZB_KGENERIC_R, false, true, true, ZB_KSCOPE_W, false, true, true>;

template <class K>
struct Lane {
  const uint32_t* pb;   // process block (LDS)
  uint2* tbl;           // LDS table base (entry t at tbl[t * K::B])
  uint32_t* q;          // LDS queue base (entry i at q[(i % K::Q) * K::B])
  uint2* stage;         // LDS record rows of this lane: record j < R at stage[j * K::B]
  uint2* rec;           // rows j >= R of this command: rec[j * B] (its chunk's output region)
  uint32_t rec_cap;
  uint32_t nrec;
  uint32_t fail;
  uint32_t transitions;
  uint32_t completed;
  int limit;
  int processed;
  int qh, qt;          // LDS ring (register pair for K::REG)
  uint32_t g;           // the lane's global FIFO behind the ring (entries beyond K::Q pending):
                        // head | tail << 16, entries in StepParams.qspill
  uint32_t ci;          // window index of the command (overflow entries, outbox, key references)
  int nt;               // table high-water mark
  uint16_t proc;
  uint16_t next_ord;
  uint16_t first_ord;
  uint16_t trig_key;    // event trigger of a completed job (EVENT_TRIGGER row), NONE if none
  uint16_t trig_evt;    // K::S: the PROCESS_EVENT key ordinal of a boundary event's trigger on trig_key
  uint32_t inc;         // the incident info of a failed exclusive gateway (find_sequence_flow)
  uint32_t n_map;       // K::S: io-mapped VARIABLE records of the batch so far (values in StepParams.map_val)
  // K::S: the value a job's document gave a multi-instance inner instance's local outputElement
  // variable in this batch (mergeDocument updated it locally): set, zbhip_doc_type, value
  uint8_t mo_set, mo_type;
  uint16_t done_job;  // the job of the last JOB:COMPLETE (its key ordinal)
  long long mo_val;
  bool pi_live;
  uint8_t pi_state;
  int pi_child;
  int pi_asf;
  uint32_t doc_begin;
  uint32_t doc_count;
  const zbhip_doc_entry* docs;
  int nvars;
  // variables and join counters are explicit scalars (not arrays): an array member indexed at
  // run time would force the whole context into scratch memory
  uint32_t vx0, vx1, vx2, vx3;  // name | scope << 16
  uint32_t vy0, vy1, vy2, vy3;  // key | type << 16
  long long vv0, vv1, vv2, vv3;
  uint32_t jw0, jw1, jw2, jw3;
  bool has_join;
  uint2 r_t0, r_t1;         // K::REG: element table entries
  uint32_t r_q0, r_q1;      // K::REG: FIFO entries
  // ---- message correlation (K::M only) ----
  uint32_t inst;            // instance whose rows are loaded (kNoInst: none, a slot lane before a
                            // local PROCESS_MESSAGE_SUBSCRIPTION command)
  uint32_t pm_x, pm_y, pm_z;// PROCESS_SUBSCRIPTION row of the loaded instance: element | state << 12
                            // (1 opening, 2 opened, 3 closing) | interrupting << 14 | partition << 16;
                            // element-instance ordinal | key ordinal << 16; correlation key
  uint32_t pm_w;            // its message name | bpmnProcessId << 16
  long long pm_msg;         // the message key the (non-interrupting) subscription's record holds: its
                            // last correlation's (updateToOpenedState), -1 before one (DevState.pms_msg)
  long long pik;            // real process-instance key of the loaded instance, or a reference
  bool slot_lane;           // primary subject is the correlation slot `slot`
  uint32_t slot;
  uint16_t s_next_ord;      // correlation-slot key space
  uint16_t i_first_ord;     // first instance-space ordinal of this batch
  uint32_t n_out, n_pay;
  uint32_t x_sum;           // sends: count (bits 0..3) | their target if one (8..23) | mixed (31)
  // pending local commands (SubscriptionCommandSender follow-ups on this partition)
  uint32_t lq_slot;         // correlation slot of a local MESSAGE_SUBSCRIPTION command
  uint32_t lq_row;          // slot row of a local PROCESS_MESSAGE_SUBSCRIPTION:CORRELATE
  long long lq_msg;         // its message key (reference)
  uint32_t lq_name_bpmn;    // message name | bpmnProcessId << 16 of the pending command
  uint32_t lq_corr;         // correlation key of the pending command
  uint32_t lq_intr;         // interrupting flag of the pending command's subscription
  long long lq_eik, lq_pik; // element / process instance keys of the pending command (references)
  uint32_t lq_eord;         // routing handle ordinal of the pending command
  // deferred correlation-slot row operations, applied at commit
  bool op_ins;              // insert a row into slot op_slot
  uint32_t op_slot;
  uint4 ins_a;
  long long ins_eik, ins_pik;
  uint32_t op_corr_mask, op_rm_mask, op_rm_slot;
  uint32_t op_open_mask, op_open_slot;  // non-interrupting rows correlated: open again (state 1)
  long long op_corr_msg, ins_key;
  const StepParams* sp;
  const uint32_t* prog;     // LDS program arena (mid-batch instance loads)
  uint16_t s_first_ord;
  // ---- the instance's timer (K::S, processes with timer catch events; DevState.tmr) ----
  bool has_tmr;
  uint32_t tm_x, tm_y;      // catch element | timer ordinal << 16; element-instance ordinal | live << 31
  long long tm_due;
};
constexpr uint32_t kNoInst = 0xFFFFFFFFu;
static_assert(kVars == 4 && kJoinWords == 4, "scalarised tables");

template <class K>
__device__ __forceinline__ uint32_t var_x(const Lane<K>& L, int i) {
  return i == 0 ? L.vx0 : i == 1 ? L.vx1 : i == 2 ? L.vx2 : L.vx3;
}
template <class K>
__device__ __forceinline__ uint32_t var_y(const Lane<K>& L, int i) {
  return i == 0 ? L.vy0 : i == 1 ? L.vy1 : i == 2 ? L.vy2 : L.vy3;
}
template <class K>
__device__ __forceinline__ long long var_v(const Lane<K>& L, int i) {
  const long long v0 = L.vv0, v1 = L.vv1, v2 = L.vv2, v3 = L.vv3;
  long long r = v3;
  r = i == 2 ? v2 : r;
  r = i == 1 ? v1 : r;
  r = i == 0 ? v0 : r;
  return r;
}
// branch-free updates: a store per field keeps every field a plain SSA value (an if/else chain
// is merged by the optimiser into one store through a selected pointer -> scratch)
template <class K>
__device__ __forceinline__ void var_put(Lane<K>& L, int i, uint32_t x, uint32_t y, long long v) {
  L.vx0 = i == 0 ? x : L.vx0; L.vy0 = i == 0 ? y : L.vy0; L.vv0 = i == 0 ? v : L.vv0;
  L.vx1 = i == 1 ? x : L.vx1; L.vy1 = i == 1 ? y : L.vy1; L.vv1 = i == 1 ? v : L.vv1;
  L.vx2 = i == 2 ? x : L.vx2; L.vy2 = i == 2 ? y : L.vy2; L.vv2 = i == 2 ? v : L.vv2;
  L.vx3 = i == 3 ? x : L.vx3; L.vy3 = i == 3 ? y : L.vy3; L.vv3 = i == 3 ? v : L.vv3;
}
template <class K>
__device__ __forceinline__ uint32_t jw_get(const Lane<K>& L, int i) {
  return i == 0 ? L.jw0 : i == 1 ? L.jw1 : i == 2 ? L.jw2 : L.jw3;
}
template <class K>
__device__ __forceinline__ void jw_put(Lane<K>& L, int i, uint32_t w) {
  L.jw0 = i == 0 ? w : L.jw0;
  L.jw1 = i == 1 ? w : L.jw1;
  L.jw2 = i == 2 ? w : L.jw2;
  L.jw3 = i == 3 ? w : L.jw3;
}

template <class K>
__device__ __forceinline__ void set_fail(Lane<K>& L, uint32_t why) {
  if (!L.fail) L.fail = why;
}

// an ACTIVATED job's record (JOB:COMPLETED / CANCELED: the stored job): its activation entry into the
// batch's cmd_act word for the drain and the device log writer (none found: the writer declines)
template <class K>
__device__ __forceinline__ void note_activation(const Lane<K>& L, uint32_t job_ord, uint32_t inst);

template <class K>
__device__ __forceinline__ uint4 elem_of(const Lane<K>& L, uint32_t e) {
  return reinterpret_cast<const uint4*>(L.pb + 8)[e];
}
__device__ __forceinline__ uint32_t etype(uint4 w) { return w.x & 0xFF; }
template <class K>
__device__ __forceinline__ uint32_t out_flow(const Lane<K>& L, uint32_t i) {
  return reinterpret_cast<const uint16_t*>(L.pb + L.pb[2])[i];
}

template <class K>
__device__ __forceinline__ uint16_t new_key(Lane<K>& L) {
  if (L.next_ord >= 0xFFF0) set_fail(L, FB_KEYS);
  return L.next_ord++;
}

template <class K>
__device__ __forceinline__ void emit(Lane<K>& L, uint32_t code, uint32_t key, uint32_t aux, uint32_t elem,
                                     uint32_t flags = 0) {
#ifdef ZB_EXP_NOEMIT  // diagnostic build: records counted, never staged
  ++L.nrec;
  if (code >= ZBHIP_PI_SEQUENCE_FLOW_TAKEN && code <= ZBHIP_PI_ELEMENT_TERMINATED) ++L.transitions;
  return;
#endif
  if (L.nrec < L.rec_cap) {
    const uint2 r = make_uint2((key & 0xFFFF) | (aux << 16), (elem & 0xFFFF) | (code << 16) | (flags << 24));
    if (L.nrec < (uint32_t)K::R) L.stage[L.nrec * K::B] = r;
    else L.rec[(size_t)L.nrec * K::B] = r;
  } else {
    set_fail(L, FB_RECORDS);
  }
  ++L.nrec;
  if (code >= ZBHIP_PI_SEQUENCE_FLOW_TAKEN && code <= ZBHIP_PI_ELEMENT_TERMINATED) ++L.transitions;
}

// ---- message records: a header row and kPayloadRows payload rows ---------------------------
template <class K>
__device__ __forceinline__ void emit_row(Lane<K>& L, uint2 r) {
  if (L.nrec < L.rec_cap) {
    if (L.nrec < (uint32_t)K::R) L.stage[L.nrec * K::B] = r;
    else L.rec[(size_t)L.nrec * K::B] = r;
  } else {
    set_fail(L, FB_RECORDS);
  }
  ++L.nrec;
}
__device__ __forceinline__ uint2 split64(long long v) {
  return make_uint2((uint32_t)((unsigned long long)v & 0xFFFFFFFFu), (uint32_t)((unsigned long long)v >> 32));
}
// Record values of MESSAGE / MESSAGE_SUBSCRIPTION / PROCESS_MESSAGE_SUBSCRIPTION records
// (protocol-impl/.../value/message/*Record.java): keys as references, resolved on drain.
template <class K>
__device__ __forceinline__ void emit_msg(Lane<K>& L, uint32_t code, long long key, long long eik, long long pik,
                                         long long msg, uint32_t corr, uint32_t name_bpmn, uint32_t part,
                                         uint32_t intr, uint32_t elem, uint32_t flags = 0) {
  emit_row(L, make_uint2(0xFFFFFFFFu, (elem & 0xFFF) | kPayloadBit | (code << 16) | (flags << 24)));
  emit_row(L, make_uint2(corr, name_bpmn));
  emit_row(L, split64(key));
  emit_row(L, split64(eik));
  emit_row(L, split64(pik));
  emit_row(L, split64(msg));
  emit_row(L, make_uint2(part | (intr << 16), 0));
  L.n_pay += kPayloadRows;
}
// key references (zb_internal.h): a subject's ordinal (resolved by the host drain through the
// subject's key history) or a key of window command ci (resolved by the device key scan)
__device__ __forceinline__ long long ref_subj(bool is_slot, uint32_t subject, uint32_t ord) {
  return -2 - (long long)((1ull << 62) | ((unsigned long long)is_slot << 61) | ((unsigned long long)subject << 16) | ord);
}
__device__ __forceinline__ long long ref_cmd(uint32_t ci, bool sec, uint32_t ord) {
  return -2 - (long long)(((unsigned long long)ci << 17) | ((unsigned long long)sec << 16) | ord);
}

// element table / FIFO storage: LDS columns, or registers for K::REG (branch-free selects keep
// every field a plain SSA value, as for the variables)
template <class K>
__device__ __forceinline__ uint2 tget(const Lane<K>& L, int t) {
  if constexpr (K::REG) {
    static_assert(K::T == 2 && K::Q == 2, "register table / FIFO");
    return t == 0 ? L.r_t0 : L.r_t1;
  } else {
    return L.tbl[t * K::B];
  }
}
template <class K>
__device__ __forceinline__ void tput(Lane<K>& L, int t, uint2 v) {
  if constexpr (K::REG) {
    L.r_t0.x = t == 0 ? v.x : L.r_t0.x; L.r_t0.y = t == 0 ? v.y : L.r_t0.y;
    L.r_t1.x = t == 1 ? v.x : L.r_t1.x; L.r_t1.y = t == 1 ? v.y : L.r_t1.y;
  } else {
    L.tbl[t * K::B] = v;
  }
}
template <class K>
__device__ __forceinline__ uint32_t qget(const Lane<K>& L, int i) {
  if constexpr (K::REG) return (i & 1) ? L.r_q1 : L.r_q0;
  else return L.q[(i % K::Q) * K::B];
}
template <class K>
__device__ __forceinline__ void qput(Lane<K>& L, int i, uint32_t v) {
  if constexpr (K::REG) {
    L.r_q0 = (i & 1) ? L.r_q0 : v;
    L.r_q1 = (i & 1) ? v : L.r_q1;
  } else {
    L.q[(i % K::Q) * K::B] = v;
  }
}

// queue entry: elem (12) | complete (1) << 12 | fs_is_pi (1) << 13 | (K::M local command; K::S with
// Q_TERM: PROCESS_INSTANCE_BATCH:TERMINATE) << 14 | terminate (K::S TERMINATE_ELEMENT) << 15 | key << 16
constexpr uint32_t Q_TERM = 1u << 15;
constexpr uint32_t Q_PIBT = 1u << 14;
__device__ __forceinline__ uint32_t qentry(uint32_t elem, bool complete, bool fs_pi, uint32_t key) {
  return elem | (complete ? 1u << 12 : 0u) | (fs_pi ? 1u << 13 : 0u) | (key << 16);
}
template <class K>
__device__ __forceinline__ int pending(const Lane<K>& L) {
  return (L.qt - L.qh) + (int)((L.g >> 16) - (L.g & 0xFFFF));
}
// entry i of the lane's global FIFO (resident lanes of the grid are interleaved: coalesced rows)
__device__ __forceinline__ uint32_t* spill_at(const StepParams& P, uint32_t i) {
  return P.qspill + ((size_t)(i % P.qspill_cap) * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
}
// the batch FIFO: the oldest K::Q pending entries in the LDS ring, newer ones (a large fan-out,
// e.g. a fork with more branches than K::Q) in the lane's global FIFO, moved into the ring as it drains
template <class K>
__device__ __forceinline__ void enqueue(Lane<K>& L, uint32_t entry) {
  const uint32_t gh = L.g & 0xFFFF, gt = L.g >> 16;
  if (L.qt - L.qh < K::Q && gt == gh) {
    qput(L, L.qt, entry);
    ++L.qt;
    return;
  }
  if constexpr (K::REG) {
    set_fail(L, FB_QUEUE);
  } else {
    if (gt - gh >= L.sp->qspill_cap || gt >= 0xFFFF) { set_fail(L, FB_QUEUE); return; }
    *spill_at(*L.sp, gt) = entry;
    L.g += 1u << 16;
  }
}
template <class K>
__device__ __forceinline__ uint32_t dequeue(Lane<K>& L) {
  const uint32_t entry = qget(L, L.qh);
  ++L.qh;
  if constexpr (!K::REG) {
    const uint32_t gh = L.g & 0xFFFF;
    if ((L.g >> 16) > gh) {
      qput(L, L.qt, *spill_at(*L.sp, gh));
      ++L.qt;
      ++L.g;
    }
  }
  return entry;
}

// ProcessingStateMachine.collectBatchProcessingStepResult (:388-417): a follow-up command is
// processed in this batch only while pending + processed + 1 + admitted < maxCommandsInBatch;
// otherwise the platform writes it to the log unprocessed and processes it later as a batch of its
// own (after the window's commands, in the order written): the record is flagged and the command
// kept in the overflow list for the runtime's continuation launches.
template <class K>
__device__ __forceinline__ void overflow(Lane<K>& L, uint32_t entry) {
  const StepParams& P = *L.sp;
  if (!P.ovf) { set_fail(L, FB_BATCH_LIMIT); return; }
  const uint32_t slot = atomicAdd(P.ovf_count, 1u);
  if (slot >= P.ovf_cap) { set_fail(L, FB_BATCH_LIMIT); return; }
  // {window index, queue entry, record ordinal | process << 16, instance slot}
  P.ovf[slot] = make_uint4(L.ci, entry, (L.nrec - 1) | ((uint32_t)L.proc << 16), P.cmds[L.ci - P.cmd_base].x);
}

// a follow-up command of the batch: its COMMAND record, then the FIFO (or the overflow list)
template <class K>
__device__ __forceinline__ void follow_up(Lane<K>& L, uint32_t code, uint32_t key, uint32_t aux, uint32_t elem,
                                          bool complete, bool fs_pi, uint32_t qkey, uint32_t qflags = 0,
                                          uint32_t rflags = 0) {
  const bool admit = pending(L) + L.processed + 1 < L.limit;
  emit(L, code, key, aux, elem, (admit ? 0u : F_UNPROCESSED) | rflags);
  const uint32_t entry = qentry(elem, complete, fs_pi, qkey) | qflags;
  if (admit) enqueue(L, entry);
  else overflow(L, entry);
}

// local subscription commands (SubscriptionCommandSender.handleFollowUpCommandBasedOnPartition,
// :304-320: receiver == this partition -> follow-up command of the batch): bit 14 + kind
enum : uint32_t { LQ_BIT = 1u << 14, LQ_MS_CREATE = 1, LQ_PMS_CREATE = 2, LQ_PMS_CORRELATE = 3, LQ_MS_CORRELATE = 4,
                  LQ_MS_DELETE = 5, LQ_PMS_DELETE = 6 };
template <class K>
__device__ __forceinline__ void push_local(Lane<K>& L, uint32_t kind) {
  // past the batch limit a local subscription command would need its pending context written to
  // the log: outside the device subset
  if (pending(L) + L.processed + 1 >= L.limit) { set_fail(L, FB_BATCH_LIMIT); return; }
  enqueue(L, LQ_BIT | kind);
}

// ---- element-instance table (LDS) ----------------------------------------------------------
template <class K>
__device__ __forceinline__ int tbl_find(const Lane<K>& L, uint32_t key) {
  for (int t = 0; t < L.nt; ++t) {
    uint2 e = tget(L, t);
    if (e.x != 0xFFFFFFFFu && (e.x >> 16) == key) return t;
  }
  return -1;
}
template <class K>
__device__ __forceinline__ int tbl_find_job(const Lane<K>& L, uint32_t job) {
  for (int t = 0; t < L.nt; ++t) {
    uint2 e = tget(L, t);
    if (e.x != 0xFFFFFFFFu && (e.y & 0xFFFF) == job && (e.y >> 24) & 1u) return t;
  }
  return -1;
}
template <class K>
__device__ __forceinline__ int tbl_insert(Lane<K>& L, uint32_t elem, uint32_t key, uint32_t state) {
  int t = 0;
  for (; t < L.nt; ++t)
    if (tget(L, t).x == 0xFFFFFFFFu) break;
  if (t == L.nt) {
    if (L.nt >= K::T) { set_fail(L, FB_TABLE); return -1; }
    ++L.nt;
  }
  tput(L, t, make_uint2(elem | (key << 16), JOB_ZERO | (state << 16)));
  return t;
}
template <class K>
__device__ __forceinline__ void tbl_set_state(Lane<K>& L, int t, uint32_t state) {
  uint2 e = tget(L, t);
  e.y = (e.y & 0xFF00FFFFu) | (state << 16);
  tput(L, t, e);
}

// ---- flow scopes (K::S: embedded sub-processes) ----------------------------------------------
// An element's container is the high half of its word 3 (0: the process).  A sub-process instance
// is an element-table entry like any other (one active instance per sub-process element; a second
// concurrent one falls back) whose job field holds childCount | activeSequenceFlows << 8
// (ElementInstance.java:23-54); the process scope keeps its counters in pi_child / pi_asf.
template <class K>
__device__ __forceinline__ uint32_t scope_of(uint4 w) {
  if constexpr (K::S) return w.w >> 16;
  else return 0;
}
template <class K>
__device__ __forceinline__ int scope_find(const Lane<K>& L, uint32_t c) {
  for (int t = 0; t < L.nt; ++t) {
    const uint2 e = tget(L, t);
    if (e.x != 0xFFFFFFFFu && (e.x & 0xFFFF) == c) return t;
  }
  return -1;
}
// key ordinal of the flow scope instance of container c (the process instance: ordinal 0)
template <class K>
__device__ __forceinline__ uint32_t scope_key(Lane<K>& L, uint32_t c) {
  if (c == 0) return 0;
  const int t = scope_find(L, c);
  if (t < 0) { set_fail(L, FB_UNSUPPORTED); return 0; }
  return tget(L, t).x >> 16;
}
// childCount += dc, activeSequenceFlows += da; decrements clamp at 0 (ElementInstance.java:203-213)
template <class K>
__device__ __forceinline__ void scope_adjust(Lane<K>& L, uint32_t c, int dc, int da) {
  if (c == 0) {
    L.pi_child += dc;
    L.pi_asf = L.pi_asf + da < 0 ? 0 : L.pi_asf + da;
    return;
  }
  const int t = scope_find(L, c);
  if (t < 0) { set_fail(L, FB_UNSUPPORTED); return; }
  uint2 e = tget(L, t);
  const int child = (int)(e.y & 0xFF) + dc;
  // a multi-instance body's second byte is its loop counter: its inner instances take no sequence
  // flows, so its activeSequenceFlows stays 0 (the activation's decrement clamps at 0)
  const bool mi = etype(elem_of(L, c)) == ZBHIP_EL_MULTI_INSTANCE_BODY;
  int asf = mi ? (int)((e.y >> 8) & 0xFF) : (int)((e.y >> 8) & 0xFF) + da;
  if (asf < 0) asf = 0;
  if (child < 0 || child > 255 || asf > 255) { set_fail(L, FB_TABLE); return; }
  e.y = (e.y & 0xFFFF0000u) | (uint32_t)child | ((uint32_t)asf << 8);
  tput(L, t, e);
}

// Complete every outstanding vector-memory operation inside the branch that issued a conditional
// load (s_waitcnt vmcnt(0); gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15).  The wait-count pass
// is conservative at control-flow joins: without this it waits at the join on every path, and
// that wait would also cover the next chunk's rows prefetched at the top of the chunk loop.
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// Retire: an empty asm reading the registers of a prefetch load.  The compiler's waitcnt pass
// waits for a load at its first use; vmcnt retires in issue order, so a first use that falls
// after stores (the next iteration's top, after the flush) would also wait for every store ack.
// Consuming the registers at a chosen point, before any store, moves that wait there.  (The
// preheader loads are consumed before the loop for the same reason: the loop header merges the
// preheader's pending loads with the back edge's pending stores.)
__device__ __forceinline__ void consume(uint32_t v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void consume(uint2 v) { asm volatile("" ::"v"(v.x), "v"(v.y)); }
__device__ __forceinline__ void consume(uint4 v) { asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w)); }

// ---- variables (registers) ------------------------------------------------------------------
template <class K>
__device__ __forceinline__ int var_find(const Lane<K>& L, uint32_t scope, uint32_t name) {
  const uint32_t want = name | (scope << 16);
  int r = -1;
  if (L.nvars > 3 && L.vx3 == want) r = 3;
  if (L.nvars > 2 && L.vx2 == want) r = 2;
  if (L.nvars > 1 && L.vx1 == want) r = 1;
  if (L.nvars > 0 && L.vx0 == want) r = 0;
  return r;
}

// VariableBehavior.setLocalVariable (VariableBehavior.java:191-200) + VariableApplier
template <class K>
__device__ __forceinline__ void set_local_variable(Lane<K>& L, uint32_t scope, const zbhip_doc_entry& d) {
  int v = var_find(L, scope, d.name_id);
  if (v < 0) {
    if (L.nvars >= kVars) { set_fail(L, FB_VARS); return; }
    uint32_t key = new_key(L);
    emit(L, C_VAR_CREATED, key, scope, d.name_id);
    var_put(L, L.nvars++, d.name_id | (scope << 16), key | ((uint32_t)d.type << 16), d.value);
  } else {
    const uint32_t y = var_y(L, v);
    if (!(((y >> 16) & 0xFF) == d.type && var_v(L, v) == d.value)) {
      emit(L, C_VAR_UPDATED, y & 0xFFFF, scope, d.name_id);
      var_put(L, v, var_x(L, v), (y & 0xFFFF) | ((uint32_t)d.type << 16), d.value);
    }
  }
}

// The key ordinal of the instance of the i-th scope above an element in container c (K::S: the
// instances of the enclosing sub-processes / multi-instance bodies; one per container element),
// NONE past the process's children.  Scope chains are at most kMaxDepth deep on the device
// (zbhip_deploy refuses io-mapped processes nested deeper).
constexpr int kMaxDepth = kMaxScopeDepth;
template <class K>
__device__ __forceinline__ uint32_t container_key(const Lane<K>& L, uint32_t& c) {
  if constexpr (K::S) {
    if (c == 0) return NONE;
    const int t = scope_find(L, c);
    c = scope_of<K>(elem_of(L, c));
    return t < 0 ? NONE : tget(L, t).x >> 16;
  } else {
    return NONE;
  }
}

// DbVariableState.getVariable (state/variable/DbVariableState.java:174-200): the scope `key`, then
// the instances of the containers from c up, then the process instance
template <class K>
__device__ __forceinline__ int var_lookup(const Lane<K>& L, uint32_t key, uint32_t c, uint32_t name) {
  int v = var_find(L, key, name);
  if constexpr (!K::IO) return v >= 0 ? v : var_find(L, 0, name);
  for (int d = 0; v < 0 && d < kMaxDepth; ++d) {
    const uint32_t k = container_key(L, c);
    if (k == NONE) break;
    v = var_find(L, k, name);
  }
  return v >= 0 ? v : var_find(L, 0, name);
}

// A multi-entry document's merge order (zbhip.h zbhip_doc_merge_order, the agrona Int2IntHashMap
// IndexedDocument iterates): position i -> document index in bits 4i..4i+3; false outside the subset (more
// than ZBHIP_DOC_MAX_ENTRIES entries, no permutation in the pad bytes, a repeated name).
template <class K>
__device__ __forceinline__ bool doc_order(const Lane<K>& L, uint32_t begin, uint32_t count, uint32_t& order,
                                          bool& displaced) {
  if (count > ZBHIP_DOC_MAX_ENTRIES) return false;
  uint32_t seen = 0;
  order = 0;
  displaced = false;
  for (uint32_t i = 0; i < count; ++i) {
    const zbhip_doc_entry e = L.docs[begin + i];
    const uint32_t j = e.pad[0];
    if (j >= count || ((seen >> j) & 1u)) return false;
    seen |= 1u << j;
    order |= j << (4 * i);
    if (i == 0) displaced = e.pad[1] & 1;
    for (uint32_t q = 0; q < i; ++q)
      if (L.docs[begin + q].name_id == e.name_id) return false;
  }
  return true;
}

// VariableBehavior.mergeLocalDocument (VariableBehavior.java:60-82): setLocalVariable of every entry in the
// IndexedDocument's order
template <class K>
__device__ __forceinline__ void merge_local_document(Lane<K>& L, uint32_t scope, uint32_t begin, uint32_t count) {
  if (count == 1) {
    const zbhip_doc_entry d = L.docs[begin];
    vm_drain();
    set_local_variable(L, scope, d);
    return;
  }
  uint32_t order;
  bool displaced;
  if (!doc_order(L, begin, count, order, displaced)) { set_fail(L, FB_DOC); return; }
  for (uint32_t i = 0; i < count && !L.fail; ++i) {
    const zbhip_doc_entry d = L.docs[begin + ((order >> (4 * i)) & 0xF)];
    vm_drain();
    set_local_variable(L, scope, d);
  }
}

// mergeDocument of a multi-entry document: every scope from the element's up to (not including) the
// process instance's iterates the entries left, updating those it holds with another value and removing
// them from the document (Iterator.remove); the process instance's scope sets the rest.  A removal from a
// table with an entry off its home slot compacts a probe chain and may reorder what is left: outside the
// subset.
template <class K>
__device__ __forceinline__ void merge_document_multi(Lane<K>& L, uint32_t scope_key, uint32_t c, uint32_t begin,
                                                     uint32_t count) {
  uint32_t order;
  bool displaced;
  if (!doc_order(L, begin, count, order, displaced)) { set_fail(L, FB_DOC); return; }
  const uint32_t all = (1u << count) - 1;
  uint32_t left = all;
  auto level = [&](uint32_t k) {
    for (uint32_t i = 0; i < count; ++i) {
      if (!((left >> i) & 1u)) continue;
      const zbhip_doc_entry d = L.docs[begin + ((order >> (4 * i)) & 0xF)];
      vm_drain();
      if constexpr (K::IO) {  // a propagated outputCollection (see merge_document_from)
        for (int q = 0; q < kVars; ++q)
          if (q < L.nvars && (var_x(L, q) & 0xFFFF) == d.name_id && ((var_y(L, q) >> 16) & 0xFF) == kDocOutList) {
            set_fail(L, FB_DOC);
            return;
          }
      }
      const int v = var_find(L, k, d.name_id);
      if (v < 0) continue;
      const uint32_t y = var_y(L, v);
      if (((y >> 16) & 0xFF) == d.type && var_v(L, v) == d.value) continue;
      emit(L, C_VAR_UPDATED, y & 0xFFFF, k, d.name_id);
      var_put(L, v, var_x(L, v), (y & 0xFFFF) | ((uint32_t)d.type << 16), d.value);
      left &= ~(1u << i);
    }
  };
  if constexpr (!K::IO) {
    if (scope_key != 0) level(scope_key);
  } else {
    uint32_t k = scope_key;
    for (int depth = 0; k != 0 && k != NONE && depth <= kMaxDepth && !L.fail; ++depth) {
      level(k);
      k = container_key(L, c);
    }
  }
  if (L.fail) return;
  if (left != all && displaced) { set_fail(L, FB_DOC); return; }
  for (uint32_t i = 0; i < count && !L.fail; ++i) {
    if (!((left >> i) & 1u)) continue;
    const zbhip_doc_entry d = L.docs[begin + ((order >> (4 * i)) & 0xF)];
    vm_drain();
    set_local_variable(L, 0, d);
  }
}

// VariableBehavior.mergeDocument (VariableBehavior.java:105-150) of the command's document from
// the scope `scope_key` of an element in container c: updated in the first scope below the process
// that holds the variable with another value, else set locally in the process instance's scope.
template <class K>
__device__ __forceinline__ void merge_document_from(Lane<K>& L, uint32_t scope_key, uint32_t c, uint32_t begin,
                                                    uint32_t count) {
  if (count == 0) return;
  if (count > 1) { merge_document_multi(L, scope_key, c, begin, count); return; }
  const zbhip_doc_entry d = L.docs[begin];
  vm_drain();
  if constexpr (K::IO) {
    // a propagated multi-instance outputCollection: its items are the host's (the value comparison of
    // setLocalVariable cannot be made here)
    for (int i = 0; i < kVars; ++i)
      if (i < L.nvars && (var_x(L, i) & 0xFFFF) == d.name_id && ((var_y(L, i) >> 16) & 0xFF) == kDocOutList) {
        set_fail(L, FB_DOC);
        return;
      }
  }
  if constexpr (!K::IO) {  // (no variables in scopes between the element and the process)
    if (scope_key != 0) {
      int v = var_find(L, scope_key, d.name_id);
      if (v >= 0) {
        const uint32_t y = var_y(L, v);
        if (!(((y >> 16) & 0xFF) == d.type && var_v(L, v) == d.value)) {
          emit(L, C_VAR_UPDATED, y & 0xFFFF, scope_key, d.name_id);
          var_put(L, v, var_x(L, v), (y & 0xFFFF) | ((uint32_t)d.type << 16), d.value);
          return;
        }
      }
    }
    set_local_variable(L, 0, d);
    return;
  }
  uint32_t k = scope_key;
  for (int depth = 0; k != 0 && k != NONE && depth <= kMaxDepth; ++depth) {
    int v = var_find(L, k, d.name_id);
    if (v >= 0) {
      const uint32_t y = var_y(L, v);
      if (!(((y >> 16) & 0xFF) == d.type && var_v(L, v) == d.value)) {
        emit(L, C_VAR_UPDATED, y & 0xFFFF, k, d.name_id);
        var_put(L, v, var_x(L, v), (y & 0xFFFF) | ((uint32_t)d.type << 16), d.value);
        return;  // consumed at this scope
      }
    }
    k = container_key(L, c);
  }
  set_local_variable(L, 0, d);
}

// ---- io mappings (K::S; BpmnVariableMappingBehavior.java:53-156) ---------------------------------
// mapping k (0 input, 1 output) of element e (runtime.cpp rebuild_program): x = type | target name
// << 16 (type 0xFE: none; ZBHIP_MAP_VARIABLE: y = the source's name id), z/w = the literal
constexpr uint32_t kIoNone = 0xFE;
template <class K>
__device__ __forceinline__ uint4 io_map(const Lane<K>& L, uint32_t e, int k) {
  if constexpr (!K::IO) return make_uint4(kIoNone, 0, 0, 0);
  if (!((L.pb[5] >> 17) & 1u)) return make_uint4(kIoNone, 0, 0, 0);
  return reinterpret_cast<const uint4*>(L.pb + (L.pb[6] >> 16))[2 * e + k];
}

// ---- multi-instance collections (K::IO: a body with a collection variable, output or condition) ----
// a body's words in its io slots (runtime.cpp rebuild_program): [0] x = collection variable | output
// collection << 16, y = outputElement | (completionCondition + 1) << 16, z / w = the numberOf* name ids;
// [1] y = the static items' list id (0xFFFFFFFF: none)
template <class K>
__device__ __forceinline__ uint4 mi_ext(const Lane<K>& L, uint32_t body) {
  if constexpr (!K::IO) return make_uint4(0xFFFFFFFFu, 0x0000FFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  if (!((L.pb[5] >> 17) & 1u)) return make_uint4(0xFFFFFFFFu, 0x0000FFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  return reinterpret_cast<const uint4*>(L.pb + (L.pb[6] >> 16))[2 * body];
}

// readInputCollectionVariable (MultiInstanceBodyProcessor.java:362-367): the item count and the list
// (0xFFFFFFFF: the static items of a body without collection words), the variable seen from the scope
// `key` in container c; a missing or non-list variable is an incident (outside the subset: fallback)
template <class K>
__device__ __forceinline__ bool mi_collection(Lane<K>& L, uint32_t body, uint4 bw, uint32_t key, uint32_t c, uint32_t& n,
                                              uint32_t& list) {
  const uint32_t coll = mi_ext(L, body).x & 0xFFFF;
  list = 0xFFFFFFFFu;
  if (coll == 0xFFFF) {
    n = (bw.z >> 12) & 0xFF;
    if constexpr (K::IO)
      if ((L.pb[5] >> 17) & 1u) list = reinterpret_cast<const uint4*>(L.pb + (L.pb[6] >> 16))[2 * body + 1].y;
    return true;
  }
  const int v = var_lookup(L, key, c, coll);
  if (v < 0 || ((var_y(L, v) >> 16) & 0xFF) != ZBHIP_DOC_LIST) { set_fail(L, FB_FEEL); return false; }
  const long long id = var_v(L, v);
  const StepParams& P = *L.sp;
  if (id < 0 || (unsigned long long)id >= P.n_lists) { set_fail(L, FB_FEEL); return false; }
  n = P.list_hdr[id].y;
  if (n > 63) { set_fail(L, FB_UNSUPPORTED); return false; }
  list = (uint32_t)id;
  return true;
}

// item i (0-based) of a list
template <class K>
__device__ __forceinline__ void list_item(const Lane<K>& L, uint32_t list, uint32_t i, uint32_t& type, long long& v) {
  const StepParams& P = *L.sp;
  const uint2 hd = P.list_hdr[list];
  type = P.list_type[hd.x + i];
  v = P.list_val[hd.x + i];
}

// ExpressionProcessor.evaluateVariableMappingExpression of a one-entry context in the scope `key` of
// an element in container c: a literal, or a copy of the variable (a missing one: outside the
// subset); FeelToMessagePackTransformer.scala:35-39 writes a whole number as an integer
template <class K>
__device__ __forceinline__ bool map_value(Lane<K>& L, uint4 m, uint32_t key, uint32_t c, uint32_t& type, long long& v) {
  type = m.x & 0xFF;
  v = (long long)(((unsigned long long)m.w << 32) | m.z);
  if (type != ZBHIP_MAP_VARIABLE) return true;
  const int i = var_lookup(L, key, c, m.y);
  if (i < 0) { set_fail(L, FB_FEEL); return false; }
  type = (var_y(L, i) >> 16) & 0xFF;
  v = var_v(L, i);
  if (type == ZBHIP_DOC_DEC && v % 1000000 == 0) {
    type = ZBHIP_DOC_INT;
    v /= 1000000;
  }
  return type <= ZBHIP_DOC_DEC || type == ZBHIP_DOC_STR;
}

// VariableBehavior.setLocalVariable of a value the engine computed: VARIABLE:CREATED (+key) or
// UPDATED, the value into the batch's map_val slot (C_VAR_MAPPED)
template <class K>
__device__ __forceinline__ void set_local_mapped(Lane<K>& L, uint32_t scope, uint32_t name, uint32_t type, long long v) {
  const StepParams& P = *L.sp;
  int i = var_find(L, scope, name);
  if (i >= 0 && ((var_y(L, i) >> 16) & 0xFF) == type && var_v(L, i) == v) return;
  if (L.n_map >= (uint32_t)kMapVals || L.ci >= P.map_cap) { set_fail(L, FB_VARS); return; }
  const bool updated = i >= 0;
  uint32_t key;
  if (!updated) {
    if (L.nvars >= kVars) { set_fail(L, FB_VARS); return; }
    key = new_key(L);
    i = L.nvars++;
  } else {
    key = var_y(L, i) & 0xFFFF;
  }
  P.map_val[(size_t)L.n_map * P.map_cap + L.ci] = v;
  emit(L, C_VAR_MAPPED, key, scope, name, type | ((updated ? 1u : 0u) << 3) | (L.n_map << 4));
  ++L.n_map;
  var_put(L, i, name | (scope << 16), key | (type << 16), v);
}

// applyInputMappings (:53-77): evaluated in the new element instance's scope, merged locally into it
template <class K>
__device__ __forceinline__ void apply_input_mapping(Lane<K>& L, uint32_t elem, uint32_t key) {
  const uint4 m = io_map(L, elem, 0);
  if ((m.x & 0xFF) == kIoNone) return;
  uint32_t type;
  long long v;
  if (!map_value(L, m, key, scope_of<K>(elem_of(L, elem)), type, v)) { set_fail(L, FB_FEEL); return; }
  set_local_mapped(L, key, m.x >> 16, type, v);
}

// the output mapping of applyOutputMappings (:86-131) after the event's variables were merged locally:
// evaluated in the element's scope, then VariableBehavior.mergeDocument from its flow scope
// (getVariableScopeKey, :157-165: no multi-instance inner activities)
template <class K>
__device__ __forceinline__ void apply_output_mapping(Lane<K>& L, uint4 m, uint32_t elem, uint32_t key) {
  uint32_t c = scope_of<K>(elem_of(L, elem));
  uint32_t type;
  long long v;
  if (!map_value(L, m, key, c, type, v)) { set_fail(L, FB_FEEL); return; }
  const uint32_t name = m.x >> 16;
  for (int depth = 0; depth < kMaxDepth; ++depth) {
    const uint32_t k = container_key(L, c);
    if (k == NONE) break;
    const int i = var_find(L, k, name);
    if (i >= 0 && !(((var_y(L, i) >> 16) & 0xFF) == type && var_v(L, i) == v)) {
      set_local_mapped(L, k, name, type, v);
      return;
    }
  }
  set_local_mapped(L, 0, name, type, v);
}

// variableState.removeScope (DbElementInstanceState.removeInstance): the element instance's own
// variables leave with it (registers closed up)
template <class K>
__device__ __forceinline__ void vars_drop_scope(Lane<K>& L, uint32_t key) {
  int n = 0;
  for (int i = 0; i < kVars; ++i) {
    if (i >= L.nvars) break;
    const uint32_t x = var_x(L, i), y = var_y(L, i);
    const long long v = var_v(L, i);
    if ((x >> 16) == key) continue;
    if (n != i) var_put(L, n, x, y, v);
    ++n;
  }
  L.nvars = n;
}

// ---- join counters (registers, 16 x u8) ----------------------------------------------------
template <class K>
__device__ __forceinline__ uint32_t join_get(const Lane<K>& L, uint32_t s) {
  return (jw_get(L, (int)(s >> 2)) >> ((s & 3) * 8)) & 0xFF;
}
template <class K>
__device__ __forceinline__ void join_set(Lane<K>& L, uint32_t s, uint32_t v) {
  const uint32_t sh = (s & 3) * 8;
  const int i = (int)(s >> 2);
  jw_put(L, i, (jw_get(L, i) & ~(0xFFu << sh)) | ((v & 0xFF) << sh));
}

// ---- FEEL condition bytecode ------------------------------------------------------------------
// Values: tag 0 NULL, 1 BOOL, 2 NUMBER (x 10^ZBHIP_DEC_SCALE), 3 STRING (never compared: an ordering
// comparison of a string with a number is NULL in feel-scala 1.17, ConditionIncidentTest).  A result
// that is not a boolean is an incident in the reference (ExpressionProcessor.java:356-368).
// The operand stack is four registers, top first (the compiler bounds the depth to 4).
// The variables a multi-instance inner instance holds without a variable-table entry (its
// inputElement, outputElement and loopCounter: setLoopVariables) and the body's numberOf* of a
// completion condition (its primary context, MultiInstanceBodyProcessor.java:396-460): names (NONE:
// none), zbhip_doc_types and values; looked up before the variable table
struct MiVars {
  uint32_t name[7];
  uint32_t type[7];
  long long val[7];
};

template <class K>
__device__ __forceinline__ bool load_var(const Lane<K>& L, uint32_t name, uint32_t scope_key, uint32_t c, uint32_t& t,
                                         long long& x, const MiVars* mv = nullptr) {
  // DbVariableState.getVariable: element scope first, then the enclosing scopes up to the process
  uint32_t ty = 0;
  long long raw = 0;
  int hit = -1;
  if (mv)
    for (int i = 0; i < 7; ++i)
      if (hit < 0 && mv->name[i] != NONE && mv->name[i] == name) hit = i;
  t = 0;
  x = 0;
  if (hit >= 0) {
    ty = mv->type[hit];
    raw = mv->val[hit];
  } else {
    const int v = var_lookup(L, scope_key, c, name);
    if (v < 0) return true;  // missing -> null
    ty = (var_y(L, v) >> 16) & 0xFF;
    raw = var_v(L, v);
  }
  if (ty == ZBHIP_DOC_NIL) return true;
  if (ty == ZBHIP_DOC_BOOL) { t = 1; x = raw != 0; return true; }
  if (ty == ZBHIP_DOC_INT) {
    if (raw > 9223372036854LL || raw < -9223372036854LL) return false;
    t = 2;
    x = raw * 1000000LL;
    return true;
  }
  if (ty == ZBHIP_DOC_DEC) { t = 2; x = raw; return true; }
  if (ty == ZBHIP_DOC_STR) { t = 3; return true; }
  return false;
}

// result: -1 outside the subset (fallback), else the tag of the value (1: boolean, in `out`)
template <class K>
__device__ __forceinline__ int eval_condition(Lane<K>& L, uint32_t cond, uint32_t scope_key, uint32_t c, bool& out,
                                              const MiVars* mv = nullptr) {
  const uint32_t* pb = L.pb;
  uint32_t pc = pb[pb[3] + cond];
  const uint32_t* code = pb + pb[4];
  uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  long long a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  int sp = 0;
  for (int guard = 0; guard < 32; ++guard) {
    const uint4 in = *reinterpret_cast<const uint4*>(code + 4 * pc++);
    const uint32_t op = in.x;
    if (op == ZBHIP_OP_END) break;
    if (op <= ZBHIP_OP_PUSH_NULL) {
      uint32_t t = 0;
      long long x = 0;
      if (op == ZBHIP_OP_PUSH_NUM) { t = 2; x = (long long)(((unsigned long long)in.w << 32) | in.z); }
      else if (op == ZBHIP_OP_PUSH_BOOL) { t = 1; x = in.y != 0; }
      else if (op == ZBHIP_OP_PUSH_VAR) { if (!load_var(L, in.y, scope_key, c, t, x, mv)) return -1; }
      if (sp >= 4) return -1;
      t3 = t2; a3 = a2; t2 = t1; a2 = a1; t1 = t0; a1 = a0; t0 = t; a0 = x;
      ++sp;
      continue;
    }
    if (op == ZBHIP_OP_NOT) {
      if (sp < 1 || t0 != 1) return -1;
      a0 = !a0;
      continue;
    }
    if (sp < 2) return -1;
    // binary: a = second, b = top
    const uint32_t ta = t1, tb = t0;
    const long long a = a1, b = a0;
    uint32_t rt = 1;
    bool r = false;
    if (op == ZBHIP_OP_AND || op == ZBHIP_OP_OR) {
      if (ta != 1 || tb != 1) return -1;
      r = op == ZBHIP_OP_AND ? (a && b) : (a || b);
    } else if (op == ZBHIP_OP_EQ || op == ZBHIP_OP_NE) {
      bool eq;
      if (ta == 3 || tb == 3) return -1;
      if (ta == 0 || tb == 0) eq = ta == tb;
      else if (ta != tb) return -1;
      else eq = a == b;
      r = op == ZBHIP_OP_EQ ? eq : !eq;
    } else if (ta == 0 || tb == 0 || (ta == 3 && tb == 2) || (ta == 2 && tb == 3)) {
      rt = 0;  // null
    } else {
      if (ta != 2 || tb != 2) return -1;
      r = op == ZBHIP_OP_LT ? a < b : op == ZBHIP_OP_LE ? a <= b : op == ZBHIP_OP_GT ? a > b : a >= b;
    }
    t0 = rt; a0 = r;
    t1 = t2; a1 = a2; t2 = t3; a2 = a3;
    --sp;
  }
  if (sp != 1) return -1;
  out = t0 == 1 && a0 != 0;
  return (int)t0;
}

// An exclusive gateway's incident (incident info in the element-table entry, bits 26..31): the
// position of the flow whose condition was not a boolean in the gateway's outgoing list (0..14) or
// 15 (none chosen, CONDITION_ERROR) | the ZBHIP_FEEL_* type of that result << 4
constexpr uint16_t FLOW_INCIDENT = 0xFFFE;
constexpr uint32_t INC_NONE_CHOSEN = 15;

// ExclusiveGatewayProcessor.findSequenceFlowToTake (:86-126); a failure returns FLOW_INCIDENT with
// the incident info in L.inc
template <class K>
__device__ __forceinline__ uint32_t find_sequence_flow(Lane<K>& L, uint4 gw, uint32_t gw_key) {
  uint32_t ob = gw.y & 0xFFFF, oc = gw.y >> 16;
  if (oc == 0) return NONE;  // implicit end
  if (oc == 1 && (elem_of(L, out_flow(L, ob)).z >> 16) == NONE) return out_flow(L, ob);
  uint32_t dflt = gw.z & 0xFFFF;
  for (uint32_t i = 0; i < oc; ++i) {
    uint32_t f = out_flow(L, ob + i);
    uint32_t cond = elem_of(L, f).z >> 16;
    if (cond == NONE || f == dflt) continue;  // outgoingWithCondition, default skipped
    bool ok;
    const int rt = eval_condition(L, cond, gw_key, scope_of<K>(gw), ok);
    if (rt < 0 || (rt != 1 && i >= INC_NONE_CHOSEN)) { set_fail(L, FB_FEEL); return NONE; }
    if (rt != 1) {  // typeCheck: EXTRACT_VALUE_ERROR
      L.inc = i | ((rt == 0 ? ZBHIP_FEEL_NULL : rt == 2 ? ZBHIP_FEEL_NUMBER : ZBHIP_FEEL_STRING) << 4);
      return FLOW_INCIDENT;
    }
    if (ok) return f;
  }
  if (dflt != NONE) return dflt;
  L.inc = INC_NONE_CHOSEN;  // NO_OUTGOING_FLOW_CHOSEN_ERROR (:121-125), CONDITION_ERROR
  return FLOW_INCIDENT;
}

// ---- appliers ------------------------------------------------------------------------------
// ProcessInstanceElementActivatingApplier.applyState (:48-204) for a child of the process
template <class K>
__device__ __forceinline__ void apply_activating_child(Lane<K>& L, uint32_t elem, uint4 w, uint32_t key) {
  uint32_t type = etype(w);
  if (type == ZBHIP_EL_PARALLEL_GATEWAY) {  // cleanupSequenceFlowsTaken: Tetris decrement
    uint32_t base = w.w & 0xFFFF, n = w.x >> 16;
    for (uint32_t s = base; s < base + n; ++s) {
      uint32_t c = join_get(L, s);
      if (c > 0) join_set(L, s, c - 1);
    }
  }
  if constexpr (K::S) {
    // a second active instance of one container element: outside the device subset
    const bool container = type == ZBHIP_EL_SUB_PROCESS || type == ZBHIP_EL_MULTI_INSTANCE_BODY;
    if (container && scope_find(L, elem) >= 0) { set_fail(L, FB_UNSUPPORTED); return; }
    const int t = tbl_insert(L, elem, key, ZBHIP_PI_ELEMENT_ACTIVATING);
    if (t < 0) return;
    if (container)  // jobKey 0; no children, no active flows (a body: loop counter 0) yet
      tput(L, t, make_uint2(elem | (key << 16), (uint32_t)ZBHIP_PI_ELEMENT_ACTIVATING << 16));
    const int da = type == ZBHIP_EL_START_EVENT || type == ZBHIP_EL_BOUNDARY_EVENT ? 0
                   : type == ZBHIP_EL_PARALLEL_GATEWAY ? -(int)(w.x >> 16) : -1;
    const uint32_t c = scope_of<K>(w);
    scope_adjust(L, c, 1, da);
    if (c != 0 && !L.fail && etype(elem_of(L, c)) == ZBHIP_EL_MULTI_INSTANCE_BODY) {
      // manageMultiInstance (ProcessInstanceElementActivatingApplier.java:237-253): the body's loop
      // counter (= childActivatedCount) + 1, the inner instance's loop counter set to it
      const int tb = scope_find(L, c);
      uint2 b = tget(L, tb);
      const uint32_t loop = ((b.y >> 8) & 0xFF) + 1;
      if (loop > 63) { set_fail(L, FB_UNSUPPORTED); return; }
      b.y = (b.y & 0xFFFF00FFu) | (loop << 8);
      tput(L, tb, b);
      uint2 e = tget(L, t);
      e.y = (e.y & 0x03FFFFFFu) | (loop << 26);
      tput(L, t, e);
    }
    return;
  }
  tbl_insert(L, elem, key, ZBHIP_PI_ELEMENT_ACTIVATING);
  ++L.pi_child;
  if (type == ZBHIP_EL_START_EVENT || (K::M && type == ZBHIP_EL_BOUNDARY_EVENT)) {  // not reached by a sequence flow
  } else if (type == ZBHIP_EL_PARALLEL_GATEWAY) {
    int n = (int)(w.x >> 16);
    L.pi_asf = L.pi_asf > n ? L.pi_asf - n : 0;  // decrementActiveSequenceFlows clamps at 0
  } else if (L.pi_asf > 0) {
    --L.pi_asf;
  }
}

// ProcessInstanceElementCompletedApplier.applyState (:45-73) -> DbElementInstanceState.removeInstance
template <class K>
__device__ __forceinline__ void apply_completed_child(Lane<K>& L, int t, uint32_t key) {
  if (L.trig_key == key) L.trig_key = NONE;  // eventScopeInstanceState.deleteInstance (triggers)
  if constexpr (K::S) {
    const uint4 w = elem_of(L, tget(L, t).x & 0xFFFF);
    tput(L, t, make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu));
    if constexpr (K::IO)
      if (L.nvars) vars_drop_scope(L, key);
    if (etype(w) == ZBHIP_EL_SUB_PROCESS) {  // its taken-flow counters go with it (removeInstance)
      const uint32_t m = w.z >> 16;
      for (uint32_t s = 0; s < (uint32_t)kMaxJoinSlots; ++s)
        if ((m >> s) & 1u) join_set(L, s, 0);
    }
    scope_adjust(L, scope_of<K>(w), -1, 0);
    return;
  }
  tput(L, t, make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu));
  --L.pi_child;
}

// takeSequenceFlow (:243-263) + activateElementInstanceInFlowScope (:326-339)
template <class K>
__device__ __forceinline__ void take_sequence_flow(Lane<K>& L, uint32_t flow) {
  uint4 fw = elem_of(L, flow);
  const uint32_t c = scope_of<K>(fw);
  const uint32_t fsk = K::S ? scope_key(L, c) : 0u;
  uint32_t sft = new_key(L);
  emit(L, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, sft, fsk, flow);
  if constexpr (K::S) scope_adjust(L, c, 0, 1);  // ProcessInstanceSequenceFlowTakenApplier
  else ++L.pi_asf;
  uint32_t target = fw.z & 0xFFFF;
  if (etype(elem_of(L, target)) == ZBHIP_EL_PARALLEL_GATEWAY) {
    uint32_t s = fw.w & 0xFFFF;
    uint32_t c = join_get(L, s);
    if (c >= 255) set_fail(L, FB_JOIN);
    join_set(L, s, c + 1);
  }
  uint32_t k = new_key(L);
  follow_up(L, ZBHIP_PI_ACTIVATE_ELEMENT, k, fsk, target, false, true, k);
}

// MultiInstanceBodyProcessor.beforeExecutionPathCompleted (:160-191) of the inner instance `key` (table
// entry t) of body c: updateOutputCollection (MultiInstanceOutputCollectionBehavior.java:57-141: the
// outputElement's value at loopCounter - 1 -- C_MI_OUT, the host completes the array), then the
// completion condition (satisfiesCompletionCondition :380-394), then for a sequential body the input
// collection read again (its size in n).  Returns whether the condition is satisfied.
template <class K>
__device__ __forceinline__ bool mi_before_completed(Lane<K>& L, int t, uint32_t c, uint32_t key, uint32_t& n) {
  const uint4 bw = elem_of(L, c), ext = mi_ext(L, c);
  uint32_t list;
  if (!mi_collection(L, c, bw, key, c, n, list)) return false;
  const uint32_t loop = tget(L, t).y >> 26;
  if (loop < 1 || loop > n) { set_fail(L, FB_UNSUPPORTED); return false; }
  const uint32_t in = bw.x >> 16, ln = bw.w & 0xFFFF, oe = ext.y & 0xFFFF, oc = ext.x >> 16;
  const uint32_t cond = ext.y >> 16;  // completionCondition + 1
  if (oc == 0xFFFF && cond == 0) return false;
  // the inner instance's own variables (not in the variable table)
  MiVars mv;
  for (int i = 0; i < 7; ++i) { mv.name[i] = NONE; mv.type[i] = 0; mv.val[i] = 0; }
  if (in != 0xFFFF) {
    if (list == 0xFFFFFFFFu) { set_fail(L, FB_UNSUPPORTED); return false; }
    uint32_t ty;
    long long v;
    list_item(L, list, loop - 1, ty, v);
    mv.name[0] = in;
    mv.type[0] = ty;
    mv.val[0] = v;
  }
  mv.name[1] = ln;
  mv.type[1] = ZBHIP_DOC_INT;
  mv.val[1] = loop;
  if (oe != 0xFFFF && oe != in && oe != ln) {
    mv.name[2] = oe;
    mv.type[2] = L.mo_set ? L.mo_type : ZBHIP_DOC_NIL;
    mv.val[2] = L.mo_set ? L.mo_val : 0;
  }
  if (oc != 0xFFFF) {
    // the outputElement `= name` evaluated in the inner instance's scope
    uint32_t ty = 0;
    long long v = 0;
    int hit = -1;
    for (int i = 0; i < 3; ++i)
      if (hit < 0 && mv.name[i] == oe) hit = i;
    if (hit >= 0) {
      ty = mv.type[hit];
      v = mv.val[hit];
    } else {
      const int vi = var_lookup(L, key, c, oe);
      if (vi < 0) { set_fail(L, FB_FEEL); return false; }  // null for a missing variable: unpinned
      ty = (var_y(L, vi) >> 16) & 0xFF;
      v = var_v(L, vi);
    }
    if (ty > ZBHIP_DOC_STR || ty == ZBHIP_DOC_OTHER) { set_fail(L, FB_UNSUPPORTED); return false; }
    const StepParams& P = *L.sp;
    if (L.n_map >= (uint32_t)kMapVals || L.ci >= P.map_cap) { set_fail(L, FB_VARS); return false; }
    P.map_val[(size_t)L.n_map * P.map_cap + L.ci] = v;
    emit(L, C_MI_OUT, loop - 1, scope_key(L, c), c, ty | (L.n_map << 4));
    ++L.n_map;
  }
  if (cond == 0) return false;
  // the body's numberOf* (the completing instance is still counted active, not yet completed)
  const int tb = scope_find(L, c);
  if (tb < 0) { set_fail(L, FB_UNSUPPORTED); return false; }
  const uint2 be = tget(L, tb);
  const uint32_t active = be.y & 0xFF, activated = (be.y >> 8) & 0xFF;
  const long long nv[4] = {(long long)activated, (long long)active - 1, (long long)activated - (long long)active + 1, 0};
  const uint32_t nn[4] = {ext.z & 0xFFFF, ext.z >> 16, ext.w & 0xFFFF, ext.w >> 16};
  for (int k = 0; k < 4; ++k) {
    mv.name[3 + k] = nn[k] == 0xFFFF ? NONE : nn[k];
    mv.type[3 + k] = ZBHIP_DOC_INT;
    mv.val[3 + k] = nv[k];
  }
  bool ok = false;
  const int rt = eval_condition(L, cond - 1, key, c, ok, &mv);
  if (rt != 1) { set_fail(L, FB_FEEL); return false; }  // not a boolean: an incident
  return ok;
}

// transitionToCompleted (:158-191) + afterExecutionPathCompleted -> ProcessProcessor (:130-140)
template <class K>
__device__ __forceinline__ void transition_to_completed_child(Lane<K>& L, int t, uint32_t elem, uint4 w, uint32_t key) {
  const uint32_t c = scope_of<K>(w);
  const uint32_t fsk = K::S ? scope_key(L, c) : 0u;
  // beforeExecutionPathCompleted (BpmnStateTransitionBehavior.java:171-178): a multi-instance body's
  // checks before the COMPLETED record
  bool satisfied = false;
  uint32_t n_items = 0;
  if constexpr (K::S)
    if ((w.y >> 16) == 0 && c != 0 && etype(elem_of(L, c)) == ZBHIP_EL_MULTI_INSTANCE_BODY) {
      satisfied = mi_before_completed(L, t, c, key, n_items);
      if (L.fail) return;
    }
  emit(L, ZBHIP_PI_ELEMENT_COMPLETED, key, fsk, elem);
  apply_completed_child(L, t, key);
  if ((w.y >> 16) == 0) {  // end of the execution path
    if (c == 0) {
      if (L.pi_live && L.pi_child + L.pi_asf == 0) {  // BpmnStateBehavior.canBeCompleted
        follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, 0, NONE, 0, true, false, 0);
      }
    } else if constexpr (K::S) {
      const int ts = scope_find(L, c);
      const uint4 cw = elem_of(L, c);
      if (etype(cw) == ZBHIP_EL_MULTI_INSTANCE_BODY) {
        // MultiInstanceBodyProcessor.afterExecutionPathCompleted (:193-230): a satisfied completion
        // condition terminates the other active children (terminateChildInstances,
        // BpmnStateTransitionBehavior.java:348-363: PROCESS_INSTANCE_BATCH:TERMINATE) and completes the
        // body at once when none is (else onChildTerminated does, child_terminated); otherwise a
        // sequential body activates its next inner instance while items are left, and the body
        // completes once no child is active
        if (ts < 0) { set_fail(L, FB_UNSUPPORTED); return; }
        const uint2 be = tget(L, ts);
        const uint32_t sk = be.x >> 16, loop = (be.y >> 8) & 0xFF;
        if (satisfied) {
          const uint32_t pc = scope_of<K>(cw), nch = be.y & 0xFF;
          if (nch != 0) {
            // (the terminations and the body's completion stay in this batch: their context is the lane's)
            if (pending(L) + L.processed + 3 + nch >= L.limit) { set_fail(L, FB_BATCH_LIMIT); return; }
            const uint32_t kb = new_key(L);
            follow_up(L, C_PIB_TERMINATE, kb, sk, c, false, false, sk, Q_TERM | Q_PIBT);
            return;
          }
          follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, sk, scope_key(L, pc), c, true, pc == 0, sk);
          return;
        }
        if (((cw.z >> 20) & 1u) && loop < n_items) {
          const uint32_t k = new_key(L);  // createInnerInstance -> activateChildInstanceWithKey
          follow_up(L, ZBHIP_PI_ACTIVATE_ELEMENT, k, sk, cw.z & 0xFFF, false, false, k);
        } else if ((be.y & 0xFF) == 0) {
          const uint32_t pc = scope_of<K>(cw);
          follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, sk, scope_key(L, pc), c, true, pc == 0, sk);
        }
        return;
      }
      // SubProcessProcessor.afterExecutionPathCompleted (:97-106): completeElement(flow scope)
      if (ts >= 0 && (tget(L, ts).y & 0xFFFF) == 0) {
        const uint32_t sk = tget(L, ts).x >> 16;
        const uint32_t pc = scope_of<K>(elem_of(L, c));
        follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, sk, scope_key(L, pc), c, true, pc == 0, sk);
      }
    }
  }
}

template <class K>
__device__ __forceinline__ void take_outgoing(Lane<K>& L, uint4 w) {
  uint32_t ob = w.y & 0xFFFF, oc = w.y >> 16;
  for (uint32_t i = 0; i < oc && !L.fail; ++i) take_sequence_flow(L, out_flow(L, ob + i));
}


// =============================================================================================
// Message correlation (K::M variant only)
// =============================================================================================
// Partition of a correlation key: SubscriptionUtil.getSubscriptionPartitionId
// (protocol-impl/.../SubscriptionUtil.java:22-44) over the host-computed Java hashCode.
__device__ __forceinline__ uint32_t subscription_partition(int32_t h, int32_t partitions) {
  const int32_t r = h % partitions;
  return (uint32_t)((r < 0 ? -r : r) + 1);
}

template <class K>
__device__ __forceinline__ uint16_t new_slot_key(Lane<K>& L) {
  if (L.s_next_ord >= 0xFFF0) set_fail(L, FB_KEYS);
  return L.s_next_ord++;
}

// payload references of the loaded instance's keys / of the lane's correlation slot keys
template <class K>
__device__ __forceinline__ long long iref(const Lane<K>& L, uint32_t ord) { return ref_subj(false, L.inst, ord); }
template <class K>
__device__ __forceinline__ long long sref(const Lane<K>& L, uint32_t ord) { return ref_subj(true, L.slot, ord); }
// device-resolved reference of a key the loaded instance generated in this batch
template <class K>
__device__ __forceinline__ long long cref_inst(const Lane<K>& L, uint32_t ord) { return ref_cmd(L.ci, L.slot_lane, ord); }

// one cross-partition send (post-commit side effect: InterPartitionCommandSender.sendCommand)
template <class K>
__device__ __forceinline__ void send_xpart(Lane<K>& L, uint32_t kind, uint32_t target, long long eik, long long pik,
                                           long long msg, uint32_t corr, uint32_t inst, uint32_t eord,
                                           uint32_t name_bpmn, uint32_t intr) {
  // one entry kept for a row patch; continuation batches (ci past the window) never send
  if (L.n_out >= (uint32_t)kOut - 1 || L.ci >= L.sp->xcap) { set_fail(L, FB_MESSAGE); return; }
  zbhip_xpart_cmd x;
  x.element_instance_key = eik;
  x.process_instance_key = pik;
  x.message_key = msg;
  x.correlation_key = corr;
  x.instance = inst;
  x.element_ord = (uint16_t)eord;
  x.message_name = (uint16_t)(name_bpmn & 0xFFFF);
  x.bpmn_process_id = (uint16_t)(name_bpmn >> 16);
  x.kind = (uint8_t)kind;
  x.interrupting = (uint8_t)intr;
  x.source_partition = (int16_t)L.sp->partition_id;
  x.target_partition = (int16_t)target;
  x.pad = 0;
  L.sp->xout[(size_t)L.n_out++ * L.sp->xcap + L.ci] = x;
  const uint32_t ns = L.x_sum & 0xF, t0 = (L.x_sum >> 8) & 0xFFFF;
  const bool mixed = (L.x_sum >> 31) || (ns && t0 != (target & 0xFFFF));
  L.x_sum = (ns + 1) | ((ns ? t0 : target & 0xFFFF) << 8) | (mixed ? 0x80000000u : 0u);
}

// CatchEventBehavior.subscribeToEvents -> subscribeToMessageEvent (processing/common/
// CatchEventBehavior.java:111-125,155-178,248-283): correlation key `= var` (STRING), the
// PROCESS_MESSAGE_SUBSCRIPTION:CREATING event (+key), then MESSAGE_SUBSCRIPTION:CREATE to the
// subscription partition -- a follow-up command here, or an outbox entry for another partition.
// A boundary event's correlation key is evaluated in the activity's flow scope (evaluateCorrelationKey,
// CatchEventBehavior.java:187-205): `boundary` skips the element's own scope.
template <class K>
__device__ __forceinline__ void subscribe_message(Lane<K>& L, uint32_t elem, uint4 w, uint32_t key, bool boundary = false) {
  const StepParams& P = *L.sp;
  const uint32_t name = w.z & 0xFFFF, var = w.z >> 16;
  int v = boundary ? -1 : var_find(L, key, var);  // DbVariableState.getVariable: element scope, then the process
  if (v < 0) v = var_find(L, 0, var);
  // ExpressionProcessor.evaluateMessageCorrelationKeyExpression: STRING (NUMBER / null -> outside)
  if (v < 0 || ((var_y(L, v) >> 16) & 0xFF) != ZBHIP_DOC_STR || L.slot_lane) { set_fail(L, FB_MESSAGE); return; }
  const long long sv = var_v(L, v);
  if (sv < 0 || sv >= (long long)P.n_strs || ((L.pm_x >> 12) & 3) != 0) { set_fail(L, FB_MESSAGE); return; }
  const uint32_t corr = (uint32_t)sv;
  const uint32_t part = subscription_partition((int32_t)P.str_hash[corr], P.partition_count);
  const uint32_t nb = name | ((L.pb[5] & 0xFFFF) << 16);
  const uint32_t sub = new_key(L);
  // ExecutableCatchEvent.isInterrupting: a catch event always, a boundary event as cancelActivity says
  const uint32_t intr = boundary ? (w.w & 1u) : 1u;
  L.pm_x = elem | (1u << 12) | (intr << 14) | (part << 16);  // ProcessMessageSubscriptionCreatingApplier
  L.pm_y = key | (sub << 16);
  L.pm_z = corr;
  L.pm_w = nb;
  L.pm_msg = -1;
  emit_msg(L, C_PMS_CREATING, iref(L, sub), iref(L, key), iref(L, 0), -1, corr, nb, part, intr, elem);
  if ((int32_t)part == P.partition_id) {
    emit_msg(L, C_MS_CREATE, -1, iref(L, key), iref(L, 0), -1, corr, nb, 0, intr, kNoElem);
    L.lq_slot = corr;
    L.lq_corr = corr;
    L.lq_intr = intr;
    L.lq_name_bpmn = nb;
    L.lq_eord = key;
    L.lq_eik = cref_inst(L, key);
    L.lq_pik = L.pik;
    push_local(L, LQ_MS_CREATE);
  } else {
    send_xpart(L, ZBHIP_CMD_MSG_SUB_CREATE, part, cref_inst(L, key), L.pik, -1, corr, L.inst, key, nb, intr);
  }
}

// a correlation key whose message state the engine holds (zbhip_evict_correlation_slots: slot_hdr.x bit 31):
// every message command of it -- a local follow-up of an instance's batch too -- is the engine's
__device__ __forceinline__ bool engine_owned(const StepParams& P, uint32_t slot) {
  return (P.st.slot_hdr[slot].x >> 31) != 0;
}

// a row of correlation slot `slot`: state != free, same subscriber (PI partition, instance, ord), same name
template <class K>
__device__ __forceinline__ int find_row(const Lane<K>& L, uint32_t slot, uint32_t pi_part, uint32_t inst, uint32_t eord,
                                        uint32_t name) {
  const StepParams& P = *L.sp;
  int found = -1;
  for (int r = kSubs - 1; r >= 0; --r) {
    const uint4 a = P.st.sub_a[sub_ri(r, slot)];
    if (((a.x & 0xFF) == 1 || (a.x & 0xFF) == 2) && (a.x >> 16) == pi_part && a.z == inst && (a.w & 0xFFFF) == eord && (a.y & 0xFFFF) == name)
      found = r;
  }
  if (L.op_ins && L.op_slot == slot && (L.ins_a.x >> 16) == pi_part && L.ins_a.z == inst &&
      (L.ins_a.w & 0xFFFF) == eord && (L.ins_a.y & 0xFFFF) == name)
    found = kSubs;  // inserted by this batch
  return found;
}

// MessageSubscriptionCreateProcessor.processRecord (processing/message/MessageSubscriptionCreateProcessor.java:66-104)
// values: eik / pik references as received, routing handle (pi_part, inst, eord)
template <class K>
__device__ __forceinline__ void ms_create(Lane<K>& L, uint32_t slot, uint32_t corr, uint32_t nb, uint32_t intr,
                                          uint32_t pi_part, uint32_t inst, uint32_t eord, long long eik,
                                          long long pik, long long eik_p, long long pik_p) {
  const StepParams& P = *L.sp;
  if (slot >= P.st.n_slots || engine_owned(P, slot)) { set_fail(L, FB_MESSAGE); return; }
  const bool dup = find_row(L, slot, pi_part, inst, eord, nb & 0xFFFF) >= 0;
  uint32_t key = NONE;
  if (!dup) {
    key = L.slot_lane ? new_slot_key(L) : new_key(L);
    const long long kp = L.slot_lane ? sref(L, key) : iref(L, key);
    emit_msg(L, C_MS_CREATED, kp, eik_p, pik_p, -1, corr, nb, 0, intr, kNoElem);
    if (L.op_ins) { set_fail(L, FB_MESSAGE); return; }
    // MessageSubscriptionCreatedApplier -> DbMessageSubscriptionState.put (row written at commit)
    L.op_ins = true;
    L.op_slot = slot;
    L.ins_a = make_uint4(1u | (intr << 8) | ((L.slot_lane ? 0u : 1u) << 9) | (pi_part << 16), nb, inst,
                         eord | (key << 16));
    L.ins_eik = eik;
    L.ins_pik = pik;
    L.ins_key = ref_cmd(L.ci, false, key);  // the batch's primary key space (instance or slot)
  }
  // MessageCorrelator.correlateNextMessage: no message outlives its PUBLISH batch in the subset
  // (time-to-live 0) -> acknowledge: SubscriptionCommandSender.openProcessMessageSubscription
  if ((int32_t)pi_part == P.partition_id) {
    emit_msg(L, C_PMS_CREATE, -1, eik_p, pik_p, -1, ZBHIP_NO_STRING,
             (nb & 0xFFFF) | 0xFFFF0000u, (uint32_t)P.partition_id, intr, kNoElem);
    L.lq_eord = eord;
    L.lq_name_bpmn = nb;
    L.lq_eik = eik;
    L.lq_pik = pik;
    L.lq_row = inst;  // the instance to load in a slot lane
    L.lq_intr = intr;
    push_local(L, LQ_PMS_CREATE);
  } else {
    send_xpart(L, ZBHIP_CMD_PMS_CREATE, pi_part, eik, pik, -1, corr, inst, eord, nb, intr);
  }
  if (dup)
    emit_msg(L, kRejectBit | C_MS_CREATE, -1, eik_p, pik_p, -1, corr, nb, 0, intr, kNoElem, ZBHIP_REASON_MS_ALREADY_OPEN);
}

// ProcessMessageSubscriptionCreateProcessor.processRecord: OPENING -> CREATED (subscription key)
template <class K>
__device__ __forceinline__ void pms_create(Lane<K>& L, uint32_t eord, uint32_t name, long long eik_p, long long pik_p,
                                           uint32_t part, uint32_t intr) {
  const uint32_t st = (L.pm_x >> 12) & 3;
  const uint32_t pm_elem = L.pm_x & 0xFFF;
  const bool match = st != 0 && (L.pm_y & 0xFFFF) == eord && (L.pm_w & 0xFFFF) == name;
  if (match && st == 1) {
    emit_msg(L, C_PMS_CREATED, iref(L, L.pm_y >> 16), iref(L, eord), iref(L, 0), -1, L.pm_z, L.pm_w, L.pm_x >> 16,
             (L.pm_x >> 14) & 1, pm_elem);
    L.pm_x = (L.pm_x & ~(3u << 12)) | (2u << 12);  // ProcessMessageSubscriptionCreatedApplier: OPENED
    // the acknowledgement of another partition carries the real element-instance key: kept for the
    // MESSAGE_SUBSCRIPTION:DELETE of a later window (the instance's keys are references in this one)
    if ((int32_t)part != L.sp->partition_id && L.inst < L.sp->st.n) L.sp->st.pms_eik[L.inst] = eik_p;
    return;
  }
  emit_msg(L, kRejectBit | C_PMS_CREATE, -1, eik_p, pik_p, -1, ZBHIP_NO_STRING, name | 0xFFFF0000u, part, intr,
           kNoElem, match ? (ZBHIP_REASON_PMS_CREATE_NOT_OPENING | ((st == 2 ? 1u : 0u) << 4)) : ZBHIP_REASON_PMS_CREATE_NOT_FOUND);
}

// ProcessMessageSubscriptionCorrelateProcessor.processRecord: CORRELATED, EventHandle.activateElement
// (processing/common/EventHandle.java:109-150: PROCESS_EVENT:TRIGGERING +key, COMPLETE_ELEMENT),
// then the acknowledgement MESSAGE_SUBSCRIPTION:CORRELATE to the message partition
template <class K>
__device__ __forceinline__ void pms_correlate(Lane<K>& L, uint32_t eord, uint32_t nb, long long eik_p, long long pik_p,
                                              long long msg_p, uint32_t corr, uint32_t part, long long eik,
                                              long long pik) {
  const uint32_t st = (L.pm_x >> 12) & 3;
  const uint32_t elem = L.pm_x & 0xFFF;
  const uint32_t name = nb & 0xFFFF;
  // no subscription, or a closing one: a rejection and MESSAGE_SUBSCRIPTION:REJECT (outside the subset)
  if (st == 0 || st == 3 || (L.pm_y & 0xFFFF) != eord || (L.pm_w & 0xFFFF) != name) { set_fail(L, FB_MESSAGE); return; }
  const int t = tbl_find(L, eord);  // canTriggerElement: the catch event is ACTIVATED with its event scope
  if (t < 0 || ((tget(L, t).y >> 16) & 0xFF) != ZBHIP_PI_ELEMENT_ACTIVATED) { set_fail(L, FB_MESSAGE); return; }
  const uint32_t intr = (L.pm_x >> 14) & 1;
  const bool boundary = etype(elem_of(L, elem)) == ZBHIP_EL_BOUNDARY_EVENT;
  // an interrupting boundary event terminates its activity first (the command's context travels in
  // the lane: past the batch limit it would be written unprocessed -- outside the device subset)
  if (boundary && intr && pending(L) + L.processed + 1 >= L.limit) { set_fail(L, FB_BATCH_LIMIT); return; }
  emit_msg(L, C_PMS_CORRELATED, iref(L, L.pm_y >> 16), eik_p, pik_p, msg_p, corr, nb, part, intr, elem);
  // ProcessMessageSubscriptionCorrelatedApplier (:27-37): interrupting -> removed; otherwise
  // updateToOpenedState(record): open, the record the CORRELATED one (its message key)
  if (intr) L.pm_x = L.pm_y = L.pm_z = L.pm_w = 0;
  else L.pm_msg = msg_p;
  const uint32_t pe = new_key(L);
  emit(L, C_PE_TRIGGERING, pe, eord, elem);
  L.trig_key = (uint16_t)eord;
  if (boundary && !intr) {
    // a non-interrupting boundary event: EventHandle.activateElement -> activateTriggeredEvent in this
    // batch; the activity stays active (its EVENT_TRIGGER row is deleted by TRIGGERED)
    L.trig_key = NONE;
    activate_triggered_event(L, pe, eord, elem, scope_key(L, 0));
  } else if (boundary) {
    // EventHandle.activateElement for a boundary event: TERMINATE_ELEMENT of the activity (its
    // onTerminate activates the event with the trigger's PROCESS_EVENT key)
    L.trig_evt = (uint16_t)pe;
    follow_up(L, ZBHIP_PI_TERMINATE_ELEMENT, eord, 0, tget(L, t).x & 0xFFFF, false, true, eord, Q_TERM);
  } else {
    follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, eord, 0, elem, true, true, eord);
  }
  // sendAcknowledgeCommand -> SubscriptionCommandSender.correlateMessageSubscription (sender partition)
  if ((int32_t)part == L.sp->partition_id) {
    emit_msg(L, C_MS_CORRELATE, -1, eik_p, pik_p, -1, ZBHIP_NO_STRING, nb, 0, 1, kNoElem);
    L.lq_slot = corr;
    L.lq_eord = eord;
    L.lq_name_bpmn = nb;
    L.lq_eik = eik_p;
    L.lq_pik = pik_p;
    L.lq_row = L.inst;
    push_local(L, LQ_MS_CORRELATE);
  } else {
    send_xpart(L, ZBHIP_CMD_MSG_SUB_CORRELATE, part, eik, pik, -1, corr, L.inst, eord, nb, 1);
  }
}

// MessageSubscriptionCorrelateProcessor.processRecord: CORRELATED (the stored record) or NOT_FOUND
template <class K>
__device__ __forceinline__ void ms_correlate(Lane<K>& L, uint32_t slot, uint32_t pi_part, uint32_t inst, uint32_t eord,
                                             uint32_t nb, long long eik_p, long long pik_p) {
  const StepParams& P = *L.sp;
  if (slot < P.st.n_slots && engine_owned(P, slot)) { set_fail(L, FB_MESSAGE); return; }
  const int r = slot < P.st.n_slots ? find_row(L, slot, pi_part, inst, eord, nb & 0xFFFF) : -1;
  if (r < 0) {
    emit_msg(L, kRejectBit | C_MS_CORRELATE, -1, eik_p, pik_p, -1, ZBHIP_NO_STRING, nb, 0, 1, kNoElem,
             ZBHIP_REASON_MS_CORR_NOT_FOUND);
    return;
  }
  if (r == kSubs) { set_fail(L, FB_MESSAGE); return; }  // correlate of a row opened in this very batch
  const size_t ri = sub_ri(r, slot);
  const uint4 a = P.st.sub_a[ri];
  const longlong2 b = P.st.sub_b[ri];
  const longlong2 k = P.st.sub_k[ri];
  const long long msg = (L.op_corr_mask >> r) & 1 ? L.op_corr_msg : k.y;
  const uint32_t intr = (a.x >> 8) & 1;
  emit_msg(L, C_MS_CORRELATED, k.x, b.x, b.y, msg, slot, a.y, 0, intr, kNoElem);
  if (!intr) {
    // MessageSubscriptionCorrelatedApplier (:26-37), non-interrupting: updateToCorrelatedState -- open
    // again, the message key kept (at commit); correlateNextMessage finds no buffered message (the
    // subset's messages live for their PUBLISH batch only)
    if (L.op_open_mask && L.op_open_slot != slot) { set_fail(L, FB_MESSAGE); return; }
    L.op_open_mask |= 1u << r;
    L.op_open_slot = slot;
    return;
  }
  // MessageSubscriptionCorrelatedApplier: interrupting -> removed (at commit)
  if (L.op_rm_mask && L.op_rm_slot != slot) { set_fail(L, FB_MESSAGE); return; }
  L.op_rm_mask |= 1u << r;
  L.op_rm_slot = slot;
}

// CatchEventBehavior.unsubscribeFromMessageEvent (processing/common/CatchEventBehavior.java:407-432):
// PROCESS_MESSAGE_SUBSCRIPTION:DELETING with the stored subscription (ProcessMessageSubscriptionDeletingApplier
// -> updateToClosingState), then MESSAGE_SUBSCRIPTION:DELETE to the subscription partition
// (SubscriptionCommandSender.closeMessageSubscription, :220-236: pik, eik, messageKey -1, name)
template <class K>
__device__ __forceinline__ void unsubscribe_message(Lane<K>& L) {
  const uint32_t eord = L.pm_y & 0xFFFF, part = L.pm_x >> 16, corr = L.pm_z, nb = L.pm_w, st0 = (L.pm_x >> 12) & 3;
  emit_msg(L, C_PMS_DELETING, iref(L, L.pm_y >> 16), iref(L, eord), iref(L, 0), L.pm_msg, corr, nb, part,
           (L.pm_x >> 14) & 1, L.pm_x & 0xFFF);
  L.pm_x |= 3u << 12;
  const uint32_t name_only = (nb & 0xFFFF) | 0xFFFF0000u;
  if ((int32_t)part == L.sp->partition_id) {
    emit_msg(L, C_MS_DELETE, -1, iref(L, eord), iref(L, 0), -1, ZBHIP_NO_STRING, name_only, 0, 1, kNoElem);
    L.lq_slot = corr;
    L.lq_name_bpmn = nb;
    L.lq_eord = eord;
    L.lq_eik = cref_inst(L, eord);
    L.lq_pik = L.pik;
    push_local(L, LQ_MS_DELETE);
  } else {
    // the real key the acknowledgement brought (an OPENING subscription -- the job completed before the
    // acknowledgement arrived -- has none here: outside the subset)
    const long long eik = L.inst < L.sp->st.n ? L.sp->st.pms_eik[L.inst] : -1;
    if (eik < 0 || st0 != 2) { set_fail(L, FB_MESSAGE); return; }
    // (the entry carries the subscription's bpmnProcessId as the other sends do; the DELETE's record
    // value leaves it empty -- the receiver builds it per kind)
    send_xpart(L, ZBHIP_CMD_MSG_SUB_DELETE, part, eik, L.pik, -1, corr, L.inst, eord, nb, 1);
  }
}

// MessageSubscriptionDeleteProcessor.processRecord (processing/message/MessageSubscriptionDeleteProcessor.java:50-68):
// MESSAGE_SUBSCRIPTION:DELETED with the stored subscription (MessageSubscriptionDeletedApplier removes the
// row at commit), then the acknowledgement PROCESS_MESSAGE_SUBSCRIPTION:DELETE (closeProcessMessageSubscription,
// SubscriptionCommandSender.java:267-283).  No such subscription (NOT_FOUND) is outside the subset.
template <class K>
__device__ __forceinline__ void ms_delete(Lane<K>& L, uint32_t slot, uint32_t pi_part, uint32_t inst, uint32_t eord,
                                          uint32_t nb, long long eik_p, long long pik_p, long long eik, long long pik) {
  const StepParams& P = *L.sp;
  const int r = slot < P.st.n_slots && !engine_owned(P, slot) ? find_row(L, slot, pi_part, inst, eord, nb & 0xFFFF) : -1;
  if (r < 0 || r == kSubs) { set_fail(L, FB_MESSAGE); return; }
  const size_t ri = sub_ri(r, slot);
  const uint4 a = P.st.sub_a[ri];
  const longlong2 b = P.st.sub_b[ri];
  const longlong2 k = P.st.sub_k[ri];
  const long long msg = (L.op_corr_mask >> r) & 1 ? L.op_corr_msg : k.y;
  emit_msg(L, C_MS_DELETED, k.x, b.x, b.y, msg, slot, a.y, 0, (a.x >> 8) & 1, kNoElem);
  if (L.op_rm_mask && L.op_rm_slot != slot) { set_fail(L, FB_MESSAGE); return; }
  L.op_rm_mask |= 1u << r;
  L.op_rm_slot = slot;
  const uint32_t name_only = (nb & 0xFFFF) | 0xFFFF0000u;
  if ((int32_t)pi_part == P.partition_id) {
    emit_msg(L, C_PMS_DELETE, -1, eik_p, pik_p, -1, ZBHIP_NO_STRING, name_only, (uint32_t)P.partition_id, 1, kNoElem);
    L.lq_eord = eord;
    L.lq_name_bpmn = nb;
    L.lq_eik = eik;
    L.lq_pik = pik;
    L.lq_row = inst;
    push_local(L, LQ_PMS_DELETE);
  } else {
    send_xpart(L, ZBHIP_CMD_PMS_DELETE, pi_part, eik, pik, -1, ZBHIP_NO_STRING, inst, eord, name_only, 1);
  }
}

// ProcessMessageSubscriptionDeleteProcessor.processRecord (processing/message/
// ProcessMessageSubscriptionDeleteProcessor.java:39-56): PROCESS_MESSAGE_SUBSCRIPTION:DELETED with the stored
// subscription (ProcessMessageSubscriptionDeletedApplier removes it) -- also after the instance ended
template <class K>
__device__ __forceinline__ void pms_delete(Lane<K>& L, uint32_t eord, uint32_t name) {
  const uint32_t st = (L.pm_x >> 12) & 3;
  if (st == 0 || (L.pm_y & 0xFFFF) != eord || (L.pm_w & 0xFFFF) != name) { set_fail(L, FB_MESSAGE); return; }
  emit_msg(L, C_PMS_DELETED, iref(L, L.pm_y >> 16), iref(L, eord), iref(L, 0), L.pm_msg, L.pm_z, L.pm_w, L.pm_x >> 16,
           (L.pm_x >> 14) & 1, L.pm_x & 0xFFF);
  L.pm_x = L.pm_y = L.pm_z = L.pm_w = 0;
  L.pm_msg = -1;
}

// sort key of a subscription's element instance key for the visit order of
// MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY [tenant, name, correlationKey, elementInstanceKey]:
// (partition, pending-in-this-window, key or (command, ordinal)) -- a key this window generated is
// newer than every real key of its partition
__device__ __forceinline__ unsigned long long eik_order(long long eik, uint32_t part) {
  if (eik >= 0) return (unsigned long long)eik;
  const unsigned long long v = (unsigned long long)(-2 - eik);
  return ((unsigned long long)part << 51) | (1ull << 50) | (v & ((1ull << 50) - 1));
}

// MessagePublishProcessor.handleNewMessage (processing/message/MessagePublishProcessor.java):
// PUBLISHED (+key), CORRELATING per open subscription (first per bpmnProcessId, element instance
// key order), PROCESS_MESSAGE_SUBSCRIPTION:CORRELATE sends, EXPIRED (time-to-live 0)
template <class K>
__device__ __forceinline__ void publish_message(Lane<K>& L, uint32_t slot, uint32_t name) {
  const StepParams& P = *L.sp;
  if (slot >= P.st.n_slots || engine_owned(P, slot)) { set_fail(L, FB_MESSAGE); return; }
  const uint32_t msg = new_slot_key(L);
  const uint32_t nb_msg = name | 0xFFFF0000u;
  emit_msg(L, C_MSG_PUBLISHED, sref(L, msg), -1, -1, -1, slot, nb_msg, 0, 0, kNoElem);
  const long long msg_ref = ref_cmd(L.ci, false, msg);
  // selection sort of the slot's open rows by element instance key
  uint32_t done = 0, chosen[kSubs], nch = 0, bpmn_seen[kSubs];
  for (int it = 0; it < kSubs; ++it) {
    int best = -1;
    unsigned long long bk = ~0ull;
    for (int r = 0; r < kSubs; ++r) {
      if ((done >> r) & 1) continue;
      const size_t ri = sub_ri(r, slot);
      const uint4 a = P.st.sub_a[ri];
      if (!((a.x & 0xFF) == 1 || (a.x & 0xFF) == 2) || (a.y & 0xFFFF) != name) { done |= 1u << r; continue; }
      const unsigned long long o = eik_order(P.st.sub_b[ri].x, a.x >> 16);
      if (o < bk) { bk = o; best = r; }
    }
    if (best < 0) break;
    done |= 1u << best;
    const size_t ri = sub_ri(best, slot);
    const uint4 a = P.st.sub_a[ri];
    bool seen = false;
    for (uint32_t j = 0; j < nch; ++j) seen |= bpmn_seen[j] == (a.y >> 16);
    if ((a.x & 0xFF) == 2 || seen) continue;  // correlating, or this process already correlates
    const longlong2 b = P.st.sub_b[ri];
    emit_msg(L, C_MS_CORRELATING, P.st.sub_k[ri].x, b.x, b.y, sref(L, msg), slot, a.y, 0, (a.x >> 8) & 1, kNoElem);
    bpmn_seen[nch] = a.y >> 16;
    chosen[nch++] = (uint32_t)best;
    L.op_corr_mask |= 1u << best;  // MessageSubscriptionCorrelatingApplier (at commit)
  }
  L.op_corr_msg = msg_ref;
  // sendCorrelateCommand: SubscriptionCommandSender.correlateProcessMessageSubscription
  for (uint32_t j = 0; j < nch; ++j) {
    const size_t ri = sub_ri(chosen[j], slot);
    const uint4 a = P.st.sub_a[ri];
    const longlong2 b = P.st.sub_b[ri];
    const uint32_t target = a.x >> 16;
    if ((int32_t)target == P.partition_id) {
      emit_msg(L, C_PMS_CORRELATE, -1, b.x, b.y, sref(L, msg), slot, a.y, (uint32_t)P.partition_id, 1, kNoElem);
      if (L.lq_row != kNoInst) { set_fail(L, FB_MESSAGE); return; }  // one local instance per batch
      L.lq_row = a.z;
      L.lq_eord = a.w & 0xFFFF;
      L.lq_name_bpmn = a.y;
      L.lq_eik = b.x;
      L.lq_pik = b.y;
      L.lq_msg = sref(L, msg);
      L.lq_corr = slot;
      push_local(L, LQ_PMS_CORRELATE);
    } else {
      send_xpart(L, ZBHIP_CMD_PMS_CORRELATE, target, b.x, b.y, msg_ref, slot, a.z, a.w & 0xFFFF, a.y, (a.x >> 8) & 1);
    }
  }
  emit_msg(L, C_MSG_EXPIRED, sref(L, msg), -1, -1, -1, slot, nb_msg, 0, 0, kNoElem);
}

// ---- TIMER:TRIGGER (K::S) --------------------------------------------------------------------
// EventTriggerBehavior.activateTriggeredEvent (processing/common/EventTriggerBehavior.java:191-244):
// PROCESS_EVENT:TRIGGERED under the trigger's key (aux: its event scope), the triggered event's
// ACTIVATING + ACTIVATED (+key, flow scope fsa) and its COMPLETE_ELEMENT
template <class K>
__device__ __forceinline__ void activate_triggered_event(Lane<K>& L, uint32_t pe, uint32_t scope, uint32_t target,
                                                         uint32_t fsa) {
  emit(L, C_PE_TRIGGERED, pe, scope, target);
  const uint32_t bk = new_key(L);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, bk, fsa, target);
  apply_activating_child(L, target, elem_of(L, target), bk);
  if (L.fail) return;
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, bk, fsa, target);
  tbl_set_state(L, tbl_find(L, bk), ZBHIP_PI_ELEMENT_ACTIVATED);
  follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, bk, fsa, target, true, true, bk);
}

// TriggerTimerProcessor.processRecord (processing/timer/TriggerTimerProcessor.java:81-114) for the
// instance's timer: NOT_FOUND / INVALID_STATE rejections, TIMER:TRIGGERED (the command's key),
// TimerTriggeredApplier (the row removed), then EventHandle.activateElement (EventHandle.java:104-131):
// PROCESS_EVENT:TRIGGERING (+key, no variables) and COMPLETE_ELEMENT for the catch event
template <class K>
__device__ __forceinline__ void trigger_timer(Lane<K>& L, uint32_t tord, long long cmd_due) {
  if (L.proc == NONE || !L.pi_live || !(L.tm_y >> 31) || (L.tm_x >> 16) != tord) {
    emit(L, kRejectBit | C_TIMER_TRIGGER, tord, NONE, NONE, ZBHIP_REASON_TIMER_NOT_FOUND);
    return;
  }
  const uint32_t eord = L.tm_y & 0xFFFF, elem = L.tm_x & 0xFFF;
  const int t = tbl_find(L, eord);  // canTriggerElement: the catch event is ACTIVATED, its scope accepting
  if (t < 0 || ((tget(L, t).y >> 16) & 0xFF) != ZBHIP_PI_ELEMENT_ACTIVATED) {
    emit(L, kRejectBit | C_TIMER_TRIGGER, tord, NONE, NONE, ZBHIP_REASON_TIMER_NOT_ACTIVE);
    return;
  }
  const uint32_t reps = (L.tm_y >> 16) & 0xFF;  // TimerRecord.repetitions (255: infinite)
  emit(L, C_TIMER_TRIGGERED, tord, eord, elem, reps);
  L.tm_x = L.tm_y = 0;
  L.tm_due = 0;
  const uint32_t pe = new_key(L);
  emit(L, C_PE_TRIGGERING, pe, eord, elem);
  L.trig_key = (uint16_t)eord;  // ProcessEventTriggeringApplier: EVENT_TRIGGER row (no variables)
  const uint4 bw = elem_of(L, elem);
  if (etype(bw) == ZBHIP_EL_BOUNDARY_EVENT && (bw.w & 1) == 0) {
    // a non-interrupting boundary event: EventHandle.activateElement -> activateTriggeredEvent in
    // this batch; the activity stays active (its EVENT_TRIGGER row is deleted by TRIGGERED)
    L.trig_key = NONE;
    const uint32_t task = tget(L, t).x & 0xFFFF;
    const uint32_t c = scope_of<K>(elem_of(L, task));
    activate_triggered_event(L, pe, eord, elem, scope_key(L, c));
    // shouldReschedule / rescheduleTimer (TriggerTimerProcessor.java:116-160): a cycle's next timer
    // from the command's dueDate (refreshTimer: Interval.withStart), one repetition fewer; a start
    // already past counts from the clock instead (Interval.toEpochMilli, Interval.java:77-93)
    if (reps == 255 || reps > 1) {
      const uint32_t nr = reps == 255 ? 255u : reps - 1;
      const uint32_t tk = new_key(L);
      L.tm_x = elem | (tk << 16);
      L.tm_y = eord | (nr << 16) | (1u << 31);
      L.tm_due = next_cycle_due(cmd_due, (long long)bw.z, L.sp->now_ms);
      emit(L, C_TIMER_NEXT, tk, eord, elem, nr);
    }
    return;
  }
  if (etype(bw) == ZBHIP_EL_BOUNDARY_EVENT) {
    // an interrupting boundary event: TERMINATE_ELEMENT of the activity it is attached to (the
    // activation of the boundary event follows its termination, terminate_pi); the trigger's
    // PROCESS_EVENT key travels with the EVENT_TRIGGER row.  Past the batch limit the command
    // would be written unprocessed with that context: outside the device subset.
    if (pending(L) + L.processed + 1 >= L.limit) { set_fail(L, FB_BATCH_LIMIT); return; }
    L.trig_evt = (uint16_t)pe;
    const uint32_t task = tget(L, t).x & 0xFFFF;
    const uint32_t c = scope_of<K>(elem_of(L, task));
    follow_up(L, ZBHIP_PI_TERMINATE_ELEMENT, eord, scope_key(L, c), task, false, c == 0, eord, Q_TERM);
    // a cycle reschedules here too (shouldReschedule does not look at the activity): TIMER:CREATED after the
    // TERMINATE_ELEMENT command; the activity's termination cancels that timer again
    if (reps == 255 || reps > 1) {
      const uint32_t nr = reps == 255 ? 255u : reps - 1;
      const uint32_t tk = new_key(L);
      L.tm_x = elem | (tk << 16);
      L.tm_y = eord | (nr << 16) | (1u << 31);
      L.tm_due = next_cycle_due(cmd_due, (long long)bw.z, L.sp->now_ms);
      emit(L, C_TIMER_NEXT, tk, eord, elem, nr);
    }
    return;
  }
  const uint32_t c = scope_of<K>(elem_of(L, elem));
  follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, eord, scope_key(L, c), elem, true, c == 0, eord);
}

// CatchEventBehavior.unsubscribeFromTimerEvent (processing/common/CatchEventBehavior.java:380-392):
// TIMER:CANCELED with the timer's key and stored value; TimerCancelledApplier removes the row.  The
// dueDate of a timer stored before the batch goes to the command's cmd_due entry (one timer row per
// instance: at most one such cancel per batch); a timer the batch created itself is due at the clock
// plus its duration, which the host and the log writer derive from the key (one of the batch's own)
template <class K>
__device__ __forceinline__ void cancel_timer(Lane<K>& L) {
  emit(L, C_TIMER_CANCELED, L.tm_x >> 16, L.tm_y & 0xFFFF, L.tm_x & 0xFFF, (L.tm_y >> 16) & 0xFF);
  if ((L.tm_x >> 16) < L.first_ord) L.sp->cmd_due[L.ci] = L.tm_due;
  L.tm_x = L.tm_y = 0;
  L.tm_due = 0;
}

// BpmnStateTransitionBehavior.onElementTerminated (:419-441) of a child of container c: the
// container's onChildTerminated.  A sub-process (SubProcessProcessor.onChildTerminated :108-160) with no
// active child left: with its boundary event's trigger (the flow scope active) transitionToTerminated
// and activateTriggeredEvent; terminated by its own flow scope, transitionToTerminated and the same one
// level up.  Children of the process (a cancel) or of a multi-instance body: outside the subset.
template <class K>
__device__ __forceinline__ void child_terminated(Lane<K>& L, uint32_t c) {
  if constexpr (K::S) {
    for (int d = 0; d < kMaxDepth; ++d) {
      if (c == 0) { set_fail(L, FB_UNSUPPORTED); return; }
      const uint4 cw = elem_of(L, c);
      const uint32_t ct = etype(cw);
      if (ct != ZBHIP_EL_SUB_PROCESS && ct != ZBHIP_EL_MULTI_INSTANCE_BODY) { set_fail(L, FB_UNSUPPORTED); return; }
      const int tc = scope_find(L, c);
      if (tc < 0) { set_fail(L, FB_UNSUPPORTED); return; }
      const uint2 ce = tget(L, tc);
      const uint32_t ckey = ce.x >> 16, cst = (ce.y >> 16) & 0xFF;
      const uint32_t pc = scope_of<K>(cw);
      const uint32_t pfsa = scope_key(L, pc);
      if (ct == ZBHIP_EL_MULTI_INSTANCE_BODY) {
        // MultiInstanceBodyProcessor.onChildTerminated (:232-247): a body that is not terminating (its
        // completion condition was met) completes once no child is active
        if (cst != ZBHIP_PI_ELEMENT_TERMINATING) {
          if ((ce.y & 0xFF) == 0) follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, ckey, pfsa, c, true, pc == 0, ckey);
          return;
        }
        // a terminating body (:244-247, terminate :282-315) once no inner instance is active:
        // transitionToTerminated and onElementTerminated; with its own boundary event's trigger
        // (activateTriggeredEvent in between) outside the subset
        if ((ce.y & 0xFF) != 0) return;
        if (L.trig_key == ckey && L.trig_evt != NONE) { set_fail(L, FB_UNSUPPORTED); return; }
        emit(L, ZBHIP_PI_ELEMENT_TERMINATED, ckey, pfsa, c);
        apply_completed_child(L, tc, ckey);
        c = pc;
        continue;
      }
      if ((ce.y & 0xFF) != 0) return;  // canBeTerminated: a child is still active
      const uint32_t pst = pc == 0 ? (L.pi_live ? (uint32_t)L.pi_state : 0u) : (tget(L, scope_find(L, pc)).y >> 16) & 0xFF;
      const uint32_t target = cw.w & 0xFFFF;  // the sub-process's boundary event
      if (L.trig_key == ckey && L.trig_evt != NONE && pst == ZBHIP_PI_ELEMENT_ACTIVATED && target != 0xFFFF) {
        const uint32_t pe = L.trig_evt;
        emit(L, ZBHIP_PI_ELEMENT_TERMINATED, ckey, pfsa, c);
        apply_completed_child(L, tc, ckey);
        L.trig_evt = NONE;
        activate_triggered_event(L, pe, ckey, target, pfsa);
        return;
      }
      if (cst != ZBHIP_PI_ELEMENT_TERMINATING) return;
      emit(L, ZBHIP_PI_ELEMENT_TERMINATED, ckey, pfsa, c);
      apply_completed_child(L, tc, ckey);
      c = pc;
    }
    set_fail(L, FB_UNSUPPORTED);
  } else {
    (void)c;
    set_fail(L, FB_UNSUPPORTED);
  }
}

// TERMINATE_ELEMENT (ProcessInstanceStateTransitionGuard :60-64, transitionToTerminating), then the
// processor's onTerminate:
// - a job worker task (JobWorkerTaskProcessor.onTerminate, task/JobWorkerTaskProcessor.java:77-104):
//   cancelJob (JOB:CANCELED, BpmnJobBehavior.java:251-274), unsubscribeFromEvents, then findEventTrigger
//   while its flow scope is active: transitionToTerminated (the instance removed like a completed one)
//   and EventTriggerBehavior.activateTriggeredEvent (EventTriggerBehavior.java:191-244: PROCESS_EVENT
//   :TRIGGERED, the boundary event ACTIVATING + ACTIVATED (+key, the activity's flow scope),
//   COMPLETE_ELEMENT); without one (terminated by its flow scope) transitionToTerminated and
//   onElementTerminated;
// - an intermediate catch event: unsubscribeFromEvents, transitionToTerminated, onElementTerminated;
// - a sub-process (SubProcessProcessor.onTerminate :84-95): unsubscribeFromEvents (its boundary
//   timer), terminateChildInstances (BpmnStateTransitionBehavior.java:348-363): with children
//   PROCESS_INSTANCE_BATCH:TERMINATE (+key), else onChildTerminated at once
template <class K>
__device__ __forceinline__ void terminate_pi(Lane<K>& L, uint32_t elem, uint4 w, uint32_t key, uint32_t fsa) {
  const int t = tbl_find(L, key);
  const uint32_t st = t < 0 ? 0u : (tget(L, t).y >> 16) & 0xFF;
  const uint32_t type = etype(w);
  const bool ok_type = ZBHIP_IS_JOB_WORKER(type) || (K::S && (type == ZBHIP_EL_SUB_PROCESS || type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT ||
                                                              type == ZBHIP_EL_MULTI_INSTANCE_BODY));
  if (t < 0 || !ok_type ||
      (st != ZBHIP_PI_ELEMENT_ACTIVATING && st != ZBHIP_PI_ELEMENT_ACTIVATED && st != ZBHIP_PI_ELEMENT_COMPLETING)) {
    set_fail(L, FB_UNSUPPORTED);
    return;
  }
  const uint32_t c = scope_of<K>(w);
  if constexpr (K::S) {
    if (type == ZBHIP_EL_SUB_PROCESS || type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
      // (a multi-instance body the same way: MultiInstanceBodyProcessor.onTerminate :116-125)
      const uint32_t nch = tget(L, t).y & 0xFF;  // childCount
      // the termination's commands stay in this batch (the trigger's context travels in the lane)
      if (pending(L) + L.processed + 2 + nch >= L.limit) { set_fail(L, FB_BATCH_LIMIT); return; }
      emit(L, ZBHIP_PI_ELEMENT_TERMINATING, key, fsa, elem);
      tbl_set_state(L, t, ZBHIP_PI_ELEMENT_TERMINATING);
      if ((L.tm_y >> 31) && (L.tm_y & 0xFFFF) == key) cancel_timer(L);
      if (nch == 0) {
        child_terminated(L, elem);  // onChildTerminated(element, terminating, null)
      } else {
        const uint32_t kb = new_key(L);
        follow_up(L, C_PIB_TERMINATE, kb, key, elem, false, false, key, Q_TERM | Q_PIBT);
      }
      return;
    }
  }
  emit(L, ZBHIP_PI_ELEMENT_TERMINATING, key, fsa, elem);
  tbl_set_state(L, t, ZBHIP_PI_ELEMENT_TERMINATING);
  const uint2 e = tget(L, t);
  if (ZBHIP_IS_JOB_WORKER(type)) {
    const uint32_t job = e.y & 0xFFFF;
    // (flag 1: the job was ACTIVATED -- its record carries the stored deadline and worker)
    if (((e.y >> 24) & 1u) && job != JOB_ZERO && job != JOB_MINUS1) {
      emit(L, C_JOB_CANCELED, job, key, elem, (e.y >> 25) & 1u);
      if ((e.y >> 25) & 1u) note_activation(L, job, L.inst);
    }
  }
  if constexpr (K::S) {  // unsubscribeFromEvents: the timer, then message subscriptions
    if ((L.tm_y >> 31) && (L.tm_y & 0xFFFF) == key) cancel_timer(L);
  }
  if constexpr (K::M) {
    if (((L.pm_x >> 12) & 3) != 0 && (L.pm_y & 0xFFFF) == key) unsubscribe_message(L);
    if (L.fail) return;
  }
  const uint32_t fst = c == 0 ? (L.pi_live ? (uint32_t)L.pi_state : 0u) : (tget(L, scope_find(L, c)).y >> 16) & 0xFF;
  const uint32_t target = ZBHIP_IS_JOB_WORKER(type) ? w.w & 0xFFFF : 0xFFFFu;  // the activity's boundary event
  if (L.trig_key == key && L.trig_evt != NONE && fst == ZBHIP_PI_ELEMENT_ACTIVATED && target != 0xFFFF) {
    const uint32_t pe = L.trig_evt;
    emit(L, ZBHIP_PI_ELEMENT_TERMINATED, key, fsa, elem);
    apply_completed_child(L, t, key);  // removeInstance; the event scope with its trigger
    L.trig_evt = NONE;
    activate_triggered_event(L, pe, key, target, fsa);
    return;
  }
  // terminated by its flow scope: transitionToTerminated, onElementTerminated
  emit(L, ZBHIP_PI_ELEMENT_TERMINATED, key, fsa, elem);
  apply_completed_child(L, t, key);
  child_terminated(L, c);
}

// TerminateProcessInstanceBatchProcessor (processing/processinstance/TerminateProcessInstanceBatchProcessor
// .java:38-85): TERMINATE_ELEMENT of every child of the container that can terminate (ACTIVATING /
// ACTIVATED / COMPLETING), in ELEMENT_INSTANCE_PARENT_CHILD (child key) order
template <class K>
__device__ __forceinline__ void terminate_batch(Lane<K>& L, uint32_t container, uint32_t ckey) {
  if constexpr (K::S) {
    static_assert(K::T <= 32, "one mask bit per table entry");
    uint32_t done = 0;
    for (int it = 0; it < K::T && !L.fail; ++it) {
      int best = -1;
      uint32_t bk = 0xFFFFFFFFu;
      for (int t = 0; t < L.nt; ++t) {
        if ((done >> t) & 1u) continue;
        const uint2 e = tget(L, t);
        if (e.x == 0xFFFFFFFFu) continue;
        const uint32_t el = e.x & 0xFFFF, k = e.x >> 16, st = (e.y >> 16) & 0xFF;
        if (scope_of<K>(elem_of(L, el)) != container || (st != ZBHIP_PI_ELEMENT_ACTIVATING &&
            st != ZBHIP_PI_ELEMENT_ACTIVATED && st != ZBHIP_PI_ELEMENT_COMPLETING))
          continue;
        if (k < bk) { bk = k; best = t; }
      }
      if (best < 0) return;
      done |= 1u << best;
      const uint32_t el = tget(L, best).x & 0xFFFF;
      follow_up(L, ZBHIP_PI_TERMINATE_ELEMENT, bk, ckey, el, false, false, bk, Q_TERM);
    }
  } else {
    (void)container;
    (void)ckey;
    set_fail(L, FB_UNSUPPORTED);
  }
}

// ActivateProcessInstanceBatchProcessor.processRecord (processing/processinstance/
// ActivateProcessInstanceBatchProcessor.java:44-60): an ACTIVATE_ELEMENT of the inner activity per
// child still to activate, each with a new key, flow scope = the body (createChildInstanceRecord
// :62-84); never split into a follow-up batch command at these record sizes (canWriteCommands)
template <class K>
__device__ __forceinline__ void activate_batch(Lane<K>& L, uint32_t body, uint4 w) {
  const int tb = scope_find(L, body);
  if (tb < 0) { set_fail(L, FB_UNSUPPORTED); return; }
  const uint32_t bk = tget(L, tb).x >> 16, inner = w.z & 0xFFF;
  uint32_t n, list;  // (ActivateProcessInstanceBatchProcessor: the record's index -- the collection's size)
  if (!mi_collection(L, body, w, bk, scope_of<K>(w), n, list)) return;
  for (uint32_t i = 0; i < n && !L.fail; ++i) {
    const uint32_t k = new_key(L);
    follow_up(L, ZBHIP_PI_ACTIVATE_ELEMENT, k, bk, inner, false, false, k);
  }
}

// ---- BpmnStreamProcessor.processRecord for one PI command ----------------------------------
template <class K>
__device__ __forceinline__ void reject_pi(Lane<K>& L, bool complete, uint32_t elem, uint32_t key, uint32_t aux,
                                          uint32_t reason, uint32_t arg) {
  emit(L, kRejectBit | (complete ? ZBHIP_PI_COMPLETE_ELEMENT : ZBHIP_PI_ACTIVATE_ELEMENT), key, aux, elem,
       reason | (arg << 4));
}

template <class K>
__device__ __forceinline__ void process_pi(Lane<K>& L, uint32_t entry) {
  const uint32_t elem = entry & 0xFFF;
  const bool complete = (entry >> 12) & 1;
  const bool fs_pi = (entry >> 13) & 1;
  const uint32_t cmd_key = entry >> 16;
  const uint4 w = elem_of(L, elem);
  const uint32_t type = etype(w);
  // flowScopeKey of the element's records and rejections: the process's children 0 (K::S: the
  // instance of the element's container), the process itself -1
  const uint32_t c = scope_of<K>(w);
  uint32_t fsa = 0, raux = fs_pi ? 0u : (uint32_t)NONE;
  if constexpr (K::S) {
    if (type != ZBHIP_EL_PROCESS) {
      fsa = scope_key(L, c);  // a container without an instance (never in the subset): fallback
      if (L.fail) return;
      raux = fsa;
    }
    if (entry & Q_TERM) {
      if (entry & Q_PIBT) terminate_batch(L, elem, cmd_key);  // PROCESS_INSTANCE_BATCH:TERMINATE of a container
      else if (complete) activate_batch(L, elem, w);         // PROCESS_INSTANCE_BATCH:ACTIVATE of a body
      else terminate_pi(L, elem, w, cmd_key, fsa);
      return;
    }
  } else if constexpr (K::M) {
    if (entry & Q_TERM) {  // TERMINATE_ELEMENT of an activity whose message boundary event was triggered
      if (complete) set_fail(L, FB_UNSUPPORTED);
      else terminate_pi(L, elem, w, cmd_key, fsa);
      return;
    }
  }

  if (!complete) {
    // ---- ACTIVATE_ELEMENT: guard (:47-70) ----
    if (type != ZBHIP_EL_PROCESS) {
      if (c != 0) {  // K::S: the flow scope is a sub-process instance (found by scope_key)
        const uint32_t fst = (tget(L, scope_find(L, c)).y >> 16) & 0xFF;
        if (fst != ZBHIP_PI_ELEMENT_ACTIVATED) { reject_pi(L, false, elem, cmd_key, raux, ZBHIP_REASON_FS_STATE, fst); return; }
      } else if (!L.pi_live) {
        reject_pi(L, false, elem, cmd_key, raux, ZBHIP_REASON_FS_NOT_FOUND, 0);
        return;
      } else if (L.pi_state != ZBHIP_PI_ELEMENT_ACTIVATED) {
        reject_pi(L, false, elem, cmd_key, raux, ZBHIP_REASON_FS_STATE, L.pi_state);
        return;
      }
      if (type == ZBHIP_EL_PARALLEL_GATEWAY) {  // canActivateParallelGateway (:169-186)
        uint32_t base = w.w & 0xFFFF, n = w.x >> 16, taken = 0;
        for (uint32_t s = base; s < base + n; ++s) taken += join_get(L, s) > 0;
        if (taken < n) { reject_pi(L, false, elem, cmd_key, raux, ZBHIP_REASON_PGW_NOT_ALL_TAKEN, 0); return; }
      }
    }
    // transitionToActivating (:72-100)
    if (type == ZBHIP_EL_PROCESS) {
      if (L.pi_live) { set_fail(L, FB_UNSUPPORTED); return; }
      emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, cmd_key, NONE, 0);
      L.pi_live = true;
      L.pi_state = ZBHIP_PI_ELEMENT_ACTIVATING;
      L.pi_child = 0;
      L.pi_asf = 0;
      // ProcessProcessor.onActivate (:55-61,119-128)
      emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, cmd_key, NONE, 0);
      L.pi_state = ZBHIP_PI_ELEMENT_ACTIVATED;
      uint32_t start = L.pb[0] >> 16;
      follow_up(L, ZBHIP_PI_ACTIVATE_ELEMENT, NONE, 0, start, false, true, NONE);  // activateChildInstance: key -1
      return;
    }
    if (cmd_key != NONE && tbl_find(L, cmd_key) >= 0) { set_fail(L, FB_UNSUPPORTED); return; }
    // an error end event (EndEventProcessor.ErrorEndEventBehavior): its error is thrown by the engine -- the
    // command that reaches it hands the instance off
    if (type == ZBHIP_EL_END_EVENT && ((w.x >> 8) & 0xFF) == ZBHIP_EV_ERROR) { set_fail(L, FB_UNSUPPORTED); return; }
    const uint32_t key = cmd_key == NONE ? new_key(L) : cmd_key;
    emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, key, fsa, elem);
    apply_activating_child(L, elem, w, key);
    if (L.fail) return;
    const int t = L.nt > 0 ? tbl_find(L, key) : -1;
    if constexpr (K::S) {
      const uint4 bw = elem_of(L, c);
      if (c != 0 && etype(bw) == ZBHIP_EL_MULTI_INSTANCE_BODY) {
        // onElementActivating -> MultiInstanceBodyProcessor.onChildActivating (:129-158) ->
        // setLoopVariables (:270-305): the item at loopCounter - 1 as the inputElement (if any), then
        // loopCounter, local to the inner instance (VARIABLE:CREATED, values from the program)
        const uint32_t loop = tget(L, t).y >> 26;
        const uint4 ext = mi_ext(L, c);
        uint32_t n, list;  // readInputCollectionVariable again: the item at loopCounter - 1
        if (!mi_collection(L, c, bw, key, c, n, list)) return;
        if (loop < 1 || loop > n) { set_fail(L, FB_FEEL); return; }  // (an EXTRACT_VALUE_ERROR incident)
        if ((bw.x >> 16) != 0xFFFFu) {
          const uint32_t ki = new_key(L);
          if ((ext.x & 0xFFFF) == 0xFFFF) emit(L, C_MI_ITEM, ki, key, c, loop);
          else emit(L, C_MI_LIST_ITEM, ki, list & 0xFFFF, list >> 16);
        }
        // the outputElement variable nil-initialized locally, unless it is the inputElement or loopCounter
        const uint32_t oe = ext.y & 0xFFFF;
        if (oe != 0xFFFF && oe != (bw.x >> 16) && oe != (bw.w & 0xFFFF)) emit(L, C_MI_OUTEL, new_key(L), key, c);
        const uint32_t kl = new_key(L);
        emit(L, C_MI_LOOP, kl, key, c, loop);
        if (!ZBHIP_IS_JOB_WORKER(type)) {  // no job: the job field keeps the variables' key
          uint2 e = tget(L, t);
          e.y = (e.y & 0xFFFF0000u) | kl;
          tput(L, t, e);
        }
      }
    }
    switch (type) {
      case ZBHIP_EL_START_EVENT:  // StartEventProcessor.onActivate (:45-50)
      case ZBHIP_EL_TASK:         // UndefinedTaskProcessor.onActivate (task/UndefinedTaskProcessor.java:37-42)
      case ZBHIP_EL_MANUAL_TASK:  // ManualTaskProcessor extends UndefinedTaskProcessor
      case ZBHIP_EL_INTERMEDIATE_THROW_EVENT:  // NoneIntermediateThrowEventBehavior.onActivate (:120-126)
        emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
        tbl_set_state(L, t, ZBHIP_PI_ELEMENT_ACTIVATED);
        follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, key, fsa, elem, true, true, key);
        return;
      case ZBHIP_EL_END_EVENT:  // NoneEndEventBehavior.onActivate/onComplete (:110-134)
        emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
        emit(L, ZBHIP_PI_ELEMENT_COMPLETING, key, fsa, elem);
        transition_to_completed_child(L, t, elem, w, key);
        take_outgoing(L, w);
        return;
      case ZBHIP_EL_SERVICE_TASK:  // JobWorkerTaskProcessor.onActivate (:49-61); the job worker
      case ZBHIP_EL_SEND_TASK:     // send / script / business-rule tasks (BpmnElementProcessors.java:46-60)
      case ZBHIP_EL_SCRIPT_TASK:
      case ZBHIP_EL_BUSINESS_RULE_TASK: {
        if constexpr (K::S) {
          // applyInputMappings, then eventSubscriptionBehavior.subscribeToEvents: the attached
          // boundary event's timer (CatchEventBehavior.subscribeToTimerEvent) before the job; one
          // timer per instance
          if constexpr (K::IO) {
            apply_input_mapping(L, elem, key);
            if (L.fail) return;
          }
          const uint32_t b = w.w & 0xFFFF;
          // (an error boundary event subscribes to nothing: JOB:THROW_ERROR looks it up)
          if (b != 0xFFFF && ((elem_of(L, b).x >> 8) & 0xFF) != ZBHIP_EV_ERROR) {
            if (!L.has_tmr || (L.tm_y >> 31)) { set_fail(L, FB_UNSUPPORTED); return; }
            const uint4 bw = elem_of(L, b);
            const uint32_t reps = (bw.w >> 8) & 0xFF;  // 1 a duration, a cycle's count, 255 infinite
            const uint32_t tk = new_key(L);
            L.tm_x = b | (tk << 16);
            L.tm_y = key | (reps << 16) | (1u << 31);
            L.tm_due = L.sp->now_ms + (long long)bw.z;
            emit(L, C_TIMER_CREATED, tk, key, b, reps);
          }
        }
        if constexpr (K::M) {
          // subscribeToEvents: the attached message boundary event's subscription before the job
          const uint32_t b = w.w & 0xFFFF;
          if (b != 0xFFFF && ((elem_of(L, b).x >> 8) & 0xFF) != ZBHIP_EV_ERROR) {
            const uint4 bw = elem_of(L, b);
            if (((bw.x >> 8) & 0xFF) != ZBHIP_EV_MESSAGE) { set_fail(L, FB_UNSUPPORTED); return; }
            subscribe_message(L, b, bw, key, true);
            if (L.fail) return;
          }
        }
        uint32_t job = new_key(L);     // BpmnJobBehavior.writeJobCreatedEvent (:194-218)
        emit(L, C_JOB_CREATED, job, key, elem);
        uint2 e = tget(L, t);   // JobCreatedApplier: element instance jobKey
        e.y = (job & 0xFFFF) | (e.y & 0xFCFF0000u) | (1u << 24);  // (a multi-instance loop counter stays)
        if ((w.z >> 16) != 0xFFFF) {
          // BpmnJobActivationBehavior.publishWork (:61-100): a job stream of the type -- JOB_BATCH:ACTIVATED
          // (key = nextKey) of this job, ACTIVATED from now on (its deadline and worker: the host's stream
          // table; runtime.cpp track_jobs)
          emit(L, C_JOB_PUSHED, new_key(L), job, elem);
          e.y |= 2u << 24;
        }
        tput(L, t, e);
        emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
        tbl_set_state(L, t, ZBHIP_PI_ELEMENT_ACTIVATED);
        return;
      }
      case ZBHIP_EL_EXCLUSIVE_GATEWAY: {  // ExclusiveGatewayProcessor.onActivate (:47-66)
        if constexpr (!K::X) { set_fail(L, FB_UNSUPPORTED); return; }
        uint32_t flow = find_sequence_flow(L, w, key);
        if (L.fail) return;
        if (flow == FLOW_INCIDENT) {
          // BpmnIncidentBehavior.createIncident (behavior/BpmnIncidentBehavior.java:51-71): INCIDENT:CREATED
          // (key = nextKey), IncidentCreatedApplier; the gateway stays ELEMENT_ACTIVATING (a persistent
          // element instance: its job field holds the incident key, bits 26..31 the incident info)
          const uint32_t ik = new_key(L);
          emit(L, C_INCIDENT_CREATED, ik, key, elem, L.inc);
          uint2 e = tget(L, t);
          e.y = (ik & 0xFFFF) | (e.y & 0x00FF0000u) | (L.inc << 26);
          tput(L, t, e);
          return;
        }
        emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
        emit(L, ZBHIP_PI_ELEMENT_COMPLETING, key, fsa, elem);
        transition_to_completed_child(L, t, elem, w, key);
        if (flow != NONE) take_sequence_flow(L, flow);
        return;
      }
      case ZBHIP_EL_INTERMEDIATE_CATCH_EVENT:  // IntermediateCatchEventProcessor.onActivate
        if constexpr (K::M) {
          if (((w.x >> 8) & 0xFF) != ZBHIP_EV_MESSAGE) { set_fail(L, FB_UNSUPPORTED); return; }
          subscribe_message(L, elem, w, key);
          if (L.fail) return;
          emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
          tbl_set_state(L, t, ZBHIP_PI_ELEMENT_ACTIVATED);
        } else if constexpr (K::S) {
          // timer: CatchEventBehavior.subscribeToTimerEvent (CatchEventBehavior.java:303-330):
          // dueDate = now + duration, TIMER:CREATED (+key), TimerCreatedApplier; one timer per
          // instance on the device (a second one falls back)
          if (((w.x >> 8) & 0xFF) != ZBHIP_EV_TIMER || !L.has_tmr || (L.tm_y >> 31)) { set_fail(L, FB_UNSUPPORTED); return; }
          const uint32_t tk = new_key(L);
          L.tm_x = elem | (tk << 16);
          L.tm_y = key | (1u << 16) | (1u << 31);  // one repetition (a duration)
          L.tm_due = L.sp->now_ms + (long long)w.z;
          emit(L, C_TIMER_CREATED, tk, key, elem, 1);
          emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
          tbl_set_state(L, t, ZBHIP_PI_ELEMENT_ACTIVATED);
        } else {
          set_fail(L, FB_UNSUPPORTED);
        }
        return;
      case ZBHIP_EL_MULTI_INSTANCE_BODY:  // MultiInstanceBodyProcessor.onActivate (:83-98) -> activate (:229-252)
        if constexpr (K::S) {
          // readInputCollectionVariable (a static collection always evaluates); no event subscriptions
          // on the body
          uint32_t n, list;
          if (!mi_collection(L, elem, w, key, c, n, list)) return;
          emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
          tbl_set_state(L, t, ZBHIP_PI_ELEMENT_ACTIVATED);
          if ((mi_ext(L, elem).x >> 16) != 0xFFFF)  // initializeOutputCollection (:43-55): [nil] * n, local
            emit(L, C_MI_OUT, new_key(L), key, elem, 0x80u | n);
          if (n == 0) {  // an empty collection: completeElement
            follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, key, fsa, elem, true, true, key);
          } else if ((w.z >> 20) & 1u) {  // createInnerInstance -> activateChildInstanceWithKey (:292-307)
            const uint32_t k = new_key(L);
            follow_up(L, ZBHIP_PI_ACTIVATE_ELEMENT, k, key, w.z & 0xFFF, false, false, k);
          } else {  // activateChildInstancesInBatches (:315-324): PROCESS_INSTANCE_BATCH:ACTIVATE
            const uint32_t kb = new_key(L);
            follow_up(L, C_PIB_ACTIVATE, kb, key, elem, true, false, kb, Q_TERM, n);  // (index: the size)
          }
        } else {
          set_fail(L, FB_UNSUPPORTED);
        }
        return;
      case ZBHIP_EL_SUB_PROCESS:  // SubProcessProcessor.onActivate (container/SubProcessProcessor.java:49-66)
        if constexpr (K::S) {
          if constexpr (K::IO) {
            apply_input_mapping(L, elem, key);  // applyInputMappings, then ACTIVATED
            if (L.fail) return;
          }
          emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
          tbl_set_state(L, t, ZBHIP_PI_ELEMENT_ACTIVATED);
          // activateChildInstance: the none start event, key -1, flow scope = this instance
          follow_up(L, ZBHIP_PI_ACTIVATE_ELEMENT, NONE, key, w.z & 0xFFFF, false, false, NONE);
        } else {
          set_fail(L, FB_UNSUPPORTED);
        }
        return;
      case ZBHIP_EL_PARALLEL_GATEWAY:  // ParallelGatewayProcessor.onActivate (:34-50)
        emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, key, fsa, elem);
        emit(L, ZBHIP_PI_ELEMENT_COMPLETING, key, fsa, elem);
        transition_to_completed_child(L, t, elem, w, key);
        take_outgoing(L, w);
        return;
      default:
        set_fail(L, FB_UNSUPPORTED);
        return;
    }
  }

  // ---- COMPLETE_ELEMENT: guard (:56-63) ----
  if (type == ZBHIP_EL_PROCESS) {
    if (!L.pi_live) { reject_pi(L, true, elem, cmd_key, raux, ZBHIP_REASON_EI_NOT_FOUND, 0); return; }
    if (L.pi_state != ZBHIP_PI_ELEMENT_ACTIVATED && L.pi_state != ZBHIP_PI_ELEMENT_COMPLETING) {
      reject_pi(L, true, elem, cmd_key, raux, ZBHIP_REASON_EI_STATE, L.pi_state);
      return;
    }
    if (L.pi_state == ZBHIP_PI_ELEMENT_COMPLETING) { set_fail(L, FB_UNSUPPORTED); return; }
    // ProcessProcessor.onComplete (:63-76): COMPLETING, COMPLETED (never end of path)
    emit(L, ZBHIP_PI_ELEMENT_COMPLETING, 0, NONE, 0);
    L.pi_state = ZBHIP_PI_ELEMENT_COMPLETING;
    emit(L, ZBHIP_PI_ELEMENT_COMPLETED, 0, NONE, 0);
    L.pi_live = false;  // removeInstance: variables, taken-flow counters of the scope go with it
    L.nvars = 0;
    L.jw0 = L.jw1 = L.jw2 = L.jw3 = 0;
    ++L.completed;
    return;
  }
  const int t = tbl_find(L, cmd_key);
  if (t < 0) { reject_pi(L, true, elem, cmd_key, raux, ZBHIP_REASON_EI_NOT_FOUND, 0); return; }
  const uint32_t st = (tget(L, t).y >> 16) & 0xFF;
  if (st != ZBHIP_PI_ELEMENT_ACTIVATED && st != ZBHIP_PI_ELEMENT_COMPLETING) {
    reject_pi(L, true, elem, cmd_key, raux, ZBHIP_REASON_EI_STATE, st);
    return;
  }
  if (c != 0) {  // K::S: the flow scope is a sub-process instance
    const uint32_t fst = (tget(L, scope_find(L, c)).y >> 16) & 0xFF;
    if (fst != ZBHIP_PI_ELEMENT_ACTIVATED) { reject_pi(L, true, elem, cmd_key, raux, ZBHIP_REASON_FS_STATE, fst); return; }
  } else if (!L.pi_live) {
    reject_pi(L, true, elem, cmd_key, raux, ZBHIP_REASON_FS_NOT_FOUND, 0);
    return;
  } else if (L.pi_state != ZBHIP_PI_ELEMENT_ACTIVATED) {
    reject_pi(L, true, elem, cmd_key, raux, ZBHIP_REASON_FS_STATE, L.pi_state);
    return;
  }
  if (st == ZBHIP_PI_ELEMENT_COMPLETING) { set_fail(L, FB_UNSUPPORTED); return; }
  emit(L, ZBHIP_PI_ELEMENT_COMPLETING, cmd_key, fsa, elem);
  tbl_set_state(L, t, ZBHIP_PI_ELEMENT_COMPLETING);
  if constexpr (K::M) {
    if (type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT) {
      // IntermediateCatchEventProcessor.onComplete -> unsubscribeFromEvents: a subscription still
      // open here would write PROCESS_MESSAGE_SUBSCRIPTION:DELETING (outside the subset)
      if (((L.pm_x >> 12) & 3) != 0 && (L.pm_y & 0xFFFF) == cmd_key) { set_fail(L, FB_MESSAGE); return; }
    } else if (type != ZBHIP_EL_START_EVENT && !ZBHIP_IS_JOB_WORKER(type) && !pass_through(type) &&
               type != ZBHIP_EL_BOUNDARY_EVENT) {
      // BoundaryEventProcessor.onComplete (event/BoundaryEventProcessor.java:47-56): no mappings
      set_fail(L, FB_UNSUPPORTED);
      return;
    }
  } else if (K::S && type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT) {
    // IntermediateCatchEventProcessor.onComplete -> unsubscribeFromEvents: a timer still open here
    // would be canceled (TIMER:CANCELED, outside the subset)
    if ((L.tm_y >> 31) && (L.tm_y & 0xFFFF) == cmd_key) { set_fail(L, FB_UNSUPPORTED); return; }
  } else if (type != ZBHIP_EL_START_EVENT && !ZBHIP_IS_JOB_WORKER(type) && !pass_through(type) &&
             !(K::S && (type == ZBHIP_EL_SUB_PROCESS || type == ZBHIP_EL_BOUNDARY_EVENT ||
                        type == ZBHIP_EL_MULTI_INSTANCE_BODY))) {
    // SubProcessProcessor.onComplete (:68-82): no output mappings or subscriptions in the subset;
    // BoundaryEventProcessor.onComplete (event/BoundaryEventProcessor.java:47-56): no mappings
    set_fail(L, FB_UNSUPPORTED);
    return;
  }
  // applyOutputMappings (BpmnVariableMappingBehavior.java:86-156): with an output mapping the event
  // trigger's variables become local (mergeLocalDocument), then the mapping goes to the flow scope;
  // without one the trigger's variables are merged from the element's scope
  bool mapped = false;
  if constexpr (K::IO) {
    const uint4 om = io_map(L, elem, 1);
    if ((om.x & 0xFF) != kIoNone) {
      if (L.trig_key == cmd_key && L.doc_count) {
        merge_local_document(L, cmd_key, L.doc_begin, L.doc_count);
        if (L.fail) return;
      }
      apply_output_mapping(L, om, elem, cmd_key);
      if (L.fail) return;
      mapped = true;
    }
  }
  if (!mapped && L.trig_key == cmd_key) {
    if constexpr (K::S) {
      // an inner instance's own loop variables would be updated in its scope (mergeDocument): they
      // are not in the variable table (derived from the slot), so such a document falls back
      const uint4 bw = elem_of(L, c);
      // (several entries: the loop variables' names are not checked one by one -- outside the subset)
      if (c != 0 && L.doc_count > 1 && etype(bw) == ZBHIP_EL_MULTI_INSTANCE_BODY) { set_fail(L, FB_DOC); return; }
      if (c != 0 && L.doc_count == 1 && etype(bw) == ZBHIP_EL_MULTI_INSTANCE_BODY) {
        const zbhip_doc_entry d = L.docs[L.doc_begin];
        const uint32_t name = d.name_id;
        vm_drain();
        if (name == (bw.x >> 16) || name == (bw.w & 0xFFFF)) { set_fail(L, FB_DOC); return; }
        const uint4 ext = mi_ext(L, c);
        const uint32_t oe = ext.y & 0xFFFF;
        // the collections themselves: the body's output (held on the host) and the input variable (read
        // again on every activation and completion) stay as they are on the device
        if (name == (ext.x >> 16) || name == (ext.x & 0xFFFF)) { set_fail(L, FB_DOC); return; }
        if (oe != 0xFFFF && name == oe) {
          // the local outputElement variable (nil): updated in the inner instance's scope; its key is
          // right below the loopCounter's (a job worker: two below the job's)
          if (d.type == ZBHIP_DOC_LIST) { set_fail(L, FB_DOC); return; }
          if (d.type != ZBHIP_DOC_NIL) {
            // (a job worker's job field is -1 after JOB:COMPLETED: the completed job's key)
            const uint32_t job = ZBHIP_IS_JOB_WORKER(type) ? L.done_job : tget(L, t).y & 0xFFFF;
            emit(L, C_VAR_UPDATED, ZBHIP_IS_JOB_WORKER(type) ? job - 2 : job - 1, cmd_key, name);
          }
          L.mo_set = 1;
          L.mo_type = d.type;
          L.mo_val = d.type == ZBHIP_DOC_NIL ? 0 : d.value;
          goto merged;
        }
      }
    }
    merge_document_from(L, cmd_key, c, L.doc_begin, L.doc_count);
  merged:;
  }
  if constexpr (K::S) {
    // JobWorkerTaskProcessor.onComplete (:63-75), SubProcessProcessor.onComplete (:68-82):
    // unsubscribeFromEvents -- the boundary event's timer
    if ((ZBHIP_IS_JOB_WORKER(type) || type == ZBHIP_EL_SUB_PROCESS) && (L.tm_y >> 31) && (L.tm_y & 0xFFFF) == cmd_key)
      cancel_timer(L);
    // StartEventProcessor.onComplete (:52-67): subscribeToEvents of the flow scope -- a sub-process's
    // timer boundary event (CatchEventBehavior.subscribeToTimerEvent: dueDate = now + duration)
    if (type == ZBHIP_EL_START_EVENT && c != 0) {
      const uint4 cw = elem_of(L, c);
      const uint32_t b = cw.w & 0xFFFF;
      // (an error boundary event subscribes to nothing)
      if (etype(cw) == ZBHIP_EL_SUB_PROCESS && b != 0xFFFF && ((elem_of(L, b).x >> 8) & 0xFF) != ZBHIP_EV_ERROR) {
        if (!L.has_tmr || (L.tm_y >> 31)) { set_fail(L, FB_UNSUPPORTED); return; }
        const uint32_t ck = scope_key(L, c);
        const uint4 bw = elem_of(L, b);
        const uint32_t reps = (bw.w >> 8) & 0xFF;  // 1 a duration, a cycle's count, 255 infinite
        const uint32_t tk = new_key(L);
        L.tm_x = b | (tk << 16);
        L.tm_y = ck | (reps << 16) | (1u << 31);
        L.tm_due = L.sp->now_ms + (long long)bw.z;
        emit(L, C_TIMER_CREATED, tk, ck, b, reps);
      }
    }
  }
  if constexpr (K::IO) {
    // MultiInstanceBodyProcessor.onComplete (:100-114): propagateVariable of the outputCollection
    // (BpmnStateBehavior.java:163-178 -> mergeDocument from the flow scope): created in the process
    // instance's scope, or UPDATED where it exists -- unless equal (VariableBehavior.java:134).  The
    // device holds an output array's length (the variable's value), not its items: an existing array
    // of another length or a scalar differs; one of the same length, a list variable, or a variable
    // of a sub-process scope is outside the subset
    if (type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
      const uint32_t oc = mi_ext(L, elem).x >> 16;
      if (oc != 0xFFFF) {
        uint32_t n, list;
        if (!mi_collection(L, elem, w, cmd_key, c, n, list)) return;
        const int vi = var_lookup(L, cmd_key, c, oc);
        if (vi >= 0) {
          const uint32_t vy = var_y(L, vi), vt = (vy >> 16) & 0xFF;
          if ((var_x(L, vi) >> 16) != 0 || vt == ZBHIP_DOC_LIST || (vt == kDocOutList && var_v(L, vi) == (long long)n)) {
            set_fail(L, FB_VARS);
            return;
          }
          emit(L, C_MI_PROP, vy & 0xFFFF, cmd_key, elem, 1u);  // (flags 1: UPDATED)
          var_put(L, vi, var_x(L, vi), (vy & 0xFFFF) | ((uint32_t)kDocOutList << 16), (long long)n);
        } else {
          if (L.nvars >= kVars) { set_fail(L, FB_VARS); return; }
          const uint32_t kv = new_key(L);
          emit(L, C_MI_PROP, kv, cmd_key, elem);
          var_put(L, L.nvars++, oc, kv | ((uint32_t)kDocOutList << 16), (long long)n);
        }
      }
    }
  }
  if constexpr (K::M) {
    // JobWorkerTaskProcessor.onComplete: unsubscribeFromEvents -- the boundary event's subscription
    if (ZBHIP_IS_JOB_WORKER(type) && ((L.pm_x >> 12) & 3) != 0 && (L.pm_y & 0xFFFF) == cmd_key) unsubscribe_message(L);
    if (L.fail) return;
  }
  transition_to_completed_child(L, t, elem, w, cmd_key);
  take_outgoing(L, w);
}

template <class K>
__device__ __forceinline__ void note_activation(const Lane<K>& L, uint32_t job_ord, uint32_t inst) {
  const StepParams& P = *L.sp;
  if (!P.cmd_act || !P.st.act || inst >= P.st.n) return;
  uint4 f = make_uint4(0, 0, 0, 0);
  for (uint32_t k = 0; k < (uint32_t)kSlots; ++k) {
    const uint4 a = P.st.act[(size_t)k * P.st.n + inst];
    if ((a.x >> 31) && (a.x & 0xFFFF) == job_ord) f = a;
  }
  P.cmd_act[L.ci] = f;
}

// ---- straight-line segments of linear chains (K::REG) --------------------------------------
// The arena's segment word of a start event or service task (runtime.cpp rebuild_program) says
// that leaving it is deterministic: one unconditional outgoing flow `f` into a service task or a
// none end event `n` without outgoing flows.  From the canonical waiting state (the scope
// ACTIVATED with that one child) the whole batch of a JOB:COMPLETE -- and of a CREATE whose start
// event leads into a task -- is then a fixed record sequence: exactly what the general path
// (JobCompleteProcessor, the FIFO over BpmnStreamProcessor, ProcessProcessor, the appliers)
// emits, written here with static stage rows and no FIFO, element table or guard dispatch.  Any
// other state, a variable document, a tight batch limit or record capacity takes the general path.
constexpr uint32_t SEG_VALID = 1u << 31, SEG_FROM_TASK = 1u << 30, SEG_TO_END = 1u << 24;
// a segment whose task carries a timer boundary event (source: canceled on completion) or whose next
// task does (target: created on activation) -- KScope's segments only (fast_scope_job)
constexpr uint32_t SEG_SRC_TIMER = 1u << 25, SEG_DST_TIMER = 1u << 26;
// a task into a joining parallel gateway, and such a gateway's own word (its one flow onwards): the
// joins of KGeneric (fast_join_job)
constexpr uint32_t SEG_TO_JOIN = 1u << 27, SEG_FROM_GW = 1u << 28;
// a none start event into a forking parallel gateway whose flows all lead into tasks (fast_fork_create)
constexpr uint32_t SEG_TO_FORK = 1u << 29;

template <class K>
__device__ __forceinline__ void put(Lane<K>& L, int j, uint32_t code, uint32_t key, uint32_t aux, uint32_t elem) {
  L.stage[j * K::B] = make_uint2((key & 0xFFFF) | (aux << 16), (elem & 0xFFFF) | (code << 16));
}

// records of the segment tail from the flow's SFT on (row j0 onwards), keys from ordinal k;
// ProcessInstanceSequenceFlowTakenApplier, then ACTIVATE_ELEMENT(n) processed as in process_pi
template <class K>
__device__ __forceinline__ void seg_enter(Lane<K>& L, int j0, uint32_t sg, uint32_t k) {
  const uint32_t f = sg & 0xFFF, n = (sg >> 12) & 0xFFF;
  put(L, j0, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, k, 0, f);
  put(L, j0 + 1, ZBHIP_PI_ACTIVATE_ELEMENT, k + 1, 0, n);
  put(L, j0 + 2, ZBHIP_PI_ELEMENT_ACTIVATING, k + 1, 0, n);
}

template <class K>
__device__ __forceinline__ bool fast_command(Lane<K>& L, uint32_t kind, uint32_t ref, uint32_t doc_count) {
  if (L.fail || L.proc == NONE || doc_count != 0 || L.limit <= 4 || L.rec_cap < 16 || L.next_ord >= 0xFFE0)
    return false;
  const uint32_t* seg = L.pb + (L.pb[6] & 0xFFFF);
  if (kind == ZBHIP_CMD_JOB_COMPLETE) {
    if (!(L.pi_live && L.pi_state == ZBHIP_PI_ELEMENT_ACTIVATED && L.nt == 1 && L.pi_child == 1 && L.pi_asf == 0))
      return false;
    const uint2 e = L.r_t0;
    if (e.x == 0xFFFFFFFFu || (e.y & 0xFFFF) != ref || !((e.y >> 24) & 1u) ||
        ((e.y >> 16) & 0xFF) != ZBHIP_PI_ELEMENT_ACTIVATED)
      return false;
    const uint32_t te = e.x & 0xFFFF, tk = e.x >> 16;
    const uint32_t sg = seg[te];
    if ((sg & (SEG_VALID | SEG_FROM_TASK | SEG_SRC_TIMER | SEG_DST_TIMER | SEG_TO_JOIN)) != (SEG_VALID | SEG_FROM_TASK)) return false;
    const uint32_t k = L.next_ord, n = (sg >> 12) & 0xFFF;
    // JobCompleteProcessor + EventTriggerBehavior.triggeringProcessEvent, then COMPLETE_ELEMENT(task)
    put(L, 0, C_JOB_COMPLETED | (((e.y >> 25) & 1u) << 8), ref, tk, te);  // (flag 1: an ACTIVATED job)
    if ((e.y >> 25) & 1u) note_activation(L, ref, L.inst);
    put(L, 1, C_PE_TRIGGERING, k, tk, te);
    put(L, 2, ZBHIP_PI_COMPLETE_ELEMENT, tk, 0, te);
    put(L, 3, ZBHIP_PI_ELEMENT_COMPLETING, tk, 0, te);
    put(L, 4, ZBHIP_PI_ELEMENT_COMPLETED, tk, 0, te);
    seg_enter(L, 5, sg, k + 1);
    if (!(sg & SEG_TO_END)) {  // JobWorkerTaskProcessor.onActivate: the next wait state
      put(L, 8, C_JOB_CREATED, k + 3, k + 2, n);
      put(L, 9, ZBHIP_PI_ELEMENT_ACTIVATED, k + 2, 0, n);
      L.r_t0 = make_uint2(n | ((k + 2) << 16), ((k + 3) & 0xFFFF) | (ZBHIP_PI_ELEMENT_ACTIVATED << 16) | (1u << 24));
      L.next_ord = (uint16_t)(k + 4);
      L.nrec = 10;
      L.transitions = 5;
    } else {  // NoneEndEventBehavior, end of the path -> ProcessProcessor.onComplete
      put(L, 8, ZBHIP_PI_ELEMENT_ACTIVATED, k + 2, 0, n);
      put(L, 9, ZBHIP_PI_ELEMENT_COMPLETING, k + 2, 0, n);
      put(L, 10, ZBHIP_PI_ELEMENT_COMPLETED, k + 2, 0, n);
      put(L, 11, ZBHIP_PI_COMPLETE_ELEMENT, 0, NONE, 0);
      put(L, 12, ZBHIP_PI_ELEMENT_COMPLETING, 0, NONE, 0);
      put(L, 13, ZBHIP_PI_ELEMENT_COMPLETED, 0, NONE, 0);
      L.r_t0 = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
      L.next_ord = (uint16_t)(k + 3);
      L.pi_child = 0;
      L.pi_live = false;
      L.pi_state = ZBHIP_PI_ELEMENT_COMPLETING;
      L.nvars = 0;
      L.nrec = 14;
      L.transitions = 9;
      L.completed = 1;
    }
    return true;
  }
  if (kind == ZBHIP_CMD_CREATE) {  // CreateProcessInstanceProcessor, ProcessProcessor, StartEventProcessor
    const uint32_t start = L.pb[0] >> 16;
    if (start == NONE) return false;
    const uint32_t sg = seg[start];
    if ((sg & (SEG_VALID | SEG_FROM_TASK | SEG_TO_END | SEG_DST_TIMER | SEG_TO_FORK)) != SEG_VALID) return false;
    const uint32_t n = (sg >> 12) & 0xFFF;
    put(L, 0, ZBHIP_PI_ACTIVATE_ELEMENT, 0, NONE, 0);
    put(L, 1, C_PIC_CREATED, 1, 0, 0);
    put(L, 2, ZBHIP_PI_ELEMENT_ACTIVATING, 0, NONE, 0);
    put(L, 3, ZBHIP_PI_ELEMENT_ACTIVATED, 0, NONE, 0);
    put(L, 4, ZBHIP_PI_ACTIVATE_ELEMENT, NONE, 0, start);
    put(L, 5, ZBHIP_PI_ELEMENT_ACTIVATING, 2, 0, start);
    put(L, 6, ZBHIP_PI_ELEMENT_ACTIVATED, 2, 0, start);
    put(L, 7, ZBHIP_PI_COMPLETE_ELEMENT, 2, 0, start);
    put(L, 8, ZBHIP_PI_ELEMENT_COMPLETING, 2, 0, start);
    put(L, 9, ZBHIP_PI_ELEMENT_COMPLETED, 2, 0, start);
    seg_enter(L, 10, sg, 3);
    put(L, 13, C_JOB_CREATED, 5, 4, n);
    put(L, 14, ZBHIP_PI_ELEMENT_ACTIVATED, 4, 0, n);
    L.r_t0 = make_uint2(n | (4u << 16), 5u | (ZBHIP_PI_ELEMENT_ACTIVATED << 16) | (1u << 24));
    L.nt = 1;
    L.next_ord = 6;
    L.pi_live = true;
    L.pi_state = ZBHIP_PI_ELEMENT_ACTIVATED;
    L.pi_child = 1;
    L.pi_asf = 0;
    L.nrec = 15;
    L.transitions = 9;
    return true;
  }
  return false;
}

// ---- straight-line JOB:COMPLETE batches of KScope ---------------------------------------------
// The same segments for processes with timers (KScope: boundary10 and the like): a task at the
// process level completing into the next task or a none end event, either task with a timer boundary
// event.  From the canonical waiting state (the process ACTIVATED with that task as its only child,
// the job unclaimed by a pending trigger, the instance's timer row the task's own or free) the batch
// is the general path's exact sequence -- JOB:COMPLETED, PROCESS_EVENT:TRIGGERING, COMPLETE_ELEMENT,
// COMPLETING, [TIMER:CANCELED], COMPLETED, SEQUENCE_FLOW_TAKEN, ACTIVATE_ELEMENT, ACTIVATING,
// [TIMER:CREATED], JOB:CREATED, ACTIVATED (or the end event's and the process's completion) -- written
// without the FIFO, guard dispatch or table search; the appliers' effects on the element table, the
// process scope's counters and the timer row are set directly.  Anything else: the general path.
template <class K>
__device__ __forceinline__ bool fast_scope_job(Lane<K>& L, uint32_t ref, uint32_t doc_count) {
  if (L.fail || L.proc == NONE || doc_count != 0 || L.limit <= 4 || L.rec_cap < 16 || L.next_ord >= 0xFFE0)
    return false;
  if (!(L.pi_live && L.pi_state == ZBHIP_PI_ELEMENT_ACTIVATED && L.nt == 1 && L.pi_child == 1 && L.pi_asf == 0 &&
        L.trig_key == NONE))
    return false;
  const uint2 e = tget(L, 0);
  if (e.x == 0xFFFFFFFFu || (e.y & 0xFFFF) != ref || !((e.y >> 24) & 1u) || ((e.y >> 16) & 0xFF) != ZBHIP_PI_ELEMENT_ACTIVATED)
    return false;
  const uint32_t te = e.x & 0xFFFF, tk = e.x >> 16;
  const uint32_t sg = L.pb[(L.pb[6] & 0xFFFF) + te];
  if ((sg & (SEG_VALID | SEG_FROM_TASK | SEG_TO_JOIN)) != (SEG_VALID | SEG_FROM_TASK)) return false;
  const bool src_tmr = sg & SEG_SRC_TIMER, dst_tmr = sg & SEG_DST_TIMER;
  const bool live_tmr = L.has_tmr && (L.tm_y >> 31);
  if ((src_tmr || dst_tmr) && !L.has_tmr) return false;
  if (src_tmr ? !(live_tmr && (L.tm_y & 0xFFFF) == tk) : live_tmr) return false;
  const uint32_t n = (sg >> 12) & 0xFFF, f = sg & 0xFFF;
  // JobCompleteProcessor: JOB:COMPLETED (the job row deleted), triggeringProcessEvent, COMPLETE_ELEMENT
  emit(L, C_JOB_COMPLETED, ref, tk, te, (e.y >> 25) & 1u);  // (flag 1: an ACTIVATED job)
  if ((e.y >> 25) & 1u) note_activation(L, ref, L.inst);
  const uint32_t pe = new_key(L);
  emit(L, C_PE_TRIGGERING, pe, tk, te);
  emit(L, ZBHIP_PI_COMPLETE_ELEMENT, tk, 0, te);
  // JobWorkerTaskProcessor.onComplete: COMPLETING, unsubscribeFromEvents (the boundary timer),
  // COMPLETED (the instance and its trigger removed), the one outgoing flow
  emit(L, ZBHIP_PI_ELEMENT_COMPLETING, tk, 0, te);
  if (src_tmr) cancel_timer(L);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETED, tk, 0, te);
  const uint32_t sft = new_key(L);
  emit(L, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, sft, 0, f);
  const uint32_t nk = new_key(L);
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, nk, 0, n);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, nk, 0, n);
  if (!(sg & SEG_TO_END)) {
    // JobWorkerTaskProcessor.onActivate: the boundary event's timer, the job, ACTIVATED
    if (dst_tmr) {
      const uint32_t b = elem_of(L, n).w & 0xFFFF;
      const uint4 bw = elem_of(L, b);
      const uint32_t reps = (bw.w >> 8) & 0xFF;
      const uint32_t tmk = new_key(L);
      L.tm_x = b | (tmk << 16);
      L.tm_y = nk | (reps << 16) | (1u << 31);
      L.tm_due = L.sp->now_ms + (long long)bw.z;
      emit(L, C_TIMER_CREATED, tmk, nk, b, reps);
    }
    const uint32_t job = new_key(L);
    emit(L, C_JOB_CREATED, job, nk, n);
    emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, nk, 0, n);
    tput(L, 0, make_uint2(n | (nk << 16), (job & 0xFFFF) | ((uint32_t)ZBHIP_PI_ELEMENT_ACTIVATED << 16) | (1u << 24)));
  } else {
    // NoneEndEventBehavior, the end of the path -> ProcessProcessor.onComplete
    emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, nk, 0, n);
    emit(L, ZBHIP_PI_ELEMENT_COMPLETING, nk, 0, n);
    emit(L, ZBHIP_PI_ELEMENT_COMPLETED, nk, 0, n);
    emit(L, ZBHIP_PI_COMPLETE_ELEMENT, 0, NONE, 0);
    emit(L, ZBHIP_PI_ELEMENT_COMPLETING, 0, NONE, 0);
    emit(L, ZBHIP_PI_ELEMENT_COMPLETED, 0, NONE, 0);
    tput(L, 0, make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu));
    L.pi_child = 0;
    L.pi_live = false;
    L.pi_state = ZBHIP_PI_ELEMENT_COMPLETING;
    L.nvars = 0;
    L.jw0 = L.jw1 = L.jw2 = L.jw3 = 0;
    ++L.completed;
  }
  return !L.fail;
}

// ---- straight-line JOB:COMPLETE batches into a join (KGeneric) -------------------------------
// A branch task completing into a joining parallel gateway (fork/join with a task per branch): the
// general path's records -- JOB:COMPLETED, PROCESS_EVENT:TRIGGERING, COMPLETE_ELEMENT, COMPLETING,
// COMPLETED, SEQUENCE_FLOW_TAKEN (the join counter), ACTIVATE_ELEMENT of the gateway, then either its
// rejection (ProcessInstanceStateTransitionGuard.canActivateParallelGateway: not all flows taken) or
// its activation (the counters' Tetris decrement), completion and the one flow onwards into a task or a
// none end event (the process completed when nothing else is active) -- with the appliers' effects set
// directly: no FIFO, guard dispatch or element lookups beyond the segment words.
template <class K>
__device__ __forceinline__ bool fast_join_job(Lane<K>& L, uint32_t ref, uint32_t doc_count) {
  if (L.fail || L.proc == NONE || doc_count != 0 || L.limit <= 6 || L.rec_cap < 24 || L.next_ord >= 0xFFE0 ||
      !L.has_join)
    return false;
  if (!(L.pi_live && L.pi_state == ZBHIP_PI_ELEMENT_ACTIVATED && L.trig_key == NONE)) return false;
  const int t = tbl_find_job(L, ref);
  if (t < 0) return false;
  const uint2 e = tget(L, t);
  if (((e.y >> 16) & 0xFF) != ZBHIP_PI_ELEMENT_ACTIVATED) return false;
  const uint32_t te = e.x & 0xFFFF, tk = e.x >> 16;
  const uint32_t* seg = L.pb + (L.pb[6] & 0xFFFF);
  const uint32_t sg = seg[te];
  if ((sg & (SEG_VALID | SEG_FROM_TASK | SEG_TO_JOIN)) != (SEG_VALID | SEG_FROM_TASK | SEG_TO_JOIN)) return false;
  const uint32_t g = (sg >> 12) & 0xFFF, f = sg & 0xFFF;
  const uint32_t sg2 = seg[g];
  if ((sg2 & (SEG_VALID | SEG_FROM_GW)) != (SEG_VALID | SEG_FROM_GW)) return false;
  // JobCompleteProcessor, triggeringProcessEvent, COMPLETE_ELEMENT of the task and its completion
  emit(L, C_JOB_COMPLETED, ref, tk, te, (e.y >> 25) & 1u);  // (flag 1: an ACTIVATED job)
  if ((e.y >> 25) & 1u) note_activation(L, ref, L.inst);
  const uint32_t pe = new_key(L);
  emit(L, C_PE_TRIGGERING, pe, tk, te);
  emit(L, ZBHIP_PI_COMPLETE_ELEMENT, tk, 0, te);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETING, tk, 0, te);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETED, tk, 0, te);
  tput(L, t, make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu));
  --L.pi_child;
  // takeSequenceFlow into the gateway: the taken-flow counter, then ACTIVATE_ELEMENT
  const uint32_t sft = new_key(L);
  emit(L, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, sft, 0, f);
  ++L.pi_asf;
  const uint4 fw = elem_of(L, f);
  const uint32_t js = fw.w & 0xFFFF, jc = join_get(L, js);
  if (jc >= 255) set_fail(L, FB_JOIN);
  join_set(L, js, jc + 1);
  const uint32_t gk = new_key(L);
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, gk, 0, g);
  const uint4 gw = elem_of(L, g);
  const uint32_t base = gw.w & 0xFFFF, nin = gw.x >> 16;
  uint32_t taken = 0;
  for (uint32_t s = base; s < base + nin; ++s) taken += join_get(L, s) > 0;
  if (taken < nin) {  // canActivateParallelGateway: the command is rejected
    emit(L, kRejectBit | ZBHIP_PI_ACTIVATE_ELEMENT, gk, 0, g, ZBHIP_REASON_PGW_NOT_ALL_TAKEN);
    return !L.fail;
  }
  // ACTIVATING (cleanupSequenceFlowsTaken, the activation's counters), ACTIVATED, COMPLETING, COMPLETED
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, gk, 0, g);
  for (uint32_t s = base; s < base + nin; ++s) {
    const uint32_t c = join_get(L, s);
    if (c > 0) join_set(L, s, c - 1);
  }
  L.pi_asf = L.pi_asf > (int)nin ? L.pi_asf - (int)nin : 0;
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, gk, 0, g);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETING, gk, 0, g);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETED, gk, 0, g);
  // the gateway's one flow onwards
  const uint32_t n = (sg2 >> 12) & 0xFFF, f2 = sg2 & 0xFFF;
  const uint32_t sft2 = new_key(L);
  emit(L, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, sft2, 0, f2);
  const uint32_t nk = new_key(L);
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, nk, 0, n);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, nk, 0, n);  // (the flow's +1 and the activation's -1 cancel)
  if (!(sg2 & SEG_TO_END)) {
    const int tn = tbl_insert(L, n, nk, ZBHIP_PI_ELEMENT_ACTIVATING);
    if (tn < 0) return false;
    ++L.pi_child;
    const uint32_t job = new_key(L);
    emit(L, C_JOB_CREATED, job, nk, n);
    tput(L, tn, make_uint2(n | (nk << 16), (job & 0xFFFF) | ((uint32_t)ZBHIP_PI_ELEMENT_ACTIVATED << 16) | (1u << 24)));
    emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, nk, 0, n);
    return !L.fail;
  }
  // NoneEndEventBehavior; the end of the path -> ProcessProcessor.onComplete once nothing is active
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, nk, 0, n);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETING, nk, 0, n);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETED, nk, 0, n);
  if (L.pi_child + L.pi_asf == 0) {
    emit(L, ZBHIP_PI_COMPLETE_ELEMENT, 0, NONE, 0);
    emit(L, ZBHIP_PI_ELEMENT_COMPLETING, 0, NONE, 0);
    emit(L, ZBHIP_PI_ELEMENT_COMPLETED, 0, NONE, 0);
    L.pi_live = false;
    L.pi_state = ZBHIP_PI_ELEMENT_COMPLETING;
    L.nvars = 0;
    L.jw0 = L.jw1 = L.jw2 = L.jw3 = 0;
    ++L.completed;
  }
  return !L.fail;
}

// A CREATE whose none start event leads into a forking parallel gateway with a task on every outgoing
// flow (fork/join with a task per branch): the general path's records -- the process, the start event,
// the gateway (its incoming flow's counter up and down again), SEQUENCE_FLOW_TAKEN + ACTIVATE_ELEMENT per
// outgoing flow, then each task's ACTIVATING, JOB:CREATED, ACTIVATED in flow order -- no variables.
template <class K>
__device__ __forceinline__ bool fast_fork_create(Lane<K>& L, uint32_t doc_count) {
  if (L.fail || L.proc == NONE || doc_count != 0 || L.limit <= 16 || L.pi_live || L.nt != 0 || !L.has_join)
    return false;
  const uint32_t start = L.pb[0] >> 16;
  if (start == NONE) return false;
  const uint32_t sg = L.pb[(L.pb[6] & 0xFFFF) + start];
  if ((sg & (SEG_VALID | SEG_FROM_TASK | SEG_TO_FORK)) != (SEG_VALID | SEG_TO_FORK)) return false;
  const uint32_t g = (sg >> 12) & 0xFFF, f = sg & 0xFFF;
  const uint4 gw = elem_of(L, g);
  const uint32_t ob = gw.y & 0xFFFF, oc = gw.y >> 16;
  if (oc > (uint32_t)K::T || oc > 8 || L.rec_cap < 16 + 5 * oc) return false;
  const uint32_t pi = new_key(L);  // 0
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, pi, NONE, 0);
  const uint32_t created = new_key(L);  // CommandProcessorImpl.accept: entityKey = nextKey
  emit(L, C_PIC_CREATED, created, pi, 0);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, pi, NONE, 0);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, pi, NONE, 0);
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, NONE, 0, start);  // activateChildInstance: key -1
  const uint32_t sk = new_key(L);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, sk, 0, start);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, sk, 0, start);
  emit(L, ZBHIP_PI_COMPLETE_ELEMENT, sk, 0, start);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETING, sk, 0, start);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETED, sk, 0, start);
  // the flow into the gateway counts on its join slot; the activation's Tetris decrement takes it off
  const uint32_t sft = new_key(L);
  emit(L, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, sft, 0, f);
  const uint32_t gk = new_key(L);
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, gk, 0, g);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, gk, 0, g);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, gk, 0, g);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETING, gk, 0, g);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETED, gk, 0, g);
  uint32_t first = 0;
  for (uint32_t i = 0; i < oc; ++i) {
    const uint32_t fi = out_flow(L, ob + i);
    const uint32_t ki = new_key(L);
    emit(L, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, ki, 0, fi);
    const uint32_t kt = new_key(L);
    if (i == 0) first = kt;
    emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, kt, 0, elem_of(L, fi).z & 0xFFFF);
  }
  for (uint32_t i = 0; i < oc; ++i) {
    const uint32_t t = elem_of(L, out_flow(L, ob + i)).z & 0xFFFF;
    const uint32_t kt = first + 2 * i;  // the task keys: every second key after the first flow's
    emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, kt, 0, t);
    const uint32_t job = new_key(L);
    emit(L, C_JOB_CREATED, job, kt, t);
    emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, kt, 0, t);
    tput(L, (int)i, make_uint2(t | (kt << 16), (job & 0xFFFF) | ((uint32_t)ZBHIP_PI_ELEMENT_ACTIVATED << 16) | (1u << 24)));
  }
  L.nt = (int)oc;
  L.pi_live = true;
  L.pi_state = ZBHIP_PI_ELEMENT_ACTIVATED;
  L.pi_child = (int)oc;
  L.pi_asf = 0;
  return !L.fail;
}

// A CREATE whose none start event leads into a task (with or without a timer boundary event):
// CreateProcessInstanceProcessor, ProcessProcessor, StartEventProcessor and the task's activation in
// the general path's order; no variables (a document takes the general path).
template <class K>
__device__ __forceinline__ bool fast_scope_create(Lane<K>& L, uint32_t doc_count) {
  if (L.fail || L.proc == NONE || doc_count != 0 || L.limit <= 4 || L.rec_cap < 18 || L.pi_live || L.nt != 0)
    return false;
  const uint32_t start = L.pb[0] >> 16;
  if (start == NONE) return false;
  const uint32_t sg = L.pb[(L.pb[6] & 0xFFFF) + start];
  if ((sg & (SEG_VALID | SEG_FROM_TASK | SEG_TO_END | SEG_TO_FORK)) != SEG_VALID) return false;
  const bool dst_tmr = sg & SEG_DST_TIMER;
  if (dst_tmr && !L.has_tmr) return false;
  const uint32_t n = (sg >> 12) & 0xFFF, f = sg & 0xFFF;
  const uint32_t pi = new_key(L);  // 0
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, pi, NONE, 0);
  const uint32_t created = new_key(L);  // CommandProcessorImpl.accept: entityKey = nextKey
  emit(L, C_PIC_CREATED, created, pi, 0);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, pi, NONE, 0);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, pi, NONE, 0);
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, NONE, 0, start);  // activateChildInstance: key -1
  const uint32_t sk = new_key(L);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, sk, 0, start);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, sk, 0, start);
  emit(L, ZBHIP_PI_COMPLETE_ELEMENT, sk, 0, start);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETING, sk, 0, start);
  emit(L, ZBHIP_PI_ELEMENT_COMPLETED, sk, 0, start);
  const uint32_t sft = new_key(L);
  emit(L, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, sft, 0, f);
  const uint32_t nk = new_key(L);
  emit(L, ZBHIP_PI_ACTIVATE_ELEMENT, nk, 0, n);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATING, nk, 0, n);
  if (dst_tmr) {
    const uint32_t b = elem_of(L, n).w & 0xFFFF;
    const uint4 bw = elem_of(L, b);
    const uint32_t reps = (bw.w >> 8) & 0xFF;
    const uint32_t tmk = new_key(L);
    L.tm_x = b | (tmk << 16);
    L.tm_y = nk | (reps << 16) | (1u << 31);
    L.tm_due = L.sp->now_ms + (long long)bw.z;
    emit(L, C_TIMER_CREATED, tmk, nk, b, reps);
  }
  const uint32_t job = new_key(L);
  emit(L, C_JOB_CREATED, job, nk, n);
  emit(L, ZBHIP_PI_ELEMENT_ACTIVATED, nk, 0, n);
  L.nt = 1;
  tput(L, 0, make_uint2(n | (nk << 16), (job & 0xFFFF) | ((uint32_t)ZBHIP_PI_ELEMENT_ACTIVATED << 16) | (1u << 24)));
  L.pi_live = true;
  L.pi_state = ZBHIP_PI_ELEMENT_ACTIVATED;
  L.pi_child = 1;
  L.pi_asf = 0;
  return !L.fail;
}

// ---- CREATE batch templates (non-register variants) -------------------------------------------
// A process whose CREATE batch never waits (runtime.cpp create_template_word: every element
// reachable from the none start event is an event without wait state, a flow or a gateway; at most
// one exclusive gateway, right behind the start event) completes the instance inside the batch, and
// the batch's compact records depend only on the process, the name of the document's variable and
// the flow that gateway takes: key ordinals restart at 0 for a CREATE, and variable values never
// appear in the compact rows.  The first lane of a launch that runs such a batch through the general
// path (BpmnStreamProcessor FIFO) records its rows as the template of (process, variant); from the
// next launch on, a CREATE with the same variant only evaluates the gateway's condition and copies
// the rows.  A template written in the running launch is never read in it (launch_seq), so no
// fence is needed: launches are ordered by the stream.
constexpr int kTplReplayed = 0x7FFF;

template <class K>
__device__ __forceinline__ uint2* tpl_at(const StepParams& P, uint32_t proc, uint32_t v) {
  return P.tpl + ((size_t)proc * kTplVar + v) * kTplWords;
}
template <class K>
constexpr bool kTplOn = !K::REG && !K::M;
template <class K>
constexpr size_t tpl_lds_bytes() {
  return kTplOn<K> ? (size_t)kTplLdsProcs * kTplVar * kTplLdsWords * sizeof(uint2) : 0;
}

// -> kTplReplayed (the batch is in the lane), a variant to record after the general path, or -1
template <class K>
__device__ __forceinline__ int tpl_create(Lane<K>& L, uint32_t doc_count, uint32_t doc_begin, uint32_t& name,
                                          const uint2* tpl_lds) {
  const StepParams& P = *L.sp;
  const uint32_t tw = L.pb[7];
  name = 0xFFFF;
  if (!(tw & TPL_OK) || doc_count > 1 || L.limit <= 0 || L.limit > 0xFFFF || L.proc >= P.n_procs) return -1;
  uint32_t v = 0;
  const uint32_t gw = tw & 0xFFF;
  if (doc_count == 1) {
    const zbhip_doc_entry d = P.docs[doc_begin];
    vm_drain();
    name = d.name_id;
    // the variable as set_local_variable puts it (process scope, key ordinal 1): the condition's input
    L.vx0 = d.name_id;
    L.vy0 = 1u | ((uint32_t)d.type << 16);
    L.vv0 = d.value;
    L.nvars = 1;
  }
  if (gw != 0xFFF) {
    const uint4 w = elem_of(L, gw);
    const uint32_t f = find_sequence_flow(L, w, NONE);  // ExclusiveGatewayProcessor.findSequenceFlowToTake
    const uint32_t ob = w.y & 0xFFFF, oc = w.y >> 16;
    v = kTplVar;
    for (uint32_t i = 0; i < oc && i < (uint32_t)kTplVar; ++i)
      if (out_flow(L, ob + i) == f) v = i;
  }
  L.nvars = 0;
  L.vx0 = 0xFFFFFFFFu;
  L.vy0 = 0;
  L.vv0 = 0;
  if (L.fail || v >= (uint32_t)kTplVar) {  // an incident or no flow: the general path decides
    L.fail = 0;
    return -1;
  }
  // the workgroup's LDS copy (taken at kernel start: templates of earlier launches, complete) for
  // the first processes, HBM otherwise or for rows past the copy
  const bool in_lds = L.proc < (uint32_t)kTplLdsProcs;
  const uint2* tl = tpl_lds + ((size_t)L.proc * kTplVar + v) * kTplLdsWords;
  const uint2* t = tpl_at<K>(P, L.proc, v);
  const uint4 hd = *reinterpret_cast<const uint4*>(in_lds ? tl : t);
  // hd.x = state (2 valid) | variable name << 16, hd.y = launch it was recorded in,
  // hd.z = records | keys << 16, hd.w = transitions | batch limit << 16
  const uint32_t n = hd.z & 0xFFFF;
  if (hd.x != (2u | (name << 16)) || hd.y == P.launch_seq || (hd.w >> 16) != (uint32_t)L.limit || n > L.rec_cap ||
      n > (uint32_t)kTplRec)
    return (int)v;
  const uint2* rows = in_lds && n + 2 <= kTplLdsWords ? tl : t;
  for (uint32_t j = 0; j < n; ++j) {
    const uint2 r = rows[2 + j];
    if (j < (uint32_t)K::R) L.stage[j * K::B] = r;
    else L.rec[(size_t)j * K::B] = r;
  }
  L.nrec = n;
  L.transitions = hd.w & 0xFFFF;
  L.completed = 1;
  L.next_ord = (uint16_t)(hd.z >> 16);
  L.pi_live = false;
  L.pi_state = ZBHIP_PI_ELEMENT_COMPLETING;
  L.pi_child = L.pi_asf = 0;
  L.nt = 0;
  return kTplReplayed;
}

// after the general path: the batch's rows become the template of variant v, if it completed the
// instance and nothing was left for later batches (no row written unprocessed).  At most one lane
// per wave and chunk tries, and a workgroup tries a template once (its LDS copy's header marks the
// attempt): a first window of 10^7 CREATEs would otherwise send 10^7 CAS to one address (measured:
// the recording launch 20x slower than a replaying one).
template <class K>
__device__ __forceinline__ void tpl_record(Lane<K>& L, uint32_t v, uint32_t name, uint2* tpl_lds) {
  const StepParams& P = *L.sp;
  uint2* t = tpl_at<K>(P, L.proc, v);
  uint2* tl = L.proc < (uint32_t)kTplLdsProcs ? tpl_lds + ((size_t)L.proc * kTplVar + v) * kTplLdsWords : nullptr;
  // candidates: a recordable batch whose template this workgroup has not seen recorded or tried
  const bool want = !(L.fail || L.pi_live || !L.completed || L.nrec > (uint32_t)kTplRec || L.nrec > L.rec_cap) &&
                    (!tl || tl[0].x == 0) && *reinterpret_cast<volatile uint32_t*>(t) == 0u;
  const unsigned long long m = __ballot(want);
  if (!want || (threadIdx.x & 63) != (uint32_t)__builtin_ctzll(m)) return;
  if (tl) tl[0].x = 1;  // tried by this workgroup
  if (atomicCAS(reinterpret_cast<uint32_t*>(t), 0u, 1u) != 0u) return;  // recorded (or claimed) already
  bool clean = true;
  for (uint32_t j = 0; j < L.nrec; ++j) {
    const uint2 r = j < (uint32_t)K::R ? L.stage[j * K::B] : L.rec[(size_t)j * K::B];
    clean &= ((r.y >> 24) & F_UNPROCESSED) == 0;
    t[2 + j] = r;
  }
  t[1] = make_uint2(L.nrec | ((uint32_t)L.next_ord << 16), L.transitions | ((uint32_t)L.limit << 16));
  t[0] = make_uint2(clean ? 2u | (name << 16) : 3u, P.launch_seq);  // state and launch: one 8-byte store
}

// ---------------------------------------------------------------------------------------------
// k_step
// ---------------------------------------------------------------------------------------------
// ---- instance rows of one command, fetched ahead of its chunk --------------------------------
constexpr uint32_t kNoCmd = 0xFFFFFFFFu;

template <class K>
__device__ __forceinline__ uint32_t cmd_index(const StepParams& P, uint32_t chunk) {
  const uint32_t lane_id = chunk * K::B + threadIdx.x;
  if (lane_id >= P.n_launch) return kNoCmd;
  return P.order ? P.order[lane_id] : lane_id;
}
__device__ __forceinline__ uint4 load_cmd(const StepParams& P, uint32_t ci) {
  return ci != kNoCmd ? P.cmds[ci - P.cmd_base] : make_uint4(0, 0, 0, 0);
}
// header row, and the first element-instance slot of a waiting instance (a CREATE reads none).
// (Prefetching a CREATE's document entry here too was measured: -11 % on configs[2], the wider
// pipeline registers cost more than the dependent load they save.)
__device__ __forceinline__ void load_rows(const StepParams& P, uint32_t ci, const uint4& cw, uint4& h, uint2& s0) {
  h = make_uint4(0xFFFFFFFFu, 0, 0, 0);
  s0 = make_uint2(0xFFFFFFFFu, 0);
  if (ci != kNoCmd && cw.x < P.st.n) {
    h = P.st.hdr[cw.x];
    if ((cw.y & 0xFF) != ZBHIP_CMD_CREATE) s0 = P.st.slots[cw.x];
  }
}

struct Counters {
  uint32_t rec, trans, comp, keys, fb, cmd, tpl;
};


// ---- message path: instance loaded in the middle of a batch (a slot lane's local
// PROCESS_MESSAGE_SUBSCRIPTION command for an instance of this partition) --------------------
template <class K>
__device__ __forceinline__ void load_instance_mid(Lane<K>& L, uint32_t inst) {
  const StepParams& P = *L.sp;
  const uint32_t N = P.st.n;
  if (L.inst != kNoInst) { if (L.inst != inst) set_fail(L, FB_MESSAGE); return; }
  if (inst >= N) { set_fail(L, FB_MESSAGE); return; }
  const uint4 h = P.st.hdr[inst];
  const uint32_t proc = h.x & 0xFFFF;
  if (h.w == P.stamp) { set_fail(L, FB_FENCED); return; }
  if (proc == NONE || !((h.y >> 24) & 1) || proc >= P.n_procs) { set_fail(L, FB_MESSAGE); return; }
  const uint32_t nslots = (h.y >> 8) & 0xFF, nvars = (h.y >> 16) & 0xFF;
  if (nslots > (uint32_t)K::T) { set_fail(L, FB_TABLE); return; }
  L.inst = inst;
  L.proc = (uint16_t)proc;
  L.next_ord = h.x >> 16;
  L.i_first_ord = L.next_ord;
  L.pi_state = h.y & 0xFF;
  L.pi_live = true;
  L.pi_child = h.z & 0xFFFF;
  L.pi_asf = h.z >> 16;
  for (uint32_t sl = 0; sl < nslots; ++sl) tput(L, (int)sl, P.st.slots[(size_t)sl * N + inst]);
  L.nt = (int)nslots;
  L.nvars = (int)nvars;
#pragma unroll
  for (int v = 0; v < kVars; ++v)
    if (v < L.nvars) {
      const uint2 m = P.st.var_meta[(size_t)v * N + inst];
      var_put(L, v, m.x, m.y, P.st.var_val[(size_t)v * N + inst]);
    }
  L.pb = L.prog + L.prog[1 + proc];
  L.has_join = K::J && (L.pb[1] & 0xFFFF) != 0;
  if (L.has_join) {
    L.jw0 = P.st.join[inst];
    L.jw1 = P.st.join[(size_t)N + inst];
    L.jw2 = P.st.join[(size_t)2 * N + inst];
    L.jw3 = P.st.join[(size_t)3 * N + inst];
  }
  const uint4 pm = P.st.pms[inst];
  L.pm_x = pm.x;
  L.pm_y = pm.y;
  L.pm_z = pm.z;
  L.pm_w = pm.w;
  L.pm_msg = P.st.pms_msg[inst];
  L.pik = P.st.pi_key[inst];
  vm_drain();
}

// a follow-up subscription command of this partition (queue entry LQ_BIT | kind)
template <class K>
__device__ __forceinline__ void process_local(Lane<K>& L, uint32_t kind) {
  const uint32_t own = (uint32_t)L.sp->partition_id;
  switch (kind) {
    case LQ_MS_CREATE:  // from a catch event of the loaded instance
      ms_create(L, L.lq_slot, L.lq_corr, L.lq_name_bpmn, L.lq_intr, own, L.inst, L.lq_eord, L.lq_eik, L.lq_pik,
                iref(L, L.lq_eord), iref(L, 0));
      return;
    case LQ_PMS_CREATE: {  // acknowledgement of a subscription this partition opened
      const bool was_loaded = L.inst != kNoInst;
      load_instance_mid(L, L.lq_row);
      if (L.fail) return;
      const long long eik_p = was_loaded && !L.slot_lane ? iref(L, L.lq_eord) : L.lq_eik;
      const long long pik_p = was_loaded && !L.slot_lane ? iref(L, 0) : L.lq_pik;
      pms_create(L, L.lq_eord, L.lq_name_bpmn & 0xFFFF, eik_p, pik_p, own, L.lq_intr);
      return;
    }
    case LQ_PMS_CORRELATE:  // a message published on this partition for one of its instances
      load_instance_mid(L, L.lq_row);
      if (L.fail) return;
      pms_correlate(L, L.lq_eord, L.lq_name_bpmn, L.lq_eik, L.lq_pik, L.lq_msg, L.lq_corr, own, L.lq_eik, L.lq_pik);
      return;
    case LQ_MS_CORRELATE:
      ms_correlate(L, L.lq_slot, own, L.lq_row, L.lq_eord, L.lq_name_bpmn, L.lq_eik, L.lq_pik);
      return;
    case LQ_MS_DELETE:  // from an activity of the loaded instance closing its subscription
      ms_delete(L, L.lq_slot, own, L.inst, L.lq_eord, L.lq_name_bpmn, iref(L, L.lq_eord), iref(L, 0), L.lq_eik, L.lq_pik);
      return;
    case LQ_PMS_DELETE:  // the acknowledgement, back on the subscriber's instance (loaded: it sent the DELETE)
      if (L.inst != L.lq_row) { set_fail(L, FB_MESSAGE); return; }
      pms_delete(L, L.lq_eord, L.lq_name_bpmn & 0xFFFF);
      return;
    default:
      set_fail(L, FB_UNSUPPORTED);
  }
}

// an ended instance's header whose closing subscription waits for its PROCESS_MESSAGE_SUBSCRIPTION:DELETE
// (k_step's commit; a never-used slot's header is all ones)
__device__ __forceinline__ bool closing_pending(uint4 h) { return (h.x & 0xFFFF) == 0xFFFF && h.y == (1u << 25); }

// the initial command of a batch that is a message / subscription command
template <class K>
__device__ __forceinline__ void message_command(Lane<K>& L, uint32_t kind, uint32_t subject, uint32_t ref, uint32_t xi) {
  const StepParams& P = *L.sp;
  if (kind == ZBHIP_CMD_PUBLISH) { publish_message(L, subject, ref); return; }
  if (xi >= P.n_xparts) { set_fail(L, FB_UNSUPPORTED); return; }
  const zbhip_xpart_cmd x = P.xparts[xi];
  const uint32_t nb = (uint32_t)x.message_name | ((uint32_t)x.bpmn_process_id << 16);
  const uint32_t src = (uint32_t)x.source_partition;
  switch (kind) {
    case ZBHIP_CMD_MSG_SUB_CREATE:
      ms_create(L, subject, x.correlation_key, nb, x.interrupting, src, x.instance, x.element_ord,
                x.element_instance_key, x.process_instance_key, x.element_instance_key, x.process_instance_key);
      return;
    case ZBHIP_CMD_MSG_SUB_CORRELATE:
      ms_correlate(L, subject, src, x.instance, x.element_ord, nb, x.element_instance_key, x.process_instance_key);
      return;
    case ZBHIP_CMD_PMS_CREATE:
      pms_create(L, x.element_ord, x.message_name, x.element_instance_key, x.process_instance_key, src, x.interrupting);
      return;
    case ZBHIP_CMD_PMS_CORRELATE:
      if (L.proc == NONE) { set_fail(L, FB_MESSAGE); return; }
      pms_correlate(L, x.element_ord, nb, x.element_instance_key, x.process_instance_key, x.message_key,
                    x.correlation_key, src, x.element_instance_key, x.process_instance_key);
      return;
    case ZBHIP_CMD_MSG_SUB_DELETE:
      ms_delete(L, subject, src, x.instance, x.element_ord, nb, x.element_instance_key, x.process_instance_key,
                x.element_instance_key, x.process_instance_key);
      return;
    case ZBHIP_CMD_PMS_DELETE:
      pms_delete(L, x.element_ord, x.message_name);
      return;
    default:
      set_fail(L, FB_UNSUPPORTED);
  }
}

// deferred correlation-slot row writes (DbMessageSubscriptionState put / updateToCorrelatingState /
// remove).  Rows are claimed with a CAS so lanes of one launch inserting into the same slot never
// collide; readers only see states 1 (open) and 2 (correlating), never a row being written (3).
template <class K>
__device__ __forceinline__ void commit_slot_rows(Lane<K>& L) {
  const StepParams& P = *L.sp;
  uint32_t patch_mask = 0, patch_slot = L.op_slot, patch_what = 0;  // bit 0: sub_b, bit 1: sub_k
  if (L.op_ins) {
    int got = -1;
    for (int r = 0; r < kSubs && got < 0; ++r)
      if (atomicCAS(&P.st.sub_a[sub_ri(r, L.op_slot)].x, 0u, 3u) == 0u) got = r;
    if (got < 0) { set_fail(L, FB_MESSAGE); return; }  // correlation slot full
    const size_t ri = sub_ri(got, L.op_slot);
    P.st.sub_b[ri] = make_longlong2(L.ins_eik, L.ins_pik);
    P.st.sub_k[ri] = make_longlong2(L.ins_key, -1);
    // the row in one 16-byte store, state included.  No release fence: on gfx950 an agent-scope
    // fence writes back the XCD's whole L2 (buffer_wbl2), once per wave -- and nothing needs it.
    // Rows are read by later launches (kernel boundaries order them); a lane of this launch that
    // reads the slot meanwhile (another subscriber's duplicate check) matches only its own
    // (partition, instance, element) triple, which no concurrent insert carries, and removed rows
    // are zeroed, so even a torn read of a row being written matches nothing.
    P.st.sub_a[ri] = L.ins_a;
    patch_mask |= 1u << got;
    // the subscription key is always a reference of this window; the element / process instance
    // keys only when this window generated them (a received command carries real keys)
    patch_what |= 2u | (L.ins_eik < -1 || L.ins_pik < -1 ? 1u : 0u);
  }
  if (L.op_corr_mask) {
    for (int r = 0; r < kSubs; ++r)
      if ((L.op_corr_mask >> r) & 1) {
        const size_t ri = sub_ri(r, L.slot);
        P.st.sub_k[ri].y = L.op_corr_msg;
        uint4 a = P.st.sub_a[ri];
        P.st.sub_a[ri].x = (a.x & ~0xFFu) | 2u;
      }
    patch_mask |= L.op_corr_mask;
    patch_slot = L.slot;
    patch_what |= 2u;  // the correlating message key
  }
  if (L.op_open_mask) {  // non-interrupting rows correlated (after their CORRELATING of this batch, if any)
    for (int r = 0; r < kSubs; ++r)
      if ((L.op_open_mask >> r) & 1) {
        const size_t ri = sub_ri(r, L.op_open_slot);
        P.st.sub_a[ri].x = (P.st.sub_a[ri].x & ~0xFFu) | 1u;
      }
  }
  if (L.op_rm_mask) {
    for (int r = 0; r < kSubs; ++r)
      if ((L.op_rm_mask >> r) & 1) P.st.sub_a[sub_ri(r, L.op_rm_slot)] = make_uint4(0, 0, 0, 0);
    patch_mask &= ~(L.op_rm_slot == patch_slot ? L.op_rm_mask : 0u);
  }
  if (patch_mask && L.ci >= P.xcap) { set_fail(L, FB_MESSAGE); return; }
  if (patch_mask) {  // the key scan replaces this window's key references in these rows
    zbhip_xpart_cmd x = {};
    x.kind = XK_PATCH;
    x.correlation_key = patch_slot;
    x.instance = patch_mask;
    x.element_ord = (uint16_t)patch_what;
    P.xout[(size_t)L.n_out++ * P.xcap + L.ci] = x;
  }
  if (L.slot_lane) P.st.slot_hdr[L.slot].x = L.s_next_ord;
}

#ifdef ZB_STAMPS
// run_command phases (summed over waves, cycles): [0] row loads, [1] initial command,
// [2] FIFO: PI entries, [3] FIFO: local subscription entries, [4] commit, [5] FIFO entries
__device__ unsigned long long g_stamps_run[8];
#define ZB_RSTAMP(v) const unsigned long long v = clock64()
#else
#define ZB_RSTAMP(v)
#endif

// One command's whole batch on one lane; returns the number of records it staged.
template <class K, class Retire>
__device__ __forceinline__ uint32_t run_command(const StepParams& P, const uint32_t* prog, uint2* tbl_base,
                                                uint2* stage_base, uint32_t* q_base, uint2* region, uint32_t ci,
                                                uint4 cw, uint4 h, uint2 s0, Counters& acc, const Retire& retire,
                                                uint2* tpl_lds) {
  const uint32_t inst = cw.x;
  const uint32_t kind = cw.y & 0xFF;
  const uint32_t doc_count = (cw.y >> 8) & 0xFF;
  const uint32_t ref = cw.y >> 16;
  const uint32_t doc_begin = cw.z;
  const uint32_t N = P.st.n;
  ZB_RSTAMP(r0);
#ifdef ZB_STAMPS
  unsigned long long r_pi = 0, r_lq = 0, r_n = 0;
#endif

  Lane<K> L;
  L.tbl = tbl_base + threadIdx.x;
  L.q = q_base + threadIdx.x;
  L.r_t0 = L.r_t1 = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
  L.r_q0 = L.r_q1 = 0;
  L.stage = stage_base + threadIdx.x;
  // rows j >= R go straight to the chunk's output region, at j * B + lane (above the packed
  // rows, which never exceed B * R): each emit of a wave is one coalesced 512-byte store, and
  // the drain gather puts them in order
  L.rec = region + threadIdx.x;
  L.rec_cap = P.rec_cap;
  L.nrec = 0;
  L.fail = 0;
  L.transitions = 0;
  L.completed = 0;
  L.limit = P.max_cmds_in_batch;
  L.processed = 0;
  L.qh = L.qt = 0;
  L.g = 0;
  L.ci = ci;
  L.sp = &P;
  L.nt = 0;
  L.trig_key = NONE;
  L.trig_evt = NONE;
  L.n_map = 0;
  L.mo_set = 0;
  L.mo_type = 0;
  L.mo_val = 0;
  L.docs = P.docs;
  L.doc_begin = doc_begin;
  L.doc_count = doc_count;
  L.has_join = false;
  L.jw0 = L.jw1 = L.jw2 = L.jw3 = 0;
  L.nvars = 0;
  L.vx0 = L.vx1 = L.vx2 = L.vx3 = 0xFFFFFFFFu;
  L.vy0 = L.vy1 = L.vy2 = L.vy3 = 0;
  L.vv0 = L.vv1 = L.vv2 = L.vv3 = 0;
  if constexpr (K::S) {
    L.has_tmr = false;
    L.tm_x = L.tm_y = 0;
    L.tm_due = 0;
  }
  bool slot_kind = false;
  L.inst = inst;  // (K::M: a slot lane loads its instance later)
  if constexpr (K::M) {
    L.prog = prog;
    L.inst = inst;
    L.pm_x = L.pm_y = L.pm_z = L.pm_w = 0;
    L.pm_msg = -1;
    L.pik = -1;
    L.slot_lane = false;
    L.slot = 0;
    L.s_next_ord = L.s_first_ord = 0;
    L.n_out = L.n_pay = 0;
    L.x_sum = 0;
    L.lq_slot = L.lq_corr = L.lq_name_bpmn = L.lq_eord = 0;
    L.lq_row = kNoInst;
    L.lq_msg = L.lq_eik = L.lq_pik = -1;
    L.op_ins = false;
    L.op_slot = 0;
    L.ins_a = make_uint4(0, 0, 0, 0);
    L.ins_eik = L.ins_pik = L.ins_key = -1;
    L.op_corr_mask = L.op_rm_mask = L.op_rm_slot = 0;
    L.op_open_mask = L.op_open_slot = 0;
    L.op_corr_msg = -1;
    slot_kind = zb_slot_kind(kind);
  }

  const bool bad_cmd = (slot_kind ? inst >= P.st.n_slots : inst >= N) ||
                       (doc_count && (uint64_t)doc_begin + doc_count > P.n_docs);
  // fence: an earlier command of this subject in the window fell back (its state was left as it
  // was), so this one must follow it on the CPU engine in log order
  uint2 slot_row = make_uint2(0, 0);
  if constexpr (K::M) {
    if (slot_kind && !bad_cmd) slot_row = P.st.slot_hdr[inst];
  }
  const bool fenced = !bad_cmd && (slot_kind ? slot_row.y == P.stamp : h.w == P.stamp);
  if (fenced) set_fail(L, FB_FENCED);
  if (slot_kind) h = make_uint4(0xFFFFFFFFu, 0, 0, 0);
  if (bad_cmd) h = make_uint4(0xFFFFFFFFu, 0, 0, 0);
  L.proc = h.x & 0xFFFF;
  L.next_ord = h.x >> 16;
  L.pi_state = h.y & 0xFF;
  L.pi_live = (h.y >> 24) & 1;
  L.pi_child = h.z & 0xFFFF;
  L.pi_asf = h.z >> 16;
  const uint32_t nslots0 = (h.y >> 8) & 0xFF;
  const uint32_t nvars0 = (h.y >> 16) & 0xFF;

  if (bad_cmd) {
    set_fail(L, FB_UNSUPPORTED);  // never touches HBM outside the partition's arrays
    L.proc = NONE;
  } else if (slot_kind) {
    if constexpr (K::M) {  // a correlation slot: its rows are read on demand, instance loaded later
      L.slot_lane = true;
      L.slot = inst;
      L.inst = kNoInst;
      L.s_next_ord = L.s_first_ord = (uint16_t)slot_row.x;
      L.proc = NONE;
    }
  } else if (kind == CMD_FOLLOWUP && L.proc == NONE) {
    // a follow-up command read back from the log after its instance ended: the guard rejects it
    if (ref >= P.n_procs) set_fail(L, FB_BAD_PROCESS);
    L.proc = ref;
    L.pi_live = false;
  } else if (kind == ZBHIP_CMD_CREATE) {
    // CreateProcessInstanceProcessor.createProcessInstance (:129-158)
    if (L.proc != NONE || (K::M && closing_pending(h))) set_fail(L, FB_SLOT_IN_USE);
    else if (ref >= P.n_procs) set_fail(L, FB_BAD_PROCESS);
    L.proc = ref;
    L.next_ord = 0;
    L.pi_live = false;
    L.pi_state = 0;
    L.pi_child = L.pi_asf = 0;
  } else if (L.proc != NONE) {
    // load the waiting instance: element-instance slots -> LDS table, variables, join counters
    if (nslots0 > (uint32_t)K::T) set_fail(L, FB_TABLE);
    if (nslots0 > 0) tput(L, 0, s0);
    if (nslots0 > 1) {
      for (uint32_t s = 1; s < nslots0 && s < (uint32_t)K::T; ++s)
        tput(L, (int)s, P.st.slots[(size_t)s * N + inst]);
      vm_drain();
    }
    L.nt = (int)nslots0;
    L.nvars = (int)nvars0;
    if (L.nvars > 0) {
#pragma unroll
      for (int v = 0; v < kVars; ++v)
        if (v < L.nvars) {
          const uint2 m = P.st.var_meta[(size_t)v * N + inst];
          var_put(L, v, m.x, m.y, P.st.var_val[(size_t)v * N + inst]);
        }
      vm_drain();
    }
  }
  L.first_ord = L.next_ord;
  if constexpr (K::M) {
    L.i_first_ord = L.next_ord;
    if (!bad_cmd && !slot_kind) {
      if (kind == ZBHIP_CMD_CREATE) {
        L.pik = ref_cmd(ci, false, 0);
      } else if (L.proc != NONE || closing_pending(h)) {  // (an ended instance: its closing subscription)
        const uint4 pm = P.st.pms[inst];
        L.pm_x = pm.x;
        L.pm_y = pm.y;
        L.pm_z = pm.z;
        L.pm_w = pm.w;
        L.pm_msg = P.st.pms_msg[inst];
        L.pik = P.st.pi_key[inst];
        vm_drain();
      }
    }
  }
  if (!L.fail && L.proc != NONE) {
    L.pb = prog + prog[1 + L.proc];
    L.has_join = K::J && (L.pb[1] & 0xFFFF) != 0;
    if constexpr (K::S) {
      L.has_tmr = (L.pb[5] >> 16) & 1;
      if (L.has_tmr && kind != ZBHIP_CMD_CREATE) {
        const uint4 tr = P.st.tmr[inst];
        L.tm_x = tr.x;
        L.tm_y = tr.y;
        L.tm_due = (long long)(((unsigned long long)tr.w << 32) | tr.z);
        vm_drain();
      }
    }
    if (L.has_join && kind != ZBHIP_CMD_CREATE) {
      L.jw0 = P.st.join[inst];
      L.jw1 = P.st.join[(size_t)N + inst];
      L.jw2 = P.st.join[(size_t)2 * N + inst];
      L.jw3 = P.st.join[(size_t)3 * N + inst];
      vm_drain();
    }
  }

  ZB_RSTAMP(r1);
  // deploy-time compiled straight-line segments (linear chains): the batch is emitted without
  // the FIFO; anything outside the canonical states takes the general path below
  bool fast = false;
  if constexpr (K::REG) fast = fast_command(L, kind, ref, doc_count);
  if constexpr (K::J && !K::S && !K::M && !K::REG) {
    if (kind == ZBHIP_CMD_JOB_COMPLETE && !P.no_fast_scope) fast = fast_join_job(L, ref, doc_count);
    else if (kind == ZBHIP_CMD_CREATE && !P.no_fast_scope) fast = fast_fork_create(L, doc_count);
  }
  if constexpr (K::S && !K::IO) {
    if (kind == ZBHIP_CMD_JOB_COMPLETE && !P.no_fast_scope) fast = fast_scope_job(L, ref, doc_count);
    else if (kind == ZBHIP_CMD_CREATE && !P.no_fast_scope) fast = fast_scope_create(L, doc_count);
  }
  int tpl_v = -1;
  uint32_t tpl_name = 0xFFFF;
  bool tpl_hit = false;
  if constexpr (!K::REG && !K::M) {
    if (P.tpl && !fast && !L.fail && kind == ZBHIP_CMD_CREATE && L.proc != NONE) {
      tpl_v = tpl_create(L, doc_count, doc_begin, tpl_name, tpl_lds);
      if (tpl_v == kTplReplayed) {
        fast = true;
        tpl_v = -1;
        tpl_hit = true;
      }
    }
  }
  if (fast) {
#ifdef ZB_EXP_FASTONLY  // diagnostic build: the general path compiled out (its commands fall back)
  } else if (K::REG) {
    set_fail(L, FB_UNSUPPORTED);
#endif
  } else if (!L.fail && kind == ZBHIP_CMD_CREATE) {
    if ((L.pb[0] >> 16) == NONE) set_fail(L, FB_BAD_PROCESS);
    uint32_t pi = new_key(L);  // = ordinal 0
    // setVariablesFromDocument -> VariableBehavior.mergeLocalDocument (:60-82)
    if (doc_count) merge_local_document(L, pi, doc_begin, doc_count);
    follow_up(L, ZBHIP_PI_ACTIVATE_ELEMENT, pi, NONE, 0, false, false, pi);
    uint32_t created = new_key(L);  // CommandProcessorImpl.accept: entityKey = nextKey
    emit(L, C_PIC_CREATED, created, pi, 0);
  } else if (!L.fail && kind == ZBHIP_CMD_JOB_COMPLETE) {
    // JobCompleteProcessor (:47-92) + DefaultJobCommandPreconditionGuard (:26-46)
    const int t = L.proc == NONE ? -1 : tbl_find_job(L, ref);
    if (t < 0) {
      emit(L, kRejectBit | C_JOB_COMPLETE, ref, NONE, NONE, ZBHIP_REASON_JOB_NOT_FOUND);
    } else {
      uint2 e = tget(L, t);
      const uint32_t task_key = e.x >> 16, task_elem = e.x & 0xFFFF;
      emit(L, C_JOB_COMPLETED, ref, task_key, task_elem, (e.y >> 25) & 1u);  // (flag 1: an ACTIVATED job)
      if ((e.y >> 25) & 1u) note_activation(L, ref, inst);
      // the task's flow scope: the process instance, or (K::S) the sub-process instance around it
      bool fs_active = L.pi_live && L.pi_state == ZBHIP_PI_ELEMENT_ACTIVATED;
      uint32_t fsk = 0;
      if constexpr (K::S) {
        const uint32_t c = scope_of<K>(elem_of(L, task_elem));
        if (c != 0) {
          const int ts = scope_find(L, c);
          fs_active = ts >= 0 && ((tget(L, ts).y >> 16) & 0xFF) == ZBHIP_PI_ELEMENT_ACTIVATED;
          fsk = ts >= 0 ? tget(L, ts).x >> 16 : 0u;
          // a multi-instance inner instance whose COMPLETE_ELEMENT would be written unprocessed
          // would wait with jobKey -1 and no key of its loop variables left in its slot: fallback
          if (etype(elem_of(L, c)) == ZBHIP_EL_MULTI_INSTANCE_BODY && pending(L) + L.processed + 1 >= L.limit)
            set_fail(L, FB_BATCH_LIMIT);
        }
      }
      // JobCompletedApplier: job rows deleted; jobKey = -1 while the flow scope is active
      e.y &= ~(3u << 24);  // the job row (and its ACTIVATED state) is deleted
      L.done_job = e.y & 0xFFFF;  // (an inner instance's loop variables: keys below the job's)
      if (fs_active) e.y = (e.y & 0xFFFF0000u) | JOB_MINUS1;
      tput(L, t, e);
      if (fs_active) {  // afterAccept
        uint32_t pe = new_key(L);  // EventTriggerBehavior.triggeringProcessEvent
        emit(L, C_PE_TRIGGERING, pe, task_key, task_elem);
        L.trig_key = task_key;       // ProcessEventTriggeringApplier: EVENT_TRIGGER row
        follow_up(L, ZBHIP_PI_COMPLETE_ELEMENT, task_key, fsk, task_elem, true, true, task_key);
      }
    }
  } else if (!L.fail && kind == ZBHIP_CMD_TIMER_TRIGGER) {
    if constexpr (K::S) trigger_timer(L, ref, (long long)(((unsigned long long)cw.w << 32) | cw.z));
    else set_fail(L, FB_UNSUPPORTED);
  } else if (!L.fail && kind == CMD_FOLLOWUP) {
    // written to the log past the batch limit: the command is this batch's initial command
    enqueue(L, doc_begin);
  } else if (!L.fail) {
    if constexpr (K::M) message_command(L, kind, inst, ref, doc_begin);
    else set_fail(L, FB_UNSUPPORTED);
  }
  L.processed = kind == CMD_FOLLOWUP ? 0 : 1;
  ZB_RSTAMP(r2);

  // ---- the batch FIFO (ProcessingStateMachine.batchProcessing :328-374) ----
#ifdef ZB_EXP_FASTONLY
  if (K::REG) fast = true;
#endif
  while (!fast && L.qh < L.qt && !L.fail) {
    const uint32_t entry = dequeue(L);
#ifdef ZB_STAMPS
    ++r_n;
#endif
    if constexpr (K::M) {
      if (entry & LQ_BIT) {
        ZB_RSTAMP(q0);
        process_local(L, entry & 0xF);
        ++L.processed;
#ifdef ZB_STAMPS
        ZB_RSTAMP(q1); r_lq += q1 - q0;
#endif
        continue;
      }
    }
    ZB_RSTAMP(p0);
    process_pi(L, entry);
    ++L.processed;
#ifdef ZB_STAMPS
    ZB_RSTAMP(p1); r_pi += p1 - p0;
#endif
  }
  ZB_RSTAMP(r3);
  if constexpr (!K::REG && !K::M) {
    if (tpl_v >= 0) tpl_record(L, (uint32_t)tpl_v, tpl_name, tpl_lds);
  }

  retire();  // the caller's prefetch loads: retired before the first store of the commit
  // ---- commit: write back the instance (or leave it untouched on fallback) ----
  uint32_t ns = 0;
  if (!L.fail && L.pi_live) {
    for (int t = 0; t < L.nt; ++t)
      if (tget(L, t).x != 0xFFFFFFFFu) ++ns;
    if (ns > (uint32_t)kSlots) set_fail(L, FB_SLOTS);
  }
  uint32_t winst = inst;
  if constexpr (K::M) {
    winst = L.inst;
    if (!L.fail) commit_slot_rows(L);
  }
  // the counters are updated branch-free: per-branch updates are merged by the optimiser into a
  // store through a selected pointer, which puts the whole accumulator in scratch
  const bool ok = !L.fail;
  if (ok && L.pi_live && winst != kNoInst) {
    uint32_t s = 0;
    for (int t = 0; t < L.nt; ++t) {
      uint2 e = tget(L, t);
      if (e.x != 0xFFFFFFFFu) P.st.slots[(size_t)(s++) * N + winst] = e;
    }
#pragma unroll
    for (int v = 0; v < kVars; ++v)
      if (v < L.nvars) {
        P.st.var_meta[(size_t)v * N + winst] = make_uint2(var_x(L, v), var_y(L, v));
        P.st.var_val[(size_t)v * N + winst] = var_v(L, v);
      }
  }
  if (ok && L.has_join && winst != kNoInst) {
    const bool live = L.pi_live;  // a completed instance's counters are removed with it
    P.st.join[winst] = live ? L.jw0 : 0u;
    P.st.join[(size_t)N + winst] = live ? L.jw1 : 0u;
    P.st.join[(size_t)2 * N + winst] = live ? L.jw2 : 0u;
    P.st.join[(size_t)3 * N + winst] = live ? L.jw3 : 0u;
  }
  if constexpr (K::M) {
    // an ended instance keeps a closing subscription until its PROCESS_MESSAGE_SUBSCRIPTION:DELETE
    const bool keep = L.pi_live || ((L.pm_x >> 12) & 3) == 3;
    if (ok && winst != kNoInst) {
      P.st.pms[winst] = keep ? make_uint4(L.pm_x, L.pm_y, L.pm_z, L.pm_w) : make_uint4(0, 0, 0, 0);
      P.st.pms_msg[winst] = keep && ((L.pm_x >> 12) & 3) ? L.pm_msg : -1;
    }
  }
  if constexpr (K::S) {
    if (ok && winst != kNoInst && L.has_tmr) {
      const bool keep = L.pi_live && (L.tm_y >> 31);
      const unsigned long long d = (unsigned long long)L.tm_due;
      P.st.tmr[winst] = keep ? make_uint4(L.tm_x, L.tm_y, (uint32_t)d, (uint32_t)(d >> 32)) : make_uint4(0, 0, 0, 0);
    }
  }
  if (ok && winst != kNoInst) {
    // a completed instance frees its slot (rows removed with the instance) but keeps next_ord,
    // so late commands for the instance relabel consistently; bit 25: a closing subscription waits
    // for its PROCESS_MESSAGE_SUBSCRIPTION:DELETE (the slot is not free for a CREATE yet)
    const bool live = L.pi_live;
    bool pms_pending = false;
    if constexpr (K::M) pms_pending = ((L.pm_x >> 12) & 3) == 3;
    P.st.hdr[winst] = live ? make_uint4(L.proc | ((uint32_t)L.next_ord << 16),
                                       L.pi_state | (ns << 8) | ((uint32_t)L.nvars << 16) | (1u << 24),
                                       (uint32_t)L.pi_child | ((uint32_t)L.pi_asf << 16), 0)
                          : make_uint4(0xFFFFu | ((uint32_t)L.next_ord << 16), pms_pending ? (1u << 25) : 0u, 0, 0);
  }
  uint32_t nkeys = ok ? (uint16_t)(L.next_ord - L.first_ord) : 0u;
  uint32_t first = L.first_ord, npay = 0;
  if constexpr (K::M) {
    // slot lanes: the slot's keys first, then the instance loaded in the middle of the batch
    const uint32_t nsec = ok && L.slot_lane && L.inst != kNoInst ? (uint16_t)(L.next_ord - L.i_first_ord) : 0u;
    if (L.slot_lane) {
      nkeys = ok ? (uint16_t)(L.s_next_ord - L.s_first_ord) + nsec : 0u;
      first = L.s_first_ord;
    }
    npay = ok ? L.n_pay : 0u;
    // z: outbox entries (bits 0..3; sends first, a row patch last), sends (4..7), their common
    // target (8..23) unless mixed (31) -- the bucketing reads the outbox only for mixed targets
    P.cmd_hdr2[ci] = make_uint4(L.inst, L.i_first_ord | (nsec << 16),
                                ok ? L.n_out | ((L.x_sum & 0xF) << 4) | (L.x_sum & 0xFFFFFF00u) : 0u, npay);
  }
  if (!ok && !bad_cmd) {  // fence the subject(s) for the rest of the window
    if (slot_kind) {
      if constexpr (K::M) P.st.slot_hdr[inst].y = P.stamp;
    } else {
      P.st.hdr[inst].w = P.stamp;
    }
    if constexpr (K::M) {
      if (slot_kind && L.inst != kNoInst && L.inst < N) P.st.hdr[L.inst].w = P.stamp;
    }
  }
  const bool ended = ok && !L.pi_live && winst != kNoInst && L.proc != NONE;
  const uint32_t nrec = ok ? L.nrec : 0u;
  P.cmd_hdr[ci] = make_uint2(nrec | (nkeys << 16),
                             first | ((uint32_t)(ok ? ST_OK : ST_FALLBACK) << 16) | (L.fail << 24) |
                                 (ended ? HDR_ENDED : 0u));
  acc.cmd += 1;
  acc.fb += ok ? 0u : 1u;
  acc.tpl += tpl_hit && ok ? 1u : 0u;
#ifdef ZB_STAMPS
  {
    ZB_RSTAMP(r4);
    if ((threadIdx.x & 63) == 0) {
      const unsigned long long v[6] = {r1 - r0, r2 - r1, r_pi, r_lq, r4 - r3, r_n};
      for (int k = 0; k < 6; ++k) atomicAdd(&g_stamps_run[k], v[k]);
    }
  }
#endif
  acc.rec += nrec - npay;
  acc.trans += ok ? L.transitions : 0u;
  acc.comp += ok ? L.completed : 0u;
  acc.keys += nkeys;
  return nrec;
}

#ifdef ZB_STAMPS
// cycle stamps per phase (summed over waves): [0] top-of-chunk wait, [1] run_command,
// [2] scan + barrier, [3] flush issue, [4] chunks, [5] prologue (program staging + first loads)
__device__ unsigned long long g_stamps[8];
#define ZB_STAMP(v) const unsigned long long v = clock64()
#else
#define ZB_STAMP(v)
#endif

// k_step: workgroup g processes chunks g, g + G, g + 2G, ... of B commands (G = grid size,
// sized by the host to the resident workgroups).  The rows of a command are fetched two chunks
// ahead (command index three, command word two, header + first slot one chunk ahead), so the
// dependent load chain command -> instance rows overlaps the previous chunk's processing.
// Chunk c's records are compacted by a wavefront scan into output region region_base + c.
template <class K>
__global__ __launch_bounds__(K::B) __attribute__((amdgpu_waves_per_eu(K::W ? K::W : 1))) void k_step(StepParams P) {
  extern __shared__ __align__(16) uint32_t smem[];
  const uint32_t prog_words = (P.prog_words + 3) & ~3u;
  uint32_t* prog = smem;
  uint2* tbl_base = reinterpret_cast<uint2*>(smem + prog_words);
  uint2* stage_base = tbl_base + (K::REG ? 0 : K::T * K::B);
  uint32_t* q_base = reinterpret_cast<uint32_t*>(stage_base + K::R * K::B);
  // the flush's prefix array and owner map alias the FIFO and the element table, idle by then
  // (K::REG: table and FIFO are registers; the flush scratch follows the stage)
  uint32_t* pre = q_base;                                   // [B] first output record of each lane
  uint8_t* own = K::REG ? reinterpret_cast<uint8_t*>(q_base + K::B) : reinterpret_cast<uint8_t*>(tbl_base);
  static_assert(K::B <= 256, "owner map holds lane ids in bytes");
  static_assert(K::REG || (K::T * 8 >= K::R && K::Q >= 1), "flush scratch fits the table / FIFO regions");
  __shared__ uint32_t wsum[2][K::B / 64];
  ZB_STAMP(t_start);
#ifdef ZB_STAMPS
  unsigned long long acc_t[6] = {0, 0, 0, 0, 0, 0};
#endif
  // a speculatively launched untrusted window whose subject check found a repeat: no lane touches
  // state or output (uniform: the whole grid returns; the host replans and runs the window again)
  if (P.guard) {
    // an untrusted device window's subject check (k_subject_check): its verdict to the host (once per
    // launch), and a faulty window does nothing (the host replans it)
    const uint32_t g = *reinterpret_cast<const volatile uint32_t*>(P.guard);
    const uint32_t f = (g >> 2) == P.guard_stamp ? g & 3u : 0u;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      *reinterpret_cast<volatile uint32_t*>(P.guard_host) = (P.guard_stamp << 2) | f;
      __threadfence_system();
    }
    if (f) return;
  }
  const uint32_t n_chunks = (P.n_launch + K::B - 1) / K::B;
  const uint32_t G = gridDim.x;
  const uint32_t lane = threadIdx.x & 63;
  Counters acc = {0, 0, 0, 0, 0, 0, 0};

  // the first commands are requested before the program is staged, so the two latencies overlap
  // (the chain program -> command -> instance rows becomes max(program, command) -> rows)
  uint32_t c = blockIdx.x;
  uint32_t ci1 = cmd_index<K>(P, c);
  uint4 cw1 = load_cmd(P, ci1);
  uint32_t ci2 = cmd_index<K>(P, c + G);
  uint4 cw2 = load_cmd(P, ci2);
  uint32_t ci3 = cmd_index<K>(P, c + 2 * G);
  for (uint32_t i = threadIdx.x; i < P.prog_words; i += K::B) prog[i] = P.prog[i];
  // CREATE templates of the first processes (after the FIFO; alias nothing)
  uint2* tpl_lds = reinterpret_cast<uint2*>(q_base + (K::REG ? 0 : K::Q * K::B));
  if constexpr (kTplOn<K>) {
    constexpr uint32_t words = (uint32_t)kTplLdsProcs * kTplVar * kTplLdsWords;
    for (uint32_t i = threadIdx.x; i < words; i += K::B) {
      const uint32_t pv = i / kTplLdsWords, w = i % kTplLdsWords;
      tpl_lds[i] = P.tpl && pv / kTplVar < P.n_procs ? P.tpl[(size_t)pv * kTplWords + w] : make_uint2(0, 0);
    }
  }
  uint4 h1;
  uint2 s1;
  load_rows(P, ci1, cw1, h1, s1);
  __syncthreads();
  consume(ci1); consume(cw1); consume(h1); consume(s1); consume(cw2); consume(ci3);
#ifdef ZB_STAMPS
  { const uint32_t u = __builtin_amdgcn_readfirstlane(cw1.x + h1.x + s1.x);
    ZB_STAMP(t_pro); acc_t[5] += t_pro - t_start + (u == 0x12345678u); }
#endif

  for (uint32_t it = 0; c < n_chunks; c += G, ++it) {
    ZB_STAMP(t0);
    const uint32_t ci = ci1;
    const uint4 cw = cw1, h = h1;
    const uint2 s0 = s1;
    // advance the pipeline before touching the current command
    ci1 = ci2;
    cw1 = cw2;
    load_rows(P, ci1, cw1, h1, s1);
    ci2 = ci3;
    cw2 = load_cmd(P, ci2);
    ci3 = cmd_index<K>(P, c + 3 * G);
    ZB_STAMP(t1);

    uint2* out = P.out + (size_t)(P.region_base + c) * P.region_stride;
    uint32_t my_nrec = 0;
    // The prefetch loads just issued are retired inside run_command, right before its commit stores
    // (see Retire): by then they have had the whole batch logic to arrive, and no store is ahead of
    // them in the vmcnt queue.
    const auto retire = [&]() { consume(h1); consume(s1); consume(cw2); consume(ci3); };
    if (ci != kNoCmd)
      my_nrec = run_command<K>(P, prog, tbl_base, stage_base, q_base, out, ci, cw, h, s0, acc, retire, tpl_lds);
    else retire();
    ZB_STAMP(t2);

    // ---- wavefront scan compaction: the chunk's staged rows (j < R) go out contiguously, once;
    // rows j >= R are already in the region, above the packed run ----
    const uint32_t mc = min(my_nrec, (uint32_t)K::R);
    uint32_t inc = mc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(inc, off);
      if (lane >= (uint32_t)off) inc += o;
    }
    uint32_t* ws = wsum[it & 1];  // double-buffered: one barrier per chunk
    const bool wave_ovf = __ballot(my_nrec > (uint32_t)K::R) != 0;
    if (lane == 63) ws[threadIdx.x >> 6] = inc | (wave_ovf ? 0x80000000u : 0u);
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    bool ovf = false;
#pragma unroll
    for (int w = 0; w < K::B / 64; ++w) {
      const uint32_t v = ws[w] & 0x7FFFFFFFu;
      if (w < (int)(threadIdx.x >> 6)) wbase += v;
      total += v;
      ovf |= (ws[w] >> 31) != 0;
    }
    ZB_STAMP(t3);
    const uint32_t my_off = wbase + inc - mc;
    // homogeneous single-wave chunk (every lane staged the same n rows -- a window of one
    // command kind at one element, the common case of straight-line segments): record o of the
    // run is row o % n of lane o / n, so the copy needs no owner map; o / n by a 16-bit
    // reciprocal, exact for o < 2^16 / n
    const uint32_t n0 = __builtin_amdgcn_readfirstlane(mc);
    if (K::REG && n0 > 0 && __ballot(mc != n0) == 0 && total == K::B * n0) {
      const uint32_t m = (65536u + n0 - 1) / n0;
      for (uint32_t o = 2 * threadIdx.x; o < total; o += 2 * K::B) {
        const uint32_t l0 = (o * m) >> 16, j0 = o - l0 * n0;
        const uint32_t l1 = j0 + 1 == n0 ? l0 + 1 : l0, j1 = j0 + 1 == n0 ? 0 : j0 + 1;
        const uint2 r0 = stage_base[j0 * K::B + l0];
        const uint2 r1 = stage_base[j1 * K::B + l1];
        *reinterpret_cast<uint4*>(out + o) = make_uint4(r0.x, r0.y, r1.x, r1.y);
      }
      __builtin_amdgcn_wave_barrier();  // the next chunk reuses the stage
    } else {
      // packed copy: an owner map in LDS turns the lanes' columns into one contiguous run
      // (at most B * R rows) that the workgroup stores with 16-byte, fully coalesced writes.
      // The copy reads LDS alone, so its stores never wait on vector memory.
      pre[threadIdx.x] = my_off;
      for (uint32_t j = 0; j < mc; ++j) own[my_off + j] = (uint8_t)threadIdx.x;
      __syncthreads();
      // four output records per thread and iteration: one 4-byte owner read, then four
      // independent prefix reads and four independent row reads (no dependent LDS chain per
      // record), two 16-byte stores
#ifdef ZB_EXP_NOFLUSH  // diagnostic build: records staged but never copied out
      if (total == 0xFFFFFFFFu)
#endif
      for (uint32_t o = 4 * threadIdx.x; o < total; o += 4 * K::B) {
        const uint32_t ow = *reinterpret_cast<const uint32_t*>(own + o);
        const uint32_t n4 = total - o;  // >= 1
        const uint32_t l0 = ow & 0xFF;
        const uint32_t l1 = n4 > 1 ? (ow >> 8) & 0xFF : l0;
        const uint32_t l2 = n4 > 2 ? (ow >> 16) & 0xFF : l0;
        const uint32_t l3 = n4 > 3 ? ow >> 24 : l0;
        const uint32_t p0 = pre[l0], p1 = pre[l1], p2 = pre[l2], p3 = pre[l3];
        const uint2 r0 = stage_base[(o - p0) * K::B + l0];
        const uint2 r1 = stage_base[(n4 > 1 ? o + 1 - p1 : o - p0) * K::B + l1];
        const uint2 r2 = stage_base[(n4 > 2 ? o + 2 - p2 : o - p0) * K::B + l2];
        const uint2 r3 = stage_base[(n4 > 3 ? o + 3 - p3 : o - p0) * K::B + l3];
        if (n4 >= 4) {
          *reinterpret_cast<uint4*>(out + o) = make_uint4(r0.x, r0.y, r1.x, r1.y);
          *reinterpret_cast<uint4*>(out + o + 2) = make_uint4(r2.x, r2.y, r3.x, r3.y);
        } else {
          out[o] = r0;
          if (n4 > 1) out[o + 1] = r1;
          if (n4 > 2) out[o + 2] = r2;
        }
      }
      __syncthreads();  // the next chunk reuses the stage columns and the owner map
    }
    // region total; a region holding rows j >= R is flagged instead (bit 31) and leaves its lanes'
    // record counts for the drain path to total and interleave
    if (ovf) P.region_lanes[(size_t)(P.region_base + c) * K::B + threadIdx.x] = (uint16_t)my_nrec;
    if (threadIdx.x == 0) P.region_total[P.region_base + c] = ovf ? 0x80000000u : total;
#ifdef ZB_STAMPS
    ZB_STAMP(t4);
    acc_t[0] += t1 - t0; acc_t[1] += t2 - t1; acc_t[2] += t3 - t2; acc_t[3] += t4 - t3; acc_t[4] += 1;
#endif
  }
#ifdef ZB_STAMPS
  if (lane == 0)
    for (int k = 0; k < 6; ++k) atomicAdd(&g_stamps[k], acc_t[k]);
#endif

  // ---- statistics: wave64 reduction, waves through LDS, one add per counter into one of 64
  // spread rows (non-returning atomics, no hot line) ----
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    acc.rec += __shfl_xor(acc.rec, off);
    acc.trans += __shfl_xor(acc.trans, off);
    acc.comp += __shfl_xor(acc.comp, off);
    acc.keys += __shfl_xor(acc.keys, off);
    acc.fb += __shfl_xor(acc.fb, off);
    acc.cmd += __shfl_xor(acc.cmd, off);
    acc.tpl += __shfl_xor(acc.tpl, off);
  }
  __shared__ uint32_t wstat[K::B / 64][8];
  if (lane == 0) {
    uint32_t* w = wstat[threadIdx.x >> 6];
    w[0] = acc.rec; w[1] = acc.trans; w[2] = acc.comp; w[3] = acc.keys; w[4] = acc.fb; w[5] = acc.cmd;
    w[6] = acc.tpl;
  }
  __syncthreads();
  if (threadIdx.x < 7) {
    uint32_t sum = 0;
#pragma unroll
    for (int w = 0; w < K::B / 64; ++w) sum += wstat[w][threadIdx.x];
    if (sum) atomicAdd(&P.stats[(blockIdx.x & 63) * 8 + threadIdx.x], (unsigned long long)sum);
  }
}

// ---------------------------------------------------------------------------------------------
// drain path (not in the hot loop): gather the workgroup regions into one contiguous buffer
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t o = __shfl_up(v, off);
    if (lane >= (uint32_t)off) v += o;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan_u(uint32_t v) { return wave_incl_scan(v); }

// single workgroup: exclusive scan of the region totals (64-bit total); a flagged region's total
// is the sum of its B lane counts
__global__ __launch_bounds__(1024) void k_scan_regions(const uint32_t* tot, const uint16_t* lanes, uint32_t B,
                                                      uint32_t nr, unsigned long long* off,
                                                      unsigned long long* total) {
  __shared__ unsigned long long ws[16];
  __shared__ unsigned long long carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nr; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    uint32_t v = i < nr ? tot[i] : 0;
    if (v >> 31) {
      v = 0;
      for (uint32_t l = 0; l < B; ++l) v += lanes[(size_t)i * B + l];
    }
    const uint32_t inc = wave_incl_scan(v);
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = inc;
    __syncthreads();
    unsigned long long wb = 0;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) wb += ws[w];
    const unsigned long long c = carry;
    if (i < nr) off[i] = c + wb + inc - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = c + wb + inc;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// region g starts at g * region_stride records (the workgroup size B of the run x rec_cap).  A
// region without rows j >= R is one packed run; one with them (bit 31 of its total) holds the
// lanes' first R rows packed at the front and row j >= R of lane l at j * B + l, and the lanes'
// record counts in lanes[g * B ..]: each lane's records are copied in order (drain path only).
__global__ __launch_bounds__(256) void k_gather(const uint2* regions, const uint32_t* tot, const uint16_t* lanes,
                                                const unsigned long long* off, size_t region_stride, uint32_t B,
                                                uint32_t R, uint2* out) {
  const uint32_t g = blockIdx.x;
  const uint32_t t = tot[g];
  const uint2* src = regions + (size_t)g * region_stride;
  uint2* dst = out + off[g];
  if (!(t >> 31)) {
    for (uint32_t i = threadIdx.x; i < t; i += 256) dst[i] = src[i];
    return;
  }
  __shared__ uint32_t wc[4], wn[4];
  const uint32_t l = threadIdx.x;
  const uint32_t n = l < B ? lanes[(size_t)g * B + l] : 0u;
  const uint32_t c = min(n, R);
  const uint32_t ic = wave_incl_scan(c), in = wave_incl_scan(n);
  if ((l & 63) == 63) {
    wc[l >> 6] = ic;
    wn[l >> 6] = in;
  }
  __syncthreads();
  uint32_t bc = 0, bn = 0;
  for (uint32_t w = 0; w < (l >> 6); ++w) {
    bc += wc[w];
    bn += wn[w];
  }
  const uint32_t cp = bc + ic - c, fp = bn + in - n;
  for (uint32_t j = 0; j < n; ++j) dst[fp + j] = j < R ? src[cp + j] : src[(size_t)j * B + l];
}


// ---------------------------------------------------------------------------------------------
// message path, after the k_step launches of a window (KMsg partitions only)
// ---------------------------------------------------------------------------------------------
// Key scan: DbKeyGenerator hands out keys in log order, so command c's keys start at
// counter + sum_{c' < c} nkeys(c') (exclusive scan over the window, 64-bit).  With the bases the
// device resolves the window's key references in the outbox and in the correlation-slot rows,
// writes each created instance's real process-instance key, and advances the counter -- so the
// cross-partition exchange never needs the host.
struct KeyScanParams {
  const uint2* cmd_hdr;
  const uint4* cmd_hdr2;
  const uint4* cmds;
  uint32_t n;
  unsigned long long* block_sum;  // [blocks]
  unsigned long long* base;       // [n] key counter value before command c's first key
  unsigned long long* counter;    // [1] the partition's key counter (last generated value)
  zbhip_xpart_cmd* xout;
  uint32_t xcap;
  long long* pi_key;
  uint32_t n_inst;
  uint4* sub_a;
  longlong2* sub_b;
  longlong2* sub_k;
  uint32_t n_slots;
  long long pbits;
};

constexpr int kScanB = 1024;

__global__ __launch_bounds__(kScanB) void k_key_block_sums(KeyScanParams K) {
  const uint32_t i = blockIdx.x * kScanB + threadIdx.x;
  uint32_t v = i < K.n ? K.cmd_hdr[i].x >> 16 : 0u;
  v = wave_incl_scan_u(v);
  __shared__ uint32_t ws[kScanB / 64];
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kScanB / 64; ++w) t += ws[w];
    K.block_sum[blockIdx.x] = t;
  }
}

// single workgroup: exclusive scan of the block sums (in place), counter advanced at the end
__global__ __launch_bounds__(1024) void k_key_scan_sums(KeyScanParams K, uint32_t nb) {
  __shared__ unsigned long long ws[16];
  __shared__ unsigned long long carry;
  if (threadIdx.x == 0) carry = *K.counter;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint32_t i = b0 + threadIdx.x;
    const unsigned long long v = i < nb ? K.block_sum[i] : 0ull;
    unsigned long long inc = v;
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned long long o = __shfl_up(inc, off);
      if (lane >= (uint32_t)off) inc += o;
    }
    if (lane == 63) ws[threadIdx.x >> 6] = inc;
    __syncthreads();
    unsigned long long wb = 0;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) wb += ws[w];
    const unsigned long long c = carry;
    if (i < nb) K.block_sum[i] = c + wb + inc - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = c + wb + inc;
    __syncthreads();
  }
  if (threadIdx.x == 0) *K.counter = carry;
}

// a key reference of window command rc, given that command's headers and key base
__device__ __forceinline__ long long resolve_with(unsigned long long v, uint2 h, uint4 h2, unsigned long long base,
                                                  long long pbits) {
  const uint32_t sec = (v >> 16) & 1, ord = v & 0xFFFF;
  const uint32_t nsec = h2.y >> 16;
  const uint32_t nprim = (h.x >> 16) - nsec;
  const unsigned long long off = sec ? nprim + (uint16_t)(ord - (h2.y & 0xFFFF)) : (uint16_t)(ord - (h.y & 0xFFFF));
  return pbits + (long long)(base + 1 + off);
}

__device__ __forceinline__ long long resolve_cmd_ref(const KeyScanParams& K, long long ref) {
  if (ref >= -1) return ref;
  const unsigned long long v = (unsigned long long)(-2 - ref);
  if ((v >> 62) & 1) return ref;  // a subject ordinal: resolved by the host drain
  const uint32_t c = (uint32_t)(v >> 17);
  if (c >= K.n) return ref;
  return resolve_with(v, K.cmd_hdr[c], K.cmd_hdr2[c], K.base[c], K.pbits);
}

// the common case: a reference of the patching command itself, from the registers holding its
// headers (every reference k_step writes names its own command; another command's only when a
// lane copied a row that a concurrent lane of the launch had just inserted)
__device__ __forceinline__ long long resolve_own(const KeyScanParams& K, long long ref, uint32_t c, uint2 h, uint4 h2,
                                                 unsigned long long base) {
  if (ref >= -1) return ref;
  const unsigned long long v = (unsigned long long)(-2 - ref);
  if ((v >> 62) & 1) return ref;
  if ((uint32_t)(v >> 17) != c) return resolve_cmd_ref(K, ref);
  return resolve_with(v, h, h2, base, K.pbits);
}

__global__ __launch_bounds__(kScanB) void k_key_apply(KeyScanParams K) {
  const uint32_t i = blockIdx.x * kScanB + threadIdx.x;
  const uint32_t v = i < K.n ? K.cmd_hdr[i].x >> 16 : 0u;
  const uint32_t inc = wave_incl_scan_u(v);
  __shared__ uint32_t ws[kScanB / 64];
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = inc;
  __syncthreads();
  unsigned long long b = K.block_sum[blockIdx.x];
  for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) b += ws[w];
  if (i < K.n) K.base[i] = b + inc - v;
}

__device__ __forceinline__ long long ll_of(uint32_t lo, uint32_t hi) {
  return (long long)(((unsigned long long)hi << 32) | lo);
}

// second pass (all bases known): patch references that may point at any command of the window.
// Every load of a command is issued before its first store (an outbox entry as three 16-byte
// loads), so a thread waits for one round of loads, not for a chain through its own stores.
__global__ __launch_bounds__(256) void k_key_patch(KeyScanParams K) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= K.n) return;
  const uint2 h = K.cmd_hdr[c];
  const uint4 h2 = K.cmd_hdr2[c];
  const uint4 cw = K.cmds[c];
  const unsigned long long base = K.base[c];
  if (((h.y >> 16) & 0xFF) != ST_OK) return;
  if ((cw.y & 0xFF) == ZBHIP_CMD_CREATE && cw.x < K.n_inst)  // ordinal 0 of the CREATE batch
    K.pi_key[cw.x] = K.pbits + (long long)(base + 1 + (uint16_t)(0 - (h.y & 0xFFFF)));
  const uint32_t nout = min(h2.z & 0xF, (uint32_t)kOut);
  for (uint32_t j = 0; j < nout; ++j) {
    uint4* xp = reinterpret_cast<uint4*>(K.xout + (size_t)j * K.xcap + c);
    const uint4 q0 = xp[0];  // element / process instance keys
    const uint4 q1 = xp[1];  // message key, correlation key (row patch: slot), instance (row mask)
    const uint4 q2 = xp[2];  // element_ord (row patch: fields), name, bpmn process id, kind, ...
    if (((q2.y >> 16) & 0xFF) == XK_PATCH) {
      const uint32_t slot = q1.z, mask = q1.w, what = q2.x & 0xFFFF;
      if (slot >= K.n_slots) continue;
      // only the row fields that may hold references of this window: random rows, so every
      // array left alone saves a read-modify-write of a line
      for (int r = 0; r < kSubs; ++r)
        if ((mask >> r) & 1) {
          const size_t ri = sub_ri(r, slot);
          if (what & 1) {
            const longlong2 bb = K.sub_b[ri];
            K.sub_b[ri] = make_longlong2(resolve_own(K, bb.x, c, h, h2, base), resolve_own(K, bb.y, c, h, h2, base));
          }
          if (what & 2) {
            const longlong2 kk = K.sub_k[ri];
            K.sub_k[ri] = make_longlong2(resolve_own(K, kk.x, c, h, h2, base), resolve_own(K, kk.y, c, h, h2, base));
          }
        }
      continue;
    }
    const long long eik = ll_of(q0.x, q0.y), pik = ll_of(q0.z, q0.w), msg = ll_of(q1.x, q1.y);
    const long long e2 = resolve_own(K, eik, c, h, h2, base), p2 = resolve_own(K, pik, c, h, h2, base),
                    m2 = resolve_own(K, msg, c, h, h2, base);
    if (e2 != eik || p2 != pik)
      xp[0] = make_uint4((uint32_t)e2, (uint32_t)((unsigned long long)e2 >> 32), (uint32_t)p2,
                         (uint32_t)((unsigned long long)p2 >> 32));
    if (m2 != msg) reinterpret_cast<long long*>(xp + 1)[0] = m2;
  }
}

// Outbox buckets by target partition, stable in log order (what the all-to-all sends):
// per-block counts, a scan (target-major), then a scatter that keeps each block's order.
struct BucketParams {
  const uint2* cmd_hdr;
  const uint4* cmd_hdr2;
  const zbhip_xpart_cmd* xout;
  uint32_t xcap;
  uint32_t n;
  uint32_t parts;
  uint32_t* blk_cnt;     // [blocks][parts] -> exclusive offsets
  uint32_t* counts;      // [parts]
  zbhip_xpart_cmd* out;
};
constexpr int kBucketB = 256;

// The targets (1-based partition ids, 0 = none) of command c's sent entries.  The command header
// summarises them (count and common target); only a command whose sends go to several partitions
// has its outbox read: the bpmn_process_id/kind/interrupting word (bytes 36..39) and the
// source/target word (40..43) of each entry.
__device__ __forceinline__ void load_targets(const BucketParams& Q, uint32_t c, uint32_t (&tg)[kOut]) {
  uint32_t z = 0;
  if (c < Q.n && ((Q.cmd_hdr[c].y >> 16) & 0xFF) == ST_OK) z = Q.cmd_hdr2[c].z;
  const uint32_t nout = min(z & 0xF, (uint32_t)kOut), nsend = (z >> 4) & 0xF, tgt = (z >> 8) & 0xFFFF;
  const bool mixed = z >> 31;
#pragma unroll
  for (int j = 0; j < kOut; ++j) {
    tg[j] = !mixed && (uint32_t)j < nsend ? tgt : 0u;
    if (mixed && (uint32_t)j < nout) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(Q.xout + (size_t)j * Q.xcap + c);
      const uint32_t kw = w[9], tw = w[10];
      if (((kw >> 16) & 0xFF) != XK_PATCH) tg[j] = (uint32_t)(int32_t)(int16_t)(tw >> 16);
    }
  }
}

__device__ __forceinline__ uint32_t count_to(const uint32_t (&tg)[kOut], uint32_t t) {
  uint32_t k = 0;
#pragma unroll
  for (int j = 0; j < kOut; ++j) k += tg[j] == t + 1;
  return k;
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t& total) {
  __shared__ uint32_t ws[kBucketB / 64];
  const uint32_t inc = wave_incl_scan_u(v);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t b = 0;
  total = 0;
  for (int w = 0; w < kBucketB / 64; ++w) {
    if (w < (int)(threadIdx.x >> 6)) b += ws[w];
    total += ws[w];
  }
  __syncthreads();
  return b + inc - v;
}

// per-block counts by target: an LDS histogram (one pass over the outbox, any partition count)
constexpr uint32_t kMaxParts = 1024;
__global__ __launch_bounds__(kBucketB) void k_bucket_count(BucketParams Q) {
  __shared__ uint32_t hist[kMaxParts];
  for (uint32_t t = threadIdx.x; t < Q.parts; t += kBucketB) hist[t] = 0;
  __syncthreads();
  uint32_t tg[kOut];
  load_targets(Q, blockIdx.x * kBucketB + threadIdx.x, tg);
#pragma unroll
  for (int j = 0; j < kOut; ++j)
    if (tg[j] - 1u < Q.parts) atomicAdd(&hist[tg[j] - 1], 1u);
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < Q.parts; t += kBucketB) Q.blk_cnt[(size_t)blockIdx.x * Q.parts + t] = hist[t];
}

// The scan of the per-block counts, target-major (bucket t after buckets 0..t-1, blocks in order):
// k_bucket_scan_groups scans groups of 1024 block counts per target in parallel (local offsets,
// group totals), k_bucket_scan_bases turns the few group totals into group bases and the counts.
constexpr int kScanG = 1024;
__global__ __launch_bounds__(kScanG) void k_bucket_scan_groups(BucketParams Q, uint32_t nb, uint32_t* grp) {
  const uint32_t b = blockIdx.x * kScanG + threadIdx.x;
  __shared__ uint32_t ws[kScanG / 64];
  for (uint32_t t = 0; t < Q.parts; ++t) {
    const uint32_t v = b < nb ? Q.blk_cnt[(size_t)b * Q.parts + t] : 0u;
    const uint32_t inc = wave_incl_scan_u(v);
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint32_t base = 0, total = 0;
    for (int w = 0; w < kScanG / 64; ++w) {
      if (w < (int)(threadIdx.x >> 6)) base += ws[w];
      total += ws[w];
    }
    if (b < nb) Q.blk_cnt[(size_t)b * Q.parts + t] = base + inc - v;
    if (threadIdx.x == 0) grp[(size_t)blockIdx.x * Q.parts + t] = total;
    __syncthreads();
  }
}

__global__ __launch_bounds__(64) void k_bucket_scan_bases(BucketParams Q, uint32_t ng, uint32_t* grp) {
  if (threadIdx.x != 0) return;
  uint32_t off = 0;
  for (uint32_t t = 0; t < Q.parts; ++t) {
    const uint32_t start = off;
    for (uint32_t g = 0; g < ng; ++g) {
      const uint32_t v = grp[(size_t)g * Q.parts + t];
      grp[(size_t)g * Q.parts + t] = off;
      off += v;
    }
    Q.counts[t] = off - start;
  }
}

// the scatter visits only the targets present in the block (an LDS bit set), in target order; the
// block scan per target keeps log order (command, then entry) inside each bucket
__global__ __launch_bounds__(kBucketB) void k_bucket_scatter(BucketParams Q, const uint32_t* grp) {
  __shared__ uint32_t present[kMaxParts / 32];
  for (uint32_t t = threadIdx.x; t < kMaxParts / 32; t += kBucketB) present[t] = 0;
  __syncthreads();
  const uint32_t c = blockIdx.x * kBucketB + threadIdx.x;
  const uint32_t g = blockIdx.x / kScanG;
  uint32_t tg[kOut];
  load_targets(Q, c, tg);
#pragma unroll
  for (int j = 0; j < kOut; ++j)
    if (tg[j] - 1u < Q.parts) atomicOr(&present[(tg[j] - 1) >> 5], 1u << ((tg[j] - 1) & 31));
  __syncthreads();
  for (uint32_t wi = 0; wi < (Q.parts + 31) / 32; ++wi) {
    uint32_t bits = present[wi];  // the same for every thread: uniform loop
    while (bits) {
      const uint32_t t = wi * 32 + __builtin_ctz(bits);
      bits &= bits - 1;
      uint32_t tot;
      const uint32_t mine = count_to(tg, t);
      uint32_t o = grp[(size_t)g * Q.parts + t] + Q.blk_cnt[(size_t)blockIdx.x * Q.parts + t] + block_excl_scan(mine, tot);
      if (mine) {
#pragma unroll
        for (int j = 0; j < kOut; ++j)
          if (tg[j] == t + 1) Q.out[o++] = Q.xout[(size_t)j * Q.xcap + c];
      }
    }
  }
}

// zbhip_exchange_gather: one block row per (source, target) pair, a grid-stride copy of the pair's
// 48-byte entries from the source's bucket for the target to its place in the target's inbox
__global__ __launch_bounds__(256) void k_xgather(XGather A) {
  const uint32_t s = blockIdx.y / A.P, t = blockIdx.y % A.P;
  uint32_t so = 0, dof = 0;
  for (uint32_t q = 0; q < A.P; ++q) {
    if (q < t) so += A.counts[s * A.P + q];
    if (q < s) dof += A.counts[q * A.P + t];
  }
  const uint32_t n = A.counts[s * A.P + t];
  const uint4* src = reinterpret_cast<const uint4*>(A.src[s] + so);
  uint4* dst = reinterpret_cast<uint4*>(A.dst[t] + dof);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < 3 * n; i += gridDim.x * 256) dst[i] = src[i];
}

// window of received cross-partition commands (exchange receiving side): one command per entry
__global__ __launch_bounds__(256) void k_xpart_window(const zbhip_xpart_cmd* xp, uint32_t n, uint4* cmds) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const zbhip_xpart_cmd x = xp[i];
  const bool pms = zb_pms_kind(x.kind);
  cmds[i] = make_uint4(pms ? x.instance : x.correlation_key, x.kind, i, 0);  // zbhip_command layout
}

constexpr uint32_t kCheckPerThread = 1;

// Subject check of a device-resident window (zbhip_submit_device*): every command claims its
// subject (instance slot, or correlation slot for MESSAGE / MESSAGE_SUBSCRIPTION commands) with the
// window's stamp; a second claim in the window flags a duplicate (bit 0), a subject out of range or
// an unknown kind bit 1.  A flagged lane raises the window's guard word gw to stamp << 2 | flags
// (atomicMax: stamps grow, so the word needs no reset between windows, and clean windows write nothing;
// the host alternates two words by stamp parity).  The
// window's k_step reads the verdict (StepParams.guard) and publishes it to the host; a caller that
// needs it before any k_step runs launches k_check_publish.
__global__ __launch_bounds__(256) void k_subject_check(const uint4* cmds, uint32_t n, uint32_t n_inst, uint32_t n_slots,
                                                       uint32_t* seen, uint32_t stamp, uint32_t* gw) {
  // kCheckPerThread commands a thread, strided by the grid (coalesced loads and claims)
  const uint32_t stride = gridDim.x * 256;
  uint32_t f = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCheckPerThread; ++k) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x + k * stride;
    if (i >= n) break;
    const uint4 c = cmds[i];
    const uint32_t kind = c.y & 0xFF;
    const bool sk = zb_slot_kind(kind);
    const bool known = (kind >= ZBHIP_CMD_CREATE && kind <= ZBHIP_CMD_MSG_SUB_CORRELATE) ||
                       kind == ZBHIP_CMD_MSG_SUB_DELETE || kind == ZBHIP_CMD_PMS_DELETE;
    if (!known || (sk ? c.x >= n_slots : c.x >= n_inst)) {
      f |= 2;
    } else if (atomicExch(&seen[(sk ? n_inst : 0u) + c.x], stamp) == stamp) {
      f |= 1;
    }
  }
  if (f) atomicMax(gw, (stamp << 2) | f);  // rare: a faulty window
}

// The verdict of the window checked with `stamp` into host-mapped memory (stamp << 2 | flags)
__global__ void k_check_publish(const uint32_t* gw, uint32_t stamp, uint32_t* host) {
  if (threadIdx.x != 0) return;
  const uint32_t g = *reinterpret_cast<const volatile uint32_t*>(gw);
  *reinterpret_cast<volatile uint32_t*>(host) = (stamp << 2) | ((g >> 2) == stamp ? g & 3u : 0u);
  __threadfence_system();
}

// A device window's launch order by subject (instance slots, then correlation slots): the stable
// radix sort keeps a subject's commands in log order, and a wave's lanes then read neighbouring
// instance rows (an exchange inbox arrives as one run per sending partition, each spread over the
// receiver's slots).  The records still come out per command (the drain and the key scan index
// commands, not lanes).
__global__ __launch_bounds__(256) void k_subject_keys(const uint4* cmds, uint32_t n, uint32_t n_inst, uint32_t* keys,
                                                      uint32_t* idx) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4 c = cmds[i];
  const uint32_t kind = c.y & 0xFF;
  const bool sk = zb_slot_kind(kind);
  keys[i] = (sk ? n_inst : 0u) + c.x;
  idx[i] = i;
}
size_t subject_sort_temp_bytes(uint32_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 32);
  return bytes;
}
hipError_t launch_subject_sort(const uint4* cmds, uint32_t n, uint32_t n_inst, uint32_t n_subjects, uint32_t* k0,
                               uint32_t* k1, uint32_t* v0, uint32_t* order, void* temp, size_t temp_bytes,
                               hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_subject_keys, dim3((n + 255) / 256), dim3(256), 0, s, cmds, n, n_inst, k0, v0);
  int bits = 1;
  while (bits < 32 && (1ull << bits) < n_subjects) ++bits;
  return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k0, k1, v0, order, (int)n, 0, bits, s);
}

// JOB_BATCH:ACTIVATE on the device (JobBatchActivatedApplier -> DbJobState.activate): the jobs the
// host picked from its JOB_ACTIVATABLE index are marked ACTIVATED in their element-instance slot
// (flags bit 1), and each job's element-instance slot word, process, and the instance's variables
// (JobVariablesCollector's input) are gathered for the JOB_BATCH:ACTIVATED record.
struct ActivatedOut {
  uint4 a;             // x = slot word (elem | key ord << 16), y = hdr.x, z = hdr.y, w = 1 found
  uint2 meta[kVars];
  long long val[kVars];
  uint2 slots[kSlots]; // the instance's element instances (the job's enclosing scopes: variables)
};
__global__ __launch_bounds__(256) void k_activate_jobs(DevState st, const uint2* jobs, uint32_t n, ActivatedOut* out,
                                                      uint32_t worker, unsigned long long deadline) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  // y bit 16: the host's state says ACTIVATABLE although the row holds a stored activation (a timed-out
  // job, DbJobState.timeout keeps the deadline and worker): activate it again
  // y bit 17: peek (zbhip_job_variables: a pushed job's variables, nothing written)
  const uint32_t inst = jobs[i].x, ord = jobs[i].y & 0xFFFF, again = (jobs[i].y >> 16) & 1u, peek = (jobs[i].y >> 17) & 1u;
  ActivatedOut o = {};
  if (inst < st.n) {
    const uint4 h = st.hdr[inst];
    const uint32_t nslots = (h.y >> 8) & 0xFF, nvars = (h.y >> 16) & 0xFF;
    bool marked = false;
    for (uint32_t s = 0; s < nslots && s < (uint32_t)kSlots; ++s) {
      uint2 e = st.slots[(size_t)s * st.n + inst];
      if ((e.y & 0xFFFF) != ord) continue;
      if (peek ? ((e.y >> 24) & 1u) != 0u : (((e.y >> 24) & 3u) == 1u || (again && ((e.y >> 24) & 3u) == 3u))) {
        if (!peek) {
          e.y |= 2u << 24;
          st.slots[(size_t)s * st.n + inst] = e;
          marked = true;
        }
        o.a = make_uint4(e.x, h.x, h.y, e.y);  // (e.y != 0: its state; a multi-instance loop counter)
      }
    }
    // the activation (DbJobState.activate stores the deadline and worker): an entry of the instance's
    // activation table -- the one already naming this ordinal (a stale one of an earlier instance in
    // the slot), or one whose job is gone
    if (marked && st.act) {
      int pick = -1;
      for (uint32_t k = 0; k < (uint32_t)kSlots && pick < 0; ++k)
        if ((st.act[(size_t)k * st.n + inst].x & 0xFFFF) == ord) pick = (int)k;
      for (uint32_t k = 0; k < (uint32_t)kSlots && pick < 0; ++k) {
        const uint4 a = st.act[(size_t)k * st.n + inst];
        bool live = false;
        for (uint32_t s = 0; s < nslots && s < (uint32_t)kSlots; ++s) {
          const uint2 e = st.slots[(size_t)s * st.n + inst];
          live |= (a.x >> 31) && (e.y & 0xFFFF) == (a.x & 0xFFFF) && ((e.y >> 24) & 3u) == 3u;
        }
        if (!live) pick = (int)k;
      }
      if (pick >= 0)
        st.act[(size_t)pick * st.n + inst] = make_uint4(ord | (1u << 31), worker, (uint32_t)deadline, (uint32_t)(deadline >> 32));
    }
    for (uint32_t v = 0; v < nvars && v < (uint32_t)kVars; ++v) {
      o.meta[v] = st.var_meta[(size_t)v * st.n + inst];
      o.val[v] = st.var_val[(size_t)v * st.n + inst];
    }
    for (uint32_t s = 0; s < (uint32_t)kSlots; ++s)
      o.slots[s] = s < nslots ? st.slots[(size_t)s * st.n + inst] : make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
  }
  out[i] = o;
}

hipError_t launch_activate_jobs(const DevState& st, const uint2* jobs, uint32_t n, void* out, uint32_t worker,
                                long long deadline, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_activate_jobs, dim3((n + 255) / 256), dim3(256), 0, s, st, jobs, n,
                            static_cast<ActivatedOut*>(out), worker, (unsigned long long)deadline);
  return hipGetLastError();
}
size_t activated_out_bytes() { return sizeof(ActivatedOut); }

// The engine's due-date checker over the device's timers (zbhip_due_timers): DueDateTimerChecker ->
// DbTimerInstanceState.processTimersWithDueDateBefore (:87-116) visits TIMER_DUE_DATES while dueDate <=
// now and returns the first later dueDate.  One coalesced pass over the instances' timer rows (16 B
// each): due rows are compacted into `out` (one atomic per wave: ballot + prefix count; the host sorts
// them into (dueDate, elementInstanceKey, key) order), later dueDates reduce to one atomic min per wave.
__global__ __launch_bounds__(256) void k_due_timers(const uint4* tmr, const uint4* hdr, uint32_t n, long long now,
                                                   DueTimer* out, uint32_t* count, unsigned long long* next_due) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  bool due = false;
  unsigned long long later = ~0ull;
  uint4 t = make_uint4(0, 0, 0, 0);
  uint32_t proc = 0;
  if (i < n) {
    t = tmr[i];
    if (t.y >> 31) {
      const uint4 hd = hdr[i];
      if ((hd.y >> 24) & 1u) {  // a live instance's live timer
        const long long d = (long long)(((unsigned long long)t.w << 32) | t.z);
        due = d <= now;
        if (!due) later = (unsigned long long)d;
        proc = hd.x & 0xFFFF;
      }
    }
  }
  const uint64_t m = __ballot(due);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == 0 && m) base = atomicAdd(count, (uint32_t)__popcll(m));
  base = __shfl(base, 0);
  if (due) out[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = DueTimer{t, i, proc};
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long u = __shfl_xor(later, o);
    later = u < later ? u : later;
  }
  if (lane == 0 && later != ~0ull) atomicMin(next_due, later);
}

hipError_t launch_due_timers(const DevState& st, long long now, DueTimer* out, uint32_t* count,
                             unsigned long long* next_due, hipStream_t s) {
  if (st.tmr && st.n)
    hipLaunchKernelGGL(k_due_timers, dim3((st.n + 255) / 256), dim3(256), 0, s, st.tmr, st.hdr, st.n, now, out, count,
                       next_due);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// launch wrappers (host)
// ---------------------------------------------------------------------------------------------
template <class K>
static size_t lds_bytes(uint32_t prog_words) {
  if (K::REG)  // program | stage | flush prefix array + owner map
    return (size_t)((prog_words + 3) & ~3u) * 4 + (size_t)K::R * K::B * sizeof(uint2) + (size_t)K::B * 4 +
           (((size_t)K::B * K::R + 3) & ~(size_t)3);
  return (size_t)((prog_words + 3) & ~3u) * 4 + (size_t)K::T * K::B * sizeof(uint2) +
         (size_t)K::R * K::B * sizeof(uint2) + (size_t)K::Q * K::B * sizeof(uint32_t) + tpl_lds_bytes<K>();
}

static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// Grid of a launch: as many workgroups as are resident at once (occupancy x CUs), each looping
// over an equal share of the chunks; ZBHIP_CHUNKS_PER_WG=k instead gives every workgroup k chunks.
constexpr size_t kLdsPerCu = 160 * 1024;
constexpr size_t kLdsGranule = 1280;  // 160 KB / 128

template <class K>
static uint32_t resident_for(size_t lds) {
  static int cus = 0;
  static size_t cached_lds = ~(size_t)0;
  static int per_cu = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  if (lds != cached_lds) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_step<K>, K::B, lds) != hipSuccess || per_cu <= 0) per_cu = 1;
    // the occupancy query counts LDS in bytes; the CU allocates it in kLdsGranule blocks, so near
    // the limit it promises one workgroup more than fits (measured: 13 600 B x 12 and
    // 27 008 B x 6 workgroups ran as 11 and 5) and the grid's last workgroups ran after the rest
    const size_t granted = (lds + kLdsGranule - 1) / kLdsGranule * kLdsGranule;
    if (granted) per_cu = std::max(1, std::min(per_cu, (int)(kLdsPerCu / granted)));
    const int forced = env_int("ZBHIP_WG_PER_CU", 0);
    if (forced > 0) per_cu = forced;
    if (env_int("ZBHIP_DEBUG", 0)) fprintf(stderr, "[zbhip] k_step B=%d R=%d lds=%zu per_cu=%d\n", K::B, K::R, lds, per_cu);
    cached_lds = lds;
  }
  return (uint32_t)(per_cu * cus);
}

template <class K>
static uint32_t grid_for(uint32_t n_chunks, size_t lds) {
  const int fixed = env_int("ZBHIP_CHUNKS_PER_WG", 0);
  if (fixed > 0) return (n_chunks + fixed - 1) / fixed;
  const uint32_t resident = resident_for<K>(lds);
  if (n_chunks <= resident) return n_chunks;
  const uint32_t per_wg = (n_chunks + resident - 1) / resident;
  return (n_chunks + per_wg - 1) / per_wg;
}

template <class K>
static hipError_t launch_k(const StepParams& P, hipStream_t s) {
  const uint32_t n_chunks = (P.n_launch + K::B - 1) / K::B;
  const size_t lds = lds_bytes<K>(P.prog_words);
  hipLaunchKernelGGL(k_step<K>, dim3(grid_for<K>(n_chunks, lds)), dim3(K::B), lds, s, P);
  return hipGetLastError();
}

// the largest grid of a k_step launch (its resident workgroups; ZBHIP_CHUNKS_PER_WG aside)
uint32_t step_resident(int variant, uint32_t prog_words) {
  return variant == 3   ? resident_for<KLinear>(lds_bytes<KLinear>(prog_words))
         : variant == 2 ? resident_for<KMsg>(lds_bytes<KMsg>(prog_words))
         : variant == 4 ? resident_for<KScope>(lds_bytes<KScope>(prog_words))
         : variant == 5 ? resident_for<KScopeIO>(lds_bytes<KScopeIO>(prog_words))
         : variant      ? resident_for<KGeneric>(lds_bytes<KGeneric>(prog_words))
                        : resident_for<KSimple>(lds_bytes<KSimple>(prog_words));
}
uint32_t step_queue(int variant) {
  return variant == 3 ? KLinear::Q : variant == 2 ? KMsg::Q : variant ? KGeneric::Q : KSimple::Q;
}

// variants: 0 KSimple, 1 KGeneric, 2 KMsg, 3 KLinear, 4 KScope, 5 KScopeIO (KGeneric's B, T, Q, R)
static_assert(KScope::B == KGeneric::B && KScope::Q == KGeneric::Q && KScope::R == KGeneric::R, "KScope shapes");
uint32_t step_block(int variant) {
  return variant == 3 ? KLinear::B : variant == 2 ? KMsg::B : variant ? KGeneric::B : KSimple::B;
}

size_t step_lds_bytes(int variant, uint32_t prog_words) {
  return variant == 3   ? lds_bytes<KLinear>(prog_words)
         : variant == 2 ? lds_bytes<KMsg>(prog_words)
         : variant == 4 ? lds_bytes<KScope>(prog_words)
         : variant == 5 ? lds_bytes<KScopeIO>(prog_words)
         : variant      ? lds_bytes<KGeneric>(prog_words)
                        : lds_bytes<KSimple>(prog_words);
}

hipError_t launch_keyscan(const uint2* cmd_hdr, const uint4* cmd_hdr2, const uint4* cmds, uint32_t n,
                          unsigned long long* block_sum, unsigned long long* base, unsigned long long* counter,
                          zbhip_xpart_cmd* xout, uint32_t xcap, const DevState& st, long long pbits, hipStream_t s) {
  if (n == 0) return hipSuccess;
  KeyScanParams K{cmd_hdr, cmd_hdr2, cmds, n, block_sum, base, counter, xout, xcap, st.pi_key, st.n,
                  st.sub_a, st.sub_b, st.sub_k, st.n_slots, pbits};
  const uint32_t nb = (n + kScanB - 1) / kScanB;
  hipLaunchKernelGGL(k_key_block_sums, dim3(nb), dim3(kScanB), 0, s, K);
  hipLaunchKernelGGL(k_key_scan_sums, dim3(1), dim3(1024), 0, s, K, nb);
  hipLaunchKernelGGL(k_key_apply, dim3(nb), dim3(kScanB), 0, s, K);
  hipLaunchKernelGGL(k_key_patch, dim3((n + 255) / 256), dim3(256), 0, s, K);
  return hipGetLastError();
}

hipError_t launch_subject_check(const uint4* cmds, uint32_t n, uint32_t n_inst, uint32_t n_slots, uint32_t* seen,
                                uint32_t stamp, uint32_t* gw, hipStream_t s) {
  const uint32_t per_block = 256 * kCheckPerThread;
  if (n) hipLaunchKernelGGL(k_subject_check, dim3((n + per_block - 1) / per_block), dim3(256), 0, s, cmds, n, n_inst, n_slots,
                            seen, stamp, gw);
  return hipGetLastError();
}

hipError_t launch_check_publish(const uint32_t* gw, uint32_t stamp, uint32_t* host, hipStream_t s) {
  hipLaunchKernelGGL(k_check_publish, dim3(1), dim3(64), 0, s, gw, stamp, host);
  return hipGetLastError();
}

hipError_t launch_xpart_window(const zbhip_xpart_cmd* xp, uint32_t n, uint4* cmds, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_xpart_window, dim3((n + 255) / 256), dim3(256), 0, s, xp, n, cmds);
  return hipGetLastError();
}

hipError_t launch_xgather(const XGather& A, uint32_t max_count, hipStream_t s) {
  if (A.P == 0 || max_count == 0) return hipSuccess;
  const uint32_t gx = std::min<uint32_t>(1024, (3 * max_count + 255) / 256);
  hipLaunchKernelGGL(k_xgather, dim3(gx, A.P * A.P), dim3(256), 0, s, A);
  return hipGetLastError();
}

hipError_t launch_bucket(const uint2* cmd_hdr, const uint4* cmd_hdr2, const zbhip_xpart_cmd* xout, uint32_t xcap,
                         uint32_t n, uint32_t parts, uint32_t* blk_cnt, uint32_t* counts, zbhip_xpart_cmd* out,
                         hipStream_t s) {
  BucketParams Q{cmd_hdr, cmd_hdr2, xout, xcap, n, parts, blk_cnt, counts, out};
  const uint32_t nb = (n + kBucketB - 1) / kBucketB;
  const uint32_t ng = (nb + kScanG - 1) / kScanG;
  uint32_t* grp = blk_cnt + (size_t)std::max(nb, 1u) * parts;  // [ng][parts] after the block counts
  if (nb) hipLaunchKernelGGL(k_bucket_count, dim3(nb), dim3(kBucketB), 0, s, Q);
  if (nb) hipLaunchKernelGGL(k_bucket_scan_groups, dim3(ng), dim3(kScanG), 0, s, Q, nb, grp);
  hipLaunchKernelGGL(k_bucket_scan_bases, dim3(1), dim3(64), 0, s, Q, ng, grp);
  if (nb) hipLaunchKernelGGL(k_bucket_scatter, dim3(nb), dim3(kBucketB), 0, s, Q, grp);
  return hipGetLastError();
}

void dump_stamps() {
#ifdef ZB_STAMPS
  unsigned long long h[8] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_stamps), sizeof h) != hipSuccess) return;
  const unsigned long long z8[8] = {};
  const double waves = 1.0;  // sums are per wave (lane 0)
  unsigned long long q[8] = {};
  if (hipMemcpyFromSymbol(q, HIP_SYMBOL(g_stamps_run), sizeof q) == hipSuccess && h[4])
    fprintf(stderr, "[stamps] run_command per chunk: loads %.0f initial %.0f fifo-pi %.0f fifo-local %.0f commit %.0f | entries/lane0 %.2f\n",
            q[0] / (double)h[4], q[1] / (double)h[4], q[2] / (double)h[4], q[3] / (double)h[4], q[4] / (double)h[4],
            q[5] / (double)h[4]);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps_run), z8, sizeof z8);
  fprintf(stderr, "[stamps] chunks %llu | per chunk cycles: top-wait %.0f run %.0f scan+barrier %.0f flush %.0f | prologue sum %.3g\n",
          h[4], h[0] / (double)h[4] * waves, h[1] / (double)h[4], h[2] / (double)h[4], h[3] / (double)h[4], (double)h[5]);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z8, sizeof z8);
#endif
}

hipError_t launch_step(int variant, const StepParams& P, hipStream_t s) {
  if (P.n_launch == 0) return hipSuccess;
  switch (variant) {
    case 3: return launch_k<KLinear>(P, s);
    case 2: return launch_k<KMsg>(P, s);
    case 1: return launch_k<KGeneric>(P, s);
    case 4: return launch_k<KScope>(P, s);
    case 5: return launch_k<KScopeIO>(P, s);
    default: return launch_k<KSimple>(P, s);
  }
}

uint32_t step_rows(int variant) {
  return variant == 3 ? KLinear::R : variant == 2 ? KMsg::R : variant ? KGeneric::R : KSimple::R;
}

hipError_t launch_gather(const uint2* regions, const uint32_t* tot, const uint16_t* lanes, uint32_t n_regions,
                         unsigned long long* off, size_t region_stride, uint32_t B, uint32_t R, uint2* out,
                         unsigned long long* total, hipStream_t s) {
  if (B > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_scan_regions, dim3(1), dim3(1024), 0, s, tot, lanes, B, n_regions, off, total);
  if (n_regions)
    hipLaunchKernelGGL(k_gather, dim3(n_regions), dim3(256), 0, s, regions, tot, lanes, off, region_stride, B, R,
                       out);
  return hipGetLastError();
}

}  // namespace zb
