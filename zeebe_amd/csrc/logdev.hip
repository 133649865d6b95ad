// Log bytes on the device: the window's compact records -> the bytes the reference's log stream
// holds for them, written into HBM.  The same format as the host serialiser (logwriter.cpp:
// SequencedBatchSerializer.java:33-67, LogAppendEntrySerializer.java:40-111, LogEntryDescriptor,
// RecordMetadata + protocol.xml:137-152, MsgPackWriter.java:62-316, the record values of
// ProcessInstanceRecord / JobRecord / VariableRecord / ProcessEventRecord /
// ProcessInstanceCreationRecord) for configs 1-4; the host builds the constant byte runs at deploy
// time (zb::log_device_tables) and the per-command table of the window (key base, positions).
//
// Keys.  A record names keys by (instance, ordinal).  Ordinals of the command's own batch resolve
// from its key base; older ordinals from an earlier command of the same instance in this window
// (`prev` chain) or from the instance's key ring in HBM: the last kRing ordinals of every instance,
// each entry tagged with its ordinal (ordinal << 48 | key counter), filled after each window, plus
// the process-instance key (ordinal 0).  An ordinal the ring no longer holds flags the window, and
// the host serialiser takes it instead.
//
// Entry templates.  Most entries of the path have a fixed layout once their keys are fixed-width
// (PROCESS_INSTANCE events and commands, JOB:CREATED, document-less JOB:COMPLETED / PROCESS_EVENT /
// PROCESS_INSTANCE_CREATION:CREATED; keys >= 2^32 always take msgpack's 9-byte form): the host
// serialises each (process, element, kind) once with sentinel keys (logwriter.cpp
// log_device_templates), and the device copies the template and patches the header's position,
// sourcePosition, key and timestamp and the value's big-endian processInstanceKey / scope key.
//
// Passes: k_log_sizes (one thread per command: entry sizes) -> u64 scan over commands -> k_log_write
// (one lane per command resolves its next record; a templated entry is then copied by half a wave,
// 16 B per lane, two entries per store instruction, so the stores cover whole consecutive lines and
// no lane composes bytes; other entries are composed by their lane directly) -> k_ring_fill
// (CREATEs reset their instance's ring, then every command adds its ordinals).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "zb_internal.h"

namespace zb {

constexpr uint32_t kRing = 16;

// global byte runs of the device tables (logwriter.cpp log_device_tables builds them in this order)
enum LogRun : uint32_t {
  G_AUTH, G_TENANT, G_FLOWSCOPE, G_EMPTY_BIN, G_JREJ_HEAD, G_JREJ_TAIL, G_VAR_A, G_VAR_VALUE, G_VAR_SCOPE,
  G_K_PIK, G_K_DEF, G_K_BPMN, G_PE_A, G_PE_TARGET, G_K_VARS, G_PIC_A, G_K_VERSION, G_PIC_TAIL,
  G_RS_PGW_A, G_RS_PGW_B, G_RS_FSNF_A, G_RS_NF_B, G_RS_FSST_A, G_RS_Q, G_RS_EINF_A, G_RS_EIST_A, G_RS_JOB_A,
  G_RS_JOB_B, G_RS_TNF_A, G_RS_TNF_B, G_RS_TNA_A, G_RS_TNA_B, G_TIMER_A, G_TIMER_DUE, G_TIMER_REPS, G_JACT_A,
  G_JACT_W, G_ST0,
  G_COUNT = G_ST0 + 16
};
// element runs (proc block word 6 + 16 e); E_DUR is the timer duration in ms (.x), not a byte run
// (E_JOB_REST: E_JOB_HEAD after its deadline and worker entries -- an ACTIVATED job's head is composed)
enum ElRun : uint32_t { E_PI_HEAD, E_PI_TAIL, E_JOB_HEAD, E_JOB_MID, E_JOB_TAIL, E_ID_STR, E_ID_RAW, E_JOB_REST, E_DUR,
                        E_COUNT };

struct LogParams {
  const uint2* rows;            // gathered compact rows (launch order)
  const LogCmd* cmds;           // [n]
  uint32_t n;
  const uint8_t* arena;         // byte runs, each 4-aligned
  const uint32_t* idx;          // run table (see log_device_tables)
  uint32_t arena_words, idx_words;  // sizes (the kernels stage both in LDS when they fit)
  const zbhip_doc_entry* docs;  // the window's document entries
  uint32_t n_docs;
  const uint16_t* inst_proc;    // [n_inst] process of each instance slot (NONE: free)
  unsigned long long* ring;     // [kRing][n_inst]
  unsigned long long* kpi;      // [n_inst] bit 63 | key counter of ordinal 0
  uint32_t n_inst;
  long long pbits;              // partition_id << 51
  long long first_position, timestamp;
  int32_t broker[3];
  unsigned long long* bytes;    // [n] entry bytes of each command, then (scanned) byte offsets
  uint64_t* out;                // log bytes (8-byte aligned entries)
  uint32_t* flag;               // bit 0: an unresolved key / unsupported value (host serialiser instead)
  long long now_ms;             // the run's clock: TIMER:CREATED dueDate = clock + duration
  const long long* cmd_due;     // [n] dueDate of the timer each batch canceled
  const uint8_t* tpl;           // entry templates (logwriter.cpp log_device_templates)
  const uint4* tpl_desc;
  const uint32_t* tpl_idx;
  uint32_t* rinfo;              // [rows] per record: template id << 16 | entry bytes, or kSlow | bytes
  unsigned long long out_cap;   // bytes at `out` (0: unchecked)
  LogKeys* wkeys;               // [n] per command: the older keys its records name (k_log_sizes)
  uint32_t tpl_lds;             // bytes of the templates + their descriptors (k_log_stream stages both)
  const uint4* cmd_act;         // [n] the ACTIVATED job a batch completed / canceled (StepParams.cmd_act)
  const uint8_t* strs;          // the value dictionary's bytes (workers of activated jobs) ...
  const unsigned long long* str_off;  // ... string i at [str_off[i], str_off[i + 1])
  uint32_t n_strs;
};
constexpr uint32_t kSlow = 1u << 31;

__device__ __forceinline__ uint2 run(const LogParams& L, uint32_t i) {
  return make_uint2(L.idx[2 * i], L.idx[2 * i + 1]);
}
__device__ __forceinline__ uint32_t proc_block(const LogParams& L, uint32_t p) {
  const uint32_t p0 = 2 * G_COUNT + 1 + 2 * L.idx[2 * G_COUNT];
  return p < L.idx[p0] ? L.idx[p0 + 1 + p] : 0u;
}
__device__ __forceinline__ uint2 el_run(const LogParams& L, uint32_t pb, uint32_t e, uint32_t k) {
  const uint32_t w = pb + 6 + E_COUNT * 2 * e + 2 * k;
  return make_uint2(L.idx[w], L.idx[w + 1]);
}
__device__ __forceinline__ uint2 name_run(const LogParams& L, uint32_t id) {
  const uint32_t nn = L.idx[2 * G_COUNT];
  return id < nn ? make_uint2(L.idx[2 * G_COUNT + 1 + 2 * id], L.idx[2 * G_COUNT + 2 + 2 * id]) : make_uint2(0, 0);
}

// ---- byte sinks: a counter, or 8-byte little-endian stores ---------------------------------
struct Count {
  unsigned long long n = 0;
  __device__ __forceinline__ void put(uint32_t, uint32_t k) { n += k; }
  __device__ __forceinline__ void b(uint32_t) { ++n; }
  __device__ __forceinline__ void bytes(const LogParams&, uint2 r) { n += r.y; }
  __device__ __forceinline__ void zeros(uint32_t k) { n += k; }
  __device__ __forceinline__ void raw(const uint8_t*, uint32_t k) { n += k; }
};
// appends up to four bytes at a time into a 128-bit accumulator, stored with one 16-byte store
// when it fills (a lane writes its own command's bytes: every store is a separate transaction, so
// fewer, wider stores); a command's bytes start 8-byte aligned, so the first store may be 8 bytes
struct Write {
  uint64_t* p;
  uint64_t a0 = 0, a1 = 0;  // pending bytes 0..7 and 8..15
  uint32_t nb = 0;
  uint32_t cap = 16;        // 8 until p is 16-byte aligned
  __device__ __forceinline__ void start(uint64_t* q) {
    p = q;
    cap = (reinterpret_cast<uintptr_t>(q) & 15) ? 8u : 16u;
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t k) {  // the k (1..4) low bytes of v
    const uint64_t x = k == 4 ? (uint64_t)v : (uint64_t)(v & ((1u << (8 * k)) - 1));
    if (nb < 8) {
      a0 |= x << (8 * nb);
      if (nb + k > 8) a1 |= x >> (8 * (8 - nb));
    } else {
      a1 |= x << (8 * (nb - 8));
    }
    nb += k;
    if (nb < cap) return;
    if (cap == 16) {
      *reinterpret_cast<ulonglong2*>(p) = make_ulonglong2(a0, a1);
      p += 2;
      nb -= 16;
      a0 = nb ? x >> (8 * (k - nb)) : 0;
      a1 = 0;
    } else {
      *p++ = a0;
      nb -= 8;
      a0 = a1;
      a1 = 0;
      cap = 16;
    }
  }
  __device__ __forceinline__ void finish() {  // entries end 8-byte aligned: at most one word pending
    if (nb) *p++ = a0;
    nb = 0;
    a0 = a1 = 0;
  }
  __device__ __forceinline__ void b(uint32_t x) { put(x, 1); }
  __device__ __forceinline__ void bytes(const LogParams& L, uint2 r) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(L.arena + r.x);
    for (uint32_t i = 0; i < r.y; i += 4) put(w[i >> 2], r.y - i < 4 ? r.y - i : 4);
  }
  __device__ __forceinline__ void zeros(uint32_t k) {
    for (uint32_t i = 0; i < k; i += 4) put(0, k - i < 4 ? k - i : 4);
  }
  __device__ __forceinline__ void raw(const uint8_t* p, uint32_t k) {  // (unaligned bytes)
    for (uint32_t i = 0; i < k; ++i) put(p[i], 1);
  }
};

template <class S>
__device__ __forceinline__ void le(S& s, unsigned long long v, int n) {
  if (n == 8) { s.put((uint32_t)v, 4); s.put((uint32_t)(v >> 32), 4); }
  else s.put((uint32_t)v, (uint32_t)n);
}
template <class S>
__device__ __forceinline__ void be(S& s, unsigned long long v, int n) {
  if (n == 8) { s.put(__builtin_bswap32((uint32_t)(v >> 32)), 4); s.put(__builtin_bswap32((uint32_t)v), 4); }
  else if (n == 4) s.put(__builtin_bswap32((uint32_t)v), 4);
  else if (n == 2) s.put(((uint32_t)(v >> 8) & 0xFF) | (((uint32_t)v & 0xFF) << 8), 2);
  else s.put((uint32_t)v, 1);
}

// MsgPackWriter.writeInteger (:154-212): the smallest encoding
template <class S>
__device__ __forceinline__ void mp_int(S& s, long long v) {
  if (v < -(1LL << 5)) {
    if (v < -(1LL << 15)) {
      if (v < -(1LL << 31)) { s.b(0xd3); be(s, (unsigned long long)v, 8); }
      else { s.b(0xd2); be(s, (unsigned long long)v, 4); }
    } else if (v < -(1LL << 7)) { s.b(0xd1); be(s, (unsigned long long)v, 2); }
    else { s.b(0xd0); s.b((uint32_t)v); }
  } else if (v < (1LL << 7)) {
    s.b((uint32_t)v);
  } else if (v < (1LL << 16)) {
    if (v < (1LL << 8)) { s.b(0xcc); s.b((uint32_t)v); }
    else { s.b(0xcd); be(s, (unsigned long long)v, 2); }
  } else if (v < (1LL << 32)) { s.b(0xce); be(s, (unsigned long long)v, 4); }
  else { s.b(0xcf); be(s, (unsigned long long)v, 8); }
}
__device__ __forceinline__ uint32_t mp_int_len(long long v) {
  if (v < -(1LL << 5)) return v < -(1LL << 31) ? 9 : v < -(1LL << 15) ? 5 : v < -(1LL << 7) ? 3 : 2;
  if (v < (1LL << 7)) return 1;
  return v < (1LL << 8) ? 2 : v < (1LL << 16) ? 3 : v < (1LL << 32) ? 5 : 9;
}

// decimal text of a signed 64-bit integer (the "%lld" of the reason texts)
template <class S>
__device__ __forceinline__ void dec(S& s, long long v) {
  char d[20];
  int n = 0;
  unsigned long long u = v < 0 ? 0ull - (unsigned long long)v : (unsigned long long)v;
  do { d[n++] = (char)('0' + u % 10); u /= 10; } while (u);
  if (v < 0) s.b('-');
  while (n) s.b((uint32_t)d[--n]);
}

// ---- one record -------------------------------------------------------------------------------
struct Rec {
  long long key, scope, pik;
  long long due;            // TIMER: dueDate
  int reps;                 // TIMER: repetitions (-1 infinite)
  uint32_t proc, elem;      // NONE when not applicable
  uint8_t rt, vt, intent, rej_type, reason, reason_arg, skip;
  bool act;                 // JOB: an ACTIVATED job's record (deadline, worker below)
  long long deadline;
  uint32_t worker;
};

// key of ordinal `ord` of instance `inst` as seen by command c (see the header comment)
__device__ __forceinline__ bool key_of(const LogParams& L, uint32_t c, uint32_t inst, uint32_t ord, long long& key) {
  if (ord == NONE) { key = -1; return true; }
  for (int hop = 0; hop < 64 && c != 0xFFFFFFFFu; ++hop) {
    const LogCmd& m = L.cmds[c];
    if (ord >= m.first_ord && m.nkeys) {  // this batch (ordinals grow within an instance generation)
      key = L.pbits + (long long)(m.key0 + (uint16_t)(ord - m.first_ord));
      return true;
    }
    if (m.first_ord == 0) break;  // a CREATE: nothing older in this generation
    c = m.prev;
  }
  if (inst >= L.n_inst) return false;
  if (ord == 0) {
    const unsigned long long k = L.kpi[inst];
    if (!(k >> 63)) return false;
    key = L.pbits + (long long)(k & ((1ull << 63) - 1));
    return true;
  }
  const unsigned long long e = L.ring[(size_t)(ord % kRing) * L.n_inst + inst];
  if ((e >> 48) != ord) return false;
  key = L.pbits + (long long)(e & ((1ull << 48) - 1));
  return true;
}

// The same for the lane's own command m (in registers): its batch's keys need no memory, and the
// older keys it names (the process instance, the element instances it continues) are looked up once
// per command and kept -- every record of a batch repeats them, and re-reading them per record missed
// L2 under the write stream (PMC: ~200 B fetched per written entry).
struct KeyCache {
  uint32_t o0 = NONE, o1 = NONE, o2 = NONE;
  long long k0 = -1, k1 = -1, k2 = -1;
  bool has_pi = false;  // the process instance's key (ordinal 0), kept apart: every record names it
  long long kpi = -1;
};
__device__ __forceinline__ bool key_of_lane(const LogParams& L, const LogCmd& m, uint32_t ord, long long& key,
                                            KeyCache& kc) {
  if (ord == NONE) { key = -1; return true; }
  if (ord >= m.first_ord && m.nkeys) {
    key = L.pbits + (long long)(m.key0 + (uint16_t)(ord - m.first_ord));
    return true;
  }
  if (ord == 0 && kc.has_pi) { key = kc.kpi; return true; }
  if (ord == kc.o0) { key = kc.k0; return true; }
  if (ord == kc.o1) { key = kc.k1; return true; }
  if (ord == kc.o2) { key = kc.k2; return true; }
  if (!key_of(L, m.first_ord == 0 ? 0xFFFFFFFFu : m.prev, m.instance, ord, key)) return false;
  if (ord == 0) {
    kc.has_pi = true;
    kc.kpi = key;
    return true;
  }
  kc.o2 = kc.o1;
  kc.k2 = kc.k1;
  kc.o1 = kc.o0;
  kc.k1 = kc.k0;
  kc.o0 = ord;
  kc.k0 = key;
  return true;
}

__device__ __forceinline__ bool decode(const LogParams& L, uint32_t c, const LogCmd& m, uint2 w, Rec& r, KeyCache& kc) {
  const uint32_t key_ord = w.x & 0xFFFF, aux_ord = w.x >> 16, elem = w.y & 0xFFFF;
  const uint32_t code = (w.y >> 16) & 0xFF, fl = w.y >> 24;
  const bool rej = code & kRejectBit;
  const uint32_t c6 = code & 0x3F;
  const uint32_t inst = m.instance;
  r.proc = inst < L.n_inst ? L.inst_proc[inst] : NONE;
  r.elem = elem;
  if (!key_of_lane(L, m, key_ord, r.key, kc) || !key_of_lane(L, m, aux_ord, r.scope, kc) ||
      !key_of_lane(L, m, 0, r.pik, kc))
    return false;
  r.rej_type = ZBHIP_REJ_NONE;
  r.reason = r.reason_arg = 0;
  r.skip = 0;
  r.act = false;
  r.deadline = -1;
  r.worker = ZBHIP_NO_STRING;
  if (c6 >= 1 && c6 <= 10) {
    r.vt = ZBHIP_VT_PROCESS_INSTANCE;
    r.intent = (uint8_t)c6;
    r.rt = rej ? ZBHIP_RT_REJECTION : (c6 >= 8 ? ZBHIP_RT_COMMAND : ZBHIP_RT_EVENT);
    r.skip = !rej && c6 >= 8 && !(fl & F_UNPROCESSED) ? 1 : 0;  // a follow-up command processed in its batch
  } else if (c6 == C_JOB_CREATED || c6 == C_JOB_COMPLETED || c6 == C_JOB_COMPLETE || c6 == C_JOB_CANCELED) {
    // an ACTIVATED job's record: the stored job's deadline and worker from the batch's activation
    // word (missing, or naming another job: the host serialiser)
    if (!rej && (fl & 1u) && (c6 == C_JOB_COMPLETED || c6 == C_JOB_CANCELED)) {
      const uint4 a = L.cmd_act ? L.cmd_act[c] : make_uint4(0, 0, 0, 0);
      if (!(a.x >> 31) || (a.x & 0xFFFF) != key_ord || (a.y != ZBHIP_NO_STRING && (a.y >= L.n_strs || !L.strs)))
        return false;
      r.act = true;
      r.deadline = (long long)(((unsigned long long)a.w << 32) | a.z);
      r.worker = a.y;
    }
    r.vt = ZBHIP_VT_JOB;
    r.intent = c6 == C_JOB_CREATED ? ZBHIP_JOB_CREATED : c6 == C_JOB_COMPLETED ? ZBHIP_JOB_COMPLETED
               : c6 == C_JOB_CANCELED ? ZBHIP_JOB_CANCELED : ZBHIP_JOB_COMPLETE;
    r.rt = rej ? ZBHIP_RT_REJECTION : ZBHIP_RT_EVENT;
  } else if (c6 == C_VAR_CREATED || c6 == C_VAR_UPDATED) {
    r.vt = ZBHIP_VT_VARIABLE;
    r.intent = c6 == C_VAR_CREATED ? ZBHIP_VAR_CREATED : ZBHIP_VAR_UPDATED;
    r.rt = ZBHIP_RT_EVENT;
  } else if (c6 == C_PE_TRIGGERING || c6 == C_PE_TRIGGERED) {
    r.vt = ZBHIP_VT_PROCESS_EVENT;
    r.intent = c6 == C_PE_TRIGGERING ? ZBHIP_PE_TRIGGERING : ZBHIP_PE_TRIGGERED;
    r.rt = ZBHIP_RT_EVENT;
  } else if (c6 == C_TIMER_CREATED || c6 == C_TIMER_NEXT || c6 == C_TIMER_TRIGGERED || c6 == C_TIMER_TRIGGER ||
             c6 == C_TIMER_CANCELED) {
    // TimerRecord (runtime.cpp expand_plain): CREATED from the clock, a cycle's next timer from the
    // TRIGGER command's dueDate, TRIGGERED / a rejected TRIGGER the command's, CANCELED the stored one
    r.vt = ZBHIP_VT_TIMER;
    r.intent = c6 == C_TIMER_CREATED || c6 == C_TIMER_NEXT ? ZBHIP_TIMER_CREATED
               : c6 == C_TIMER_TRIGGERED ? ZBHIP_TIMER_TRIGGERED : c6 == C_TIMER_CANCELED ? ZBHIP_TIMER_CANCELED
               : ZBHIP_TIMER_TRIGGER;
    r.rt = rej ? ZBHIP_RT_REJECTION : ZBHIP_RT_EVENT;
    const long long cmd = (long long)(((unsigned long long)m.pad << 32) | m.doc_begin);
    long long dur = 0;
    // (a timer created in this batch and canceled in it: the clock plus its duration, as CREATED --
    // cmd_due holds only the dueDate of a timer stored before the batch)
    const bool fresh = c6 == C_TIMER_CANCELED && m.nkeys && key_ord >= m.first_ord && key_ord < (uint32_t)m.first_ord + m.nkeys;
    bool next = c6 == C_TIMER_NEXT;
    if (c6 == C_TIMER_CREATED || c6 == C_TIMER_NEXT || fresh) {
      const uint32_t pb = r.proc != NONE ? proc_block(L, r.proc) : 0u;
      if (!pb || elem >= L.idx[pb + 5]) return false;
      const uint2 d = el_run(L, pb, elem, E_DUR);
      dur = (long long)d.x;
      // (a fresh cancel of an interrupting boundary cycle's next timer: only a TIMER:TRIGGER batch -- a
      // nonzero command dueDate -- reschedules one; due as its CREATED)
      if (fresh && d.y && cmd != 0) next = true;
    }
    r.due = next ? next_cycle_due(cmd, dur, L.now_ms) : c6 == C_TIMER_CREATED || fresh ? L.now_ms + dur
            : c6 == C_TIMER_CANCELED ? L.cmd_due[c] : cmd;
    r.reps = rej ? 1 : fl == 255 ? -1 : (int)fl;
  } else if (c6 == C_PIC_CREATED) {
    r.vt = ZBHIP_VT_PROCESS_INSTANCE_CREATION;
    r.intent = ZBHIP_PIC_CREATED;
    r.rt = ZBHIP_RT_EVENT;
  } else {
    return false;  // a message record or a corrupt row: the host serialiser
  }
  if (rej) {
    r.reason = fl & 0xF;
    r.reason_arg = fl >> 4;
    if (r.vt == ZBHIP_VT_JOB) {
      r.rej_type = ZBHIP_REJ_NOT_FOUND;
      r.proc = NONE;
      r.elem = NONE;
      r.scope = -1;
      r.pik = -1;
    } else if (r.vt == ZBHIP_VT_TIMER) {  // the TIMER:TRIGGER command's value
      r.rej_type = r.reason == ZBHIP_REASON_TIMER_NOT_FOUND ? ZBHIP_REJ_NOT_FOUND : ZBHIP_REJ_INVALID_STATE;
      r.proc = NONE;
      r.elem = NONE;
      r.scope = -1;
      r.pik = -1;
    } else {
      r.rej_type = ZBHIP_REJ_INVALID_STATE;
    }
  }
  return true;
}

// msgpack of one document value (logwriter.cpp doc_value); strings are not on the device
template <class S>
__device__ __forceinline__ bool doc_value(S& s, const zbhip_doc_entry& d) {
  switch (d.type) {
    case ZBHIP_DOC_NIL: s.b(0xc0); return true;
    case ZBHIP_DOC_BOOL: s.b(d.value ? 0xc3 : 0xc2); return true;
    case ZBHIP_DOC_INT: mp_int(s, d.value); return true;
    case ZBHIP_DOC_DEC: {
      const double v = (double)d.value / 1e6;
      s.b(0xcb);
      be(s, (unsigned long long)__double_as_longlong(v), 8);
      return true;
    }
    default: return false;
  }
}
__device__ __forceinline__ uint32_t doc_value_len(const zbhip_doc_entry& d) {
  return d.type == ZBHIP_DOC_INT ? mp_int_len(d.value) : d.type == ZBHIP_DOC_DEC ? 9u : 1u;
}
__device__ __forceinline__ bool doc_ok(const zbhip_doc_entry& d) {
  return d.type == ZBHIP_DOC_NIL || d.type == ZBHIP_DOC_BOOL || d.type == ZBHIP_DOC_INT || d.type == ZBHIP_DOC_DEC;
}

// mp_bin of the command's document (DocumentValue: empty -> EMPTY_DOCUMENT; else its map, entries in
// document order); false for a document the device does not write (a string or list value, more than
// ZBHIP_DOC_MAX_ENTRIES entries)
template <class S>
__device__ __forceinline__ bool src_doc_bin(S& s, const LogParams& L, const LogCmd& m) {
  if (m.doc_count == 0) { s.bytes(L, run(L, G_EMPTY_BIN)); return true; }
  if (m.doc_count > ZBHIP_DOC_MAX_ENTRIES) return false;
  uint32_t len = 1;  // fixmap header
  for (uint32_t i = 0; i < m.doc_count; ++i) {
    const zbhip_doc_entry d = L.docs[m.doc_begin + i];
    if (!doc_ok(d)) return false;
    len += name_run(L, d.name_id).y + doc_value_len(d);
  }
  if (len < 256) {  // MsgPackWriter.writeBinaryHeader: bin8 / bin16
    s.b(0xc4);
    s.b(len);
  } else {
    s.b(0xc5);
    be(s, len, 2);
  }
  s.b(0x80 | m.doc_count);
  for (uint32_t i = 0; i < m.doc_count; ++i) {
    const zbhip_doc_entry d = L.docs[m.doc_begin + i];
    s.bytes(L, name_run(L, d.name_id));
    doc_value(s, d);
  }
  return true;
}

template <class S>
__device__ __forceinline__ void reason_text(S& s, const LogParams& L, const Rec& r, uint32_t pb) {
  switch (r.reason) {
    case ZBHIP_REASON_PGW_NOT_ALL_TAKEN:
      s.bytes(L, run(L, G_RS_PGW_A));
      if (pb && r.elem != NONE) s.bytes(L, el_run(L, pb, r.elem, E_ID_RAW));
      s.bytes(L, run(L, G_RS_PGW_B));
      return;
    case ZBHIP_REASON_FS_NOT_FOUND:
      s.bytes(L, run(L, G_RS_FSNF_A)); dec(s, r.scope); s.bytes(L, run(L, G_RS_NF_B));
      return;
    case ZBHIP_REASON_FS_STATE:
      s.bytes(L, run(L, G_RS_FSST_A)); s.bytes(L, run(L, G_ST0 + (r.reason_arg & 15))); s.bytes(L, run(L, G_RS_Q));
      return;
    case ZBHIP_REASON_EI_NOT_FOUND:
      s.bytes(L, run(L, G_RS_EINF_A)); dec(s, r.key); s.bytes(L, run(L, G_RS_NF_B));
      return;
    case ZBHIP_REASON_EI_STATE:
      s.bytes(L, run(L, G_RS_EIST_A)); s.bytes(L, run(L, G_ST0 + (r.reason_arg & 15))); s.bytes(L, run(L, G_RS_Q));
      return;
    case ZBHIP_REASON_JOB_NOT_FOUND:
      s.bytes(L, run(L, G_RS_JOB_A)); dec(s, r.key); s.bytes(L, run(L, G_RS_JOB_B));
      return;
    case ZBHIP_REASON_TIMER_NOT_FOUND:
      s.bytes(L, run(L, G_RS_TNF_A)); dec(s, r.key); s.bytes(L, run(L, G_RS_TNF_B));
      return;
    case ZBHIP_REASON_TIMER_NOT_ACTIVE:
      s.bytes(L, run(L, G_RS_TNA_A)); dec(s, r.key); s.bytes(L, run(L, G_RS_TNA_B));
      return;
    default:
      return;
  }
}

// the record value (msgpack); false: outside what the device writes
template <class S>
__device__ __forceinline__ bool value(S& s, const LogParams& L, const LogCmd& m, const Rec& r, uint32_t pb) {
  const bool has_el = pb && r.elem != NONE && r.elem < L.idx[pb + 5];
  switch (r.vt) {
    case ZBHIP_VT_PROCESS_INSTANCE:
      if (!has_el) return false;
      s.bytes(L, el_run(L, pb, r.elem, E_PI_HEAD));
      mp_int(s, r.pik);
      s.bytes(L, run(L, G_FLOWSCOPE));
      mp_int(s, r.scope);
      s.bytes(L, el_run(L, pb, r.elem, E_PI_TAIL));
      return true;
    case ZBHIP_VT_JOB:
      if (r.rt == ZBHIP_RT_REJECTION) {
        s.bytes(L, run(L, G_JREJ_HEAD));
        if (!src_doc_bin(s, L, m)) return false;
        s.bytes(L, run(L, G_JREJ_TAIL));
        return true;
      }
      if (!has_el || el_run(L, pb, r.elem, E_JOB_HEAD).y == 0) return false;
      if (r.act) {  // the stored job of an ACTIVATED job: its deadline and worker
        s.bytes(L, run(L, G_JACT_A));
        mp_int(s, r.deadline);
        s.bytes(L, run(L, G_JACT_W));
        const unsigned long long b = r.worker == ZBHIP_NO_STRING ? 0 : L.str_off[r.worker];
        const uint32_t n = r.worker == ZBHIP_NO_STRING ? 0u : (uint32_t)(L.str_off[r.worker + 1] - b);
        if (n < 32) s.b(0xa0 | n);  // MsgPackWriter.writeStringHeader (:214-240)
        else if (n < 256) { s.b(0xd9); s.b(n); }
        else if (n < 65536) { s.b(0xda); be(s, n, 2); }
        else { s.b(0xdb); be(s, n, 4); }
        if (n) s.raw(L.strs + b, n);
        s.bytes(L, el_run(L, pb, r.elem, E_JOB_REST));
      } else {
        s.bytes(L, el_run(L, pb, r.elem, E_JOB_HEAD));
      }
      if (r.intent != ZBHIP_JOB_COMPLETED) s.bytes(L, run(L, G_EMPTY_BIN));
      else if (!src_doc_bin(s, L, m)) return false;
      s.bytes(L, el_run(L, pb, r.elem, E_JOB_MID));
      mp_int(s, r.pik);
      s.bytes(L, el_run(L, pb, r.elem, E_JOB_TAIL));
      mp_int(s, r.scope);
      s.bytes(L, run(L, G_TENANT));
      return true;
    case ZBHIP_VT_VARIABLE: {
      // the batch's source document entry of that name (VariableRecord.java:35-41; names are distinct)
      if (!pb || m.doc_count == 0 || m.doc_count > ZBHIP_DOC_MAX_ENTRIES) return false;
      uint32_t at = 0;
      while (at + 1 < m.doc_count && L.docs[m.doc_begin + at].name_id != r.elem) ++at;
      const zbhip_doc_entry d = L.docs[m.doc_begin + at];
      if (d.name_id != r.elem || !doc_ok(d)) return false;
      const uint2 nr = name_run(L, r.elem);
      s.bytes(L, run(L, G_VAR_A));
      s.bytes(L, nr);
      s.bytes(L, run(L, G_VAR_VALUE));
      s.b(0xc4);
      s.b(doc_value_len(d));
      doc_value(s, d);
      s.bytes(L, run(L, G_VAR_SCOPE));
      mp_int(s, r.scope);
      s.bytes(L, run(L, G_K_PIK));
      mp_int(s, r.pik);
      s.bytes(L, run(L, G_K_DEF));
      mp_int(s, (long long)(((unsigned long long)L.idx[pb + 3] << 32) | L.idx[pb + 2]));
      s.bytes(L, run(L, G_K_BPMN));
      s.bytes(L, make_uint2(L.idx[pb], L.idx[pb + 1]));
      s.bytes(L, run(L, G_TENANT));
      return true;
    }
    case ZBHIP_VT_PROCESS_EVENT:
      if (!has_el) return false;
      s.bytes(L, run(L, G_PE_A));
      mp_int(s, r.scope);
      s.bytes(L, run(L, G_PE_TARGET));
      s.bytes(L, el_run(L, pb, r.elem, E_ID_STR));
      s.bytes(L, run(L, G_K_VARS));
      if (r.intent == ZBHIP_PE_TRIGGERED) s.bytes(L, run(L, G_EMPTY_BIN));  // processEventTriggered: reset record
      else if (!src_doc_bin(s, L, m)) return false;
      s.bytes(L, run(L, G_K_DEF));
      mp_int(s, (long long)(((unsigned long long)L.idx[pb + 3] << 32) | L.idx[pb + 2]));
      s.bytes(L, run(L, G_K_PIK));
      mp_int(s, r.pik);
      s.bytes(L, run(L, G_TENANT));
      return true;
    case ZBHIP_VT_TIMER:  // TimerRecord.java:24-40
      if (r.rt != ZBHIP_RT_REJECTION && !has_el) return false;
      s.bytes(L, run(L, G_TIMER_A));
      mp_int(s, r.scope);
      s.bytes(L, run(L, G_K_PIK));
      mp_int(s, r.pik);
      s.bytes(L, run(L, G_TIMER_DUE));
      mp_int(s, r.due);
      s.bytes(L, run(L, G_PE_TARGET));
      if (has_el) s.bytes(L, el_run(L, pb, r.elem, E_ID_STR));
      else s.b(0xa0);  // ""
      s.bytes(L, run(L, G_TIMER_REPS));
      mp_int(s, r.reps);
      s.bytes(L, run(L, G_K_DEF));
      mp_int(s, has_el ? (long long)(((unsigned long long)L.idx[pb + 3] << 32) | L.idx[pb + 2]) : -1LL);
      s.bytes(L, run(L, G_TENANT));
      return true;
    case ZBHIP_VT_PROCESS_INSTANCE_CREATION:
      if (!pb) return false;
      s.bytes(L, run(L, G_PIC_A));
      s.bytes(L, make_uint2(L.idx[pb], L.idx[pb + 1]));
      s.bytes(L, run(L, G_K_DEF));
      mp_int(s, (long long)(((unsigned long long)L.idx[pb + 3] << 32) | L.idx[pb + 2]));
      s.bytes(L, run(L, G_K_PIK));
      mp_int(s, r.scope);
      s.bytes(L, run(L, G_K_VERSION));
      mp_int(s, (long long)(int32_t)L.idx[pb + 4]);
      s.bytes(L, run(L, G_K_VARS));
      if (!src_doc_bin(s, L, m)) return false;
      s.bytes(L, run(L, G_PIC_TAIL));
      s.bytes(L, run(L, G_TENANT));
      return true;
    default:
      return false;
  }
}

// one log entry: dispatcher frame + LogEntryDescriptor header + SBE RecordMetadata + value, 8-aligned
// (logwriter.cpp zbhip_serialize_log); `S` counts in the first pass and writes in the second.
template <class S>
__device__ __forceinline__ bool entry(S& s, const LogParams& L, const LogCmd& m, const Rec& r, long long pos) {
  const uint32_t pb = r.proc != NONE ? proc_block(L, r.proc) : 0u;
  Count vc, rc;
  if (!value(vc, L, m, r, pb)) return false;
  const bool rej = r.rt == ZBHIP_RT_REJECTION;
  if (rej) reason_text(rc, L, r, pb);
  const uint2 auth = run(L, G_AUTH);  // le32 length + AuthInfo msgpack
  const uint32_t md = 8 + 32 + 4 + (uint32_t)rc.n + auth.y;
  const uint32_t framed = 12 + 40 + md + (uint32_t)vc.n;
  const uint32_t aligned = (framed + 7) & ~7u;
  le(s, framed, 4);
  s.zeros(8);
  s.b(0); s.b(0); s.b(r.skip); s.b(0);
  le(s, (unsigned long long)pos, 8);
  le(s, (unsigned long long)m.src_pos, 8);
  le(s, (unsigned long long)r.key, 8);
  le(s, (unsigned long long)L.timestamp, 8);
  le(s, md, 2);
  s.zeros(2);
  // RecordMetadata: messageHeader (blockLength 32, templateId 200, schemaId 0, version 4) + block
  le(s, 32, 2); le(s, 200, 2); le(s, 0, 2); le(s, 4, 2);
  s.b(r.rt);
  le(s, 0x80000000u, 4);          // requestStreamId: null
  le(s, ~0ull, 8);                // requestId: null
  le(s, 4, 2);                    // protocolVersion
  s.b(r.vt);
  s.b(r.intent);
  le(s, (uint32_t)L.broker[0], 4); le(s, (uint32_t)L.broker[1], 4); le(s, (uint32_t)L.broker[2], 4);
  le(s, 1, 2);                    // recordVersion
  s.b(rej ? r.rej_type : 255);
  le(s, rc.n, 4);
  if (rej) reason_text(s, L, r, pb);
  s.bytes(L, auth);
  value(s, L, m, r, pb);
  s.zeros(aligned - framed);
  return true;
}

// the tables in LDS (every run is read byte by byte; from HBM each word is a dependent round trip)
constexpr uint32_t kLdsTableWords = 12 * 1024;  // 48 KB
__device__ __forceinline__ void stage_tables(LogParams& L, uint32_t* lds) {
  if (L.arena_words + L.idx_words > kLdsTableWords) return;
  const uint32_t* a = reinterpret_cast<const uint32_t*>(L.arena);
  for (uint32_t i = threadIdx.x; i < L.arena_words; i += blockDim.x) lds[i] = a[i];
  for (uint32_t i = threadIdx.x; i < L.idx_words; i += blockDim.x) lds[L.arena_words + i] = L.idx[i];
  __syncthreads();
  L.arena = reinterpret_cast<const uint8_t*>(lds);
  L.idx = lds + L.arena_words;
}

// the record's entry template (id + 1, 0: composed instead): its kind (zb_internal.h kLogTplKinds),
// the keys the template can take (patched in its 9-byte msgpack form, or a process element's -1
// flowScopeKey that is part of the template)
__device__ __forceinline__ uint32_t tpl_of(const LogParams& L, const LogCmd& m, const Rec& r, uint4& d) {
  if (r.rt == ZBHIP_RT_REJECTION || r.act || r.proc >= L.tpl_idx[0] || L.pbits < (1LL << 32)) return 0;
  uint32_t k;
  switch (r.vt) {
    case ZBHIP_VT_PROCESS_INSTANCE: k = r.skip ? 10u + r.intent - 8u : r.intent - 1u; break;
    case ZBHIP_VT_JOB:
      k = r.intent == ZBHIP_JOB_CREATED ? 13u : r.intent == ZBHIP_JOB_COMPLETED && !m.doc_count ? 17u : NONE;
      break;
    case ZBHIP_VT_PROCESS_EVENT:
      k = r.intent == ZBHIP_PE_TRIGGERED ? 15u : r.intent == ZBHIP_PE_TRIGGERING && !m.doc_count ? 14u : NONE;
      break;
    case ZBHIP_VT_PROCESS_INSTANCE_CREATION: k = m.doc_count ? NONE : 16u; break;
    default: return 0;
  }
  if (k >= kLogTplKinds) return 0;
  const uint32_t pb = proc_block(L, r.proc);
  if (!pb || r.elem >= L.idx[pb + 5]) return 0;
  const uint32_t id = L.tpl_idx[L.tpl_idx[1 + r.proc] + r.elem * kLogTplKinds + k];
  if (!id) return 0;
  d = L.tpl_desc[id - 1];
  const long long big = 1LL << 32;
  if ((d.y >> 16) && r.pik < big) return 0;
  if (d.z ? r.scope < big : (r.vt != ZBHIP_VT_PROCESS_INSTANCE || r.scope != -1)) return 0;
  return id;
}

// pass 1: entry sizes per command, and per record its template or kSlow (flag bit 1: some record is
// composed, k_log_compose runs; bit 0: a key or value outside the device writer)
__global__ __launch_bounds__(256) void k_log_sizes(LogParams L) {
  extern __shared__ uint32_t tables[];
  stage_tables(L, tables);
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  bool slow = false;
  if (c < L.n) {
    const LogCmd m = L.cmds[c];
    Count s;
    KeyCache kc, kp;
    long long pik = -1;
    if (!key_of_lane(L, m, 0, pik, kp)) pik = -1;
    for (uint32_t j = 0; j < m.nrec; ++j) {
      Rec r;
      uint4 d;
      if (!decode(L, c, m, L.rows[m.rec_off + j], r, kc)) {
        atomicOr(L.flag, 1u);
        for (; j < m.nrec; ++j) L.rinfo[m.rec_off + j] = kSlow;  // (no stale info behind a declined record)
        break;
      }
      const uint32_t id = tpl_of(L, m, r, d);
      if (id && id < 0x8000u) {
        s.n += d.y & 0xFFFF;
        L.rinfo[m.rec_off + j] = id << 16 | (d.y & 0xFFFF);
      } else {
        Count e;
        if (!entry(e, L, m, r, 0) || e.n >= 0x10000) {
          atomicOr(L.flag, 1u);
          for (; j < m.nrec; ++j) L.rinfo[m.rec_off + j] = kSlow;
          break;
        }
        s.n += e.n;
        L.rinfo[m.rec_off + j] = kSlow | (uint32_t)e.n;
        slow = true;
      }
    }
    L.bytes[c] = s.n;
    if (L.wkeys) {
      LogKeys k;
      k.pik = pik;
      k.k0 = kc.k0;
      k.k1 = kc.k1;
      k.k2 = kc.k2;
      k.o0 = kc.o0;
      k.o1 = kc.o1;
      k.o2 = kc.o2;
      L.wkeys[c] = k;
    }
  }
  const unsigned long long b = __ballot(slow);
  if (b && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(b)) atomicOr(L.flag, 2u);
}

// x (8 bytes in memory order) placed at byte d of a 16-byte chunk (lo = bytes 0..7, hi = 8..15)
__device__ __forceinline__ void patch8(unsigned long long& lo, unsigned long long& hi, unsigned long long x, int d) {
  const unsigned long long M = ~0ull;
  if (d <= -8 || d >= 16) return;
  if (d < 0) {
    const int sh = -8 * d;
    lo = (lo & ~(M >> sh)) | (x >> sh);
  } else if (d < 8) {
    const int sh = 8 * d;
    lo = (lo & ~(M << sh)) | (x << sh);
    if (sh) hi = (hi & ~(M >> (64 - sh))) | (x >> (64 - sh));
  } else {
    const int sh = 8 * (d - 8);
    hi = (hi & ~(M << sh)) | (x << sh);
  }
}

// pass 2: the templated entries, written as one byte stream per command.  A half wave (32 lanes)
// takes a command at a time: lane l resolves record g*32 + l of group g (its template, keys, entry
// start by a half-wave scan of the entry sizes) into the half wave's LDS slots, then the 32 lanes
// write the group's bytes as consecutive 16-byte chunks -- every store instruction covers 1 KB of
// whole lines (entries are 8-aligned, so each 8-byte half of a chunk belongs to one entry; the
// halves outside the group, or in a composed entry, are left to their writer).  Writing each
// command's ~4 KB contiguously instead of entry by entry from scattered lanes leaves one partial
// line per command instead of one per entry.
struct StreamEnt {
  unsigned long long start;    // byte offset in the output
  long long key, scope, pik, lpos;
  uint32_t off, slow, pa, sa;  // template offset (16-aligned), composed entry, key patch positions
};
constexpr uint32_t kLogWriteB = 256;
constexpr uint32_t kHalf = 32;

// x (8 bytes in memory order) placed at byte d of an 8-byte word (branch-free; |d| >= 8: unchanged)
__device__ __forceinline__ unsigned long long patch_word(unsigned long long w, unsigned long long x, int d) {
  const unsigned long long M = ~0ull;
  const int sh = 8 * (d < 0 ? -d : d);
  const unsigned long long keep = d < 0 ? ~(M >> sh) : ~(M << sh);
  const unsigned long long put = d < 0 ? (x >> sh) : (x << sh);
  return d <= -8 || d >= 8 ? w : (w & keep) | put;
}

// the 8-byte word at byte rel (a multiple of 8) of a templated entry: template bytes (`tb`: the
// templates, LDS-staged), the header's position / source position / key / timestamp, the
// big-endian process instance and scope keys
__device__ __forceinline__ unsigned long long tpl_word(const uint8_t* tb, const StreamEnt& e, uint32_t rel,
                                                       long long src, unsigned long long ts) {
  unsigned long long w = *reinterpret_cast<const unsigned long long*>(tb + e.off + rel);
  w = rel == 16 ? (unsigned long long)e.lpos : rel == 24 ? (unsigned long long)src
      : rel == 32 ? (unsigned long long)e.key : rel == 40 ? ts : w;
  if (e.pa) w = patch_word(w, __builtin_bswap64((unsigned long long)e.pik), (int)e.pa - (int)rel);
  if (e.sa) w = patch_word(w, __builtin_bswap64((unsigned long long)e.scope), (int)e.sa - (int)rel);
  return w;
}

// Each half wave stages a group of its command's entries -- as many as fit kStage bytes -- in LDS
// exactly as they go out (template bytes, then the header fields and keys patched in), then copies
// the stage to the output in 16-byte chunks.  The copy loop issues no vector-memory load, so no
// s_waitcnt vmcnt (on gfx950 it counts the stores too) holds its streaming stores back; the stores
// drain once per group, when the next group's template loads are waited for.  Composed entries'
// bytes are staged as garbage and written over by k_log_compose, which runs after this kernel.
constexpr uint32_t kStage = 4096;  // bytes per half wave (+16 for the chunk alignment): 3 workgroups per CU
constexpr uint32_t kStageAlloc = kStage + 16;

__global__ __launch_bounds__(kLogWriteB) void k_log_write(LogParams L, uint32_t) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t lane = threadIdx.x & (kHalf - 1), hw = threadIdx.x / kHalf;
  uint8_t* const stage = reinterpret_cast<uint8_t*>(smem) + hw * kStageAlloc;
  uint8_t* const out = reinterpret_cast<uint8_t*>(L.out);
  const unsigned long long ts = (unsigned long long)L.timestamp;
  const uint32_t c0 = blockIdx.x * kLogWriteB + hw * kHalf;
  // a speculative launch (before the host read the size pass's results) writes nothing when the
  // window outgrew the buffer or the size pass declined it (its entry sizes are then incomplete)
  if (L.out_cap && ((*L.flag & 1u) || L.bytes[L.n] > L.out_cap)) return;
  // the half wave's 32 command rows and byte offsets, loaded at once (lane l: command c0 + l) and
  // handed to the whole half wave command by command: one coalesced load instead of a dependent
  // HBM round trip per command
  LogCmd mine{};
  unsigned long long mine_bytes = 0;
  if (c0 + lane < L.n) {
    mine = L.cmds[c0 + lane];
    mine_bytes = L.bytes[c0 + lane];
  }
  for (uint32_t ci = 0; ci < kHalf; ++ci) {
    const uint32_t c = c0 + ci;  // (half-wave uniform)
    if (c >= L.n) break;
    LogCmd m;
    m.rec_off = __shfl(mine.rec_off, ci, kHalf);
    m.out_rec = __shfl(mine.out_rec, ci, kHalf);
    m.key0 = __shfl(mine.key0, ci, kHalf);
    m.src_pos = __shfl(mine.src_pos, ci, kHalf);
    m.instance = __shfl(mine.instance, ci, kHalf);
    m.prev = __shfl(mine.prev, ci, kHalf);
    m.first_ord = (uint16_t)__shfl((uint32_t)mine.first_ord, ci, kHalf);
    m.nkeys = (uint16_t)__shfl((uint32_t)mine.nkeys, ci, kHalf);
    m.nrec = (uint16_t)__shfl((uint32_t)mine.nrec, ci, kHalf);
    m.doc_count = m.doc_begin = m.pad = 0;  // (templated entries carry no documents)
    unsigned long long gbase = __shfl(mine_bytes, ci, kHalf);
    KeyCache kc;
    for (uint32_t g = 0; g < m.nrec;) {
      const uint32_t j = g + lane;
      StreamEnt e;
      e.off = e.pa = e.sa = 0;
      e.slow = 1;
      e.key = e.scope = e.pik = e.lpos = 0;
      uint32_t size = 0;
      if (j < m.nrec) {
        const uint32_t info = L.rinfo[m.rec_off + j];
        size = info & 0xFFFF;
        if (!(info & kSlow)) {
          const uint2 w = L.rows[m.rec_off + j];
          const uint4 d = L.tpl_desc[(info >> 16) - 1];
          const bool ok = key_of_lane(L, m, w.x & 0xFFFF, e.key, kc) && key_of_lane(L, m, w.x >> 16, e.scope, kc) &&
                          key_of_lane(L, m, 0, e.pik, kc);
          e.slow = ok ? 0u : 1u;  // (k_log_sizes flagged a missing key already)
          e.off = d.x;
          e.pa = d.y >> 16;
          e.sa = d.z;
        }
        e.lpos = L.first_position + (long long)(m.out_rec + j);
      }
      // inclusive scan of the entry sizes over the half wave
      unsigned long long incl = size;
      for (uint32_t d = 1; d < kHalf; d <<= 1) {
        const unsigned long long y = __shfl_up(incl, d, kHalf);
        if (lane >= d) incl += y;
      }
      const uint32_t lead = (uint32_t)(gbase & 15);  // stage byte of gbase
      // the entries of this group: the prefix that fits the stage (at least one)
      const unsigned long long fits = __ballot(j < m.nrec && lead + incl <= kStage);
      const uint32_t hmask = (uint32_t)(fits >> (threadIdx.x & 32));
      uint32_t take = (uint32_t)__builtin_popcount(hmask);
      const bool staged = take > 0;
      if (!staged) take = 1;  // one entry larger than the stage: written from the templates directly
      const unsigned long long gsize = __shfl(incl, take - 1, kHalf);
      e.start = gbase + incl - size;
      const unsigned long long gend = gbase + gsize;
      if (staged) {
        if (lane < take && !e.slow) {  // the lane's entry into the stage
          uint8_t* const dst = stage + lead + (uint32_t)(incl - size);
          const uint8_t* const src = L.tpl + e.off;
          const uint32_t n8 = size / 8;
          uint32_t i = 0;
          for (; i + 8 <= n8; i += 8) {  // four 16-byte loads in flight per round trip
            uint4 t[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) t[k] = *reinterpret_cast<const uint4*>(src + 8 * i + 16 * k);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              reinterpret_cast<uint2*>(dst)[i + 2 * k] = make_uint2(t[k].x, t[k].y);
              reinterpret_cast<uint2*>(dst)[i + 2 * k + 1] = make_uint2(t[k].z, t[k].w);
            }
          }
          for (; i < n8; ++i) reinterpret_cast<uint2*>(dst)[i] = *reinterpret_cast<const uint2*>(src + 8 * i);
          unsigned long long* const w = reinterpret_cast<unsigned long long*>(dst);
          w[2] = (unsigned long long)e.lpos;  // LogEntryDescriptor: position, source position, key, timestamp
          w[3] = (unsigned long long)m.src_pos;
          w[4] = (unsigned long long)e.key;
          w[5] = ts;
          if (e.pa) {
            const uint32_t q = e.pa / 8;
            const unsigned long long x = __builtin_bswap64((unsigned long long)e.pik);
            w[q] = patch_word(w[q], x, (int)e.pa - (int)(8 * q));
            if (q + 1 < n8) w[q + 1] = patch_word(w[q + 1], x, (int)e.pa - (int)(8 * q + 8));
          }
          if (e.sa) {
            const uint32_t q = e.sa / 8;
            const unsigned long long x = __builtin_bswap64((unsigned long long)e.scope);
            w[q] = patch_word(w[q], x, (int)e.sa - (int)(8 * q));
            if (q + 1 < n8) w[q + 1] = patch_word(w[q + 1], x, (int)e.sa - (int)(8 * q + 8));
          }
        }
        // (the half wave's LDS writes precede its reads: one wave's LDS operations complete in order)
        __builtin_amdgcn_wave_barrier();
        const unsigned long long o0 = gbase & ~15ull;
        for (unsigned long long o = o0 + 16ull * lane; o < gend; o += 16ull * kHalf) {
          const uint4 v = *reinterpret_cast<const uint4*>(stage + (o - o0));
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
          if (o >= gbase && o + 16 <= gend) {
            u32x4 q;
            q.x = v.x; q.y = v.y; q.z = v.z; q.w = v.w;
            __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(out + o));
          } else {  // a chunk shared with the neighbouring group: only this group's half
            u32x2 q;
            if (o >= gbase) { q.x = v.x; q.y = v.y; __builtin_nontemporal_store(q, reinterpret_cast<u32x2*>(out + o)); }
            else { q.x = v.z; q.y = v.w; __builtin_nontemporal_store(q, reinterpret_cast<u32x2*>(out + o + 8)); }
          }
        }
      } else {
        // one oversized entry (lane 0's): 8-byte words straight from its template
        StreamEnt x;
        x.start = __shfl(e.start, 0, kHalf);
        x.key = __shfl(e.key, 0, kHalf);
        x.scope = __shfl(e.scope, 0, kHalf);
        x.pik = __shfl(e.pik, 0, kHalf);
        x.lpos = __shfl(e.lpos, 0, kHalf);
        x.off = __shfl(e.off, 0, kHalf);
        x.slow = __shfl(e.slow, 0, kHalf);
        x.pa = __shfl(e.pa, 0, kHalf);
        x.sa = __shfl(e.sa, 0, kHalf);
        if (!x.slow)
          for (unsigned long long a = gbase + 8ull * lane; a < gend; a += 8ull * kHalf)
            __builtin_nontemporal_store(tpl_word(L.tpl, x, (uint32_t)(a - gbase), m.src_pos, ts),
                                        reinterpret_cast<unsigned long long*>(out + a));
      }
      g += take;
      gbase = gend;
      __builtin_amdgcn_wave_barrier();  // the slots and the stage are rewritten by the next group
    }
  }
}

// pass 2, block form (the templates and their descriptors fit LDS beside the waves' areas): one
// wave per contiguous range of commands -- one contiguous byte range of the output -- taken in
// blocks of up to kBlkCmds commands / kBlkRecs records.  A block's command rows and key sets go into
// the lanes' registers (lane k: command k), its records' template info and key ordinals into the
// wave's LDS by direct global->LDS loads.  Those are the wave's only vector-memory loads, so it waits
// for its outstanding stores once per block, not once per group as k_log_write does (on gfx950
// s_waitcnt vmcnt counts stores too: k_log_write's waves spent 62 % of their cycles there).  The
// block's entries form one stream: lane j of a group of 64 takes entry e0 + j, its command's fields
// by permutes from the command lanes, and resolves its template and keys; the prefix of the group
// that fits the wave's stage is then composed in three steps -- the template words, word-parallel
// (lane x: stage word x, its entry found from one ballot of the entry starts; consecutive words, no
// bank conflicts), the header fields and big-endian keys, one lane per entry, and the stage out in
// 16-byte non-temporal chunks, 1 KB of whole lines per store instruction.  Scans are DPP (no LDS
// round trip).  (Round 4's k_log_stream composed entry by entry with the whole wave: ~100
// wave-instructions per entry; round 5's word-only form, no stage, ~150 per 512 bytes: both slower.)
// default-policy stores: measured 1.07 ms per window against 1.24 ms with non-temporal stores
// (scripts/ab_logstores.sh; ZB_LOG_NT_STORES builds the other)
#ifdef ZB_LOG_NT_STORES
#define ZB_LOG_STORE(v, p) __builtin_nontemporal_store(v, p)
#else
#define ZB_LOG_STORE(v, p) (*(p) = (v))
#endif
constexpr uint32_t kBlkCmds = 32;
constexpr uint32_t kBlkRecs = 192;
constexpr uint32_t kBlkLdsMax = 160 * 1024;

typedef __attribute__((address_space(1))) void g_void;
typedef __attribute__((address_space(3))) void l_void;

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ unsigned long long rl64(unsigned long long v, uint32_t k) {
  return (unsigned long long)rl((uint32_t)v, k) | (unsigned long long)rl((uint32_t)(v >> 32), k) << 32;
}
// orders one wave's LDS accesses across its lanes for the compiler (the hardware keeps a wave's LDS
// operations in order)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// inclusive scan over the wave by DPP (row shifts within rows of 16, then the row broadcasts): VALU
// only, where __shfl_up is an LDS permute and its round trip per step
__device__ __forceinline__ uint32_t wave_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}
template <uint32_t NW, uint32_t ST>
struct BlkShape {
  static constexpr uint32_t kWaveLds = kBlkRecs * 8 + ST + 16;  // rinfo, rows (their first words), stage
  static constexpr uint32_t kLds = NW * kWaveLds;
};

template <uint32_t NW, uint32_t ST>
__global__ __launch_bounds__(NW * 64) void k_log_blocks(LogParams L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint8_t* const lds = reinterpret_cast<uint8_t*>(smem);
  if (L.out_cap && ((*L.flag & 1u) || L.bytes[L.n] > L.out_cap)) return;  // (as k_log_write)
  // LDS: the waves' record areas first (the direct global->LDS loads address LDS through M0: kept in
  // the low 64 KB), then their stages, then the templates and descriptors
  const uint32_t T = (L.tpl_lds + 15u) & ~15u;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* const lri = reinterpret_cast<uint32_t*>(lds + wv * (kBlkRecs * 8));
  uint32_t* const lrow = lri + kBlkRecs;  // the first word of each record's row (its key ordinals)
  uint8_t* const stage = lds + NW * (kBlkRecs * 8) + wv * (ST + 16);
  uint8_t* const tpl = lds + BlkShape<NW, ST>::kLds;
  for (uint32_t i = threadIdx.x; i < T / 16; i += blockDim.x)
    reinterpret_cast<uint4*>(tpl)[i] = reinterpret_cast<const uint4*>(L.tpl)[i];
  __syncthreads();
  const uint4* const desc = reinterpret_cast<const uint4*>(tpl + (reinterpret_cast<const uint8_t*>(L.tpl_desc) - L.tpl));
  uint8_t* const out = reinterpret_cast<uint8_t*>(L.out);
  const unsigned long long ts = (unsigned long long)L.timestamp;
  const unsigned long long W = (unsigned long long)gridDim.x * NW;
  const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * NW + wv);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const uint32_t ce = (uint32_t)((unsigned long long)L.n * (w + 1) / W);
  uint32_t c = (uint32_t)((unsigned long long)L.n * w / W);
  uint32_t j0 = 0;              // records of command c already written (a command longer than a block)
  unsigned long long gpos = 0;  // and the byte position after them
  bool carry = false;           // the stage's first word holds the 8 bytes before gpos, not yet written
  auto flush_carry = [&](unsigned long long at) {  // (the carried word is the 8 bytes before `at`)
    if (carry && lane == 0) {
      u32x2 q;
      const uint2 v = *reinterpret_cast<const uint2*>(stage);
      q.x = v.x; q.y = v.y;
      ZB_LOG_STORE(q, reinterpret_cast<u32x2*>(out + at - 8));
    }
    carry = false;
  };
  while (c < ce) {
    const uint32_t nb = ce - c < kBlkCmds ? ce - c : kBlkCmds;
    LogCmd m{};
    unsigned long long mb = 0;
    LogKeys mk{};
    if (lane < nb) {
      m = L.cmds[c + lane];
      mb = L.bytes[c + lane];
      mk = L.wkeys[c + lane];
    }
    const uint32_t cnt = lane < nb ? (uint32_t)m.nrec - (lane == 0 ? j0 : 0u) : 0u;
    const uint32_t incl = wave_scan(cnt);
    uint32_t take = (uint32_t)__builtin_popcountll(__ballot(lane < nb && incl <= kBlkRecs));
    uint32_t first = rl(cnt, 0);
    const bool partial = take == 0;  // command c alone has more records than a block: its next kBlkRecs
    if (partial) {
      take = 1;
      first = kBlkRecs;
    }
    // the block's record info and rows into the wave's LDS
    uint32_t p = 0;
    for (uint32_t k = 0; k < take; ++k) {
      const uint32_t rk = rl((uint32_t)m.rec_off, k) + (k == 0 ? j0 : 0u);
      const uint32_t nk = k == 0 ? first : rl(cnt, k);
      for (uint32_t q = 0; q < nk; q += 64)
        if (q + lane < nk)
          __builtin_amdgcn_global_load_lds((g_void*)(L.rinfo + rk + q + lane), (l_void*)(lri + p + q), 4, 0, 0);
      const uint32_t* const rw = reinterpret_cast<const uint32_t*>(L.rows) + 2ull * rk;
      for (uint32_t q = 0; q < nk; q += 64)
        if (q + lane < nk) __builtin_amdgcn_global_load_lds((g_void*)(rw + 2 * (q + lane)), (l_void*)(lrow + p + q), 4, 0, 0);
      p += nk;
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the loads above have landed in LDS
    wave_lds_sync();
    // the block's entries as one stream (the commands' bytes follow each other): lane j of a group
    // takes entry e0 + j, its command's fields by permutes from the command lanes
    const uint32_t P = partial ? first : rl(incl, take - 1);
    const uint32_t ks = incl - cnt;  // (command lane k: its first entry in the block)
    unsigned long long pos = j0 ? gpos : rl64(mb, 0);  // output byte of the next entry
    for (uint32_t e0 = 0; e0 < P; e0 += 64) {
      const uint32_t ng = P - e0 < 64 ? P - e0 : 64u;
      const uint32_t e = e0 + lane;
      // the entry's command: the last one starting at or before it
      uint32_t kk = (uint32_t)__builtin_popcountll(__ballot(lane < take && ks <= e0)) - 1u;
      unsigned long long S = __ballot(lane < take && ks > e0 && ks < e0 + 64);
      while (S) {
        const uint32_t j = (uint32_t)__builtin_ctzll(S);
        S &= S - 1;
        kk += e >= rl(ks, j) ? 1u : 0u;
      }
      const int ki = (int)kk;
      const unsigned long long out_rec = __shfl(m.out_rec, ki), key0 = __shfl(m.key0, ki);
      const unsigned long long src = (unsigned long long)__shfl(m.src_pos, ki);
      const uint32_t fo_nk = __shfl((uint32_t)m.first_ord | (uint32_t)m.nkeys << 16, ki);
      const uint32_t first_ord = fo_nk & 0xFFFF, nkeys = fo_nk >> 16;
      const long long pik = __shfl(mk.pik, ki), k0 = __shfl(mk.k0, ki), k1 = __shfl(mk.k1, ki), k2 = __shfl(mk.k2, ki);
      const uint32_t o0 = __shfl(mk.o0, ki), o1 = __shfl(mk.o1, ki), o2 = __shfl(mk.o2, ki);
      const uint32_t prev = __shfl(m.prev, ki), inst = __shfl(m.instance, ki);
      const uint32_t ie = e - __shfl(ks, ki) + (kk == 0 ? j0 : 0u);  // the entry's index in its command
      auto wkey = [&](uint32_t ord) -> long long {
        if (ord == NONE) return -1;
        if (nkeys && ord >= first_ord) return L.pbits + (long long)(key0 + (uint16_t)(ord - first_ord));
        if (ord == 0) return pik;
        if (ord == o0) return k0;
        if (ord == o1) return k1;
        if (ord == o2) return k2;
        long long key = 0;  // (a fourth older ordinal: the key chain in memory)
        key_of(L, first_ord == 0 ? 0xFFFFFFFFu : prev, inst, ord, key);
        return key;
      };
      {
        // lane j: entry e0 + j (its template, keys, size)
        uint32_t size = 0, off = 0, pa = 0, sa = 0;
        bool slow = true;
        long long key = 0, scope = 0;
        if (lane < ng) {
          const uint32_t info = lri[e];
          size = info & 0xFFFF;
          if (!(info & kSlow)) {
            const uint32_t rx = lrow[e];
            const uint4 d = desc[(info >> 16) - 1];
            off = d.x;
            pa = d.y >> 16;
            sa = d.z;
            key = wkey(rx & 0xFFFF);
            scope = wkey(rx >> 16);
            slow = false;
          }
        }
        const uint32_t end = wave_scan(size);  // entry j ends at byte `end` of the group
        const unsigned long long lpos = (unsigned long long)(L.first_position + (long long)(out_rec + ie));
        const unsigned long long pik_be = __builtin_bswap64((unsigned long long)pik);
        const unsigned long long scope_be = __builtin_bswap64((unsigned long long)scope);
        uint32_t g = 0;     // entries of the group written
        uint32_t gb = 0;    // and their bytes
        while (g < ng) {
          const uint32_t lead = (uint32_t)(pos & 15);  // stage byte of pos
          // the entries that fit the stage from entry g on (at least one)
          const unsigned long long fits = __ballot(lane >= g && lane < ng && lead + (end - gb) <= ST);
          const uint32_t t = (uint32_t)__builtin_popcountll(fits);
          if (!t) {
            flush_carry(pos);
            // entry g alone is larger than the stage: its words straight from the template
            const uint32_t sz = rl(size, g), o = rl(off, g), a = rl(pa, g), b = rl(sa, g);
            if (!(rl((uint32_t)slow, g))) {
              const unsigned long long kg = rl64((unsigned long long)key, g), sb = rl64(scope_be, g), lp = rl64(lpos, g);
              const unsigned long long sg = rl64(src, g), pb = rl64(pik_be, g);
              for (uint32_t x = 8 * lane; x < sz; x += 512) {
                unsigned long long v = *reinterpret_cast<const unsigned long long*>(tpl + o + x);
                v = x == 16 ? lp : x == 24 ? sg : x == 32 ? kg : x == 40 ? ts : v;
                if (a) v = patch_word(v, pb, (int)a - (int)x);
                if (b) v = patch_word(v, sb, (int)b - (int)x);
                __builtin_nontemporal_store(v, reinterpret_cast<unsigned long long*>(out + pos + x));
              }
            }
            pos += sz;
            gb += sz;
            ++g;
            continue;
          }
          const uint32_t ge = rl(end, g + t - 1) - gb;  // the staged entries' bytes
          const bool mine = lane >= g && lane < g + t;
          // the template words into the stage, word-parallel (lane x: stage word cb + x, consecutive
          // words: no bank conflicts): its entry is the last one starting at or before it
          const uint32_t sw = (lead + end - size - gb) >> 3;  // the lane's entry's first stage word
          const uint32_t ew = (lead + ge) >> 3;
          const uint32_t dl = (slow ? 0u : off) - 8 * sw;  // (mod 2^32)
          for (uint32_t cb = lead >> 3; cb < ew; cb += 128) {  // (two words per lane in flight)
            const uint32_t x0 = cb + lane, x1 = x0 + 64;
            uint32_t r0 = (uint32_t)__builtin_popcountll(__ballot(mine && sw <= cb)) + g - 1u, r1 = r0;
            unsigned long long S = __ballot(mine && sw > cb && sw < cb + 128);
            while (S) {
              const uint32_t j = (uint32_t)__builtin_ctzll(S);
              S &= S - 1;
              const uint32_t v = rl(sw, j);
              r0 += x0 >= v ? 1u : 0u;
              r1 += x1 >= v ? 1u : 0u;
            }
            // (one permute per word: the entry's template byte minus its stage byte)
            const uint32_t d0 = __shfl(dl, (int)r0), d1 = __shfl(dl, (int)r1);
            // (a composed entry's words read template 0's bytes: garbage k_log_compose writes over;
            // words past the group go to the stage's spare last word: no branches)
            const unsigned long long t0 = *reinterpret_cast<const unsigned long long*>(tpl + d0 + 8 * x0);
            const unsigned long long t1 = *reinterpret_cast<const unsigned long long*>(tpl + d1 + 8 * x1);
            *reinterpret_cast<unsigned long long*>(stage + (x0 < ew ? 8 * x0 : ST + 8)) = t0;
            *reinterpret_cast<unsigned long long*>(stage + (x1 < ew ? 8 * x1 : ST + 8)) = t1;
          }
          wave_lds_sync();
          if (mine && !slow) {
            // the lane's entry: header fields and keys over the template words
            unsigned long long* const d64 = reinterpret_cast<unsigned long long*>(stage) + sw;
            const uint32_t n8 = size / 8;
            d64[2] = lpos;  // LogEntryDescriptor: position, source position, key, timestamp
            d64[3] = src;
            d64[4] = (unsigned long long)key;
            d64[5] = ts;
            // (each key's two words read together, then written: one round trip per key)
            if (pa) {
              const uint32_t q = pa / 8, q1 = q + 1 < n8 ? q + 1 : q;
              const unsigned long long a0 = d64[q], a1 = d64[q1];
              d64[q1] = patch_word(a1, pik_be, (int)pa - (int)(8 * q1));
              d64[q] = patch_word(a0, pik_be, (int)pa - (int)(8 * q));
            }
            if (sa) {
              const uint32_t q = sa / 8, q1 = q + 1 < n8 ? q + 1 : q;
              const unsigned long long a0 = d64[q], a1 = d64[q1];
              d64[q1] = patch_word(a1, scope_be, (int)sa - (int)(8 * q1));
              d64[q] = patch_word(a0, scope_be, (int)sa - (int)(8 * q));
            }
          }
          wave_lds_sync();
          // the stage out: 16-byte chunks of whole lines, the 8-byte half of a chunk shared with the
          // neighbouring group alone
          uint8_t* const ob = out + (pos & ~15ull);
          const uint32_t e = lead + ge;
          // (a trailing half chunk is not written: its 8 bytes move to the stage's first word and go
          // out with the next group's first chunk -- `carry` -- so every store is a whole chunk but
          // the upper half at the start of the wave's range and the last word at its end)
          auto put = [&](uint32_t o, uint4 v) {
            if (o + 16 > e) return;  // (the trailing half: carried)
            if (o >= lead || carry) {
              u32x4 q;
              q.x = v.x; q.y = v.y; q.z = v.z; q.w = v.w;
              ZB_LOG_STORE(q, reinterpret_cast<u32x4*>(ob + o));
            } else {
              u32x2 q;
              q.x = v.z; q.y = v.w;
              ZB_LOG_STORE(q, reinterpret_cast<u32x2*>(ob + o + 8));
            }
          };
          for (uint32_t o = 16u * lane; o < e; o += 2048u) {  // (two chunks per lane in flight)
            // (both reads before the stores; a read past the stage reads a neighbour's bytes, unused)
            const uint4 v0 = *reinterpret_cast<const uint4*>(stage + o);
            const uint4 v1 = *reinterpret_cast<const uint4*>(stage + o + 1024);
            put(o, v0);
            if (o + 1024 < e) put(o + 1024, v1);
          }
          carry = (e & 15) != 0;
          if (carry && lane == 0)
            *reinterpret_cast<unsigned long long*>(stage) = *reinterpret_cast<const unsigned long long*>(stage + e - 8);
          wave_lds_sync();
          pos += ge;
          gb += ge;
          g += t;
        }
      }
    }
    gpos = pos;
    if (partial) {
      j0 += first;
      if (j0 >= rl(m.nrec, 0)) {
        ++c;
        j0 = 0;
      }
    } else {
      c += take;
      j0 = 0;
    }
  }
  flush_carry(gpos);
}

// pass 2b (flag bit 1 only): the entries without a template, composed by their command's lane
__global__ __launch_bounds__(256) void k_log_compose(LogParams L) {
  extern __shared__ uint32_t tables[];
  stage_tables(L, tables);
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= L.n) return;
  const LogCmd m = L.cmds[c];
  unsigned long long pos = L.bytes[c];
  KeyCache kc;
  for (uint32_t j = 0; j < m.nrec; ++j) {
    const uint32_t info = L.rinfo[m.rec_off + j];
    if (info & kSlow) {
      Rec r;
      if (!decode(L, c, m, L.rows[m.rec_off + j], r, kc)) return;
      Write w;
      w.start(L.out + (pos >> 3));
      entry(w, L, m, r, L.first_position + (long long)(m.out_rec + j));
      w.finish();
    }
    pos += info & 0xFFFF;
  }
}

// exclusive scan of the per-command byte counts (in place), total at bytes[n]
constexpr int kLogScanB = 1024;
__global__ __launch_bounds__(kLogScanB) void k_log_block_sums(unsigned long long* v, uint32_t n, unsigned long long* bs) {
  const uint32_t i = blockIdx.x * kLogScanB + threadIdx.x;
  __shared__ unsigned long long ws[kLogScanB / 64];
  unsigned long long x = i < n ? v[i] : 0ull;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(x, off);
    if ((threadIdx.x & 63) >= (uint32_t)off) x += y;
  }
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kLogScanB / 64; ++w) t += ws[w];
    bs[blockIdx.x] = t;
  }
}
// exclusive scan of the block sums in place (one workgroup, kLogScanB at a time), total at *total
__global__ __launch_bounds__(kLogScanB) void k_log_scan_sums(unsigned long long* bs, uint32_t nb, unsigned long long* total) {
  __shared__ unsigned long long ws[kLogScanB / 64];
  __shared__ unsigned long long carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nb; base += kLogScanB) {
    const uint32_t i = base + threadIdx.x;
    const unsigned long long x0 = i < nb ? bs[i] : 0ull;
    unsigned long long x = x0;
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned long long y = __shfl_up(x, off);
      if ((threadIdx.x & 63) >= (uint32_t)off) x += y;
    }
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    unsigned long long b = carry;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) b += ws[w];
    if (i < nb) bs[i] = b + x - x0;
    __syncthreads();
    if (threadIdx.x == kLogScanB - 1) carry = b + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}
__global__ __launch_bounds__(kLogScanB) void k_log_apply(unsigned long long* v, uint32_t n, const unsigned long long* bs) {
  const uint32_t i = blockIdx.x * kLogScanB + threadIdx.x;
  __shared__ unsigned long long ws[kLogScanB / 64];
  const unsigned long long x0 = i < n ? v[i] : 0ull;
  unsigned long long x = x0;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(x, off);
    if ((threadIdx.x & 63) >= (uint32_t)off) x += y;
  }
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  unsigned long long b = bs[blockIdx.x];
  for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) b += ws[w];
  if (i < n) v[i] = b + x - x0;
}

// The command table of a one-round window whose rows were gathered in log order, on the device:
// rec_off = out_rec = the exclusive scan of the record counts, key0 = the key counter + 1 + the
// exclusive scan of the key counts (runtime.cpp builds the same on the host for other windows).
// Block sums pack records (low half) and keys (high half): neither passes 2^32 in a window.
__global__ __launch_bounds__(kLogScanB) void k_table_block_sums(const uint2* hdr, uint32_t n, unsigned long long* bs) {
  const uint32_t i = blockIdx.x * kLogScanB + threadIdx.x;
  __shared__ unsigned long long ws[kLogScanB / 64];
  const uint2 h = i < n ? hdr[i] : make_uint2(0, 0);
  unsigned long long x = (unsigned long long)(h.x & 0xFFFF) | ((unsigned long long)(h.x >> 16) << 32);
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(x, off);
    if ((threadIdx.x & 63) >= (uint32_t)off) x += y;
  }
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kLogScanB / 64; ++w) t += ws[w];
    bs[blockIdx.x] = t;
  }
}
__global__ __launch_bounds__(kLogScanB) void k_table_build(LogParams L, const uint2* hdr, const zbhip_command* cmds,
                                                          const long long* src_pos, unsigned long long key_base,
                                                          const unsigned long long* bs, LogCmd* out,
                                                          uint16_t* inst_proc, uint4* jrn) {
  const uint32_t i = blockIdx.x * kLogScanB + threadIdx.x;
  __shared__ unsigned long long ws[kLogScanB / 64];
  const uint2 h = i < L.n ? hdr[i] : make_uint2(0, 0);
  const unsigned long long x0 = (unsigned long long)(h.x & 0xFFFF) | ((unsigned long long)(h.x >> 16) << 32);
  unsigned long long x = x0;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(x, off);
    if ((threadIdx.x & 63) >= (uint32_t)off) x += y;
  }
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  unsigned long long b = bs[blockIdx.x];
  for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) b += ws[w];
  if (i >= L.n) return;
  const unsigned long long ex = b + x - x0;  // records before | keys before << 32
  const zbhip_command cm = cmds[i];
  LogCmd m;
  m.rec_off = ex & 0xFFFFFFFFull;
  m.out_rec = m.rec_off;
  m.key0 = key_base + 1 + (ex >> 32);
  m.src_pos = src_pos ? src_pos[i] : -1;
  m.instance = cm.instance;
  m.prev = ~0u;
  m.first_ord = (uint16_t)(h.y & 0xFFFF);
  m.nkeys = ((h.y >> 16) & 0xFF) == ST_OK ? (uint16_t)(h.x >> 16) : (uint16_t)0;
  m.nrec = (uint16_t)(h.x & 0xFFFF);
  m.doc_count = cm.doc_count;
  m.doc_begin = cm.doc_begin;
  m.pad = cm.pad;
  out[i] = m;
  // a CREATE starts its slot's instance (one command per instance in a one-round window)
  if (cm.kind == ZBHIP_CMD_CREATE && cm.instance < L.n_inst) inst_proc[cm.instance] = cm.ref;
  // the window's key bookkeeping journal (runtime.cpp fold_journal): first key, its ordinal, the
  // instance and whether the batch ended it, the key count and a CREATE's process
  if (jrn)
    jrn[i] = make_uint4((uint32_t)m.key0, ((uint32_t)(m.key0 >> 32) & 0xFFFFu) | (uint32_t)m.first_ord << 16,
                        cm.instance | (h.y & HDR_ENDED), (uint32_t)m.nkeys |
                        (uint32_t)(cm.kind == ZBHIP_CMD_CREATE ? cm.ref : 0xFFFFu) << 16);
}

// ring fill after the window: CREATEs reset their instance (a new generation), then every command
// adds its batch's ordinals (atomicMax: a later batch of the instance carries larger ordinals)
__global__ __launch_bounds__(256) void k_ring_create(LogParams L) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= L.n) return;
  const LogCmd m = L.cmds[c];
  if (!m.nkeys || m.first_ord != 0 || m.instance >= L.n_inst) return;
  for (uint32_t s = 0; s < kRing; ++s) L.ring[(size_t)s * L.n_inst + m.instance] = 0ull;
  L.kpi[m.instance] = (1ull << 63) | (unsigned long long)m.key0;
}
__global__ __launch_bounds__(256) void k_ring_add(LogParams L) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= L.n) return;
  const LogCmd m = L.cmds[c];
  if (!m.nkeys || m.instance >= L.n_inst) return;
  const uint32_t k0 = m.nkeys > kRing ? m.nkeys - kRing : 0u;  // the last kRing ordinals of the batch
  for (uint32_t k = k0; k < m.nkeys; ++k) {
    const uint32_t ord = (uint16_t)(m.first_ord + k);
    const unsigned long long e = ((unsigned long long)ord << 48) | (unsigned long long)(m.key0 + k);
    atomicMax(&L.ring[(size_t)(ord % kRing) * L.n_inst + m.instance], e);
  }
}

hipError_t launch_log_device(const LogLaunch& a, hipStream_t s) {
  LogParams L{a.rows, a.cmds, a.n, a.arena, a.idx, a.arena_words, a.idx_words, a.docs, a.n_docs, a.inst_proc, a.ring,
              a.kpi, a.n_inst, a.pbits, a.first_position, a.timestamp, {a.broker[0], a.broker[1], a.broker[2]},
              a.bytes, a.out, a.flag, a.now_ms, a.cmd_due, a.tpl, a.tpl_desc, a.tpl_idx, a.rinfo, a.out_cap,
              a.wkeys, a.tpl_lds, a.cmd_act, a.strs, a.str_off, a.n_strs};
  const uint32_t g = (a.n + 255) / 256;
  const size_t lds = a.arena_words + a.idx_words <= kLdsTableWords ? (size_t)(a.arena_words + a.idx_words) * 4 : 0;
  if (a.phase == 0) {  // sizes and byte offsets
    if (a.n) hipLaunchKernelGGL(k_log_sizes, dim3(g), dim3(256), lds, s, L);
    const uint32_t nb = (a.n + kLogScanB - 1) / kLogScanB;
    if (a.n) hipLaunchKernelGGL(k_log_block_sums, dim3(nb), dim3(kLogScanB), 0, s, a.bytes, a.n, a.block_sums);
    hipLaunchKernelGGL(k_log_scan_sums, dim3(1), dim3(kLogScanB), 0, s, a.block_sums, nb, a.bytes + a.n);
    if (a.n) hipLaunchKernelGGL(k_log_apply, dim3(nb), dim3(kLogScanB), 0, s, a.bytes, a.n, a.block_sums);
  } else if (a.phase == 3) {  // the command table (block sums, their scan, the rows)
    const uint32_t nb = (a.n + kLogScanB - 1) / kLogScanB;
    if (a.n) hipLaunchKernelGGL(k_table_block_sums, dim3(nb), dim3(kLogScanB), 0, s, a.hdr, a.n, a.table_sums);
    hipLaunchKernelGGL(k_log_scan_sums, dim3(1), dim3(kLogScanB), 0, s, a.table_sums, nb, a.table_sums + nb);
    if (a.n)
      hipLaunchKernelGGL(k_table_build, dim3(nb), dim3(kLogScanB), 0, s, L, a.hdr, a.wcmds, a.src_pos, a.key_base,
                         a.table_sums, a.table, a.inst_proc_w, a.jrn);
  } else if (a.phase == 1) {
    // k_log_blocks when the templates fit LDS beside the waves' areas (k_log_write otherwise: it reads
    // them from memory; ZBHIP_LOG_HALFWAVE=1 forces it).  Two shapes: 8 waves with 8 KB stages, or 16
    // waves with 3 KB stages (ZBHIP_LOG_BLOCKS=16)
    static int cus = 0;
    static bool attr8 = false, attr12 = false, attr16 = false;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus <= 0)
        cus = 256;
      attr8 = hipFuncSetAttribute(reinterpret_cast<const void*>(k_log_blocks<8, 8192>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)kBlkLdsMax) == hipSuccess;
      attr12 = hipFuncSetAttribute(reinterpret_cast<const void*>(k_log_blocks<12, 6144>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)kBlkLdsMax) == hipSuccess;
      attr16 = hipFuncSetAttribute(reinterpret_cast<const void*>(k_log_blocks<16, 4096>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)kBlkLdsMax) == hipSuccess;
      (void)hipGetLastError();
    }
    const int want = getenv("ZBHIP_LOG_BLOCKS") ? atoi(getenv("ZBHIP_LOG_BLOCKS")) : 16;
    const uint32_t nw = want == 8 ? 8u : want == 12 ? 12u : 16u;
    const size_t T = (size_t)((a.tpl_lds + 15u) & ~15u);
    const size_t blds = T + (nw == 8 ? BlkShape<8, 8192>::kLds : nw == 12 ? BlkShape<12, 6144>::kLds : BlkShape<16, 4096>::kLds);
    const bool attr = nw == 8 ? attr8 : nw == 12 ? attr12 : attr16;
    const bool blocks = attr && a.wkeys && a.tpl_lds && blds <= kBlkLdsMax && !getenv("ZBHIP_LOG_HALFWAVE");
    static bool told = false;
    if (!told && getenv("ZBHIP_DEBUG")) {
      told = true;
      fprintf(stderr, "[zbhip] log write pass: %s, %u waves (templates + descriptors %u B, LDS %zu B)\n",
              blocks ? "k_log_blocks" : "k_log_write", nw, a.tpl_lds, blds);
    }
    if (a.n && a.compose != 2 && blocks) {
      uint32_t grid = (uint32_t)cus * (kBlkLdsMax / blds >= 2 ? 2u : 1u);
      const uint32_t need = (a.n + nw * 16 - 1) / (nw * 16);  // >= 16 commands per wave
      if (need < grid) grid = need;
      if (nw == 16) hipLaunchKernelGGL((k_log_blocks<16, 4096>), dim3(grid), dim3(16 * 64), blds, s, L);
      else if (nw == 12) hipLaunchKernelGGL((k_log_blocks<12, 6144>), dim3(grid), dim3(12 * 64), blds, s, L);
      else hipLaunchKernelGGL((k_log_blocks<8, 8192>), dim3(grid), dim3(8 * 64), blds, s, L);
    } else if (a.n && a.compose != 2) {
      hipLaunchKernelGGL(k_log_write, dim3((a.n + kLogWriteB - 1) / kLogWriteB), dim3(kLogWriteB),
                         (size_t)(kLogWriteB / kHalf) * kStageAlloc, s, L, 0u);
    }
    if (a.n && a.compose) hipLaunchKernelGGL(k_log_compose, dim3(g), dim3(256), lds, s, L);
  } else {
    if (a.n) hipLaunchKernelGGL(k_ring_create, dim3(g), dim3(256), 0, s, L);
    if (a.n) hipLaunchKernelGGL(k_ring_add, dim3(g), dim3(256), 0, s, L);
  }
  return hipGetLastError();
}

}  // namespace zb
