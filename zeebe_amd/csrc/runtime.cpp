// Host runtime of libzbhip.so: partition handles, deployment into the LDS program arena,
// command windows, kernel launches, key relabelling, record drain and state export.
//
// The handle is one Zeebe partition (StreamProcessor + Engine of one partition,
// broker/.../steps/StreamProcessorTransitionStep.java:127-165); all device memory it needs is
// allocated at open (HBM is sized for the instance capacity, SoA), nothing is allocated in
// the run path.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <tuple>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <deque>
#include <iterator>
#include <new>
#include <vector>

#include "zb_internal.h"

namespace zb {
uint32_t step_block(int variant);
uint32_t step_resident(int variant, uint32_t prog_words);
uint32_t step_queue(int variant);
size_t step_lds_bytes(int variant, uint32_t prog_words);
hipError_t launch_step(int variant, const StepParams& P, hipStream_t s);
void dump_stamps();
uint32_t step_rows(int variant);
hipError_t launch_gather(const uint2* regions, const uint32_t* tot, const uint16_t* lanes, uint32_t n_regions,
                         unsigned long long* off, size_t region_stride, uint32_t B, uint32_t R, uint2* out,
                         unsigned long long* total, hipStream_t s);
hipError_t launch_keyscan(const uint2* cmd_hdr, const uint4* cmd_hdr2, const uint4* cmds, uint32_t n,
                          unsigned long long* block_sum, unsigned long long* base, unsigned long long* counter,
                          zbhip_xpart_cmd* xout, uint32_t xcap, const DevState& st, long long pbits, hipStream_t s);
hipError_t launch_xpart_window(const zbhip_xpart_cmd* xp, uint32_t n, uint4* cmds, hipStream_t s);
hipError_t launch_activate_jobs(const DevState& st, const uint2* jobs, uint32_t n, void* out, uint32_t worker,
                                long long deadline, hipStream_t s);
hipError_t launch_log_device(const LogLaunch& a, hipStream_t s);
int log_device_tables(const zbhip_serializer* s, std::vector<uint8_t>& arena, std::vector<uint32_t>& idx);
int log_device_templates(zbhip_serializer* s, std::vector<uint8_t>& bytes, std::vector<uint32_t>& desc,
                         std::vector<uint32_t>& idx);
void serializer_broker(const zbhip_serializer* s, int32_t out[3]);
size_t activated_out_bytes();
size_t subject_sort_temp_bytes(uint32_t n);
hipError_t launch_subject_sort(const uint4* cmds, uint32_t n, uint32_t n_inst, uint32_t n_subjects, uint32_t* k0,
                               uint32_t* k1, uint32_t* v0, uint32_t* order, void* temp, size_t temp_bytes,
                               hipStream_t s);
hipError_t launch_subject_check(const uint4* cmds, uint32_t n, uint32_t n_inst, uint32_t n_slots, uint32_t* seen,
                                uint32_t stamp, uint32_t* w, hipStream_t s);
hipError_t launch_check_publish(const uint32_t* w, uint32_t stamp, uint32_t* host, hipStream_t s);
hipError_t launch_bucket(const uint2* cmd_hdr, const uint4* cmd_hdr2, const zbhip_xpart_cmd* xout, uint32_t xcap,
                         uint32_t n, uint32_t parts, uint32_t* blk_cnt, uint32_t* counts, zbhip_xpart_cmd* out,
                         hipStream_t s);
hipError_t launch_xgather(const XGather& A, uint32_t max_count, hipStream_t s);
hipError_t launch_due_timers(const DevState& st, long long now, DueTimer* out, uint32_t* count,
                             unsigned long long* next_due, hipStream_t s);
constexpr uint32_t kExtraRegions = 64;
constexpr size_t kBulkDrainMin = 1 << 16;  // records: below this the drain stays on the calling thread
constexpr uint32_t kRegionPad = 0;  // regions for the extra workgroups of multi-round windows
}  // namespace zb

using namespace zb;

namespace {

// hex of a string inside a state row (error messages may hold ',' and '|')
std::string hex_of(const std::string& v) {
  static const char* d = "0123456789abcdef";
  std::string o;
  for (unsigned char c : v) {
    o += d[c >> 4];
    o += d[c & 15];
  }
  return o;
}

struct Proc {
  std::vector<zbhip_element> els;
  std::vector<uint16_t> out;
  std::vector<uint32_t> cond_begin;
  std::vector<zbhip_insn> code;
  std::vector<std::string> strings;
  uint16_t none_start = NONE;
  uint16_t n_join_slots = 0;
  int64_t def_key = 0;
  int32_t version = 1;
  uint16_t bpmn_id = 0;
  uint16_t bpmn_name = NONE;  // name id of the bpmnProcessId (processes with message catch events)
  bool has_msg = false;
  bool has_timer = false;     // timer catch events (KScope, the instance timer row)
  std::vector<uint32_t> job_type_id;  // per element: id of its job type (service tasks), else ~0
  // multi-instance bodies (ExecutableMultiInstanceBody): the inner activity, isSequential, the
  // inputElement's name id (NONE: none), the loopCounter name id, the static inputCollection
  // (zbhip_doc_type, value; strings as value-dictionary ids)
  struct Mi {
    uint16_t body, inner;
    bool seq;
    uint16_t input_name, loop_name;
    std::vector<std::pair<uint8_t, int64_t>> items;
    // the inputCollection variable (ZBHIP_OP_COLLECTION; NONE: the static items), the outputCollection
    // and outputElement names (ZBHIP_OP_OUTPUT), the completionCondition's condition index (-1 none),
    // the name ids of numberOfInstances / ActiveInstances / CompletedInstances / TerminatedInstances
    // (NONE: the condition does not read it)
    uint16_t coll_name = NONE, out_coll = NONE, out_elem = NONE;
    int32_t cond = -1;
    uint32_t static_list = 0xFFFFFFFFu;  // the static items as a list (a body with collection words)
    uint16_t n_names[4] = {NONE, NONE, NONE, NONE};
    // the outputElement is a local nil-initialized variable of the inner instance (not the inputElement
    // or loopCounter: setLoopVariables :283-300)
    bool out_local() const { return out_elem != NONE && out_elem != input_name && out_elem != loop_name; }
    bool ext() const { return coll_name != NONE || out_coll != NONE || cond >= 0; }
  };
  std::vector<Mi> mi;
  std::vector<int16_t> mi_of;  // per element: its body's index in `mi` (the body and its inner activity), -1
  const Mi* mi_body(uint32_t e) const { return e < mi_of.size() && mi_of[e] >= 0 ? &mi[mi_of[e]] : nullptr; }
  // the body around inner activity e (nullptr: e is not an inner activity)
  const Mi* mi_inner(uint32_t e) const {
    const Mi* m = mi_body(e);
    return m && m->inner == e ? m : nullptr;
  }
  const std::string& id(uint32_t e) const { return strings[els[e].id]; }
  // zeebe:ioMapping per element ([0] input, [1] output; kernels.hip io_map): type kIoNone, ZBHIP_MAP_VARIABLE
  // (src = the source variable's name id) or a literal's zbhip_doc_type (STR: value-dictionary id in lit)
  struct Io {
    uint8_t type = 0xFE;
    uint16_t src = NONE, tgt = NONE;
    int64_t lit = 0;
  };
  std::vector<std::array<Io, 2>> io;
  bool has_io = false;
  bool io_of(uint32_t e) const { return has_io && e < io.size() && (io[e][0].type != 0xFE || io[e][1].type != 0xFE); }
};
constexpr uint8_t kIoNone = 0xFE;
// device limit of a multi-instance body: loop counters live in 6 bits of the inner instance's slot
// (kernels.hip apply_activating_child), children in 8 bits of the body's
constexpr size_t kMaxMiItems = 63;

// Host threads a bulk host pass may use: the CPUs this process may run on (affinity mask, which
// honours taskset / cgroup cpusets), at most 16.
// CPUs this process may keep busy: its affinity set, its cgroup's CPU quota (cpu.max, v2; cfs
// quota / period, v1) -- a busy pool past the quota is throttled by the kernel for the rest of the
// 100 ms period, which showed as 10-45 ms stalls of single windows -- at most 16, or
// ZBHIP_HOST_THREADS.  One CPU of a quota is left to the calling thread and the runtime's own.
static unsigned detect_host_threads() {
  if (const char* e = getenv("ZBHIP_HOST_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return (unsigned)std::min(v, 64);
  }
  cpu_set_t set;
  CPU_ZERO(&set);
  int n = sched_getaffinity(0, sizeof set, &set) == 0 ? CPU_COUNT(&set) : (int)std::thread::hardware_concurrency();
  double quota = 0;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) quota = atof(q) / (double)period;
    fclose(f);
  } else if (FILE* fq = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    long long q = -1, period = 0;
    if (fscanf(fq, "%lld", &q) != 1) q = -1;
    fclose(fq);
    if (FILE* fp = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (fscanf(fp, "%lld", &period) != 1) period = 0;
      fclose(fp);
    }
    if (q > 0 && period > 0) quota = (double)q / (double)period;
  }
  if (quota > 0) n = std::min(n, std::max(1, (int)quota - 1));
  return (unsigned)std::max(1, std::min(16, n));
}
unsigned host_threads() {
  static const unsigned n = detect_host_threads();
  return n;
}

// A process-wide pool of host worker threads, started once (thread creation cost ~0.3 ms per
// 16-thread fork/join, several times per window on the log-byte path).  One job at a time: a call
// that finds the pool busy (another handle's call on another thread) forks its own threads.
// set on the pool's workers and on a caller's own share while a pool job runs: a parallel_for
// nested inside a job runs serially instead of touching the pool (whose busy mutex that thread may
// already own)
static thread_local bool tl_in_pool_job = false;

class WorkerPool {
 public:
  static WorkerPool& get() {
    static WorkerPool p;
    return p;
  }
  // runs job(t, T) for t in [1, T) on the workers (T - 1 <= workers()); false when busy
  bool run(unsigned T, const std::function<void(unsigned, unsigned)>& job, const std::function<void()>& own) {
    std::unique_lock<std::mutex> busy(busy_, std::try_to_lock);
    if (!busy.owns_lock() || T - 1 > workers_.size()) return false;
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &job;
      T_ = T;
      remaining_ = T - 1;
      ++gen_;
    }
    cv_.notify_all();
    tl_in_pool_job = true;
    own();
    tl_in_pool_job = false;
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return remaining_ == 0; });
    job_ = nullptr;
    return true;
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  WorkerPool() {
    const unsigned n = host_threads();
    for (unsigned i = 1; i < n; ++i) {
      try {
        workers_.emplace_back([this, i] { loop(i); });
      } catch (...) {
        break;
      }
    }
  }
  void loop(unsigned idx) {
    tl_in_pool_job = true;
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(unsigned, unsigned)>* job;
      unsigned T;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
        T = T_;
      }
      if (idx < T) {
        (*job)(idx, T);
        std::lock_guard<std::mutex> g(m_);
        if (--remaining_ == 0) done_.notify_one();
      }
    }
  }
  std::mutex busy_, m_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> workers_;
  const std::function<void(unsigned, unsigned)>* job_ = nullptr;
  unsigned T_ = 0, remaining_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// fn(t, T) for t in [0, T) on up to T threads (the pool's, else threads of its own); a thread that
// cannot be started runs its share on the calling thread (no exception leaves the C ABI, no
// joinable thread is destroyed)
template <class F>
void parallel_for(unsigned T, const F& fn) {
  if (T <= 1 || tl_in_pool_job) {
    for (unsigned t = 0; t < std::max(T, 1u); ++t) fn(t, std::max(T, 1u));
    return;
  }
  const std::function<void(unsigned, unsigned)> job = [&fn](unsigned t, unsigned TT) { fn(t, TT); };
  if (WorkerPool::get().run(T, job, [&] { fn(0u, T); })) return;
  std::vector<std::thread> pool;
  pool.reserve(T);
  unsigned t = 1;
  for (; t < T; ++t) {
    try {
      pool.emplace_back(fn, t, T);
    } catch (...) {
      break;
    }
  }
  for (unsigned u = t; u < T; ++u) fn(u, T);
  fn(0u, T);
  for (auto& th : pool) th.join();
}

// Java String#hashCode over signed bytes (SubscriptionUtil.getSubscriptionHashCode, :22-30)
int32_t java_hash(const char* b, size_t n) {
  uint32_t h = 0;
  for (size_t i = 0; i < n; ++i) h = 31u * h + (uint32_t)(int32_t)(int8_t)b[i];
  return (int32_t)h;
}

struct BatchRef {
  int64_t base;  // first generated key counter value (key = (p << 51) + base + i)
  uint32_t inst;
  uint16_t first_ord;
  uint16_t nkeys;
  uint32_t gen;  // generation of the subject when the keys were generated (inst_gen)
  // not zero-filled when a window's segment of 10^6 entries is allocated (every entry is written)
  BatchRef() {}
  BatchRef(int64_t b, uint32_t i, uint16_t f, uint16_t n, uint32_t g) : base(b), inst(i), first_ord(f), nkeys(n), gen(g) {}
};

// A std::vector-like buffer in pinned host memory: the window's commands are uploaded from it by
// DMA, without the driver's synchronous staging of a pageable source.  (Trivially copyable T; grows
// by reallocation, new elements zeroed as std::vector value-initialises them.)
template <class T>
struct PinnedVec {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  PinnedVec() = default;
  PinnedVec(const PinnedVec&) = delete;
  PinnedVec& operator=(const PinnedVec&) = delete;
  ~PinnedVec() {
    if (p) (void)hipHostFree(p);
  }
  void reserve(size_t c) {
    if (c <= cap) return;
    const size_t nc = std::max(c, cap * 2);
    T* q = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&q), nc * sizeof(T), hipHostMallocDefault) != hipSuccess) throw std::bad_alloc();
    if (n) memcpy(q, p, n * sizeof(T));
    if (p) (void)hipHostFree(p);
    p = q;
    cap = nc;
  }
  void resize(size_t m) {
    reserve(m);
    if (m > n) memset(static_cast<void*>(p + n), 0, (m - n) * sizeof(T));
    n = m;
  }
  void clear() { n = 0; }
  template <class It>
  void insert(T* at, It first, It last) {  // (appending only)
    const size_t k = (size_t)std::distance(first, last);
    (void)at;
    reserve(n + k);
    std::copy(first, last, p + n);
    n += k;
  }
  T* data() { return p; }
  const T* data() const { return p; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  T* begin() { return p; }
  T* end() { return p + n; }
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  void swap(PinnedVec& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
  }
};

// The resolve_key table: BatchRefs in key order, in segments (one per plain window, or appended
// entries), so appending 10^6 entries never moves the older ones and a compaction runs segment by
// segment on host threads.  Lookup: the segment by its first key, then within it.
struct KeyTable {
  std::vector<std::vector<BatchRef>> seg;
  size_t count = 0;
  size_t size() const { return count; }
  // a new segment of n entries, filled by the caller (indexes 0 .. n-1, from any thread)
  // emptied segments' buffers, reused by the next windows (freeing and re-faulting 24 MB per
  // window cost milliseconds of page-table work on the bookkeeping's critical path)
  std::vector<std::vector<BatchRef>> spare;
  BatchRef* append_segment(size_t n) {
    if (n == 0) return nullptr;
    size_t best = spare.size();
    for (size_t i = 0; i < spare.size(); ++i)
      if (spare[i].capacity() >= n && (best == spare.size() || spare[i].capacity() < spare[best].capacity())) best = i;
    if (best < spare.size()) {
      seg.push_back(std::move(spare[best]));
      spare.erase(spare.begin() + best);
      seg.back().resize(n);
    } else {
      seg.emplace_back(n);
    }
    count += n;
    return seg.back().data();
  }
  void push_back(const BatchRef& b) {
    if (seg.empty() || seg.back().size() >= (1u << 20)) {
      seg.emplace_back();
      seg.back().reserve(1024);
    }
    seg.back().push_back(b);
    ++count;
  }
  const BatchRef* find(int64_t v) const {  // the last entry with base <= v
    auto s = std::upper_bound(seg.begin(), seg.end(), v,
                              [](int64_t x, const std::vector<BatchRef>& g) { return x < g.front().base; });
    if (s == seg.begin()) return nullptr;
    --s;
    auto it = std::upper_bound(s->begin(), s->end(), v, [](int64_t x, const BatchRef& b) { return x < b.base; });
    return it == s->begin() ? nullptr : &*(it - 1);
  }
  // in 64 Ki-entry chunks over the host threads (whole segments per thread left one thread with two
  // 10^6-entry segments: 36 ms stalls every ~11 windows), then each segment's kept runs closed up
  template <class Live>
  void compact(const Live& live) {
    constexpr size_t kChunk = size_t(1) << 16;
    std::vector<std::pair<uint32_t, size_t>> chunks;  // (segment, first entry)
    std::vector<size_t> seg_chunk(seg.size() + 1, 0);
    for (size_t i = 0; i < seg.size(); ++i) {
      seg_chunk[i] = chunks.size();
      for (size_t b = 0; b < seg[i].size(); b += kChunk) chunks.emplace_back((uint32_t)i, b);
    }
    seg_chunk[seg.size()] = chunks.size();
    std::vector<size_t> kept(chunks.size(), 0);
    parallel_for(host_threads(), [&](unsigned t, unsigned T) {
      for (size_t k = t; k < chunks.size(); k += T) {
        std::vector<BatchRef>& g = seg[chunks[k].first];
        const size_t b = chunks[k].second, e = std::min(b + kChunk, g.size());
        size_t o = b;
        for (size_t x = b; x < e; ++x)
          if (live(g[x])) g[o++] = g[x];
        kept[k] = o - b;
      }
    });
    parallel_for(host_threads(), [&](unsigned t, unsigned T) {
      for (size_t i = t; i < seg.size(); i += T) {
        std::vector<BatchRef>& g = seg[i];
        size_t o = 0;
        for (size_t k = seg_chunk[i]; k < seg_chunk[i + 1]; ++k) {
          if (o != chunks[k].second && kept[k]) memmove(&g[o], &g[chunks[k].second], kept[k] * sizeof(BatchRef));
          o += kept[k];
        }
        g.resize(o);
      }
    });
    std::vector<std::vector<BatchRef>> keep;
    keep.reserve(seg.size());
    for (auto& g : seg) {
      if (!g.empty()) keep.push_back(std::move(g));
      else spare.push_back(std::move(g));
    }
    trim_spare();
    seg.swap(keep);
    count = 0;
    for (auto& g : seg) count += g.size();
  }
  // spare buffers are kept up to twice the largest live segment's capacity in total (a window or
  // two), largest first: a table that shrank gives its memory back
  void trim_spare() {
    size_t live = 0;
    for (auto& g : seg) live = std::max(live, g.capacity());
    std::sort(spare.begin(), spare.end(),
              [](const std::vector<BatchRef>& a, const std::vector<BatchRef>& b) { return a.capacity() > b.capacity(); });
    size_t kept = 0, total = 0;
    while (kept < spare.size() && kept < 4 && total + spare[kept].capacity() <= 2 * std::max<size_t>(live, 1u << 16)) {
      total += spare[kept].capacity();
      ++kept;
    }
    spare.resize(kept);
  }
  void sort_all() {  // (imports: one segment again)
    std::vector<BatchRef> all;
    all.reserve(count);
    for (auto& g : seg) all.insert(all.end(), g.begin(), g.end());
    std::sort(all.begin(), all.end(), [](const BatchRef& a, const BatchRef& b) { return a.base < b.base; });
    seg.clear();
    if (!all.empty()) seg.push_back(std::move(all));
  }
};

const char* state_name(int s) {
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

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) return hipSuccess;
  return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
}

}  // namespace

struct zbhip_handle {
  zbhip_config cfg{};
  zbhip_serializer* ser = nullptr;  // log serialiser, kept in step with deploy / intern (logwriter.cpp)
  hipStream_t stream = nullptr;
  bool own_stream = false;

  std::vector<Proc> procs;
  std::vector<uint32_t> prog;
  uint32_t* d_prog = nullptr;
  size_t d_prog_cap = 0;
  uint2* d_tpl = nullptr;        // CREATE batch templates [procs][kTplVar][kTplWords] (kernels.hip)
  size_t tpl_procs = 0;          // processes the template table holds
  uint32_t launch_seq = 0;       // k_step launches so far (StepParams.launch_seq)

  std::vector<std::string> names;
  std::unordered_map<std::string, uint32_t> name_ids;

  DevState st{};
  uint4* d_cmds = nullptr;
  zbhip_doc_entry* d_docs = nullptr;
  uint32_t* d_order = nullptr;
  bool order_on_device = false;  // h_order is d_order's (a device window sorted by subject): copied on use
  uint32_t* d_sort = nullptr;    // [3][max_commands] subject keys in / out, indices in
  void* d_sort_temp = nullptr;
  size_t sort_temp_bytes = 0;
  uint2* d_rec = nullptr;
  uint2* d_cmd_hdr = nullptr;
  uint2* d_regions = nullptr;                // [regions][128 * rec_cap] per-workgroup record regions
  uint32_t* d_region_total = nullptr;        // [regions]
  uint16_t* d_region_lanes = nullptr;        // [regions][128] lane record counts (regions with rows j >= R)
  unsigned long long* d_region_off = nullptr;// [regions] (drain path)
  unsigned long long* d_stats = nullptr;     // [64][8] spread accumulators + [512] gather total
  uint32_t regions_cap = 0;
  size_t region_records = 0;
  uint32_t region_pad = 0;  // records between consecutive regions (region stride B * rec_cap + pad)
  int variant = 3;                           // kernel variant (zbhip_deploy): 3 KLinear, 0 KSimple, 1 KGeneric, 2 KMsg, 4 KScope
  // launches of the last run: region base, lane count, and the window index of each lane (the
  // main window's rounds: identity or h_order; continuation batches: cont_order)
  struct Launch {
    uint32_t region, first, count;
    uint8_t src;  // 0 identity, 1 h_order[first + k], 2 cont_order[first + k]
  };
  std::vector<Launch> launches;
  // follow-up commands written to the log past maxCommandsInBatch, read back as batches of their own
  // after the window (kernels.hip overflow / CMD_FOLLOWUP)
  bool may_overflow = false;           // a deployed process can exceed the batch limit (deploy-time bound)
  uint32_t max_pending = 0;            // deploy-time bound of pending follow-ups in one batch
  uint4* d_ovf = nullptr;
  uint32_t* d_ovf_count = nullptr;
  uint32_t ovf_cap = 0;                // overflow entries per run (a batch past it falls back: FB_BATCH_LIMIT)
  zbhip_command* d_cont = nullptr;     // continuation commands (window indices n ..)
  uint32_t* d_cont_order = nullptr;
  std::vector<zbhip_command> cont_cmds;
  std::vector<uint32_t> cont_order;
  // ZBHIP_OPEN_DEFER_CONTINUATIONS: a follow-up written unprocessed is not run after the window; it
  // waits here (id -> its CMD_FOLLOWUP command) until the log reader submits it (ZBHIP_CMD_CONTINUE)
  // at its own log position.  Ids follow the drain order of the unprocessed records.
  std::unordered_map<uint64_t, zbhip_command> deferred;
  std::unordered_map<uint32_t, uint32_t> deferred_per_inst;  // pending continuations per instance slot
  uint64_t next_cont_id = 1;
  uint64_t last_cont_first = 0, last_cont_n = 0;             // ids the last run deferred
  std::unordered_map<uint64_t, uint64_t> cont_ids;           // (window command << 16 | record ordinal) -> id
  bool window_continues = false;                             // the window runs deferred continuations
  bool defer() const { return cfg.flags & ZBHIP_OPEN_DEFER_CONTINUATIONS; }
  uint32_t* d_qspill = nullptr;        // batch FIFO entries beyond the LDS ring (kernels.hip enqueue)
  size_t qspill_words = 0;
  uint32_t qspill_cap = 0;
  std::vector<hipEvent_t> tev;               // timing events (pairs) since the last stats reset
  size_t tev_used = 0;
  uint32_t rec_cap = 64;
  size_t rec_slots = 0;  // commands the record buffer is sized for

  // current window
  bool external = false;
  const uint4* ext_cmds = nullptr;
  const zbhip_doc_entry* ext_docs = nullptr;
  PinnedVec<zbhip_command> h_cmds;  // (pinned: the upload source of host windows)
  PinnedVec<zbhip_command> h_cmds_next;  // the next window's, validated and copied in one pass
  hipEvent_t upload_ev = nullptr;        // recorded after a submit's uploads (h_cmds, h_docs, h_xparts,
                                         // h_order): the next submit waits on it before rewriting them
  std::vector<zbhip_doc_entry> h_docs;
  size_t n_cmds = 0, n_docs = 0;
  std::vector<uint32_t> round_begin;
  std::vector<uint32_t> h_order;
  int64_t doc_base = 0, next_doc_base = 0;
  int64_t source_base = 0, next_source = 0;
  bool ran = false;

  // results of the last run
  std::vector<uint2> h_hdr;
  std::vector<uint2> h_out;
  std::vector<uint64_t> h_off;  // record offset of each command in h_out
  bool off_ready = false;       // h_off is the last run's (compute_offsets)
  size_t out_total = 0;         // records of the last run (in d_rec; in h_out once out_host)
  bool out_host = false;
  size_t drain_cmd = 0, drain_rec = 0, drain_ord = 0;
  bool results = false;

  // key relabelling (DbKeyGenerator order)
  int64_t key_counter = 0;
  int64_t clock_ms = 0;       // zbhip_set_clock: the clock of the next runs (timer due dates)
  int64_t run_clock_ms = 0;   // the clock of the last run (drained TIMER:CREATED dueDates)
  bool relabel_ok = true;
  size_t fin_next = 0;             // the last run's key bookkeeping is done for commands < fin_next (advance)
  std::vector<uint32_t> ext_keys;  // keys the CPU engine generated for the window's fallback commands
  bool ext_ready = false;          // ext_keys / declared are the last run's (ensure_ext)
  unsigned long long fb_seen = 0;           // fallbacks counted in the statistics rows so far
  unsigned long long window_fallbacks = 0;  // ... in the last run
  std::vector<uint8_t> declared;   // ... declared by the adapter (zbhip_set_external_keys)
  // plan_rounds: (stamp, last round) per subject; window of the last command per instance slot
  std::vector<std::pair<uint32_t, uint32_t>> plan_last;
  uint32_t plan_stamp = 0;
  std::vector<uint32_t> plan_seen;
  std::vector<uint32_t> plan_round;  // round of each command of the window being planned
  uint32_t plan_window = 0;
  // fence stamps of the device windows (StepParams.stamp; hdr.w / slot_hdr.y of a fallen-back subject)
  uint32_t window_stamp = 0;
  // device-window subject check (k_subject_check)
  uint32_t* d_seen = nullptr;
  uint32_t* d_check_flag = nullptr;
  uint32_t check_stamp = 0;
  // speculative subject check of an untrusted device window (no host read before its launch): the
  // check's flag travels to pinned memory behind an event; k_step launches guarded by it, and the next
  // host call that depends on the window (resolve_guard) reads the flag -- a repeat replans and reruns
  struct GuardedWindow {
    const zbhip_command* cmds;
    size_t n;
    const zbhip_doc_entry* docs;
    size_t n_docs;
    const zbhip_xpart_cmd* xparts;
    size_t n_xparts;
    int64_t doc_base, source_base;  // the handle's counters before the window (rolled back on a replay)
    uint32_t run_flags;
  } guard_win{};
  bool guard_armed = false;    // submitted with a speculative check, not run yet
  bool guard_pending = false;  // run guarded, flag not read yet
  uint32_t* h_check_flag = nullptr;  // host-mapped: the last check's completion marker (stamp << 2 | flags)
  uint32_t* d_check_host = nullptr;  // its device address
  uint32_t guard_stamp = 0;          // the stamp of the checked window
  // resolve_key: the generation of every subject (bumped when an instance is created or ends, so
  // keys of an earlier instance in a reused slot never resolve); stale entries are compacted away
  std::vector<uint32_t> inst_gen;
  size_t batches_compacted = 0;
  std::atomic<size_t> batches_dead{0};  // entries of ended instances since the last compaction
  std::vector<std::vector<std::pair<uint16_t, int64_t>>> hist;
  std::vector<uint16_t> inst_proc;
  KeyTable batches;
  // Windows whose key bookkeeping stayed on the device (zbhip_serialize_log_device over a
  // device-built command table): k_table_build journals each command's first key, ordinal, key
  // count, instance, end and CREATE process in HBM (16 B per command), and the host tables above are
  // brought up to date from the journal (fold_journal) only when a host consumer reads them -- a
  // drain, resolve_key, an export, job activation, a host-built window -- or the journal is full.
  struct JournalWindow {
    uint32_t slot;
    size_t n;
    uint64_t window;  // windows_run of the window
  };
  uint4* d_jrn = nullptr;
  uint32_t jrn_slots = 0;
  uint32_t jrn_next = 0;
  std::deque<JournalWindow> jrn_q;
  std::vector<uint4> jrn_host;

  // ---- log bytes on the device (zbhip_serialize_log_device, logdev.hip) ----
  uint8_t* d_log_arena = nullptr;   // the serialiser's constant byte runs
  uint32_t* d_log_idx = nullptr;
  size_t log_arena_cap = 0, log_idx_cap = 0;
  size_t log_tables_procs = ~(size_t)0, log_tables_names = ~(size_t)0;
  uint32_t log_arena_words = 0, log_idx_words = 0;
  uint8_t* d_log_tpl = nullptr;     // entry templates | their descriptors (16-aligned) | the index
  size_t log_tpl_cap = 0, log_tpl_desc_off = 0, log_tpl_idx_off = 0;
  unsigned long long* d_ring = nullptr;  // [16][max_instances] key ring + [max_instances] PI keys
  uint16_t* d_inst_proc = nullptr;
  LogCmd* d_logcmd = nullptr;
  unsigned long long* d_log_bytes = nullptr;  // [max_commands + 1 + scan blocks]
  long long* d_src_pos = nullptr;             // [max_commands] source positions (device-built command table)
  std::vector<uint16_t> inst_proc_stage;      // inst_proc as uploaded for that table
  uint16_t* inst_proc_pin = nullptr;          // pinned staging of the device-table path's uploads
  size_t inst_proc_pin_cap = 0;
  long long* src_pos_pin = nullptr;
  size_t src_pos_pin_cap = 0;
  unsigned long long* d_tbl_sums = nullptr;   // scan blocks of the device-built command table
  uint64_t* d_log_out = nullptr;
  size_t log_out_cap = 0;
  // zbhip_log_copy_async: two device output buffers used in turn (window k's bytes stay put while they
  // cross PCIe and window k+1 is written into the other one) and two pinned host buffers, the copies on a
  // stream of their own ordered after the write by events
  struct LogBuf {
    uint64_t* dev = nullptr;
    size_t dev_cap = 0;
    char* host = nullptr;
    size_t host_cap = 0;
    hipEvent_t written = nullptr, copied = nullptr;
    bool pending = false;  // a copy out of this buffer was queued and not yet waited for
  } log_bufs[2];
  int log_cur = 0;
  bool log_double = false;
  hipStream_t copy_stream = nullptr;
  uint32_t* d_log_flag = nullptr;
  uint32_t* d_log_rinfo = nullptr;  // [rows] per record: template / composed, entry bytes
  LogKeys* d_log_wkeys = nullptr;   // [max_commands] older keys per command (size pass -> write pass)
  std::vector<LogCmd> h_logcmd;
  std::vector<uint64_t> log_prev;   // per instance: window | last command of the window (prev chain)
  uint64_t windows_run = 0;         // zbhip_run calls
  uint64_t ring_filled = 0;         // windows whose keys are in the ring (all of them, or the path is off)
  bool ring_ok = true;              // false once a window's keys missed the ring (or state was imported)

  // ---- job activation (zbhip_activate_jobs) ----
  // JOB_ACTIVATABLE of the GPU-resident jobs, [type, job key] -> (instance, job key ordinal): built
  // from the device rows at the first activation, then kept by the key bookkeeping (advance)
  bool job_index_on = false;
  std::map<std::pair<uint32_t, int64_t>, std::pair<uint32_t, uint16_t>> job_index;
  std::unordered_map<std::string, uint32_t> job_type_ids;
  // A job whose stored JobRecord differs from the one JOB:CREATED wrote (slot flag bit 1 on the device):
  // the deadline and worker DbJobState.activate stored, kept when the job timed out
  // (DbJobState.timeout :142-150), and its JOB_STATES value.
  enum : uint8_t { JS_ACTIVATED = 0, JS_ACTIVATABLE = 1, JS_GONE = 2, JS_FAILED = 3 };  // (GONE: completed / canceled)
  struct Activation {
    int64_t deadline;
    std::string worker;
    uint32_t inst;
    uint32_t worker_id;  // the worker in the value dictionary (ZBHIP_NO_STRING: empty)
    uint8_t state = JS_ACTIVATED;
    int64_t eik = -1, pik = -1;  // the job's element instance and process instance
    int32_t proc = -1, elem = -1;
    // JobFailProcessor.failJob stored them (zbhip_fail_job): retries and errorMessage from then on
    bool fail_fields = false;
    int32_t retries = 0;
    uint32_t error_id = ZBHIP_NO_STRING;  // the errorMessage in the value dictionary
    int64_t incident_key = -1;            // its JOB_NO_RETRIES incident (INCIDENTS, INCIDENT_JOBS)
    uint32_t incident_msg_id = ZBHIP_NO_STRING;
  };
  std::unordered_map<int64_t, Activation> activated;  // jobs with a stored activation: deadline, worker, state
  // job streams (JobStreamer.streamFor: a gateway's StreamActivatedJobs), by job type id: the jobs a
  // device batch creates of such a type are pushed (BpmnJobActivationBehavior.publishWork)
  struct Stream {
    std::string worker;
    uint32_t worker_id;
    int64_t timeout;
  };
  std::map<uint32_t, Stream> streams;
  std::map<uint32_t, Stream> run_streams;  // the streams of the last run (its pushes' deadlines / workers)
  DueTimer* d_due = nullptr;                          // zbhip_due_timers: [max_instances] due rows
  uint32_t* d_due_count = nullptr;
  unsigned long long* d_due_next = nullptr;
  std::vector<int64_t> completed_activated;           // completed in the last window (dropped next)
  uint32_t job_type(const std::string& t) {
    auto it = job_type_ids.find(t);
    if (it != job_type_ids.end()) return it->second;
    const uint32_t id = (uint32_t)job_type_ids.size();
    job_type_ids.emplace(t, id);
    return id;
  }

  // ---- the list dictionary (ZBHIP_DOC_LIST values: multi-instance inputCollection variables and
  // outputCollections), deduplicated; its items on the device (d_list_*: uploaded before a run) ----
  using Items = std::vector<std::pair<uint8_t, int64_t>>;
  std::vector<Items> lists;
  std::map<Items, uint32_t> list_ids;
  std::vector<uint2> list_hdr;      // per list: first item, item count
  std::vector<long long> list_val;  // the items' values, then their zbhip_doc_types
  std::vector<uint8_t> list_type;
  uint2* d_list_hdr = nullptr;
  long long* d_list_val = nullptr;
  uint8_t* d_list_type = nullptr;
  size_t d_list_n = 0, d_list_items = 0, d_list_cap = 0, d_litem_cap = 0;
  // multi-instance output collections (host-side: the device keeps no array): per body element
  // instance the collection variable's key and items (track_mi, from the drained records); the list
  // ids of propagated collections (variables of type kDocOutList on the device), by variable key;
  // the inline values of the window's multi-instance records, by (command, ordinal)
  struct MiOut {
    int64_t var_key;
    Items items;
  };
  std::unordered_map<int64_t, MiOut> mi_out;
  std::unordered_map<int64_t, uint32_t> outlist_var;
  struct MiRec {
    int64_t key, scope;
    int32_t name;
    uint8_t intent, type;
    int64_t value;
  };
  std::unordered_map<uint64_t, MiRec> mi_rec;
  bool mi_ext = false;  // a deployed process has a multi-instance collection variable / output / condition

  // ---- message correlation (variant 2) ----
  std::vector<std::string> strs;               // value dictionary
  std::unordered_map<std::string, uint32_t> str_ids;
  std::vector<uint32_t> str_hash;
  uint32_t* d_str_hash = nullptr;
  size_t d_str_cap = 0, d_str_n = 0;
  zbhip_xpart_cmd* d_xparts = nullptr;         // host-submitted window xparts
  const zbhip_xpart_cmd* ext_xparts = nullptr;
  std::vector<zbhip_xpart_cmd> h_xparts;
  size_t n_xparts = 0;
  uint4* d_cmd_hdr2 = nullptr;
  long long* d_cmd_due = nullptr;       // (KScope) dueDate of the timer each batch canceled
  long long* d_map_val = nullptr;       // (KScope) io-mapped variable values per batch (StepParams.map_val)
  uint4* d_cmd_act = nullptr;           // the ACTIVATED job each batch completed / canceled (StepParams.cmd_act)
  uint8_t* d_strs = nullptr;            // the value dictionary on the device (the log writer's workers)
  unsigned long long* d_str_off = nullptr;
  size_t d_strs_n = 0, d_strs_cap = 0, d_str_off_cap = 0;
  std::vector<long long> h_map_val;
  bool debug = getenv("ZBHIP_DEBUG") != nullptr;  // per-call host timing lines on stderr
  std::vector<long long> h_cmd_due;
  zbhip_xpart_cmd* d_xout = nullptr;
  zbhip_xpart_cmd* d_xbucket = nullptr;
  uint32_t* d_blk_cnt = nullptr;
  uint32_t* d_xcount = nullptr;
  unsigned long long* d_key_counter = nullptr;
  unsigned long long* d_key_base = nullptr;
  unsigned long long* d_key_blk = nullptr;
  bool bucketed = false;
  bool outbox_taken = false;  // zbhip_outbox_device already handed out the last run's outbox
  uint64_t xout_host_run = ~0ull;  // windows_run of the outbox copy in h_xout (zbhip_outbox_command)
  bool published = false;                      // a publish ran: MESSAGE_STATS row exists
  std::vector<uint4> h_hdr2;
  std::vector<int64_t> h_base;                 // key counter before each command's first key
  std::vector<zbhip_xpart_cmd> h_xout;
  bool msg() const { return variant == 2; }
  bool scope_variant() const { return variant == 4 || variant == 5; }  // KScope / KScopeIO

  zbhip_stats stats{};
  bool stats_dirty = false;
  uint32_t n_regions = 0;
  unsigned long long key_counter_approx = 0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};

  // subjects of the key history: instance slots [0, n), correlation slots [n, n + S)
  uint32_t slot_subject(uint32_t slot) const { return cfg.max_instances + slot; }
  // a key reference of a payload row / row (zb_internal.h) -> the reference's key
  long long resolve_ref(long long ref) const {
    if (ref >= -1) return ref;
    const unsigned long long v = (unsigned long long)(-2 - ref);
    const uint32_t ord = v & 0xFFFF;
    if ((v >> 62) & 1) {
      const bool is_slot = (v >> 61) & 1;
      const uint32_t subj = (uint32_t)((v >> 16) & 0xFFFFFFFFull);
      return key_of(is_slot ? slot_subject(subj) : subj, ord);
    }
    const uint32_t c = (uint32_t)(v >> 17), sec = (v >> 16) & 1;
    if (c >= h_base.size() || c >= h_hdr.size()) return -1;
    const uint32_t nsec = h_hdr2[c].y >> 16, nprim = (h_hdr[c].x >> 16) - nsec;
    const uint32_t off = sec ? nprim + (uint16_t)(ord - (h_hdr2[c].y & 0xFFFF)) : (uint16_t)(ord - (h_hdr[c].y & 0xFFFF));
    return ((int64_t)cfg.partition_id << 51) + h_base[c] + 1 + off;
  }

  long long key_of(uint32_t inst, uint32_t ord) const {
    if (ord == NONE || inst >= hist.size()) return -1;
    const auto& h = hist[inst];
    for (size_t i = h.size(); i-- > 0;)
      if (h[i].first <= ord) return ((int64_t)cfg.partition_id << 51) + h[i].second + (ord - h[i].first);
    return -1;
  }
};

#define HIPCHK(x)                                                                                \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      if (getenv("ZBHIP_DEBUG")) fprintf(stderr, "[zbhip] %s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return ZBHIP_EDEVICE;                                                                      \
    }                                                                                            \
  } while (0)

static int finalize(zbhip_handle* h);
static int settle(zbhip_handle* h);
static int log_next_buffer(zbhip_handle* h);
static int resolve_guard(zbhip_handle* h);
static int64_t intern_items(zbhip_handle* h, const zbhip_handle::Items& v);
static int sync_lists(zbhip_handle* h);

extern "C" {

const char* zbhip_build_info(void) {
  return "libzbhip gfx950 (HIP) k_step/k_block_sums/k_scan_sums/k_compact, ABI " "1";
}

int zbhip_open(const zbhip_config* cfg, zbhip_handle** out) {
  if (!cfg || !out || cfg->max_instances == 0 || cfg->max_commands == 0 || cfg->partition_id < 0 ||
      cfg->max_instances >= 0xFFFFFFF0u)
    return ZBHIP_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg->device) return ZBHIP_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) return ZBHIP_ENODEV;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ZBHIP_ENODEV;
  HIPCHK(hipSetDevice(cfg->device));
  auto* h = new zbhip_handle();
  h->cfg = *cfg;
  zbhip_serializer_new(&h->ser);
  if (h->cfg.max_commands_in_batch <= 0) h->cfg.max_commands_in_batch = 100;
  if (h->cfg.max_doc_entries == 0) h->cfg.max_doc_entries = cfg->max_commands;
  h->rec_cap = cfg->max_records_per_batch ? cfg->max_records_per_batch : 64;
  if (h->rec_cap > 0xFFFF) { delete h; return ZBHIP_EINVAL; }
  h->key_counter = cfg->initial_key;
  if (cfg->stream) {
    h->stream = reinterpret_cast<hipStream_t>(cfg->stream);
  } else {
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) { delete h; return ZBHIP_EDEVICE; }
    h->own_stream = true;
  }
  const size_t N = cfg->max_instances;
  h->st.n = (uint32_t)N;
  bool ok = dalloc(&h->st.hdr, N) == hipSuccess && dalloc(&h->st.slots, N * kSlots) == hipSuccess &&
            dalloc(&h->st.var_meta, N * kVars) == hipSuccess && dalloc(&h->st.var_val, N * kVars) == hipSuccess &&
            dalloc(&h->st.join, N * kJoinWords) == hipSuccess &&
            dalloc(&h->d_cmds, cfg->max_commands) == hipSuccess &&
            dalloc(&h->d_docs, h->cfg.max_doc_entries) == hipSuccess &&
            dalloc(&h->d_order, cfg->max_commands) == hipSuccess &&
            dalloc(&h->d_cmd_hdr, cfg->max_commands) == hipSuccess &&
            dalloc(&h->d_stats, 64 * 8 + 8) == hipSuccess &&
            dalloc(&h->d_rec, ((size_t)cfg->max_commands + 64) * h->rec_cap) == hipSuccess;
  // region pool: every workgroup of a run owns (workgroup size) * rec_cap records; sized for a
  // full window plus kExtraRegions partly filled workgroups of extra rounds (<= 256 lanes each)
  h->regions_cap = (cfg->max_commands + 63) / 64 + kExtraRegions;
  {
    const char* e = getenv("ZBHIP_REGION_PAD");
    h->region_pad = e ? (uint32_t)atoi(e) : kRegionPad;
  }
  h->region_records = ((size_t)cfg->max_commands + (size_t)kExtraRegions * 256) * h->rec_cap +
                      (size_t)h->regions_cap * h->region_pad;
  ok = ok && dalloc(&h->d_regions, h->region_records) == hipSuccess &&
       dalloc(&h->d_region_total, h->regions_cap) == hipSuccess &&
       dalloc(&h->d_region_lanes, (size_t)h->regions_cap * 128) == hipSuccess &&
       dalloc(&h->d_region_off, h->regions_cap) == hipSuccess;
  // timer rows (KScope timer catch events): one per instance
  ok = ok && dalloc(&h->st.tmr, N) == hipSuccess && dalloc(&h->d_cmd_due, cfg->max_commands) == hipSuccess &&
       dalloc(&h->d_map_val, (size_t)kMapVals * cfg->max_commands) == hipSuccess;
  // message correlation state (config 5): PROCESS_SUBSCRIPTION rows per instance, correlation slots
  const size_t S = cfg->max_correlation_keys;
  h->st.n_slots = (uint32_t)S;
  if (S) {
    ok = ok && dalloc(&h->st.pms, N) == hipSuccess && dalloc(&h->st.pi_key, N) == hipSuccess &&
         dalloc(&h->st.pms_eik, N) == hipSuccess && dalloc(&h->st.pms_msg, N) == hipSuccess &&
         dalloc(&h->st.slot_hdr, S) == hipSuccess && dalloc(&h->st.sub_a, S * kSubs) == hipSuccess &&
         dalloc(&h->st.sub_b, S * kSubs) == hipSuccess && dalloc(&h->st.sub_k, S * kSubs) == hipSuccess;
  }
  ok = ok && dalloc(&h->d_cmd_hdr2, cfg->max_commands) == hipSuccess &&
       dalloc(&h->d_xparts, cfg->max_commands) == hipSuccess &&
       dalloc(&h->d_key_counter, 1) == hipSuccess && dalloc(&h->d_key_base, cfg->max_commands) == hipSuccess &&
       dalloc(&h->d_key_blk, (cfg->max_commands + 1023) / 1024 + 1) == hipSuccess && dalloc(&h->d_xcount, 1024) == hipSuccess &&
       dalloc(&h->d_seen, N + S) == hipSuccess && dalloc(&h->d_check_flag, 4) == hipSuccess &&
       dalloc(&h->d_ovf, h->ovf_cap = std::max<uint32_t>(4096u, 4u * cfg->max_commands)) == hipSuccess &&
       dalloc(&h->d_ovf_count, 1) == hipSuccess &&
       dalloc(&h->d_cont, cfg->max_commands) == hipSuccess && dalloc(&h->d_cont_order, cfg->max_commands) == hipSuccess;
  if (S) {
    ok = ok && dalloc(&h->d_xout, (size_t)cfg->max_commands * kOut) == hipSuccess &&
         dalloc(&h->d_xbucket, (size_t)cfg->max_commands * kOut) == hipSuccess &&
         dalloc(&h->d_blk_cnt, ((size_t)cfg->max_commands / 256 + 1 + (size_t)cfg->max_commands / (256 * 1024) + 1) *
                                   (size_t)std::max(1, cfg->partition_count)) == hipSuccess;
  }
  if (!ok) { zbhip_close(h); return ZBHIP_ENOMEM; }
  if (S) {
    const unsigned long long kc = (unsigned long long)cfg->initial_key;
    if (hipMemsetAsync(h->st.pms, 0, N * sizeof(uint4), h->stream) != hipSuccess ||
        hipMemsetAsync(h->st.pi_key, 0xFF, N * sizeof(long long), h->stream) != hipSuccess ||
        hipMemsetAsync(h->st.pms_eik, 0xFF, N * sizeof(long long), h->stream) != hipSuccess ||
        hipMemsetAsync(h->st.pms_msg, 0xFF, N * sizeof(long long), h->stream) != hipSuccess ||
        hipMemsetAsync(h->st.slot_hdr, 0, S * sizeof(uint2), h->stream) != hipSuccess ||
        hipMemsetAsync(h->st.sub_a, 0, S * kSubs * sizeof(uint4), h->stream) != hipSuccess ||
        hipMemcpyAsync(h->d_key_counter, &kc, sizeof kc, hipMemcpyHostToDevice, h->stream) != hipSuccess) {
      zbhip_close(h);
      return ZBHIP_EDEVICE;
    }
  }
  h->rec_slots = cfg->max_commands;
  // every slot starts free (proc = 0xFFFF); counters zero
  if (hipMemsetAsync(h->st.hdr, 0xFF, N * sizeof(uint4), h->stream) != hipSuccess ||
      hipMemsetAsync(h->st.tmr, 0, N * sizeof(uint4), h->stream) != hipSuccess ||
      hipMemsetAsync(h->st.join, 0, N * kJoinWords * sizeof(uint32_t), h->stream) != hipSuccess ||
      hipMemsetAsync(h->d_seen, 0, (N + S) * sizeof(uint32_t), h->stream) != hipSuccess ||
      hipMemsetAsync(h->d_check_flag, 0, 4 * sizeof(uint32_t), h->stream) != hipSuccess ||
      hipMemsetAsync(h->d_ovf_count, 0, sizeof(uint32_t), h->stream) != hipSuccess ||
      hipMemsetAsync(h->d_stats, 0, (64 * 8 + 8) * sizeof(unsigned long long), h->stream) != hipSuccess ||
      hipStreamSynchronize(h->stream) != hipSuccess) {
    zbhip_close(h);
    return ZBHIP_EDEVICE;
  }
  for (auto& e : h->ev) (void)hipEventCreate(&e);
  *out = h;
  return ZBHIP_OK;
}

void zbhip_close(zbhip_handle* h) {
  if (!h) return;
  if (h->h_check_flag) {
    (void)hipStreamSynchronize(h->stream);
    (void)hipHostFree(h->h_check_flag);
  }
  (void)hipFree(h->st.hdr);
  (void)hipFree(h->st.slots);
  (void)hipFree(h->st.var_meta);
  (void)hipFree(h->st.var_val);
  (void)hipFree(h->st.join);
  (void)hipFree(h->d_prog);
  (void)hipFree(h->d_cmds);
  (void)hipFree(h->d_docs);
  (void)hipFree(h->d_order);
  (void)hipFree(h->d_sort);
  (void)hipFree(h->d_sort_temp);
  (void)hipFree(h->d_rec);
  (void)hipFree(h->d_cmd_hdr);
  (void)hipFree(h->d_regions);
  (void)hipFree(h->d_region_total);
  (void)hipFree(h->d_region_lanes);
  (void)hipFree(h->d_region_off);
  (void)hipFree(h->d_stats);
  (void)hipFree(h->st.pms);
  (void)hipFree(h->st.pms_eik);
  (void)hipFree(h->st.pms_msg);
  (void)hipFree(h->st.tmr);
  (void)hipFree(h->st.act);
  (void)hipFree(h->d_cmd_act);
  (void)hipFree(h->d_due);
  (void)hipFree(h->d_due_count);
  (void)hipFree(h->d_due_next);
  (void)hipFree(h->d_strs);
  (void)hipFree(h->d_str_off);
  (void)hipFree(h->d_cmd_due);
  (void)hipFree(h->d_map_val);
  (void)hipFree(h->st.pi_key);
  (void)hipFree(h->st.slot_hdr);
  (void)hipFree(h->st.sub_a);
  (void)hipFree(h->st.sub_b);
  (void)hipFree(h->st.sub_k);
  (void)hipFree(h->d_str_hash);
  (void)hipFree(h->d_list_hdr);
  (void)hipFree(h->d_list_val);
  (void)hipFree(h->d_list_type);
  (void)hipFree(h->d_xparts);
  (void)hipFree(h->d_cmd_hdr2);
  (void)hipFree(h->d_xout);
  (void)hipFree(h->d_xbucket);
  (void)hipFree(h->d_blk_cnt);
  (void)hipFree(h->d_xcount);
  (void)hipFree(h->d_key_counter);
  (void)hipFree(h->d_key_base);
  (void)hipFree(h->d_key_blk);
  (void)hipFree(h->d_seen);
  (void)hipFree(h->d_ovf);
  (void)hipFree(h->d_ovf_count);
  (void)hipFree(h->d_cont);
  (void)hipFree(h->d_cont_order);
  (void)hipFree(h->d_qspill);
  (void)hipFree(h->d_tpl);
  (void)hipFree(h->d_log_arena);
  (void)hipFree(h->d_log_idx);
  (void)hipFree(h->d_log_tpl);
  (void)hipFree(h->d_ring);
  (void)hipFree(h->d_inst_proc);
  (void)hipFree(h->d_logcmd);
  (void)hipFree(h->d_log_bytes);
  (void)hipFree(h->d_src_pos);
  (void)hipFree(h->d_tbl_sums);
  if (h->log_double) (void)hipFree(h->log_bufs[h->log_cur ^ 1].dev);  // (the current one is d_log_out)
  for (int b = 0; b < 2; ++b) {
    auto& L = h->log_bufs[b];
    if (L.pending && L.copied) (void)hipEventSynchronize(L.copied);
    if (L.host) (void)hipHostFree(L.host);
    if (L.written) (void)hipEventDestroy(L.written);
    if (L.copied) (void)hipEventDestroy(L.copied);
  }
  if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
  (void)hipFree(h->d_log_out);
  (void)hipFree(h->d_log_flag);
  (void)hipFree(h->d_log_rinfo);
  (void)hipFree(h->d_log_wkeys);
  (void)hipFree(h->d_jrn);
  if (h->inst_proc_pin) (void)hipHostFree(h->inst_proc_pin);
  if (h->src_pos_pin) (void)hipHostFree(h->src_pos_pin);
  (void)hipFree(h->d_check_flag);
  for (auto& e : h->tev) (void)hipEventDestroy(e);
  if (h->upload_ev) (void)hipEventDestroy(h->upload_ev);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  zbhip_serializer_free(h->ser);
  delete h;
}

int zbhip_intern(zbhip_handle* h, const char* name) {
  if (!h || !name) return ZBHIP_EINVAL;
  auto it = h->name_ids.find(name);
  if (it != h->name_ids.end()) return (int)it->second;
  if (h->names.size() >= 0xFFF0) return ZBHIP_ENOMEM;
  uint32_t id = (uint32_t)h->names.size();
  h->names.emplace_back(name);
  h->name_ids.emplace(name, id);
  if (h->ser) zbhip_serializer_intern(h->ser, name);
  return (int)id;
}

const char* zbhip_name(zbhip_handle* h, uint32_t id) {
  return h && id < h->names.size() ? h->names[id].c_str() : "";
}

const char* zbhip_string(zbhip_handle* h, uint32_t p, uint32_t s) {
  if (!h || p >= h->procs.size() || s >= h->procs[p].strings.size()) return "";
  return h->procs[p].strings[s].c_str();
}

// Deploy-time bound of the commands one batch of the process can hold (ProcessingStateMachine's
// FIFO): every token reaching a node costs at most its ACTIVATE and COMPLETE commands, a token
// count per node summed over the incoming flows (joins and exclusive gateways over-counted), plus the
// initial command, the process's ACTIVATE and COMPLETE.  A cycle has no bound.
static uint64_t batch_bound(const Proc& P) {
  if (!P.mi.empty()) return ~0ull;  // a parallel body's children: up to its collection's size per token
  const size_t E = P.els.size();
  std::vector<uint64_t> tok(E, 0);
  std::vector<uint32_t> indeg(E, 0);
  auto is_node = [&](size_t e) { return e > 0 && P.els[e].element_type != ZBHIP_EL_SEQUENCE_FLOW; };
  for (size_t f = 0; f < E; ++f)
    if (P.els[f].element_type == ZBHIP_EL_SEQUENCE_FLOW && P.els[f].flow_target < E) ++indeg[P.els[f].flow_target];
  // a sub-process activates its none start event once per token that reaches it
  for (size_t e = 1; e < E; ++e)
    if (P.els[e].element_type == ZBHIP_EL_SUB_PROCESS && P.els[e].start_event < E) ++indeg[P.els[e].start_event];
  std::vector<uint32_t> ready;
  for (size_t e = 0; e < E; ++e)
    if (is_node(e) && indeg[e] == 0) {
      tok[e] = 1;
      ready.push_back((uint32_t)e);
    }
  size_t seen = 0, nodes = 0;
  for (size_t e = 0; e < E; ++e) nodes += is_node(e);
  uint64_t total = 3;
  while (!ready.empty()) {
    const uint32_t e = ready.back();
    ready.pop_back();
    ++seen;
    total += 2 * tok[e];
    const zbhip_element& N = P.els[e];
    if (N.element_type == ZBHIP_EL_SUB_PROCESS && N.start_event < E) {
      tok[N.start_event] += tok[e];
      if (--indeg[N.start_event] == 0) ready.push_back(N.start_event);
    }
    for (uint32_t i = 0; i < N.out_count; ++i) {
      const uint32_t f = P.out[N.out_begin + i];
      const uint32_t t = P.els[f].flow_target;
      if (t >= E) continue;
      tok[t] += tok[e];
      if (tok[t] > (1u << 20)) return ~0ull;
      if (--indeg[t] == 0) ready.push_back(t);
    }
  }
  return seen == nodes ? total : ~0ull;  // nodes never reached: a cycle
}

// Builds the LDS program arena from every deployed process (layout: zb_internal.h).
// CREATE batch templates (kernels.hip tpl_create): the template word of a process whose CREATE
// batch never waits -- every element reachable from the none start event is a none start or end
// event, a sequence flow or a gateway -- so the batch completes the instance, and whose rows
// depend on at most one decision: one exclusive gateway, entered only from the start event's one
// flow (one token reaches it, once).  Anything else: 0 (no template, the general path as always).
static uint32_t create_template_word(const Proc& P) {
  const uint32_t n_el = (uint32_t)P.els.size();
  if (P.none_start == NONE || P.none_start >= n_el) return 0;
  std::vector<char> seen(n_el, 0);
  std::vector<uint32_t> todo{P.none_start};
  uint32_t xgw = 0xFFF, n_xgw = 0;
  while (!todo.empty()) {
    const uint32_t e = todo.back();
    todo.pop_back();
    if (e >= n_el) return 0;
    if (seen[e]) continue;
    seen[e] = 1;
    const zbhip_element& E = P.els[e];
    switch (E.element_type) {
      case ZBHIP_EL_SEQUENCE_FLOW:
        todo.push_back(E.flow_target);
        continue;
      case ZBHIP_EL_START_EVENT:
        if (E.event_type != ZBHIP_EV_NONE) return 0;
        break;
      case ZBHIP_EL_END_EVENT:
        if (E.event_type != ZBHIP_EV_NONE || E.out_count) return 0;
        break;
      case ZBHIP_EL_PARALLEL_GATEWAY:
        break;
      case ZBHIP_EL_EXCLUSIVE_GATEWAY:
        ++n_xgw;
        xgw = e;
        break;
      default:
        return 0;  // a wait state (task, catch event) or an element outside the subset
    }
    for (uint32_t i = 0; i < E.out_count; ++i) todo.push_back(P.out[E.out_begin + i]);
  }
  if (n_xgw > 1) return 0;
  if (n_xgw == 1) {
    const zbhip_element& S = P.els[P.none_start];
    if (S.out_count != 1 || xgw >= 0xFFF || P.els[xgw].in_count != 1) return 0;
    const uint32_t f = P.out[S.out_begin];
    if (f >= n_el || P.els[f].flow_target != xgw) return 0;
  }
  return TPL_OK | xgw;
}

static int rebuild_program(zbhip_handle* h) {
  std::vector<uint32_t> prog(1 + h->procs.size(), 0);
  prog[0] = (uint32_t)h->procs.size();
  while (prog.size() % 4) prog.push_back(0);
  for (size_t p = 0; p < h->procs.size(); ++p) {
    const Proc& P = h->procs[p];
    const uint32_t base = (uint32_t)prog.size();
    prog[1 + p] = base;
    const uint32_t n_el = (uint32_t)P.els.size();
    const uint32_t out_off = 8 + 4 * n_el;
    const uint32_t cond_off = out_off + ((uint32_t)P.out.size() + 1) / 2;
    const uint32_t n_cond = P.cond_begin.empty() ? 0 : (uint32_t)P.cond_begin.size() - 1;
    const uint32_t code_off = (cond_off + n_cond + 3) & ~3u;  // 16-byte aligned instructions (uint4 loads)
    const uint32_t seg_off = code_off + 4 * (uint32_t)P.code.size();
    const uint32_t io_off = (seg_off + n_el + 3) & ~3u;  // io mappings: 8 words per element (kernels.hip io_map)
    const uint32_t total = P.has_io ? io_off + 8 * n_el : io_off;
    prog.resize(base + total, 0);
    uint32_t* pb = prog.data() + base;
    pb[0] = n_el | ((uint32_t)P.none_start << 16);
    pb[1] = P.n_join_slots | (n_cond << 16);
    pb[2] = out_off;
    pb[3] = cond_off;
    pb[4] = code_off;
    pb[5] = P.bpmn_name | (P.has_timer ? 1u << 16 : 0u) | (P.has_io ? 1u << 17 : 0u);  // bpmnProcessId name id
    pb[6] = seg_off | (io_off << 16);
    if (io_off >= 0x10000) return ZBHIP_ENOMEM;
    if (P.has_io)
      for (uint32_t e = 0; e < n_el; ++e)
        for (int k = 0; k < 2; ++k) {
          // w0 = type | target name << 16, w1 = source name id, w2/w3 = the literal (STR: its string id)
          const Proc::Io io = e < P.io.size() ? P.io[e][k] : Proc::Io{};
          uint32_t* m = pb + io_off + 8 * e + 4 * k;
          m[0] = io.type | ((uint32_t)io.tgt << 16);
          m[1] = io.src;
          m[2] = (uint32_t)((uint64_t)io.lit & 0xFFFFFFFFu);
          m[3] = (uint32_t)((uint64_t)io.lit >> 32);
          // a multi-instance body (never io-mapped) holds its collection words in its input slot
          // (kernels.hip mi_ext): collection | outputCollection << 16, outputElement | (condition + 1) << 16,
          // numberOfInstances | numberOfActiveInstances << 16, numberOfCompletedInstances |
          // numberOfTerminatedInstances << 16
          const Proc::Mi* mb = k == 0 && P.els[e].element_type == ZBHIP_EL_MULTI_INSTANCE_BODY ? P.mi_body(e) : nullptr;
          if (mb) {
            m[0] = mb->coll_name | ((uint32_t)mb->out_coll << 16);
            m[1] = mb->out_elem | ((uint32_t)(mb->cond + 1) << 16);
            m[2] = mb->n_names[0] | ((uint32_t)mb->n_names[1] << 16);
            m[3] = mb->n_names[2] | ((uint32_t)mb->n_names[3] << 16);
          } else if (k == 1 && P.els[e].element_type == ZBHIP_EL_MULTI_INSTANCE_BODY && P.mi_body(e)) {
            m[1] = P.mi_body(e)->static_list;  // (no output mapping: m[0] stays kIoNone)
          }
        }
    pb[7] = create_template_word(P);
    // straight-line segment words (kernels.hip fast_command): a start event or service task with
    // one unconditional outgoing flow into a service task or a none end event without outgoing flows
    // (a task whose jobs a job stream takes is entered on the general path: the push record)
    auto streamed = [&](uint32_t t) { return ZBHIP_IS_JOB_WORKER(P.els[t].element_type) && h->streams.count(P.job_type_id[t]); };
    for (uint32_t e = 0; e < n_el; ++e) {
      const zbhip_element& E = P.els[e];
      uint32_t sg = 0;
      // (bits 25 / 26: the task / the next task carries a timer boundary event -- KScope's
      // fast_scope_job; KLinear never holds such processes, its fast_command refuses the bits)
      auto timer_boundary = [&](const zbhip_element& T) {
        return T.start_event != ZBHIP_NONE16 && T.start_event < n_el &&
               P.els[T.start_event].element_type == ZBHIP_EL_BOUNDARY_EVENT && P.els[T.start_event].event_type == ZBHIP_EV_TIMER;
      };
      const bool src_tmr = ZBHIP_IS_JOB_WORKER(E.element_type) && timer_boundary(E);
      if ((E.element_type == ZBHIP_EL_START_EVENT || ZBHIP_IS_JOB_WORKER(E.element_type)) && E.out_count == 1 &&
          E.flow_scope == 0 && !(ZBHIP_IS_JOB_WORKER(E.element_type) && E.start_event != ZBHIP_NONE16 && !src_tmr) &&
          !P.io_of(e) && !P.mi_inner(e)) {
        const uint32_t f = P.out[E.out_begin];
        const zbhip_element& F = P.els[f];
        const uint32_t n = F.flow_target;
        if (F.element_type == ZBHIP_EL_SEQUENCE_FLOW && F.condition == ZBHIP_NONE16 && n < n_el && f < 0xFFF && n < 0xFFF) {
          const zbhip_element& N = P.els[n];
          const bool dst_tmr = ZBHIP_IS_JOB_WORKER(N.element_type) && timer_boundary(N);
          const bool task = ZBHIP_IS_JOB_WORKER(N.element_type) && (N.start_event == ZBHIP_NONE16 || dst_tmr) &&
                            !P.io_of(n) && !P.mi_inner(n) && !streamed(n);
          const bool end = N.element_type == ZBHIP_EL_END_EVENT && N.event_type == ZBHIP_EV_NONE && N.out_count == 0;
          // bit 29: a start event into a forking parallel gateway whose every outgoing flow is
          // unconditional into a task without boundary event (KGeneric's fast_fork_create)
          bool fork = E.element_type == ZBHIP_EL_START_EVENT && N.element_type == ZBHIP_EL_PARALLEL_GATEWAY &&
                      N.in_count == 1 && N.out_count >= 2 && N.out_count <= 8 && N.flow_scope == 0;
          for (uint32_t i = 0; fork && i < N.out_count; ++i) {
            const zbhip_element& G = P.els[P.out[N.out_begin + i]];
            const uint32_t t = G.flow_target;
            fork = G.element_type == ZBHIP_EL_SEQUENCE_FLOW && G.condition == ZBHIP_NONE16 && t < n_el &&
                   ZBHIP_IS_JOB_WORKER(P.els[t].element_type) && P.els[t].start_event == ZBHIP_NONE16 &&
                   !P.io_of(t) && !P.mi_inner(t) && P.els[t].element_type != ZBHIP_EL_PARALLEL_GATEWAY && !streamed(t);
          }
          if (fork) sg = (1u << 31) | (1u << 29) | (n << 12) | f;
          // bit 27: a task into a joining parallel gateway (KGeneric's fast_join_job)
          const bool join = ZBHIP_IS_JOB_WORKER(E.element_type) && !src_tmr && N.element_type == ZBHIP_EL_PARALLEL_GATEWAY &&
                            N.in_count >= 2 && N.out_count == 1 && N.flow_scope == 0;
          if (task || end || join)
            sg = (1u << 31) | (ZBHIP_IS_JOB_WORKER(E.element_type) ? 1u << 30 : 0u) | (end ? 1u << 24 : 0u) |
                 (src_tmr ? 1u << 25 : 0u) | (dst_tmr ? 1u << 26 : 0u) | (join ? 1u << 27 : 0u) | (n << 12) | f;
        }
      } else if (E.element_type == ZBHIP_EL_PARALLEL_GATEWAY && E.in_count >= 2 && E.out_count == 1 && E.flow_scope == 0) {
        // bit 28: a joining gateway's one unconditional flow into a task (no boundary event) or a none
        // end event (the continuation of fast_join_job)
        const uint32_t f = P.out[E.out_begin];
        const zbhip_element& F = P.els[f];
        const uint32_t n = F.flow_target;
        if (F.element_type == ZBHIP_EL_SEQUENCE_FLOW && F.condition == ZBHIP_NONE16 && n < n_el && f < 0xFFF && n < 0xFFF) {
          const zbhip_element& N = P.els[n];
          const bool task = ZBHIP_IS_JOB_WORKER(N.element_type) && N.start_event == ZBHIP_NONE16 && !P.io_of(n) &&
                            !P.mi_inner(n) && !streamed(n);
          const bool end = N.element_type == ZBHIP_EL_END_EVENT && N.event_type == ZBHIP_EV_NONE && N.out_count == 0;
          if (task || end) sg = (1u << 31) | (1u << 28) | (end ? 1u << 24 : 0u) | (n << 12) | f;
        }
      }
      pb[seg_off + e] = sg;
    }
    // NUMBER_OF_TAKEN_SEQUENCE_FLOWS rows of a sub-process's own gateways: removed with the
    // sub-process instance (DbElementInstanceState.removeInstance)
    std::vector<uint32_t> join_mask(n_el, 0);
    for (uint32_t f = 0; f < n_el; ++f) {
      const zbhip_element& F = P.els[f];
      if (F.element_type == ZBHIP_EL_SEQUENCE_FLOW && F.join_slot < 16 && F.flow_scope)
        join_mask[F.flow_scope] |= 1u << F.join_slot;
    }
    for (uint32_t e = 0; e < n_el; ++e) {
      const zbhip_element& E = P.els[e];
      uint32_t* w = pb + 8 + 4 * e;
      w[0] = E.element_type | ((uint32_t)E.event_type << 8) | ((uint32_t)E.in_count << 16);
      w[1] = E.out_begin | ((uint32_t)E.out_count << 16);
      if (E.element_type == ZBHIP_EL_SEQUENCE_FLOW) w[2] = E.flow_target | ((uint32_t)E.condition << 16);
      else if (E.element_type == ZBHIP_EL_EXCLUSIVE_GATEWAY) w[2] = E.default_flow | (0xFFFFu << 16);
      else if (ZBHIP_IS_JOB_WORKER(E.element_type))  // job type | 0 when a job stream takes its jobs (0xFFFF none)
        w[2] = E.job_type | ((h->streams.count(P.job_type_id[e]) ? 0u : 0xFFFFu) << 16);
      else if ((E.element_type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT || E.element_type == ZBHIP_EL_BOUNDARY_EVENT) &&
               E.event_type == ZBHIP_EV_MESSAGE)
        w[2] = E.message_name | ((uint32_t)E.correlation_var << 16);  // name ids (zbhip_deploy)
      else if (E.element_type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT || E.element_type == ZBHIP_EL_BOUNDARY_EVENT)
        w[2] = E.duration_ms;
      else if (E.element_type == ZBHIP_EL_SUB_PROCESS) w[2] = E.start_event | (join_mask[e] << 16);
      else w[2] = 0xFFFFFFFFu;
      // a job worker's join_slot half: its boundary event (zbhip_element.start_event), 0xFFFF if none;
      // a sub-process's: its boundary event (zbhip_element.default_flow); a boundary event's: 1 if
      // interrupting (zbhip_element.job_retries)
      const uint32_t low = ZBHIP_IS_JOB_WORKER(E.element_type) ? E.start_event
                           : E.element_type == ZBHIP_EL_SUB_PROCESS ? E.default_flow
                           : E.element_type == ZBHIP_EL_BOUNDARY_EVENT ? E.job_retries : E.join_slot;
      w[3] = low | ((uint32_t)E.flow_scope << 16);
      if (const Proc::Mi* m = E.element_type == ZBHIP_EL_MULTI_INSTANCE_BODY ? P.mi_body(e) : nullptr) {
        // a multi-instance body: w0 high half its inputElement's name id, w2 inner activity |
        // collection size << 12 | isSequential << 20, w3 low half the loopCounter name id
        w[0] = E.element_type | ((uint32_t)E.event_type << 8) | ((uint32_t)m->input_name << 16);
        w[2] = m->inner | ((uint32_t)m->items.size() << 12) | (m->seq ? 1u << 20 : 0u);
        w[3] = m->loop_name | ((uint32_t)E.flow_scope << 16);
      }
    }
    uint16_t* outw = reinterpret_cast<uint16_t*>(pb + out_off);
    for (size_t i = 0; i < P.out.size(); ++i) outw[i] = P.out[i];
    for (uint32_t c = 0; c < n_cond; ++c) pb[cond_off + c] = P.cond_begin[c];
    for (size_t i = 0; i < P.code.size(); ++i) {
      uint32_t* in = pb + code_off + 4 * i;
      in[0] = P.code[i].op;
      in[1] = P.code[i].arg;
      in[2] = (uint32_t)((uint64_t)P.code[i].literal & 0xFFFFFFFFu);
      in[3] = (uint32_t)((uint64_t)P.code[i].literal >> 32);
    }
  }
  if (prog.size() > kMaxProgWords) return ZBHIP_ENOMEM;
  if (prog.size() > h->d_prog_cap) {
    (void)hipFree(h->d_prog);
    h->d_prog = nullptr;
    if (dalloc(&h->d_prog, prog.size()) != hipSuccess) return ZBHIP_ENOMEM;
    h->d_prog_cap = prog.size();
  }
  if (h->procs.size() > h->tpl_procs && h->variant != 2 && h->variant != 3) {
    // a larger template table (templates are relearned: the next launches record them again)
    (void)hipFree(h->d_tpl);
    h->d_tpl = nullptr;
    h->tpl_procs = 0;
    const size_t cap = std::max<size_t>(16, h->procs.size() * 2);
    const size_t words = cap * kTplVar * kTplWords;
    if (dalloc(&h->d_tpl, words) != hipSuccess) return ZBHIP_ENOMEM;
    HIPCHK(hipMemsetAsync(h->d_tpl, 0, words * sizeof(uint2), h->stream));
    h->tpl_procs = cap;
  }
  HIPCHK(hipMemcpyAsync(h->d_prog, prog.data(), prog.size() * 4, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->prog.swap(prog);
  return ZBHIP_OK;
}

int zbhip_deploy(zbhip_handle* h, const zbhip_process_csr* csr, uint32_t* idx_out) {
  if (!h || !csr || csr->n_elements == 0 || csr->n_elements > (uint32_t)kMaxElements) return ZBHIP_EINVAL;
  if (csr->n_join_slots > kMaxJoinSlots) return ZBHIP_EUNSUPP;
  if (h->procs.size() >= 0xFFF0) return ZBHIP_ENOMEM;
  Proc P;
  P.els.assign(csr->elements, csr->elements + csr->n_elements);
  P.out.assign(csr->out_flow, csr->out_flow + csr->n_out);
  if (csr->n_conditions) P.cond_begin.assign(csr->cond_begin, csr->cond_begin + csr->n_conditions + 1);
  P.code.assign(csr->code, csr->code + csr->n_code);
  for (uint32_t i = 0; i < csr->n_strings; ++i) P.strings.emplace_back(csr->strings[i]);
  P.none_start = csr->none_start;
  P.n_join_slots = csr->n_join_slots;
  P.def_key = csr->process_definition_key;
  P.version = csr->version;
  P.bpmn_id = csr->bpmn_process_id;
  for (auto& e : P.els)
    if (e.element_type != ZBHIP_EL_PROCESS && e.element_type != ZBHIP_EL_START_EVENT &&
        e.element_type != ZBHIP_EL_END_EVENT && !ZBHIP_IS_JOB_WORKER(e.element_type) &&
        e.element_type != ZBHIP_EL_EXCLUSIVE_GATEWAY && e.element_type != ZBHIP_EL_PARALLEL_GATEWAY &&
        e.element_type != ZBHIP_EL_SEQUENCE_FLOW && e.element_type != ZBHIP_EL_INTERMEDIATE_CATCH_EVENT &&
        e.element_type != ZBHIP_EL_SUB_PROCESS && e.element_type != ZBHIP_EL_BOUNDARY_EVENT &&
        e.element_type != ZBHIP_EL_MULTI_INSTANCE_BODY && e.element_type != ZBHIP_EL_EVENT_SUB_PROCESS &&
        !pass_through(e.element_type))
      return ZBHIP_EUNSUPP;
  // event sub-processes (error start events only): never entered on the device -- a JOB:THROW_ERROR hands
  // the instance to the engine, which activates them -- so their contents are held to elements that need
  // no deploy-time device state (no catch or boundary events, no nested containers); an error start event
  // lives only there
  for (size_t e = 1; e < P.els.size(); ++e) {
    const zbhip_element& E = P.els[e];
    if (E.flow_scope >= P.els.size()) return ZBHIP_EINVAL;
    if (E.element_type == ZBHIP_EL_START_EVENT && E.event_type != ZBHIP_EV_NONE &&
        (E.event_type != ZBHIP_EV_ERROR || P.els[E.flow_scope].element_type != ZBHIP_EL_EVENT_SUB_PROCESS))
      return ZBHIP_EINVAL;
    bool inside = false;
    for (uint32_t c = E.flow_scope, d = 0; c != 0 && c < P.els.size() && d < 64; c = P.els[c].flow_scope, ++d)
      inside |= P.els[c].element_type == ZBHIP_EL_EVENT_SUB_PROCESS;
    if (!inside) continue;
    const bool ok = E.element_type == ZBHIP_EL_START_EVENT || E.element_type == ZBHIP_EL_END_EVENT ||
                    (ZBHIP_IS_JOB_WORKER(E.element_type) && E.start_event == ZBHIP_NONE16) ||
                    E.element_type == ZBHIP_EL_EXCLUSIVE_GATEWAY || E.element_type == ZBHIP_EL_PARALLEL_GATEWAY ||
                    E.element_type == ZBHIP_EL_SEQUENCE_FLOW || pass_through(E.element_type);
    if (!ok) return ZBHIP_EUNSUPP;
  }
  // timer and message boundary events: one per job worker task, in the task's container (message
  // boundary events: the process's, KMsg has no flow scopes)
  for (size_t e = 0; e < P.els.size(); ++e) {
    const zbhip_element& E = P.els[e];
    if (E.element_type == ZBHIP_EL_BOUNDARY_EVENT) {
      const bool msg = E.event_type == ZBHIP_EV_MESSAGE && E.flow_scope == 0;
      // (an error boundary event: nothing on the device -- JOB:THROW_ERROR hands the instance off)
      if ((E.event_type != ZBHIP_EV_TIMER && E.event_type != ZBHIP_EV_ERROR && !msg) || E.flow_source >= P.els.size())
        return ZBHIP_EUNSUPP;
      const zbhip_element& A = P.els[E.flow_source];
      // (a timer or error boundary event on an embedded sub-process: zbhip_element.default_flow of the
      // sub-process)
      const bool on_sub = A.element_type == ZBHIP_EL_SUB_PROCESS &&
                          (E.event_type == ZBHIP_EV_TIMER || E.event_type == ZBHIP_EV_ERROR) && A.default_flow == e;
      // (further error boundary events of an activity: outside its slot, found by flow_source)
      const uint16_t slot = A.element_type == ZBHIP_EL_SUB_PROCESS ? A.default_flow : A.start_event;
      const bool extra_error = E.event_type == ZBHIP_EV_ERROR &&
                               ((slot != ZBHIP_NONE16 && slot < P.els.size() &&
                                 (ZBHIP_IS_JOB_WORKER(A.element_type) || A.element_type == ZBHIP_EL_SUB_PROCESS)) ||
                                A.element_type == ZBHIP_EL_MULTI_INSTANCE_BODY);  // (a body: no slot)
      if ((!ZBHIP_IS_JOB_WORKER(A.element_type) || A.start_event != e) && !on_sub && !extra_error) return ZBHIP_EINVAL;
      if (A.flow_scope != E.flow_scope) return ZBHIP_EINVAL;
    } else if (ZBHIP_IS_JOB_WORKER(E.element_type) && E.start_event != ZBHIP_NONE16) {
      if (E.start_event >= P.els.size() || P.els[E.start_event].element_type != ZBHIP_EL_BOUNDARY_EVENT) return ZBHIP_EINVAL;
    }
  }
  for (size_t e = 0; e < P.els.size(); ++e) {  // containers: a sub-process element, before its children
    const zbhip_element& E = P.els[e];
    if (e > 0 && (E.flow_scope >= e || (E.flow_scope && P.els[E.flow_scope].element_type != ZBHIP_EL_SUB_PROCESS &&
                                        P.els[E.flow_scope].element_type != ZBHIP_EL_MULTI_INSTANCE_BODY &&
                                        P.els[E.flow_scope].element_type != ZBHIP_EL_EVENT_SUB_PROCESS)))
      return ZBHIP_EINVAL;
    if (E.element_type == ZBHIP_EL_EVENT_SUB_PROCESS &&
        (E.start_event >= P.els.size() || P.els[E.start_event].flow_scope != e ||
         P.els[E.start_event].event_type != ZBHIP_EV_ERROR ||
         (E.flow_scope != 0 && P.els[E.flow_scope].element_type != ZBHIP_EL_SUB_PROCESS)))
      return ZBHIP_EINVAL;
    if (E.flow_scope && P.els[E.flow_scope].element_type == ZBHIP_EL_MULTI_INSTANCE_BODY &&
        P.els[E.flow_scope].start_event != e)
      return ZBHIP_EINVAL;  // a body contains exactly its inner activity
    if (E.element_type == ZBHIP_EL_SUB_PROCESS &&
        (E.start_event >= P.els.size() || P.els[E.start_event].flow_scope != e))
      return ZBHIP_EINVAL;
  }
  for (auto& e : P.els)
    if ((e.element_type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT || e.element_type == ZBHIP_EL_BOUNDARY_EVENT) &&
        e.event_type == ZBHIP_EV_TIMER) {
      P.has_timer = true;
    } else if (e.element_type == ZBHIP_EL_BOUNDARY_EVENT && e.event_type == ZBHIP_EV_ERROR) {
      // error boundary events: no device state (the instance moves to the engine for JOB:THROW_ERROR)
    } else if (e.element_type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT || e.element_type == ZBHIP_EL_BOUNDARY_EVENT) {
      // message catch events and message boundary events (KMsg)
      if (e.event_type != ZBHIP_EV_MESSAGE) return ZBHIP_EINVAL;
      if (!h->st.n_slots) return ZBHIP_EUNSUPP;  // the handle was opened without message state
      if (e.message_name >= P.strings.size() || e.correlation_var >= P.strings.size()) return ZBHIP_EINVAL;
      P.has_msg = true;
    }
  // multi-instance bodies (MultiInstanceActivityTransformer): the inner activity right behind the body,
  // a job worker (no boundary event: those attach to the body, outside the subset) or an undefined
  // task; a static collection of at most kMaxMiItems items (ZBHIP_OP_ITEM, then ZBHIP_OP_END)
  P.mi_of.assign(P.els.size(), -1);
  for (size_t e = 0; e < P.els.size(); ++e) {
    const zbhip_element& E = P.els[e];
    if (E.element_type != ZBHIP_EL_MULTI_INSTANCE_BODY) continue;
    if (E.start_event != e + 1 || e + 1 >= P.els.size() || e >= 0xFFF) return ZBHIP_EINVAL;
    const zbhip_element& I = P.els[e + 1];
    if (I.flow_scope != e || I.out_count || I.in_count) return ZBHIP_EINVAL;
    if (!(ZBHIP_IS_JOB_WORKER(I.element_type) && I.start_event == ZBHIP_NONE16) && I.element_type != ZBHIP_EL_TASK &&
        I.element_type != ZBHIP_EL_MANUAL_TASK)
      return ZBHIP_EUNSUPP;
    if (E.condition == ZBHIP_NONE16 || (size_t)E.condition + 1 >= P.cond_begin.size()) return ZBHIP_EINVAL;
    Proc::Mi m;
    m.body = (uint16_t)e;
    m.inner = (uint16_t)(e + 1);
    m.seq = E.job_retries & 1;
    m.input_name = m.loop_name = NONE;
    const uint32_t b0 = P.cond_begin[E.condition], b1 = P.cond_begin[E.condition + 1];
    if (b1 <= b0 || b1 > P.code.size() || P.code[b1 - 1].op != ZBHIP_OP_END) return ZBHIP_EINVAL;
    for (uint32_t i = b0; i + 1 < b1; ++i) {
      const zbhip_insn& in = P.code[i];
      if (in.op == ZBHIP_OP_COLLECTION) {  // (string-table indices until the names are interned below)
        if (i != b0 || in.arg >= P.strings.size()) return ZBHIP_EINVAL;
        m.coll_name = (uint16_t)in.arg;
        continue;
      }
      if (in.op == ZBHIP_OP_OUTPUT) {
        if (i + 2 != b1 || in.arg >= P.strings.size() || in.literal < 0 || (size_t)in.literal >= P.strings.size())
          return ZBHIP_EINVAL;
        m.out_coll = (uint16_t)in.arg;
        m.out_elem = (uint16_t)in.literal;
        continue;
      }
      if (in.op != ZBHIP_OP_ITEM || m.coll_name != NONE) return ZBHIP_EINVAL;
      if (in.arg != ZBHIP_DOC_INT && in.arg != ZBHIP_DOC_BOOL && in.arg != ZBHIP_DOC_NIL && in.arg != ZBHIP_DOC_STR)
        return ZBHIP_EUNSUPP;
      if (in.arg == ZBHIP_DOC_STR && (in.literal < 0 || (size_t)in.literal >= P.strings.size())) return ZBHIP_EINVAL;
      m.items.push_back({(uint8_t)in.arg, in.literal});
    }
    if (m.items.size() > kMaxMiItems) return ZBHIP_EUNSUPP;
    if (E.default_flow != ZBHIP_NONE16) {  // the completionCondition
      if ((size_t)E.default_flow + 1 >= P.cond_begin.size()) return ZBHIP_EINVAL;
      m.cond = E.default_flow;
    }
    if (E.message_name != ZBHIP_NONE16 && E.message_name >= P.strings.size()) return ZBHIP_EINVAL;
    P.mi_of[e] = P.mi_of[e + 1] = (int16_t)P.mi.size();
    P.mi.push_back(std::move(m));
  }
  // condition variable names -> partition name ids, interned in element order (the oracle's order)
  for (auto& e : P.els) {
    if (e.element_type != ZBHIP_EL_SEQUENCE_FLOW || e.condition == ZBHIP_NONE16) continue;
    for (uint32_t i = P.cond_begin[e.condition]; i < P.cond_begin[e.condition + 1]; ++i)
      if (P.code[i].op == ZBHIP_OP_PUSH_VAR) {
        if (P.code[i].arg >= P.strings.size()) return ZBHIP_EINVAL;
        int id = zbhip_intern(h, P.strings[P.code[i].arg].c_str());
        if (id < 0) return id;
        P.code[i].arg = (uint32_t)id;
      }
  }
  // message names and correlation variables, then the bpmnProcessId, in element order (the
  // oracle's order): the name dictionary is replicated across partitions by deploy order
  if (P.has_msg) {
    for (auto& e : P.els) {
      if ((e.element_type != ZBHIP_EL_INTERMEDIATE_CATCH_EVENT && e.element_type != ZBHIP_EL_BOUNDARY_EVENT) ||
          e.event_type != ZBHIP_EV_MESSAGE)
        continue;
      int mn = zbhip_intern(h, P.strings[e.message_name].c_str());
      int cv = zbhip_intern(h, P.strings[e.correlation_var].c_str());
      if (mn < 0 || cv < 0) return ZBHIP_ENOMEM;
      e.message_name = (uint16_t)mn;
      e.correlation_var = (uint16_t)cv;
    }
    int bn = zbhip_intern(h, P.strings[P.bpmn_id].c_str());
    if (bn < 0) return ZBHIP_ENOMEM;
    P.bpmn_name = (uint16_t)bn;
  }
  // multi-instance bodies, in element order: the inputElement and loopCounter names, then the string
  // items into the value dictionary (the oracle's deploy order)
  for (Proc::Mi& m : P.mi) {
    const zbhip_element& E = P.els[m.body];
    if (E.message_name != ZBHIP_NONE16) {
      const int in = zbhip_intern(h, P.strings[E.message_name].c_str());
      if (in < 0) return in;
      m.input_name = (uint16_t)in;
    }
    const int ln = zbhip_intern(h, "loopCounter");
    if (ln < 0) return ln;
    m.loop_name = (uint16_t)ln;
    for (auto& it : m.items)
      if (it.first == ZBHIP_DOC_STR) {
        const std::string& t = P.strings[(size_t)it.second];
        const int64_t sid = zbhip_intern_string(h, t.data(), t.size());
        if (sid < 0) return (int)sid;
        it.second = sid;
      }
    // then the collection variable, the outputCollection and outputElement names, the completion
    // condition's variables (the oracle's deploy order); numberOf* are the condition's primary context
    for (uint16_t* nm : {&m.coll_name, &m.out_coll, &m.out_elem})
      if (*nm != NONE) {
        const int id = zbhip_intern(h, P.strings[*nm].c_str());
        if (id < 0) return id;
        *nm = (uint16_t)id;
      }
    if (m.cond >= 0) {
      static const char* kNumberOf[4] = {"numberOfInstances", "numberOfActiveInstances", "numberOfCompletedInstances",
                                         "numberOfTerminatedInstances"};
      for (uint32_t i = P.cond_begin[m.cond]; i < P.cond_begin[m.cond + 1]; ++i)
        if (P.code[i].op == ZBHIP_OP_PUSH_VAR) {
          if (P.code[i].arg >= P.strings.size()) return ZBHIP_EINVAL;
          const std::string& vn = P.strings[P.code[i].arg];
          const int id = zbhip_intern(h, vn.c_str());
          if (id < 0) return id;
          P.code[i].arg = (uint32_t)id;
          for (int k = 0; k < 4; ++k)
            if (vn == kNumberOf[k]) m.n_names[k] = (uint16_t)id;
          // the outputCollection is not held on the device
          if (id == m.out_coll) return ZBHIP_EUNSUPP;
        }
    }
    if (m.ext()) {
      P.has_io = true;  // the body's words in its io slot (rebuild_program): KScopeIO
      if (m.coll_name == NONE) {  // the static items as a list: the device reads item values from it
        const int64_t id = intern_items(h, m.items);
        if (id < 0) return (int)id;
        m.static_list = (uint32_t)id;
      }
    }
  }
  // io mappings (zbhip_mapping): job worker tasks (not multi-instance inner activities) and embedded
  // sub-processes, one input and one output each; names interned in element order, the input's source
  // and target before the output's (the oracle's deploy order), string literals into the value
  // dictionary
  if (csr->n_mappings) {
    if (!csr->mappings) return ZBHIP_EINVAL;
    P.io.assign(P.els.size(), {});
    for (uint32_t i = 0; i < csr->n_mappings; ++i) {
      const zbhip_mapping& M = csr->mappings[i];
      if (M.element >= P.els.size() || M.output > 1 || M.target >= P.strings.size()) return ZBHIP_EINVAL;
      const zbhip_element& E = P.els[M.element];
      if (!(ZBHIP_IS_JOB_WORKER(E.element_type) || E.element_type == ZBHIP_EL_SUB_PROCESS) || P.mi_inner(M.element))
        return ZBHIP_EUNSUPP;
      Proc::Io& io = P.io[M.element][M.output];
      if (io.type != kIoNone) return ZBHIP_EUNSUPP;  // one mapping of each kind
      if (M.source_type == ZBHIP_MAP_VARIABLE || M.source_type == ZBHIP_DOC_STR) {
        if (M.source >= P.strings.size()) return ZBHIP_EINVAL;
      } else if (M.source_type != ZBHIP_DOC_NIL && M.source_type != ZBHIP_DOC_BOOL && M.source_type != ZBHIP_DOC_INT) {
        return ZBHIP_EUNSUPP;
      }
      io.type = M.source_type;
      io.src = M.source;
      io.tgt = M.target;
      io.lit = M.literal;
    }
    for (size_t e = 0; e < P.els.size(); ++e)
      for (Proc::Io& io : P.io[e]) {
        if (io.type == kIoNone) continue;
        if (io.type == ZBHIP_MAP_VARIABLE) {
          const int id = zbhip_intern(h, P.strings[io.src].c_str());
          if (id < 0) return id;
          io.src = (uint16_t)id;
        } else if (io.type == ZBHIP_DOC_STR) {
          const std::string& t = P.strings[io.src];
          const int64_t sid = zbhip_intern_string(h, t.data(), t.size());
          if (sid < 0) return (int)sid;
          io.lit = sid;
        }
        const int tid = zbhip_intern(h, P.strings[io.tgt].c_str());
        if (tid < 0) return tid;
        io.tgt = (uint16_t)tid;
        P.has_io = true;
      }
  }
  // kernel variant, the smallest that covers every deployed process (kernels.hip KCfg):
  //   3 KLinear  -- linear chains: every node <= 1 outgoing flow, no gateways (4 waves/SIMD)
  //   0 KSimple  -- one token per instance (no parallel gateway / multi-outgoing node but an XOR)
  //   1 KGeneric -- everything else in the subset
  //   4 KScope   -- embedded sub-processes (flow scopes below the process), timers
  //   5 KScopeIO -- KScope plus zeebe:ioMapping (variables in element-instance scopes)
  //   2 KMsg     -- message catch events and subscription commands (config 5); a sub-process
  //                 deployed next to them falls back (KMsg has no flow scopes)
  int cls = 3;
  bool scopes = false;
  for (auto& e : P.els) {
    if (e.element_type == ZBHIP_EL_EXCLUSIVE_GATEWAY && cls == 3) cls = 0;
    if (e.element_type == ZBHIP_EL_PARALLEL_GATEWAY) cls = 1;
    if (e.element_type != ZBHIP_EL_EXCLUSIVE_GATEWAY && e.element_type != ZBHIP_EL_SEQUENCE_FLOW && e.out_count > 1)
      cls = 1;
    scopes |= e.element_type == ZBHIP_EL_SUB_PROCESS || e.element_type == ZBHIP_EL_MULTI_INSTANCE_BODY;
  }
  // timer catch events: KScope as well (the instance's timer row); io mappings: KScopeIO (variables
  // in the scopes of element instances)
  if (scopes || P.has_timer) cls = 4;
  if (P.has_io) cls = 5;
  if (P.has_msg) cls = 2;
  if (P.has_io) {
    // the device walks io-mapped scope chains at most kMaxScopeDepth containers up (kernels.hip
    // var_lookup, merge_document_from, apply_output_mapping); a deeper nesting stays with the engine,
    // whose DbVariableState walks the whole parent chain
    for (uint32_t e = 0; e < P.els.size(); ++e) {
      int depth = 0;
      for (uint32_t c = P.els[e].flow_scope; c != 0 && c < P.els.size() && depth <= kMaxScopeDepth; c = P.els[c].flow_scope)
        ++depth;
      if (depth > kMaxScopeDepth) return ZBHIP_EUNSUPP;
    }
  }
  auto rank = [](int v) { return v == 3 ? 0 : v == 0 ? 1 : v == 1 ? 2 : v == 4 ? 3 : v == 5 ? 4 : 5; };
  if ((P.has_msg && (h->variant == 5 || P.has_io)) || (P.has_io && h->msg())) return ZBHIP_EUNSUPP;  // KMsg has no io
  const int old_variant = h->variant;
  if (h->procs.empty() || rank(cls) > rank(h->variant)) h->variant = cls;
  if (const char* fv = getenv("ZBHIP_FORCE_VARIANT")) {  // experiments: never below what the processes need
    const int f = atoi(fv);
    if (rank(f) >= rank(h->variant)) h->variant = f;
  }
  P.job_type_id.assign(P.els.size(), ~0u);
  for (size_t e = 0; e < P.els.size(); ++e)
    if (ZBHIP_IS_JOB_WORKER(P.els[e].element_type) && P.els[e].job_type < P.strings.size())
      P.job_type_id[e] = h->job_type(P.strings[P.els[e].job_type]);
  const bool mi_ext = std::any_of(P.mi.begin(), P.mi.end(), [](const Proc::Mi& m) { return m.ext(); });
  h->procs.push_back(std::move(P));
  if (mi_ext) {
    h->mi_ext = true;
    h->ring_ok = false;  // list values: the host serialiser writes such windows
  }
  {
    const uint64_t limit = (uint64_t)h->cfg.max_commands_in_batch;
    bool over = false;
    uint64_t pend = 0;
    for (const Proc& Q : h->procs) {
      const uint64_t b = batch_bound(Q);
      over |= b >= limit;
      pend = std::max(pend, std::min(b, limit));
    }
    h->may_overflow = over;
    h->max_pending = (uint32_t)pend;
  }
  int rc = rebuild_program(h);
  if (rc != ZBHIP_OK) {
    h->procs.pop_back();
    h->variant = old_variant;
    return rc;
  }
  zbhip_serializer_deploy(h->ser, csr, nullptr);  // same index: both append in deploy order
  if (idx_out) *idx_out = (uint32_t)h->procs.size() - 1;
  return ZBHIP_OK;
}

static bool slot_kind(uint8_t k) { return zb_slot_kind(k); }

// Splits the window into rounds so that each subject (instance slot; correlation slot for message
// commands) appears at most once per launch; commands of one subject keep their log order across
// rounds (the reference processes them in log order).  Message commands may touch an instance of
// this partition and instance commands a correlation slot, so a change between the two classes
// starts a new epoch: every later command goes to a round after all earlier ones.
// A large plain window's subjects are claimed on the host threads first (one atomic stamp exchange
// each): the common window addresses every instance once and needs no ordered pass.
static int plan_rounds(zbhip_handle* h) {
  h->round_begin.clear();
  h->h_order.clear();
  // a CREATE into an instance slot that an earlier command of the same window addressed is refused:
  // the adapter reuses a slot only after the window that ended its instance was drained (records of
  // both instances would otherwise share the slot's key history)
  // (message partitions: a window-wide stamp table, the round stamps below restart per epoch;
  // otherwise the round table's own stamp says "addressed earlier in this window")
  const bool msg = h->msg();
  if (msg) {
    const size_t n_inst0 = h->cfg.max_instances;
    if (h->plan_seen.size() < n_inst0) h->plan_seen.assign(n_inst0, 0u);
    if (++h->plan_window == 0) {
      std::fill(h->plan_seen.begin(), h->plan_seen.end(), 0u);
      h->plan_window = 1;
    }
    for (size_t i = 0; i < h->n_cmds; ++i) {
      const zbhip_command& c = h->h_cmds[i];
      if (slot_kind(c.kind)) continue;
      if (c.kind == ZBHIP_CMD_CREATE && h->plan_seen[c.instance] == h->plan_window) return ZBHIP_EINVAL;
      h->plan_seen[c.instance] = h->plan_window;
    }
  }
  // last round per subject in a flat table (instances, then correlation slots), valid where its
  // stamp is the current one: no hashing and no clearing per window
  const size_t n_inst = h->cfg.max_instances;
  if (h->plan_last.size() < n_inst + h->st.n_slots) h->plan_last.assign(n_inst + h->st.n_slots, {0u, 0u});
  auto next_stamp = [h]() {
    if (++h->plan_stamp == 0) {  // wrapped: forget every entry
      std::fill(h->plan_last.begin(), h->plan_last.end(), std::make_pair(0u, 0u));
      h->plan_stamp = 1;
    }
    return h->plan_stamp;
  };
  uint32_t stamp = next_stamp();
  if (!msg && h->n_cmds >= (1u << 16)) {
    // the common window addresses every instance once: claim the subjects on the worker threads
    // (an atomic stamp exchange each); a repeat falls through to the ordered pass below, with a
    // fresh stamp
    std::atomic<bool> repeat{false};
    const size_t n = h->n_cmds;
    parallel_for(host_threads(), [&](unsigned t, unsigned TT) {
      for (size_t i = n * t / TT; i < n * (t + 1) / TT; ++i) {
        auto& e = h->plan_last[h->h_cmds[i].instance];  // bounds: validate()
        if (__atomic_exchange_n(&e.first, stamp, __ATOMIC_RELAXED) == stamp) {
          repeat = true;
          return;
        }
      }
    });
    if (!repeat) return ZBHIP_OK;  // one round: identity order
    stamp = next_stamp();
  }
  std::vector<uint32_t>& round_of = h->plan_round;
  if (round_of.size() < h->n_cmds) round_of.resize(h->n_cmds);
  uint32_t max_round = 0, epoch = 0;
  int cls = -1;
  for (size_t i = 0; i < h->n_cmds; ++i) {
    const bool sk = slot_kind(h->h_cmds[i].kind);
    if (msg && cls >= 0 && (int)sk != cls && i > 0) {
      epoch = max_round + 1;
      stamp = next_stamp();
    }
    cls = (int)sk;
    auto& e = h->plan_last[(sk ? n_inst : 0) + h->h_cmds[i].instance];  // bounds: validate()
    if (!msg && e.first == stamp && h->h_cmds[i].kind == ZBHIP_CMD_CREATE) return ZBHIP_EINVAL;
    const uint32_t r = e.first == stamp ? e.second + 1 : epoch;
    e = {stamp, r};
    round_of[i] = r;
    max_round = std::max(max_round, r);
  }
  if (max_round == 0) return ZBHIP_OK;  // single round: identity order
  std::vector<uint32_t> cnt(max_round + 2, 0);
  for (size_t i = 0; i < h->n_cmds; ++i) cnt[round_of[i] + 1]++;
  for (size_t r = 1; r < cnt.size(); ++r) cnt[r] += cnt[r - 1];
  h->round_begin.assign(cnt.begin(), cnt.end());
  h->h_order.resize(h->n_cmds);
  std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1);
  for (size_t i = 0; i < h->n_cmds; ++i) h->h_order[pos[round_of[i]]++] = (uint32_t)i;
  return ZBHIP_OK;
}

static int validate(zbhip_handle* h, const zbhip_command* cmds, size_t n, size_t n_docs,
                    const zbhip_xpart_cmd* xp, size_t n_xp) {
  for (size_t i = 0; i < n; ++i) {
    const zbhip_command& c = cmds[i];
    if (slot_kind(c.kind) || zb_pms_kind(c.kind)) {
      if (!h->msg()) return ZBHIP_EUNSUPP;
      if (c.doc_count) return ZBHIP_EINVAL;
      if (slot_kind(c.kind) ? c.instance >= h->st.n_slots : c.instance >= h->cfg.max_instances) return ZBHIP_EINVAL;
      if (c.kind == ZBHIP_CMD_PUBLISH) {
        if (c.ref >= h->names.size() || c.instance >= h->strs.size()) return ZBHIP_EINVAL;
      } else {
        if (c.doc_begin >= n_xp || xp[c.doc_begin].kind != c.kind) return ZBHIP_EINVAL;
      }
      continue;
    }
    if (c.instance >= h->cfg.max_instances) return ZBHIP_EINVAL;
    if (c.kind == ZBHIP_CMD_CREATE) {
      if (c.ref >= h->procs.size()) return ZBHIP_EINVAL;
      // the slot's instance still has follow-ups waiting in the log: it is not free yet
      if (!h->deferred_per_inst.empty() && h->deferred_per_inst.count(c.instance)) return ZBHIP_EINVAL;
    } else if (c.kind == ZBHIP_CMD_JOB_COMPLETE) {
      if (c.ref >= 0xFFF0) return ZBHIP_EINVAL;
    } else if (c.kind == ZBHIP_CMD_TIMER_TRIGGER) {
      if (c.ref >= 0xFFF0 || c.doc_count) return ZBHIP_EINVAL;  // doc_begin | pad << 32 = dueDate
      continue;
    } else if (c.kind == ZBHIP_CMD_CONTINUE) {
      // a deferred continuation read back from the log: known id, its own instance, no document
      if (!h->defer() || c.doc_count) return ZBHIP_EINVAL;
      auto it = h->deferred.find((uint64_t)c.doc_begin | ((uint64_t)c.pad << 32));
      if (it == h->deferred.end() || it->second.instance != c.instance) return ZBHIP_EINVAL;
      continue;
    } else {
      return ZBHIP_EINVAL;
    }
    if (c.doc_count && (size_t)c.doc_begin + c.doc_count > n_docs) return ZBHIP_EINVAL;
  }
  return ZBHIP_OK;
}

// uploads the Java hashCodes of strings interned since the last run
static int sync_strings(zbhip_handle* h) {
  if (h->d_str_n == h->strs.size()) return ZBHIP_OK;
  if (h->strs.size() > h->d_str_cap) {
    size_t cap = std::max<size_t>(1024, h->strs.size() * 2);
    uint32_t* d = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&d), cap * sizeof(uint32_t)) != hipSuccess) return ZBHIP_ENOMEM;
    if (h->d_str_n)
      HIPCHK(hipMemcpyAsync(d, h->d_str_hash, h->d_str_n * sizeof(uint32_t), hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    (void)hipFree(h->d_str_hash);
    h->d_str_hash = d;
    h->d_str_cap = cap;
  }
  HIPCHK(hipMemcpyAsync(h->d_str_hash + h->d_str_n, h->str_hash.data() + h->d_str_n,
                        (h->strs.size() - h->d_str_n) * sizeof(uint32_t), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->d_str_n = h->strs.size();
  return ZBHIP_OK;
}

int zbhip_submit(zbhip_handle* h, const zbhip_command* cmds, size_t n, const zbhip_doc_entry* docs, size_t n_docs) {
  return zbhip_submit_ex(h, cmds, n, docs, n_docs, nullptr, 0);
}

int zbhip_submit_ex(zbhip_handle* h, const zbhip_command* cmds, size_t n, const zbhip_doc_entry* docs, size_t n_docs,
                    const zbhip_xpart_cmd* xparts, size_t n_xparts) {
  if (!h || (n && !cmds) || (n_docs && !docs) || (n_xparts && !xparts)) return ZBHIP_EINVAL;
  if (n > h->cfg.max_commands || n_docs > h->cfg.max_doc_entries || n_xparts > h->cfg.max_commands) return ZBHIP_ENOMEM;
  const bool dbg = h->debug;
  auto now = [] { return std::chrono::steady_clock::now(); };
  const auto t0 = now();
  // the previous submit's uploads read the handle's staging buffers: done before they are rewritten
  // (a run in between has waited for them already; two submits in a row wait here)
  if (int rc0 = resolve_guard(h)) return rc0;  // the last window's speculative check
  if (h->upload_ev) HIPCHK(hipEventSynchronize(h->upload_ev));
  int rc = settle(h);  // the previous window's keys are fixed before its commands are replaced
  if (rc) return rc;
  const auto t1 = now();
  // validation, then the host copy, on the worker threads by ranges (a refused window leaves the
  // handle as it was); the first failing command's code wins, as in one pass
  std::atomic<bool> continues_any{false};
  {
    // one pass over the caller's commands: each block validated, then copied (into the next
    // window's pinned buffer, swapped in once the whole window validated: a refused window leaves the
    // handle as it was)
    const unsigned T = n >= (1u << 16) ? host_threads() : 1u;
    std::vector<std::pair<size_t, int>> fail(T, {~(size_t)0, ZBHIP_OK});
    h->h_cmds_next.resize(n);
    zbhip_command* const dst = h->h_cmds_next.data();
    parallel_for(T, [&](unsigned t, unsigned TT) {
      const size_t lo = n * t / TT, hi = n * (t + 1) / TT;
      bool cont = false;
      for (size_t b = lo; b < hi; b += 4096) {
        const size_t e = std::min(hi, b + 4096);
        if (validate(h, cmds + b, e - b, n_docs, xparts, n_xparts) != ZBHIP_OK) {
          for (size_t i = b; i < e; ++i)  // the block's first failing command
            if (int ri = validate(h, cmds + i, 1, n_docs, xparts, n_xparts)) {
              fail[t] = {i, ri};
              return;
            }
        }
        memcpy(dst + b, cmds + b, (e - b) * sizeof(zbhip_command));
        for (size_t i = b; i < e; ++i) cont |= cmds[i].kind == ZBHIP_CMD_CONTINUE;
      }
      if (cont) continues_any = true;
    });
    for (const auto& f : fail)
      if (f.second) return f.second;  // ranges in log order: the first range's failure is the first
    h->external = false;
    h->h_cmds.swap(h->h_cmds_next);
  }
  bool continues = continues_any.load();
  if (continues) {
    // duplicates of one id in a window are refused before anything is consumed
    std::unordered_map<uint64_t, int> seen;
    for (const auto& c : h->h_cmds)
      if (c.kind == ZBHIP_CMD_CONTINUE && seen[(uint64_t)c.doc_begin | ((uint64_t)c.pad << 32)]++) return ZBHIP_EINVAL;
  }
  h->h_docs.assign(docs, docs + n_docs);
  h->h_xparts.assign(xparts, xparts + n_xparts);
  h->n_xparts = n_xparts;
  h->ext_xparts = nullptr;
  if (n_xparts)  // (from the handle's copy: the caller's buffers are free once this returns)
    HIPCHK(hipMemcpyAsync(h->d_xparts, h->h_xparts.data(), n_xparts * sizeof(zbhip_xpart_cmd), hipMemcpyHostToDevice,
                          h->stream));
  h->n_cmds = n;
  h->n_docs = n_docs;
  const auto t2 = now();
  // the host has the window: its subjects are claimed on the host threads (no device round trip)
  rc = plan_rounds(h);
  if (rc) {
    h->n_cmds = h->n_docs = h->n_xparts = 0;
    return rc;
  }
  const auto t3 = now();
  h->doc_base = h->next_doc_base;
  h->next_doc_base += (int64_t)n_docs;
  h->source_base = h->next_source;
  h->next_source += (int64_t)n;
  if (continues) {
    // each continuation becomes the CMD_FOLLOWUP batch it was deferred as (the kernel runs it
    // against the instance's state at this log position, as the reference does when it reads the
    // command back)
    for (auto& c : h->h_cmds) {
      if (c.kind != ZBHIP_CMD_CONTINUE) continue;
      auto it = h->deferred.find((uint64_t)c.doc_begin | ((uint64_t)c.pad << 32));
      c = it->second;
      h->deferred.erase(it);
      auto pi = h->deferred_per_inst.find(c.instance);
      if (pi != h->deferred_per_inst.end() && --pi->second == 0) h->deferred_per_inst.erase(pi);
    }
    cmds = h->h_cmds.data();
  }
  h->window_continues = continues;
  if (n) HIPCHK(hipMemcpyAsync(h->d_cmds, h->h_cmds.data(), n * sizeof(zbhip_command), hipMemcpyHostToDevice, h->stream));
  if (n_docs)
    HIPCHK(hipMemcpyAsync(h->d_docs, h->h_docs.data(), n_docs * sizeof(zbhip_doc_entry), hipMemcpyHostToDevice,
                          h->stream));
  if (!h->h_order.empty())
    HIPCHK(hipMemcpyAsync(h->d_order, h->h_order.data(), n * 4, hipMemcpyHostToDevice, h->stream));
  // no wait here: the uploads read only the handle's own buffers (h_cmds pinned, h_docs, h_xparts,
  // h_order), which the next submit rewrites after waiting on this event
  if (!h->upload_ev) HIPCHK(hipEventCreateWithFlags(&h->upload_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(h->upload_ev, h->stream));
  h->ran = false;
  h->results = false;
  if (dbg) {
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr, "[zbhip] submit n=%zu: finalize %.2f ms, validate+copy %.2f ms, plan %.2f ms, upload %.2f ms\n", n,
            ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, now()));
  }
  return ZBHIP_OK;
}

int zbhip_submit_device(zbhip_handle* h, const zbhip_command* dev_cmds, size_t n, const zbhip_doc_entry* dev_docs,
                        size_t n_docs) {
  return zbhip_submit_device_ex(h, dev_cmds, n, dev_docs, n_docs, nullptr, 0);
}

static int replan_device_window(zbhip_handle* h, const zbhip_command* dev_cmds, size_t n, const zbhip_doc_entry* dev_docs,
                                size_t n_docs, const zbhip_xpart_cmd* dev_xparts, size_t n_xparts, bool* replanned);

// The subject check's verdict of the last checked window: its marker in host-mapped memory (stamp << 2
// | flags: the window's guarded k_step, or k_check_publish, writes it); a spin, bounded by the stream's
// own completion (a device fault ends it)
static int64_t read_check_marker(zbhip_handle* h) {
  const volatile uint32_t* m = h->h_check_flag;
  const uint32_t want = h->guard_stamp & 0x3FFFFFFFu;
  for (uint32_t spin = 0; (*m >> 2) != want; ++spin) {
    if (spin > (1u << 16)) {  // slow: let the runtime wait for the stream instead
      HIPCHK(hipStreamSynchronize(h->stream));
      if ((*m >> 2) != want) return ZBHIP_EDEVICE;
      break;
    }
  }
  return *m & 3u;
}

// The flag of a speculatively checked device window (check_device_window): read once, before anything
// depends on the window.  Clean: nothing to do.  A repeated subject: the guarded launch did nothing; the
// window is replanned on the host and run again with its run flags (before any later window).  A subject
// out of range: the window is refused (nothing of it ran) and this call reports ZBHIP_EINVAL.
static int resolve_guard(zbhip_handle* h) {
  if (h->guard_armed) {  // submitted, never run: a new submit replaces it
    h->guard_armed = false;
    return ZBHIP_OK;
  }
  if (!h->guard_pending) return ZBHIP_OK;
  h->guard_pending = false;
  const int64_t fl = read_check_marker(h);
  if (fl < 0) return (int)fl;
  const uint32_t flag = (uint32_t)fl;
  if (!flag) return ZBHIP_OK;
  const auto w = h->guard_win;
  h->next_doc_base = w.doc_base;  // the window's log positions and documents are given again
  h->next_source = w.source_base;
  h->ran = false;
  h->results = false;
  h->n_cmds = 0;
  if (flag & 2) return ZBHIP_EINVAL;
  bool replanned = false;
  if (int rc = replan_device_window(h, w.cmds, w.n, w.docs, w.n_docs, w.xparts, w.n_xparts, &replanned)) return rc;
  const int rc = zbhip_run(h, w.run_flags);
  return rc < 0 ? rc : ZBHIP_OK;
}

// A device window's subjects are checked on the device (k_subject_check): a window that addresses
// one subject twice is copied to the host and planned into rounds like a host window (so it runs
// in log order per subject); a subject out of range refuses the window.  Handles opened with
// ZBHIP_OPEN_TRUSTED_DEVICE_WINDOWS skip the check (the caller guarantees one command per subject).
static int check_device_window(zbhip_handle* h, const zbhip_command* dev_cmds, size_t n, const zbhip_doc_entry* dev_docs,
                               size_t n_docs, const zbhip_xpart_cmd* dev_xparts, size_t n_xparts, bool* replanned) {
  *replanned = false;
  if ((h->cfg.flags & ZBHIP_OPEN_TRUSTED_DEVICE_WINDOWS) || n == 0) return ZBHIP_OK;
  // (on the handle's stream: in order after whatever produced the window)
  hipStream_t cs = h->stream;
  if (++h->check_stamp >= (1u << 30)) {  // (30-bit stamps: the guard word's and the marker's)
    HIPCHK(hipMemsetAsync(h->d_seen, 0, ((size_t)h->cfg.max_instances + h->st.n_slots) * sizeof(uint32_t), cs));
    HIPCHK(hipMemsetAsync(h->d_check_flag, 0, 4 * sizeof(uint32_t), cs));
    h->check_stamp = 1;
  }
  if (!h->h_check_flag) {  // the host-mapped completion marker (stamp << 2 | flags)
    if (hipHostMalloc(reinterpret_cast<void**>(&h->h_check_flag), sizeof(uint32_t), hipHostMallocMapped) != hipSuccess)
      return ZBHIP_ENOMEM;
    *h->h_check_flag = 0;
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->d_check_host), h->h_check_flag, 0));
  }
  HIPCHK(launch_subject_check(reinterpret_cast<const uint4*>(dev_cmds), (uint32_t)n, h->cfg.max_instances, h->st.n_slots,
                              h->d_seen, h->check_stamp, h->d_check_flag + 2, cs));
  h->guard_win = {dev_cmds, n, dev_docs, n_docs, dev_xparts, n_xparts, h->next_doc_base, h->next_source, 0};
  h->guard_stamp = h->check_stamp;
  if (!h->msg() && !getenv("ZBHIP_SYNC_SUBJECT_CHECK")) {
    // speculative: nobody waits now; the run launches its k_step guarded by the device's verdict
    // (resolve_guard reads the marker later)
    h->guard_armed = true;
    return ZBHIP_OK;
  }
  HIPCHK(launch_check_publish(h->d_check_flag + 2, h->check_stamp, h->d_check_host, cs));
  int64_t flag = read_check_marker(h);
  if (flag < 0) return (int)flag;
  if (flag & 2) return ZBHIP_EINVAL;
  if (!(flag & 1)) return ZBHIP_OK;
  return replan_device_window(h, dev_cmds, n, dev_docs, n_docs, dev_xparts, n_xparts, replanned);
}

// the window copied to the host and submitted as a host window (planned into rounds in log order)
static int replan_device_window(zbhip_handle* h, const zbhip_command* dev_cmds, size_t n, const zbhip_doc_entry* dev_docs,
                                size_t n_docs, const zbhip_xpart_cmd* dev_xparts, size_t n_xparts, bool* replanned) {
  std::vector<zbhip_command> c(n);
  std::vector<zbhip_doc_entry> d(n_docs);
  std::vector<zbhip_xpart_cmd> x(n_xparts);
  HIPCHK(hipMemcpy(c.data(), dev_cmds, n * sizeof(zbhip_command), hipMemcpyDeviceToHost));
  if (n_docs) HIPCHK(hipMemcpy(d.data(), dev_docs, n_docs * sizeof(zbhip_doc_entry), hipMemcpyDeviceToHost));
  if (n_xparts) HIPCHK(hipMemcpy(x.data(), dev_xparts, n_xparts * sizeof(zbhip_xpart_cmd), hipMemcpyDeviceToHost));
  *replanned = true;
  return zbhip_submit_ex(h, c.data(), n, d.data(), n_docs, x.data(), n_xparts);
}

int zbhip_submit_device_ex(zbhip_handle* h, const zbhip_command* dev_cmds, size_t n, const zbhip_doc_entry* dev_docs,
                           size_t n_docs, const zbhip_xpart_cmd* dev_xparts, size_t n_xparts) {
  if (!h || (n && !dev_cmds)) return ZBHIP_EINVAL;
  if (n > h->rec_slots) return ZBHIP_ENOMEM;
  if (int rc0 = resolve_guard(h)) return rc0;  // the last window's speculative check
  if (h->upload_ev) HIPCHK(hipEventSynchronize(h->upload_ev));  // (h_order is rewritten by the planning)
  if (int rc0 = settle(h)) return rc0;
  bool replanned = false;
  const int rc = check_device_window(h, dev_cmds, n, dev_docs, n_docs, dev_xparts, n_xparts, &replanned);
  if (rc || replanned) return rc;
  h->external = true;
  h->window_continues = false;  // (ZBHIP_CMD_CONTINUE is a host-window command)
  h->ext_xparts = dev_xparts;
  h->n_xparts = n_xparts;
  h->h_xparts.clear();
  h->ext_cmds = reinterpret_cast<const uint4*>(dev_cmds);
  h->ext_docs = dev_docs;
  h->h_cmds.clear();
  h->h_docs.clear();
  h->n_cmds = n;
  h->n_docs = n_docs;
  h->round_begin.clear();
  h->h_order.clear();
  h->order_on_device = false;
  // a message partition's window in subject order (one round: its subjects are distinct) -- opt-in
  // until measured (ZBHIP_SUBJECT_SORT=1)
  const char* sort_env = getenv("ZBHIP_SUBJECT_SORT");  // (its value: the smallest window sorted)
  if (h->msg() && sort_env && n >= (size_t)std::max(1, atoi(sort_env))) {
    const size_t cap = h->cfg.max_commands;
    if (!h->d_sort) {
      h->sort_temp_bytes = subject_sort_temp_bytes((uint32_t)cap);
      if (dalloc(&h->d_sort, 3 * cap) != hipSuccess || hipMalloc(&h->d_sort_temp, h->sort_temp_bytes + 256) != hipSuccess)
        return ZBHIP_ENOMEM;
    }
    HIPCHK(launch_subject_sort(reinterpret_cast<const uint4*>(dev_cmds), (uint32_t)n, h->cfg.max_instances,
                               h->cfg.max_instances + h->st.n_slots, h->d_sort, h->d_sort + cap, h->d_sort + 2 * cap,
                               h->d_order, h->d_sort_temp, h->sort_temp_bytes, h->stream));
    h->round_begin = {0u, (uint32_t)n};
    h->order_on_device = true;
  }
  h->doc_base = h->next_doc_base;
  h->next_doc_base += (int64_t)n_docs;
  h->source_base = h->next_source;
  h->next_source += (int64_t)n;
  h->ran = false;
  h->results = false;
  return ZBHIP_OK;
}

static hipEvent_t next_event(zbhip_handle* h) {
  if (h->tev_used == h->tev.size()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    h->tev.push_back(e);
  }
  return h->tev[h->tev_used++];
}

// record offset of every command of the last run in the gathered records: regions follow launch
// order, lanes follow the launch order
static int compute_offsets(zbhip_handle* h) {
  if (h->off_ready) return ZBHIP_OK;
  if (h->order_on_device) {  // the launch order of a subject-sorted device window
    h->h_order.resize(h->round_begin.empty() ? 0 : h->round_begin.back());
    if (!h->h_order.empty())
      HIPCHK(hipMemcpy(h->h_order.data(), h->d_order, h->h_order.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    h->order_on_device = false;
  }
  const uint32_t n = (uint32_t)h->n_cmds;
  const uint64_t total = h->out_total;
  h->h_off.resize(n + 1);
  uint64_t off = 0;
  if (h->launches.size() == 1 && h->launches[0].src == 0 && n >= (1u << 16)) {
    // one launch in log order: a prefix sum of the record counts, by ranges on host threads
    const unsigned T = host_threads();
    std::vector<uint64_t> part(T + 1, 0);
    parallel_for(T, [&](unsigned t, unsigned TT) {
      uint64_t sum = 0;
      for (size_t c = (size_t)n * t / TT; c < (size_t)n * (t + 1) / TT; ++c) sum += h->h_hdr[c].x & 0xFFFF;
      part[t + 1] = sum;
    });
    for (unsigned t = 0; t < T; ++t) part[t + 1] += part[t];
    parallel_for(T, [&](unsigned t, unsigned TT) {
      uint64_t o = part[t];
      for (size_t c = (size_t)n * t / TT; c < (size_t)n * (t + 1) / TT; ++c) {
        h->h_off[c] = o;
        o += h->h_hdr[c].x & 0xFFFF;
      }
    });
    off = part[T];
  } else {
    for (const auto& l : h->launches)
      for (uint32_t k = 0; k < l.count; ++k) {
        const uint32_t c = l.src == 0 ? l.first + k : l.src == 1 ? h->h_order[l.first + k] : h->cont_order[l.first + k];
        h->h_off[c] = off;
        off += h->h_hdr[c].x & 0xFFFF;
      }
  }
  h->h_off[n] = 0;
  if (off != total) return ZBHIP_EDEVICE;
  h->off_ready = true;
  return ZBHIP_OK;
}

// the last run's records in host memory (ZBHIP_RUN_DEVICE_RECORDS left them in HBM)
static int ensure_out(zbhip_handle* h) {
  if (int rc = compute_offsets(h)) return rc;
  if (h->out_host) return ZBHIP_OK;
  h->h_out.resize(h->out_total);
  if (h->out_total)
    HIPCHK(hipMemcpy(h->h_out.data(), h->d_rec, h->out_total * sizeof(uint2), hipMemcpyDeviceToHost));
  h->out_host = true;
  return ZBHIP_OK;
}

// JOB_ACTIVATABLE bookkeeping of one processed command from its records: JOB:CREATED adds a job,
// JOB:COMPLETED removes it (its ACTIVATED entry is dropped at the next window)
static void track_jobs(zbhip_handle* h, size_t c, uint32_t inst) {
  const uint32_t nrec = h->h_hdr[c].x & 0xFFFF;
  const uint2* rows = h->h_out.data() + h->h_off[c];
  const uint16_t proc = inst < h->inst_proc.size() ? h->inst_proc[inst] : NONE;
  if (proc == NONE || proc >= h->procs.size()) return;
  const Proc& P = h->procs[proc];
  uint32_t task_ord = NONE;
  for (uint32_t i = 0; i < nrec; ++i) {
    const uint2 w = rows[i];
    const uint32_t elem = w.y & 0xFFFF, code = (w.y >> 16) & 0x3F;
    if (h->msg() && elem != NONE && (elem & kPayloadBit)) {  // message record + payload rows
      i += kPayloadRows;
      continue;
    }
    if (((w.y >> 16) & kRejectBit) ||
        (code != C_JOB_CREATED && code != C_JOB_COMPLETED && code != C_JOB_CANCELED && code != C_JOB_PUSHED) ||
        elem >= P.els.size())
      continue;
    const uint32_t tid = P.job_type_id[elem];
    if (code == C_JOB_PUSHED) {  // publishWork: the job ACTIVATED with the stream's deadline and worker
      const int64_t jk = h->key_of(inst, w.x >> 16);
      const auto st = h->run_streams.find(tid);
      if (h->job_index_on) h->job_index.erase({tid, jk});
      if (st == h->run_streams.end()) continue;
      zbhip_handle::Activation& a = h->activated[jk];
      a.deadline = h->run_clock_ms + st->second.timeout;
      a.worker = st->second.worker;
      a.inst = inst;
      a.worker_id = st->second.worker_id;
      a.state = zbhip_handle::JS_ACTIVATED;
      a.eik = h->key_of(inst, task_ord);
      a.pik = h->key_of(inst, 0);
      a.proc = (int32_t)proc;
      a.elem = (int32_t)elem;
      continue;
    }
    const int64_t key = h->key_of(inst, w.x & 0xFFFF);
    if (code == C_JOB_CREATED) task_ord = w.x >> 16;  // (its element instance: a push follows)
    if (code == C_JOB_CREATED) {
      if (h->job_index_on) h->job_index[{tid, key}] = {inst, (uint16_t)(w.x & 0xFFFF)};
    } else {
      if (h->job_index_on) h->job_index.erase({tid, key});
      auto it = h->activated.find(key);
      if (it != h->activated.end()) {  // gone (the drain still reads its deadline and worker)
        it->second.state = zbhip_handle::JS_GONE;
        h->completed_activated.push_back(key);
      }
    }
  }
}

// the window's fallback key declarations, cleared on first use after a run (a window without fallback
// commands never reads them)
static void ensure_ext(zbhip_handle* h) {
  if (h->ext_ready) return;
  const size_t n = h->n_cmds;
  h->ext_keys.resize(n);
  h->declared.resize(n);
  if (n >= (1u << 16)) {
    parallel_for(host_threads(), [&](unsigned t, unsigned T) {
      const size_t lo = n * t / T, hi = n * (t + 1) / T;
      std::fill(h->ext_keys.begin() + lo, h->ext_keys.begin() + hi, 0);
      std::fill(h->declared.begin() + lo, h->declared.begin() + hi, 0);
    });
  } else {
    std::fill(h->ext_keys.begin(), h->ext_keys.end(), 0);
    std::fill(h->declared.begin(), h->declared.end(), 0);
  }
  h->ext_ready = true;
}

// The whole bookkeeping of a plain window at once (no message subjects, no job index): key bases
// in log order (a sequential prefix), then the per-instance histories, processes and generations on
// host threads -- each thread owns the instances i % T == t and walks the window in log order, so
// every instance sees its commands in order -- and the resolve table filled at precomputed places.
static void advance_window_parallel(zbhip_handle* h) {
  const size_t n = h->n_cmds;
  const unsigned T = host_threads();
  // key bases and resolve-table positions in log order: per-range sums, then each range from its base
  std::vector<int64_t> kbase(T + 1, 0);
  std::vector<size_t> bbase(T + 1, 0);
  auto range = [n](unsigned t, unsigned TT) { return std::make_pair(n * t / TT, n * (t + 1) / TT); };
  const uint32_t N = h->cfg.max_instances;
  // a resolve-table entry for every processed command with keys whose subject is an instance slot
  // (the entries are written at these places below; none is left unwritten)
  auto has_entry = [h, N](size_t c, uint2 hd) { return (hd.x >> 16) != 0 && h->h_cmds[c].instance < N; };
  parallel_for(T, [&](unsigned t, unsigned TT) {
    int64_t k = 0;
    size_t b = 0;
    const auto [lo, hi] = range(t, TT);
    for (size_t c = lo; c < hi; ++c) {
      const uint2 hd = h->h_hdr[c];
      if (((hd.y >> 16) & 0xFF) == ST_OK) {
        k += hd.x >> 16;
        b += has_entry(c, hd);
      } else {
        k += h->ext_keys[c];
      }
    }
    kbase[t + 1] = k;
    bbase[t + 1] = b;
  });
  kbase[0] = h->key_counter;
  for (unsigned t = 0; t < T; ++t) {
    kbase[t + 1] += kbase[t];
    bbase[t + 1] += bbase[t];
  }
  BatchRef* const tbl = h->batches.append_segment(bbase[T]);
  // one subject per command in a one-round window: every range updates its own instances; with
  // rounds, each thread owns the instances i % T == t and walks the window in log order
  const bool one_round = h->round_begin.empty() && h->cont_cmds.empty();
  auto apply = [&](size_t c, size_t bpos, size_t& dead) {
    const zbhip_command& cm = h->h_cmds[c];
    const uint32_t inst = cm.instance;
    const uint2 hd = h->h_hdr[c];
    const uint32_t nkeys = hd.x >> 16, first = hd.y & 0xFFFF;
    if (cm.kind == ZBHIP_CMD_CREATE) {  // a new instance in the slot: its own key history
      h->hist[inst].clear();
      h->inst_proc[inst] = cm.ref;
      ++h->inst_gen[inst];
    }
    if (nkeys) {
      h->hist[inst].push_back({(uint16_t)first, h->h_base[c] + 1});
      tbl[bpos] = {h->h_base[c] + 1, inst, (uint16_t)first, (uint16_t)nkeys, h->inst_gen[inst]};
    }
    if (hd.y & HDR_ENDED) {  // completed: its job keys no longer resolve
      ++h->inst_gen[inst];
      dead += h->hist[inst].size();  // (summed per thread: no shared counter in the loop)
    }
  };
  std::vector<uint32_t> bpos(one_round ? 0 : n, ~0u);
  parallel_for(T, [&](unsigned t, unsigned TT) {
    int64_t kc = kbase[t];
    size_t nb = bbase[t], dead = 0;
    const auto [lo, hi] = range(t, TT);
    for (size_t c = lo; c < hi; ++c) {
      const uint2 hd = h->h_hdr[c];
      h->h_base[c] = kc;
      const bool ok = ((hd.y >> 16) & 0xFF) == ST_OK;
      kc += ok ? (int64_t)(hd.x >> 16) : h->ext_keys[c];
      if (!ok) continue;
      if (h->h_cmds[c].instance >= N) continue;
      const size_t here = nb;
      nb += has_entry(c, hd);
      if (!one_round) {
        bpos[c] = (uint32_t)here;
      } else {
        apply(c, here, dead);
      }
    }
    h->batches_dead.fetch_add(dead, std::memory_order_relaxed);
  });
  if (!one_round) {
    parallel_for(T, [&](unsigned t, unsigned TT) {
      size_t dead = 0;
      for (size_t c = 0; c < n; ++c) {
        const uint32_t inst = h->h_cmds[c].instance;
        if (inst >= N || inst % TT != t || bpos[c] == ~0u) continue;
        apply(c, bpos[c], dead);
      }
      h->batches_dead.fetch_add(dead, std::memory_order_relaxed);
    });
  }
  h->key_counter = kbase[T];
  h->fin_next = n;
}

// One journaled window into the host tables (the per-instance histories, processes and generations,
// and a resolve-table segment), as advance_window_parallel books a one-round window: each command
// is the only one of its instance, so ranges of commands go to host threads.  The current window's
// key bases are set too.
static void fold_journal(zbhip_handle* h, const uint4* e, size_t n, bool current) {
  const unsigned T = host_threads();
  const uint32_t N = h->cfg.max_instances;
  auto range = [n](unsigned t, unsigned TT) { return std::make_pair(n * t / TT, n * (t + 1) / TT); };
  auto has_entry = [N](const uint4& x) { return (x.w & 0xFFFF) != 0 && (x.z & 0x7FFFFFFFu) < N; };
  std::vector<size_t> bbase(T + 1, 0);
  parallel_for(T, [&](unsigned t, unsigned TT) {
    size_t b = 0;
    const auto [lo, hi] = range(t, TT);
    for (size_t c = lo; c < hi; ++c) b += has_entry(e[c]);
    bbase[t + 1] = b;
  });
  for (unsigned t = 0; t < T; ++t) bbase[t + 1] += bbase[t];
  BatchRef* const tbl = h->batches.append_segment(bbase[T]);
  if (current) h->h_base.resize(std::max(h->h_base.size(), n));
  parallel_for(T, [&](unsigned t, unsigned TT) {
    size_t nb = bbase[t], dead = 0;
    const auto [lo, hi] = range(t, TT);
    for (size_t c = lo; c < hi; ++c) {
      const uint4 x = e[c];
      const int64_t base = (int64_t)((uint64_t)x.x | (uint64_t)(x.y & 0xFFFF) << 32);
      const uint16_t first = (uint16_t)(x.y >> 16), nkeys = (uint16_t)(x.w & 0xFFFF), proc = (uint16_t)(x.w >> 16);
      const uint32_t inst = x.z & 0x7FFFFFFFu;
      if (current) h->h_base[c] = base - 1;
      if (inst >= N) continue;
      if (proc != 0xFFFF) {  // a CREATE: a new instance in the slot, its own key history
        h->hist[inst].clear();
        h->inst_proc[inst] = proc;
        ++h->inst_gen[inst];
      }
      if (nkeys) {
        h->hist[inst].push_back({first, base});
        tbl[nb++] = {base, inst, first, nkeys, h->inst_gen[inst]};
      }
      if (x.z >> 31) {  // the batch ended the instance: its keys no longer resolve
        ++h->inst_gen[inst];
        dead += h->hist[inst].size();
      }
    }
    h->batches_dead.fetch_add(dead, std::memory_order_relaxed);
  });
  if (h->batches.size() >= 2 * h->batches_compacted + (1u << 20) && 3 * h->batches_dead.load() >= h->batches.size()) {
    h->batches.compact([h](const BatchRef& b) { return b.gen == h->inst_gen[b.inst]; });
    h->batches_compacted = h->batches.size();
    h->batches_dead = 0;
  }
}

// every journaled window into the host tables, oldest first (keep: windows left journaled)
static int fold_journals(zbhip_handle* h, size_t keep = 0) {
  if (h->jrn_q.size() <= keep) return ZBHIP_OK;
  const size_t subjects = (size_t)h->cfg.max_instances + h->st.n_slots;
  if (h->hist.size() < subjects) {
    h->hist.resize(subjects);
    h->inst_gen.resize(subjects, 0);
  }
  if (h->inst_proc.size() < h->cfg.max_instances) h->inst_proc.resize(h->cfg.max_instances, NONE);
  while (h->jrn_q.size() > keep) {
    const zbhip_handle::JournalWindow j = h->jrn_q.front();
    h->jrn_host.resize(j.n);
    if (j.n)
      HIPCHK(hipMemcpy(h->jrn_host.data(), h->d_jrn + (size_t)j.slot * h->cfg.max_commands, j.n * sizeof(uint4),
                       hipMemcpyDeviceToHost));
    fold_journal(h, h->jrn_host.data(), j.n, h->results && j.window == h->windows_run);
    h->jrn_q.pop_front();
  }
  return ZBHIP_OK;
}

// The multi-instance collection records of window command c (instance `inst`), in log order: the
// values their expansion gives them (mi_rec: the device writes no list) and the host's copy of every
// body's outputCollection (mi_out) and of the propagated ones (outlist_var) -- kernels.hip C_MI_*.
static int track_mi(zbhip_handle* h, size_t c, uint32_t inst) {
  auto mi_fail = [&](int site) {
    if (getenv("ZBHIP_DEBUG_MI")) fprintf(stderr, "[track_mi] command %zu instance %u: site %d\n", c, inst, site);
    return (int)ZBHIP_EDEVICE;
  };
  const uint32_t nrec = h->h_hdr[c].x & 0xFFFF;
  const uint2* rows = h->h_out.data() + h->h_off[c];
  const uint16_t proc = inst < h->inst_proc.size() ? h->inst_proc[inst] : NONE;
  if (proc == NONE || proc >= h->procs.size()) return ZBHIP_OK;
  const Proc& P = h->procs[proc];
  for (uint32_t i = 0; i < nrec; ++i) {
    const uint2 w = rows[i];
    const uint32_t code = (w.y >> 16) & 0xFF, c6 = code & 0x3F, fl = w.y >> 24;
    if (code & kRejectBit) continue;
    const uint32_t key_ord = w.x & 0xFFFF, aux_ord = w.x >> 16, elem = w.y & 0xFFFF;
    const uint64_t at = ((uint64_t)c << 16) | i;
    if (c6 == C_MI_LIST_ITEM) {  // the C_MI_LOOP row that follows: the scope, the body, the loop counter
      uint32_t j = i + 1;
      while (j < nrec && ((rows[j].y >> 16) & 0x3F) != C_MI_LOOP) ++j;
      if (j >= nrec) return mi_fail(1);
      const uint32_t body = rows[j].y & 0xFFFF, loop = rows[j].y >> 24, list = aux_ord | (elem << 16);
      const Proc::Mi* m = P.mi_body(body);
      if (!m || list >= h->lists.size() || loop < 1 || loop > h->lists[list].size()) return mi_fail(2);
      const auto& it = h->lists[list][loop - 1];
      h->mi_rec[at] = {h->key_of(inst, key_ord), h->key_of(inst, rows[j].x >> 16), (int32_t)m->input_name,
                       (uint8_t)ZBHIP_VAR_CREATED, it.first, it.second};
    } else if (c6 == C_MI_OUTEL) {  // the outputElement variable, nil
      const Proc::Mi* m = P.mi_body(elem);
      if (!m) return mi_fail(3);
      h->mi_rec[at] = {h->key_of(inst, key_ord), h->key_of(inst, aux_ord), (int32_t)m->out_elem,
                       (uint8_t)ZBHIP_VAR_CREATED, (uint8_t)ZBHIP_DOC_NIL, 0};
    } else if (c6 == C_MI_OUT) {
      const Proc::Mi* m = P.mi_body(elem);
      if (!m) return mi_fail(4);
      const int64_t body_key = h->key_of(inst, aux_ord);
      uint8_t intent = ZBHIP_VAR_CREATED;
      if (fl & 0x80) {  // initializeOutputCollection: [nil] * n
        auto& o = h->mi_out[body_key];
        o.var_key = h->key_of(inst, key_ord);
        o.items.assign(fl & 0x7F, {(uint8_t)ZBHIP_DOC_NIL, 0});
      } else {  // updateOutputCollection: the item at index key_ord
        auto f = h->mi_out.find(body_key);
        const size_t slot = (fl >> 4) & 3, vat = slot * h->cfg.max_commands + c;
        if (f == h->mi_out.end() || key_ord >= f->second.items.size() || c >= h->cfg.max_commands ||
            vat >= h->h_map_val.size())
          return mi_fail(5);
        f->second.items[key_ord] = {(uint8_t)(fl & 7), (fl & 7) == ZBHIP_DOC_NIL ? 0 : (int64_t)h->h_map_val[vat]};
        intent = ZBHIP_VAR_UPDATED;
      }
      const auto& o = h->mi_out[body_key];
      const int64_t id = intern_items(h, o.items);
      if (id < 0) return (int)id;
      h->mi_rec[at] = {o.var_key, body_key, (int32_t)m->out_coll, intent, (uint8_t)ZBHIP_DOC_LIST, id};
    } else if (c6 == C_MI_PROP) {  // propagateVariable: created in the process instance's scope, or
      // (flags 1) the variable there updated
      const Proc::Mi* m = P.mi_body(elem);
      auto f = h->mi_out.find(h->key_of(inst, aux_ord));
      if (!m || f == h->mi_out.end()) return mi_fail(6);
      const int64_t id = intern_items(h, f->second.items);
      if (id < 0) return (int)id;
      const int64_t vk = h->key_of(inst, key_ord);
      h->outlist_var[vk] = (uint32_t)id;
      h->mi_rec[at] = {vk, h->key_of(inst, 0), (int32_t)m->out_coll,
                       (uint8_t)(fl & 1 ? ZBHIP_VAR_UPDATED : ZBHIP_VAR_CREATED), (uint8_t)ZBHIP_DOC_LIST, id};
    } else if ((c6 == ZBHIP_PI_ELEMENT_COMPLETED || c6 == ZBHIP_PI_ELEMENT_TERMINATED) && elem < P.els.size() &&
               P.els[elem].element_type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
      h->mi_out.erase(h->key_of(inst, key_ord));  // the body's variables leave with it
    }
  }
  return ZBHIP_OK;
}

// Key relabelling bookkeeping of the last run, in log (source) order: each command's first key
// (DbKeyGenerator order), the subjects' key histories and the resolve_key table.  It advances
// lazily, command by command: up to `limit`, and never past a fallback command whose CPU-engine keys
// were not declared yet (zbhip_set_external_keys), unless `force` (then it generated none) -- so the
// adapter can hand a fallback instance over (its earlier commands' keys are fixed) and declare the
// keys the CPU engine generated before the keys of the window's later commands are fixed.
static int advance(zbhip_handle* h, size_t limit, bool force) {
  if (int rc = resolve_guard(h)) return rc;
  if (int rc = fold_journals(h)) return rc;
  if (!h->results || h->fin_next >= h->n_cmds) return ZBHIP_OK;
  ensure_ext(h);
  if (h->fin_next == 0) {  // a new window: jobs completed in the previous one are gone
    for (int64_t k : h->completed_activated) h->activated.erase(k);
    h->completed_activated.clear();
    h->mi_rec.clear();
  }
  if (h->job_index_on || !h->activated.empty() || !h->streams.empty() || h->mi_ext)
    if (int rc = ensure_out(h)) return rc;
  const size_t subjects = (size_t)h->cfg.max_instances + h->st.n_slots;
  if (h->hist.size() < subjects) {
    h->hist.resize(subjects);
    h->inst_proc.resize(h->cfg.max_instances, NONE);
    h->inst_gen.resize(subjects, 0);
  }
  const size_t n = std::min(limit, h->n_cmds);
  if (h->fin_next == 0 && n == h->n_cmds && !h->msg() && !h->job_index_on && h->activated.empty() &&
      h->streams.empty() && !h->mi_ext && n >= (1u << 16)) {
    bool all_declared = true;  // the whole window can be done now (fallback keys declared, or forced)
    if (!force)
      for (size_t c = 0; c < n && all_declared; ++c)
        all_declared = ((h->h_hdr[c].y >> 16) & 0xFF) == ST_OK || h->declared[c];
    if (all_declared) advance_window_parallel(h);
  }
  for (size_t c = h->fin_next; c < n; ++c) {
    const uint2 hd = h->h_hdr[c];
    const zbhip_command& cm = h->h_cmds[c];
    const uint32_t nkeys = hd.x >> 16, first = hd.y & 0xFFFF;
    if (((hd.y >> 16) & 0xFF) != ST_OK) {  // processed by the CPU engine: the keys it declared
      if (!h->declared[c] && !force) return ZBHIP_OK;
      h->h_base[c] = h->key_counter;
      h->key_counter += h->ext_keys[c];
      h->fin_next = c + 1;
      continue;
    }
    h->h_base[c] = h->key_counter;
    h->fin_next = c + 1;
    if (h->msg() && slot_kind(cm.kind)) {
      // the correlation slot's keys first, then the instance a local command loaded
      const uint4 h2 = h->h_hdr2[c];
      const uint32_t nsec = h2.y >> 16, nprim = nkeys - nsec;
      const uint32_t subj = h->slot_subject(cm.instance);
      if (nprim) {
        h->hist[subj].push_back({(uint16_t)first, h->key_counter + 1});
        h->batches.push_back({h->key_counter + 1, subj, (uint16_t)first, (uint16_t)nprim, h->inst_gen[subj]});
      }
      if (nsec) {
        h->hist[h2.x].push_back({(uint16_t)(h2.y & 0xFFFF), h->key_counter + 1 + nprim});
        h->batches.push_back({h->key_counter + 1 + nprim, h2.x, (uint16_t)(h2.y & 0xFFFF), (uint16_t)nsec, h->inst_gen[h2.x]});
      }
      if ((h->job_index_on || !h->activated.empty() || !h->streams.empty()) && h2.x < h->cfg.max_instances)
        track_jobs(h, c, h2.x);
      if ((hd.y & HDR_ENDED) && h2.x < h->cfg.max_instances) {
        ++h->inst_gen[h2.x];
        h->batches_dead.fetch_add(h->hist[h2.x].size(), std::memory_order_relaxed);
      }
      h->key_counter += nkeys;
      continue;
    }
    if (cm.kind == ZBHIP_CMD_CREATE) {  // a new instance in the slot: its own key history
      h->hist[cm.instance].clear();
      h->inst_proc[cm.instance] = cm.ref;
      ++h->inst_gen[cm.instance];
    }
    if (nkeys) {
      h->hist[cm.instance].push_back({(uint16_t)first, h->key_counter + 1});
      h->batches.push_back({h->key_counter + 1, cm.instance, (uint16_t)first, (uint16_t)nkeys, h->inst_gen[cm.instance]});
    }
    if (h->job_index_on || !h->activated.empty() || !h->streams.empty()) track_jobs(h, c, cm.instance);
    if (h->mi_ext)
      if (int rc = track_mi(h, c, cm.instance)) return rc;
    if (hd.y & HDR_ENDED) {  // completed: its job keys no longer resolve
      ++h->inst_gen[cm.instance];
      h->batches_dead.fetch_add(h->hist[cm.instance].size(), std::memory_order_relaxed);
    }
    h->key_counter += nkeys;
  }
  if (h->fin_next < h->n_cmds) return ZBHIP_OK;
  // window done: drop the key-table entries of ended / replaced instances once they outnumber the rest
  // (once ended instances' entries are a third of the table: a scan that finds nothing is not paid for)
  if (h->batches.size() >= 2 * h->batches_compacted + (1u << 20) && 3 * h->batches_dead.load() >= h->batches.size()) {
    h->batches.compact([h](const BatchRef& b) { return b.gen == h->inst_gen[b.inst]; });
    h->batches_compacted = h->batches.size();
    h->batches_dead = 0;
  }
  return ZBHIP_OK;
}

// the whole window (undeclared fallback commands generated no keys)
static int finalize(zbhip_handle* h) { return advance(h, ~(size_t)0, true); }

// before a new window replaces the last one's commands: its keys fixed -- booked here, or journaled
// on the device (left there)
static int settle(zbhip_handle* h) {
  if (!h->results || h->fin_next >= h->n_cmds) return ZBHIP_OK;
  return finalize(h);
}

int zbhip_set_clock(zbhip_handle* h, int64_t now_ms) {
  if (!h) return ZBHIP_EINVAL;
  h->clock_ms = now_ms;
  return ZBHIP_OK;
}

int zbhip_run(zbhip_handle* h, uint32_t flags) {
  if (!h) return ZBHIP_EINVAL;
  if (h->ran) return ZBHIP_ESTATE;
  if (h->procs.empty()) return ZBHIP_ESTATE;
  const uint32_t* guard = nullptr;
  if (h->guard_armed) {
    h->guard_armed = false;
    if (flags & ZBHIP_RUN_NO_RESULTS) {
      // speculative: k_step runs guarded by the check's flag; resolve_guard reads it later
      guard = h->d_check_flag + 2;  // the guard word (k_subject_check's faulty lanes raise it)
      h->guard_win.run_flags = flags;
      h->guard_pending = true;
    } else {
      // results are read back in this call anyway: decide now
      HIPCHK(launch_check_publish(h->d_check_flag + 2, h->guard_stamp, h->d_check_host, h->stream));
      const int64_t fl = read_check_marker(h);
      if (fl < 0) return (int)fl;
      const uint32_t flag = (uint32_t)fl;
      if (flag) {
        const auto w = h->guard_win;
        h->next_doc_base = w.doc_base;
        h->next_source = w.source_base;
        if (flag & 2) {
          h->n_cmds = 0;
          return ZBHIP_EINVAL;
        }
        bool replanned = false;
        if (int rc = replan_device_window(h, w.cmds, w.n, w.docs, w.n_docs, w.xparts, w.n_xparts, &replanned)) return rc;
      }
    }
  }
  if (h->ring_filled != h->windows_run) h->ring_ok = false;  // the previous window's keys are not in the ring
  ++h->windows_run;
  const bool timed = flags & ZBHIP_RUN_TIMED;
  const bool want = !(flags & ZBHIP_RUN_NO_RESULTS);
  const bool accumulate = flags & ZBHIP_RUN_ACCUMULATE;
  const uint32_t n = (uint32_t)h->n_cmds;
  const uint32_t B = step_block(h->variant);
  // fence stamp of this window (0 and 0xFFFFFFFF are never stamps: open-time values of hdr.w and
  // slot_hdr.y); on wrap-around every stale stamp is cleared first
  if (++h->window_stamp == 0xFFFFFFFFu) {
    HIPCHK(hipMemset2DAsync(reinterpret_cast<char*>(h->st.hdr) + 12, sizeof(uint4), 0, 4, h->st.n, h->stream));
    if (h->st.n_slots)
      HIPCHK(hipMemset2DAsync(reinterpret_cast<char*>(h->st.slot_hdr) + 4, sizeof(uint2), 0, 4, h->st.n_slots, h->stream));
    h->window_stamp = 1;
  }
  if (!accumulate) {
    HIPCHK(hipMemsetAsync(h->d_stats, 0, 64 * 8 * sizeof(unsigned long long), h->stream));
    h->tev_used = 0;
  }

  StepParams P{};
  P.cmds = h->external ? h->ext_cmds : h->d_cmds;
  P.docs = h->external ? h->ext_docs : h->d_docs;
  P.n_docs = (uint32_t)h->n_docs;
  P.prog = h->d_prog;
  P.prog_words = (uint32_t)h->prog.size();
  P.n_procs = (uint32_t)h->procs.size();
  P.st = h->st;
  P.rec_cap = h->rec_cap;
  P.region_stride = B * h->rec_cap + h->region_pad;
  P.out = h->d_regions;
  P.region_total = h->d_region_total;
  P.region_lanes = h->d_region_lanes;
  P.cmd_hdr = h->d_cmd_hdr;
  P.stats = h->d_stats;
  P.max_cmds_in_batch = h->cfg.max_commands_in_batch;
  P.stamp = h->window_stamp;
  P.now_ms = h->clock_ms;
  // the straight-line KScope / KGeneric batches (ZBHIP_NO_FAST_SCOPE=1: the general path, for A/B)
  P.no_fast_scope = getenv("ZBHIP_NO_FAST_SCOPE") ? 1u : 0u;
  P.cmd_due = h->d_cmd_due;
  P.map_val = h->d_map_val;
  P.map_cap = h->cfg.max_commands;
  P.cmd_act = h->st.act ? h->d_cmd_act : nullptr;
  P.guard = guard;
  P.guard_stamp = h->guard_stamp & 0x3FFFFFFFu;
  P.guard_host = h->d_check_host;
  if (h->d_list_n != h->lists.size())
    if (int rc = sync_lists(h)) return rc;
  P.list_hdr = h->d_list_hdr;
  P.list_val = h->d_list_val;
  P.list_type = h->d_list_type;
  P.n_lists = (uint32_t)h->d_list_n;
  h->run_clock_ms = h->clock_ms;
  if (!h->streams.empty() || !h->run_streams.empty()) h->run_streams = h->streams;  // (the pushes' deadlines / workers)
  P.tpl = (h->variant == 0 || h->variant == 1 || h->scope_variant()) && !getenv("ZBHIP_NO_TEMPLATES") ? h->d_tpl : nullptr;
  if (h->msg()) {
    int rc = sync_strings(h);
    if (rc) return rc;
    P.xparts = h->external ? h->ext_xparts : h->d_xparts;
    P.n_xparts = (uint32_t)h->n_xparts;
    P.str_hash = h->d_str_hash;
    P.n_strs = (uint32_t)h->d_str_n;
    P.cmd_hdr2 = h->d_cmd_hdr2;
    P.xout = h->d_xout;
    P.xcap = (uint32_t)h->cfg.max_commands;
    P.partition_id = h->cfg.partition_id;
    P.partition_count = std::max(1, h->cfg.partition_count);
  }

  // launches: one per round (commands of one instance are serialised in log order)
  h->launches.clear();
  uint32_t region = 0;
  auto add_launch = [&](uint32_t first, uint32_t count, uint8_t src) {
    h->launches.push_back({region, first, count, src});
    region += (count + B - 1) / B;
  };
  if (h->round_begin.empty()) {
    if (n) add_launch(0, n, 0);
  } else {
    for (size_t r = 0; r + 1 < h->round_begin.size(); ++r)
      add_launch(h->round_begin[r], h->round_begin[r + 1] - h->round_begin[r], 1);
  }
  if (region > h->regions_cap || (size_t)region * P.region_stride > h->region_records)
    return ZBHIP_ENOMEM;  // too many rounds for the region pool
  // follow-up commands past the batch limit (not for message partitions: their local commands
  // carry context the log entry would need -> FB_BATCH_LIMIT); batch FIFO spill for fan-outs
  // larger than the LDS ring
  const bool overflow = h->may_overflow && !h->msg();
  if (overflow) {
    P.ovf = h->d_ovf;
    P.ovf_count = h->d_ovf_count;
    P.ovf_cap = h->ovf_cap;
  }
  if (h->max_pending > step_queue(h->variant) && h->variant != 3 && !getenv("ZBHIP_CHUNKS_PER_WG")) {
    const uint32_t cap = h->max_pending;
    const size_t words = (size_t)step_resident(h->variant, P.prog_words) * B * cap;
    if (words > h->qspill_words) {
      (void)hipFree(h->d_qspill);
      h->d_qspill = nullptr;
      h->qspill_words = 0;
      if (dalloc(&h->d_qspill, words) != hipSuccess) return ZBHIP_ENOMEM;
      h->qspill_words = words;
    }
    P.qspill = h->d_qspill;
    P.qspill_cap = cap;
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (timed) {
    e0 = next_event(h);
    e1 = next_event(h);
    if (!e0 || !e1) return ZBHIP_EDEVICE;
    HIPCHK(hipEventRecord(e0, h->stream));
  }
  for (const auto& l : h->launches) {
    P.order = l.src == 0 ? nullptr : h->d_order + l.first;
    P.n_launch = l.count;
    P.region_base = l.region;
    P.launch_seq = ++h->launch_seq;
    HIPCHK(launch_step(h->variant, P, h->stream));
  }
  // continuation: the follow-up commands written to the log unprocessed become batches of their
  // own after the window, in the order written (source command, then record ordinal); theirs may
  // overflow again
  uint32_t n_all = n;
  h->cont_cmds.clear();
  h->cont_order.clear();
  h->last_cont_first = h->next_cont_id;
  h->last_cont_n = 0;
  h->cont_ids.clear();
  std::vector<uint2> hdr_tmp;
  if (overflow && h->defer()) {
    // deferred: the follow-ups written unprocessed wait for their own log positions
    uint32_t cnt = 0;
    HIPCHK(hipMemcpyAsync(&cnt, h->d_ovf_count, sizeof cnt, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    // entries past the list's capacity were not written: their batches fell back (FB_BATCH_LIMIT)
    cnt = std::min(cnt, h->ovf_cap);
    if (cnt) {
      std::vector<uint4> ov(cnt);
      HIPCHK(hipMemcpy(ov.data(), h->d_ovf, cnt * sizeof(uint4), hipMemcpyDeviceToHost));
      HIPCHK(hipMemsetAsync(h->d_ovf_count, 0, sizeof(uint32_t), h->stream));
      hdr_tmp.resize(n);
      HIPCHK(hipMemcpy(hdr_tmp.data(), h->d_cmd_hdr, n * sizeof(uint2), hipMemcpyDeviceToHost));
      ov.erase(std::remove_if(ov.begin(), ov.end(), [&](const uint4& e) {
                 return e.x >= n || ((hdr_tmp[e.x].y >> 16) & 0xFF) != ST_OK;
               }), ov.end());
      std::sort(ov.begin(), ov.end(), [](const uint4& a, const uint4& b) {
        return a.x != b.x ? a.x < b.x : (a.z & 0xFFFF) < (b.z & 0xFFFF);
      });
      for (const uint4& e : ov) {
        zbhip_command c{};
        c.instance = e.w;
        c.kind = CMD_FOLLOWUP;
        c.ref = (uint16_t)(e.z >> 16);
        c.doc_begin = e.y;
        h->cont_ids.emplace(((uint64_t)e.x << 16) | (e.z & 0xFFFF), h->next_cont_id);
        h->deferred.emplace(h->next_cont_id++, c);
        ++h->deferred_per_inst[c.instance];
      }
      h->last_cont_n = ov.size();
    }
  }
  while (overflow && !h->defer()) {
    uint32_t cnt = 0;
    HIPCHK(hipMemcpyAsync(&cnt, h->d_ovf_count, sizeof cnt, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    if (cnt == 0) break;
    cnt = std::min(cnt, h->ovf_cap);  // past the capacity: those batches fell back
    std::vector<uint4> ov(cnt);
    HIPCHK(hipMemcpy(ov.data(), h->d_ovf, cnt * sizeof(uint4), hipMemcpyDeviceToHost));
    HIPCHK(hipMemsetAsync(h->d_ovf_count, 0, sizeof(uint32_t), h->stream));
    hdr_tmp.resize(n_all);
    HIPCHK(hipMemcpy(hdr_tmp.data(), h->d_cmd_hdr, n_all * sizeof(uint2), hipMemcpyDeviceToHost));
    // entries of batches that fell back are void (their records were dropped)
    ov.erase(std::remove_if(ov.begin(), ov.end(), [&](const uint4& e) {
               return e.x >= n_all || ((hdr_tmp[e.x].y >> 16) & 0xFF) != ST_OK;
             }), ov.end());
    if (ov.empty()) break;
    std::sort(ov.begin(), ov.end(), [](const uint4& a, const uint4& b) {
      return a.x != b.x ? a.x < b.x : (a.z & 0xFFFF) < (b.z & 0xFFFF);
    });
    if ((size_t)n_all + ov.size() > h->cfg.max_commands) return ZBHIP_ENOMEM;
    // the continuation window: rounds so that an instance appears once per launch, in order
    const uint32_t first_new = (uint32_t)h->cont_cmds.size();
    std::unordered_map<uint32_t, uint32_t> rounds_of;
    std::vector<uint32_t> round(ov.size());
    uint32_t max_round = 0;
    for (size_t k = 0; k < ov.size(); ++k) {
      zbhip_command c{};
      c.instance = ov[k].w;
      c.kind = CMD_FOLLOWUP;
      c.ref = (uint16_t)(ov[k].z >> 16);
      c.doc_begin = ov[k].y;
      h->cont_cmds.push_back(c);
      round[k] = rounds_of[c.instance]++;
      max_round = std::max(max_round, round[k]);
    }
    HIPCHK(hipMemcpyAsync(h->d_cont + first_new, h->cont_cmds.data() + first_new, ov.size() * sizeof(zbhip_command),
                          hipMemcpyHostToDevice, h->stream));
    for (uint32_t r = 0; r <= max_round; ++r) {
      const uint32_t begin = (uint32_t)h->cont_order.size();
      for (size_t k = 0; k < ov.size(); ++k)
        if (round[k] == r) h->cont_order.push_back(n_all + (uint32_t)k);
      add_launch(begin, (uint32_t)h->cont_order.size() - begin, 2);
    }
    if (region > h->regions_cap || (size_t)region * P.region_stride > h->region_records) return ZBHIP_ENOMEM;
    HIPCHK(hipMemcpyAsync(h->d_cont_order, h->cont_order.data(), h->cont_order.size() * sizeof(uint32_t),
                          hipMemcpyHostToDevice, h->stream));
    P.cmds = reinterpret_cast<const uint4*>(h->d_cont);
    P.cmd_base = n;
    for (size_t l = h->launches.size() - (max_round + 1); l < h->launches.size(); ++l) {
      P.order = h->d_cont_order + h->launches[l].first;
      P.n_launch = h->launches[l].count;
      P.region_base = h->launches[l].region;
      P.launch_seq = ++h->launch_seq;
      HIPCHK(launch_step(h->variant, P, h->stream));
    }
    n_all += (uint32_t)ov.size();
  }
  h->next_source += (int64_t)(n_all - n);  // the continuation batches' log positions follow
  if (h->msg()) {
    // keys of the window in log order: real process-instance keys, outbox and slot-row references
    HIPCHK(launch_keyscan(h->d_cmd_hdr, h->d_cmd_hdr2, P.cmds, n, h->d_key_blk, h->d_key_base, h->d_key_counter,
                          h->d_xout, (uint32_t)h->cfg.max_commands, h->st, (long long)h->cfg.partition_id << 51,
                          h->stream));
    h->bucketed = false;
    h->outbox_taken = false;
  }
  if (timed) HIPCHK(hipEventRecord(e1, h->stream));
  h->stats.launches = (uint32_t)h->launches.size();
  h->stats.rounds = (uint32_t)h->launches.size();
  h->n_regions = region;
  h->ran = true;
  h->drain_cmd = 0;
  h->drain_rec = 0;
  h->drain_ord = 0;
  h->results = false;

  if (!want) {
    // benchmarking mode: nothing is copied back and nothing waits; keys are not relabelled
    h->relabel_ok = false;
    h->stats_dirty = true;
    h->n_cmds = n_all;
    return (int)n_all;
  }
  if (h->external) {
    // a device-resident window with results (e.g. an exchange inbox in drain mode): the host
    // bookkeeping below reads the window's commands, documents and received commands
    h->h_cmds.resize(n);
    h->h_docs.resize(h->n_docs);
    h->h_xparts.resize(h->n_xparts);
    if (n) HIPCHK(hipMemcpyAsync(h->h_cmds.data(), P.cmds, n * sizeof(zbhip_command), hipMemcpyDeviceToHost, h->stream));
    if (h->n_docs && P.docs)
      HIPCHK(hipMemcpyAsync(h->h_docs.data(), P.docs, h->n_docs * sizeof(zbhip_doc_entry), hipMemcpyDeviceToHost, h->stream));
    if (h->n_xparts && h->ext_xparts)
      HIPCHK(hipMemcpyAsync(h->h_xparts.data(), h->ext_xparts, h->n_xparts * sizeof(zbhip_xpart_cmd),
                            hipMemcpyDeviceToHost, h->stream));
  }
  if (h->msg()) {
    HIPCHK(hipStreamSynchronize(h->stream));
    for (auto& c : h->h_cmds) h->published |= c.kind == ZBHIP_CMD_PUBLISH;
  }
  h->h_cmds.resize(n);
  h->h_cmds.insert(h->h_cmds.end(), h->cont_cmds.begin(), h->cont_cmds.end());
  h->n_cmds = n_all;
  {
  const uint32_t n = n_all;  // the window and its continuation batches

  // ---- results: headers + records gathered into log order (drain path, off the hot loop) ----
  auto now = [] { return std::chrono::steady_clock::now(); };
  const auto t0 = now();
  h->h_hdr.resize(n);
  if (n) HIPCHK(hipMemcpyAsync(h->h_hdr.data(), h->d_cmd_hdr, n * sizeof(uint2), hipMemcpyDeviceToHost, h->stream));
  // secondary headers: message partitions only (slot batches, outbox counts, payload rows)
  if (h->msg()) h->h_hdr2.assign(n, make_uint4(0, 0, 0, 0));
  else h->h_hdr2.clear();
  if (n && h->scope_variant()) {  // dueDates of canceled timers (TIMER:CANCELED values)
    h->h_cmd_due.resize(n);
    HIPCHK(hipMemcpyAsync(h->h_cmd_due.data(), h->d_cmd_due, n * sizeof(long long), hipMemcpyDeviceToHost, h->stream));
  }
  if (n && h->variant == 5) {  // io-mapped variable values (C_VAR_MAPPED records)
    const size_t m = std::min<size_t>(n, h->cfg.max_commands);
    h->h_map_val.resize((size_t)kMapVals * h->cfg.max_commands);
    HIPCHK(hipMemcpy2DAsync(h->h_map_val.data(), h->cfg.max_commands * sizeof(long long), h->d_map_val,
                            h->cfg.max_commands * sizeof(long long), m * sizeof(long long), kMapVals,
                            hipMemcpyDeviceToHost, h->stream));
  }
  if (n && h->msg())
    HIPCHK(hipMemcpyAsync(h->h_hdr2.data(), h->d_cmd_hdr2, n * sizeof(uint4), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(launch_gather(h->d_regions, h->d_region_total, h->d_region_lanes, region, h->d_region_off,
                       P.region_stride, B, step_rows(h->variant), h->d_rec, h->d_stats + 64 * 8, h->stream));
  unsigned long long total = 0;
  HIPCHK(hipMemcpyAsync(&total, h->d_stats + 64 * 8, sizeof total, hipMemcpyDeviceToHost, h->stream));
  // the statistics rows: this window's fallback count (whether every command ran on the device)
  unsigned long long srows[64 * 8];
  HIPCHK(hipMemcpyAsync(srows, h->d_stats, sizeof srows, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  {
    unsigned long long fb = 0;
    for (int r = 0; r < 64; ++r) fb += srows[r * 8 + 4];
    if (!accumulate) h->fb_seen = 0;
    h->window_fallbacks = fb - h->fb_seen;
    h->fb_seen = fb;
  }
  const auto t1 = now();
  h->out_total = total;
  h->out_host = false;
  h->h_out.clear();
  if (!(flags & ZBHIP_RUN_DEVICE_RECORDS)) {
    h->h_out.resize(total);
    if (total) HIPCHK(hipMemcpy(h->h_out.data(), h->d_rec, total * sizeof(uint2), hipMemcpyDeviceToHost));
    h->out_host = true;
  }
  h->stats_dirty = true;

  // record offset of every command (the host needs them to read records; with the records left in
  // HBM they are computed when a host reader first asks)
  h->off_ready = false;
  if (!(flags & ZBHIP_RUN_DEVICE_RECORDS))
    if (int rc = compute_offsets(h)) return rc;
  if (h->debug) {
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr, "[zbhip] run n=%u: kernels + headers + gather %.2f ms, records copy + offsets %.2f ms\n", n,
            ms(t0, t1), ms(t1, now()));
  }

  // fallback key declarations start empty (cleared when first read: ensure_ext); key bases are
  // written by advance() before any read
  h->ext_ready = false;
  h->h_base.resize(n);
  h->fin_next = 0;
  h->results = true;
  }
  return (int)n_all;
}

int64_t zbhip_pending_records(zbhip_handle* h) {
  if (!h || !h->results) return 0;
  int64_t pay = 0;
  for (auto& x : h->h_hdr2) pay += x.w;  // payload rows of message records
  return (int64_t)h->out_total - pay;
}

int zbhip_get_stats(zbhip_handle* h, zbhip_stats* out) {
  if (getenv("ZBHIP_STAMPS")) dump_stamps();
  if (!h || !out) return ZBHIP_EINVAL;
  if (int rc = resolve_guard(h)) return rc;
  if (h->stats_dirty) {
    unsigned long long rows[64 * 8];
    HIPCHK(hipMemcpyAsync(rows, h->d_stats, sizeof rows, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    unsigned long long c[8] = {0};
    for (int r = 0; r < 64; ++r)
      for (int k = 0; k < 8; ++k) c[k] += rows[r * 8 + k];
    h->stats.records = c[0];
    h->stats.transitions = c[1];
    h->stats.completed_instances = c[2];
    h->stats.keys = c[3];
    h->stats.fallback = c[4];
    h->stats.commands = c[5];
    h->stats.template_batches = c[6];
    double ms = 0;
    for (size_t i = 0; i + 1 < h->tev_used; i += 2) {
      float a = 0;
      if (hipEventElapsedTime(&a, h->tev[i], h->tev[i + 1]) == hipSuccess) ms += a;
    }
    h->stats.step_ms = ms;
    h->stats.compact_ms = 0;  // compaction is fused into k_step
    if (!h->relabel_ok) h->key_counter_approx = c[3];
    h->stats_dirty = false;
  }
  *out = h->stats;
  return ZBHIP_OK;
}

// message record codes -> (record type, value type, intent)
static bool message_code(uint32_t c6, zbhip_record& r) {
  switch (c6) {
    case C_PMS_CREATING: r.value_type = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_PMS_CREATING; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_PMS_CREATE: r.value_type = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_PMS_CREATE; r.record_type = ZBHIP_RT_COMMAND; return true;
    case C_PMS_CREATED: r.value_type = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_PMS_CREATED; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_PMS_CORRELATE: r.value_type = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_PMS_CORRELATE; r.record_type = ZBHIP_RT_COMMAND; return true;
    case C_PMS_CORRELATED: r.value_type = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_PMS_CORRELATED; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_MS_CREATE: r.value_type = ZBHIP_VT_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_MS_CREATE; r.record_type = ZBHIP_RT_COMMAND; return true;
    case C_MS_CREATED: r.value_type = ZBHIP_VT_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_MS_CREATED; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_MS_CORRELATING: r.value_type = ZBHIP_VT_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_MS_CORRELATING; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_MS_CORRELATE: r.value_type = ZBHIP_VT_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_MS_CORRELATE; r.record_type = ZBHIP_RT_COMMAND; return true;
    case C_MS_CORRELATED: r.value_type = ZBHIP_VT_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_MS_CORRELATED; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_PMS_DELETING: r.value_type = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_PMS_DELETING; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_PMS_DELETE: r.value_type = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_PMS_DELETE; r.record_type = ZBHIP_RT_COMMAND; return true;
    case C_PMS_DELETED: r.value_type = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_PMS_DELETED; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_MS_DELETE: r.value_type = ZBHIP_VT_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_MS_DELETE; r.record_type = ZBHIP_RT_COMMAND; return true;
    case C_MS_DELETED: r.value_type = ZBHIP_VT_MESSAGE_SUBSCRIPTION; r.intent = ZBHIP_MS_DELETED; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_MSG_PUBLISHED: r.value_type = ZBHIP_VT_MESSAGE; r.intent = ZBHIP_MSG_PUBLISHED; r.record_type = ZBHIP_RT_EVENT; return true;
    case C_MSG_EXPIRED: r.value_type = ZBHIP_VT_MESSAGE; r.intent = ZBHIP_MSG_EXPIRED; r.record_type = ZBHIP_RT_EVENT; return true;
    default: return false;
  }
}

static uint8_t rejection_type_of(uint32_t reason) {
  switch (reason) {
    case ZBHIP_REASON_JOB_NOT_FOUND:
    case ZBHIP_REASON_PMS_CREATE_NOT_FOUND:
    case ZBHIP_REASON_PMS_CORR_NOT_FOUND:
    case ZBHIP_REASON_MS_CORR_NOT_FOUND:
    case ZBHIP_REASON_TIMER_NOT_FOUND:
      return ZBHIP_REJ_NOT_FOUND;
    default:
      return ZBHIP_REJ_INVALID_STATE;
  }
}

static void stored_job_record(const zbhip_handle::Activation& a, int64_t key, uint8_t rt, uint8_t intent,
                              zbhip_record& r);

// One compact row of a plain (non-message) record -> zbhip_record: relabelled keys, record /
// value type and intent from the row code, document references.  Read-only on the handle, so the
// bulk drain runs it from several threads.
static int expand_plain(const zbhip_handle* h, size_t c, uint32_t inst, uint2 w, uint32_t ord, zbhip_record& r) {
  const zbhip_command& cm = h->h_cmds[c];
  const int64_t doc = cm.doc_count ? h->doc_base + cm.doc_begin : -1;
  const uint32_t key_ord = w.x & 0xFFFF, aux_ord = w.x >> 16, elem = w.y & 0xFFFF;
  const uint32_t code = (w.y >> 16) & 0xFF, fl = w.y >> 24;
  const bool rej = code & kRejectBit;
  const uint32_t c6 = code & 0x3F;
  const uint16_t proc = inst < h->inst_proc.size() ? h->inst_proc[inst] : NONE;
  r = zbhip_record{};
  r.source_index = h->source_base + (int64_t)c;
  r.rejection_type = ZBHIP_REJ_NONE;
  r.ordinal = (uint16_t)ord;
  r.aux = -1;
  r.message_key = -1;
  r.correlation_key = ZBHIP_NO_STRING;
  r.message_name = 0xFFFF;
  r.bpmn_process_id = 0xFFFF;
    r.key = h->key_of(inst, key_ord);
    r.scope_key = aux_ord == NONE ? -1 : h->key_of(inst, aux_ord);
    r.process_instance_key = h->key_of(inst, 0);
    r.process_idx = proc == NONE ? -1 : proc;
    r.element_idx = elem == NONE ? -1 : (int32_t)elem;
    r.reason = 0;
    r.reason_arg = 0;
    if (c6 >= 1 && c6 <= 10) {
      r.value_type = ZBHIP_VT_PROCESS_INSTANCE;
      r.intent = (uint8_t)c6;
      r.record_type = rej ? ZBHIP_RT_REJECTION : (c6 >= 8 ? ZBHIP_RT_COMMAND : ZBHIP_RT_EVENT);
      r.unprocessed = !rej && c6 >= 8 && (fl & F_UNPROCESSED) ? 1 : 0;
      if (r.unprocessed && !h->cont_ids.empty()) {  // deferred: the continuation's id
        auto it = h->cont_ids.find(((uint64_t)c << 16) | ord);
        if (it != h->cont_ids.end()) r.aux = (int64_t)it->second;
      }
    } else if (c6 == C_JOB_PUSHED) {
      // JOB_BATCH:ACTIVATED of a job stream's push: aux = the job, the job's fields as a JOB record's
      r.value_type = ZBHIP_VT_JOB_BATCH;
      r.intent = ZBHIP_JOB_BATCH_ACTIVATED;
      r.record_type = ZBHIP_RT_EVENT;
      r.aux = h->key_of(inst, aux_ord);
      auto it = h->activated.find(r.aux);
      if (it == h->activated.end()) return ZBHIP_EDEVICE;
      const zbhip_record k = r;
      stored_job_record(it->second, r.aux, ZBHIP_RT_EVENT, ZBHIP_JOB_BATCH_ACTIVATED, r);
      r.key = k.key;
      r.value_type = ZBHIP_VT_JOB_BATCH;
      r.aux = k.aux;
      r.source_index = k.source_index;
      r.ordinal = k.ordinal;
    } else if (c6 == C_JOB_CREATED || c6 == C_JOB_COMPLETED || c6 == C_JOB_COMPLETE || c6 == C_JOB_CANCELED) {
      r.value_type = ZBHIP_VT_JOB;
      r.intent = c6 == C_JOB_CREATED ? ZBHIP_JOB_CREATED : c6 == C_JOB_COMPLETED ? ZBHIP_JOB_COMPLETED
                 : c6 == C_JOB_CANCELED ? ZBHIP_JOB_CANCELED : ZBHIP_JOB_COMPLETE;
      r.record_type = rej ? ZBHIP_RT_REJECTION : ZBHIP_RT_EVENT;
      if (c6 == C_JOB_COMPLETED || c6 == C_JOB_COMPLETE) r.aux = doc;
      if (!rej && (fl & 1u) && (c6 == C_JOB_COMPLETED || c6 == C_JOB_CANCELED)) {
        // the stored job of an ACTIVATED job: its deadline and worker (DbJobState.activate)
        auto it = h->activated.find(r.key);
        if (it != h->activated.end()) {
          r.message_key = it->second.deadline;
          r.correlation_key = it->second.worker_id;
          if (it->second.fail_fields) {  // a failed job's retries and errorMessage
            r.reason_arg = 1;
            r.partition = it->second.retries;
            r.message_name = (uint16_t)(it->second.error_id & 0xFFFF);
            r.bpmn_process_id = (uint16_t)(it->second.error_id >> 16);
          }
        }
      }
    } else if (c6 == C_VAR_CREATED || c6 == C_VAR_UPDATED) {
      r.value_type = ZBHIP_VT_VARIABLE;
      r.intent = c6 == C_VAR_CREATED ? ZBHIP_VAR_CREATED : ZBHIP_VAR_UPDATED;
      r.record_type = ZBHIP_RT_EVENT;
      // the value comes from the batch's source document entry of that name
      for (uint32_t j = 0; j < cm.doc_count; ++j)
        if (h->h_docs[cm.doc_begin + j].name_id == elem) r.aux = h->doc_base + cm.doc_begin + j;
    } else if (c6 == C_MI_ITEM || c6 == C_MI_LOOP) {
      // MultiInstanceBodyProcessor.setLoopVariables: VARIABLE:CREATED in the inner instance's scope,
      // the value inline -- the body's item at loopCounter - 1, or loopCounter itself
      const Proc::Mi* m = proc != NONE ? h->procs[proc].mi_body(elem) : nullptr;
      if (!m || fl < 1 || (c6 == C_MI_ITEM && fl > m->items.size())) return ZBHIP_EDEVICE;
      r.value_type = ZBHIP_VT_VARIABLE;
      r.intent = ZBHIP_VAR_CREATED;
      r.record_type = ZBHIP_RT_EVENT;
      r.element_idx = c6 == C_MI_ITEM ? m->input_name : m->loop_name;
      r.aux = ZBHIP_AUX_INLINE;
      r.partition = c6 == C_MI_ITEM ? m->items[fl - 1].first : ZBHIP_DOC_INT;
      r.message_key = c6 == C_MI_ITEM ? m->items[fl - 1].second : (int64_t)fl;
    } else if (c6 == C_MI_LIST_ITEM || c6 == C_MI_OUTEL || c6 == C_MI_OUT || c6 == C_MI_PROP) {
      // multi-instance collection variables: their values from the log-order pass (track_mi)
      auto it = h->mi_rec.find(((uint64_t)c << 16) | ord);
      if (it == h->mi_rec.end()) {
        if (getenv("ZBHIP_DEBUG_MI")) fprintf(stderr, "[expand] command %zu ordinal %u: no multi-instance record\n", c, ord);
        return ZBHIP_EDEVICE;
      }
      const zbhip_handle::MiRec& m = it->second;
      r.key = m.key;
      r.scope_key = m.scope;
      r.element_idx = m.name;
      r.value_type = ZBHIP_VT_VARIABLE;
      r.intent = m.intent;
      r.record_type = ZBHIP_RT_EVENT;
      r.aux = ZBHIP_AUX_INLINE;
      r.partition = m.type;
      r.message_key = m.value;
    } else if (c6 == C_VAR_MAPPED) {
      // BpmnVariableMappingBehavior (behavior/BpmnVariableMappingBehavior.java:53-156): the value the
      // mapping computed, inline (its zbhip_doc_type in flags bits 0..2, its map_val slot in bit 4)
      const size_t slot = (fl >> 4) & 1;
      const size_t at = slot * h->cfg.max_commands + c;
      if (c >= h->cfg.max_commands || at >= h->h_map_val.size()) return ZBHIP_EDEVICE;
      r.value_type = ZBHIP_VT_VARIABLE;
      r.intent = (fl >> 3) & 1 ? ZBHIP_VAR_UPDATED : ZBHIP_VAR_CREATED;
      r.record_type = ZBHIP_RT_EVENT;
      r.aux = ZBHIP_AUX_INLINE;
      r.partition = (int32_t)(fl & 7);
      r.message_key = h->h_map_val[at];
    } else if (c6 == C_PIB_ACTIVATE) {
      // PROCESS_INSTANCE_BATCH:ACTIVATE (activateChildInstancesInBatches): batchElementInstanceKey =
      // the body (scope_key), index = its collection's size
      const Proc::Mi* m = proc != NONE ? h->procs[proc].mi_body(elem) : nullptr;
      if (!m) return ZBHIP_EDEVICE;
      r.value_type = ZBHIP_VT_PROCESS_INSTANCE_BATCH;
      r.intent = ZBHIP_PIB_ACTIVATE;
      r.record_type = ZBHIP_RT_COMMAND;
      r.partition = (int32_t)(fl & 0x3F);  // the collection's size (the row's flags)
      r.unprocessed = (fl & F_UNPROCESSED) ? 1 : 0;
      if (r.unprocessed && !h->cont_ids.empty()) {
        auto it = h->cont_ids.find(((uint64_t)c << 16) | ord);
        if (it != h->cont_ids.end()) r.aux = (int64_t)it->second;
      }
    } else if (c6 == C_PIB_TERMINATE) {
      // PROCESS_INSTANCE_BATCH:TERMINATE (terminateChildInstances): batchElementInstanceKey = the
      // container (scope_key), index -1
      r.value_type = ZBHIP_VT_PROCESS_INSTANCE_BATCH;
      r.intent = ZBHIP_PIB_TERMINATE;
      r.record_type = ZBHIP_RT_COMMAND;
      r.partition = -1;
      r.unprocessed = (fl & F_UNPROCESSED) ? 1 : 0;
      if (r.unprocessed) return ZBHIP_EDEVICE;  // (the kernel keeps terminations in their batch)
    } else if (c6 == C_PE_TRIGGERING || c6 == C_PE_TRIGGERED) {
      r.value_type = ZBHIP_VT_PROCESS_EVENT;
      r.intent = c6 == C_PE_TRIGGERING ? ZBHIP_PE_TRIGGERING : ZBHIP_PE_TRIGGERED;
      r.record_type = ZBHIP_RT_EVENT;
      r.aux = c6 == C_PE_TRIGGERING ? doc : -1;
    } else if (c6 == C_PIC_CREATED) {
      r.value_type = ZBHIP_VT_PROCESS_INSTANCE_CREATION;
      r.intent = ZBHIP_PIC_CREATED;
      r.record_type = ZBHIP_RT_EVENT;
      r.aux = doc;
    } else if (c6 == C_INCIDENT_CREATED) {
      // BpmnIncidentBehavior.createIncident: elementInstanceKey = variableScopeKey = the gateway's
      // (scope_key); the ErrorType in partition, the failing flow in aux, its result type in reason_arg
      const Proc* P = proc != NONE ? &h->procs[proc] : nullptr;
      if (!P || elem >= P->els.size()) return ZBHIP_EDEVICE;
      const zbhip_element& G = P->els[elem];
      const uint32_t pos = fl & 15;
      r.value_type = ZBHIP_VT_INCIDENT;
      r.intent = ZBHIP_INCIDENT_CREATED;
      r.record_type = ZBHIP_RT_EVENT;
      r.partition = pos == 15 ? ZBHIP_ERR_CONDITION_ERROR : ZBHIP_ERR_EXTRACT_VALUE_ERROR;
      if (pos != 15) {
        if (pos >= G.out_count || (size_t)G.out_begin + pos >= P->out.size()) return ZBHIP_EDEVICE;
        r.aux = P->out[G.out_begin + pos];
        r.reason_arg = (uint8_t)(fl >> 4);
      }
    } else if (c6 == C_TIMER_CANCELED) {
      // CatchEventBehavior.unsubscribeFromTimerEvent: the stored timer's dueDate (cmd_due)
      r.value_type = ZBHIP_VT_TIMER;
      r.intent = ZBHIP_TIMER_CANCELED;
      r.record_type = ZBHIP_RT_EVENT;
      r.aux = c < h->h_cmd_due.size() ? h->h_cmd_due[c] : -1;
      if (c < h->h_hdr.size()) {
        // a timer created in this batch and canceled in it: the clock plus its duration (as its
        // CREATED); cmd_due holds only the dueDate of a timer stored before the batch
        const uint32_t first = h->h_hdr[c].y & 0xFFFF, nkeys = h->h_hdr[c].x >> 16;
        const zbhip_element* E = proc != NONE && elem < h->procs[proc].els.size() ? &h->procs[proc].els[elem] : nullptr;
        if (E && nkeys && key_ord >= first && key_ord < first + nkeys) {
          // (an interrupting boundary event's cycle: the next timer TIMER:TRIGGER rescheduled before the
          // activity's termination canceled it -- due from the command's dueDate, as its CREATED)
          const bool next = cm.kind == ZBHIP_CMD_TIMER_TRIGGER && E->element_type == ZBHIP_EL_BOUNDARY_EVENT &&
                            (E->job_retries & 1) && (E->job_retries >> 8) != 1;
          const int64_t cmd_due = (int64_t)((uint64_t)cm.doc_begin | ((uint64_t)cm.pad << 32));
          r.aux = next ? next_cycle_due(cmd_due, (int64_t)E->duration_ms, h->run_clock_ms)
                       : h->run_clock_ms + (int64_t)E->duration_ms;
        }
      }
      r.partition = fl == 255 ? -1 : (int32_t)fl;  // TimerRecord.repetitions
    } else if (c6 == C_TIMER_CREATED || c6 == C_TIMER_NEXT || c6 == C_TIMER_TRIGGERED || c6 == C_TIMER_TRIGGER) {
      // TimerRecord: elementInstanceKey (scope_key), dueDate in aux -- CREATED: the run's clock plus
      // the element's duration (CatchEventBehavior.java:310); TRIGGERED / a rejected TRIGGER: the
      // command's TimerRecord (TriggerTimerProcessor.java:108: the TIMER:TRIGGER value)
      r.value_type = ZBHIP_VT_TIMER;
      r.intent = c6 == C_TIMER_CREATED || c6 == C_TIMER_NEXT ? ZBHIP_TIMER_CREATED
                 : c6 == C_TIMER_TRIGGERED ? ZBHIP_TIMER_TRIGGERED : ZBHIP_TIMER_TRIGGER;
      r.record_type = rej ? ZBHIP_RT_REJECTION : ZBHIP_RT_EVENT;
      const int64_t cmd_due = (int64_t)((uint64_t)cm.doc_begin | ((uint64_t)cm.pad << 32));
      const zbhip_element* E = proc != NONE && elem < h->procs[proc].els.size() ? &h->procs[proc].els[elem] : nullptr;
      // a cycle's next timer counts from the TRIGGER command's dueDate (refreshTimer), others from the clock
      const int64_t dur = E ? (int64_t)E->duration_ms : 0;
      r.aux = c6 == C_TIMER_CREATED ? h->run_clock_ms + dur
               : c6 == C_TIMER_NEXT ? next_cycle_due(cmd_due, dur, h->run_clock_ms) : cmd_due;
      if (!rej) r.partition = fl == 255 ? -1 : (int32_t)fl;  // TimerRecord.repetitions
    } else {
      return ZBHIP_EDEVICE;  // corrupt record
    }
    if (rej) {
      r.reason = fl & 0xF;
      r.reason_arg = fl >> 4;
      if (r.value_type == ZBHIP_VT_TIMER) {  // the TIMER:TRIGGER command's value
        r.rejection_type = rejection_type_of(r.reason);
        r.process_idx = -1;
        r.element_idx = -1;
        r.scope_key = -1;
        r.process_instance_key = -1;
      } else if (r.value_type == ZBHIP_VT_JOB) {
        r.rejection_type = ZBHIP_REJ_NOT_FOUND;
        r.process_idx = -1;
        r.element_idx = -1;
        r.scope_key = -1;
        r.process_instance_key = -1;
      } else {
        r.rejection_type = ZBHIP_REJ_INVALID_STATE;
      }
    }
  return ZBHIP_OK;
}

// Record drain_rec of window command c as a zbhip_record (ordinal ord), keys relabelled; advances
// rec past the row(s) it used (a message record and its payload rows) and ord by one.
static int expand_row(zbhip_handle* h, size_t c, size_t& rec, size_t& ord, zbhip_record& r) {
  const uint2 hd = h->h_hdr[c];
  const uint32_t nrec = hd.x & 0xFFFF;
  const zbhip_command& cm = h->h_cmds[c];
  // the instance the records refer to: the command's, or the one a message batch loaded
  const uint32_t inst = h->msg() && slot_kind(cm.kind) ? h->h_hdr2[c].x : cm.instance;
  const uint2* rows = h->h_out.data() + h->h_off[c];
  const uint2 w = rows[rec];
  const uint32_t elem = w.y & 0xFFFF;
  const uint32_t code = (w.y >> 16) & 0xFF, fl = w.y >> 24;
  const bool rej = code & kRejectBit;
  const uint32_t c6 = code & 0x3F;
  const uint16_t proc = inst < h->inst_proc.size() ? h->inst_proc[inst] : NONE;
  r = zbhip_record{};
  r.source_index = h->source_base + (int64_t)c;
  r.rejection_type = ZBHIP_REJ_NONE;
  r.ordinal = (uint16_t)ord;
  r.aux = -1;
  r.message_key = -1;
  r.correlation_key = ZBHIP_NO_STRING;
  r.message_name = 0xFFFF;
  r.bpmn_process_id = 0xFFFF;
  if (h->msg() && elem != NONE && (elem & kPayloadBit)) {
    // message record: 6 payload rows (kernels.hip emit_msg)
    if (rec + kPayloadRows >= nrec) return ZBHIP_EDEVICE;
    const uint2* pl = rows + rec + 1;
    auto ll = [](uint2 v) { return (long long)(((unsigned long long)v.y << 32) | v.x); };
    if (!message_code(c6, r)) return ZBHIP_EDEVICE;
    const uint32_t el = elem & 0xFFF;
    r.correlation_key = pl[0].x;
    r.message_name = (uint16_t)(pl[0].y & 0xFFFF);
    r.bpmn_process_id = (uint16_t)(pl[0].y >> 16);
    r.key = h->resolve_ref(ll(pl[1]));
    r.scope_key = h->resolve_ref(ll(pl[2]));
    r.process_instance_key = h->resolve_ref(ll(pl[3]));
    r.message_key = h->resolve_ref(ll(pl[4]));
    r.partition = (int32_t)(pl[5].x & 0xFFFF);
    r.interrupting = (uint8_t)(pl[5].x >> 16);
    r.element_idx = el == kNoElem ? -1 : (int32_t)el;
    r.process_idx = el == kNoElem || proc == NONE ? -1 : proc;
    if (rej) {
      r.record_type = ZBHIP_RT_REJECTION;
      r.reason = fl & 0xF;
      r.reason_arg = fl >> 4;
      r.rejection_type = rejection_type_of(r.reason);
    }
    rec += 1 + kPayloadRows;
    ++ord;
    return ZBHIP_OK;
  }
  if (int rc = expand_plain(h, c, inst, w, ord, r)) return rc;
  ++rec;
  ++ord;
  return ZBHIP_OK;
}

int zbhip_drain(zbhip_handle* h, zbhip_record* out, size_t cap, size_t* n_out) {
  if (!h || (cap && !out)) return ZBHIP_EINVAL;
  if (n_out) *n_out = 0;
  if (!h->results) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  if (int rc = ensure_out(h)) return rc;
  if (!h->msg() && h->drain_cmd == 0 && h->drain_rec == 0 && h->h_out.size() >= kBulkDrainMin &&
      cap >= h->h_out.size()) {
    // whole window at once: record i of command c goes to out[first(c) + i] (one row per record
    // without message payloads), so command ranges expand independently on host threads
    const size_t n = h->n_cmds;
    std::vector<size_t> first(n + 1, 0);
    for (size_t c = 0; c < n; ++c) first[c + 1] = first[c] + (h->h_hdr[c].x & 0xFFFF);
    if (first[n] != h->h_out.size()) return ZBHIP_EDEVICE;
    std::atomic<int> err{0};
    parallel_for(host_threads(), [&](unsigned t, unsigned T) {
      // commands split by record count, so every thread expands about total / T records
      const size_t lo = std::lower_bound(first.begin(), first.end(), first[n] * t / T) - first.begin();
      const size_t hi = std::lower_bound(first.begin(), first.end(), first[n] * (t + 1) / T) - first.begin();
      for (size_t c = lo; c < hi && c < n; ++c) {
        const uint2* rows = h->h_out.data() + h->h_off[c];
        const uint32_t nrec = h->h_hdr[c].x & 0xFFFF;
        for (uint32_t i = 0; i < nrec; ++i) {
          const int rc = expand_plain(h, c, h->h_cmds[c].instance, rows[i], i, out[first[c] + i]);
          if (rc) { err.store(rc); return; }
        }
      }
    });
    if (err.load()) return err.load();
    h->drain_cmd = n;
    if (n_out) *n_out = first[n];
    return ZBHIP_OK;
  }
  size_t k = 0;
  while (k < cap && h->drain_cmd < h->n_cmds) {
    const size_t c = h->drain_cmd;
    const uint2 hd = h->h_hdr[c];
    const uint32_t nrec = hd.x & 0xFFFF;
    if (h->drain_rec >= nrec) {
      ++h->drain_cmd;
      h->drain_rec = 0;
      h->drain_ord = 0;
      continue;
    }
    zbhip_record r;
    if (int rc = expand_row(h, c, h->drain_rec, h->drain_ord, r)) return rc;
    out[k++] = r;
  }
  if (n_out) *n_out = k;
  return ZBHIP_OK;
}

int zbhip_rejection_reason(zbhip_handle* h, const zbhip_record* r, char* buf, size_t cap) {
  if (!h || !r || !buf) return ZBHIP_EINVAL;
  return zbhip_serializer_rejection_reason(h->ser, r, buf, cap);
}

zbhip_serializer* zbhip_handle_serializer(zbhip_handle* h) { return h ? h->ser : nullptr; }

namespace {
struct DbExport {
  zbhip_serializer* ser;
  zbhip_db_sink sink;
  void* ctx;
  int rc;
};
void db_row(void* c, const char* row) {
  auto* e = static_cast<DbExport*>(c);
  const int r = zbhip_serializer_encode_state_row(e->ser, row, e->sink, e->ctx);
  if (r < 0 && e->rc == ZBHIP_OK) e->rc = r;
}
}  // namespace

int zbhip_export_state_db(zbhip_handle* h, zbhip_db_sink sink, void* ctx) {
  if (!h || !sink) return ZBHIP_EINVAL;
  DbExport e{h->ser, sink, ctx, ZBHIP_OK};
  const int rc = zbhip_export_state(h, db_row, &e);
  return rc < 0 ? rc : e.rc;
}

// The records of window command i only (a plain window: no message payloads), keys relabelled: the
// adapter emits a window command's batch when the platform reaches it, and keys of commands after a
// fallback command are fixed only once the CPU engine's keys for it are declared -- so this advances
// the key bookkeeping up to i without forcing (ZBHIP_ESTATE while an earlier fallback is undeclared).
int zbhip_drain_command(zbhip_handle* h, size_t i, zbhip_record* out, size_t cap, size_t* n_out) {
  if (!h || (cap && !out) || !n_out) return ZBHIP_EINVAL;
  *n_out = 0;
  if (!h->results) return ZBHIP_ESTATE;
  if (i >= h->n_cmds) return ZBHIP_EINVAL;
  if (int rc = advance(h, i + 1, false)) {
    if (getenv("ZBHIP_DEBUG_MI")) fprintf(stderr, "[drain_command] advance to %zu: %d\n", i + 1, rc);
    return rc;
  }
  if (h->fin_next <= i) return ZBHIP_ESTATE;
  if (int rc = ensure_out(h)) return rc;
  const uint32_t nrec = h->h_hdr[i].x & 0xFFFF;
  if (h->msg()) {  // message records span payload rows: count them first
    size_t need = 0;
    const uint2* rows = h->h_out.data() + h->h_off[i];
    for (uint32_t k = 0; k < nrec; ++need) {
      const uint32_t elem = rows[k].y & 0xFFFF;
      k += elem != NONE && (elem & kPayloadBit) ? 1 + kPayloadRows : 1;
    }
    if (cap < need) {
      *n_out = need;
      return ZBHIP_ENOMEM;
    }
    size_t rec = 0, ord = 0;
    for (size_t k = 0; k < need; ++k)
      if (int rc = expand_row(h, i, rec, ord, out[k])) return rc;
    *n_out = need;
    return ZBHIP_OK;
  }
  if (cap < nrec) {
    *n_out = nrec;
    return ZBHIP_ENOMEM;
  }
  const uint2* rows = h->h_out.data() + h->h_off[i];
  for (uint32_t k = 0; k < nrec; ++k)
    if (int rc = expand_plain(h, i, h->h_cmds[i].instance, rows[k], k, out[k])) {
      if (getenv("ZBHIP_DEBUG_MI"))
        fprintf(stderr, "[drain_command] command %zu row %u code %u flags %u elem %u: %d\n", i, k, (rows[k].y >> 16) & 0xFF,
                rows[k].y >> 24, rows[k].y & 0xFFFF, rc);
      return rc;
    }
  *n_out = nrec;
  return ZBHIP_OK;
}

int zbhip_resolve_key(zbhip_handle* h, int64_t key, uint32_t* instance, uint16_t* ordinal) {
  if (!h || !instance || !ordinal) return ZBHIP_EINVAL;
  // keys of commands after a fallback command whose CPU-engine keys are not declared yet resolve
  // once the window is drained
  if (int rc = advance(h, ~(size_t)0, false)) return rc;
  const int64_t v = key - ((int64_t)h->cfg.partition_id << 51);
  const BatchRef* it = h->batches.find(v);
  if (!it) return ZBHIP_EINVAL;
  if (v >= it->base + it->nkeys) return ZBHIP_EINVAL;
  if (it->inst < h->inst_gen.size() && it->gen != h->inst_gen[it->inst]) return ZBHIP_EINVAL;  // instance ended
  *instance = it->inst;
  *ordinal = (uint16_t)(it->first_ord + (v - it->base));
  return ZBHIP_OK;
}

// ---- value dictionary ------------------------------------------------------------------------
int64_t zbhip_intern_string(zbhip_handle* h, const char* bytes, size_t len) {
  if (!h || (len && !bytes)) return ZBHIP_EINVAL;
  std::string v(bytes ? bytes : "", len);
  auto it = h->str_ids.find(v);
  if (it != h->str_ids.end()) return it->second;
  if (h->strs.size() >= 0xFFFFFFF0u) return ZBHIP_ENOMEM;
  const uint32_t id = (uint32_t)h->strs.size();
  if (h->ser) zbhip_serializer_intern_string(h->ser, v.data(), v.size());
  h->str_hash.push_back((uint32_t)java_hash(v.data(), v.size()));
  h->strs.push_back(std::move(v));
  h->str_ids.emplace(h->strs.back(), id);
  return id;
}

static int64_t intern_items(zbhip_handle* h, const zbhip_handle::Items& v) {
  auto it = h->list_ids.find(v);
  if (it != h->list_ids.end()) return it->second;
  if (h->lists.size() >= 0x7FFFFFF0u) return ZBHIP_ENOMEM;
  const uint32_t id = (uint32_t)h->lists.size();
  h->list_hdr.push_back(make_uint2((uint32_t)h->list_val.size(), (uint32_t)v.size()));
  std::vector<zbhip_doc_entry> rows(v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    h->list_val.push_back(v[i].second);
    h->list_type.push_back(v[i].first);
    rows[i] = zbhip_doc_entry{};
    rows[i].type = v[i].first;
    rows[i].value = v[i].second;
  }
  if (h->ser) zbhip_serializer_intern_list(h->ser, rows.data(), rows.size());
  h->lists.push_back(v);
  h->list_ids.emplace(v, id);
  return id;
}

extern "C" int64_t zbhip_intern_list(zbhip_handle* h, const zbhip_doc_entry* items, size_t n) {
  if (!h || (n && !items)) return ZBHIP_EINVAL;
  zbhip_handle::Items v;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t t = items[i].type;
    if (t != ZBHIP_DOC_NIL && t != ZBHIP_DOC_BOOL && t != ZBHIP_DOC_INT && t != ZBHIP_DOC_DEC && t != ZBHIP_DOC_STR)
      return ZBHIP_EUNSUPP;  // nested lists / documents
    if (t == ZBHIP_DOC_STR && (items[i].value < 0 || (size_t)items[i].value >= h->strs.size())) return ZBHIP_EINVAL;
    v.push_back({t, t == ZBHIP_DOC_NIL ? 0 : items[i].value});
  }
  return intern_items(h, v);
}

extern "C" int zbhip_list_items(zbhip_handle* h, int64_t id, zbhip_doc_entry* out, size_t cap, size_t* n_out) {
  if (!h || !n_out || (cap && !out)) return ZBHIP_EINVAL;
  if (id < 0 || (size_t)id >= h->lists.size()) return ZBHIP_EINVAL;
  const auto& v = h->lists[(size_t)id];
  *n_out = v.size();
  for (size_t i = 0; i < v.size() && i < cap; ++i) {
    out[i] = zbhip_doc_entry{};
    out[i].type = v[i].first;
    out[i].value = v[i].second;
  }
  return ZBHIP_OK;
}

// IndexedDocument.index (state/variable/IndexedDocument.java:44-56) puts (key offset -> value offset) into
// an agrona Int2IntHashMap (org.agrona 1.19.2, parent/pom.xml:38): a table of 2^k slots (8 at first)
// probed from evenHash(key) = ((key << 1) - (key << 8)) & (2 * slots - 1) over (key, value) int pairs, by
// pairs upwards; past (int)(slots * 0.65f) entries it doubles, re-putting the old pairs in slot order.
// Its iterator walks the slots downwards from the top one, or -- when the top slot is taken, so a probe
// chain may wrap -- from just below the first free slot, once around.  Only the slot of each entry
// matters here: slot = pair index / 2.
extern "C" int zbhip_doc_merge_order(const uint32_t* key_offsets, size_t n, zbhip_doc_entry* entries) {
  if ((n && (!key_offsets || !entries)) || n > 256) return ZBHIP_EINVAL;
  for (size_t i = 1; i < n; ++i)
    if (key_offsets[i] <= key_offsets[i - 1]) return ZBHIP_EINVAL;
  for (size_t i = 0; i < n; ++i) entries[i].pad[0] = entries[i].pad[1] = 0;
  if (n < 2) return ZBHIP_OK;
  auto home = [](uint32_t key, uint32_t slots) {  // evenHash / 2
    return ((((key << 1) - (key << 8)) & (2 * slots - 1)) >> 1);
  };
  uint32_t slots = 8;
  std::vector<int> table(slots, -1);  // slot -> document index
  size_t size = 0;
  auto place = [&](std::vector<int>& t, uint32_t sl, int doc) {
    uint32_t i = home(key_offsets[doc], sl);
    while (t[i] >= 0) i = (i + 1) & (sl - 1);
    t[i] = doc;
  };
  for (size_t d = 0; d < n; ++d) {
    place(table, slots, (int)d);  // (offsets are distinct: no replacement)
    if (++size > (size_t)(int)(slots * 0.65f)) {
      std::vector<int> grown(2 * slots, -1);
      for (uint32_t i = 0; i < slots; ++i)
        if (table[i] >= 0) place(grown, 2 * slots, table[i]);
      table.swap(grown);
      slots *= 2;
    }
  }
  uint32_t start = slots;  // AbstractIterator.reset
  if (table[slots - 1] >= 0)
    for (start = 0; start < slots && table[start] >= 0; ++start) {
    }
  bool displaced = false;
  size_t k = 0;
  for (uint32_t step = 1; step <= slots && k < n; ++step) {  // findNext: downwards, once around
    const uint32_t i = (start + slots - step) & (slots - 1);
    if (table[i] < 0) continue;
    entries[k++].pad[0] = (uint8_t)table[i];
    displaced = displaced || home(key_offsets[table[i]], slots) != i;
  }
  entries[0].pad[1] = displaced ? 1 : 0;
  return ZBHIP_OK;
}

// uploads the lists interned since the last run (their headers and items)
static int sync_lists(zbhip_handle* h) {
  if (h->d_list_n == h->lists.size()) return ZBHIP_OK;
  if (h->lists.size() > h->d_list_cap || h->list_val.size() > h->d_litem_cap) {
    const size_t lc = std::max<size_t>(1024, h->lists.size() * 2), ic = std::max<size_t>(4096, h->list_val.size() * 2);
    HIPCHK(hipStreamSynchronize(h->stream));
    (void)hipFree(h->d_list_hdr);
    (void)hipFree(h->d_list_val);
    (void)hipFree(h->d_list_type);
    h->d_list_hdr = nullptr;
    h->d_list_val = nullptr;
    h->d_list_type = nullptr;
    if (dalloc(&h->d_list_hdr, lc) != hipSuccess || dalloc(&h->d_list_val, ic) != hipSuccess ||
        dalloc(&h->d_list_type, ic) != hipSuccess)
      return ZBHIP_ENOMEM;
    h->d_list_cap = lc;
    h->d_litem_cap = ic;
    h->d_list_n = h->d_list_items = 0;
  }
  HIPCHK(hipMemcpyAsync(h->d_list_hdr + h->d_list_n, h->list_hdr.data() + h->d_list_n,
                        (h->lists.size() - h->d_list_n) * sizeof(uint2), hipMemcpyHostToDevice, h->stream));
  const size_t ni = h->list_val.size() - h->d_list_items;
  if (ni) {
    HIPCHK(hipMemcpyAsync(h->d_list_val + h->d_list_items, h->list_val.data() + h->d_list_items, ni * sizeof(long long),
                          hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->d_list_type + h->d_list_items, h->list_type.data() + h->d_list_items, ni,
                          hipMemcpyHostToDevice, h->stream));
  }
  HIPCHK(hipStreamSynchronize(h->stream));  // (the host vectors may grow before the next run)
  h->d_list_n = h->lists.size();
  h->d_list_items = h->list_val.size();
  return ZBHIP_OK;
}

int zbhip_intern_strings(zbhip_handle* h, const char* bytes, const uint64_t* offsets, size_t n, uint32_t* ids_out) {
  if (!h || (n && (!bytes || !offsets))) return ZBHIP_EINVAL;
  h->strs.reserve(h->strs.size() + n);
  h->str_hash.reserve(h->str_hash.size() + n);
  for (size_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i]) return ZBHIP_EINVAL;
    int64_t id = zbhip_intern_string(h, bytes + offsets[i], offsets[i + 1] - offsets[i]);
    if (id < 0) return (int)id;
    if (ids_out) ids_out[i] = (uint32_t)id;
  }
  return ZBHIP_OK;
}

const char* zbhip_string_value(zbhip_handle* h, uint32_t id, size_t* len) {
  if (!h || id >= h->strs.size()) {
    if (len) *len = 0;
    return "";
  }
  if (len) *len = h->strs[id].size();
  return h->strs[id].c_str();
}

int32_t zbhip_subscription_partition(const char* bytes, size_t len, int32_t partition_count) {
  if (partition_count <= 0) return ZBHIP_EINVAL;
  const int32_t r = java_hash(bytes, len) % partition_count;
  return (r < 0 ? -r : r) + 1;
}

// ---- outbox --------------------------------------------------------------------------------------
int zbhip_outbox(zbhip_handle* h, zbhip_xpart_cmd* out, size_t cap, size_t* n_out) {
  if (!h || !n_out) return ZBHIP_EINVAL;
  *n_out = 0;
  if (!h->results) return h->msg() ? ZBHIP_ESTATE : ZBHIP_OK;
  if (!h->msg()) return ZBHIP_OK;
  if (int rc = finalize(h)) return rc;
  const size_t n = h->n_cmds;
  h->h_xout.resize(n * kOut);
  if (n) {  // entry-major on the device (entry j of command c at j * max_commands + c)
    HIPCHK(hipMemcpy2DAsync(h->h_xout.data(), n * sizeof(zbhip_xpart_cmd), h->d_xout,
                            (size_t)h->cfg.max_commands * sizeof(zbhip_xpart_cmd), n * sizeof(zbhip_xpart_cmd), kOut,
                            hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  size_t k = 0;
  for (size_t c = 0; c < n; ++c) {
    if (((h->h_hdr[c].y >> 16) & 0xFF) != ST_OK) continue;
    for (uint32_t j = 0; j < (h->h_hdr2[c].z & 0xF) && j < (uint32_t)kOut; ++j) {
      const zbhip_xpart_cmd& x = h->h_xout[j * n + c];
      if (x.kind == XK_PATCH) continue;
      if (out && k < cap) out[k] = x;
      ++k;
    }
  }
  *n_out = k;
  return ZBHIP_OK;
}

// The sends of window command i (its batch's post-commit side effects, in batch order): what a host
// adapter hands to InterPartitionCommandSender once the platform committed command i's batch.
int zbhip_outbox_command(zbhip_handle* h, size_t i, zbhip_xpart_cmd* out, size_t cap, size_t* n_out) {
  if (!h || !n_out || (cap && !out)) return ZBHIP_EINVAL;
  *n_out = 0;
  if (!h->results) return h->msg() ? ZBHIP_ESTATE : ZBHIP_OK;
  if (!h->msg()) return ZBHIP_OK;
  if (i >= h->n_cmds) return ZBHIP_EINVAL;
  if (int rc = advance(h, i + 1, false)) return rc;
  const size_t n = h->n_cmds;
  if (h->xout_host_run != h->windows_run || h->h_xout.size() != n * kOut) {
    h->h_xout.resize(n * kOut);
    if (n) {
      HIPCHK(hipMemcpy2DAsync(h->h_xout.data(), n * sizeof(zbhip_xpart_cmd), h->d_xout,
                              (size_t)h->cfg.max_commands * sizeof(zbhip_xpart_cmd), n * sizeof(zbhip_xpart_cmd), kOut,
                              hipMemcpyDeviceToHost, h->stream));
      HIPCHK(hipStreamSynchronize(h->stream));
    }
    h->xout_host_run = h->windows_run;
  }
  if (((h->h_hdr[i].y >> 16) & 0xFF) != ST_OK) return ZBHIP_OK;
  size_t k = 0;
  for (uint32_t j = 0; j < (h->h_hdr2[i].z & 0xF) && j < (uint32_t)kOut; ++j) {
    const zbhip_xpart_cmd& x = h->h_xout[j * n + i];
    if (x.kind == XK_PATCH) continue;
    if (k < cap) out[k] = x;
    ++k;
  }
  *n_out = k;
  return k > cap ? ZBHIP_ENOMEM : ZBHIP_OK;
}

int zbhip_outbox_device(zbhip_handle* h, const zbhip_xpart_cmd** dev_out, uint32_t* counts) {
  if (!h || !dev_out || !counts) return ZBHIP_EINVAL;
  if (!h->msg() || !h->ran) return ZBHIP_ESTATE;
  const uint32_t parts = (uint32_t)std::max(1, h->cfg.partition_count);
  if (parts > 1024) return ZBHIP_EINVAL;
  if (!h->bucketed) {
    HIPCHK(launch_bucket(h->d_cmd_hdr, h->d_cmd_hdr2, h->d_xout, (uint32_t)h->cfg.max_commands, (uint32_t)h->n_cmds, parts, h->d_blk_cnt,
                         h->d_xcount, h->d_xbucket, h->stream));
    h->bucketed = true;
  }
  *dev_out = h->d_xbucket;
  if (h->outbox_taken) {  // sent already: nothing new until the next run
    memset(counts, 0, parts * sizeof(uint32_t));
    return ZBHIP_OK;
  }
  HIPCHK(hipMemcpyAsync(counts, h->d_xcount, parts * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->outbox_taken = true;
  return ZBHIP_OK;
}

void* zbhip_stream(zbhip_handle* h) { return h ? reinterpret_cast<void*>(h->stream) : nullptr; }

int zbhip_outbox_device_async(zbhip_handle* h, const zbhip_xpart_cmd** dev_out, void* dev_counts) {
  if (!h || !dev_out || !dev_counts) return ZBHIP_EINVAL;
  if (!h->msg() || !h->ran) return ZBHIP_ESTATE;
  const uint32_t parts = (uint32_t)std::max(1, h->cfg.partition_count);
  if (parts > 1024) return ZBHIP_EINVAL;
  if (!h->bucketed) {
    HIPCHK(launch_bucket(h->d_cmd_hdr, h->d_cmd_hdr2, h->d_xout, (uint32_t)h->cfg.max_commands, (uint32_t)h->n_cmds, parts, h->d_blk_cnt,
                         h->d_xcount, h->d_xbucket, h->stream));
    h->bucketed = true;
  }
  *dev_out = h->d_xbucket;
  if (h->outbox_taken) {
    HIPCHK(hipMemsetAsync(dev_counts, 0, parts * sizeof(uint32_t), h->stream));
  } else {
    HIPCHK(hipMemcpyAsync(dev_counts, h->d_xcount, parts * sizeof(uint32_t), hipMemcpyDeviceToDevice, h->stream));
    h->outbox_taken = true;
  }
  return ZBHIP_OK;
}

int zbhip_outbox_copy(zbhip_handle* h, void* dev_dst, size_t first, size_t count) {
  if (!h || (count && !dev_dst)) return ZBHIP_EINVAL;
  if (!h->msg() || !h->bucketed) return ZBHIP_ESTATE;
  if (first + count > h->n_cmds * kOut) return ZBHIP_EINVAL;
  if (count)
    HIPCHK(hipMemcpyAsync(dev_dst, h->d_xbucket + first, count * sizeof(zbhip_xpart_cmd), hipMemcpyDeviceToDevice,
                          h->stream));
  return ZBHIP_OK;
}

int zbhip_exchange_gather(const zbhip_xpart_cmd* const* src, uint32_t P, const uint32_t* dev_counts,
                          zbhip_xpart_cmd* const* dst, uint32_t max_count, void* stream) {
  if (P > kMaxGatherParts || (P && (!src || !dst || !dev_counts))) return ZBHIP_EINVAL;
  XGather A{};
  A.P = P;
  A.counts = dev_counts;
  for (uint32_t q = 0; q < P; ++q) {
    A.src[q] = src[q];
    A.dst[q] = dst[q];
  }
  HIPCHK(launch_xgather(A, max_count, reinterpret_cast<hipStream_t>(stream)));
  return ZBHIP_OK;
}

int zbhip_submit_xparts_device(zbhip_handle* h, const zbhip_xpart_cmd* dev_xparts, size_t n) {
  if (!h || (n && !dev_xparts)) return ZBHIP_EINVAL;
  if (!h->msg()) return ZBHIP_EUNSUPP;
  if (n > h->cfg.max_commands) return ZBHIP_ENOMEM;
  HIPCHK(launch_xpart_window(dev_xparts, (uint32_t)n, h->d_cmds, h->stream));
  return zbhip_submit_device_ex(h, reinterpret_cast<const zbhip_command*>(h->d_cmds), n, nullptr, 0, dev_xparts, n);
}

int64_t zbhip_incident_message(zbhip_handle* h, const zbhip_record* r, char* out, size_t cap) {
  if (!h || !h->ser) return ZBHIP_EINVAL;
  return zbhip_serializer_incident_message(h->ser, r, out, cap);
}

int zbhip_string_partitions(zbhip_handle* h, const uint32_t* ids, size_t n, int32_t partition_count, int32_t* out) {
  if (!h || partition_count <= 0 || (n && (!ids || !out))) return ZBHIP_EINVAL;
  for (size_t i = 0; i < n; ++i) {
    if (ids[i] >= h->str_hash.size()) return ZBHIP_EINVAL;
    const int32_t r = (int32_t)h->str_hash[ids[i]] % partition_count;
    out[i] = (r < 0 ? -r : r) + 1;
  }
  return ZBHIP_OK;
}

int zbhip_command_status(zbhip_handle* h, size_t i, uint32_t* status, uint32_t* reason) {
  if (!h || !status || !reason) return ZBHIP_EINVAL;
  if (!h->results) return ZBHIP_ESTATE;
  if (i >= h->n_cmds) return ZBHIP_EINVAL;
  *status = (h->h_hdr[i].y >> 16) & 0xFF;
  *reason = (h->h_hdr[i].y >> 24) & 0x7F;
  return ZBHIP_OK;
}

int zbhip_fallback(zbhip_handle* h, uint32_t* instances, size_t cap, size_t* n_out) {
  if (!h || !n_out) return ZBHIP_EINVAL;
  *n_out = 0;
  if (!h->results) return h->stats.fallback ? ZBHIP_ESTATE : ZBHIP_OK;
  size_t k = 0;
  for (size_t c = 0; c < h->n_cmds; ++c)
    if (((h->h_hdr[c].y >> 16) & 0xFF) != ST_OK) {
      if (k < cap && instances) instances[k] = h->h_cmds[c].instance;
      ++k;
    }
  *n_out = k;
  return ZBHIP_OK;
}

// Canonical CF rows (same text format as the oracle's state dump).
namespace {
struct InstRows {  // the SoA rows of one instance slot
  uint4 hdr;
  uint2 slots[kSlots];
  uint2 vm[kVars];
  long long vv[kVars];
  uint32_t join[kJoinWords];
  uint4 pms;
  long long pms_msg = -1;  // DevState.pms_msg
  bool has_pms;
  uint4 tmr;  // the instance's timer row (DevState.tmr)
};
}  // namespace

// PROCESS_SUBSCRIPTION_BY_KEY [eik, name] (DbProcessMessageSubscriptionState) of an instance slot's
// subscription row -- also after the instance ended, while a closing subscription waits for its
// PROCESS_MESSAGE_SUBSCRIPTION:DELETE
static void emit_pms(zbhip_handle* h, uint32_t inst, const InstRows& R, const Proc& P, long long pik,
                     zbhip_state_sink sink, void* ctx) {
  char buf[768];
  if (R.has_pms && ((R.pms.x >> 12) & 3)) {  // PROCESS_SUBSCRIPTION_BY_KEY [eik, name] (DbProcessMessageSubscriptionState)
    const uint4 m = R.pms;
    const uint32_t el = m.x & 0xFFF;
    const zbhip_element& E = P.els[el];
    snprintf(buf, sizeof buf,
             "PROCESS_SUBSCRIPTION_BY_KEY|%lld|%s|key=%lld,state=%s,subscriptionPartitionId=%u,processInstanceKey=%lld,"
             "bpmnProcessId=%s,messageKey=%lld,correlationKey=%s,elementId=%s,interrupting=%u",
             h->key_of(inst, m.y & 0xFFFF), zbhip_name(h, E.message_name), h->key_of(inst, m.y >> 16),
             ((m.x >> 12) & 3) == 1 ? "OPENING" : ((m.x >> 12) & 3) == 3 ? "CLOSING" : "OPENED", m.x >> 16, pik, zbhip_name(h, P.bpmn_name),
             h->resolve_ref(R.pms_msg), zbhip_string_value(h, m.z, nullptr), P.id(el).c_str(), (m.x >> 14) & 1);
    sink(ctx, buf);
  }
}

// a list's items in a state row: "type:value;..." (the oracle's format, zb_oracle.cpp list_text)
static std::string list_text(const zbhip_handle::Items& items) {
  std::string o;
  for (size_t i = 0; i < items.size(); ++i) {
    if (i) o += ';';
    o += std::to_string((int)items[i].first) + ":" + std::to_string((long long)items[i].second);
  }
  return o;
}

// a multi-instance body's collection as the instance holds it: the static items, or the list variable
// (seen from the body: its containers' scopes, then the process instance's; nullptr: none)
static const zbhip_handle::Items* mi_items_of(const zbhip_handle* h, const Proc& P, const Proc::Mi& m, const InstRows& R,
                                              uint32_t inst) {
  (void)inst;
  if (m.coll_name == NONE) return &m.items;
  const uint32_t nslots = (R.hdr.y >> 8) & 0xFF, nvars = (R.hdr.y >> 16) & 0xFF;
  std::vector<uint32_t> chain;  // the scope ordinals from the body's container up, then the process (0)
  for (uint32_t c = P.els[m.body].flow_scope, d = 0; c != 0 && c < P.els.size() && d < 16; c = P.els[c].flow_scope, ++d)
    for (uint32_t s = 0; s < nslots && s < (uint32_t)kSlots; ++s)
      if ((R.slots[s].x & 0xFFFF) == c) chain.push_back(R.slots[s].x >> 16);
  chain.push_back(0);
  for (uint32_t sc : chain)
    for (uint32_t v = 0; v < nvars && v < (uint32_t)kVars; ++v)
      if ((R.vm[v].x & 0xFFFF) == m.coll_name && (R.vm[v].x >> 16) == sc) {
        if (((R.vm[v].y >> 16) & 0xFF) != ZBHIP_DOC_LIST || R.vv[v] < 0 || (size_t)R.vv[v] >= h->lists.size())
          return nullptr;
        return &h->lists[(size_t)R.vv[v]];
      }
  return nullptr;
}

// the rows of one process instance (ELEMENT_INSTANCE_KEY ... NUMBER_OF_TAKEN_SEQUENCE_FLOWS,
// PROCESS_SUBSCRIPTION_BY_KEY); nothing for a free slot
static void emit_instance(zbhip_handle* h, uint32_t inst, const InstRows& R, zbhip_state_sink sink, void* ctx) {
  char buf[768];
  const uint4 hd = R.hdr;
  if (!((hd.y >> 24) & 1)) {  // an ended instance: only a subscription still closing (header bit 25)
    const uint32_t ip = inst < h->inst_proc.size() ? h->inst_proc[inst] : NONE;
    if (hd.y == (1u << 25) && ip != NONE && ip < h->procs.size())
      emit_pms(h, inst, R, h->procs[ip], h->key_of(inst, 0), sink, ctx);
    return;
  }
  const uint32_t proc = hd.x & 0xFFFF;
  if (proc == NONE || proc >= h->procs.size()) return;
  const Proc& P = h->procs[proc];
  const long long pik = h->key_of(inst, 0);
  const uint32_t nslots = (hd.y >> 8) & 0xFF, nvars = (hd.y >> 16) & 0xFF;
  snprintf(buf, sizeof buf,
           "ELEMENT_INSTANCE_KEY|%lld|parentKey=-1,childCount=%u,childActivatedCount=0,childCompletedCount=0,"
           "childTerminatedCount=0,jobKey=0,multiInstanceLoopCounter=0,interruptingElementId=,"
           "calledChildInstanceKey=-1,state=%u,elementId=%s,bpmnElementType=%d,bpmnEventType=%d,flowScopeKey=-1,"
           "processInstanceKey=%lld,processDefinitionKey=%lld,activeSequenceFlows=%u",
           pik, hd.z & 0xFFFF, hd.y & 0xFF, P.id(0).c_str(), ZBHIP_EL_PROCESS, ZBHIP_EV_UNSPECIFIED, pik,
           (long long)P.def_key, hd.z >> 16);
  sink(ctx, buf);
  snprintf(buf, sizeof buf, "ELEMENT_INSTANCE_PARENT_CHILD|-1|%lld", pik);
  sink(ctx, buf);
  snprintf(buf, sizeof buf, "ELEMENT_INSTANCE_CHILD_PARENT|%lld|-1", pik);
  sink(ctx, buf);
  snprintf(buf, sizeof buf, "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY|%lld|%lld", (long long)P.def_key, pik);
  sink(ctx, buf);
  // the start events of the event sub-processes attached to container c (SubProcessTransformer: after
  // the boundary events), the interrupting ones (job_retries bit 0)
  auto esp_ids = [&](uint32_t c, std::string& intr, bool& any) {
    for (size_t x = 0; x < P.els.size(); ++x)
      if (P.els[x].element_type == ZBHIP_EL_EVENT_SUB_PROCESS && P.els[x].flow_scope == c &&
          P.els[x].start_event < P.els.size()) {
        any = true;
        if (P.els[P.els[x].start_event].job_retries & 1)
          intr += (intr.empty() ? "" : ";") + P.id(P.els[x].start_event);
      }
  };
  {  // the process instance's event scope: only with event sub-processes (createEventScope: hasEvents)
    std::string intr;
    bool any = false;
    esp_ids(0, intr, any);
    if (any) {
      snprintf(buf, sizeof buf, "EVENT_SCOPE|%lld|accepting=1,interrupted=0,interrupting=%s,boundaryElementIds=", pik,
               intr.c_str());
      sink(ctx, buf);
    }
  }
  // the key of the instance of container c (an element's flow scope): the process instance, or the
  // slot of the sub-process element c (one active instance per sub-process element)
  auto scope_key = [&](uint32_t c) -> long long {
    if (c == 0) return pik;
    for (uint32_t s = 0; s < nslots && s < (uint32_t)kSlots; ++s)
      if ((R.slots[s].x & 0xFFFF) == c) return h->key_of(inst, R.slots[s].x >> 16);
    return pik;
  };
  for (uint32_t s = 0; s < nslots; ++s) {
    const uint2 e = R.slots[s];
    const uint32_t elem = e.x & 0xFFFF;
    const long long k = h->key_of(inst, e.x >> 16);
    const uint32_t job = e.y & 0xFFFF, state = (e.y >> 16) & 0xFF;
    const bool job_row = (e.y >> 24) & 1;
    const zbhip_element& E = P.els[elem];
    const bool sub = E.element_type == ZBHIP_EL_SUB_PROCESS;  // job field: childCount | activeSequenceFlows << 8
    const bool body = E.element_type == ZBHIP_EL_MULTI_INSTANCE_BODY;  // childCount | loop counter << 8
    const Proc::Mi* im = P.mi_inner(elem);  // a multi-instance inner instance: its loop counter in the flags
    const bool jw = ZBHIP_IS_JOB_WORKER(E.element_type);
    // an exclusive gateway waits only with an incident: its job field is the incident key
    const bool xgw = E.element_type == ZBHIP_EL_EXCLUSIVE_GATEWAY;
    const long long jk = sub || body || xgw || (im && !jw) ? 0 : job == JOB_ZERO ? 0 : job == JOB_MINUS1 ? -1 : h->key_of(inst, job);
    const long long fs = scope_key(E.flow_scope);
    const uint32_t child = sub || body ? job & 0xFF : 0u, loop = body ? (job >> 8) & 0xFF : im ? e.y >> 26 : 0u;
    snprintf(buf, sizeof buf,
             "ELEMENT_INSTANCE_KEY|%lld|parentKey=%lld,childCount=%u,childActivatedCount=%u,childCompletedCount=%u,"
             "childTerminatedCount=0,jobKey=%lld,multiInstanceLoopCounter=%u,interruptingElementId=,"
             "calledChildInstanceKey=-1,state=%u,elementId=%s,bpmnElementType=%d,bpmnEventType=%d,flowScopeKey=%lld,"
             "processInstanceKey=%lld,processDefinitionKey=%lld,activeSequenceFlows=%u",
             k, fs, child, body ? loop : 0u, body ? loop - child : 0u, jk, loop, state, P.id(elem).c_str(),
             E.element_type, E.event_type, fs, pik, (long long)P.def_key, sub ? (job >> 8) & 0xFF : 0u);
    sink(ctx, buf);
    const zbhip_handle::Items* coll = im ? mi_items_of(h, P, *im, R, inst) : nullptr;
    if (im && coll && loop >= 1 && loop <= coll->size() && (jw ? job_row : job != JOB_ZERO)) {
      // the inner instance's loop variables (setLoopVariables): keys right before its job's (a job
      // worker) or the loopCounter key in its job field (an undefined task) -- the inputElement, the
      // local outputElement (nil: a job's document updates it only in the batch that completes the
      // instance), the loopCounter -- values from the collection
      const uint32_t kl = jw ? job - 1 : job;
      const uint32_t ko = im->out_local() ? 1u : 0u;
      if (im->input_name != NONE) {
        snprintf(buf, sizeof buf, "VARIABLES|%lld|%s|key=%lld,type=%u,value=%lld", k, h->names[im->input_name].c_str(),
                 h->key_of(inst, kl - 1 - ko), (unsigned)(*coll)[loop - 1].first, (long long)(*coll)[loop - 1].second);
        sink(ctx, buf);
      }
      if (ko) {
        snprintf(buf, sizeof buf, "VARIABLES|%lld|%s|key=%lld,type=%u,value=0", k, h->names[im->out_elem].c_str(),
                 h->key_of(inst, kl - 1), (unsigned)ZBHIP_DOC_NIL);
        sink(ctx, buf);
      }
      snprintf(buf, sizeof buf, "VARIABLES|%lld|%s|key=%lld,type=%u,value=%u", k, h->names[im->loop_name].c_str(),
               h->key_of(inst, kl), (unsigned)ZBHIP_DOC_INT, loop);
      sink(ctx, buf);
    }
    if (body && P.mi_body(elem) && P.mi_body(elem)->out_coll != NONE) {
      // the body's local outputCollection (initializeOutputCollection / updateOutputCollection): the host's
      const auto o = h->mi_out.find(k);
      if (o != h->mi_out.end()) {
        snprintf(buf, sizeof buf, "VARIABLES|%lld|%s|key=%lld,type=%u,value=", k,
                 h->names[P.mi_body(elem)->out_coll].c_str(), (long long)o->second.var_key, (unsigned)ZBHIP_DOC_LIST);
        sink(ctx, (std::string(buf) + list_text(o->second.items)).c_str());
      }
    }
    snprintf(buf, sizeof buf, "ELEMENT_INSTANCE_PARENT_CHILD|%lld|%lld", fs, k);
    sink(ctx, buf);
    snprintf(buf, sizeof buf, "ELEMENT_INSTANCE_CHILD_PARENT|%lld|%lld", k, fs);
    sink(ctx, buf);
    if (xgw) {  // IncidentCreatedApplier -> DbIncidentState.createIncident (INCIDENTS, INCIDENT_PROCESS_INSTANCES)
      const uint32_t info = e.y >> 26, pos = info & 15;
      const long long ik = h->key_of(inst, job);
      const int flow = pos == 15 || (size_t)E.out_begin + pos >= P.out.size() ? -1 : (int)P.out[E.out_begin + pos];
      snprintf(buf, sizeof buf,
               "INCIDENTS|%lld|errorType=%d,flow=%d,result=%u,processDefinitionKey=%lld,processInstanceKey=%lld,"
               "elementId=%s,elementInstanceKey=%lld",
               ik, pos == 15 ? ZBHIP_ERR_CONDITION_ERROR : ZBHIP_ERR_EXTRACT_VALUE_ERROR, flow, pos == 15 ? 0u : info >> 4,
               (long long)P.def_key, pik, P.id(elem).c_str(), k);
      sink(ctx, buf);
      snprintf(buf, sizeof buf, "INCIDENT_PROCESS_INSTANCES|%lld|%lld", k, ik);
      sink(ctx, buf);
    }
    std::string esp_intr;
    bool has_esp = false;
    if (E.element_type == ZBHIP_EL_SUB_PROCESS) esp_ids(elem, esp_intr, has_esp);
    bool body_bnd = false;  // a multi-instance body with (error) boundary events: an event scope
    if (body)
      for (size_t b = 0; b < P.els.size() && !body_bnd; ++b)
        body_bnd = P.els[b].element_type == ZBHIP_EL_BOUNDARY_EVENT && P.els[b].flow_source == elem;
    const bool sub_bnd = E.element_type == ZBHIP_EL_SUB_PROCESS && E.default_flow != ZBHIP_NONE16 &&
                         E.default_flow < P.els.size();
    if (ZBHIP_IS_JOB_WORKER(E.element_type) || E.element_type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT ||
        E.element_type == ZBHIP_EL_BOUNDARY_EVENT || sub_bnd || has_esp || body_bnd) {
      // EventScopeInstance.java:25-35: a catch / boundary event's interrupting ids are its own id
      // (ExecutableCatchEventElement.java:124-132), a job worker's (a sub-process's: an event scope
      // only with events) those of its interrupting boundary event, which is also its
      // boundaryElementIds (ExecutableActivity.java:28-38)
      const bool own = E.element_type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT || E.element_type == ZBHIP_EL_BOUNDARY_EVENT;
      const bool bnd = (ZBHIP_IS_JOB_WORKER(E.element_type) && E.start_event != ZBHIP_NONE16) || sub_bnd || body_bnd;
      // an activity's boundary events in attach order (element order), the cancelActivity ones interrupting
      std::string ids = own ? P.id(elem) : std::string(), intr_ids = own ? ids : std::string();
      if (bnd)
        for (size_t b = 0; b < P.els.size(); ++b)
          if (P.els[b].element_type == ZBHIP_EL_BOUNDARY_EVENT && P.els[b].flow_source == elem) {
            ids += (ids.empty() ? "" : ";") + P.id((uint32_t)b);
            if (P.els[b].job_retries & 1) intr_ids += (intr_ids.empty() ? "" : ";") + P.id((uint32_t)b);
          }
      if (!esp_intr.empty()) intr_ids += (intr_ids.empty() ? "" : ";") + esp_intr;
      snprintf(buf, sizeof buf, "EVENT_SCOPE|%lld|accepting=1,interrupted=0,interrupting=%s,boundaryElementIds=%s", k,
               intr_ids.c_str(), bnd ? ids.c_str() : "");
      sink(ctx, buf);
    }
    if (job_row) {
      const char* type = P.strings[E.job_type].c_str();
      const bool stored = (e.y >> 25) & 1;  // a stored activation (zbhip_activate_jobs): deadline, worker, state on the host
      const auto ait = stored ? h->activated.find(jk) : h->activated.end();
      const zbhip_handle::Activation* A = ait != h->activated.end() ? &ait->second : nullptr;
      const long long deadline = A ? (long long)A->deadline : -1;
      const bool act = A && A->state == zbhip_handle::JS_ACTIVATED;
      const bool failed = A && A->state == zbhip_handle::JS_FAILED;
      std::string fail_suffix;  // a failed job's stored fields (errorMessage in hex: it may hold ',' or '|')
      if (A && A->fail_fields)
        fail_suffix = ",errorMessageHex=" + hex_of(A->error_id == ZBHIP_NO_STRING ? std::string() : h->strs[A->error_id]) +
                      ",retryBackoff=0,recurringTime=-1";
      snprintf(buf, sizeof buf,
               "JOBS|%lld|type=%s,retries=%d,elementId=%s,elementInstanceKey=%lld,processInstanceKey=%lld,"
               "bpmnProcessId=%s,processDefinitionKey=%lld,processDefinitionVersion=%d,tenantId=<default>,"
               "deadline=%lld,worker=",
               jk, type, A && A->fail_fields ? A->retries : (int)E.job_retries, P.id(elem).c_str(), k, pik,
               P.strings[P.bpmn_id].c_str(), (long long)P.def_key, P.version, deadline);
      // (worker and errorMessage appended unbounded: a message holds up to 10 000 characters)
      const std::string row = std::string(buf) + (A ? A->worker : std::string()) + fail_suffix;
      sink(ctx, row.c_str());
      snprintf(buf, sizeof buf, "JOB_STATES|%lld|%s", jk, failed ? "FAILED" : act ? "ACTIVATED" : "ACTIVATABLE");
      sink(ctx, buf);
      if (act) {
        snprintf(buf, sizeof buf, "JOB_DEADLINES|%lld|%lld", deadline, jk);
        sink(ctx, buf);
      } else if (!failed) {
        snprintf(buf, sizeof buf, "JOB_ACTIVATABLE|%s|<default>|%lld", type, jk);
        sink(ctx, buf);
      }
      if (A && A->incident_key >= 0) {  // its JOB_NO_RETRIES incident (DbIncidentState.createIncident)
        snprintf(buf, sizeof buf,
                 "INCIDENTS|%lld|errorType=%d,flow=-1,result=0,processDefinitionKey=%lld,processInstanceKey=%lld,"
                 "elementId=%s,elementInstanceKey=%lld,jobKey=%lld,messageHex=",
                 (long long)A->incident_key, (int)ZBHIP_ERR_JOB_NO_RETRIES, (long long)P.def_key, pik, P.id(elem).c_str(),
                 k, jk);
        const std::string row =
            std::string(buf) + hex_of(A->incident_msg_id == ZBHIP_NO_STRING ? std::string() : h->strs[A->incident_msg_id]);
        sink(ctx, row.c_str());
        snprintf(buf, sizeof buf, "INCIDENT_JOBS|%lld|%lld", jk, (long long)A->incident_key);
        sink(ctx, buf);
      }
    }
  }
  for (uint32_t v = 0; v < nvars; ++v) {
    const uint2 m = R.vm[v];
    const uint32_t scope = m.x >> 16, type = (m.y >> 16) & 0xFF;
    const long long vk = h->key_of(inst, m.y & 0xFFFF);
    if (type == ZBHIP_DOC_LIST || type == kDocOutList) {  // a list: its items in the row
      const auto ov = type == kDocOutList ? h->outlist_var.find(vk) : h->outlist_var.end();
      const long long id = type == kDocOutList ? (ov == h->outlist_var.end() ? -1 : (long long)ov->second) : R.vv[v];
      if (id < 0 || (size_t)id >= h->lists.size()) continue;
      snprintf(buf, sizeof buf, "VARIABLES|%lld|%s|key=%lld,type=%u,value=", h->key_of(inst, scope),
               h->names[m.x & 0xFFFF].c_str(), vk, (unsigned)ZBHIP_DOC_LIST);
      sink(ctx, (std::string(buf) + list_text(h->lists[(size_t)id])).c_str());
      continue;
    }
    snprintf(buf, sizeof buf, "VARIABLES|%lld|%s|key=%lld,type=%u,value=%lld", h->key_of(inst, scope),
             h->names[m.x & 0xFFFF].c_str(), vk, type, R.vv[v]);
    sink(ctx, buf);
  }
  if (R.tmr.y >> 31) {  // TIMERS [eik, timerKey] -> TimerInstance, TIMER_DUE_DATES [dueDate, eik, timerKey] (DbTimerInstanceState)
    const long long eik = h->key_of(inst, R.tmr.y & 0xFFFF), tk = h->key_of(inst, R.tmr.x >> 16);
    const long long due = (long long)(((unsigned long long)R.tmr.w << 32) | R.tmr.z);
    snprintf(buf, sizeof buf,
             "TIMERS|%lld|%lld|handlerNodeId=%s,processDefinitionKey=%lld,key=%lld,elementInstanceKey=%lld,"
             "processInstanceKey=%lld,dueDate=%lld,repetitions=%d,tenantId=<default>",
             eik, tk, P.id(R.tmr.x & 0xFFF).c_str(), (long long)P.def_key, tk, eik, pik, due,
             ((R.tmr.y >> 16) & 0xFF) == 255 ? -1 : (int)((R.tmr.y >> 16) & 0xFF));
    sink(ctx, buf);
    snprintf(buf, sizeof buf, "TIMER_DUE_DATES|%lld|%lld|%lld", due, eik, tk);
    sink(ctx, buf);
  }
  emit_pms(h, inst, R, P, pik, sink, ctx);
  if (P.n_join_slots) {
    for (uint32_t f = 0; f < P.els.size(); ++f) {
      const zbhip_element& E = P.els[f];
      if (E.element_type != ZBHIP_EL_SEQUENCE_FLOW || E.join_slot == ZBHIP_NONE16) continue;
      const uint32_t s = E.join_slot;
      const uint32_t cnt = (R.join[s >> 2] >> ((s & 3) * 8)) & 0xFF;
      if (!cnt) continue;
      snprintf(buf, sizeof buf, "NUMBER_OF_TAKEN_SEQUENCE_FLOWS|%lld|%s|%s|%u", scope_key(E.flow_scope),
               P.id(E.flow_target).c_str(), P.id(f).c_str(), cnt);
      sink(ctx, buf);
    }
  }
}

// one instance's rows gathered from HBM (small copies: the hand-off path of a few instances)
static int gather_instance(zbhip_handle* h, uint32_t i, InstRows& R) {
  const size_t N = h->st.n;
  HIPCHK(hipMemcpy(&R.hdr, h->st.hdr + i, sizeof(uint4), hipMemcpyDeviceToHost));
  const uint32_t nslots = (R.hdr.y >> 8) & 0xFF, nvars = (R.hdr.y >> 16) & 0xFF;
  for (uint32_t s = 0; s < nslots && s < (uint32_t)kSlots; ++s)
    HIPCHK(hipMemcpy(&R.slots[s], h->st.slots + s * N + i, sizeof(uint2), hipMemcpyDeviceToHost));
  for (uint32_t v = 0; v < nvars && v < (uint32_t)kVars; ++v) {
    HIPCHK(hipMemcpy(&R.vm[v], h->st.var_meta + v * N + i, sizeof(uint2), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&R.vv[v], h->st.var_val + v * N + i, sizeof(long long), hipMemcpyDeviceToHost));
  }
  for (int w = 0; w < kJoinWords; ++w)
    HIPCHK(hipMemcpy(&R.join[w], h->st.join + w * N + i, sizeof(uint32_t), hipMemcpyDeviceToHost));
  R.has_pms = h->st.n_slots != 0;
  if (R.has_pms) {
    HIPCHK(hipMemcpy(&R.pms, h->st.pms + i, sizeof(uint4), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&R.pms_msg, h->st.pms_msg + i, sizeof(long long), hipMemcpyDeviceToHost));
  }
  HIPCHK(hipMemcpy(&R.tmr, h->st.tmr + i, sizeof(uint4), hipMemcpyDeviceToHost));
  return ZBHIP_OK;
}

// MESSAGE_SUBSCRIPTION_BY_KEY / _BY_NAME_AND_CORRELATION_KEY rows of one correlation slot's kSubs rows
static void emit_slot_rows(zbhip_handle* h, uint32_t slot, const uint4* sa, const longlong2* sb, const longlong2* sk,
                           zbhip_state_sink sink, void* ctx) {
  char buf[768];
  for (int r = 0; r < kSubs; ++r) {
    const uint4 a = sa[r];
    const uint32_t st = a.x & 0xFF;
    if (st != 1 && st != 2) continue;
    const char* name = zbhip_name(h, a.y & 0xFFFF);
    const char* corr = zbhip_string_value(h, slot, nullptr);
    snprintf(buf, sizeof buf,
             "MESSAGE_SUBSCRIPTION_BY_KEY|%lld|%s|key=%lld,correlating=%d,processInstanceKey=%lld,bpmnProcessId=%s,"
             "messageKey=%lld,correlationKey=%s,interrupting=%u",
             (long long)sb[r].x, name, (long long)sk[r].x, st == 2 ? 1 : 0, (long long)sb[r].y,
             zbhip_name(h, a.y >> 16), (long long)sk[r].y, corr, (a.x >> 8) & 1);
    sink(ctx, buf);
    snprintf(buf, sizeof buf, "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY|<default>|%s|%s|%lld", name, corr,
             (long long)sb[r].x);
    sink(ctx, buf);
  }
}

int zbhip_export_state(zbhip_handle* h, zbhip_state_sink sink, void* ctx) {
  if (!h || !sink) return ZBHIP_EINVAL;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  const size_t N = h->st.n;
  std::vector<uint4> hdr(N);
  std::vector<uint2> slots(N * kSlots), vm(N * kVars);
  std::vector<long long> vv(N * kVars);
  std::vector<uint32_t> join(N * kJoinWords);
  std::vector<uint4> tmr(N);
  const size_t S = h->st.n_slots;
  std::vector<uint4> pms(S ? N : 0), sub_a(S * kSubs);
  std::vector<longlong2> sub_b(S * kSubs), sub_k(S * kSubs);
  HIPCHK(hipStreamSynchronize(h->stream));
  std::vector<long long> pms_msg(S ? N : 0, -1);
  if (S) {
    HIPCHK(hipMemcpy(pms.data(), h->st.pms, N * sizeof(uint4), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(pms_msg.data(), h->st.pms_msg, N * sizeof(long long), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(sub_a.data(), h->st.sub_a, S * kSubs * sizeof(uint4), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(sub_b.data(), h->st.sub_b, S * kSubs * sizeof(longlong2), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(sub_k.data(), h->st.sub_k, S * kSubs * sizeof(longlong2), hipMemcpyDeviceToHost));
  }
  HIPCHK(hipMemcpy(hdr.data(), h->st.hdr, N * sizeof(uint4), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(slots.data(), h->st.slots, N * kSlots * sizeof(uint2), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(vm.data(), h->st.var_meta, N * kVars * sizeof(uint2), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(vv.data(), h->st.var_val, N * kVars * sizeof(long long), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(join.data(), h->st.join, N * kJoinWords * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(tmr.data(), h->st.tmr, N * sizeof(uint4), hipMemcpyDeviceToHost));
  char buf[768];
  snprintf(buf, sizeof buf, "KEY|latestKey|%lld", (long long)(((int64_t)h->cfg.partition_id << 51) + h->key_counter));
  sink(ctx, buf);
  InstRows R{};
  for (size_t i = 0; i < N; ++i) {
    R.hdr = hdr[i];
    const uint32_t proc = R.hdr.x & 0xFFFF;
    // (an ended instance whose subscription is closing: header bit 25, its row only)
    const bool closing = proc == NONE && R.hdr.y == (1u << 25) && S;
    if (!closing && (proc == NONE || !((R.hdr.y >> 24) & 1))) continue;
    for (int k = 0; k < kSlots; ++k) R.slots[k] = slots[(size_t)k * N + i];
    for (int k = 0; k < kVars; ++k) {
      R.vm[k] = vm[(size_t)k * N + i];
      R.vv[k] = vv[(size_t)k * N + i];
    }
    for (int k = 0; k < kJoinWords; ++k) R.join[k] = join[(size_t)k * N + i];
    R.has_pms = S != 0;
    if (S) {
      R.pms = pms[i];
      R.pms_msg = pms_msg[i];
    }
    R.tmr = tmr[i];
    emit_instance(h, (uint32_t)i, R, sink, ctx);
  }
  // MESSAGE_SUBSCRIPTION_BY_KEY [eik, name] and MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY
  // [tenant, name, correlationKey, eik] of this (message) partition (DbMessageSubscriptionState)
  for (size_t slot = 0; slot < S; ++slot)
    emit_slot_rows(h, (uint32_t)slot, &sub_a[sub_ri(0, slot)], &sub_b[sub_ri(0, slot)], &sub_k[sub_ri(0, slot)], sink, ctx);
  if (h->published) sink(ctx, "MESSAGE_STATS|messagesDeadlineCount|0");
  return ZBHIP_OK;
}

// The message state of correlation slots (one owner per correlation key): the slots'
// MESSAGE_SUBSCRIPTION rows as zbhip_export_state writes them, for the engine's state.
int zbhip_export_correlation_slots(zbhip_handle* h, const uint32_t* slots, size_t n, zbhip_state_sink sink, void* ctx) {
  if (!h || !sink || (n && !slots)) return ZBHIP_EINVAL;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  const size_t S = h->st.n_slots;
  HIPCHK(hipStreamSynchronize(h->stream));
  for (size_t i = 0; i < n; ++i) {
    if (slots[i] >= S) return ZBHIP_EINVAL;
    uint4 a[kSubs];
    longlong2 b[kSubs], k[kSubs];
    const size_t r0 = sub_ri(0, slots[i]);
    HIPCHK(hipMemcpy(a, h->st.sub_a + r0, sizeof a, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(b, h->st.sub_b + r0, sizeof b, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(k, h->st.sub_k + r0, sizeof k, hipMemcpyDeviceToHost));
    emit_slot_rows(h, slots[i], a, b, k, sink, ctx);
  }
  return ZBHIP_OK;
}

int zbhip_export_correlation_slots_db(zbhip_handle* h, const uint32_t* slots, size_t n, zbhip_db_sink sink, void* ctx) {
  if (!h || !sink) return ZBHIP_EINVAL;
  DbExport e{h->ser, sink, ctx, ZBHIP_OK};
  const int rc = zbhip_export_correlation_slots(h, slots, n, db_row, &e);
  return rc ? rc : e.rc;
}

// The slots' MESSAGE_SUBSCRIPTION rows leave the device (after zbhip_export_correlation_slots put them into
// the engine's state): zeroed rows are free rows.
int zbhip_evict_correlation_slots(zbhip_handle* h, const uint32_t* slots, size_t n) {
  if (!h || (n && !slots)) return ZBHIP_EINVAL;
  const size_t S = h->st.n_slots;
  for (size_t i = 0; i < n; ++i) {
    if (slots[i] >= S) return ZBHIP_EINVAL;
    const size_t r0 = sub_ri(0, slots[i]);
    HIPCHK(hipMemsetAsync(h->st.sub_a + r0, 0, kSubs * sizeof(uint4), h->stream));
    HIPCHK(hipMemsetAsync(h->st.sub_b + r0, 0, kSubs * sizeof(longlong2), h->stream));
    HIPCHK(hipMemsetAsync(h->st.sub_k + r0, 0, kSubs * sizeof(longlong2), h->stream));
    // slot_hdr.x bit 31: the engine owns the key -- the device declines its commands (local follow-ups
    // of an instance's batch included: FB_MESSAGE), so the adapter hands such an instance to the engine
    uint2 sh;
    HIPCHK(hipMemcpyAsync(&sh, h->st.slot_hdr + slots[i], sizeof sh, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    sh.x |= 1u << 31;
    HIPCHK(hipMemcpyAsync(h->st.slot_hdr + slots[i], &sh, sizeof sh, hipMemcpyHostToDevice, h->stream));
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return ZBHIP_OK;
}

int zbhip_export_instances_db(zbhip_handle* h, const uint32_t* instances, size_t n, zbhip_db_sink sink, void* ctx) {
  if (!h || !sink) return ZBHIP_EINVAL;
  DbExport e{h->ser, sink, ctx, ZBHIP_OK};
  const int rc = zbhip_export_instances(h, instances, n, db_row, &e);
  return rc < 0 ? rc : e.rc;
}

// Hand-off of instances to the CPU engine: their slots are freed on the device (as a completed
// instance's: rows gone, the key ordinal kept) and their keys no longer resolve.
int zbhip_evict_instances(zbhip_handle* h, const uint32_t* instances, size_t n) {
  if (!h || (n && !instances)) return ZBHIP_EINVAL;
  if (int rc = advance(h, ~(size_t)0, false)) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  for (size_t k = 0; k < n; ++k) {
    const uint32_t i = instances[k];
    if (i >= h->st.n) return ZBHIP_EINVAL;
    uint4 hd;
    HIPCHK(hipMemcpy(&hd, h->st.hdr + i, sizeof hd, hipMemcpyDeviceToHost));
    const uint4 freed = make_uint4(0xFFFFu | (hd.x & 0xFFFF0000u), 0, 0, hd.w);  // the fence stays
    HIPCHK(hipMemcpy(h->st.hdr + i, &freed, sizeof freed, hipMemcpyHostToDevice));
    const uint32_t zero[kJoinWords] = {0, 0, 0, 0};
    for (int w = 0; w < kJoinWords; ++w)
      HIPCHK(hipMemcpy(h->st.join + (size_t)w * h->st.n + i, &zero[w], sizeof(uint32_t), hipMemcpyHostToDevice));
    const uint4 z = make_uint4(0, 0, 0, 0);
    if (h->st.n_slots) HIPCHK(hipMemcpy(h->st.pms + i, &z, sizeof z, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->st.tmr + i, &z, sizeof z, hipMemcpyHostToDevice));
    if (i < h->inst_gen.size()) ++h->inst_gen[i];
    for (auto it = h->job_index.begin(); it != h->job_index.end();)
      it = it->second.first == i ? h->job_index.erase(it) : std::next(it);
    for (auto it = h->activated.begin(); it != h->activated.end();)
      it = it->second.inst == i ? h->activated.erase(it) : std::next(it);
    // its follow-ups still waiting in the log now belong to the CPU engine, which reads them back
    if (h->deferred_per_inst.erase(i))
      for (auto it = h->deferred.begin(); it != h->deferred.end();)
        it = it->second.instance == i ? h->deferred.erase(it) : std::next(it);
  }
  return ZBHIP_OK;
}

int zbhip_continuations(zbhip_handle* h, uint64_t* first_id, uint64_t* n) {
  if (!h || !first_id || !n) return ZBHIP_EINVAL;
  *first_id = h->last_cont_first;
  *n = h->last_cont_n;
  return ZBHIP_OK;
}

int zbhip_pending_continuations(zbhip_handle* h, uint32_t instance) {
  if (!h) return ZBHIP_EINVAL;
  auto it = h->deferred_per_inst.find(instance);
  return it == h->deferred_per_inst.end() ? 0 : (int)it->second;
}

// DbKeyGenerator's current key after the last window (its key bookkeeping finished: the CPU
// engine's declared keys included, undeclared fallbacks counted as none)
int zbhip_current_key(zbhip_handle* h, int64_t* key) {
  if (!h || !key) return ZBHIP_EINVAL;
  if (h->ran && !h->results) return ZBHIP_ESTATE;  // a benchmarking run: keys were not counted
  if (int rc = finalize(h)) return rc;
  *key = ((int64_t)h->cfg.partition_id << 51) + h->key_counter;
  return ZBHIP_OK;
}

// KeyGeneratorControls.setKeyIfHigher (stream-platform/.../state/DbKeyGenerator.java:54-61): keys the
// CPU engine generated between two windows; the next window's keys follow them
int zbhip_set_key_if_higher(zbhip_handle* h, int64_t key) {
  if (!h) return ZBHIP_EINVAL;
  if (h->ran && !h->results) return ZBHIP_ESTATE;
  const int64_t pbits = (int64_t)h->cfg.partition_id << 51;
  if (key < pbits || key - pbits >= (1LL << 51)) return ZBHIP_EINVAL;  // another partition's key
  if (int rc = finalize(h)) return rc;
  if (key - pbits > h->key_counter) {
    h->key_counter = key - pbits;
    const unsigned long long kc = (unsigned long long)h->key_counter;
    HIPCHK(hipMemcpyAsync(h->d_key_counter, &kc, sizeof kc, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return ZBHIP_OK;
}

// DbKeyGenerator's value before window command i: the keys of the commands before it, the CPU
// engine's declared ones included
int zbhip_key_before(zbhip_handle* h, size_t i, int64_t* key) {
  if (!h || !key) return ZBHIP_EINVAL;
  if (!h->results) return ZBHIP_ESTATE;
  if (i > h->n_cmds) return ZBHIP_EINVAL;
  if (int rc = advance(h, i, false)) return rc;
  if (i < h->fin_next) {
    *key = ((int64_t)h->cfg.partition_id << 51) + h->h_base[i];
    return ZBHIP_OK;
  }
  int64_t c = h->key_counter;  // after commands < fin_next
  ensure_ext(h);
  for (size_t k = h->fin_next; k < i; ++k) {
    const uint2 hd = h->h_hdr[k];
    c += ((hd.y >> 16) & 0xFF) == ST_OK ? (int64_t)(hd.x >> 16) : (int64_t)h->ext_keys[k];
  }
  *key = ((int64_t)h->cfg.partition_id << 51) + c;
  return ZBHIP_OK;
}

int zbhip_set_external_keys(zbhip_handle* h, size_t i, uint32_t nkeys) {
  if (!h) return ZBHIP_EINVAL;
  if (!h->results) return ZBHIP_ESTATE;
  if (i >= h->n_cmds || ((h->h_hdr[i].y >> 16) & 0xFF) == ST_OK) return ZBHIP_EINVAL;
  if (i < h->fin_next) return ZBHIP_ESTATE;  // the keys after it are fixed already
  // config 5: the device key scan fixed this window's keys already (outbox, slot rows): the engine's keys
  // can only come after the window's last device key -- no later command of the window generated one (the
  // adapter runs a process-instance command last in its window when a fallback may take engine keys); the
  // next window starts after them (zbhip_set_key_if_higher)
  if (h->msg() && nkeys) {
    for (size_t j = i + 1; j < h->n_cmds; ++j)
      if (((h->h_hdr[j].y >> 16) & 0xFF) == ST_OK && (h->h_hdr[j].x >> 16) != 0) return ZBHIP_EUNSUPP;
    return ZBHIP_OK;
  }
  ensure_ext(h);
  h->ext_keys[i] = nkeys;
  h->declared[i] = 1;
  return ZBHIP_OK;
}

int zbhip_export_instances(zbhip_handle* h, const uint32_t* instances, size_t n, zbhip_state_sink sink, void* ctx) {
  if (!h || !sink || (n && !instances)) return ZBHIP_EINVAL;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  // the keys up to the first undeclared fallback command (a fallback instance's own history ends
  // before its fallback command: later commands of it are fenced)
  if (int rc = advance(h, ~(size_t)0, false)) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  for (size_t k = 0; k < n; ++k) {
    if (instances[k] >= h->st.n) return ZBHIP_EINVAL;
    InstRows R{};
    if (int rc = gather_instance(h, instances[k], R)) return rc;
    emit_instance(h, instances[k], R, sink, ctx);
  }
  return ZBHIP_OK;
}

}  // extern "C"

// ---- import: canonical rows / zb-db entries -> SoA rows ---------------------
namespace {
std::vector<std::string> split_row(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t a = 0;
  for (;;) {
    const size_t b = s.find(sep, a);
    out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
    if (b == std::string::npos) break;
    a = b + 1;
  }
  return out;
}
std::unordered_map<std::string, std::string> row_fields(const std::string& s) {
  std::unordered_map<std::string, std::string> f;
  for (const auto& kv : split_row(s, ',')) {
    const size_t e = kv.find('=');
    if (e != std::string::npos) f[kv.substr(0, e)] = kv.substr(e + 1);
  }
  return f;
}
int64_t to_ll(const std::string& s) { return strtoll(s.c_str(), nullptr, 10); }

struct ImpElement {
  int64_t key = 0, job = 0, pik = 0, fs = 0, def = 0, child_count = 0, asf = 0;
  int64_t activated = 0, completed = 0, terminated = 0, loop = 0;  // multi-instance counters
  uint32_t state = 0, type = 0;
  std::string id;
};
struct ImpVar {
  int64_t scope = 0, key = 0, value = 0;
  std::string name;
  uint32_t type = 0;
};
struct ImpTimer {
  int64_t eik = 0, key = 0, due = 0;
  std::string handler;
  uint32_t reps = 1;  // repetitions as the timer row holds them (255 infinite)
};
struct ImpPms {
  int64_t eik = 0, key = 0;
  std::string name, corr, elem_id;
  uint32_t state = 0, part = 0, intr = 0;
  int64_t msg = -1;  // messageKey of the stored record (a non-interrupting subscription's last correlation)
};
int64_t string_interner(void* ctx, const char* b, size_t n) {
  return zbhip_intern_string(static_cast<zbhip_handle*>(ctx), b, n);
}
}  // namespace

extern "C" int zbhip_import_state(zbhip_handle* h, const char* text, size_t len, uint32_t first_slot,
                                  uint32_t* n_instances) {
  if (!h || (len && !text)) return ZBHIP_EINVAL;
  if (n_instances) *n_instances = 0;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  h->ring_ok = false;  // imported keys are not in the device key ring: the host serialiser from now on
  if (h->st.act)  // (activations of earlier instances in the slots no longer apply)
    HIPCHK(hipMemset(h->st.act, 0, (size_t)kSlots * h->cfg.max_instances * sizeof(uint4)));
  std::map<int64_t, ImpElement> els;
  std::vector<ImpVar> vars;
  std::vector<std::tuple<int64_t, std::string, std::string, uint32_t>> taken;
  std::set<int64_t> job_rows;
  std::map<int64_t, std::pair<int64_t, std::string>> job_act;  // ACTIVATED jobs: deadline, worker
  std::set<int64_t> job_activated_state;
  struct JobMeta {
    int64_t eik, pik;
    std::string element_id;
    int32_t elem;  // (set where the job's element instance is rebuilt)
    bool failed_fields;  // JobFailProcessor stored retries / errorMessage (hex in the row)
    int32_t retries;
    std::string error_hex;
  };
  std::map<int64_t, JobMeta> job_meta;
  std::vector<ImpPms> pms;
  std::vector<ImpTimer> timers;
  int64_t latest = -1;
  bool stats_row = false;
  for (const std::string& row : split_row(std::string(text, len), '\n')) {
    if (row.empty()) continue;
    const auto p = split_row(row, '|');
    const std::string& cf = p[0];
    if (cf == "KEY" && p.size() >= 3) {
      latest = to_ll(p[2]);
    } else if (cf == "ELEMENT_INSTANCE_KEY" && p.size() >= 3) {
      auto f = row_fields(p[2]);
      ImpElement e;
      e.key = to_ll(p[1]);
      e.job = to_ll(f["jobKey"]);
      e.pik = to_ll(f["processInstanceKey"]);
      e.fs = to_ll(f["flowScopeKey"]);
      e.def = to_ll(f["processDefinitionKey"]);
      e.child_count = to_ll(f["childCount"]);
      e.asf = to_ll(f["activeSequenceFlows"]);
      e.activated = to_ll(f["childActivatedCount"]);
      e.completed = to_ll(f["childCompletedCount"]);
      e.terminated = to_ll(f["childTerminatedCount"]);
      e.loop = to_ll(f["multiInstanceLoopCounter"]);
      e.state = (uint32_t)to_ll(f["state"]);
      e.type = (uint32_t)to_ll(f["bpmnElementType"]);
      e.id = f["elementId"];
      els[e.key] = e;
    } else if (cf == "VARIABLES" && p.size() >= 4) {
      auto f = row_fields(p[3]);
      const uint32_t type = (uint32_t)to_ll(f["type"]);
      int64_t value = to_ll(f["value"]);
      if (type == ZBHIP_DOC_LIST) {  // a list: its items in the row
        zbhip_handle::Items items;
        for (const std::string& it : split_row(f["value"], ';')) {
          if (it.empty()) continue;
          const size_t c = it.find(':');
          if (c == std::string::npos) return ZBHIP_EINVAL;
          items.push_back({(uint8_t)to_ll(it.substr(0, c)), to_ll(it.substr(c + 1))});
        }
        value = intern_items(h, items);
        if (value < 0) return (int)value;
      }
      vars.push_back({to_ll(p[1]), to_ll(f["key"]), value, p[2], type});
    } else if (cf == "NUMBER_OF_TAKEN_SEQUENCE_FLOWS" && p.size() >= 5) {
      taken.emplace_back(to_ll(p[1]), p[2], p[3], (uint32_t)to_ll(p[4]));
    } else if (cf == "JOBS" && p.size() >= 3) {
      job_rows.insert(to_ll(p[1]));
      auto f = row_fields(p[2]);
      job_act[to_ll(p[1])] = {f.count("deadline") ? to_ll(f["deadline"]) : -1, f["worker"]};
      job_meta[to_ll(p[1])] = {to_ll(f["elementInstanceKey"]), to_ll(f["processInstanceKey"]), f["elementId"], -1,
                               f.count("errorMessageHex") != 0, (int32_t)to_ll(f["retries"]), f["errorMessageHex"]};
    } else if (cf == "JOB_STATES" && p.size() >= 3) {
      if (p[2] == "ACTIVATED") job_activated_state.insert(to_ll(p[1]));
      else if (p[2] != "ACTIVATABLE") return ZBHIP_EUNSUPP;  // failed / error-thrown jobs: outside the subset
    } else if (cf == "PROCESS_SUBSCRIPTION_BY_KEY" && p.size() >= 4) {
      auto f = row_fields(p[3]);
      ImpPms m;
      m.eik = to_ll(p[1]);
      m.name = p[2];
      m.key = to_ll(f["key"]);
      // a closing subscription (its element instance may be gone) is outside the import subset
      if (f["state"] == "CLOSING") return ZBHIP_EUNSUPP;
      m.state = f["state"] == "OPENING" ? 1u : 2u;
      m.part = (uint32_t)to_ll(f["subscriptionPartitionId"]);
      m.corr = f["correlationKey"];
      m.elem_id = f["elementId"];
      m.intr = (uint32_t)to_ll(f["interrupting"]);
      m.msg = f.count("messageKey") ? to_ll(f["messageKey"]) : -1;
      pms.push_back(m);
    } else if (cf == "TIMERS" && p.size() >= 4) {
      auto f = row_fields(p[3]);
      const int64_t reps = to_ll(f["repetitions"]);  // -1 (infinite) or 1..254 on the device
      if (reps != -1 && (reps < 1 || reps > 254)) return ZBHIP_EUNSUPP;
      timers.push_back({to_ll(p[1]), to_ll(p[2]), to_ll(f["dueDate"]), f["handlerNodeId"], reps == -1 ? 255u : (uint32_t)reps});
    } else if (cf == "MESSAGE_SUBSCRIPTION_BY_KEY" || cf == "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY") {
      return ZBHIP_EUNSUPP;  // message-partition rows: no routing handle to the subscriber's slot
    } else if (cf == "MESSAGE_STATS") {
      stats_row = true;
    }
    // ELEMENT_INSTANCE_PARENT_CHILD / _CHILD_PARENT, PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY,
    // EVENT_SCOPE, JOB_STATES, JOB_ACTIVATABLE follow from the rows above
  }
  if (!pms.empty() && !h->st.n_slots) return ZBHIP_EUNSUPP;
  std::vector<int64_t> piks;
  for (const auto& kv : els)
    if (kv.second.type == ZBHIP_EL_PROCESS) piks.push_back(kv.first);  // map order: key order
  const size_t N = h->st.n;
  if ((size_t)first_slot + piks.size() > N) return ZBHIP_ENOMEM;
  if (piks.empty() && latest < 0) return ZBHIP_OK;

  // the partition's SoA rows, edited on the host and written back once
  std::vector<uint4> hdr(N);
  std::vector<uint2> slots(N * kSlots), vm(N * kVars);
  std::vector<long long> vv(N * kVars);
  std::vector<uint32_t> join(N * kJoinWords);
  std::vector<uint4> pmsrow(h->st.n_slots ? N : 0);
  std::vector<long long> pmseik(h->st.n_slots ? N : 0, -1);
  std::vector<long long> pmsmsg(h->st.n_slots ? N : 0, -1);
  std::vector<long long> pikrow(h->st.n_slots ? N : 0);
  std::vector<uint4> tmrrow(N);
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(hdr.data(), h->st.hdr, N * sizeof(uint4), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(slots.data(), h->st.slots, N * kSlots * sizeof(uint2), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(vm.data(), h->st.var_meta, N * kVars * sizeof(uint2), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(vv.data(), h->st.var_val, N * kVars * sizeof(long long), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(join.data(), h->st.join, N * kJoinWords * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(tmrrow.data(), h->st.tmr, N * sizeof(uint4), hipMemcpyDeviceToHost));
  if (h->st.n_slots) {
    HIPCHK(hipMemcpy(pmsrow.data(), h->st.pms, N * sizeof(uint4), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(pmseik.data(), h->st.pms_eik, N * sizeof(long long), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(pmsmsg.data(), h->st.pms_msg, N * sizeof(long long), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(pikrow.data(), h->st.pi_key, N * sizeof(long long), hipMemcpyDeviceToHost));
  }
  const int64_t pbits = (int64_t)h->cfg.partition_id << 51;
  const size_t subjects = (size_t)h->cfg.max_instances + h->st.n_slots;
  if (h->hist.size() < subjects) {
    h->hist.resize(subjects);
    h->inst_proc.resize(h->cfg.max_instances, NONE);
    h->inst_gen.resize(subjects, 0);
  }
  struct Done {
    uint32_t slot;
    std::vector<int64_t> keys;
  };
  std::vector<Done> done;
  for (size_t k = 0; k < piks.size(); ++k) {
    const uint32_t inst = first_slot + (uint32_t)k;
    const ImpElement& pe = els[piks[k]];
    if ((hdr[inst].x & 0xFFFF) != NONE) return ZBHIP_EINVAL;  // the slot holds an instance
    int proc = -1;
    for (size_t q = 0; q < h->procs.size(); ++q)
      if (h->procs[q].def_key == pe.def) proc = (int)q;
    if (proc < 0) return ZBHIP_EINVAL;  // not deployed
    const Proc& P = h->procs[proc];
    // an element by id and type (a multi-instance body and its inner activity share the id)
    auto elem_of_id = [&](const std::string& id, uint32_t type = ~0u) -> int {
      for (size_t e = 0; e < P.els.size(); ++e)
        if (P.els[e].element_type != ZBHIP_EL_SEQUENCE_FLOW && P.id((uint32_t)e) == id &&
            (type == ~0u || P.els[e].element_type == type))
          return (int)e;
      return -1;
    };
    // keys of the instance: ordinal 0 the instance, then every other key in key order
    std::vector<const ImpElement*> children;
    std::vector<int64_t> keys;
    std::set<int64_t> subs;  // embedded sub-process instances of this process instance
    for (const auto& kv : els) {
      const ImpElement& e = kv.second;
      if (e.pik != pe.key || e.key == pe.key) continue;
      children.push_back(&e);
      keys.push_back(e.key);
      if (e.type == ZBHIP_EL_SUB_PROCESS || e.type == ZBHIP_EL_MULTI_INSTANCE_BODY) subs.insert(e.key);
      else if (e.job > 0) keys.push_back(e.job);
    }
    // flow scopes: the process instance or one of its sub-process / multi-instance body instances
    // (KScope slots); a container's counters live in its slot's job field
    for (const ImpElement* c : children) {
      if (c->fs != pe.key && !subs.count(c->fs)) return ZBHIP_EUNSUPP;
      if (c->type == ZBHIP_EL_SUB_PROCESS && (c->child_count < 0 || c->child_count > 255 || c->asf < 0 || c->asf > 255))
        return ZBHIP_EUNSUPP;
      if (c->terminated != 0) return ZBHIP_EUNSUPP;
      // an exclusive gateway waits only with an incident (INCIDENTS rows are not imported): CPU engine
      if (c->type == ZBHIP_EL_EXCLUSIVE_GATEWAY) return ZBHIP_EUNSUPP;
      if (c->type == ZBHIP_EL_MULTI_INSTANCE_BODY &&  // childActivatedCount = loop, completed = loop - active
          (c->loop < 0 || c->loop > (int64_t)kMaxMiItems || c->asf != 0 || c->activated != c->loop ||
           c->child_count < 0 || c->completed != c->loop - c->child_count))
        return ZBHIP_EUNSUPP;
      if (c->type != ZBHIP_EL_MULTI_INSTANCE_BODY && c->loop != 0 &&
          !(subs.count(c->fs) && els[c->fs].type == ZBHIP_EL_MULTI_INSTANCE_BODY))
        return ZBHIP_EUNSUPP;
    }
    std::vector<const ImpVar*> ivars;
    auto scope_of = [&](int64_t s) { return s == pe.key || std::any_of(children.begin(), children.end(), [&](const ImpElement* c) { return c->key == s; }); };
    // a multi-instance inner instance's own variables: its loop variables, derived from its slot on
    // the device (checked against the program below); their keys take ordinals like any other.  A
    // body's local outputCollection is the host's (mi_out)
    std::map<int64_t, std::map<std::string, const ImpVar*>> loop_vars;
    std::vector<std::pair<int64_t, const ImpVar*>> out_colls;
    for (const auto& v : vars)
      if (scope_of(v.scope)) {
        if (subs.count(v.scope) && els[v.scope].type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
          const int be = elem_of_id(els[v.scope].id, ZBHIP_EL_MULTI_INSTANCE_BODY);
          const Proc::Mi* bm = be < 0 ? nullptr : P.mi_body((uint32_t)be);
          if (!bm || bm->out_coll == NONE || h->names[bm->out_coll] != v.name || v.type != ZBHIP_DOC_LIST)
            return ZBHIP_EUNSUPP;
          keys.push_back(v.key);
          out_colls.push_back({v.scope, &v});
          continue;
        }
        // container-local variables: written by a sub-process's input mapping (KScopeIO) only
        if (subs.count(v.scope) && (!P.has_io || els[v.scope].type != ZBHIP_EL_SUB_PROCESS)) return ZBHIP_EUNSUPP;
        keys.push_back(v.key);
        if (v.scope != pe.key) {
          const ImpElement& se = els[v.scope];
          if (subs.count(se.fs) && els[se.fs].type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
            loop_vars[v.scope][v.name] = &v;
            continue;
          }
        }
        ivars.push_back(&v);
      }
    const ImpTimer* tmr = nullptr;  // the instance's timer (one per instance on the device)
    for (const auto& t : timers)
      if (std::any_of(children.begin(), children.end(), [&](const ImpElement* c) { return c->key == t.eik; })) {
        if (tmr) return ZBHIP_EUNSUPP;
        tmr = &t;
        keys.push_back(t.key);
      }
    const ImpPms* sub = nullptr;
    for (const auto& m : pms)
      if (std::any_of(children.begin(), children.end(), [&](const ImpElement* c) { return c->key == m.eik; })) {
        if (sub) return ZBHIP_EUNSUPP;  // one open subscription per instance
        sub = &m;
        keys.push_back(m.key);
      }
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    keys.erase(std::remove(keys.begin(), keys.end(), pe.key), keys.end());
    keys.insert(keys.begin(), pe.key);
    if (keys.size() >= 0xFFF0) return ZBHIP_ENOMEM;
    auto ord = [&](int64_t key) -> uint32_t {
      return (uint32_t)(std::lower_bound(keys.begin() + 1, keys.end(), key) - keys.begin());
    };
    if (children.size() > (size_t)kSlots || ivars.size() > (size_t)kVars) return ZBHIP_ENOMEM;
    for (size_t c = 0; c < children.size(); ++c) {
      const ImpElement& e = *children[c];
      const int el = elem_of_id(e.id, e.type);
      if (el < 0 || P.els[el].element_type != e.type) return ZBHIP_EINVAL;
      const bool in_container = e.fs != pe.key && (els[e.fs].type == ZBHIP_EL_SUB_PROCESS ||
                                                   els[e.fs].type == ZBHIP_EL_MULTI_INSTANCE_BODY);
      if (P.els[el].flow_scope != (e.fs == pe.key ? 0u : in_container ? (uint32_t)elem_of_id(els[e.fs].id, els[e.fs].type)
                                                                      : ~0u))
        return ZBHIP_EINVAL;  // the flow scope instance is not the element's container
      const bool sub_el = e.type == ZBHIP_EL_SUB_PROCESS, body = e.type == ZBHIP_EL_MULTI_INSTANCE_BODY;
      uint32_t job = sub_el ? (uint32_t)e.child_count | ((uint32_t)e.asf << 8)
                     : body ? (uint32_t)e.child_count | ((uint32_t)e.loop << 8)
                     : e.job == 0 ? JOB_ZERO : e.job == -1 ? JOB_MINUS1 : ord(e.job);
      // (flag bit 1: a stored activation -- ACTIVATED, or timed out with its deadline and worker kept)
      const auto ja = job_act.find(e.job);
      const auto jmf = job_meta.find(e.job);
      // a failure that left errorMessage, retryBackoff and recurringTime at their defaults shows in its
      // retries alone
      if (jmf != job_meta.end() && !sub_el && !body && jmf->second.retries != (int32_t)P.els[el].job_retries)
        jmf->second.failed_fields = true;
      const bool stored = job_activated_state.count(e.job) ||
                          (ja != job_act.end() && (ja->second.first != -1 || !ja->second.second.empty())) ||
                          (jmf != job_meta.end() && jmf->second.failed_fields);
      uint32_t row = !sub_el && !body && e.job > 0 && job_rows.count(e.job) ? (stored ? 3u : 1u) : 0u;
      if (row) {
        const auto jm = job_meta.find(e.job);
        if (jm != job_meta.end()) jm->second.elem = el;
      }
      if (const Proc::Mi* m = P.mi_inner((uint32_t)el)) {
        // the loop counter in the flags; its loop variables exactly what setLoopVariables wrote,
        // keyed right below the job's key (a job worker) or kept in the job field (an undefined task);
        // the items: the static ones or the imported collection variable's (the process instance's)
        const zbhip_handle::Items* coll = &m->items;
        if (m->coll_name != NONE) {
          coll = nullptr;
          for (const auto& v : vars)
            if (v.scope == pe.key && v.name == h->names[m->coll_name] && v.type == ZBHIP_DOC_LIST)
              coll = &h->lists[(size_t)v.value];
          if (!coll) return ZBHIP_EUNSUPP;
        }
        if (e.loop < 1 || e.loop > (int64_t)coll->size()) return ZBHIP_EUNSUPP;
        const uint32_t ko = m->out_local() ? 1u : 0u;
        const auto lv = loop_vars.find(e.key);
        if (lv == loop_vars.end() || lv->second.size() != (m->input_name != NONE ? 2u : 1u) + ko) return ZBHIP_EUNSUPP;
        const auto li = lv->second.find(h->names[m->loop_name]);
        if (li == lv->second.end() || li->second->type != ZBHIP_DOC_INT || li->second->value != e.loop) return ZBHIP_EUNSUPP;
        const uint32_t kl = ord(li->second->key);
        if (ko) {  // the local outputElement: nil until the batch that completes the instance
          const auto oi = lv->second.find(h->names[m->out_elem]);
          if (oi == lv->second.end() || oi->second->type != ZBHIP_DOC_NIL || ord(oi->second->key) + 1 != kl)
            return ZBHIP_EUNSUPP;
        }
        if (m->input_name != NONE) {
          const auto ii = lv->second.find(h->names[m->input_name]);
          const auto& item = (*coll)[(size_t)e.loop - 1];
          if (ii == lv->second.end() || ii->second->type != item.first || ii->second->value != item.second ||
              ord(ii->second->key) + 1 + ko != kl)
            return ZBHIP_EUNSUPP;
        }
        if (ZBHIP_IS_JOB_WORKER(e.type) ? !(row & 1) || job != kl + 1 : e.job != 0) return ZBHIP_EUNSUPP;
        if (!ZBHIP_IS_JOB_WORKER(e.type)) job = kl;
        row |= (uint32_t)e.loop << 2;
      } else if (!loop_vars.empty() && loop_vars.count(e.key)) {
        return ZBHIP_EUNSUPP;
      }
      slots[c * N + inst] = make_uint2((uint32_t)el | (ord(e.key) << 16), job | (e.state << 16) | (row << 24));
    }
    for (size_t v = 0; v < ivars.size(); ++v) {
      const ImpVar& x = *ivars[v];
      const int name = zbhip_intern(h, x.name.c_str());
      if (name < 0) return name;
      const uint32_t scope = x.scope == pe.key ? 0u : ord(x.scope);
      vm[v * N + inst] = make_uint2((uint32_t)name | (scope << 16), ord(x.key) | (x.type << 16));
      vv[v * N + inst] = x.value;
    }
    for (int w = 0; w < kJoinWords; ++w) join[(size_t)w * N + inst] = 0;
    for (const auto& t : taken) {
      if (std::get<0>(t) != pe.key && !subs.count(std::get<0>(t))) continue;
      int slot = -1;
      for (size_t f = 0; f < P.els.size(); ++f) {
        const zbhip_element& F = P.els[f];
        if (F.element_type == ZBHIP_EL_SEQUENCE_FLOW && P.id((uint32_t)f) == std::get<2>(t) && F.flow_target < P.els.size() &&
            P.id(F.flow_target) == std::get<1>(t))
          slot = F.join_slot == ZBHIP_NONE16 ? -1 : F.join_slot;
      }
      if (slot < 0 || std::get<3>(t) > 255) return ZBHIP_EUNSUPP;
      join[(size_t)(slot >> 2) * N + inst] |= std::get<3>(t) << ((slot & 3) * 8);
    }
    if (h->st.n_slots) {
      pmsrow[inst] = make_uint4(0, 0, 0, 0);
      pmseik[inst] = -1;
      pmsmsg[inst] = -1;
      pikrow[inst] = pe.key;
      if (sub) {
        const int el = elem_of_id(sub->elem_id);
        if (el < 0) return ZBHIP_EINVAL;
        const int64_t corr = zbhip_intern_string(h, sub->corr.data(), sub->corr.size());
        if (corr < 0) return (int)corr;
        const int name = zbhip_intern(h, sub->name.c_str());
        if (name < 0) return name;
        pmsrow[inst] = make_uint4((uint32_t)el | (sub->state << 12) | (sub->intr << 14) | (sub->part << 16),
                                  ord(sub->eik) | (ord(sub->key) << 16), (uint32_t)corr,
                                  (uint32_t)name | ((uint32_t)P.bpmn_name << 16));
        pmsmsg[inst] = sub->msg;
        // an opened subscription of another partition: its real element-instance key (the later DELETE's)
        if (sub->state == 2 && (int32_t)sub->part != h->cfg.partition_id) pmseik[inst] = sub->eik;
      }
    } else if (sub) {
      return ZBHIP_EUNSUPP;
    }
    tmrrow[inst] = make_uint4(0, 0, 0, 0);
    if (tmr) {
      const int el = elem_of_id(tmr->handler);
      if (el < 0 || !P.has_timer) return ZBHIP_EINVAL;
      tmrrow[inst] = make_uint4((uint32_t)el | (ord(tmr->key) << 16), ord(tmr->eik) | (tmr->reps << 16) | (1u << 31),
                                (uint32_t)(uint64_t)tmr->due, (uint32_t)((uint64_t)tmr->due >> 32));
    }
    hdr[inst] = make_uint4((uint32_t)proc | ((uint32_t)keys.size() << 16),
                           pe.state | ((uint32_t)children.size() << 8) | ((uint32_t)ivars.size() << 16) | (1u << 24),
                           (uint32_t)pe.child_count | ((uint32_t)pe.asf << 16), 0);
    for (const auto& [body_key, v] : out_colls) h->mi_out[body_key] = {v->key, h->lists[(size_t)v->value]};
    done.push_back({inst, std::move(keys)});
  }
  HIPCHK(hipMemcpy(h->st.hdr, hdr.data(), N * sizeof(uint4), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->st.slots, slots.data(), N * kSlots * sizeof(uint2), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->st.var_meta, vm.data(), N * kVars * sizeof(uint2), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->st.var_val, vv.data(), N * kVars * sizeof(long long), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->st.join, join.data(), N * kJoinWords * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->st.tmr, tmrrow.data(), N * sizeof(uint4), hipMemcpyHostToDevice));
  if (h->st.n_slots) {
    HIPCHK(hipMemcpy(h->st.pms, pmsrow.data(), N * sizeof(uint4), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->st.pms_eik, pmseik.data(), N * sizeof(long long), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->st.pms_msg, pmsmsg.data(), N * sizeof(long long), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->st.pi_key, pikrow.data(), N * sizeof(long long), hipMemcpyHostToDevice));
  }
  // key histories and the resolve_key table: one entry per imported key
  for (const Done& d : done) {
    auto& hs = h->hist[d.slot];
    hs.clear();
    ++h->inst_gen[d.slot];
    h->inst_proc[d.slot] = (uint16_t)(hdr[d.slot].x & 0xFFFF);
    for (size_t o = 0; o < d.keys.size(); ++o) {
      hs.push_back({(uint16_t)o, d.keys[o] - pbits});
      h->batches.push_back({d.keys[o] - pbits, d.slot, (uint16_t)o, 1, h->inst_gen[d.slot]});
    }
  }
  h->batches.sort_all();
  if (latest >= 0 && latest - pbits > h->key_counter) h->key_counter = latest - pbits;
  if (h->st.n_slots) {
    const unsigned long long kc = (unsigned long long)h->key_counter;
    HIPCHK(hipMemcpy(h->d_key_counter, &kc, sizeof kc, hipMemcpyHostToDevice));
  }
  h->published |= stats_row;
  for (const Done& d : done)
    for (int64_t k : d.keys)
      if (job_act.count(k) && (job_activated_state.count(k) || job_act[k].first != -1 || !job_act[k].second.empty() ||
                               (job_meta.count(k) && job_meta[k].failed_fields))) {
        const std::string& wk = job_act[k].second;
        const int64_t wid = wk.empty() ? (int64_t)ZBHIP_NO_STRING : zbhip_intern_string(h, wk.data(), wk.size());
        if (wid < 0) return (int)wid;
        zbhip_handle::Activation& a = h->activated[k];
        a = {job_act[k].first, wk, d.slot, (uint32_t)wid};
        a.state = job_activated_state.count(k) ? zbhip_handle::JS_ACTIVATED : zbhip_handle::JS_ACTIVATABLE;
        const auto jm = job_meta.find(k);
        if (jm != job_meta.end()) {
          a.eik = jm->second.eik;
          a.pik = jm->second.pik;
          a.proc = (int32_t)(hdr[d.slot].x & 0xFFFF);
          a.elem = jm->second.elem;
          if (jm->second.failed_fields) {  // a failed job with retries left (a FAILED one is refused above)
            std::string msg;
            const std::string& hx = jm->second.error_hex;
            for (size_t q = 0; q + 1 < hx.size(); q += 2) msg += (char)std::stoi(hx.substr(q, 2), nullptr, 16);
            const int64_t eid = msg.empty() ? (int64_t)ZBHIP_NO_STRING : zbhip_intern_string(h, msg.data(), msg.size());
            if (eid < 0) return (int)eid;
            a.fail_fields = true;
            a.retries = jm->second.retries;
            a.error_id = (uint32_t)eid;
            h->ring_ok = false;
          }
        }
      }
  h->job_index_on = false;  // rebuilt from the device rows at the next activation
  if (n_instances) *n_instances = (uint32_t)done.size();
  return ZBHIP_OK;
}

extern "C" int zbhip_import_state_db(zbhip_handle* h, const uint8_t* entries, size_t len, uint32_t first_slot,
                                     uint32_t* n_instances) {
  if (!h || (len && !entries)) return ZBHIP_EINVAL;
  std::string rows;
  std::vector<char> row(4096);
  size_t off = 0;
  while (off < len) {
    if (len - off < 12) return ZBHIP_EINVAL;
    uint32_t hd[3];
    memcpy(hd, entries + off, 12);
    off += 12;
    if (len - off < (size_t)hd[1] + hd[2]) return ZBHIP_EINVAL;
    int n = zbhip_serializer_decode_state_entry(h->ser, hd[0], entries + off, hd[1], entries + off + hd[1], hd[2],
                                                string_interner, h, row.data(), row.size());
    while (n == ZBHIP_ENOMEM && row.size() < ((size_t)1 << 26)) {  // a long value (an errorMessage: 10 000 chars)
      row.resize(row.size() * 8);
      n = zbhip_serializer_decode_state_entry(h->ser, hd[0], entries + off, hd[1], entries + off + hd[1], hd[2],
                                              string_interner, h, row.data(), row.size());
    }
    if (n < 0) return n;
    if (n > 0) {
      rows.append(row.data(), (size_t)n);
      rows.push_back('\n');
    }
    off += (size_t)hd[1] + hd[2];
  }
  return zbhip_import_state(h, rows.data(), rows.size(), first_slot, n_instances);
}

// After recovery (StreamProcessorLifecycleAware.onRecovered) the engine's state holds every instance:
// this marks the entries of the instances the handle can take over -- process instances of processes
// deployed on the handle, minus `exclude` (instances a command still waiting in the log addresses) --
// so the adapter imports exactly those (zbhip_import_state_db) and deletes them from RocksDB.  An
// entry belongs to the instance of its element instance / job / scope (the column families' keys).
extern "C" int zbhip_select_instances_db(zbhip_handle* h, const uint8_t* entries, size_t len, const int64_t* exclude,
                                         size_t n_exclude, uint8_t* take, size_t n_take, size_t* n_entries) {
  if (!h || (len && !entries) || (n_exclude && !exclude) || (n_take && !take)) return ZBHIP_EINVAL;
  std::vector<std::string> rows;
  std::vector<char> row(4096);
  size_t off = 0;
  while (off < len) {
    if (len - off < 12) return ZBHIP_EINVAL;
    uint32_t hd[3];
    memcpy(hd, entries + off, 12);
    off += 12;
    if (len - off < (size_t)hd[1] + hd[2]) return ZBHIP_EINVAL;
    int n = zbhip_serializer_decode_state_entry(h->ser, hd[0], entries + off, hd[1], entries + off + hd[1], hd[2],
                                                string_interner, h, row.data(), row.size());
    while (n == ZBHIP_ENOMEM && row.size() < ((size_t)1 << 26)) {  // a long value (an errorMessage: 10 000 chars)
      row.resize(row.size() * 8);
      n = zbhip_serializer_decode_state_entry(h->ser, hd[0], entries + off, hd[1], entries + off + hd[1], hd[2],
                                              string_interner, h, row.data(), row.size());
    }
    if (n < 0) return n;
    rows.emplace_back(row.data(), (size_t)n);
    off += (size_t)hd[1] + hd[2];
  }
  if (n_entries) *n_entries = rows.size();
  if (n_take < rows.size()) return ZBHIP_ENOMEM;
  auto split = [](const std::string& r) {
    std::vector<std::string> p;
    size_t s = 0;
    for (size_t i = 0; i <= r.size(); ++i)
      if (i == r.size() || r[i] == '|') { p.push_back(r.substr(s, i - s)); s = i + 1; }
    return p;
  };
  auto field = [](const std::string& f, const char* name) -> std::string {
    const std::string k = std::string(name) + "=";
    size_t a = 0;
    while (a < f.size()) {
      size_t e = f.find(',', a);
      if (e == std::string::npos) e = f.size();
      if (f.compare(a, k.size(), k) == 0) return f.substr(a + k.size(), e - a - k.size());
      a = e + 1;
    }
    return std::string();
  };
  std::unordered_set<int64_t> device_keys, excluded(exclude, exclude + n_exclude), eligible;
  for (const Proc& p : h->procs) device_keys.insert(p.def_key);
  std::unordered_map<int64_t, int64_t> ei, jobs;  // element instance / job key -> process instance key
  std::vector<std::vector<std::string>> parts(rows.size());
  for (size_t i = 0; i < rows.size(); ++i) {
    if (rows[i].empty()) continue;
    parts[i] = split(rows[i]);
    const auto& p = parts[i];
    if (p[0] == "ELEMENT_INSTANCE_KEY" && p.size() > 2) {
      const int64_t pik = std::stoll(field(p[2], "processInstanceKey"));
      ei[std::stoll(p[1])] = pik;
      if (field(p[2], "bpmnElementType") == "1" && device_keys.count(std::stoll(field(p[2], "processDefinitionKey"))) &&
          !excluded.count(pik))
        eligible.insert(pik);
    } else if (p[0] == "JOBS" && p.size() > 2) {
      jobs[std::stoll(p[1])] = std::stoll(field(p[2], "processInstanceKey"));
    }
  }
  auto owner = [&](const std::vector<std::string>& p) -> int64_t {
    auto in = [](const std::unordered_map<int64_t, int64_t>& m, const std::string& k) -> int64_t {
      auto it = m.find(std::stoll(k));
      return it == m.end() ? -1 : it->second;
    };
    const std::string& cf = p[0];
    if (p.size() < 2) return -1;
    if (cf == "ELEMENT_INSTANCE_KEY" || cf == "ELEMENT_INSTANCE_CHILD_PARENT" || cf == "NUMBER_OF_TAKEN_SEQUENCE_FLOWS" ||
        cf == "VARIABLES" || cf == "EVENT_SCOPE" || cf == "EVENT_TRIGGER" || cf == "TIMERS")
      return in(ei, p[1]);
    if (cf == "ELEMENT_INSTANCE_PARENT_CHILD" && p.size() > 2) return in(ei, p[2]);  // [parent, child]: the child's
    if (cf == "TIMER_DUE_DATES" && p.size() > 2) return in(ei, p[2]);
    if (cf == "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY" && p.size() > 2) return std::stoll(p[2]);
    if (cf == "JOBS" || cf == "JOB_STATES") return in(jobs, p[1]);
    if (cf == "JOB_ACTIVATABLE" && p.size() > 3) return in(jobs, p[3]);
    if (cf == "JOB_DEADLINES" && p.size() > 2) return in(jobs, p[2]);
    return -1;
  };
  try {
    for (size_t i = 0; i < rows.size(); ++i)
      take[i] = !parts[i].empty() && eligible.count(owner(parts[i])) ? 1 : 0;
  } catch (const std::exception&) {
    return ZBHIP_EINVAL;
  }
  return (int)eligible.size();
}

// ---- job activation ----------------------------------------------------------
// JOB_BATCH:ACTIVATE: the host's JOB_ACTIVATABLE index picks the jobs (type, then job key), the device
// marks them ACTIVATED and gathers their element instances and variables (k_activate_jobs).
static int build_job_index(zbhip_handle* h) {
  const size_t N = h->st.n;
  std::vector<uint4> hdr(N);
  std::vector<uint2> slots(N * kSlots);
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(hdr.data(), h->st.hdr, N * sizeof(uint4), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(slots.data(), h->st.slots, N * kSlots * sizeof(uint2), hipMemcpyDeviceToHost));
  h->job_index.clear();
  for (size_t i = 0; i < N; ++i) {
    const uint32_t proc = hdr[i].x & 0xFFFF;
    if (proc == NONE || proc >= h->procs.size() || !((hdr[i].y >> 24) & 1)) continue;
    const Proc& P = h->procs[proc];
    const uint32_t ns = (hdr[i].y >> 8) & 0xFF;
    for (uint32_t s = 0; s < ns && s < (uint32_t)kSlots; ++s) {
      const uint2 e = slots[s * N + i];
      const uint32_t elem = e.x & 0xFFFF, job = e.y & 0xFFFF, fl = e.y >> 24;
      if (!(fl & 1u) || elem >= P.els.size()) continue;  // a job row ...
      const int64_t jk = h->key_of((uint32_t)i, job);
      if (fl & 2u) {  // ... with a stored activation: activatable again once it timed out
        const auto ait = h->activated.find(jk);
        if (ait == h->activated.end() || ait->second.state != zbhip_handle::JS_ACTIVATABLE) continue;
      }
      h->job_index[{P.job_type_id[elem], jk}] = {(uint32_t)i, (uint16_t)job};
    }
  }
  h->job_index_on = true;
  return ZBHIP_OK;
}

// JobVariablesCollector.setJobVariables (DbVariableState.getVariablesAsDocument :193-247) over one job's
// gathered rows (k_activate_jobs' ActivatedOut): the element's scope, its enclosing containers', then the
// process instance's; names in DbString key order (length, bytes), each once, `requested` only if any.
static void collect_job_variables(zbhip_handle* h, const uint4& a, const uint2* meta, const long long* val,
                                  const uint2* slots, const std::vector<uint32_t>& requested, zbhip_activated_job& j) {
  auto name_less = [h](uint32_t x_, uint32_t y_) {
    const std::string& x = h->names[x_];
    const std::string& y = h->names[y_];
    return x.size() != y.size() ? x.size() < y.size() : x < y;
  };
  const uint32_t proc = a.y & 0xFFFF, elem = a.x & 0xFFFF, eord = a.x >> 16;
  // DbVariableState.visitVariables: the element's scope, then the process instance's
  const uint32_t nv = std::min<uint32_t>((a.z >> 16) & 0xFF, (uint32_t)kVars);
  std::vector<uint32_t> taken;
  const Proc::Mi* m = proc < h->procs.size() ? h->procs[proc].mi_inner(elem) : nullptr;
  const uint32_t loop = a.w >> 26;
  // the collection the inner instance's item comes from: the static items or the list variable's
  const zbhip_handle::Items* coll = m ? &m->items : nullptr;
  if (m && m->coll_name != NONE) {
    coll = nullptr;
    for (uint32_t v = 0; v < nv; ++v)
      if ((meta[v].x & 0xFFFF) == m->coll_name && ((meta[v].y >> 16) & 0xFF) == ZBHIP_DOC_LIST && val[v] >= 0 &&
          (size_t)val[v] < h->lists.size())
        coll = &h->lists[(size_t)val[v]];
  }
  if (m && coll && loop >= 1 && loop <= coll->size()) {
    // a multi-instance inner instance's scope: its loop variables (setLoopVariables: the inputElement,
    // the local outputElement -- nil --, the loopCounter), then the body's (its outputCollection),
    // then the process instance's
    std::vector<zbhip_doc_entry> local;
    if (m->input_name != NONE)
      local.push_back({m->input_name, (*coll)[loop - 1].first, {0, 0, 0}, (*coll)[loop - 1].second});
    if (m->out_local()) local.push_back({m->out_elem, (uint8_t)ZBHIP_DOC_NIL, {0, 0, 0}, 0});
    local.push_back({m->loop_name, (uint8_t)ZBHIP_DOC_INT, {0, 0, 0}, (int64_t)loop});
    std::sort(local.begin(), local.end(),
              [&](const zbhip_doc_entry& p, const zbhip_doc_entry& q) { return name_less(p.name_id, q.name_id); });
    for (const zbhip_doc_entry& d : local) {
      if (!requested.empty() && std::find(requested.begin(), requested.end(), d.name_id) == requested.end()) continue;
      if (j.n_variables >= 6) break;
      taken.push_back(d.name_id);
      j.variables[j.n_variables++] = d;
    }
    // the body's local outputCollection (the host's copy)
    if (m->out_coll != NONE && j.n_variables < 6 &&
        (requested.empty() || std::find(requested.begin(), requested.end(), m->out_coll) != requested.end()))
      for (uint32_t s = 0; s < (uint32_t)kSlots; ++s)
        if (slots[s].x != 0xFFFFFFFFu && (slots[s].x & 0xFFFF) == m->body) {
          const auto o = h->mi_out.find(h->key_of(j.instance, slots[s].x >> 16));
          if (o == h->mi_out.end()) break;
          const int64_t id = intern_items(h, o->second.items);
          if (id < 0) break;
          taken.push_back(m->out_coll);
          j.variables[j.n_variables++] = {m->out_coll, (uint8_t)ZBHIP_DOC_LIST, {0, 0, 0}, id};
          break;
        }
  }
  // the element's scope, the instances of its enclosing containers (sub-processes with io-mapped
  // variables), then the process instance's
  std::vector<uint32_t> chain{eord};
  if (proc < h->procs.size() && elem < h->procs[proc].els.size())
    for (uint32_t c = h->procs[proc].els[elem].flow_scope, d = 0; c != 0 && c < h->procs[proc].els.size() && d < 16;
         c = h->procs[proc].els[c].flow_scope, ++d)
      for (uint32_t si = 0; si < (uint32_t)kSlots; ++si)
        if (slots[si].x != 0xFFFFFFFFu && (slots[si].x & 0xFFFF) == c) chain.push_back(slots[si].x >> 16);
  chain.push_back(0u);
  for (uint32_t scope : chain) {
    std::vector<uint32_t> local;
    for (uint32_t v = 0; v < nv; ++v)
      if ((meta[v].x >> 16) == scope) local.push_back(v);
    std::sort(local.begin(), local.end(),
              [&](uint32_t p, uint32_t q) { return name_less(meta[p].x & 0xFFFF, meta[q].x & 0xFFFF); });
    for (uint32_t v : local) {
      const uint32_t name = meta[v].x & 0xFFFF;
      if (std::find(taken.begin(), taken.end(), name) != taken.end()) continue;
      if (!requested.empty() && std::find(requested.begin(), requested.end(), name) == requested.end()) continue;
      if (j.n_variables >= 6) break;
      taken.push_back(name);
      zbhip_doc_entry& d = j.variables[j.n_variables++];
      d.name_id = name;
      d.type = (uint8_t)((meta[v].y >> 16) & 0xFF);
      d.value = val[v];
      if (d.type == kDocOutList) {  // a propagated outputCollection: the host's list
        const auto ov = h->outlist_var.find(h->key_of(j.instance, meta[v].y & 0xFFFF));
        d.type = ZBHIP_DOC_LIST;
        d.value = ov == h->outlist_var.end() ? 0 : ov->second;
      }
    }
  }
}

extern "C" int zbhip_activate_jobs(zbhip_handle* h, const zbhip_job_activation* cmd, zbhip_activated_job* jobs,
                                   size_t cap, zbhip_job_batch* res) {
  if (!h || !cmd || !res || (cap && !jobs) || (cmd->type_len && !cmd->type) || (cmd->worker_len && !cmd->worker) ||
      (cmd->n_variables && !cmd->variables))
    return ZBHIP_EINVAL;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  *res = zbhip_job_batch{};
  res->key = -1;
  res->rejection_type = ZBHIP_REJ_NONE;
  // JobBatchActivateProcessor.isValid / rejectCommand (:68-118): INVALID_ARGUMENT, no key
  const uint8_t reason = cmd->max_jobs < 1 ? 1 : cmd->timeout < 1 ? 2 : cmd->type_len == 0 ? 3 : 0;
  if (reason) {
    res->rejection_type = ZBHIP_REJ_INVALID_ARGUMENT;
    res->reason = reason;
    return ZBHIP_OK;
  }
  if (!h->job_index_on)
    if (int rc = build_job_index(h)) return rc;
  // the worker into the value dictionary: the activated jobs' records name it
  const int64_t worker_wid = cmd->worker_len ? zbhip_intern_string(h, cmd->worker, cmd->worker_len) : (int64_t)ZBHIP_NO_STRING;
  if (worker_wid < 0) return (int)worker_wid;
  const uint32_t worker_id = (uint32_t)worker_wid;
  res->key = ((int64_t)h->cfg.partition_id << 51) + ++h->key_counter;  // keyGenerator.nextKey
  if (h->st.n_slots) {
    const unsigned long long kc = (unsigned long long)h->key_counter;
    HIPCHK(hipMemcpy(h->d_key_counter, &kc, sizeof kc, hipMemcpyHostToDevice));
  }
  const std::string type(cmd->type, cmd->type_len), worker(cmd->worker ? cmd->worker : "", cmd->worker_len);
  auto tit = h->job_type_ids.find(type);
  std::vector<std::pair<int64_t, std::pair<uint32_t, uint16_t>>> pick;
  if (tit != h->job_type_ids.end()) {
    const size_t want = std::min<size_t>((size_t)cmd->max_jobs, cap);
    for (auto it = h->job_index.lower_bound({tit->second, INT64_MIN});
         it != h->job_index.end() && it->first.first == tit->second && pick.size() < want; ++it)
      pick.push_back({it->first.second, it->second});
    if (!pick.empty() && pick.size() == cap && cap < (size_t)cmd->max_jobs) {  // the caller's buffer was the limit
      const auto nx = h->job_index.upper_bound({tit->second, pick.back().first});
      res->truncated = nx != h->job_index.end() && nx->first.first == tit->second;
    }
  }
  res->n_jobs = (uint32_t)pick.size();
  if (pick.empty()) return ZBHIP_OK;
  const size_t n = pick.size(), ob = activated_out_bytes();
  std::vector<uint2> list(n);
  for (size_t i = 0; i < n; ++i) {  // (y bit 16: a timed-out job, its row keeps the stored activation)
    const auto ait = h->activated.find(pick[i].first);
    list[i] = make_uint2(pick[i].second.first, pick[i].second.second | (ait != h->activated.end() ? 1u << 16 : 0u));
  }
  uint2* d_list = nullptr;
  void* d_out = nullptr;
  std::vector<uint8_t> outb(n * ob);
  if (hipMalloc(reinterpret_cast<void**>(&d_list), n * sizeof(uint2)) != hipSuccess) return ZBHIP_ENOMEM;
  if (hipMalloc(&d_out, n * ob) != hipSuccess) {
    (void)hipFree(d_list);
    return ZBHIP_ENOMEM;
  }
  // the device's activation table (the deadline and worker of ACTIVATED jobs, for their later records)
  hipError_t e = hipSuccess;
  if (!h->st.act && !getenv("ZBHIP_NO_DEVICE_ACTIVATIONS")) {  // (off: activated jobs' windows go to the host serialiser)
    const size_t words = (size_t)kSlots * h->cfg.max_instances;
    if (dalloc(&h->st.act, words) != hipSuccess || dalloc(&h->d_cmd_act, (size_t)h->cfg.max_commands) != hipSuccess) {
      (void)hipFree(d_list);
      (void)hipFree(d_out);
      return ZBHIP_ENOMEM;
    }
    e = hipMemsetAsync(h->st.act, 0, words * sizeof(uint4), h->stream);
  }
  if (e == hipSuccess) e = hipMemcpyAsync(d_list, list.data(), n * sizeof(uint2), hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess)
    e = launch_activate_jobs(h->st, d_list, (uint32_t)n, d_out, worker_id, cmd->timestamp + cmd->timeout, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(outb.data(), d_out, n * ob, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d_list);
  (void)hipFree(d_out);
  if (e != hipSuccess) return ZBHIP_EDEVICE;
  std::vector<uint32_t> requested(cmd->variables, cmd->variables + cmd->n_variables);
  for (size_t i = 0; i < n; ++i) {
    const uint8_t* o = outb.data() + i * ob;
    uint4 a;
    uint2 meta[kVars];
    long long val[kVars];
    uint2 slots[kSlots];
    memcpy(&a, o, sizeof a);
    memcpy(meta, o + sizeof(uint4), sizeof meta);
    memcpy(val, o + sizeof(uint4) + sizeof meta, sizeof val);
    memcpy(slots, o + sizeof(uint4) + sizeof meta + sizeof val, sizeof slots);
    const uint32_t inst = pick[i].second.first;
    if (!a.w) return ZBHIP_EDEVICE;  // the index and the device rows disagree
    const uint32_t proc = a.y & 0xFFFF, elem = a.x & 0xFFFF, eord = a.x >> 16;
    zbhip_activated_job& j = jobs[i];
    j = zbhip_activated_job{};
    j.key = pick[i].first;
    j.element_instance_key = h->key_of(inst, eord);
    j.process_instance_key = h->key_of(inst, 0);
    j.deadline = cmd->timestamp + cmd->timeout;
    j.instance = inst;
    j.process_idx = (int32_t)proc;
    j.element_idx = (int32_t)elem;
    j.retries = proc < h->procs.size() && elem < h->procs[proc].els.size() ? h->procs[proc].els[elem].job_retries : 0;
    collect_job_variables(h, a, meta, val, slots, requested, j);
    // JobBatchActivatedApplier -> DbJobState.activate: ACTIVATED, out of JOB_ACTIVATABLE, deadline
    h->job_index.erase({tit->second, j.key});
    zbhip_handle::Activation& act = h->activated[j.key];  // (a failed job keeps its retries / errorMessage)
    act.deadline = j.deadline;
    act.worker = worker;
    act.inst = inst;
    act.worker_id = worker_id;
    act.state = zbhip_handle::JS_ACTIVATED;
    if (act.fail_fields) j.retries = act.retries;
    act.eik = j.element_instance_key;
    act.pik = j.process_instance_key;
    act.proc = j.process_idx;
    act.elem = j.element_idx;
  }
  return ZBHIP_OK;
}

// JOB_ACTIVATABLE of one type over the device's jobs, in key order (the host's job index)
extern "C" int zbhip_activatable_jobs(zbhip_handle* h, const char* type, size_t type_len, int64_t* keys, size_t cap,
                                      size_t* n_out) {
  if (!h || !n_out || (type_len && !type) || (cap && !keys)) return ZBHIP_EINVAL;
  *n_out = 0;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  if (!h->job_index_on)
    if (int rc = build_job_index(h)) return rc;
  const auto tit = h->job_type_ids.find(std::string(type ? type : "", type_len));
  if (tit == h->job_type_ids.end()) return ZBHIP_OK;
  size_t n = 0;
  for (auto it = h->job_index.lower_bound({tit->second, INT64_MIN});
       it != h->job_index.end() && it->first.first == tit->second && n < cap; ++it)
    keys[n++] = it->first.second;
  *n_out = n;
  return ZBHIP_OK;
}

// The push side effect's ActivatedJob (BpmnJobActivationBehavior.publishWork :83-97: JobVariablesCollector
// over the stream's fetchVariables, then jobStream.push): the stored activation of each pushed job and its
// variables, gathered in one k_activate_jobs launch in peek mode (nothing written).  A key that is not a
// live device job comes back with key -1.
extern "C" int zbhip_job_variables(zbhip_handle* h, const int64_t* job_keys, size_t n, const uint32_t* names,
                                   size_t n_names, zbhip_activated_job* out) {
  if (!h || (n && (!job_keys || !out)) || (n_names && !names)) return ZBHIP_EINVAL;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  if (!n) return ZBHIP_OK;
  std::vector<uint2> list(n);
  std::vector<uint8_t> live(n, 0);
  for (size_t i = 0; i < n; ++i) {
    uint32_t inst = 0xFFFFFFFFu;
    uint16_t ord = 0;
    if (zbhip_resolve_key(h, job_keys[i], &inst, &ord) == ZBHIP_OK && inst < h->cfg.max_instances) live[i] = 1;
    list[i] = make_uint2(live[i] ? inst : 0xFFFFFFFFu, (uint32_t)ord | 1u << 17);
  }
  const size_t ob = activated_out_bytes();
  std::vector<uint8_t> outb(n * ob);
  uint2* d_list = nullptr;
  void* d_out = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&d_list), n * sizeof(uint2)) != hipSuccess) return ZBHIP_ENOMEM;
  if (hipMalloc(&d_out, n * ob) != hipSuccess) {
    (void)hipFree(d_list);
    return ZBHIP_ENOMEM;
  }
  hipError_t e = hipMemcpyAsync(d_list, list.data(), n * sizeof(uint2), hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = launch_activate_jobs(h->st, d_list, (uint32_t)n, d_out, 0, 0, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(outb.data(), d_out, n * ob, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d_list);
  (void)hipFree(d_out);
  if (e != hipSuccess) return ZBHIP_EDEVICE;
  const std::vector<uint32_t> requested(names, names + n_names);
  for (size_t i = 0; i < n; ++i) {
    zbhip_activated_job& j = out[i];
    j = zbhip_activated_job{};
    j.key = -1;
    const uint8_t* o = outb.data() + i * ob;
    uint4 a;
    uint2 meta[kVars];
    long long val[kVars];
    uint2 slots[kSlots];
    memcpy(&a, o, sizeof a);
    memcpy(meta, o + sizeof(uint4), sizeof meta);
    memcpy(val, o + sizeof(uint4) + sizeof meta, sizeof val);
    memcpy(slots, o + sizeof(uint4) + sizeof meta + sizeof val, sizeof slots);
    if (!live[i] || !a.w) continue;
    const uint32_t inst = list[i].x, proc = a.y & 0xFFFF, elem = a.x & 0xFFFF;
    j.key = job_keys[i];
    j.element_instance_key = h->key_of(inst, a.x >> 16);
    j.process_instance_key = h->key_of(inst, 0);
    j.instance = inst;
    j.process_idx = (int32_t)proc;
    j.element_idx = (int32_t)elem;
    j.retries = proc < h->procs.size() && elem < h->procs[proc].els.size() ? h->procs[proc].els[elem].job_retries : 0;
    j.deadline = -1;
    const auto ait = h->activated.find(j.key);
    if (ait != h->activated.end()) {
      j.deadline = ait->second.deadline;
      if (ait->second.fail_fields) j.retries = (uint16_t)ait->second.retries;
    }
    collect_job_variables(h, a, meta, val, slots, requested, j);
  }
  return ZBHIP_OK;
}

extern "C" int zbhip_job_batch_rejection_reason(const zbhip_job_activation* cmd, const zbhip_job_batch* res, char* buf,
                                               size_t cap) {
  if (!cmd || !res || !buf || !cap) return ZBHIP_EINVAL;
  const char* f = "Expected to activate job batch with %s to be %s, but it was %s";  // rejectCommand (:91-118)
  char v[64];
  switch (res->reason) {
    case 1:
      snprintf(v, sizeof v, "'%d'", cmd->max_jobs);
      snprintf(buf, cap, f, "max jobs to activate", "greater than zero", v);
      break;
    case 2:
      snprintf(v, sizeof v, "'%lld'", (long long)cmd->timeout);
      snprintf(buf, cap, f, "timeout", "greater than zero", v);
      break;
    case 3: snprintf(buf, cap, f, "type", "present", "blank"); break;
    default: buf[0] = 0;
  }
  return ZBHIP_OK;
}

// ---- the engine's scheduled tasks over device-held state -------------------------------------------
// The reference's scheduled checkers read RocksDB; the device's timers and activated jobs live in HBM
// and in the handle.  These calls are what a host adapter's checkers read instead.

// a TIMER:TRIGGER command of a due device timer, as WriteTriggerTimerCommandVisitor writes it
// (DueDateTimerChecker.java:115-129): key = the timer, the TimerRecord of the TimerInstance
static void timer_trigger_record(zbhip_handle* h, const DueTimer& d, zbhip_record& r) {
  r = zbhip_record{};
  r.record_type = ZBHIP_RT_COMMAND;
  r.value_type = ZBHIP_VT_TIMER;
  r.intent = ZBHIP_TIMER_TRIGGER;
  r.rejection_type = ZBHIP_REJ_NONE;
  r.key = h->key_of(d.inst, d.tmr.x >> 16);
  r.scope_key = h->key_of(d.inst, d.tmr.y & 0xFFFF);
  r.process_instance_key = h->key_of(d.inst, 0);
  r.process_idx = (int32_t)d.proc;
  r.element_idx = (int32_t)(d.tmr.x & 0xFFF);  // the handler node (catch / boundary event)
  r.aux = (int64_t)(((unsigned long long)d.tmr.w << 32) | d.tmr.z);  // dueDate
  const uint32_t reps = (d.tmr.y >> 16) & 0xFF;
  r.partition = reps == 255 ? -1 : (int32_t)reps;
  r.source_index = -1;
  r.message_key = -1;
  r.correlation_key = ZBHIP_NO_STRING;
  r.message_name = r.bpmn_process_id = 0xFFFF;
}

extern "C" int zbhip_due_timers(zbhip_handle* h, int64_t now, zbhip_record* out, size_t cap, size_t* n_out, int64_t* next_due) {
  if (!h || !n_out || (cap && !out)) return ZBHIP_EINVAL;
  *n_out = 0;
  if (next_due) *next_due = -1;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  const uint32_t N = h->cfg.max_instances;
  if (!h->d_due) {
    if (dalloc(&h->d_due, N) != hipSuccess || dalloc(&h->d_due_count, 1) != hipSuccess ||
        dalloc(&h->d_due_next, 1) != hipSuccess)
      return ZBHIP_ENOMEM;
  }
  const unsigned long long none = ~0ull;
  HIPCHK(hipMemsetAsync(h->d_due_count, 0, sizeof(uint32_t), h->stream));
  HIPCHK(hipMemcpyAsync(h->d_due_next, &none, sizeof none, hipMemcpyHostToDevice, h->stream));
  HIPCHK(launch_due_timers(h->st, (long long)now, h->d_due, h->d_due_count, h->d_due_next, h->stream));
  uint32_t count = 0;
  unsigned long long later = none;
  HIPCHK(hipMemcpyAsync(&count, h->d_due_count, sizeof count, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(&later, h->d_due_next, sizeof later, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  std::vector<DueTimer> due(count);
  if (count) HIPCHK(hipMemcpy(due.data(), h->d_due, count * sizeof(DueTimer), hipMemcpyDeviceToHost));
  // TIMER_DUE_DATES order: [dueDate, [elementInstanceKey, timerKey]] (DbTimerInstanceState :52-56)
  std::vector<zbhip_record> recs(count);
  for (uint32_t i = 0; i < count; ++i) timer_trigger_record(h, due[i], recs[i]);
  std::sort(recs.begin(), recs.end(), [](const zbhip_record& a, const zbhip_record& b) {
    return std::tie(a.aux, a.scope_key, a.key) < std::tie(b.aux, b.scope_key, b.key);
  });
  const size_t n = std::min<size_t>(cap, count);
  for (size_t i = 0; i < n; ++i) out[i] = recs[i];
  *n_out = n;
  // processTimersWithDueDateBefore's result: the first dueDate it did not consume
  if (next_due) *next_due = n < count ? recs[n].aux : later != none ? (int64_t)later : -1;
  return ZBHIP_OK;
}

// a JOB record of a device job with a stored activation: the stored JobRecord (type, retries,
// element and keys from the deployment and the handle, deadline and worker as DbJobState stored them)
static void stored_job_record(const zbhip_handle::Activation& a, int64_t key, uint8_t rt, uint8_t intent,
                              zbhip_record& r) {
  r = zbhip_record{};
  r.key = key;
  r.record_type = rt;
  r.value_type = ZBHIP_VT_JOB;
  r.intent = intent;
  r.rejection_type = ZBHIP_REJ_NONE;
  r.scope_key = a.eik;
  r.process_instance_key = a.pik;
  r.process_idx = a.proc;
  r.element_idx = a.elem;
  r.source_index = -1;
  r.aux = -1;
  r.message_key = a.deadline;
  r.correlation_key = a.worker_id;
  r.message_name = r.bpmn_process_id = 0xFFFF;
  if (a.fail_fields) {  // a failed job's retries and errorMessage (zbhip_record, JOB records)
    r.reason_arg = 1;
    r.partition = a.retries;
    r.message_name = (uint16_t)(a.error_id & 0xFFFF);
    r.bpmn_process_id = (uint16_t)(a.error_id >> 16);
  }
}

extern "C" int zbhip_timed_out_jobs(zbhip_handle* h, int64_t now, zbhip_record* out, size_t cap, size_t* n_out,
                                    int64_t* next_deadline) {
  if (!h || !n_out || (cap && !out)) return ZBHIP_EINVAL;
  *n_out = 0;
  if (next_deadline) *next_deadline = -1;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  // DbJobState.forEachTimedOutEntry (:286-298): JOB_DEADLINES [deadline, jobKey] while deadline < now
  std::vector<std::pair<int64_t, int64_t>> due;
  for (const auto& [k, a] : h->activated)
    if (a.state == zbhip_handle::JS_ACTIVATED && a.deadline < now) due.push_back({a.deadline, k});
  std::sort(due.begin(), due.end());
  const size_t n = std::min(cap, due.size());
  for (size_t i = 0; i < n; ++i)
    stored_job_record(h->activated.at(due[i].second), due[i].second, ZBHIP_RT_COMMAND, ZBHIP_JOB_TIME_OUT, out[i]);
  *n_out = n;
  // the first timed-out deadline not returned (a merge with the engine's JOB_DEADLINES stops before it)
  if (next_deadline && n < due.size()) *next_deadline = due[n].first;
  return ZBHIP_OK;
}

// BpmnJobActivationBehavior.publishWork of a job the host side made ACTIVATABLE (a time-out, a failure
// with retries left): with a job stream for its type, JOB_BATCH:ACTIVATED (key = nextKey) of the job,
// ACTIVATED again with the stream's deadline and worker.  Returns the records written (0 or 1).
static size_t push_job(zbhip_handle* h, int64_t job_key, int64_t now, zbhip_record* out) {
  auto it = h->activated.find(job_key);
  if (it == h->activated.end() || it->second.proc < 0 || (size_t)it->second.proc >= h->procs.size()) return 0;
  zbhip_handle::Activation& a = it->second;
  const Proc& P = h->procs[a.proc];
  if (a.elem < 0 || (size_t)a.elem >= P.els.size()) return 0;
  const uint32_t tid = P.job_type_id[a.elem];
  const auto st = h->streams.find(tid);
  if (st == h->streams.end()) return 0;
  a.deadline = now + st->second.timeout;
  a.worker = st->second.worker;
  a.worker_id = st->second.worker_id;
  a.state = zbhip_handle::JS_ACTIVATED;
  if (h->job_index_on) h->job_index.erase({tid, job_key});
  const int64_t key = ((int64_t)h->cfg.partition_id << 51) + ++h->key_counter;
  if (h->st.n_slots) {
    const unsigned long long kc = (unsigned long long)h->key_counter;
    if (hipMemcpy(h->d_key_counter, &kc, sizeof kc, hipMemcpyHostToDevice) != hipSuccess) return 0;
  }
  stored_job_record(a, job_key, ZBHIP_RT_EVENT, ZBHIP_JOB_BATCH_ACTIVATED, *out);
  out->key = key;
  out->value_type = ZBHIP_VT_JOB_BATCH;
  out->aux = job_key;
  return 1;
}

extern "C" int zbhip_time_out_job(zbhip_handle* h, int64_t job_key, int64_t now, zbhip_record* out, size_t cap,
                                  size_t* n_out) {
  if (!h || !out || !n_out || cap < 2) return ZBHIP_EINVAL;
  *n_out = 1;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  // JobTimeOutProcessor.processRecord (:46-69): an ACTIVATED job past its deadline times out, anything
  // else is rejected NOT_FOUND with the job's state
  auto it = h->activated.find(job_key);
  uint8_t why = 0;  // reason_arg: 0 no such job, 1 not activated, 2 not timed out, 3 failed
  if (it != h->activated.end()) {
    if (it->second.state == zbhip_handle::JS_ACTIVATED) {
      if (it->second.deadline < now) {
        zbhip_handle::Activation& a = it->second;
        stored_job_record(a, job_key, ZBHIP_RT_EVENT, ZBHIP_JOB_TIMED_OUT, *out);
        // JobTimedOutApplier -> DbJobState.timeout: ACTIVATABLE again, the record kept, no deadline row
        a.state = zbhip_handle::JS_ACTIVATABLE;
        uint32_t inst;
        uint16_t ord;
        if (h->job_index_on && a.proc >= 0 && (size_t)a.proc < h->procs.size() && a.elem >= 0 &&
            (size_t)a.elem < h->procs[a.proc].els.size() && zbhip_resolve_key(h, job_key, &inst, &ord) == ZBHIP_OK)
          h->job_index[{h->procs[a.proc].job_type_id[a.elem], job_key}] = {inst, ord};
        *n_out += push_job(h, job_key, now, out + 1);  // publishWork (JobTimeOutProcessor.java:55)
        return ZBHIP_OK;
      }
      why = 2;
    } else {
      why = it->second.state == zbhip_handle::JS_GONE ? 0 : it->second.state == zbhip_handle::JS_FAILED ? 3 : 1;
    }
  } else {
    // no stored activation: an ACTIVATABLE job of a live instance, or none at all
    uint32_t inst;
    uint16_t ord;
    if (zbhip_resolve_key(h, job_key, &inst, &ord) == ZBHIP_OK && inst < h->cfg.max_instances) {
      InstRows R{};
      if (int rc = gather_instance(h, inst, R)) return rc;
      const uint32_t nslots = (R.hdr.y >> 8) & 0xFF;
      for (uint32_t s = 0; s < nslots && s < (uint32_t)kSlots; ++s)
        if ((R.slots[s].y & 0xFFFF) == ord && ((R.slots[s].y >> 24) & 1u) && ((R.hdr.y >> 24) & 1u)) why = 1;
    }
  }
  *out = zbhip_record{};
  out->key = job_key;
  out->record_type = ZBHIP_RT_REJECTION;
  out->value_type = ZBHIP_VT_JOB;
  out->intent = ZBHIP_JOB_TIME_OUT;
  out->rejection_type = ZBHIP_REJ_NOT_FOUND;
  out->reason = ZBHIP_REASON_JOB_TIME_OUT;
  out->reason_arg = why;
  out->scope_key = out->process_instance_key = out->aux = out->message_key = out->source_index = -1;
  out->process_idx = out->element_idx = -1;
  out->correlation_key = ZBHIP_NO_STRING;
  out->message_name = out->bpmn_process_id = 0xFFFF;
  return ZBHIP_OK;
}

// StringUtil.limitString(message, maxLength) (util/.../StringUtil.java:50-56) on the UTF-8 bytes of a Java
// String: the length counts UTF-16 code units (a character beyond the BMP is two); a cut inside a
// surrogate pair keeps the lone high surrogate, which String.getBytes(UTF_8) writes as '?'
static std::string limit_java_string(const std::string& s, size_t max_units) {
  size_t units = 0, i = 0;
  while (i < s.size()) {
    const unsigned char c = (unsigned char)s[i];
    const size_t len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : 4;
    const size_t u = len == 4 ? 2 : 1;
    if (units + u > max_units) return s.substr(0, i) + (units < max_units ? "?" : "") + "...";
    units += u;
    i += len;
  }
  return s;
}

extern "C" int zbhip_fail_job(zbhip_handle* h, const zbhip_job_fail* cmd, zbhip_record* out, size_t cap, size_t* n_out) {
  if (!h || !cmd || !n_out || (cap && !out) || (cmd->error_message_len && !cmd->error_message)) return ZBHIP_EINVAL;
  *n_out = 0;
  if (cap < 2) return ZBHIP_ENOMEM;
  if (!h->relabel_ok) return ZBHIP_ESTATE;
  if (int rc = finalize(h)) return rc;
  const int64_t job_key = cmd->job_key;
  auto reject = [&](uint8_t type, uint8_t state) {  // JobCommandPreconditionChecker.check (:33-49)
    zbhip_record& r = out[0];
    r = zbhip_record{};
    r.key = job_key;
    r.record_type = ZBHIP_RT_REJECTION;
    r.value_type = ZBHIP_VT_JOB;
    r.intent = ZBHIP_JOB_FAIL;
    r.rejection_type = type;
    r.reason = ZBHIP_REASON_JOB_STATE;
    r.reason_arg = state;
    r.scope_key = r.process_instance_key = r.aux = r.message_key = r.source_index = -1;
    r.process_idx = r.element_idx = -1;
    r.correlation_key = ZBHIP_NO_STRING;
    r.message_name = r.bpmn_process_id = 0xFFFF;
    *n_out = 1;
    return ZBHIP_OK;
  };
  auto it = h->activated.find(job_key);
  if (it != h->activated.end() && it->second.state == zbhip_handle::JS_GONE) return reject(ZBHIP_REJ_NOT_FOUND, 3);
  if (it != h->activated.end() && it->second.state == zbhip_handle::JS_FAILED) return reject(ZBHIP_REJ_INVALID_STATE, 2);
  // the job row on the device (ACTIVATABLE, or ACTIVATED with a stored activation)
  uint32_t inst;
  uint16_t ord;
  if (zbhip_resolve_key(h, job_key, &inst, &ord) != ZBHIP_OK || inst >= h->cfg.max_instances)
    return reject(ZBHIP_REJ_NOT_FOUND, 3);
  InstRows R{};
  if (int rc = gather_instance(h, inst, R)) return rc;
  const uint32_t nslots = (R.hdr.y >> 8) & 0xFF, proc = R.hdr.x & 0xFFFF;
  int slot = -1;
  for (uint32_t s = 0; s < nslots && s < (uint32_t)kSlots; ++s)
    if ((R.slots[s].y & 0xFFFF) == ord && ((R.slots[s].y >> 24) & 1u)) slot = (int)s;
  if (slot < 0 || !((R.hdr.y >> 24) & 1u) || proc >= h->procs.size()) return reject(ZBHIP_REJ_NOT_FOUND, 3);
  // the device subset: no variables (setFailedVariables), no retry back-off (JobBackoffChecker)
  if (cmd->n_variables || (cmd->retries > 0 && cmd->retry_backoff > 0)) return ZBHIP_EUNSUPP;
  std::string msg(cmd->error_message ? cmd->error_message : "", cmd->error_message_len);
  msg = limit_java_string(msg, 10000);
  const int64_t eid = msg.empty() ? (int64_t)ZBHIP_NO_STRING : zbhip_intern_string(h, msg.data(), msg.size());
  if (eid < 0) return (int)eid;
  const uint32_t elem = R.slots[slot].x & 0xFFFF;
  const Proc& P = h->procs[proc];
  if (elem >= P.els.size()) return ZBHIP_EDEVICE;
  const bool had = it != h->activated.end();
  zbhip_handle::Activation& a = h->activated[job_key];
  if (!had) {  // the first stored field of this job: the slot's flag bit 1 makes its later records read them
    a.deadline = -1;
    a.inst = inst;
    a.worker_id = ZBHIP_NO_STRING;
    a.eik = h->key_of(inst, R.slots[slot].x >> 16);
    a.pik = h->key_of(inst, 0);
    a.proc = (int32_t)proc;
    a.elem = (int32_t)elem;
    uint2 w = R.slots[slot];
    w.y |= 2u << 24;
    HIPCHK(hipMemcpy(h->st.slots + (size_t)slot * h->st.n + inst, &w, sizeof w, hipMemcpyHostToDevice));
  }
  a.fail_fields = true;
  a.retries = cmd->retries;
  a.error_id = (uint32_t)eid;
  h->ring_ok = false;  // the device log writer does not write failed jobs' fields: the host serialiser does
  // JOB:FAILED: the stored job with the command's retries / errorMessage (retryBackoff 0, no variables)
  stored_job_record(a, job_key, ZBHIP_RT_EVENT, ZBHIP_JOB_FAILED, out[0]);
  *n_out = 1;
  // JobFailedApplier -> DbJobState.fail (:191-203): ACTIVATABLE again with retries left, else FAILED
  const uint32_t tid = P.job_type_id[elem];
  if (cmd->retries > 0) {
    a.state = zbhip_handle::JS_ACTIVATABLE;
    if (h->job_index_on) h->job_index[{tid, job_key}] = {inst, ord};
    *n_out += push_job(h, job_key, cmd->timestamp, out + 1);  // retryImmediately: publishWork (:129-132)
    return ZBHIP_OK;
  }
  a.state = zbhip_handle::JS_FAILED;
  if (h->job_index_on) h->job_index.erase({tid, job_key});
  // raiseIncident (:139-162): INCIDENT:CREATED, key = keyGenerator.nextKey (no instance's ordinal)
  const std::string text = msg.empty() ? std::string("No more retries left.") : msg;
  const int64_t tid_msg = zbhip_intern_string(h, text.data(), text.size());
  if (tid_msg < 0) return (int)tid_msg;
  a.incident_key = ((int64_t)h->cfg.partition_id << 51) + ++h->key_counter;
  a.incident_msg_id = (uint32_t)tid_msg;
  if (h->st.n_slots) {
    const unsigned long long kc = (unsigned long long)h->key_counter;
    HIPCHK(hipMemcpy(h->d_key_counter, &kc, sizeof kc, hipMemcpyHostToDevice));
  }
  zbhip_record& r = out[1];
  r = zbhip_record{};
  r.key = a.incident_key;
  r.record_type = ZBHIP_RT_EVENT;
  r.value_type = ZBHIP_VT_INCIDENT;
  r.intent = ZBHIP_INCIDENT_CREATED;
  r.rejection_type = ZBHIP_REJ_NONE;
  r.scope_key = a.eik;
  r.process_instance_key = a.pik;
  r.process_idx = a.proc;
  r.element_idx = a.elem;
  r.partition = ZBHIP_ERR_JOB_NO_RETRIES;
  r.aux = job_key;
  r.correlation_key = a.incident_msg_id;
  r.source_index = r.message_key = -1;
  r.message_name = r.bpmn_process_id = 0xFFFF;
  *n_out = 2;
  return ZBHIP_OK;
}

extern "C" int zbhip_set_job_stream(zbhip_handle* h, const char* type, size_t type_len, const char* worker,
                                    size_t worker_len, int64_t timeout, int on) {
  if (!h || !type || !type_len || (worker_len && !worker) || (on && timeout < 1)) return ZBHIP_EINVAL;
  const uint32_t tid = h->job_type(std::string(type, type_len));
  if (on) {
    const std::string w(worker ? worker : "", worker_len);
    const int64_t wid = w.empty() ? (int64_t)ZBHIP_NO_STRING : zbhip_intern_string(h, w.data(), w.size());
    if (wid < 0) return (int)wid;
    const auto old = h->streams.find(tid);
    const bool same = old != h->streams.end();
    h->streams[tid] = {w, (uint32_t)wid, timeout};
    if (same) return ZBHIP_OK;  // (the program words only say whether a stream exists)
  } else if (!h->streams.erase(tid)) {
    return ZBHIP_OK;
  }
  h->ring_ok = false;  // the device log writer does not write pushes: the host serialiser does
  return rebuild_program(h);
}

extern "C" int zbhip_job_state(zbhip_handle* h, int64_t job_key) {
  if (!h) return ZBHIP_EINVAL;
  auto it = h->activated.find(job_key);
  if (it == h->activated.end()) return -1;  // none stored: ACTIVATABLE if the key is a live job's
  switch (it->second.state) {
    case zbhip_handle::JS_ACTIVATED: return 1;
    case zbhip_handle::JS_ACTIVATABLE: return 0;
    case zbhip_handle::JS_FAILED: return 2;
    default: return 3;
  }
}

// ---- log bytes on the device (logdev.hip) ----------------------------------------------------------
// After zbhip_run with results: every record of the window serialised in HBM, in drain order, the
// same bytes zbhip_serialize_log writes for the drained records.  The window's keys then go into
// the device key ring, which is why every window has to come through here for the path to stay on:
// a window that did not (or imported state, message partitions, continuation batches, string
// variables, a key older than the ring) makes this return ZBHIP_EUNSUPP -- the host serialiser
// (zbhip_drain + zbhip_serialize_log) is then the path for that window and the ones after it.
extern "C" int zbhip_serialize_log_device(zbhip_handle* h, const zbhip_log_window* w, const void** dev_bytes,
                                          size_t* used) {
  if (!h || !w || !dev_bytes || !used) return ZBHIP_EINVAL;
  *dev_bytes = nullptr;
  *used = 0;
  if (!h->results) return ZBHIP_ESTATE;
  const bool fill = h->ring_filled + 1 == h->windows_run;  // every earlier window's keys are in the ring
  if (!fill) h->ring_ok = false;
  h->ring_filled = h->windows_run;  // this window is accounted for, whether or not it is written here
  if (h->msg() || !h->cont_cmds.empty() || h->window_continues) h->ring_ok = false;
  if (w->timer_values) {  // rejected TIMER:TRIGGERs carry the commands' TimerRecords: the host writes them
    bool trig = h->h_cmds.size() < h->n_cmds;
    for (size_t c = 0; c < h->n_cmds && !trig; ++c) trig = h->h_cmds[c].kind == ZBHIP_CMD_TIMER_TRIGGER;
    if (trig) h->ring_ok = false;
  }
  if (!h->ring_ok) return ZBHIP_EUNSUPP;
  const bool dbg = getenv("ZBHIP_DEBUG") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  const auto t0 = now();
  const size_t n = h->n_cmds;
  const size_t N = h->cfg.max_instances;
  if (w->n_cmds != n) return ZBHIP_EINVAL;
  // The command table on the device (logdev.hip k_table_build) when the window is one round of
  // device-processed commands gathered in log order and its key bookkeeping has not started: the
  // host's key relabelling bookkeeping (finalize) then runs while the device builds the table and
  // sizes the entries.  Otherwise the host builds the table after finalize.
  bool dev_table = n > 0 && h->round_begin.empty() && h->fin_next == 0 && h->launches.size() == 1 &&
                   h->launches[0].src == 0 && h->launches[0].count == n && !getenv("ZBHIP_HOST_LOG_TABLE");
  if (dev_table) dev_table = h->window_fallbacks == 0;  // (every command of the window ran on the device)
  const unsigned long long key_base = (unsigned long long)h->key_counter;  // (fin_next == 0: the window's base)
  if (!dev_table)
    if (int rc = finalize(h)) return rc;
  const auto t1 = now();
  // tables of the serialiser (deployments / names changed since the last upload)
  if (h->log_tables_procs != h->procs.size() || h->log_tables_names != h->names.size()) {
    std::vector<uint8_t> arena;
    std::vector<uint32_t> idx;
    if (int rc = log_device_tables(h->ser, arena, idx)) return rc;
    if (arena.size() > h->log_arena_cap) {
      (void)hipFree(h->d_log_arena);
      h->d_log_arena = nullptr;
      if (dalloc(&h->d_log_arena, arena.size() * 2) != hipSuccess) return ZBHIP_ENOMEM;
      h->log_arena_cap = arena.size() * 2;
    }
    if (idx.size() > h->log_idx_cap) {
      (void)hipFree(h->d_log_idx);
      h->d_log_idx = nullptr;
      if (dalloc(&h->d_log_idx, idx.size() * 2) != hipSuccess) return ZBHIP_ENOMEM;
      h->log_idx_cap = idx.size() * 2;
    }
    HIPCHK(hipMemcpyAsync(h->d_log_arena, arena.data(), arena.size(), hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->d_log_idx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, h->stream));
    std::vector<uint8_t> tpl;
    std::vector<uint32_t> desc, tidx;
    if (int rc = log_device_templates(h->ser, tpl, desc, tidx)) return rc;
    const size_t desc_off = (tpl.size() + 15) & ~(size_t)15, idx_off = desc_off + desc.size() * 4;
    const size_t tpl_bytes = idx_off + tidx.size() * 4;
    if (tpl_bytes > h->log_tpl_cap) {
      (void)hipFree(h->d_log_tpl);
      h->d_log_tpl = nullptr;
      if (dalloc(&h->d_log_tpl, tpl_bytes * 2) != hipSuccess) return ZBHIP_ENOMEM;
      h->log_tpl_cap = tpl_bytes * 2;
    }
    tpl.resize(tpl_bytes, 0);
    memcpy(tpl.data() + desc_off, desc.data(), desc.size() * 4);
    memcpy(tpl.data() + idx_off, tidx.data(), tidx.size() * 4);
    HIPCHK(hipMemcpyAsync(h->d_log_tpl, tpl.data(), tpl_bytes, hipMemcpyHostToDevice, h->stream));
    h->log_tpl_desc_off = desc_off;
    h->log_tpl_idx_off = idx_off;
    HIPCHK(hipStreamSynchronize(h->stream));
    h->log_tables_procs = h->procs.size();
    h->log_tables_names = h->names.size();
    h->log_arena_words = (uint32_t)(arena.size() / 4);
    h->log_idx_words = (uint32_t)idx.size();
  }
  if (!h->d_ring) {
    const size_t words = (size_t)16 * N + N;  // logdev.hip kRing = 16
    if (dalloc(&h->d_ring, words) != hipSuccess || dalloc(&h->d_inst_proc, N) != hipSuccess ||
        dalloc(&h->d_logcmd, (size_t)h->cfg.max_commands) != hipSuccess ||
        dalloc(&h->d_log_bytes, (size_t)h->cfg.max_commands + 1 + ((size_t)h->cfg.max_commands + 1023) / 1024 + 1) != hipSuccess ||
        dalloc(&h->d_log_flag, 1) != hipSuccess || dalloc(&h->d_src_pos, (size_t)h->cfg.max_commands) != hipSuccess ||
        dalloc(&h->d_tbl_sums, ((size_t)h->cfg.max_commands + 1023) / 1024 + 2) != hipSuccess ||
        dalloc(&h->d_log_rinfo, ((size_t)h->cfg.max_commands + 64) * h->rec_cap) != hipSuccess ||
        dalloc(&h->d_log_wkeys, (size_t)h->cfg.max_commands) != hipSuccess)
      return ZBHIP_ENOMEM;
    HIPCHK(hipMemsetAsync(h->d_ring, 0, words * sizeof(unsigned long long), h->stream));
  }
  LogLaunch a{};
  a.rows = h->d_rec;
  a.cmds = h->d_logcmd;
  a.n = (uint32_t)n;
  a.arena = h->d_log_arena;
  a.idx = h->d_log_idx;
  a.arena_words = h->log_arena_words;
  a.idx_words = h->log_idx_words;
  a.tpl = h->d_log_tpl;
  a.tpl_desc = reinterpret_cast<const uint4*>(h->d_log_tpl + h->log_tpl_desc_off);
  a.tpl_idx = reinterpret_cast<const uint32_t*>(h->d_log_tpl + h->log_tpl_idx_off);
  a.docs = h->external ? h->ext_docs : h->d_docs;
  a.n_docs = (uint32_t)h->n_docs;
  a.inst_proc = h->d_inst_proc;
  a.ring = h->d_ring;
  a.kpi = h->d_ring + (size_t)16 * N;
  a.n_inst = (uint32_t)N;
  a.pbits = (long long)h->cfg.partition_id << 51;
  a.first_position = w->first_position;
  a.timestamp = w->timestamp;
  serializer_broker(h->ser, a.broker);
  a.bytes = h->d_log_bytes;
  a.block_sums = h->d_log_bytes + n + 1;
  a.flag = h->d_log_flag;
  a.now_ms = h->run_clock_ms;
  a.cmd_due = h->d_cmd_due;
  a.rinfo = h->d_log_rinfo;
  a.wkeys = h->d_log_wkeys;
  a.tpl_lds = (uint32_t)h->log_tpl_idx_off;
  if (h->st.act) {  // activated jobs' records name their workers: the dictionary's bytes on the device
    if (h->d_strs_n != h->strs.size()) {
      std::vector<unsigned long long> off(h->strs.size() + 1, 0);
      for (size_t i = 0; i < h->strs.size(); ++i) off[i + 1] = off[i] + h->strs[i].size();
      if (off.back() > h->d_strs_cap) {
        (void)hipFree(h->d_strs);
        h->d_strs = nullptr;
        h->d_strs_cap = 0;
        if (dalloc(&h->d_strs, (size_t)off.back() * 2 + 64) != hipSuccess) return ZBHIP_ENOMEM;
        h->d_strs_cap = (size_t)off.back() * 2 + 64;
      }
      if (off.size() > h->d_str_off_cap) {
        (void)hipFree(h->d_str_off);
        h->d_str_off = nullptr;
        h->d_str_off_cap = 0;
        if (dalloc(&h->d_str_off, off.size() * 2) != hipSuccess) return ZBHIP_ENOMEM;
        h->d_str_off_cap = off.size() * 2;
      }
      std::string bytes;
      bytes.reserve((size_t)off.back());
      for (const std::string& x : h->strs) bytes += x;
      if (!bytes.empty()) HIPCHK(hipMemcpy(h->d_strs, bytes.data(), bytes.size(), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(h->d_str_off, off.data(), off.size() * sizeof(unsigned long long), hipMemcpyHostToDevice));
      h->d_strs_n = h->strs.size();
    }
    a.cmd_act = h->d_cmd_act;
    a.strs = h->d_strs;
    a.str_off = h->d_str_off;
    a.n_strs = (uint32_t)h->d_strs_n;
  }
  unsigned long long total = 0;
  uint32_t flag = 0;
  auto tu = now(), tf = now();
  bool spec = false;  // k_log_write launched before the total was known
  // the window's key bookkeeping journaled on the device (fold_journal) instead of booked here
  // (ZBHIP_NO_JOURNAL=1: booked on the host after every window, as before round 4)
  bool journal = dev_table && !h->job_index_on && !h->msg() && !getenv("ZBHIP_NO_JOURNAL");
  uint32_t jslot = 0;
  if (journal && !h->d_jrn) {
    const char* e = getenv("ZBHIP_JOURNAL_WINDOWS");
    const size_t per = (size_t)h->cfg.max_commands * sizeof(uint4);
    size_t slots = e ? (size_t)atoi(e) : 64;
    slots = std::min<size_t>(slots, std::max<size_t>(1, ((size_t)2 << 30) / std::max<size_t>(per, 1)));
    if (slots && dalloc(&h->d_jrn, slots * h->cfg.max_commands) == hipSuccess) h->jrn_slots = (uint32_t)slots;
  }
  if (journal && !h->jrn_slots) journal = false;
  if (journal) {
    if (h->jrn_q.size() >= h->jrn_slots)  // full: the oldest window into the host tables
      if (int rc = fold_journals(h, h->jrn_slots - 1)) return rc;
    jslot = h->jrn_next;
    h->jrn_next = (h->jrn_next + 1) % h->jrn_slots;
  }
  unsigned long long tbl_total = 0;  // the device table's scan total: records | keys << 32
  if (dev_table) {
    // the instances' processes before this window (the table kernel adds this window's CREATEs),
    // from the host tables -- unless windows are journaled: then the device's copy is the current one
    // (a copy, since finalize updates inst_proc while the upload may still read it, through pinned
    // staging filled on the host threads: a pageable upload is copied by the driver through its own
    // bounce buffers, synchronously and with stalls of tens of ms per window)
    if (h->jrn_q.empty() && h->inst_proc.size() >= N) {
      if (h->inst_proc_pin_cap < N) {
        if (h->inst_proc_pin) (void)hipHostFree(h->inst_proc_pin);
        h->inst_proc_pin = nullptr;
        h->inst_proc_pin_cap = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&h->inst_proc_pin), N * sizeof(uint16_t), hipHostMallocDefault) != hipSuccess)
          return ZBHIP_ENOMEM;
        h->inst_proc_pin_cap = N;
      }
      memcpy(h->inst_proc_pin, h->inst_proc.data(), N * sizeof(uint16_t));
      HIPCHK(hipMemcpyAsync(h->d_inst_proc, h->inst_proc_pin, N * sizeof(uint16_t), hipMemcpyHostToDevice, h->stream));
    }
    if (w->source_positions) {
      if (h->src_pos_pin_cap < n) {
        if (h->src_pos_pin) (void)hipHostFree(h->src_pos_pin);
        h->src_pos_pin = nullptr;
        h->src_pos_pin_cap = 0;
        const size_t cap = std::max<size_t>(n, h->cfg.max_commands);
        if (hipHostMalloc(reinterpret_cast<void**>(&h->src_pos_pin), cap * sizeof(long long), hipHostMallocDefault) != hipSuccess)
          return ZBHIP_ENOMEM;
        h->src_pos_pin_cap = cap;
      }
      parallel_for(host_threads(), [&](unsigned t, unsigned TT) {
        const size_t b = n * t / TT, e = n * (t + 1) / TT;
        memcpy(h->src_pos_pin + b, w->source_positions + b, (e - b) * sizeof(long long));
      });
      HIPCHK(hipMemcpyAsync(h->d_src_pos, h->src_pos_pin, n * sizeof(long long), hipMemcpyHostToDevice, h->stream));
    }
    tu = now();
    if (int rc = log_next_buffer(h)) return rc;
    HIPCHK(hipMemsetAsync(h->d_log_flag, 0, sizeof(uint32_t), h->stream));
    a.hdr = h->d_cmd_hdr;
    a.wcmds = reinterpret_cast<const zbhip_command*>(h->external ? h->ext_cmds : h->d_cmds);
    a.src_pos = w->source_positions ? h->d_src_pos : nullptr;
    a.key_base = key_base;
    a.table = h->d_logcmd;
    a.table_sums = h->d_tbl_sums;
    a.inst_proc_w = h->d_inst_proc;
    a.jrn = journal ? h->d_jrn + (size_t)jslot * h->cfg.max_commands : nullptr;
    a.phase = 3;
    HIPCHK(launch_log_device(a, h->stream));
    a.jrn = nullptr;
    const size_t nb = (n + 1023) / 1024;  // (logdev.hip kLogScanB)
    HIPCHK(hipMemcpyAsync(&tbl_total, h->d_tbl_sums + nb, sizeof tbl_total, hipMemcpyDeviceToHost, h->stream));
    a.phase = 0;
    HIPCHK(launch_log_device(a, h->stream));
    HIPCHK(hipMemcpyAsync(&total, h->d_log_bytes + n, sizeof total, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(&flag, h->d_log_flag, sizeof flag, hipMemcpyDeviceToHost, h->stream));
    // the templated entries written right away, under the host bookkeeping below: the device table
    // needs nothing from it (k_log_write returns at once when the window outgrew the buffer; a
    // window the device cannot write is discarded after the size pass's flag is read)
    if (h->log_out_cap) {
      a.out = h->d_log_out;
      a.out_cap = h->log_out_cap;
      a.compose = 0;
      a.phase = 1;
      HIPCHK(launch_log_device(a, h->stream));
      spec = true;
    }
    if (journal) {
      tf = now();
      HIPCHK(hipStreamSynchronize(h->stream));
      h->key_counter = (int64_t)key_base + (int64_t)(tbl_total >> 32);
      h->fin_next = n;
      h->jrn_q.push_back({jslot, n, h->windows_run});
    } else {
      // meanwhile on the host: the window's key relabelling bookkeeping (the same key bases)
      if (int rc = finalize(h)) {
        (void)hipStreamSynchronize(h->stream);
        return rc;
      }
      if (h->h_base[0] + 1 != (int64_t)key_base + 1 || h->key_counter < (int64_t)key_base) return ZBHIP_EDEVICE;
      tf = now();
      HIPCHK(hipStreamSynchronize(h->stream));
      if (h->key_counter != (int64_t)key_base + (int64_t)(tbl_total >> 32)) return ZBHIP_EDEVICE;
    }
  }
  const auto t2 = now();
  // the window's command table: rows, record positions, key bases, the prev chain per instance
  // (a window of one round has one command per instance: no chain, and it is filled on host threads)
  if (!dev_table) {
  if (int rc = compute_offsets(h)) return rc;
  h->h_logcmd.resize(n);
  if (h->log_prev.size() < N) h->log_prev.assign(N, ~0ull);
  const uint64_t win = h->windows_run;
  const bool one_round = h->round_begin.empty();
  auto fill_cmd = [&](size_t c, uint64_t out_rec) {
    const uint2 hd = h->h_hdr[c];
    const zbhip_command& cm = h->h_cmds[c];
    const bool ok = ((hd.y >> 16) & 0xFF) == ST_OK;
    LogCmd& m = h->h_logcmd[c];
    m.rec_off = h->h_off[c];
    m.out_rec = out_rec;
    m.key0 = (unsigned long long)(h->h_base[c] + 1);
    m.src_pos = w->source_positions ? w->source_positions[c] : -1;
    m.instance = cm.instance;
    m.first_ord = (uint16_t)(hd.y & 0xFFFF);
    m.nkeys = ok ? (uint16_t)(hd.x >> 16) : 0;
    m.nrec = (uint16_t)(hd.x & 0xFFFF);
    m.doc_count = cm.doc_count;
    m.doc_begin = cm.doc_begin;
    m.pad = cm.pad;
    m.prev = ~0u;
    return (uint64_t)m.nrec;
  };
  if (one_round) {
    const unsigned T = host_threads();
    std::vector<uint64_t> part(T + 1, 0);
    parallel_for(T, [&](unsigned t, unsigned TT) {  // records per thread range, then each range from its base
      uint64_t s = 0;
      for (size_t c = n * t / TT; c < n * (t + 1) / TT; ++c) s += h->h_hdr[c].x & 0xFFFF;
      part[t + 1] = s;
    });
    for (unsigned t = 0; t < T; ++t) part[t + 1] += part[t];
    parallel_for(T, [&](unsigned t, unsigned TT) {
      uint64_t out_rec = part[t];
      for (size_t c = n * t / TT; c < n * (t + 1) / TT; ++c) out_rec += fill_cmd(c, out_rec);
    });
  } else {
    uint64_t out_rec = 0;
    for (size_t c = 0; c < n; ++c) {
      out_rec += fill_cmd(c, out_rec);
      const uint32_t inst = h->h_cmds[c].instance;
      if (inst < N) {
        const uint64_t lp = h->log_prev[inst];
        if ((lp >> 32) == (win & 0xFFFFFFFFu)) h->h_logcmd[c].prev = (uint32_t)lp;
        h->log_prev[inst] = ((win & 0xFFFFFFFFu) << 32) | (uint32_t)c;
      }
    }
  }
  if (int rc = log_next_buffer(h)) return rc;
  if (n) HIPCHK(hipMemcpyAsync(h->d_logcmd, h->h_logcmd.data(), n * sizeof(LogCmd), hipMemcpyHostToDevice, h->stream));
  if (h->inst_proc.size() >= N)
    HIPCHK(hipMemcpyAsync(h->d_inst_proc, h->inst_proc.data(), N * sizeof(uint16_t), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemsetAsync(h->d_log_flag, 0, sizeof(uint32_t), h->stream));
  a.phase = 0;
  HIPCHK(launch_log_device(a, h->stream));
  HIPCHK(hipMemcpyAsync(&total, h->d_log_bytes + n, sizeof total, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(&flag, h->d_log_flag, sizeof flag, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  }
  const auto t3 = now();
  int rc = ZBHIP_OK;
  if (flag & 1u) {
    rc = ZBHIP_EUNSUPP;  // a key the ring does not hold, or a value outside the device writer
  } else {
    if (spec && total <= h->log_out_cap) {  // the bytes are written: composed entries only
      if (flag & 2u) {
        a.out = h->d_log_out;
        a.out_cap = 0;
        a.compose = 2;
        a.phase = 1;
        HIPCHK(launch_log_device(a, h->stream));
      }
    } else {
    if (total > h->log_out_cap) {
      (void)hipFree(h->d_log_out);
      h->d_log_out = nullptr;
      h->log_out_cap = 0;
      const size_t cap = std::max<size_t>(total + total / 4, 1 << 20);
      if (dalloc(&h->d_log_out, cap / 8) != hipSuccess) return ZBHIP_ENOMEM;
      h->log_out_cap = cap / 8 * 8;
    }
    a.out = h->d_log_out;
    a.out_cap = 0;
    a.compose = (flag & 2u) ? 1 : 0;
    a.phase = 1;
    HIPCHK(launch_log_device(a, h->stream));
    }
    *dev_bytes = h->d_log_out;
    *used = total;
  }
  a.phase = 2;  // the window's keys into the ring, in any case
  HIPCHK(launch_log_device(a, h->stream));
  // (no wait: the bytes are complete in the handle's stream order -- zbhip_log_device_copy and the
  // next window's run wait for them, and the host meanwhile takes the next window)
  if (dbg) {
    HIPCHK(hipStreamSynchronize(h->stream));
    const auto t4 = now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr, "[zbhip] serialize_log_device n=%zu (%s table): finalize %.2f ms, table %.2f ms (uploads %.2f, "
            "key bookkeeping %.2f, wait %.2f), upload+sizes %.2f ms, write+ring %.2f ms\n", n,
            dev_table ? "device" : "host", ms(t0, t1), ms(t1, t2), dev_table ? ms(t1, tu) : 0.0,
            dev_table ? ms(tu, tf) : 0.0, dev_table ? ms(tf, t2) : 0.0, ms(t2, t3), ms(t3, t4));
  }
  return rc;
}

// Double-buffered log output (zbhip_log_copy_async): the window about to be written takes the other device
// buffer; the stream waits for the copy still reading it (two windows back).
static int log_next_buffer(zbhip_handle* h) {
  if (!h->log_double) return ZBHIP_OK;
  zbhip_handle::LogBuf& cur = h->log_bufs[h->log_cur];
  cur.dev = h->d_log_out;
  cur.dev_cap = h->log_out_cap;
  h->log_cur ^= 1;
  zbhip_handle::LogBuf& nxt = h->log_bufs[h->log_cur];
  if (nxt.pending) HIPCHK(hipStreamWaitEvent(h->stream, nxt.copied, 0));
  h->d_log_out = nxt.dev;
  h->log_out_cap = nxt.dev_cap;
  return ZBHIP_OK;
}

extern "C" int zbhip_log_copy_async(zbhip_handle* h, size_t n, const void** host_bytes) {
  if (!h || !host_bytes) return ZBHIP_EINVAL;
  *host_bytes = nullptr;
  if (n > h->log_out_cap || (n && !h->d_log_out)) return ZBHIP_EINVAL;
  if (!h->copy_stream) {
    // a high-priority stream: HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues round robin, and a copy
    // stream sharing the compute stream's queue would run its blit behind the next window's kernels (measured:
    // no overlap at all); priority streams come from a queue pool of their own
    int lo = 0, hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPCHK(hipStreamCreateWithPriority(&h->copy_stream, hipStreamNonBlocking, hi));
    for (auto& L : h->log_bufs) {
      HIPCHK(hipEventCreateWithFlags(&L.written, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&L.copied, hipEventDisableTiming));
    }
  }
  zbhip_handle::LogBuf& L = h->log_bufs[h->log_cur];
  if (L.host_cap < n) {  // (grown before its first use, or after its last copy was waited for)
    if (L.pending) HIPCHK(hipEventSynchronize(L.copied));
    L.pending = false;
    if (L.host) (void)hipHostFree(L.host);
    L.host = nullptr;
    L.host_cap = 0;
    const size_t cap = n + n / 8 + (1 << 20);
    if (hipHostMalloc(reinterpret_cast<void**>(&L.host), cap, hipHostMallocDefault) != hipSuccess) return ZBHIP_ENOMEM;
    L.host_cap = cap;
  }
  HIPCHK(hipEventRecord(L.written, h->stream));
  HIPCHK(hipStreamWaitEvent(h->copy_stream, L.written, 0));
  if (n) HIPCHK(hipMemcpyAsync(L.host, h->d_log_out, n, hipMemcpyDeviceToHost, h->copy_stream));
  HIPCHK(hipEventRecord(L.copied, h->copy_stream));
  L.pending = true;
  h->log_double = true;
  *host_bytes = L.host;
  return ZBHIP_OK;
}

extern "C" int zbhip_log_copy_wait(zbhip_handle* h, const void* host_bytes) {
  if (!h) return ZBHIP_EINVAL;
  for (auto& L : h->log_bufs)
    if (host_bytes == nullptr || L.host == host_bytes) {
      if (L.pending) HIPCHK(hipEventSynchronize(L.copied));
      L.pending = false;
      if (host_bytes) return ZBHIP_OK;
    }
  return host_bytes ? ZBHIP_EINVAL : ZBHIP_OK;
}

extern "C" int zbhip_log_device_copy(zbhip_handle* h, void* dst, size_t n) {
  if (!h || (n && !dst)) return ZBHIP_EINVAL;
  if (n > h->log_out_cap || (n && !h->d_log_out)) return ZBHIP_EINVAL;
  if (n) HIPCHK(hipMemcpyAsync(dst, h->d_log_out, n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return ZBHIP_OK;
}
