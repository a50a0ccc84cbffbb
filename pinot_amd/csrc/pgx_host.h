// libpgx host side: what its translation units share.  pgx_host.cpp holds the C ABI of include/pgx.h and query execution
// (launches, result read-back, batched and cached runs); pgx_plan.cpp the per-query planning; pgx_stage.cpp segment
// staging; pgx_part.cpp the partitioned sparse group-by runtime and the device-resident results it produces;
// pgx_plan_cache.cpp, pgx_mv.cpp, pgx_multi.cpp, pgx_realtime.cpp and pgx_fixtures.cpp as their names say.  Context,
// segment, query, result and plan types live here.
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <functional>
#include <thread>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <tuple>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/pgx.h"
#include "pgx_internal.h"
#include "pgx_jit_abi.h"

extern "C" hipError_t pgx_launch_scan(const pgx::KQuery* q, int grid, int64_t tiles_per_wg, size_t lds_bytes,
                                      hipStream_t stream);
extern "C" hipError_t pgx_launch_init_planes(unsigned long long* table, uint64_t slots, int num_planes,
                                             const pgx::KQuery* q, unsigned long long* keys, uint64_t key_words,
                                             unsigned int* key_state, hipStream_t stream);
extern "C" hipError_t pgx_launch_compact(unsigned long long* table, uint64_t slots, int num_planes,
                                         unsigned long long* counter, int64_t* out_slot,
                                         unsigned long long* out_planes, uint64_t cap_out, int reset,
                                         uint32_t min_mask, hipStream_t stream);
extern "C" hipError_t pgx_launch_gather_keys(const unsigned long long* keys, const int64_t* slot,
                                             const unsigned long long* n_dev, int64_t n, int kw, unsigned long long* out,
                                             hipStream_t stream);
extern "C" hipError_t pgx_launch_roaring(const pgx::RDesc* descs, int npairs, int maxchunks, hipStream_t stream);
extern "C" hipError_t pgx_launch_roaring_program_wave(const pgx::RProg* progs, const pgx::RDesc* descs, int nprogs,
                                                      int maxchunks, int nslots, hipStream_t stream);
extern "C" hipError_t pgx_launch_roaring_program(const pgx::RProg* progs, const pgx::RDesc* descs, int nprogs,
                                                 int maxchunks, int maxleaves, hipStream_t stream);
extern "C" hipError_t pgx_launch_synth(uint32_t* out_words, int64_t n_rows, int bits, uint32_t card, uint64_t seed,
                                       int64_t n_words, uint64_t pair_seed, uint32_t npairs, hipStream_t stream);
extern "C" hipError_t pgx_launch_partition(const uint64_t* in, const int64_t* in_off, const unsigned long long* in_cnt,
                                           int in_cstride, int nreg, int reg_div, int64_t in_cap, int chunks_per_reg,
                                           uint64_t keymask, int shift, int nbits, uint64_t* out, int64_t cap,
                                           unsigned long long* cursor, int cstride, unsigned long long* overflow,
                                           hipStream_t stream);
extern "C" hipError_t pgx_launch_mv_leaf_mask(const pgx::MvLeaf* items, int nitems, int max_words, hipStream_t stream);
extern "C" hipError_t pgx_launch_mv_aggregate(const pgx::MvAgg* items, int nitems, int max_words, hipStream_t stream);
extern "C" hipError_t pgx_launch_mv_group(const pgx::MvGroupArgs* args, int nsegs, int max_docs, int ordered,
                                          hipStream_t stream);
extern "C" hipError_t pgx_launch_part_aggregate(const uint64_t* in, const unsigned long long* in_cnt, int cstride,
                                                int nparts, int64_t cap, uint64_t keymask, int keybits, int64_t vbase,
                                                int need_sum, int need_min, int need_max, int pack_shift,
                                                uint64_t* okey, uint64_t* oplane, int64_t ocap,
                                                unsigned long long* ocount, unsigned long long* overflow,
                                                hipStream_t stream);
extern "C" hipError_t pgx_launch_part_aggregate_f64(const uint64_t* in, const unsigned long long* in_cnt, int cstride,
                                                    int nparts, int64_t cap, uint64_t keymask, int keybits,
                                                    const double* fdict, int need_min, int need_max, uint64_t* okey,
                                                    uint64_t* oplane, int64_t ocap, unsigned long long* ocount,
                                                    unsigned long long* overflow, hipStream_t stream);
extern "C" hipError_t pgx_launch_trim(const uint64_t* oplane, int64_t ocap, int64_t n, const int* kinds,
                                      const int* planes, int nf,
                                      void* states, int64_t* idx, uint64_t* keys, int64_t cap, int grid,
                                      const unsigned long long* prange, int64_t* cidx, uint64_t* ckey, int64_t ccap,
                                      hipStream_t stream);
extern "C" hipError_t pgx_launch_group_gather(const uint64_t* okey, const uint64_t* oplane, int64_t ocap, int nplanes,
                                              const int64_t* idx, int64_t m, uint64_t* out, hipStream_t stream);
extern "C" size_t pgx_trim_state_bytes(void);
extern "C" hipError_t pgx_launch_pack_remap(uint32_t* out_words, const int32_t* ids, const int32_t* remap,
                                            int64_t n_rows, int bits, int64_t n_words, hipStream_t stream);
extern "C" hipError_t pgx_launch_narrow_split(const uint32_t* lo, const uint16_t* hi, const unsigned long long* cnt1,
                                              int nbuckets, int nwg, int64_t cap1, int rb1, int k2, uint32_t* out,
                                              int64_t cap2, unsigned int* cnt2, unsigned long long* ovf, int wide,
                                              hipStream_t stream);
extern "C" hipError_t pgx_launch_narrow_aggregate(const uint32_t* in, const unsigned int* cnt2, int64_t cap2,
                                                  int nparts, int rb2, int keybits, int64_t vbase, int img_kind,
                                                  const uint32_t* img, int img_words, int img_sh, const int64_t* vdict,
                                                  int need_sum, int need_min, int need_max, int cshift, uint64_t* okey,
                                                  uint64_t* oplane, int64_t ocap, unsigned long long* ctr,
                                                  unsigned long long* prange, int grid, uint64_t* scratch,
                                                  int64_t scratch_words, int wide, hipStream_t stream);
extern "C" int64_t pgx_narrow_scratch_words(int nparts, int img_kind, int grid);
extern "C" hipError_t pgx_launch_fsm(const pgx::FsmSeg* segs, int nsegs, const uint32_t* table, int S, int L,
                                     int64_t total_chunks, uint32_t* cnt, uint16_t* stv, unsigned long long* pcount,
                                     uint16_t* pstate, int T, unsigned long long* stats, hipStream_t stream);
extern "C" hipError_t pgx_launch_dense_reduce(unsigned long long* dst, const unsigned long long* src, uint64_t slots,
                                              int nplanes, uint64_t ops, hipStream_t stream);
extern "C" hipError_t pgx_launch_join(const uint64_t* okey0, int64_t n0, const uint64_t* okey, const uint64_t* opl,
                                      int64_t ocap, int64_t n, unsigned long long* tkey, int64_t* tidx, uint64_t cap,
                                      uint64_t* comb, int64_t ccap, int base, unsigned long long* miss,
                                      hipStream_t stream);
extern "C" hipError_t pgx_launch_group_merge(const uint64_t* key, const uint64_t* pl, int64_t es, int64_t ps,
                                             int64_t n, unsigned long long* tkey, unsigned long long* tpl,
                                             uint64_t cap, int nplanes, uint64_t ops, unsigned long long* overflow,
                                             hipStream_t stream);
extern "C" hipError_t pgx_launch_group_pack(const uint64_t* okey, const uint64_t* opl, int64_t ocap, int64_t n,
                                            int nplanes, uint64_t* rec, hipStream_t stream);
extern "C" hipError_t pgx_launch_group_compact(const unsigned long long* tkey, const unsigned long long* tpl,
                                               uint64_t cap, int nplanes, uint64_t* okey, uint64_t* opl, int64_t ocap,
                                               unsigned long long* counter, hipStream_t stream);
struct pgx_ctx;
extern "C" void ctx_unref(pgx_ctx* ctx);


using namespace pgx;

namespace pgxh {

inline thread_local std::string g_last_error;

struct PgxError {
  pgx_status status;
  std::string msg;
};

[[noreturn]] inline void fail(pgx_status s, const std::string& m) { throw PgxError{s, m}; }

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) fail(PGX_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// Kernel timing of whole executions (pgx_timing_start / pgx_timing_stop; bench.py's roofline): while a window is open,
// every kernel the library launches is bracketed by two HIP events on the stream it is launched on (the query stream,
// the side stream of batched plans, a caller's stream).  At the end of the window the launches' [start, end] intervals
// give the GPU time an execution really costs: the UNION of busy intervals (concurrent kernels on two streams count
// once), next to the summed per-launch durations and the span.  Process-wide: one window at a time.
struct KTimer {
  std::atomic<bool> on{false};
  std::mutex mu;
  struct Rec {
    hipEvent_t a, b;
    const char* name;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> spare;
  hipEvent_t ref = nullptr;
  hipEvent_t take() {
    std::lock_guard<std::mutex> g(mu);
    if (!spare.empty()) {
      hipEvent_t e = spare.back();
      spare.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  void add(hipEvent_t a, hipEvent_t b, const char* name) {
    std::lock_guard<std::mutex> g(mu);
    recs.push_back({a, b, name});
  }
};
inline KTimer g_kt;

struct KScope {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t st;
  const char* name;
  KScope(hipStream_t s, const char* n) : st(s), name(n) {
    if (!g_kt.on.load(std::memory_order_relaxed)) return;
    a = g_kt.take();
    b = g_kt.take();
    if (a && b && hipEventRecord(a, st) != hipSuccess) a = nullptr;
  }
  ~KScope() {
    if (!a || !b) return;
    if (hipEventRecord(b, st) == hipSuccess) g_kt.add(a, b, name);
  }
};
// launch `call` (returning hipError_t) on stream `st` as kernel `name`, timed when a timing window is open
#define PGX_LAUNCH(st, name, call, what) \
  do {                                   \
    KScope ks_((st), (name));            \
    hip_check((call), (what));           \
  } while (0)

template <typename F>
pgx_status guarded(F&& f) {
  try {
    f();
    return PGX_OK;
  } catch (const PgxError& e) {
    g_last_error = e.msg;
    return e.status;
  } catch (const std::bad_alloc&) {
    g_last_error = "host out of memory";
    return PGX_ERR_OOM;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return PGX_ERR_INTERNAL;
  }
}

inline uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline uint64_t be64(const uint8_t* p) { return (uint64_t(be32(p)) << 32) | be32(p + 4); }

inline uint64_t fnv1a(const void* data, size_t n, uint64_t h = 1469598103934665603ull) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 1099511628211ull;
  }
  return h;
}

// Padded size of a fixed-bit forward index on device: whole tiles (each lane reads exactly `bits` dwords).
inline uint64_t padded_fwd_bytes(int64_t total_docs, int bits) {
  const int64_t tiles = (total_docs + kTileRows - 1) / kTileRows;
  return static_cast<uint64_t>(std::max<int64_t>(tiles, 1)) * (kTileRows / 8) * bits + 64;
}
}  // namespace pgxh
using namespace pgxh;

// =================================================================================================
// Context
// =================================================================================================
// Host worker pool of a context: per-segment query planning of large segment lists runs on it (C5: 4096 segments).
// run(n, f) calls f(i) for i in [0, n) on the workers and the caller; the first exception is rethrown to the caller.
struct WorkerPool {
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv, done_cv;
  const std::function<void(int)>* job = nullptr;
  int njobs = 0, pending = 0;
  std::atomic<int> next{0};
  uint64_t gen = 0;
  bool stop = false;
  std::exception_ptr err;

  void work() {
    for (int i; (i = next.fetch_add(1)) < njobs;) {
      try {
        (*job)(i);
      } catch (...) {
        std::lock_guard<std::mutex> g(m);
        if (!err) err = std::current_exception();
      }
    }
  }
  void start(int nthreads) {
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([this] {
        uint64_t seen = 0;
        for (;;) {
          {
            std::unique_lock<std::mutex> g(m);
            cv.wait(g, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
          }
          work();
          std::lock_guard<std::mutex> g(m);
          if (--pending == 0) done_cv.notify_all();
        }
      });
  }
  std::mutex run_mu;  // one job at a time: concurrent pgx_execute calls on one context take turns here
  void run(int n, const std::function<void(int)>& f) {
    std::lock_guard<std::mutex> one(run_mu);
    std::unique_lock<std::mutex> g(m);
    job = &f;
    njobs = n;
    next = 0;
    err = nullptr;
    pending = int(th.size());
    ++gen;
    cv.notify_all();
    g.unlock();
    work();
    g.lock();
    done_cv.wait(g, [&] { return pending == 0; });
    job = nullptr;
    if (err) std::rethrow_exception(err);
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
};

// Persistent host threads for independent tasks (batched plans: every batch of a long segment list is planned on its own
// thread while the submitting thread launches the batches in order).  Unlike WorkerPool (one parallel loop at a time,
// the caller blocks), submit() returns at once.
struct TaskTeam {
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  bool stop = false;
  void start(int n) {
    for (int t = 0; t < n; ++t)
      th.emplace_back([this] {
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> g(m);
            cv.wait(g, [&] { return stop || !q.empty(); });
            if (q.empty()) return;  // stop, nothing left
            f = std::move(q.front());
            q.pop_front();
          }
          f();  // tasks catch their own exceptions
        }
      });
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m);
      q.push_back(std::move(f));
    }
    cv.notify_one();
  }
  ~TaskTeam() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
};

struct DevBuf;
struct SharedDict;

struct pgx_ctx {
  std::atomic<int> refs{1};  // the caller's handle + one per staged segment
  // Numeric dictionaries (and their LDS value images) staged once per context and shared by every segment holding
  // the same dictionary (key: content hash; content compared on a hit): segments of one table usually share value
  // domains, so thousands of segments then read one L2-resident table instead of thousands of private copies.
  std::mutex dict_mu;
  std::unordered_map<uint64_t, std::weak_ptr<SharedDict>> dicts;
  WorkerPool pool;           // started lazily (first large query)
  std::once_flag pool_once;
  TaskTeam plan_team;        // batched plans (run_batched), started lazily
  std::once_flag plan_once;
  void plan_submit(std::function<void()> f) {
    std::call_once(plan_once, [this] {
      const unsigned hc = std::thread::hardware_concurrency();
      plan_team.start(int(std::min<unsigned>(8, hc > 2 ? hc - 2 : 1)));
    });
    plan_team.submit(std::move(f));
  }
  void parallel_for(int n, const std::function<void(int)>& f) {
    std::call_once(pool_once, [this] {
      const unsigned hc = std::thread::hardware_concurrency();
      pool.start(int(std::min<unsigned>(15, hc > 1 ? hc - 1 : 1)));  // + the caller: 16 (the box's CPU share)
    });
    pool.run(n, f);
  }
  int device = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;  // batched queries: argument uploads + bitmap programs run ahead of the query kernels
  std::mutex mu;
  // Pinned host blocks for the per-query argument arena (one H2D copy per query) and result read-back.
  std::multimap<size_t, void*> pinned_free;
  std::unordered_map<void*, size_t> pinned_live;

  void* pinned_alloc(size_t bytes) {
    bytes = std::max<size_t>(4096, (bytes + 4095) & ~size_t(4095));
    std::lock_guard<std::mutex> g(mu);
    auto it = pinned_free.lower_bound(bytes);
    if (it != pinned_free.end() && it->first <= bytes * 4) {
      void* p = it->second;
      pinned_live[p] = it->first;
      pinned_free.erase(it);
      return p;
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) fail(PGX_ERR_OOM, "hipHostMalloc failed");
    pinned_live[p] = bytes;
    return p;
  }
  void pinned_release(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(mu);
    auto it = pinned_live.find(p);
    if (it == pinned_live.end()) return;
    pinned_free.emplace(it->second, p);
    pinned_live.erase(it);
  }
  // Simple size-bucketed device memory pool (avoids hipMalloc/hipFree on the query path).
  std::multimap<size_t, void*> free_blocks;
  std::unordered_map<void*, size_t> live;

  void* alloc(size_t bytes) {
    bytes = std::max<size_t>(256, (bytes + 255) & ~size_t(255));
    std::lock_guard<std::mutex> g(mu);
    auto it = free_blocks.lower_bound(bytes);
    if (it != free_blocks.end() && it->first <= bytes * 2) {
      void* p = it->second;
      live[p] = it->first;
      free_blocks.erase(it);
      return p;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      // release cached blocks and retry once
      for (auto& kv : free_blocks) (void)hipFree(kv.second);
      free_blocks.clear();
      e = hipMalloc(&p, bytes);
      if (e != hipSuccess) fail(PGX_ERR_OOM, "hipMalloc(" + std::to_string(bytes) + ") failed");
    }
    live[p] = bytes;
    return p;
  }
  void release(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(mu);
    auto it = live.find(p);
    if (it == live.end()) return;
    free_blocks.emplace(it->second, p);
    live.erase(it);
  }
};

struct PinnedBuf {
  pgx_ctx* ctx = nullptr;
  void* p = nullptr;
  PinnedBuf() = default;
  PinnedBuf(pgx_ctx* c, size_t n) : ctx(c), p(c->pinned_alloc(n)) {}
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  PinnedBuf(PinnedBuf&& o) noexcept : ctx(o.ctx), p(o.p) { o.p = nullptr; }
  PinnedBuf& operator=(PinnedBuf&& o) noexcept {
    reset();
    ctx = o.ctx;
    p = o.p;
    o.p = nullptr;
    return *this;
  }
  ~PinnedBuf() { reset(); }
  void reset() {
    if (p && ctx) ctx->pinned_release(p);
    p = nullptr;
  }
  uint8_t* bytes() const { return static_cast<uint8_t*>(p); }
};

struct DevBuf {
  pgx_ctx* ctx = nullptr;
  void* p = nullptr;
  DevBuf() = default;
  DevBuf(pgx_ctx* c, size_t n) : ctx(c), p(c->alloc(n)) {}
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : ctx(o.ctx), p(o.p) { o.p = nullptr; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    reset();
    ctx = o.ctx;
    p = o.p;
    o.p = nullptr;
    return *this;
  }
  ~DevBuf() { reset(); }
  void reset() {
    if (p && ctx) ctx->release(p);
    p = nullptr;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

struct SharedDict {
  int data_type = 0;
  std::vector<uint64_t> enc;  // int64 / double bits per dictId (the device copy's content)
  DevBuf dict;
  DevBuf img;
  int img_kind = 0, img_sh = 0, img_words = 0;
  int64_t vbase = 0;
  uint64_t vrange = 0;
  // the narrow aggregation's packed image (pgx_narrow.hip IMG 4), built on first use: pk_state 0 untried, 1 built,
  // -1 does not fit (guarded by the context's dict_mu)
  DevBuf pk_img;
  int pk_state = 0, pk_sh = 0, pk_words = 0;
};
constexpr int kNarrowImg4Words = (160 * 1024 - 16 * 192 * 20 - 1024) / 4;  // pgx_narrow.hip kNAImg4Words

// =================================================================================================
// Segments
// =================================================================================================
struct StagedColumn {
  std::string name;
  int data_type = 0;
  int card = 0;
  int bits = 0;
  bool is_sorted = false;
  int dict_width = 0;
  bool has_inverted = false;
  // device
  const uint32_t* fwd = nullptr;  // packed fixed-bit (padded)
  DevBuf fwd_owned;
  const void* dict_dev = nullptr;  // int64 / double values per dictId (shared->dict)
  std::shared_ptr<SharedDict> shared;  // the context-wide copy of this dictionary and its value image
  // host
  std::vector<int32_t> sorted_first, sorted_last;  // sorted columns: inclusive doc range per dictId
  std::vector<int64_t> ivals;                      // numeric dictionary values (INT/LONG)
  std::vector<double> dvals;                       // FLOAT/DOUBLE dictionary values
  std::vector<std::string> svals;                  // STRING dictionary values (unpadded)
  int pad_char = 0;                                // STRING padding byte
  uint64_t dict_hash = 0;
  std::vector<uint8_t> inv;                        // bitmap inverted index bytes (host)
  std::vector<uint32_t> inv_off;                   // (card+1) byte offsets of the per-dictId roaring bitmaps
  DevBuf inv_dev;                                  // device copy (expanded by pgx_roaring_expand); null if unusable
  // LDS value image (pgx_jit.cpp): the dictionary re-encoded so a whole column's values fit one workgroup's LDS
  int img_kind = IMG_NONE;
  int img_sh = 0;
  int img_words = 0;
  int64_t vbase = 0;       // integer images hold value - vbase
  uint64_t vrange = 0;     // max(value) - vbase
  const void* img_dev = nullptr;  // shared->img
  // multi-value columns (<col>.mv.fwd): fwd holds the raw value section; doc d owns values [mv_start[d], mv_start[d+1])
  bool is_mv = false;
  int64_t total_entries = 0;
  DevBuf mv_start;
  int max_mv = 0;
};

inline std::atomic<uint64_t> g_segment_uid{1};
inline std::atomic<uint64_t> g_segment_frees{0};  // segments freed so far: a plan-cache entry whose segment pointers match
                                           // and no segment was freed since it was kept needs no uid comparison

struct pgx_segment {
  pgx_ctx* ctx = nullptr;
  uint64_t uid = g_segment_uid.fetch_add(1);  // never reused: keys the plan cache (a freed address may be reused)
  std::string name;
  int32_t total_docs = 0, total_raw_docs = 0;
  std::vector<StagedColumn> cols;
  std::unordered_map<std::string, int> by_name;
  std::vector<uint8_t> star_tree;
  // OFF_HEAP star tree (core/startree/StarTreeOffHeap.java:95-150, StarTreeIndexNodeOffHeap.java): BFS nodes of
  // {dimName, dimValue, startDoc, endDoc (exclusive), aggDocId, childStart, childEnd}, children sorted by value.
  struct StarNode { int32_t dim, value, start, end, agg, cbeg, cend; };
  bool st_ok = false;
  std::vector<StarNode> st_nodes;
  std::vector<std::string> st_dim_name;          // dimension index -> column name
  std::vector<std::string> st_skip;              // star.tree.skip.materialization.for.dimensions
  uint64_t device_bytes = 0;

  std::vector<std::string> names;  // column names, contiguous: planning looks columns up per segment and query column
  const StagedColumn& col(const std::string& n) const {
    if (names.size() <= 24) {  // a short scan over one or two cache lines beats hashing the name
      for (size_t i = 0; i < names.size(); ++i)
        if (names[i].size() == n.size() && std::memcmp(names[i].data(), n.data(), n.size()) == 0) return cols[i];
      fail(PGX_ERR_INVALID_ARG, "segment " + name + " has no column " + n);
    }
    auto it = by_name.find(n);
    if (it == by_name.end()) fail(PGX_ERR_INVALID_ARG, "segment " + name + " has no column " + n);
    return cols[it->second];
  }
};

// =================================================================================================
// Query
// =================================================================================================
// A caller-given key space for one group-by column (pgx_query_set_key_domain): the sorted distinct values of the column
// over every process's segments, so that every rank plans the same dense slots / packed keys.
struct KeyDomain {
  bool set = false;
  int type = PGX_INT;                 // PGX_INT / PGX_LONG -> iv, PGX_FLOAT / PGX_DOUBLE -> dv, PGX_STRING -> sv
  std::vector<int64_t> iv;
  std::vector<double> dv;
  std::vector<std::string> sv;
  int64_t size() const { return type == PGX_STRING ? int64_t(sv.size()) : (iv.empty() ? int64_t(dv.size()) : int64_t(iv.size())); }
};

struct pgx_query {
  std::vector<int> agg_fn;
  std::vector<std::string> agg_col;  // "" for COUNT(*)
  std::vector<std::string> group_cols;
  int top_n = 10;
  std::vector<pgx_filter_node> filter;
  std::vector<std::string> leaf_col;
  std::vector<int> leaf_kind;
  uint32_t flags = 0;
  std::vector<KeyDomain> key_domain;  // [group column]
  Knobs kn;                           // the PGX_* environment when the query was compiled (read_knobs)
  // global hash-table size the query's last execution needed (run_query starts there instead of at 1M slots and
  // overflowing once more): a start size only, never a result input
  struct Hint {  // an atomic that copies by value (a query is copied for its multi-value part, pgx_mv.cpp)
    mutable std::atomic<uint64_t> v{0};
    Hint() = default;
    Hint(const Hint& o) : v(o.v.load()) {}
    Hint& operator=(const Hint& o) {
      v.store(o.v.load());
      return *this;
    }
    uint64_t load() const { return v.load(); }
    void store(uint64_t x) const { v.store(x); }
  };
  Hint hash_cap_hint;
};

// =================================================================================================
// Result
// =================================================================================================
struct pgx_bindings {
  std::vector<pgx_leaf_binding> arr;
  std::vector<std::vector<uint32_t>> words;  // owned bitsets (arr[i].words points into these)
};

// pgx_execute_async: the query runs on a worker thread of the library's pool (planning, the launches on the context's
// stream, the read-back); the submitting thread returns at once.  The inputs the caller owns only for the duration of
// the call (the segment list, the bindings and their bitsets, the options) are copied here first.  The pool's threads
// live for the whole process (a thread per query cost ~20-40 us of creation and join per query: C1-sized queries).
struct AsyncState {
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  pgx_status status = PGX_OK;
  std::string msg;
  std::vector<pgx_segment*> segs;
  std::vector<pgx_leaf_binding> binds;
  std::vector<std::vector<uint32_t>> words;
  pgx_exec_opts opts{};
  bool has_opts = false;
  void join() {  // until the worker has finished with this state
    std::unique_lock<std::mutex> g(m);
    cv.wait(g, [&] { return done; });
  }
  ~AsyncState() { join(); }
};

class AsyncPool {
 public:
  static AsyncPool& get() {
    static AsyncPool* p = new AsyncPool(kThreads);  // never destroyed: workers may be blocked at process exit
    return *p;
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  static constexpr int kThreads = 8;  // queries in flight per process (bench: 3; one per device under execute_multi)
  explicit AsyncPool(int n) {
    for (int i = 0; i < n; ++i) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return !q_.empty(); });
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

struct pgx_result {
  int64_t stats[4] = {0, 0, 0, 0};
  int num_aggs = 0;
  std::vector<int> agg_fn;
  bool group_by = false;
  int top_n = 10;
  int mode = 0;
  // aggregation-only
  std::vector<double> agg_value;
  std::vector<int64_t> agg_count;
  // group-by (columnar)
  int64_t num_groups = 0;
  std::vector<std::vector<int32_t>> key_seg, key_id;  // [col][group]
  std::vector<std::vector<double>> g_value;          // [fn][group]
  std::vector<std::vector<int64_t>> g_count;         // [fn][group]
  // Partitioned group-by (run_partitioned): the groups stay in device memory until an accessor needs them.
  struct Lazy {
    pgx_ctx* ctx = nullptr;      // holds a context reference (the result may outlive the caller's handle)
    DevBuf okey, oplane;         // packed keys; planes x ocap: count, then sum, min, max per value column
    int nplanes = 4;             // 1 + 3 x value columns
    std::vector<int> agg_plane;  // per function: the plane its value is decoded from (COUNT: 0)
    std::vector<bool> agg_fp;    // per function: a FLOAT / DOUBLE column (f64 sum, ordered-f64 min / max)
    DevBuf prange;               // trim-key ranges per kind (pgx_narrow_aggregate), or none: the trim's range pass
    int64_t ocap = 0;
    std::vector<int> gshift, gbits;
    using Reps = std::shared_ptr<const std::vector<std::vector<int32_t>>>;
    Reps rep_seg, rep_id;  // [col][global id] (shared with a kept plan: every replay's result reads the same tables)
    std::vector<int> agg_kind;
    std::vector<std::vector<int64_t>> trims;  // per function: the device-selected trim, best first
    int64_t trim_size = 0;                    // the size those selections were made for
    ~Lazy() {
      okey.reset();
      oplane.reset();
      prange.reset();
      if (ctx) ctx_unref(ctx);
    }
  };
  std::unique_ptr<Lazy> lazy;
  std::unique_ptr<AsyncState> async;  // declared last: destroyed (joined) before the fields its thread writes
  void ready() const;                 // waits for an async execution; throws its error
  void materialize();
  const std::vector<int64_t>& device_trim(int fn, int64_t size);
  void decode_lazy(const uint64_t* keys, const uint64_t* planes, int64_t n, int64_t out_stride, int32_t* seg_index,
                   int32_t* dict_id, double* value, int64_t* count) const;
};


namespace pgxh {

// ----- physical filter plan (FilterPlanNode.constructPhysicalOperator + reorder, plan/FilterPlanNode.java:77-170) -----
enum PhysKind { PH_SORTED = 0, PH_AND = 1, PH_BITMAP = 2, PH_SCAN = 3, PH_OR = 4 };

struct PNode {
  int op;  // PGX_F_LEAF / AND / OR
  int leaf = -1;
  int phys = PH_SCAN;
  std::vector<PNode> kids;
};

// Global key identity for one group-by column over the executed segments (per-segment dictIds -> union
// dictionary ids).  Identity when every segment holds the same dictionary bytes.
struct GlobalDict {
  int64_t card = 0;
  bool identity = true;
  // [seg][local] -> global; segments with byte-identical dictionaries share one table (and one blob copy)
  std::vector<std::shared_ptr<const std::vector<int32_t>>> remap;
  // [global] -> a (segment, local id) holding the value; rep_seg -1: the caller's key domain, rep_id = domain index
  std::vector<int32_t> rep_seg, rep_id;
};

// Key identity of a query whose segments run on several devices (pgx_execute_multi): the global dictionaries are built
// once over ALL segments, and each device's plan takes its segments' rows of them, so a packed key or dense slot
// means the same group on every device and the per-device partials merge without a remap.
struct Domain {
  const std::vector<GlobalDict>* g = nullptr;  // per group column, over the full segment list
  std::vector<int> index;                      // this device's segment i -> position in the full list
};

inline int bits_for(int64_t card) {
  int b = 1;
  while ((int64_t(1) << b) < card) ++b;
  return b;
}

constexpr int kPart1Bits = 7;           // partitioned group-by, first pass: 128 buckets (top bits of the mix)
constexpr int kPart1N = 1 << kPart1Bits;
constexpr int kCursorStride = 16;       // u64 words between partition cursors: one 128-B line each

struct ExecPlan {
  bool serial = false;            // planned on a planner thread: no nested parallel_for on the context's pool
  KQuery kq{};
  std::vector<KSeg> ksegs;
  std::vector<int32_t> blob32;   // ranges / remaps / bitsets, uploaded as one buffer
  struct Fix { size_t seg; int kind; int slot; size_t off; };  // pointer fixups into blob32
  std::vector<Fix> fixes;
  std::vector<std::string> qcols;
  std::vector<GlobalDict> gdicts;
  std::vector<int> gbits;
  int64_t host_entries = 0;
  int64_t total_raw = 0;
  // bitmap inverted-index leaves expanded on device for the query kernels (a-7)
  bool use_docmask = false;
  std::vector<int> leaf_phys;                      // physical operator kind per leaf (FilterPlanNode choice)
  struct RoarItem {
    int seg, leaf;
    bool neg;
    size_t blob_off;
    int nb, nchunks;
    uint64_t mask_off;
    const void* inv;
    uint64_t bytes = 0;  // serialized bytes of its bitmaps (selectivity estimate)
  };
  std::vector<RoarItem> roar;
  std::vector<std::vector<int>> roar_index;        // [seg][leaf] -> index into roar or -1
  std::vector<std::vector<const StagedColumn*>> segcols;  // [seg][query column slot]
  // star-tree segments (a-18): a per-segment filter program over the query's leaves plus doc-range leaves
  struct StarPlan {
    bool on = false;
    std::vector<int> op, arg;                      // postfix program (OP_*)
    std::vector<std::pair<size_t, int>> ranges;    // extra range leaves: (blob offset, number of [a,b] pairs)
  };
  std::vector<StarPlan> star;
  std::vector<std::vector<int32_t>> star_tiles;   // per star segment: local tile ids intersecting its ranges
  size_t star_tile_cap = 0;                       // arena int32 slots reserved for them
  uint64_t mask_words = 0;
  const RDesc* rdesc_dev = nullptr;
  bool roar_early = false;  // the expansion was launched by upload_plan (before the query kernels are planned)
  // a lone query's replay (plan cache, no PGX_X_THROUGHPUT): bitmap programs and query kernel in two halves, the second
  // half's programs on the side stream beside the first half's query kernel (launch_scan)
  bool split2 = false;
  hipStream_t ctx_side = nullptr;
  struct Ev {
    hipEvent_t e = nullptr;
    hipEvent_t get() {
      if (!e) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
      return e;
    }
    ~Ev() {
      if (e) (void)hipEventDestroy(e);
    }
  } ev_pre, ev_half;
  int roar_maxchunks = 0;
  uint32_t* masks_dev = nullptr;
  int n_proj = 0;
  int mode_ref = 0;
  uint64_t dense_slots = 0;
  uint64_t hash_cap = 0;
  int grid = 0;
  int64_t tiles_per_wg = 0;
  size_t lds_bytes = 0;
  // query-specialised kernels (pgx_jit.cpp): one launch per group of segments sharing a shape
  // partitioned group-by (G_HASH64 keys, one integer value column; run_partitioned)
  Knobs kn;  // the query's (plan_query copies them in: partition sizing and launches read them from the plan)
  bool use_part = false;
  int part_vcol = -1;            // query column slot of the aggregated value (-1: COUNT only)
  int part_keybits = 0;
  int part_vbits = 0;
  int64_t part_vbase = 0;
  bool part_sum = false, part_min = false, part_max = false;
  bool part_dictid = false;      // records carry the value's dictId (sorted dictionary), values looked up at aggregation
  bool part_slab = false;        // ... into per-workgroup slabs (dictId records, LDS cursors; pass 2 reads the slabs)
  int64_t part_nwg = 0;          // slab mode: query-kernel workgroups over all launch groups (slabs per bucket)
  int64_t part_wg_rows = 0;      // slab mode: most rows one workgroup scans
  const int64_t* part_vdict = nullptr;  // device int64 value per dictId (part_dictid)
  unsigned long long* part_cursor = nullptr;   // fused first pass: bucket cursors, overflow counter, bucket capacity
  unsigned long long* part_overflow = nullptr;
  int64_t part_cap = 0;
  // narrow records (run_narrow, the default for partitioned plans that qualify): the scan writes dictId records split
  // 256 ways into per-workgroup slabs (part_slab with kNarrow1Bits), u32 in kq.table and bits 32..47 in part_hi
  bool part_narrow = false;
  uint64_t last_groups = 0;  // groups of this plan's previous execution (finish_result's first read-back size)
  std::shared_ptr<const std::vector<std::vector<int32_t>>> lazy_rep_seg, lazy_rep_id;  // part_result's key tables
  int narrow_vd = 0;              // dictId bits of the value column (0: COUNT only)
  int narrow_k2min = 0;           // second-split bits the record width needs
  int narrow_img = 0;             // value image in the aggregation's LDS: 0 none, 1 U32, 2 FOR16, 3 value offsets, 4 packed
  bool narrow_wide = false;       // second-stage records of 64 bits (value offsets too wide for 32-bit records)
  const uint32_t* narrow_imgp = nullptr;
  int narrow_img_words = 0, narrow_img_sh = 0;
  uint64_t narrow_vrange = 0;     // largest value offset (value - vbase)
  unsigned short* part_hi = nullptr;
  // FLOAT / DOUBLE value column: records carry an index into the concatenation of the segments' dictionaries
  // (part_fdict; segment s's dictionary starts at part_fbase[s]), summed in f64 by pgx_part_aggregate_f64
  bool part_fp = false;
  const double* part_fdict = nullptr;
  std::vector<int64_t> part_fbase;
  std::vector<DevBuf> part_fdict_bufs;  // owns the concatenated dictionaries (one per FLOAT / DOUBLE value column)
  // One value column's partitioned-path settings (the fields above from part_vcol to narrow_vrange).  A query whose
  // functions read several value columns runs the pipeline once per column (pgx_part.cpp run_value_columns) and joins
  // the passes' groups by key; part_cols[0] is loaded into the fields above at planning.
  struct PartCol {
    int vcol = -1, vbits = 0;
    int64_t vbase = 0;
    bool sum = false, mn = false, mx = false, dictid = false, slab = false, narrow = false;
    const int64_t* vdict = nullptr;
    int vd = 0, k2min = 0, img = 0, img_words = 0, img_sh = 0;
    bool wide = false;
    const uint32_t* imgp = nullptr;
    uint64_t vrange = 0;
    bool fp = false;
    const double* fdict = nullptr;
    std::vector<int64_t> fbase;
  };
  std::vector<PartCol> part_cols;
  PartCol save_part_col() const {
    PartCol c;
    c.vcol = part_vcol, c.vbits = part_vbits, c.vbase = part_vbase;
    c.sum = part_sum, c.mn = part_min, c.mx = part_max, c.dictid = part_dictid, c.slab = part_slab, c.narrow = part_narrow;
    c.vdict = part_vdict, c.vd = narrow_vd, c.k2min = narrow_k2min, c.img = narrow_img, c.img_words = narrow_img_words;
    c.img_sh = narrow_img_sh, c.imgp = narrow_imgp, c.vrange = narrow_vrange, c.wide = narrow_wide;
    c.fp = part_fp, c.fdict = part_fdict, c.fbase = part_fbase;
    return c;
  }
  void load_part_col(const PartCol& c) {
    part_vcol = c.vcol, part_vbits = c.vbits, part_vbase = c.vbase;
    part_sum = c.sum, part_min = c.mn, part_max = c.mx, part_dictid = c.dictid, part_slab = c.slab, part_narrow = c.narrow;
    part_vdict = c.vdict, narrow_vd = c.vd, narrow_k2min = c.k2min, narrow_img = c.img, narrow_img_words = c.img_words;
    narrow_img_sh = c.img_sh, narrow_imgp = c.imgp, narrow_vrange = c.vrange, narrow_wide = c.wide;
    part_fp = c.fp, part_fdict = c.fdict, part_fbase = c.fbase;
  }
  std::vector<int64_t> rec_base; // per segment: index of its row 0 in the record array
  int64_t rec_total = 0;
  struct JitGroup {
    void* fn = nullptr;
    int T = 256;
    int grid = 1;
    JArgs args{};
    std::vector<JSeg> segs;
  };
  std::vector<JitGroup> jit;
  // bitmap sub-trees evaluated by pgx_roaring_program into one mask each (JIT leaf L + k for program k)
  bool rprog_on = false;
  bool rchunk = false;   // ... evaluated per chunk inside the query kernels (LEAF_RCHUNK), not by a separate pass
  // multi-value scan leaves (pgx_mv_leaf_mask writes one doc mask per (segment, leaf), read as LEAF_DOCMASK)
  struct MvItem { int seg, leaf; };
  std::vector<MvItem> mv_items;
  std::vector<int> mv_neg;                 // [leaf] NEQ / NOT_IN
  std::vector<std::vector<int>> mv_index;  // [seg][leaf] -> index into mv_items or -1
  DevBuf mv_masks, mv_descs;
  std::vector<MvLeaf> mv_host;             // their descriptors (host copy, sent by send_arena)
  int mv_max_words = 0;
  // selection masks for the multi-value functions (one bit per scanned row, per segment)
  bool want_selmask = false;
  DevBuf sel_buf;
  // multi-value group-by results: per function, where its count comes from (-1: plane 0, the (doc, key) pairs; -2: its
  // own value (COUNTMV); p >= 0: plane p (AVGMV's value count))
  std::vector<int> g_count_plane;
  std::vector<int64_t> sel_off;       // [seg] word offset in sel_buf
  struct DmProg {
    std::vector<int> op, arg;  // RP_*; RP_LEAF arg = query leaf index
  };
  std::vector<DmProg> dm_progs;
  std::vector<RProg> rprogs;              // [seg * nprogs + k]
  // bitmap-program kernel choice, decided once per plan (launch_bitmaps; a replay must not walk 4096 programs again):
  // -1 undecided, 0 the wave kernel (rp_nslots mask slots), 1 the wide kernel (rp_maxleaves)
  int rp_kind = -1, rp_nslots = 1, rp_maxleaves = 0;
  const RProg* rprog_dev = nullptr;
  // numEntriesScannedInFilter automaton (pgx_stats.cpp) for filter trees whose statistic has no closed form
  bool fsm_on = false;
  FsmPlan fsm;
  std::vector<int64_t> sorted_span;     // [seg * L + leaf] -> (first << 32 | last) doc of a sorted leaf (0 = empty)
  std::vector<int64_t> lmask_off;       // [seg] word offset of its leaf masks (-1: no automaton for this segment)
  std::vector<int64_t> lmask_words;     // [seg] words per leaf
  uint64_t lmask_total = 0;
  uint32_t* lmask_dev = nullptr;
  std::vector<FsmSeg> fsm_segs;
  int64_t fsm_chunks = 0;
  DevBuf fsm_table, fsm_segbuf, fsm_cnt, fsm_stv, fsm_pcount, fsm_pstate, lmask_buf;
  int fsm_T = 1;
};

// Estimated filter selectivity below which bitmap programs run inside the query kernels (LEAF_RCHUNK).  0: only when
// forced with PGX_RCHUNK=1 (measured slower at C5 so far: the per-chunk container search stalls its workgroup).
constexpr double kRchunkMaxSel = 0.0;

constexpr size_t kOutsBytes = 256;  // agg planes [0, 72), stats [128, 144), overflow [192, 200)
// Dense group tables up to this size live in the argument arena right after the outputs block: the arena copy
// initialises them and ONE read-back returns outputs and table (no init or compaction kernel; C1 / C4 latency)
constexpr size_t kArenaTableMax = 64 * 1024;
struct ExecBuffers {
  DevBuf arena;
  PinnedBuf host;
  size_t off_ksegs = 0, off_jsegs = 0, off_tiles = 0, off_rdesc = 0, off_rprog = 0, off_outs = 0, size = 0;
  size_t tbl_bytes = 0;  // in-arena dense table at off_outs + kOutsBytes (0: none)
  bool tbl_live = false;  // this execution's table is the in-arena one (alloc_outputs)
  DevBuf table, keys, key_state, masks;
  uint64_t table_bytes = 0;  // dense table: size of `table`, kept across executions of a kept plan
  bool table_clean = false;  // ... and its slots are at their initial values (the last compaction reset them)
  uint8_t* dev() const { return arena.as<uint8_t>(); }
};

constexpr int64_t kPartGroupsPerWg = 700;   // groups per pgx_part_aggregate workgroup: LDS table load <= ~1/3 (2048 slots)
constexpr uint64_t kPartMaxBytes = uint64_t(96) << 30;  // partition buffers beyond this: fall back to the hash table
constexpr int kPartChunkRecs = 8192;    // records per pgx_partition workgroup (pgx_kernels.hip kPartChunk)

struct PartBuffers {
  int nbits2 = 7;                       // second pass: 2^nbits2 buckets per first-pass bucket (0: no second pass)
  int64_t cap1 = 0, cap2 = 0, ocap = 0;
  DevBuf out1, out2, okey, oplane, ctr;  // ctr: cursors1[kPart1N] | cursors2[nparts] (kCursorStride apart) | ocount | ovf[3]
  DevBuf prange;                         // trim-key ranges of the groups (narrow aggregation), or none
  bool pass2() const { return nbits2 > 0; }
  int64_t nparts() const { return int64_t(1) << (kPart1Bits + nbits2); }
  size_t ctr_words() const { return size_t(kPart1N + (pass2() ? nparts() : 0)) * kCursorStride + 4; }
  int64_t out1_recs() const { return int64_t(kPart1N) * cap1; }
};

constexpr int kPartMaxValueCols = 4;  // value columns of one partitioned plan (one pipeline run each)
constexpr int kNarrowSlots = 192;  // pgx_narrow.hip kNASlots: one wavefront's table
constexpr int kNarrowMaxWg = 1024; // pgx_narrow.hip kN2MaxSlabs

struct NarrowBuffers {
  int k2 = 0, rb1 = 0, rb2 = 0, cshift = 0;
  bool hib = false;
  int w2 = 1;  // u32 words per second-stage record (2: ExecPlan::narrow_wide)
  int64_t nwg = 0, cap1 = 0, cap2 = 0, ocap = 0, nparts = 0;
  DevBuf lo1, hi1, cnt1, rec2, cnt2, okey, oplane, ctr;  // ctr: ocount | overflow scan | split | aggregation
  DevBuf prange;  // trim-key ranges: [kind] smallest, [4 + kind] largest (pgx_trim.hip)
  DevBuf agg_scratch;  // the aggregation's per-wavefront output regions (pgx_narrow_scratch_words)
  int64_t agg_scratch_words = 0;
};

inline unsigned long long* devp(const DevBuf& b) { return b.as<unsigned long long>(); }
}  // namespace pgxh

namespace pgxh {
// ---- pgx_host.cpp: planning and execution pieces the partitioned runtime drives --------------------------------
bool packed_value_image(pgx_ctx* ctx, SharedDict& sd, const std::vector<int64_t>& ivals);  // pgx_stage.cpp
void alloc_outputs(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, void* dense_out, uint64_t dense_out_bytes);
void reset_outputs(ExecPlan& P, ExecBuffers& B, hipStream_t st, bool init_table = true, bool outs_only = false);
void launch_scan(ExecPlan& P, hipStream_t st);
void plan_jit(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, ExecPlan& P, ExecBuffers& B);
double decode_plane(int op, bool fp, unsigned long long x, int fn);
void upload_plan(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, hipStream_t st);
inline thread_local std::function<void(const char*)> g_prof_mark;  // PGX_DEBUG=host_profile phase marks (run_query)
void prof_mark(const char* what);
void canon_rprog(std::vector<int>& op, std::vector<int>& arg);
void resolve_binding(const StagedColumn& c, int kind, const pgx_predicate& p, int32_t& lo, int32_t& hi,
                     std::vector<uint32_t>& words);
GlobalDict domain_dict(const Domain& d, int col, int n);
uint64_t initial_hash_cap(pgx_segment* const* segs, int n, const ExecPlan& P);
void stage_dict(pgx_ctx* ctx, pgx_segment* seg, const std::vector<uint8_t>& dict_host, StagedColumn& c);
GlobalDict group_dict(const pgx_query& q, pgx_segment* const* segs, int n, int g);
int reference_mode(const pgx_query& q, const pgx_segment* seg);
void plan_query(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
                uint32_t xflags, ExecPlan& P, const Domain* dom = nullptr);
void finish_result(pgx_ctx* ctx, const pgx_query& q, ExecPlan& P, ExecBuffers& B, pgx_segment* const* segs, int n,
                   hipStream_t st, pgx_result* R, const unsigned long long* dense_host_override);
void run_query(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
               const pgx_exec_opts* opts, pgx_result* R, const Domain* dom = nullptr);

// ---- pgx_plan_cache.cpp / pgx_mv.cpp / pgx_stage.cpp ---------------------------------------------------------------
struct PlanEntry {
  pgx_ctx* ctx = nullptr;
  std::vector<uint64_t> uids;
  std::vector<pgx_segment*> ptrs;  // the segment list as passed, and g_segment_frees when last matched
  uint64_t gen = 0;
  uint64_t key = 0;
  std::unique_ptr<ExecPlan> P;
  std::unique_ptr<ExecBuffers> B;
  std::unique_ptr<NarrowBuffers> NB;  // a narrow partitioned plan's slabs and partitions (sized by its first run)
  std::unique_ptr<PartBuffers> PB;    // a radix partitioned plan's buckets and partitions (same)
  bool busy = false;
  uint64_t stamp = 0;
  ~PlanEntry() {
    NB.reset();
    PB.reset();
    B.reset();
    P.reset();
    if (ctx) ctx_unref(ctx);
  }
};


bool plan_cache_on();
uint64_t plan_key(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
                  uint32_t xflags);
std::shared_ptr<PlanEntry> plan_cache_acquire(const pgx_query* q, pgx_segment* const* segs, int n, uint64_t key);
bool plan_cache_seen_before(const pgx_query* q, uint64_t key, const std::vector<uint64_t>& uids);
void plan_cache_release(const std::shared_ptr<PlanEntry>& e);
void plan_cache_insert(const pgx_query* q, pgx_ctx* ctx, pgx_segment* const* segs, int n, std::vector<uint64_t> uids,
                       uint64_t key, std::unique_ptr<ExecPlan> P, std::unique_ptr<ExecBuffers> B,
                       std::unique_ptr<NarrowBuffers> NB = nullptr, std::unique_ptr<PartBuffers> PB = nullptr);
void plan_cache_purge(const pgx_query* q, const pgx_ctx* ctx);
bool plan_cacheable(const ExecPlan& P);

void run_mv(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
            uint32_t xflags, pgx_result* R, hipStream_t st);
void run_mv_group(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
                  uint32_t xflags, pgx_result* R, hipStream_t st, const Domain* dom = nullptr);

void parse_star_tree(pgx_segment& seg);
void stage_column(pgx_ctx* ctx, pgx_segment* seg, const pgx_column_desc& d, bool device_mem, StagedColumn& c);

// ---- pgx_multi.cpp: partials of several devices merged ----------------------------------------------------------
void merge_device_groups(pgx_ctx* ctx, hipStream_t st, const uint64_t* keys, const uint64_t* planes, int64_t es,
                         int64_t ps, int64_t n, const pgx_result::Lazy& like, pgx_result* R);
bool query_is_mv(const pgx_query& q, pgx_segment* const* segs, int n);
void run_multi(pgx_ctx* const* ctxs, int nctx, const pgx_query& q, pgx_segment* const* segs, int n,
               const pgx_leaf_binding* bindings, uint32_t xflags, pgx_result* R);

// ---- pgx_part.cpp: partitioned sparse group-by (radix records, narrow records) ----------------------------------
bool part_debug(const ExecPlan& P);
void part_size(const ExecPlan& P, PartBuffers& PB);
bool part_alloc(pgx_ctx* ctx, const ExecPlan& P, PartBuffers& PB);
void part_prepare(ExecPlan& P, PartBuffers& PB, hipStream_t st);
void part_enqueue(const ExecPlan& P, PartBuffers& PB, hipStream_t st);
bool run_partitioned(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, PartBuffers& PB, hipStream_t st);
bool replay_part(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, PartBuffers& PB, hipStream_t st);
void narrow_prepare(ExecPlan& P, NarrowBuffers& NB, hipStream_t st);
void narrow_enqueue(pgx_ctx* ctx, const ExecPlan& P, NarrowBuffers& NB, hipStream_t st);
bool run_narrow(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, NarrowBuffers& NB, hipStream_t st);
bool replay_narrow(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, NarrowBuffers& NB, hipStream_t st);
void narrow_fallback(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, ExecPlan& P, ExecBuffers& B);
void part_result(pgx_ctx* ctx, const pgx_query& q, ExecPlan& P, ExecBuffers& B, PartBuffers& PB, pgx_result* R);
bool run_value_columns(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, ExecPlan& P, ExecBuffers& B,
                       hipStream_t st, pgx_result* R);
}  // namespace pgxh
