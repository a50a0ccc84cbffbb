// Combine trim on the device for group-by results that stay in HBM (the partitioned sparse
// group-by, pgx_part.cpp run_partitioned), and the gather of selected groups.
//
// The reference trims the combined map when it holds more than 20 x max(topN, 1000) groups: per aggregation function
// a MinMaxPriorityQueue keeps the 5 x max(topN, 1000) best values, largest first, smallest first for MIN functions
// (query/aggregation/groupby/AggregationGroupByOperatorService.java:64-76, :284-440; the comparator looks at the value
// only).  Here the same selection is a radix select over a 64-bit order key per group (passes of 11-bit digits, each a
// histogram of the groups still matching the selected prefix), then one compaction pass that keeps every group above
// the threshold key and as many threshold ties as fit.  After the first digit the groups at or above the threshold's
// bin -- the only ones the later passes and the selection can keep -- are copied out (index + key) once, and the later
// passes read that short list instead of the planes (two full reads of a plane per function instead of up to eight).  Which of several tied groups at the threshold survive is
// arbitrary, as in the reference (heap order; parity unpinned); the kept values are exact.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PGX_GLOBAL __attribute__((address_space(1)))

namespace pgx {

// Plane layout of a partitioned result (pgx_part_aggregate): oplane[p * ocap + g], p = 0 count, 1 int64 sum,
// 2 ordered min, 3 ordered max.
enum TrimKind : int { TK_COUNT = 0, TK_SUM = 1, TK_MIN = 2, TK_MAX = 3, TK_AVG = 4, TK_SUMF = 5, TK_AVGF = 6 };

// Layout shared with pgx_part.cpp (device_trim writes k, kmin = ~0 and zeros before the launch).  One state per
// function: every kernel below takes an array of states and the function slot is blockIdx.y.
struct TrimState {
  unsigned long long prefix;   // selected high bits of the threshold key          (offset 0)
  unsigned long long mask;     // which bits of prefix are fixed                   (8)
  long long k;                 // groups still to take among those matching prefix (16)
  int shift;                   // bit position of the digit of the next pass       (24)
  int done;                    // threshold complete (no more histogram passes)   (28)
  unsigned long long n_sel;    // compaction cursors                               (32)
  unsigned long long n_tie;    //                                                  (40)
  unsigned long long kmin;     // key range of the groups                          (48)
  unsigned long long kmax;     //                                                  (56)
  unsigned int hist[2048];     //                                                  (64)
  unsigned long long n_cand;   // groups copied to the candidate list (pgx_trim_cand)
};
constexpr int kTrimDigit = 11;             // bits per histogram pass
constexpr int kTrimBins = 1 << kTrimDigit;
constexpr int kTrimPasses = (64 + kTrimDigit - 1) / kTrimDigit;

constexpr int kTrimMaxFns = 8;
struct TrimKinds {             // function slot -> trim key kind, and the plane holding its value (sum plane for AVG)
  int kind[kTrimMaxFns];
  int plane[kTrimMaxFns];
};

// Where a pass reads its groups: the planes (trim_key of group i), or -- once pgx_trim_cand has run and its list fit --
// function y's candidate list (cidx / ckey + y * ccap: the group's index and key).
struct TrimSrc {
  const uint64_t* oplane;
  int64_t ocap, n;
  const int64_t* cidx;
  const uint64_t* ckey;
  int64_t ccap;
};
__device__ __forceinline__ bool trim_use_cand(const TrimState* st, const TrimSrc& S) {
  return st->n_cand - 1ull < static_cast<unsigned long long>(S.ccap);  // 0 < n_cand <= ccap
}

// Larger key = better group.  Plane 0 is the count; `plane` the function's value plane.
__device__ __forceinline__ uint64_t trim_key(const PGX_GLOBAL uint64_t* pl, int64_t ocap, int64_t i, int kind,
                                             int plane) {
  const PGX_GLOBAL uint64_t* v = pl + static_cast<int64_t>(plane) * ocap;
  switch (kind) {
    case TK_COUNT:
      return pl[i];
    case TK_SUM:
      return v[i] ^ 0x8000000000000000ull;
    case TK_MIN:
      return ~v[i];
    case TK_MAX:
      return v[i];
    case TK_SUMF: {  // f64 sum bits -> ordered
      const uint64_t b = v[i];
      return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
    }
    default: {  // AVG: the ratio sum / count as an ordered double (AvgPair compares by value)
      const uint64_t c = pl[i];
      const double s = kind == TK_AVGF ? __longlong_as_double(static_cast<long long>(v[i]))
                                       : static_cast<double>(static_cast<int64_t>(v[i]));
      const double d = c ? s / static_cast<double>(c) : 0.0;
      const uint64_t b = static_cast<uint64_t>(__double_as_longlong(d));
      return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
    }
  }
}

// Key range per function: the digits above the highest bit in which the smallest and largest keys differ are the
// same for every group, so the radix passes start below them (C3's sums span ~27 bits: 4 passes instead of 8).
__global__ void __launch_bounds__(256) pgx_trim_range(const uint64_t* __restrict__ oplane, int64_t ocap, int64_t n,
                                                      const TrimKinds K, TrimState* __restrict__ sts) {
  __shared__ unsigned long long wmin[4], wmax[4];
  TrimState* st = sts + blockIdx.y;
  const int kind = K.kind[blockIdx.y], plane = K.plane[blockIdx.y];
  const PGX_GLOBAL uint64_t* pl = (const PGX_GLOBAL uint64_t*)oplane;
  unsigned long long lo = ~0ull, hi = 0ull;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const uint64_t key = trim_key(pl, ocap, i, kind, plane);
    lo = key < lo ? key : lo;
    hi = key > hi ? key : hi;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long a = __shfl_xor(lo, d, 64), b = __shfl_xor(hi, d, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    wmin[threadIdx.x >> 6] = lo;
    wmax[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      lo = wmin[w] < lo ? wmin[w] : lo;
      hi = wmax[w] > hi ? wmax[w] : hi;
    }
    atomicMin(&st->kmin, lo);
    atomicMax(&st->kmax, hi);
  }
}

// Key ranges computed by the kernel that wrote the planes (pgx_narrow_aggregate): prange[k] = smallest and
// prange[4 + k] = largest trim key of kind k (COUNT / SUM / MIN / MAX), so the range pass need not re-read the planes.
__global__ void pgx_trim_seed(const unsigned long long* __restrict__ prange, const TrimKinds K,
                              TrimState* __restrict__ sts) {
  if (threadIdx.x != 0) return;
  TrimState* st = sts + blockIdx.x;
  const int kind = K.kind[blockIdx.x];
  st->kmin = prange[kind];
  st->kmax = prange[4 + kind];
}

// One lane per function: fix the bits above the highest differing bit, first digit just below them.
__global__ void pgx_trim_begin(TrimState* __restrict__ sts) {
  if (threadIdx.x != 0) return;
  TrimState* st = sts + blockIdx.x;
  const unsigned long long x = st->kmin ^ st->kmax;
  if (st->kmin > st->kmax || x == 0ull) {  // no groups, or every key equal: all ties at kmin
    st->prefix = st->kmin;
    st->mask = ~0ull;
    st->done = 1;
    return;
  }
  const int hb = 64 - __clzll(static_cast<long long>(x));  // bits [0, hb) vary
  st->mask = hb == 64 ? 0ull : ~((1ull << hb) - 1ull);
  st->prefix = st->kmin & st->mask;
  st->shift = hb > kTrimDigit ? hb - kTrimDigit : 0;
  st->done = 0;
}

__global__ void __launch_bounds__(256) pgx_trim_hist(const TrimSrc S, const TrimKinds K, TrimState* __restrict__ sts) {
  TrimState* st = sts + blockIdx.y;
  if (st->done) return;
  const bool cand = trim_use_cand(st, S);
  const int64_t n = cand ? static_cast<int64_t>(st->n_cand) : S.n;
  if (static_cast<int64_t>(blockIdx.x) * 256 >= n) return;  // (a short candidate list: most workgroups idle)
  const PGX_GLOBAL uint64_t* ck = (const PGX_GLOBAL uint64_t*)S.ckey + static_cast<int64_t>(blockIdx.y) * S.ccap;
  __shared__ unsigned int lh[kTrimBins];
  const int tid = threadIdx.x;
  const int kind = K.kind[blockIdx.y], plane = K.plane[blockIdx.y];
  for (int b = tid; b < kTrimBins; b += 256) lh[b] = 0u;
  __syncthreads();
  const unsigned long long prefix = st->prefix, mask = st->mask;
  const int shift = st->shift;
  const PGX_GLOBAL uint64_t* pl = (const PGX_GLOBAL uint64_t*)S.oplane;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + tid; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const uint64_t key = cand ? ck[i] : trim_key(pl, S.ocap, i, kind, plane);
    if ((key & mask) == prefix) atomicAdd(&lh[(key >> shift) & (kTrimBins - 1u)], 1u);
  }
  __syncthreads();
  for (int b = tid; b < kTrimBins; b += 256)
    if (lh[b]) atomicAdd(&st->hist[b], lh[b]);
}

// After the first digit: every group at or above the threshold's bin (key >= prefix: the bits below the fixed ones are
// zero in prefix) to function y's candidate list.  A workgroup scans one contiguous range and lists its candidates in
// LDS, reserving list space with ONE device atomic per flush (a few per workgroup): a wavefront atomic per 64 groups on
// one address would serialise (~11 ns each, ~10^5 of them at C3).  A list that would run past ccap is abandoned
// (n_cand > ccap: the later passes read the planes).
constexpr int kCandLds = 2048;
__global__ void __launch_bounds__(256) pgx_trim_cand(const TrimSrc S, const TrimKinds K, TrimState* __restrict__ sts,
                                                     int64_t* __restrict__ cidx, uint64_t* __restrict__ ckey) {
  __shared__ uint32_t lidx[kCandLds];
  __shared__ uint64_t lkey[kCandLds];
  __shared__ unsigned int lcnt;
  __shared__ unsigned long long gbase;
  TrimState* st = sts + blockIdx.y;
  if (st->done) return;  // threshold complete after one digit: the selection reads the planes once
  const int kind = K.kind[blockIdx.y], plane = K.plane[blockIdx.y];
  const unsigned long long prefix = st->prefix;
  const PGX_GLOBAL uint64_t* pl = (const PGX_GLOBAL uint64_t*)S.oplane;
  cidx += static_cast<int64_t>(blockIdx.y) * S.ccap;
  ckey += static_cast<int64_t>(blockIdx.y) * S.ccap;
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t chunk = (S.n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * chunk;
  const int64_t hi = lo + chunk < S.n ? lo + chunk : S.n;
  if (tid == 0) lcnt = 0u;
  __syncthreads();
  for (int64_t b = lo; b < hi; b += 256) {
    const int64_t i = b + tid;
    const uint64_t key = i < hi ? trim_key(pl, S.ocap, i, kind, plane) : 0ull;
    const bool in = i < hi && key >= prefix;
    const unsigned long long m = __ballot(in);
    if (m) {
      const int leader = __ffsll(static_cast<long long>(m)) - 1;
      unsigned int r0 = 0u;
      if (lane == leader) r0 = atomicAdd(&lcnt, static_cast<unsigned int>(__popcll(m)));
      const unsigned int r = __shfl(r0, leader, 64) + static_cast<unsigned int>(__popcll(m & ((1ull << lane) - 1ull)));
      if (in) {  // r < kCandLds: the list is flushed while it has room for a whole round
        lidx[r] = static_cast<uint32_t>(i - lo);
        lkey[r] = key;
      }
    }
    __syncthreads();
    const unsigned int nl = lcnt;
    if (nl > static_cast<unsigned int>(kCandLds - 256) || b + 256 >= hi) {  // (uniform)
      if (tid == 0 && nl) gbase = atomicAdd(&st->n_cand, static_cast<unsigned long long>(nl));
      __syncthreads();
      for (unsigned int j = tid; j < nl; j += 256) {
        const unsigned long long p = gbase + j;
        if (p < static_cast<unsigned long long>(S.ccap)) {
          cidx[p] = lo + lidx[j];
          ckey[p] = lkey[j];
        }
      }
      __syncthreads();
      if (tid == 0) lcnt = 0u;
      __syncthreads();
    }
  }
}

// One wavefront per function: fix the next digit of the threshold from the histogram (the largest digit d whose bins
// >= d hold at least k groups), then clear the histogram for the next pass.  Lane l holds bins [32 l, 32 l + 32).
// Digits may overlap bits fixed before (the last one ends at bit 0): those bits are equal in every key matching the
// prefix, so OR-ing them in changes nothing.
__global__ void pgx_trim_step(TrimState* __restrict__ sts) {
  TrimState* st = sts + blockIdx.x;
  if (st->done) return;
  const int lane = threadIdx.x;
  constexpr int kPer = kTrimBins / 64;
  long long mine = 0;
  for (int i = 0; i < kPer; ++i) mine += st->hist[lane * kPer + i];
  // suffix sums over lanes: S(l) = bins of lanes >= l
  long long suf = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const long long y = __shfl_down(suf, d, 64);
    if (lane + d < 64) suf += y;
  }
  const long long k = st->k;
  // the highest lane whose suffix reaches k holds the threshold digit (lane 0 if none: every group is kept)
  const unsigned long long reach = __ballot(suf >= k);
  const int L = reach ? 63 - __clzll(static_cast<long long>(reach)) : 0;
  const long long above_lane = __shfl(suf - mine, L, 64);  // bins of lanes > L
  if (lane == L) {
    long long above = above_lane;
    int d = L * kPer + kPer - 1;
    for (; d > L * kPer; --d) {
      const long long h = st->hist[d];
      if (above + h >= k) break;
      above += h;
    }
    if (!reach) d = 0;
    st->prefix |= static_cast<unsigned long long>(d) << st->shift;
    st->mask |= static_cast<unsigned long long>(kTrimBins - 1) << st->shift;
    st->k -= above;
    if (st->shift == 0) st->done = 1;
    else st->shift = st->shift > kTrimDigit ? st->shift - kTrimDigit : 0;
  }
  __syncthreads();
  for (int i = 0; i < kPer; ++i) st->hist[lane * kPer + i] = 0u;
}

// Function slot y writes its selection to idx / keys + y * cap.  A workgroup scans one contiguous range of groups.
// Groups above the threshold key are taken at once (wave-aggregated reservations: at most k of them exist).  Threshold
// ties are listed in the workgroup's LDS and reserved with ONE atomic per workgroup at the end: a MIN or MAX threshold
// can tie tens of thousands of groups, and one device-scope atomic per wave on one address serialises at ~11 ns each.
// A workgroup whose range holds more than kTieCap ties reserves the rest per wave as it finds them.
constexpr int kTieCap = 2048;
__global__ void __launch_bounds__(256) pgx_trim_select(const TrimSrc S, const TrimKinds K, TrimState* __restrict__ sts,
                                                       int64_t* __restrict__ idx, uint64_t* __restrict__ keys,
                                                       int64_t cap) {
  __shared__ uint32_t tbuf[kTieCap];
  __shared__ unsigned int tcnt;
  __shared__ long long ttake, tsel;
  TrimState* st = sts + blockIdx.y;
  const int kind = K.kind[blockIdx.y], plane = K.plane[blockIdx.y];
  idx += static_cast<int64_t>(blockIdx.y) * cap;
  keys += static_cast<int64_t>(blockIdx.y) * cap;
  const unsigned long long thr = st->prefix;
  const long long ties = st->k;
  const PGX_GLOBAL uint64_t* pl = (const PGX_GLOBAL uint64_t*)S.oplane;
  const bool cand = trim_use_cand(st, S);
  const int64_t n = cand ? static_cast<int64_t>(st->n_cand) : S.n;
  const PGX_GLOBAL uint64_t* ck = (const PGX_GLOBAL uint64_t*)S.ckey + static_cast<int64_t>(blockIdx.y) * S.ccap;
  const PGX_GLOBAL int64_t* ci = (const PGX_GLOBAL int64_t*)S.cidx + static_cast<int64_t>(blockIdx.y) * S.ccap;
  auto orig = [&](int64_t i) -> int64_t { return cand ? ci[i] : i; };  // the group's index in the planes
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  if (threadIdx.x == 0) tcnt = 0u;
  __syncthreads();
  // wave-aggregated reservation of `mask` lanes on cursor c; returns this lane's slot
  auto reserve = [&](unsigned long long* c, unsigned long long mask) -> unsigned long long {
    const int leader = __ffsll(static_cast<long long>(mask)) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(c, static_cast<unsigned long long>(__popcll(mask)));
    return __shfl(base, leader, 64) + __popcll(mask & below);
  };
  for (int64_t b = lo + (threadIdx.x & ~63); b < hi; b += 256) {
    const int64_t i = b + lane;
    const bool valid = i < hi;
    const uint64_t key = valid ? (cand ? ck[i] : trim_key(pl, S.ocap, i, kind, plane)) : 0ull;
    const bool eq = valid && key == thr;
    const unsigned long long em = __ballot(eq);
    bool take = valid && key > thr;
    if (em) {
      const int ld = __ffsll(static_cast<long long>(em)) - 1;
      unsigned int r0 = 0u;
      if (lane == ld) r0 = atomicAdd(&tcnt, static_cast<unsigned int>(__popcll(em)));
      const unsigned int r = __shfl(r0, ld, 64) + static_cast<unsigned int>(__popcll(em & below));
      if (eq && r < static_cast<unsigned int>(kTieCap)) tbuf[r] = static_cast<uint32_t>(i - lo);
      const unsigned long long om = __ballot(eq && r >= static_cast<unsigned int>(kTieCap));
      if (om) {  // LDS list full: this wave reserves its overflowing ties itself
        const unsigned long long t = reserve(&st->n_tie, om);
        take = take || (eq && r >= static_cast<unsigned int>(kTieCap) && static_cast<long long>(t) < ties);
      }
    }
    const unsigned long long tm = __ballot(take);
    if (!tm) continue;
    const unsigned long long p = reserve(&st->n_sel, tm);
    if (take && p < static_cast<unsigned long long>(cap)) {
      idx[p] = orig(i);
      keys[p] = key;
    }
  }
  __syncthreads();
  const unsigned int nt = tcnt < static_cast<unsigned int>(kTieCap) ? tcnt : static_cast<unsigned int>(kTieCap);
  if (threadIdx.x == 0) {
    long long tk = 0, sb = 0;
    if (nt) {
      const long long t0 = static_cast<long long>(atomicAdd(&st->n_tie, static_cast<unsigned long long>(nt)));
      tk = ties - t0;
      tk = tk < 0 ? 0 : (tk > nt ? nt : tk);
      if (tk) sb = static_cast<long long>(atomicAdd(&st->n_sel, static_cast<unsigned long long>(tk)));
    }
    ttake = tk;
    tsel = sb;
  }
  __syncthreads();
  for (long long j = threadIdx.x; j < ttake; j += 256) {
    const long long p = tsel + j;
    if (p < cap) {
      idx[p] = orig(lo + tbuf[j]);
      keys[p] = thr;
    }
  }
}

// Gather selected groups: out[0, m) packed keys, then planes 0 .. nplanes-1 (m words each).
__global__ void __launch_bounds__(256) pgx_group_gather(const uint64_t* __restrict__ okey,
                                                        const uint64_t* __restrict__ oplane, int64_t ocap,
                                                        int nplanes, const int64_t* __restrict__ idx, int64_t m,
                                                        uint64_t* __restrict__ out) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (j >= m) return;
  const int64_t i = idx[j];
  out[j] = okey[i];
  for (int p = 0; p < nplanes; ++p) out[(p + 1) * m + j] = oplane[p * ocap + i];
}

}  // namespace pgx

// Host launchers (pgx_part.cpp device_trim).  The nf state blocks are prepared by the caller: k = groups wanted, kmin = ~0,
// everything else zero.  kinds[f]: TrimKind of function slot f.  At most 8 histogram passes (8-bit digits); passes after
// a function's threshold is complete return at once.
extern "C" hipError_t pgx_launch_trim(const uint64_t* oplane, int64_t ocap, int64_t n, const int* kinds,
                                      const int* planes, int nf,
                                      void* states, int64_t* idx, uint64_t* keys, int64_t cap, int grid,
                                      const unsigned long long* prange, int64_t* cidx, uint64_t* ckey, int64_t ccap,
                                      hipStream_t stream) {
  if (nf < 1 || nf > pgx::kTrimMaxFns || ccap < 0 || (ccap > 0 && (!cidx || !ckey))) return hipErrorInvalidValue;
  const pgx::TrimSrc S{oplane, ocap, n, cidx, ckey, ccap};
  pgx::TrimKinds K{};
  bool seeded = prange != nullptr;
  for (int f = 0; f < nf; ++f) {
    K.kind[f] = kinds[f];
    K.plane[f] = planes[f];
    seeded = seeded && kinds[f] != pgx::TK_AVG && kinds[f] < pgx::TK_SUMF;  // ratios / f64: their range needs the pass
  }
  pgx::TrimState* st = static_cast<pgx::TrimState*>(states);
  const dim3 g(grid, nf);
  if (seeded) hipLaunchKernelGGL(pgx::pgx_trim_seed, dim3(nf), dim3(64), 0, stream, prange, K, st);
  else hipLaunchKernelGGL(pgx::pgx_trim_range, g, dim3(256), 0, stream, oplane, ocap, n, K, st);
  hipLaunchKernelGGL(pgx::pgx_trim_begin, dim3(nf), dim3(64), 0, stream, st);
  for (int pass = 0; pass < pgx::kTrimPasses; ++pass) {
    hipLaunchKernelGGL(pgx::pgx_trim_hist, g, dim3(256), 0, stream, S, K, st);
    hipLaunchKernelGGL(pgx::pgx_trim_step, dim3(nf), dim3(64), 0, stream, st);
    if (pass == 0 && ccap > 0) hipLaunchKernelGGL(pgx::pgx_trim_cand, g, dim3(256), 0, stream, S, K, st, cidx, ckey);
  }
  hipLaunchKernelGGL(pgx::pgx_trim_select, g, dim3(256), 0, stream, S, K, st, idx, keys, cap);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_group_gather(const uint64_t* okey, const uint64_t* oplane, int64_t ocap, int nplanes,
                                              const int64_t* idx, int64_t m, uint64_t* out, hipStream_t stream) {
  if (m <= 0) return hipSuccess;
  if (nplanes < 1 || nplanes > 1 + 3 * 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pgx::pgx_group_gather, dim3(static_cast<unsigned>((m + 255) / 256)), dim3(256), 0, stream, okey,
                     oplane, ocap, nplanes, idx, m, out);
  return hipGetLastError();
}

extern "C" size_t pgx_trim_state_bytes(void) { return sizeof(pgx::TrimState); }
