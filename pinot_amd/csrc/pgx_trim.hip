// Combine trim on the device for group-by results that stay in HBM (the partitioned sparse
// group-by, pgx_host.cpp run_partitioned), and the gather of selected groups.
//
// The reference trims the combined map when it holds more than 20 x max(topN, 1000) groups: per aggregation function
// a MinMaxPriorityQueue keeps the 5 x max(topN, 1000) best values, largest first, smallest first for MIN functions
// (query/aggregation/groupby/AggregationGroupByOperatorService.java:64-76, :284-440; the comparator looks at the value
// only).  Here the same selection is a radix select over a 64-bit order key per group (8 passes of 8 bits, each a
// histogram of the groups still matching the selected prefix), then one compaction pass that keeps every group above
// the threshold key and as many threshold ties as fit.  Which of several tied groups at the threshold survive is
// arbitrary, as in the reference (heap order; parity unpinned); the kept values are exact.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PGX_GLOBAL __attribute__((address_space(1)))

namespace pgx {

// Plane layout of a partitioned result (pgx_part_aggregate): oplane[p * ocap + g], p = 0 count, 1 int64 sum,
// 2 ordered min, 3 ordered max.
enum TrimKind : int { TK_COUNT = 0, TK_SUM = 1, TK_MIN = 2, TK_MAX = 3, TK_AVG = 4 };

// Layout shared with pgx_host.cpp (device_trim writes prefix / mask / k / shift before the launch).
struct TrimState {
  unsigned long long prefix;   // selected high bits of the threshold key          (offset 0)
  unsigned long long mask;     // which bits of prefix are fixed                   (8)
  long long k;                 // groups still to take among those matching prefix (16)
  int shift;                   // bit position of the digit of the next pass       (24)
  int pad;
  unsigned long long n_sel;    // compaction cursors                               (32)
  unsigned long long n_tie;    //                                                  (40)
  unsigned int hist[256];      //                                                  (48)
};

// Larger key = better group.
__device__ __forceinline__ uint64_t trim_key(const PGX_GLOBAL uint64_t* pl, int64_t ocap, int64_t i, int kind) {
  switch (kind) {
    case TK_COUNT:
      return pl[i];
    case TK_SUM:
      return pl[ocap + i] ^ 0x8000000000000000ull;
    case TK_MIN:
      return ~pl[2 * ocap + i];
    case TK_MAX:
      return pl[3 * ocap + i];
    default: {  // AVG: the ratio sum / count as an ordered double (AvgPair compares by value)
      const uint64_t c = pl[i];
      const double d = c ? static_cast<double>(static_cast<int64_t>(pl[ocap + i])) / static_cast<double>(c) : 0.0;
      const uint64_t b = static_cast<uint64_t>(__double_as_longlong(d));
      return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
    }
  }
}

__global__ void __launch_bounds__(256) pgx_trim_hist(const uint64_t* __restrict__ oplane, int64_t ocap, int64_t n,
                                                     int kind, TrimState* __restrict__ st) {
  __shared__ unsigned int lh[256];
  const int tid = threadIdx.x;
  lh[tid] = 0u;
  __syncthreads();
  const unsigned long long prefix = st->prefix, mask = st->mask;
  const int shift = st->shift;
  const PGX_GLOBAL uint64_t* pl = (const PGX_GLOBAL uint64_t*)oplane;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + tid; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const uint64_t key = trim_key(pl, ocap, i, kind);
    if ((key & mask) == prefix) atomicAdd(&lh[(key >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (lh[tid]) atomicAdd(&st->hist[tid], lh[tid]);
}

// One lane: fix the next digit of the threshold from the histogram (the largest digit d whose bins >= d hold at
// least k groups), then clear the histogram for the next pass.
__global__ void pgx_trim_step(TrimState* __restrict__ st) {
  if (threadIdx.x != 0) return;
  long long above = 0;
  int d = 255;
  for (; d > 0; --d) {
    const long long h = st->hist[d];
    if (above + h >= st->k) break;
    above += h;
  }
  st->prefix |= static_cast<unsigned long long>(d) << st->shift;
  st->mask |= 255ull << st->shift;
  st->k -= above;
  st->shift -= 8;
  for (int b = 0; b < 256; ++b) st->hist[b] = 0u;
}

__global__ void __launch_bounds__(256) pgx_trim_select(const uint64_t* __restrict__ oplane, int64_t ocap, int64_t n,
                                                       int kind, TrimState* __restrict__ st, int64_t* __restrict__ idx,
                                                       uint64_t* __restrict__ keys, int64_t cap) {
  const unsigned long long thr = st->prefix;
  const long long ties = st->k;
  const PGX_GLOBAL uint64_t* pl = (const PGX_GLOBAL uint64_t*)oplane;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const uint64_t key = trim_key(pl, ocap, i, kind);
    bool take = key > thr;
    if (!take && key == thr) take = static_cast<long long>(atomicAdd(&st->n_tie, 1ull)) < ties;
    if (take) {
      const unsigned long long p = atomicAdd(&st->n_sel, 1ull);
      if (p < static_cast<unsigned long long>(cap)) {
        idx[p] = i;
        keys[p] = key;
      }
    }
  }
}

// Gather selected groups: out[0, m) packed keys, then planes 0..3 (m words each).
__global__ void __launch_bounds__(256) pgx_group_gather(const uint64_t* __restrict__ okey,
                                                        const uint64_t* __restrict__ oplane, int64_t ocap,
                                                        const int64_t* __restrict__ idx, int64_t m,
                                                        uint64_t* __restrict__ out) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (j >= m) return;
  const int64_t i = idx[j];
  out[j] = okey[i];
#pragma unroll
  for (int p = 0; p < 4; ++p) out[(p + 1) * m + j] = oplane[p * ocap + i];
}

}  // namespace pgx

// Host launchers (pgx_host.cpp).  The state block is prepared by the caller: prefix = mask = 0, k = groups wanted,
// shift = 56, everything else zero.
extern "C" hipError_t pgx_launch_trim(const uint64_t* oplane, int64_t ocap, int64_t n, int kind, void* state,
                                      int64_t* idx, uint64_t* keys, int64_t cap, int grid, hipStream_t stream) {
  pgx::TrimState* st = static_cast<pgx::TrimState*>(state);
  for (int pass = 0; pass < 8; ++pass) {
    hipLaunchKernelGGL(pgx::pgx_trim_hist, dim3(grid), dim3(256), 0, stream, oplane, ocap, n, kind, st);
    hipLaunchKernelGGL(pgx::pgx_trim_step, dim3(1), dim3(64), 0, stream, st);
  }
  hipLaunchKernelGGL(pgx::pgx_trim_select, dim3(grid), dim3(256), 0, stream, oplane, ocap, n, kind, st, idx, keys,
                     cap);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_group_gather(const uint64_t* okey, const uint64_t* oplane, int64_t ocap,
                                              const int64_t* idx, int64_t m, uint64_t* out, hipStream_t stream) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(pgx::pgx_group_gather, dim3(static_cast<unsigned>((m + 255) / 256)), dim3(256), 0, stream, okey,
                     oplane, ocap, idx, m, out);
  return hipGetLastError();
}

extern "C" size_t pgx_trim_state_bytes(void) { return sizeof(pgx::TrimState); }
