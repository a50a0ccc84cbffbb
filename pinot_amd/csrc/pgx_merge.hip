// Cross-GPU merge of per-device group-by partials, the device-side counterpart of the reference's
// combine over segments served by different executors: operator/MCombineGroupByOperator.java:166-191 merges equal
// group keys with each function's combineTwoValues (CountAggregationFunction.java:79-87 long add,
// SumAggregationFunction.java:168-176 double add, Min/Max extremes, AvgAggregationFunction.java:116-125 pair add).
//
// * pgx_dense_reduce: dst op= src over dense tables of the same layout (slot s = the same group on every device: the
//   plan's key space is the union dictionary of ALL segments of the query), one plane op per plane.  Streams both
//   tables once (16 B read + 8 B written per slot and plane), HBM-bound.
// * pgx_group_merge: sparse groups (packed key + planes: count, then per value column sum / ordered min / ordered max,
//   the layout pgx_part_aggregate / pgx_narrow_aggregate / pgx_part_aggregate_f64 and the several-column join write;
//   a FLOAT / DOUBLE column's sum plane holds f64 bits) from any number of devices, copied side by side into one
//   buffer, are inserted into an open-addressing table in HBM (linear probing on a 64-bit mix of the key, one CAS per
//   new key, then one atomic per plane with the plane's op: int64 add, f64 add, ordered min, ordered max), and
//   pgx_group_compact appends the occupied slots to okey / oplane again (wave-aggregated cursor).  A group of P planes
//   moves 8 (1 + P) B in, P + 1 random 8-B atomics, 8 (1 + P) B out: bound by the atomics' 64-B granules.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pgx {

constexpr unsigned long long kMergeEmpty = ~0ull;  // packed keys use < 64 bits (pgx_plan.cpp part_keybits <= 63)

__device__ __forceinline__ uint64_t merge_mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

// op: 0 int64 add, 1 double add, 2 ordered-u64 min, 3 ordered-u64 max (PlaneOp); ops packs 2 bits per plane.
__global__ void pgx_dense_reduce(unsigned long long* __restrict__ dst, const unsigned long long* __restrict__ src,
                                 uint64_t slots, int nplanes, uint64_t ops) {
  const uint64_t n = slots * static_cast<uint64_t>(nplanes);
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const int op = static_cast<int>((ops >> (2 * (i / slots))) & 3u);
    const unsigned long long a = dst[i], b = src[i];
    unsigned long long r;
    if (op == 0) r = a + b;
    else if (op == 1)
      r = static_cast<unsigned long long>(__double_as_longlong(__longlong_as_double(static_cast<long long>(a)) +
                                                              __longlong_as_double(static_cast<long long>(b))));
    else if (op == 2) r = a < b ? a : b;
    else r = a > b ? a : b;
    dst[i] = r;
  }
}

// Table: tkey[cap] (kMergeEmpty = free), tpl[p * cap + slot] for the planes p < nplanes (min planes start at ~0, the
// others at 0).  ops: 2 bits per plane (PlaneOp: 0 int64 add, 1 f64 add, 2 ordered min, 3 ordered max).  Input group i:
// key[i * es], plane p at pl[p * ps + i * es] (columnar: es = 1, ps = n; records of 1 + nplanes words: key = rec,
// pl = rec + 1, es = 1 + nplanes, ps = 1).  A group whose probe sequence finds no slot counts in *overflow.
__global__ void __launch_bounds__(256) pgx_group_merge(const uint64_t* __restrict__ key,
                                                       const uint64_t* __restrict__ pl, int64_t es, int64_t ps,
                                                       int64_t n, unsigned long long* __restrict__ tkey,
                                                       unsigned long long* __restrict__ tpl, uint64_t cap, int nplanes,
                                                       uint64_t ops, unsigned long long* __restrict__ overflow) {
  const uint64_t mask = cap - 1;  // cap is a power of two
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const unsigned long long k = key[i * es];
    uint64_t h = merge_mix(k) & mask;
    int64_t slot = -1;
    for (uint64_t probe = 0; probe < cap; ++probe) {
      const unsigned long long prev = atomicCAS(tkey + h, kMergeEmpty, k);
      if (prev == kMergeEmpty || prev == k) {
        slot = static_cast<int64_t>(h);
        break;
      }
      h = (h + 1) & mask;
    }
    if (slot < 0) {
      atomicAdd(overflow, 1ull);
      continue;
    }
    const uint64_t* g = pl + i * es;
    for (int p = 0; p < nplanes; ++p) {
      const unsigned long long x = static_cast<unsigned long long>(g[p * ps]);
      unsigned long long* t = tpl + p * cap + slot;
      const int op = static_cast<int>((ops >> (2 * p)) & 3u);
      if (op == 0) atomicAdd(t, x);
      else if (op == 1) atomicAdd(reinterpret_cast<double*>(t), __longlong_as_double(static_cast<long long>(x)));
      else if (op == 2) atomicMin(t, x);
      else atomicMax(t, x);
    }
  }
}

__global__ void __launch_bounds__(256) pgx_group_compact(const unsigned long long* __restrict__ tkey,
                                                         const unsigned long long* __restrict__ tpl, uint64_t cap,
                                                         int nplanes, uint64_t* __restrict__ okey,
                                                         uint64_t* __restrict__ opl, int64_t ocap,
                                                         unsigned long long* __restrict__ counter) {
  // one counter reservation per workgroup tile of 256 x 16 slots: one per wavefront serialised ~500K device atomics on
  // one address for a 33M-slot merge table (~11 ns each)
  __shared__ unsigned int scan[256];
  __shared__ unsigned long long base;
  constexpr int K = 16;
  const int tid = threadIdx.x;
  for (uint64_t t0 = blockIdx.x * static_cast<uint64_t>(256 * K); t0 < cap; t0 += static_cast<uint64_t>(gridDim.x) * 256 * K) {
    unsigned int live = 0, mine = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t s = t0 + k * 256 + tid;
      const bool l = s < cap && tkey[s] != kMergeEmpty;
      live |= (l ? 1u : 0u) << k;
      mine += l;
    }
    scan[tid] = mine;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
      const unsigned int y = tid >= d ? scan[tid - d] : 0u;
      __syncthreads();
      scan[tid] += y;
      __syncthreads();
    }
    if (tid == 255) base = scan[255] ? atomicAdd(counter, static_cast<unsigned long long>(scan[255])) : 0ull;
    __syncthreads();
    unsigned long long j = base + scan[tid] - mine;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (!((live >> k) & 1u)) continue;
      const uint64_t s = t0 + k * 256 + tid;
      if (j < static_cast<unsigned long long>(ocap)) {  // the host sized ocap from the table; cannot run over
        okey[j] = tkey[s];
        for (int p = 0; p < nplanes; ++p) opl[p * ocap + j] = tpl[p * cap + s];
      }
      ++j;
    }
    __syncthreads();  // scan / base are reused by the next tile
  }
}

// Hash-table keys of the compacted slots (kw <= 4 words per key): the host reads back only the live groups' keys.  n_dev
// (optional): the compaction's group counter -- min(*n_dev, n) keys are gathered.
__global__ void __launch_bounds__(256) pgx_gather_keys(const unsigned long long* __restrict__ keys,
                                                       const int64_t* __restrict__ slot,
                                                       const unsigned long long* __restrict__ n_dev, int64_t n, int kw,
                                                       unsigned long long* __restrict__ out) {
  if (n_dev) n = static_cast<int64_t>(*n_dev) < n ? static_cast<int64_t>(*n_dev) : n;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t s = slot[i];
    for (int w = 0; w < kw; ++w) out[i * kw + w] = keys[s * kw + w];
  }
}

// Joining the passes of a partitioned plan over several value columns (pgx_part.cpp run_value_columns): every pass
// finds the same groups (the filter and the keys are the same) in its own order.  pgx_join_build puts the first pass's
// keys in an open-addressing table (key -> index in the first pass); pgx_join_scatter looks up each group of a later
// pass and writes its sum / min / max planes into the combined planes at the first pass's index.  A key the table does
// not hold counts in *miss (cannot happen: the host fails the query if it does).
__global__ void __launch_bounds__(256) pgx_join_build(const uint64_t* __restrict__ okey, int64_t n,
                                                      unsigned long long* __restrict__ tkey,
                                                      int64_t* __restrict__ tidx, uint64_t cap) {
  const uint64_t mask = cap - 1;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const unsigned long long k = okey[i];
    uint64_t h = merge_mix(k) & mask;
    for (uint64_t probe = 0; probe < cap; ++probe) {
      if (atomicCAS(tkey + h, kMergeEmpty, k) == kMergeEmpty) {  // keys are distinct: a free slot, never our key
        tidx[h] = i;
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

__global__ void __launch_bounds__(256) pgx_join_scatter(const uint64_t* __restrict__ okey,
                                                        const uint64_t* __restrict__ opl, int64_t ocap, int64_t n,
                                                        const unsigned long long* __restrict__ tkey,
                                                        const int64_t* __restrict__ tidx, uint64_t cap,
                                                        uint64_t* __restrict__ comb, int64_t ccap, int base,
                                                        unsigned long long* __restrict__ miss) {
  const uint64_t mask = cap - 1;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const unsigned long long k = okey[i];
    uint64_t h = merge_mix(k) & mask;
    int64_t j = -1;
    for (uint64_t probe = 0; probe < cap; ++probe) {
      const unsigned long long t = tkey[h];
      if (t == k) {
        j = tidx[h];
        break;
      }
      if (t == kMergeEmpty) break;
      h = (h + 1) & mask;
    }
    if (j < 0) {
      atomicAdd(miss, 1ull);
      continue;
    }
    for (int p = 0; p < 3; ++p) comb[(base + p) * ccap + j] = opl[(1 + p) * ocap + i];  // sum, min, max
  }
}

// Columnar groups (okey, oplane[p * ocap + i]) -> records of 1 + nplanes words (key, then the planes) for an exchange.
__global__ void __launch_bounds__(256) pgx_group_pack(const uint64_t* __restrict__ okey,
                                                      const uint64_t* __restrict__ opl, int64_t ocap, int64_t n,
                                                      int nplanes, uint64_t* __restrict__ rec) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    uint64_t* r = rec + (1 + nplanes) * i;
    r[0] = okey[i];
    for (int p = 0; p < nplanes; ++p) r[1 + p] = opl[p * ocap + i];
  }
}

}  // namespace pgx

extern "C" hipError_t pgx_launch_dense_reduce(unsigned long long* dst, const unsigned long long* src, uint64_t slots,
                                              int nplanes, uint64_t ops, hipStream_t stream) {
  const uint64_t n = slots * static_cast<uint64_t>(nplanes);
  if (n == 0) return hipSuccess;
  if (nplanes > 32) return hipErrorInvalidValue;
  const unsigned grid = static_cast<unsigned>(n / 256 + 1 < 16384 ? n / 256 + 1 : 16384);
  hipLaunchKernelGGL(pgx::pgx_dense_reduce, dim3(grid), dim3(256), 0, stream, dst, src, slots, nplanes, ops);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_gather_keys(const unsigned long long* keys, const int64_t* slot,
                                             const unsigned long long* n_dev, int64_t n, int kw, unsigned long long* out,
                                             hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (kw < 1 || kw > 4) return hipErrorInvalidValue;
  const unsigned grid = static_cast<unsigned>(n / 256 + 1 < 16384 ? n / 256 + 1 : 16384);
  hipLaunchKernelGGL(pgx::pgx_gather_keys, dim3(grid), dim3(256), 0, stream, keys, slot, n_dev, n, kw, out);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_join(const uint64_t* okey0, int64_t n0, const uint64_t* okey, const uint64_t* opl,
                                      int64_t ocap, int64_t n, unsigned long long* tkey, int64_t* tidx, uint64_t cap,
                                      uint64_t* comb, int64_t ccap, int base, unsigned long long* miss,
                                      hipStream_t stream) {
  // okey0 != null: build the table from the first pass's n0 keys; else scatter a later pass's n groups
  if (cap == 0 || (cap & (cap - 1)) != 0 || !tkey || !tidx) return hipErrorInvalidValue;
  if (okey0) {
    if (n0 <= 0) return hipSuccess;
    const unsigned grid = static_cast<unsigned>(n0 / 256 + 1 < 16384 ? n0 / 256 + 1 : 16384);
    hipLaunchKernelGGL(pgx::pgx_join_build, dim3(grid), dim3(256), 0, stream, okey0, n0, tkey, tidx, cap);
    return hipGetLastError();
  }
  if (n <= 0) return hipSuccess;
  if (!okey || !opl || !comb || !miss || base < 1) return hipErrorInvalidValue;
  const unsigned grid = static_cast<unsigned>(n / 256 + 1 < 16384 ? n / 256 + 1 : 16384);
  hipLaunchKernelGGL(pgx::pgx_join_scatter, dim3(grid), dim3(256), 0, stream, okey, opl, ocap, n, tkey, tidx, cap, comb,
                     ccap, base, miss);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_group_merge(const uint64_t* key, const uint64_t* pl, int64_t es, int64_t ps,
                                             int64_t n, unsigned long long* tkey, unsigned long long* tpl,
                                             uint64_t cap, int nplanes, uint64_t ops, unsigned long long* overflow,
                                             hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (cap == 0 || (cap & (cap - 1)) != 0 || nplanes < 1 || nplanes > 32) return hipErrorInvalidValue;
  const int64_t g = (n + 255) / 256;
  hipLaunchKernelGGL(pgx::pgx_group_merge, dim3(static_cast<unsigned>(g < 65536 ? g : 65536)), dim3(256), 0, stream,
                     key, pl, es, ps, n, tkey, tpl, cap, nplanes, ops, overflow);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_group_pack(const uint64_t* okey, const uint64_t* opl, int64_t ocap, int64_t n,
                                            int nplanes, uint64_t* rec, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (nplanes < 1 || nplanes > 32) return hipErrorInvalidValue;
  const int64_t g = (n + 255) / 256;
  hipLaunchKernelGGL(pgx::pgx_group_pack, dim3(static_cast<unsigned>(g < 65536 ? g : 65536)), dim3(256), 0, stream,
                     okey, opl, ocap, n, nplanes, rec);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_group_compact(const unsigned long long* tkey, const unsigned long long* tpl,
                                               uint64_t cap, int nplanes, uint64_t* okey, uint64_t* opl, int64_t ocap,
                                               unsigned long long* counter, hipStream_t stream) {
  if (cap == 0) return hipSuccess;
  if (nplanes < 1 || nplanes > 32) return hipErrorInvalidValue;
  const uint64_t g = (cap + 4095) / 4096;
  hipLaunchKernelGGL(pgx::pgx_group_compact, dim3(static_cast<unsigned>(g < 4096 ? g : 4096)), dim3(256), 0, stream,
                     tkey, tpl, cap, nplanes, okey, opl, ocap, counter);
  return hipGetLastError();
}
