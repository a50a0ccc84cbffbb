// MI355X (gfx950) kernels of the pinot-core segment query hot path.
//
// One fused kernel (pgx_scan_kernel) replaces the reference's per-doc Java loops for a whole query:
//   a-1  fixed-bit forward-index decode     (util/PinotDataCustomBitSet.java:122-155)        -> decode32<B>
//   a-6  scan predicates                    (operator/dociditerators/SVScanDocIdIterator.java) -> leaf words
//   a-8  sorted-index ranges                (operator/filter/SortedInvertedIndexBasedFilterOperator.java) -> leaf words
//   a-9/a-10 AND / OR doc-set algebra       (operator/docidsets/{And,Or}BlockDocIdSet.java)    -> bitwise ops on words
//   a-12 doc-id compaction into blocks      (operator/BReusableFilteredDocIdSetOperator.java)  -> 32-row mask words
//   a-13/a-3 projection + dictionary decode (operator/aggregation/DataBlockCache.java, Dictionary.readDoubleValues)
//   a-14 aggregation                        (operator/aggregation/DefaultAggregationExecutor.java)
//   a-15..a-17 group-by                     (operator/aggregation/groupby/DefaultGroupByExecutor.java,
//                                            DefaultGroupKeyGenerator.java, DoubleGroupByResultHolder.java)
//   a-19 combine over segments              (operator/MCombine*Operator.java): every segment accumulates into the
//                                            same query-wide accumulators (global key ids), so the combine is free.
//
// Execution model: a workgroup (256 lanes = 4 waves) owns a TILE of 8192 consecutive rows of one segment; lane l owns
// rows [32l, 32l+32) of the tile, i.e. exactly one 32-bit doc mask word and exactly B dwords of a B-bit forward index
// (32*B bits), so no value straddles two lanes and every lane decodes from its own registers.  Workgroups walk a
// contiguous range of tiles (persistent grid) so per-workgroup accumulators (registers / LDS tables) are flushed once.
// The whole path is HBM-bound integer work: no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "pgx_internal.h"

namespace pgx {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------------------------
// K1: fixed-bit unpack.  The lane's 32 rows occupy B dwords starting at dword (row0/32)*B of the (big-endian,
// MSB-first) forward index.  Loads are as wide as the lane chunk's alignment allows.
// ---------------------------------------------------------------------------------------------
template <int B>
__device__ __forceinline__ void decode32(const uint32_t* __restrict__ p, uint32_t (&v)[32]) {
  uint32_t w[B + 1];
  if constexpr (B % 4 == 0) {
#pragma unroll
    for (int i = 0; i < B / 4; ++i) {
      u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + i);
      w[4 * i] = q.x; w[4 * i + 1] = q.y; w[4 * i + 2] = q.z; w[4 * i + 3] = q.w;
    }
  } else if constexpr (B % 2 == 0) {
#pragma unroll
    for (int i = 0; i < B / 2; ++i) {
      u32x2 q = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p) + i);
      w[2 * i] = q.x; w[2 * i + 1] = q.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < B; ++i) w[i] = __builtin_nontemporal_load(p + i);
  }
  w[B] = 0;
#pragma unroll
  for (int i = 0; i < B; ++i) w[i] = bswap32(w[i]);
  constexpr uint32_t MASK = (B == 32) ? 0xFFFFFFFFu : ((1u << (B & 31)) - 1u);
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int o = j * B;
    const int k = o >> 5;
    const int s = o & 31;
    if (s + B <= 32) {
      v[j] = (w[k] >> (32 - s - B)) & MASK;
    } else {
      const uint64_t win = (static_cast<uint64_t>(w[k]) << 32) | w[k + 1];
      v[j] = static_cast<uint32_t>(win >> (64 - s - B)) & MASK;
    }
  }
}

#define PGX_DECODE_CASES(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
  X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)

__device__ __forceinline__ void decode_dyn(int bits, const uint32_t* __restrict__ fwd, int64_t lane_chunk,
                                           uint32_t (&v)[32]) {
  const uint32_t* p = fwd + lane_chunk * bits;
  switch (bits) {
#define PGX_CASE(b) \
  case b:           \
    decode32<b>(p, v); \
    break;
    PGX_DECODE_CASES(PGX_CASE)
#undef PGX_CASE
    default:
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = 0;
  }
}

// ---------------------------------------------------------------------------------------------
// Accumulator encodings
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long ord_i64(int64_t x) {
  return static_cast<unsigned long long>(x) ^ 0x8000000000000000ull;
}
__device__ __forceinline__ unsigned long long ord_f64(double d) {
  unsigned long long b = __double_as_longlong(d);
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

// ---------------------------------------------------------------------------------------------
// Filter leaves
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ranges_word(const KLeaf& L, int32_t row0) {
  // Sorted-index doc ranges (inclusive, ascending, disjoint) -> this lane's 32-doc word.
  const int32_t* r = L.ranges;
  int lo = 0, hi = L.nranges;  // first range with end >= row0
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (r[2 * mid + 1] < row0) lo = mid + 1; else hi = mid;
  }
  uint32_t word = 0;
  const int32_t last = row0 + 31;
  for (int i = lo; i < L.nranges; ++i) {
    int32_t a = r[2 * i], b = r[2 * i + 1];
    if (a > last) break;
    int s = max(a, row0) - row0, e = min(b, last) - row0;
    uint32_t m = (e - s == 31) ? 0xFFFFFFFFu : (((1u << (e - s + 1)) - 1u) << s);
    word |= m;
  }
  return word;
}

__device__ __forceinline__ uint32_t leaf_word(const KSeg& S, const KQuery& Q, int leaf, int32_t row0,
                                              int64_t lane_chunk) {
  const KLeaf& L = S.leaf[leaf];
  if (L.mode == LEAF_NONE) return 0u;
  if (L.mode == LEAF_RANGES) return ranges_word(L, row0);
  const int c = Q.leaf_col[leaf];
  uint32_t v[32];
  decode_dyn(S.bits[c], S.fwd[c], lane_chunk, v);
  uint32_t word = 0;
  if (L.mode == LEAF_SCAN_INTERVAL) {
    const uint32_t lo = static_cast<uint32_t>(L.lo);
    const uint32_t span = static_cast<uint32_t>(L.hi - L.lo);
#pragma unroll
    for (int j = 0; j < 32; ++j) word |= static_cast<uint32_t>((v[j] - lo) <= span) << j;
  } else {
    const uint32_t* bs = L.bitset;
#pragma unroll
    for (int j = 0; j < 32; ++j) word |= ((bs[v[j] >> 5] >> (v[j] & 31)) & 1u) << j;
  }
  return word;
}

// Stack machine over 32-bit doc words, registers only (no runtime-indexed arrays -> no scratch).
struct WordStack {
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0, s7 = 0;
  __device__ __forceinline__ void push(uint32_t x) {
    s7 = s6; s6 = s5; s5 = s4; s4 = s3; s3 = s2; s2 = s1; s1 = s0; s0 = x;
  }
  __device__ __forceinline__ void fold(bool is_and) {
    s0 = is_and ? (s0 & s1) : (s0 | s1);
    s1 = s2; s2 = s3; s3 = s4; s4 = s5; s5 = s6; s6 = s7; s7 = 0;
  }
};

__device__ __forceinline__ uint32_t run_filter(const KSeg& S, const KQuery& Q, int32_t row0, int64_t lane_chunk,
                                               uint32_t valid, unsigned long long& entries) {
  if (Q.prog_len == 0) return valid;
  WordStack st;
  for (int pc = 0; pc < Q.prog_len; ++pc) {
    const int op = Q.prog_op[pc];
    const int arg = Q.prog_arg[pc];
    if (op == OP_LEAF) {
      const uint32_t w = leaf_word(S, Q, arg, row0, lane_chunk) & valid;
      if (S.lmask) S.lmask[arg * S.lmask_words + lane_chunk] = w;  // statistics automaton input
      st.push(w);
    } else if (op == OP_AND) {
      for (int k = 1; k < arg; ++k) st.fold(true);
    } else if (op == OP_OR) {
      for (int k = 1; k < arg; ++k) st.fold(false);
    } else if (op == OP_STAT) {
      entries += __popc(st.s0);
    } else if (op == OP_TRUE) {
      st.push(valid);
    }
  }
  return st.s0 & valid;
}

// ---------------------------------------------------------------------------------------------
// Hash table (LONG_MAP / ARRAY_MAP group keys): open addressing, linear probing.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

// Probe chains are bounded (kGlobalMaxProbes): at the load factors the host plans (<= 1/2) a longer chain means the
// table is (nearly) full, so the lane reports overflow at once and the host regrows the table and reruns, instead of
// walking the whole table with one device atomic per slot.
constexpr uint64_t kGlobalMaxProbes = 64;

__device__ __forceinline__ int64_t hash_slot64(const KQuery& Q, uint64_t key) {
  const uint64_t mask = Q.hash_cap - 1;
  const uint64_t lim = Q.hash_cap < kGlobalMaxProbes ? Q.hash_cap : kGlobalMaxProbes;
  uint64_t h = mix64(key) & mask;
  for (uint64_t probe = 0; probe < lim; ++probe) {
    unsigned long long prev = atomicCAS(Q.keys + h, kEmptyKey, static_cast<unsigned long long>(key));
    if (prev == kEmptyKey || prev == key) return static_cast<int64_t>(h);
    h = (h + 1) & mask;
  }
  return -1;
}

__device__ __forceinline__ int64_t hash_slot128(const KQuery& Q, uint64_t klo, uint64_t khi) {
  const uint64_t mask = Q.hash_cap - 1;
  const uint64_t lim = Q.hash_cap < kGlobalMaxProbes ? Q.hash_cap : kGlobalMaxProbes;
  uint64_t h = mix64(klo ^ mix64(khi)) & mask;
  uint64_t probes = 0;
  // Every loop iteration makes progress for every lane (no divergent spin on another lane's write).
  while (probes < lim) {
    unsigned int st = atomicCAS(Q.key_state + h, 0u, 1u);
    if (st == 0u) {
      __hip_atomic_store(Q.keys + 2 * h, klo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(Q.keys + 2 * h + 1, khi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
      atomicExch(Q.key_state + h, 2u);
      return static_cast<int64_t>(h);
    }
    if (st == 2u) {
      unsigned long long a = __hip_atomic_load(Q.keys + 2 * h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned long long b = __hip_atomic_load(Q.keys + 2 * h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a == klo && b == khi) return static_cast<int64_t>(h);
      h = (h + 1) & mask;
      ++probes;
    }
    // st == 1: another lane is publishing this slot; re-read next iteration.
  }
  return -1;
}

// Keys of W 64-bit words (G_HASHW, ARRAY_MAP keys over 126 bits): the 128-bit protocol with W words per slot.
template <int W>
__device__ __forceinline__ int64_t hash_slotw(const KQuery& Q, const uint64_t (&k)[W]) {
  const uint64_t mask = Q.hash_cap - 1;
  const uint64_t lim = Q.hash_cap < kGlobalMaxProbes ? Q.hash_cap : kGlobalMaxProbes;
  uint64_t hv = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) hv = mix64(hv ^ k[w]);
  uint64_t h = hv & mask;
  uint64_t probes = 0;
  while (probes < lim) {
    unsigned int st = atomicCAS(Q.key_state + h, 0u, 1u);
    if (st == 0u) {
#pragma unroll
      for (int w = 0; w < W; ++w)
        __hip_atomic_store(Q.keys + W * h + w, k[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
      atomicExch(Q.key_state + h, 2u);
      return static_cast<int64_t>(h);
    }
    if (st == 2u) {
      bool same = true;
#pragma unroll
      for (int w = 0; w < W; ++w)
        same = same && __hip_atomic_load(Q.keys + W * h + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k[w];
      if (same) return static_cast<int64_t>(h);
      h = (h + 1) & mask;
      ++probes;
    }
  }
  return -1;
}

// ---------------------------------------------------------------------------------------------
// Plane updates (LDS or global; the pointer's address space is known at each call site)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void plane_update_global(unsigned long long* p, int op, unsigned long long enc) {
  switch (op) {
    case P_ADD_I64: atomicAdd(p, enc); break;
    case P_ADD_F64: atomicAdd(reinterpret_cast<double*>(p), __longlong_as_double(static_cast<long long>(enc))); break;
    case P_MIN_ORD: atomicMin(p, enc); break;
    case P_MAX_ORD: atomicMax(p, enc); break;
  }
}

__device__ __forceinline__ unsigned long long value_enc(const void* dict, bool fp, int kind, uint32_t id) {
  if (fp) {
    const double d = static_cast<const double*>(dict)[id];
    if (kind == A_MIN || kind == A_MAX) return ord_f64(d);
    return static_cast<unsigned long long>(__double_as_longlong(d));
  }
  const int64_t x = static_cast<const int64_t*>(dict)[id];
  if (kind == A_MIN || kind == A_MAX) return ord_i64(x);
  return static_cast<unsigned long long>(x);
}

__device__ __forceinline__ unsigned long long combine_enc(int op, unsigned long long x, unsigned long long y) {
  if (op == P_ADD_I64) return x + y;
  if (op == P_ADD_F64)
    return static_cast<unsigned long long>(__double_as_longlong(__longlong_as_double(static_cast<long long>(x)) +
                                                                __longlong_as_double(static_cast<long long>(y))));
  if (op == P_MIN_ORD) return x < y ? x : y;
  return x > y ? x : y;
}

__device__ __forceinline__ unsigned long long wave_reduce(int op, unsigned long long x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x = combine_enc(op, x, __shfl_xor(x, off));
  return x;
}

__device__ __forceinline__ unsigned long long plane_identity(int op) { return op == P_MIN_ORD ? ~0ull : 0ull; }

// ---------------------------------------------------------------------------------------------
// The fused scan kernel.  GM selects the group-by storage at compile time:
//   G_NONE aggregation-only | G_DENSE_LDS | G_DENSE_GLOBAL | G_HASH64 | G_HASH128
// ---------------------------------------------------------------------------------------------
template <int GM>
__global__ void __launch_bounds__(kBlock) pgx_scan_kernel(const KQuery Q, int64_t tiles_per_wg) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_table[];
  __shared__ unsigned long long s_acc[kMaxAggs + 1];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int64_t t_begin = static_cast<int64_t>(blockIdx.x) * tiles_per_wg;
  const int64_t t_end = min(t_begin + tiles_per_wg, Q.total_tiles);
  if (t_begin >= t_end) return;

  if (tid <= kMaxAggs) s_acc[tid] = (tid >= 1 && tid <= Q.num_aggs) ? plane_identity(Q.plane_op[tid]) : 0ull;
  if constexpr (GM == G_DENSE_LDS) {
    const uint64_t n = Q.dense_slots * Q.num_planes;
    for (uint64_t i = tid; i < n; i += kBlock)
      lds_table[i] = plane_identity(Q.plane_op[static_cast<int>(i / Q.dense_slots)]);
  }
  __syncthreads();

  unsigned long long entries = 0;
  unsigned long long docs = 0;

  // Locate the first tile's segment (binary search, wave-uniform), then walk forward.
  int seg;
  {
    int lo = 0, hi = Q.num_segs - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (Q.segs[mid].tile_begin <= t_begin) lo = mid; else hi = mid - 1;
    }
    seg = lo;
  }

  for (int64_t t = t_begin; t < t_end; ++t) {
    while (seg + 1 < Q.num_segs && Q.segs[seg + 1].tile_begin <= t) ++seg;
    const KSeg& S = Q.segs[seg];
    const int64_t local_tile = t - S.tile_begin;
    const int32_t row0 = static_cast<int32_t>(local_tile * kTileRows + tid * kLaneRows);
    const int64_t lane_chunk = local_tile * kBlock + tid;  // lane chunk index within the segment
    uint32_t valid;
    if (row0 >= S.num_docs) valid = 0u;
    else if (row0 + 32 <= S.num_docs) valid = 0xFFFFFFFFu;
    else valid = (1u << (S.num_docs - row0)) - 1u;

    uint32_t mask = 0;
    if (valid) mask = run_filter(S, Q, row0, lane_chunk, valid, entries);
    docs += __popc(mask);

    if constexpr (GM == G_NONE) {
      // ---- aggregation-only (a-14) ----
      for (int a = 0; a < Q.num_aggs; ++a) {
        const int kind = Q.agg_kind[a];
        if (kind == A_COUNT) continue;
        const int op = Q.plane_op[a + 1];
        unsigned long long x = plane_identity(op);
        if (mask) {
          const int c = Q.agg_col[a];
          uint32_t v[32];
          decode_dyn(S.bits[c], S.fwd[c], lane_chunk, v);
          const bool fp = Q.agg_fp[a];
          if (kind == A_MIN || kind == A_MAX) {
            // Dictionaries are sorted ascending (SegmentDictionaryCreator.build), so the extreme value is the value
            // of the extreme dictId: one dictionary read per lane per tile instead of one per row.
            uint32_t best = (kind == A_MIN) ? 0xFFFFFFFFu : 0u;
#pragma unroll
            for (int j = 0; j < 32; ++j)
              if ((mask >> j) & 1u) best = (kind == A_MIN) ? min(best, v[j]) : max(best, v[j]);
            x = value_enc(S.dict[c], fp, kind, best);
          } else if (fp) {
            const double* d = static_cast<const double*>(S.dict[c]);
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < 32; ++j)
              if ((mask >> j) & 1u) s += d[v[j]];
            x = static_cast<unsigned long long>(__double_as_longlong(s));
          } else {
            const int64_t* d = static_cast<const int64_t*>(S.dict[c]);
            int64_t s = 0;
#pragma unroll
            for (int j = 0; j < 32; ++j)
              if ((mask >> j) & 1u) s += d[v[j]];
            x = static_cast<unsigned long long>(s);
          }
        }
        x = wave_reduce(op, x);
        if (lane == 0) {
          if (op == P_ADD_I64) atomicAdd(&s_acc[a + 1], x);
          else if (op == P_ADD_F64) atomicAdd(reinterpret_cast<double*>(&s_acc[a + 1]),
                                              __longlong_as_double(static_cast<long long>(x)));
          else if (op == P_MIN_ORD) atomicMin(&s_acc[a + 1], x);
          else atomicMax(&s_acc[a + 1], x);
        }
      }
    } else {
      // ---- group-by (a-15..a-17) ----
      if (!mask) continue;
      using KeyT = typename std::conditional<(GM == G_DENSE_LDS || GM == G_DENSE_GLOBAL), uint32_t, uint64_t>::type;
      KeyT klo[32];
      uint64_t khi[(GM == G_HASH128) ? 32 : 1];
#pragma unroll
      for (int j = 0; j < 32; ++j) klo[j] = 0;
      if constexpr (GM == G_HASH128) {
#pragma unroll
        for (int j = 0; j < 32; ++j) khi[j] = 0;
      }
      for (int g = 0; g < (GM == G_HASHW ? 0 : Q.num_gcols); ++g) {
        const int c = Q.gcol[g];
        uint32_t v[32];
        decode_dyn(S.bits[c], S.fwd[c], lane_chunk, v);
        const int32_t* rm = S.remap[c];
        if (rm) {
#pragma unroll
          for (int j = 0; j < 32; ++j)
            if ((mask >> j) & 1u) v[j] = static_cast<uint32_t>(rm[v[j]]);
        }
        if constexpr (GM == G_DENSE_LDS || GM == G_DENSE_GLOBAL) {
          const uint32_t mul = static_cast<uint32_t>(Q.gmul[g]);
#pragma unroll
          for (int j = 0; j < 32; ++j) klo[j] += v[j] * mul;
        } else {
          const int sh = Q.gshift[g];
          if (GM == G_HASH128 && Q.ghi[g]) {
#pragma unroll
            for (int j = 0; j < 32; ++j) khi[(GM == G_HASH128) ? j : 0] |= static_cast<uint64_t>(v[j]) << sh;
          } else {
#pragma unroll
            for (int j = 0; j < 32; ++j) klo[j] |= static_cast<uint64_t>(v[j]) << sh;
          }
        }
      }
      // Resolve hash slots in place (klo becomes the slot index).
      uint32_t live = mask;
      if constexpr (GM == G_HASHW) {
        // keys of 3-4 words: 8 rows at a time (their words in registers), each column decoded once per chunk
        for (int j0 = 0; j0 < 32; j0 += 8) {
          if (!((mask >> j0) & 0xFFu)) continue;
          uint64_t kw[8][kMaxKeyWords];
#pragma unroll
          for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int w = 0; w < kMaxKeyWords; ++w) kw[r][w] = 0;
          for (int g = 0; g < Q.num_gcols; ++g) {
            const int c = Q.gcol[g];
            uint32_t v[32];
            decode_dyn(S.bits[c], S.fwd[c], lane_chunk, v);
            const int32_t* rm = S.remap[c];
            const int sh = Q.gshift[g], wd = Q.ghi[g];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              uint32_t x = v[j0 + r];
              if (rm && ((mask >> (j0 + r)) & 1u)) x = static_cast<uint32_t>(rm[x]);
#pragma unroll
              for (int w = 0; w < kMaxKeyWords; ++w)
                if (w == wd) kw[r][w] |= static_cast<uint64_t>(x) << sh;
            }
          }
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int j = j0 + r;
            if (!((mask >> j) & 1u)) continue;
            int64_t sl;
            if (Q.key_words == 3) {
              const uint64_t k3[3] = {kw[r][0], kw[r][1], kw[r][2]};
              sl = hash_slotw<3>(Q, k3);
            } else {
              const uint64_t k4[4] = {kw[r][0], kw[r][1], kw[r][2], kw[r][3]};
              sl = hash_slotw<4>(Q, k4);
            }
            if (sl < 0) live &= ~(1u << j);
            klo[j] = static_cast<uint64_t>(sl);
          }
        }
        if (live != mask) atomicAdd(Q.overflow, static_cast<unsigned long long>(__popc(mask & ~live)));
      }
      if constexpr (GM == G_HASH64 || GM == G_HASH128) {
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          if ((mask >> j) & 1u) {
            int64_t s;
            if constexpr (GM == G_HASH64) s = hash_slot64(Q, klo[j]);
            else s = hash_slot128(Q, klo[j], khi[j]);
            if (s < 0) live &= ~(1u << j);
            klo[j] = static_cast<uint64_t>(s);
          }
        }
        if (live != mask) atomicAdd(Q.overflow, static_cast<unsigned long long>(__popc(mask & ~live)));
      }
      const uint64_t stride = (GM == G_DENSE_LDS || GM == G_DENSE_GLOBAL) ? Q.dense_slots : Q.hash_cap;  // (HASHW too)
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if ((live >> j) & 1u) {
          if constexpr (GM == G_DENSE_LDS) atomicAdd(&lds_table[klo[j]], 1ull);
          else atomicAdd(&Q.table[klo[j]], 1ull);
        }
      for (int a = 0; a < Q.num_aggs; ++a) {
        const int kind = Q.agg_kind[a];
        if (kind == A_COUNT) continue;
        const int c = Q.agg_col[a];
        uint32_t v[32];
        decode_dyn(S.bits[c], S.fwd[c], lane_chunk, v);
        const bool fp = Q.agg_fp[a];
        const int op = Q.plane_op[a + 1];
        const uint64_t pbase = static_cast<uint64_t>(a + 1) * stride;
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if ((live >> j) & 1u) {
            const unsigned long long e = value_enc(S.dict[c], fp, kind, v[j]);
            if constexpr (GM == G_DENSE_LDS) {
              unsigned long long* p = &lds_table[pbase + klo[j]];
              if (op == P_ADD_I64) atomicAdd(p, e);
              else if (op == P_ADD_F64) atomicAdd(reinterpret_cast<double*>(p), __longlong_as_double(static_cast<long long>(e)));
              else if (op == P_MIN_ORD) atomicMin(p, e);
              else atomicMax(p, e);
            } else {
              plane_update_global(&Q.table[pbase + klo[j]], op, e);
            }
          }
      }
    }
  }

  // ---- flush: statistics, aggregation-only accumulators, LDS group table ----
  unsigned long long d = wave_reduce(P_ADD_I64, docs);
  unsigned long long e = wave_reduce(P_ADD_I64, entries);
  if (lane == 0) {
    if (d) atomicAdd(Q.stats + 0, d);
    if (e) atomicAdd(Q.stats + 1, e);
    if (GM == G_NONE && d) atomicAdd(&s_acc[0], d);
  }
  __syncthreads();
  if constexpr (GM == G_NONE) {
    if (tid < Q.num_planes) {
      const int op = (tid == 0) ? P_ADD_I64 : Q.plane_op[tid];
      if (tid == 0 || Q.agg_kind[tid - 1] != A_COUNT) plane_update_global(Q.agg_out + tid, op, s_acc[tid]);
    }
  }
  if constexpr (GM == G_DENSE_LDS) {
    const uint64_t n = Q.dense_slots * Q.num_planes;
    for (uint64_t i = tid; i < n; i += kBlock) {
      const uint64_t plane = i / Q.dense_slots;
      const uint64_t s = i - plane * Q.dense_slots;
      if (lds_table[s] == 0) continue;  // slot untouched by this workgroup
      plane_update_global(Q.table + i, Q.plane_op[plane], lds_table[i]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Table initialisation and compaction
// ---------------------------------------------------------------------------------------------
__global__ void pgx_init_planes(unsigned long long* table, uint64_t slots, int num_planes, const KQuery Q,
                               unsigned long long* keys, uint64_t key_words, unsigned int* key_state) {
  const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, step = (uint64_t)gridDim.x * blockDim.x;
  for (int p = 0; p < num_planes; ++p) {  // one plane at a time: no division per element
    const unsigned long long v = (Q.plane_op[p] == P_MIN_ORD) ? ~0ull : 0ull;
    unsigned long long* t = table + (uint64_t)p * slots;
    for (uint64_t i = t0; i < slots; i += step) t[i] = v;
  }
  for (uint64_t i = t0; i < key_words; i += step) keys[i] = kEmptyKey;
  if (key_state)
    for (uint64_t i = t0; i < slots; i += step) key_state[i] = 0u;
}

// Exclusive prefix of `mine` over the workgroup's 256 threads and ONE device atomic per call: *base = the counter's
// old value (visible to every thread after the call).  Every thread of the workgroup must call it.
__device__ __forceinline__ unsigned int block_reserve(unsigned int* scan, unsigned long long* base, unsigned int mine,
                                                     unsigned long long* counter) {
  const int tid = threadIdx.x;
  scan[tid] = mine;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // Hillis-Steele inclusive scan
    const unsigned int y = tid >= d ? scan[tid - d] : 0u;
    __syncthreads();
    scan[tid] += y;
    __syncthreads();
  }
  if (tid == 255) *base = scan[255] ? atomicAdd(counter, static_cast<unsigned long long>(scan[255])) : 0ull;
  __syncthreads();
  return scan[tid] - mine;
}

// Emit occupied slots: out_slot[i] = slot index, out_planes[p*cap_out + i] = plane value.
// Small tables (dense key spaces, <= 2^20 slots): one counter reservation per wavefront, lanes in slot order.
// reset: every occupied slot is put back to its planes' initial values (ordered-min planes, bit p of min_mask: ~0; the
// others 0) once read, so the next execution of a kept plan finds the table clean (no pgx_init_planes).
__global__ void pgx_compact_wave(unsigned long long* table, uint64_t slots, int num_planes,
                                 unsigned long long* counter, int64_t* out_slot, unsigned long long* out_planes,
                                 uint64_t cap_out, int reset, uint32_t min_mask) {
  const int lane = threadIdx.x & 63;
  for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + (threadIdx.x & ~63u); b < slots;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = b + lane;
    const bool live = s < slots && table[s] != 0;
    const unsigned long long m = __ballot(live);
    if (!m) continue;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(counter, static_cast<unsigned long long>(__popcll(m)));
    const unsigned long long i = __shfl(base, 0, 64) + __popcll(m & ((1ull << lane) - 1ull));
    if (!live) continue;
    if (i < cap_out) {
      out_slot[i] = static_cast<int64_t>(s);
      for (int p = 0; p < num_planes; ++p) out_planes[p * cap_out + i] = table[p * slots + s];
    }
    if (reset)
      for (int p = 0; p < num_planes; ++p) table[p * slots + s] = ((min_mask >> p) & 1u) ? ~0ull : 0ull;
  }
}

// Large tables (hash tables, up to 2^27 slots): one counter reservation per workgroup tile of 256 x 16 slots (block_reserve): a device atomic per occupied slot
// serialises on the counter (16.7M groups ~ 24 ms), and even one per wavefront costs ~11 ns each at one L2 address.
__global__ void __launch_bounds__(256) pgx_compact(const unsigned long long* table, uint64_t slots, int num_planes,
                                                   unsigned long long* counter, int64_t* out_slot,
                                                   unsigned long long* out_planes, uint64_t cap_out) {
  __shared__ unsigned int scan[256];
  __shared__ unsigned long long base;
  constexpr int K = 16;
  for (uint64_t t0 = blockIdx.x * (uint64_t)(256 * K); t0 < slots; t0 += (uint64_t)gridDim.x * 256 * K) {
    unsigned int live = 0, mine = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t s = t0 + k * 256 + threadIdx.x;
      const bool l = s < slots && table[s] != 0;
      live |= (l ? 1u : 0u) << k;
      mine += l;
    }
    const unsigned int excl = block_reserve(scan, &base, mine, counter);
    unsigned long long i = base + excl;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (!((live >> k) & 1u)) continue;
      const uint64_t s = t0 + k * 256 + threadIdx.x;
      if (i < cap_out) {
        out_slot[i] = static_cast<int64_t>(s);
        for (int p = 0; p < num_planes; ++p) out_planes[p * cap_out + i] = table[p * slots + s];
      }
      ++i;
    }
    __syncthreads();  // base / scan are reused by the next tile
  }
}


// ---------------------------------------------------------------------------------------------
// a-7: bitmap inverted-index leaves.  The reference ORs the RoaringBitmap of every matching dictId
// (operator/filter/BitmapBasedFilterOperator.java:62-92, segment/index/readers/BitmapInvertedIndexReader.java:91-117;
// RoaringBitmap 0.5.10 portable format without run containers: cookie 12346, container count, (key, card-1) u16
// pairs, u32 offsets, then array (<= 4096 u16) or bitmap (1024 u64) containers).  One workgroup expands one
// 65536-doc chunk of one (segment, leaf): each lane binary-searches one bitmap's container keys for the chunk, then
// the workgroup ORs the found containers into an 8 KiB LDS mask (array containers bit by bit with LDS atomics, bitmap
// containers word by word) and writes the 2048 mask words to HBM with coalesced stores.  Roaring bytes are only
// 2-byte aligned inside the inverted-index file, so multi-byte fields are read as u16 pairs.
// ---------------------------------------------------------------------------------------------
#define PGX_GLOBAL __attribute__((address_space(1)))
// Global-address-space loads: flat loads would share the LDS counter with the mask atomics and serialise them.
__device__ __forceinline__ uint32_t rd16(const uint8_t* p) { return *(const PGX_GLOBAL uint16_t*)(p); }
__device__ __forceinline__ uint32_t rd32(const uint8_t* p) { return rd16(p) | (rd16(p + 2) << 16); }
// Bitmap k of a descriptor: its dictId's entry of the .bitmap.inv header (BE int offsets, 4-byte aligned) locates it.
__device__ __forceinline__ const uint8_t* rbitmap(const RDesc& D, int k) {
  const uint32_t id = D.ids[k];
  return D.inv + __builtin_bswap32(((const PGX_GLOBAL uint32_t*)(D.inv))[id]);
}

constexpr int kRoarBatch = 256;

// ORs the containers of D's bitmaps for one chunk into the LDS mask m (2048 words, zeroed by the caller).  Every
// thread of the 256-lane workgroup must call it (it synchronises).
__device__ void roar_or_chunk(const RDesc& D, int chunk, uint32_t* m, const uint8_t** cptr, int* ccard, int* cpre,
                              int* ncont, int* celems) {
  const int tid = threadIdx.x;
  for (int b0 = 0; b0 < D.nb; b0 += kRoarBatch) {
    if (tid == 0) *ncont = 0;
    __syncthreads();
    const int b = b0 + tid;
    if (b < D.nb) {
      const uint8_t* base = rbitmap(D, b);
      const int n = static_cast<int>(rd32(base + 4));
      // keys are sorted and distinct, so a bitmap with a container in every chunk holds chunk c at index c: probe
      // there first (one load for dense bitmaps), then binary-search the rest of the range
      int lo = 0, hi = n - 1, found = -1;
      const int g = min(chunk, n - 1);
      if (g >= 0) {
        const uint32_t kv = rd32(base + 8 + 4 * g);  // key | (card - 1) << 16
        const int k = static_cast<int>(kv & 0xFFFFu);
        if (k == chunk) found = g;
        else if (k < chunk) lo = g + 1;
        else hi = g - 1;
      }
      while (found < 0 && lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const int k = static_cast<int>(rd16(base + 8 + 4 * mid));
        if (k == chunk) { found = mid; break; }
        if (k < chunk) lo = mid + 1; else hi = mid - 1;
      }
      if (found >= 0) {
        const int card = static_cast<int>(rd16(base + 8 + 4 * found + 2)) + 1;
        const uint32_t off = rd32(base + 8 + 4 * n + 4 * found);
        const int slot = atomicAdd(ncont, 1);
        cptr[slot] = base + off;
        ccard[slot] = card;
      }
    }
    __syncthreads();
    const int nc = *ncont;
    // array containers: exclusive prefix of their cardinalities (wave 0, 4 entries per lane), then every lane takes
    // elements of any container with 4 loads in flight before the LDS atomics (a loop over containers would chain one
    // global-load latency per container)
    if (tid < 64) {
      int v[4], x = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = tid * 4 + j;
        v[j] = (k < nc && ccard[k] <= 4096) ? ccard[k] : 0;
        x += v[j];
      }
      int incl = x;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (tid >= d) incl += y;
      }
      int e = incl - x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cpre[tid * 4 + j] = e;
        e += v[j];
      }
      if (tid == 63) *celems = incl;
    }
    __syncthreads();
    const int ne = *celems;
    for (int e0 = 0; e0 < ne; e0 += 4 * 256) {
      uint32_t val[4];
      bool ok[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = e0 + j * 256 + tid;
        ok[j] = e < ne;
        if (ok[j]) {
          int lo = 0, hi = nc - 1;  // the last container with cpre <= e holds element e (empty parts repeat cpre)
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (cpre[mid] <= e) lo = mid; else hi = mid - 1;
          }
          val[j] = rd16(cptr[lo] + 2 * (e - cpre[lo]));
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ok[j]) atomicOr(&m[val[j] >> 5], 1u << (val[j] & 31u));
    }
    for (int k = 0; k < nc; ++k) {  // bitmap containers: 1024 x u64 LE == 2048 x u32, bit j of word w = doc 32w + j
      if (ccard[k] <= 4096) continue;
      const uint8_t* c = cptr[k];
      for (int w = tid; w < 2048; w += 256) {
        const uint32_t x = rd32(c + 4 * w);
        if (x) atomicOr(&m[w], x);
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) pgx_roaring_expand(const RDesc* __restrict__ descs, int npairs, int maxchunks) {
  const int pair = static_cast<int>(blockIdx.x / maxchunks);
  const int chunk = static_cast<int>(blockIdx.x - static_cast<unsigned>(pair) * maxchunks);
  if (pair >= npairs) return;
  const RDesc D = descs[pair];
  if (chunk >= D.nchunks) return;
  __shared__ uint32_t m[2048];
  __shared__ const uint8_t* cptr[kRoarBatch];
  __shared__ int ccard[kRoarBatch], cpre[kRoarBatch];
  __shared__ int ncont, celems;
  const int tid = threadIdx.x;
  for (int i = tid; i < 2048; i += 256) m[i] = 0u;
  roar_or_chunk(D, chunk, m, cptr, ccard, cpre, &ncont, &celems);
  uint32_t* out = D.mask + static_cast<size_t>(chunk) * 2048;
  for (int i = tid; i < 2048; i += 256) out[i] = m[i];
}

// AND / OR / NOT over bitmap leaves for one 65536-doc chunk (AndBlockDocIdSet.fastIterator's bitmap AND,
// OrBlockDocIdSet's bitmap OR, BitmapDocIdSet's exclusion flip): a stack of LDS masks, each leaf expanded with
// roar_or_chunk, the result written once.  One workgroup per (program, chunk).
constexpr int kRProgStack = 4;
__global__ void __launch_bounds__(256) pgx_roaring_program(const RProg* __restrict__ progs, const RDesc* __restrict__ descs,
                                                           int nprogs, int maxchunks) {
  const int pi = static_cast<int>(blockIdx.x / maxchunks);
  const int chunk = static_cast<int>(blockIdx.x - static_cast<unsigned>(pi) * maxchunks);
  if (pi >= nprogs) return;
  const RProg& P = progs[pi];
  if (chunk >= P.nchunks) return;
  __shared__ uint32_t stk[kRProgStack][2048];
  __shared__ const uint8_t* cptr[kRoarBatch];
  __shared__ int ccard[kRoarBatch], cpre[kRoarBatch];
  __shared__ int ncont, celems;
  const int tid = threadIdx.x;
  const int64_t doc0 = static_cast<int64_t>(chunk) << 16;
  int sp = 0;
  for (int i = 0; i < P.nops; ++i) {
    const int op = P.op[i];
    if (op == RP_LEAF) {
      uint32_t* m = stk[sp];
      for (int w = tid; w < 2048; w += 256) m[w] = 0u;
      __syncthreads();
      const int a = P.arg[i];
      if (a >= 0) roar_or_chunk(descs[a], chunk, m, cptr, ccard, cpre, &ncont, &celems);
      ++sp;
    } else if (op == RP_NOT) {
      uint32_t* m = stk[sp - 1];
      for (int w = tid; w < 2048; w += 256) {
        const int64_t d = doc0 + 32 * w;  // first doc of the word
        uint32_t keep = 0xFFFFFFFFu;       // bits inside [0, num_docs)
        if (d >= P.num_docs) keep = 0u;
        else if (d + 32 > P.num_docs) keep = (1u << (P.num_docs - d)) - 1u;
        m[w] = ~m[w] & keep;
      }
    } else {
      uint32_t* a = stk[sp - 2];
      const uint32_t* b = stk[sp - 1];
      for (int w = tid; w < 2048; w += 256) a[w] = op == RP_AND ? (a[w] & b[w]) : (a[w] | b[w]);
      --sp;
    }
    __syncthreads();
  }
  uint32_t* out = P.mask + static_cast<size_t>(chunk) * 2048;
  for (int w = tid; w < 2048; w += 256) out[w] = stk[0][w];
}

// The same program with every leaf expanded at once: one container search over ALL bitmaps of ALL leaves (a lane per
// bitmap), one pass over all their array-container elements (4 loads in flight per lane, LDS atomics into the leaf's
// own mask), the bitmap containers, then the AND / OR / NOT program evaluated per mask word in registers and written
// straight out.  The dependent global-load chain is that of ONE leaf, not one per leaf (C5: 3 leaves, 34 bitmaps), and
// the LDS holds exactly the program's leaf masks (dynamic LDS, nleaves x 8 KiB).
constexpr int kRProgMaxLeaves = 8;
__global__ void __launch_bounds__(256) pgx_roaring_program_wide(const RProg* __restrict__ progs,
                                                                const RDesc* __restrict__ descs, int nprogs,
                                                                int maxchunks) {
  const int pi = static_cast<int>(blockIdx.x / maxchunks);
  const int chunk = static_cast<int>(blockIdx.x - static_cast<unsigned>(pi) * maxchunks);
  if (pi >= nprogs) return;
  const RProg& P = progs[pi];
  if (chunk >= P.nchunks) return;
  extern __shared__ uint32_t lmask[];  // [leaf][2048]
  __shared__ const uint8_t* cptr[kRoarBatch];
  __shared__ int ccard[kRoarBatch], cpre[kRoarBatch], cleaf[kRoarBatch];
  __shared__ int ncont, celems;
  __shared__ int leaf_desc[kRProgMaxLeaves], leaf_b0[kRProgMaxLeaves + 1];
  const int tid = threadIdx.x;
  if (tid == 0) {
    int nl = 0, tot = 0;
    for (int i = 0; i < P.nops; ++i)
      if (P.op[i] == RP_LEAF) {
        const int a = P.arg[i];
        leaf_desc[nl] = a;
        leaf_b0[nl] = tot;
        tot += a >= 0 ? descs[a].nb : 0;
        ++nl;
      }
    leaf_b0[nl] = tot;
    ncont = nl;  // leaves, read below before the first batch reuses ncont
  }
  __syncthreads();
  const int nl = ncont;
  const int total_b = leaf_b0[nl];
  for (int i = tid; i < nl * 2048; i += 256) lmask[i] = 0u;
  for (int b0 = 0; b0 < total_b; b0 += kRoarBatch) {
    __syncthreads();
    if (tid == 0) ncont = 0;
    __syncthreads();
    const int b = b0 + tid;
    if (b < total_b) {
      int j = 0;
      while (leaf_b0[j + 1] <= b) ++j;  // the leaf this bitmap belongs to (<= 8 leaves)
      const RDesc& D = descs[leaf_desc[j]];
      const uint8_t* base = rbitmap(D, b - leaf_b0[j]);
      const int n = static_cast<int>(rd32(base + 4));
      int lo = 0, hi = n - 1, found = -1;
      const int g = min(chunk, n - 1);
      if (g >= 0) {
        const uint32_t kv = rd32(base + 8 + 4 * g);
        const int k = static_cast<int>(kv & 0xFFFFu);
        if (k == chunk) found = g;
        else if (k < chunk) lo = g + 1;
        else hi = g - 1;
      }
      while (found < 0 && lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const int k = static_cast<int>(rd16(base + 8 + 4 * mid));
        if (k == chunk) { found = mid; break; }
        if (k < chunk) lo = mid + 1; else hi = mid - 1;
      }
      if (found >= 0) {
        const int card = static_cast<int>(rd16(base + 8 + 4 * found + 2)) + 1;
        const uint32_t off = rd32(base + 8 + 4 * n + 4 * found);
        const int slot = atomicAdd(&ncont, 1);
        cptr[slot] = base + off;
        ccard[slot] = card;
        cleaf[slot] = j;
      }
    }
    __syncthreads();
    const int nc = ncont;
    if (tid < 64) {
      int v[4], x = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = tid * 4 + q;
        v[q] = (k < nc && ccard[k] <= 4096) ? ccard[k] : 0;
        x += v[q];
      }
      int incl = x;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (tid >= d) incl += y;
      }
      int e = incl - x;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        cpre[tid * 4 + q] = e;
        e += v[q];
      }
      if (tid == 63) celems = incl;
    }
    __syncthreads();
    const int ne = celems;
    for (int e0 = 0; e0 < ne; e0 += 4 * 256) {
      uint32_t val[4];
      int dst[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = e0 + q * 256 + tid;
        dst[q] = -1;
        if (e < ne) {
          int lo = 0, hi = nc - 1;
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (cpre[mid] <= e) lo = mid; else hi = mid - 1;
          }
          val[q] = rd16(cptr[lo] + 2 * (e - cpre[lo]));
          dst[q] = cleaf[lo] * 2048;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (dst[q] >= 0) atomicOr(&lmask[dst[q] + (val[q] >> 5)], 1u << (val[q] & 31u));
    }
    for (int k = 0; k < nc; ++k) {
      if (ccard[k] <= 4096) continue;
      const uint8_t* c = cptr[k];
      uint32_t* m = lmask + cleaf[k] * 2048;
      for (int w = tid; w < 2048; w += 256) {
        const uint32_t x = rd32(c + 4 * w);
        if (x) atomicOr(&m[w], x);
      }
    }
  }
  __syncthreads();
  // the program, per mask word, in registers
  const int64_t doc0 = static_cast<int64_t>(chunk) << 16;
  uint32_t* out = P.mask + static_cast<size_t>(chunk) * 2048;
  for (int w = tid; w < 2048; w += 256) {
    uint32_t st[kRProgStack + 4];
    int sp = 0, leaf = 0;
    const int64_t d = doc0 + 32 * w;
    const uint32_t keep = d >= P.num_docs ? 0u : (d + 32 > P.num_docs ? (1u << (P.num_docs - d)) - 1u : 0xFFFFFFFFu);
    for (int i = 0; i < P.nops; ++i) {
      const int op = P.op[i];
      if (op == RP_LEAF) {
        st[sp++] = lmask[leaf * 2048 + w];
        ++leaf;
      } else if (op == RP_NOT) {
        st[sp - 1] = ~st[sp - 1] & keep;
      } else {
        st[sp - 2] = op == RP_AND ? (st[sp - 2] & st[sp - 1]) : (st[sp - 2] | st[sp - 1]);
        --sp;
      }
    }
    out[w] = st[0];
  }
}

// One workgroup per (segment, program), walking the segment's 65536-doc chunks in order.  Every bitmap of the program
// (<= kSegRBitmaps, one lane each) keeps a cursor into its sorted container keys, and the key / cardinality / offset of
// its NEXT container are loaded while the current chunk is expanded, so a chunk costs the element and bitmap-word loads
// only (the per-chunk kernels above pay a container search of four dependent loads per chunk).  Array elements spread
// over all lanes (4 loads in flight each), bitmap-container words too; the AND / OR / NOT program is evaluated per mask
// word in registers and the chunk's mask written out.
constexpr int kSegRThreads = 512;
constexpr int kSegRBitmaps = 512;
// Workgroup barrier that orders LDS only: no s_waitcnt vmcnt(0), so global loads issued before it (next container's
// fields) and the mask stores of the previous chunk are not drained at every phase of the chunk loop.  Global memory
// is never communicated between the workgroup's threads here.
__device__ __forceinline__ void seg_lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__global__ void __launch_bounds__(kSegRThreads, 8) pgx_roaring_program_seg(const RProg* __restrict__ progs,
                                                                        const RDesc* __restrict__ descs, int nprogs,
                                                                        int parts) {
  // `parts` workgroups per segment, each walking a contiguous range of its chunks: short segment lists (a batch of a
  // long query) still put enough workgroups on the chip
  const int pi = static_cast<int>(blockIdx.x) / parts;
  if (pi >= nprogs) return;
  const RProg& P = progs[pi];
  const int per = (P.nchunks + parts - 1) / parts;
  const int c0 = (static_cast<int>(blockIdx.x) % parts) * per;
  const int c1 = min(P.nchunks, c0 + per);
  if (c0 >= c1) return;
  extern __shared__ uint32_t lmask[];  // [leaf][2048]
  __shared__ const uint8_t* cptr[kSegRBitmaps];
  __shared__ int ccard[kSegRBitmaps], cpre[kSegRBitmaps + 1], cleaf[kSegRBitmaps];
  __shared__ int ncont;
  const int tid = threadIdx.x;
  // leaves in program order (uniform loads); lane tid < total bitmaps owns bitmap (tid - first) of leaf `leaf`
  int nl = 0, tot = 0, leaf = 0, my_desc = -1, my_first = 0;
  for (int i = 0; i < P.nops; ++i)
    if (P.op[i] == RP_LEAF && nl < kRProgMaxLeaves) {
      const int a = P.arg[i];
      const int nb = a >= 0 ? descs[a].nb : 0;
      if (tid >= tot && tid < tot + nb) {
        leaf = nl;
        my_desc = a;
        my_first = tot;
      }
      tot += nb;
      ++nl;
    }
  // this lane's bitmap: header, container count and the fields of its first container (the host launches this
  // kernel only when the program's bitmaps number <= kSegRBitmaps)
  const uint8_t* base = nullptr;
  int n = 0, cur = 0, key = 1 << 30, card = 0;
  uint32_t off = 0;
  if (my_desc >= 0) {
    const RDesc& D = descs[my_desc];
    base = rbitmap(D, tid - my_first);
    n = static_cast<int>(rd32(base + 4));
    if (c0 > 0 && n > 0) {  // first container with key >= c0: keys are strictly increasing, so key[c0] == c0 settles it
      if (n > c0 && static_cast<int>(rd16(base + 8 + 4 * c0)) == c0) {
        cur = c0;
      } else {
        int lo = 0, hi = n;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (static_cast<int>(rd16(base + 8 + 4 * mid)) < c0) lo = mid + 1; else hi = mid;
        }
        cur = lo;
      }
    }
    if (cur < n) {
      key = static_cast<int>(rd16(base + 8 + 4 * cur));
      card = static_cast<int>(rd16(base + 8 + 4 * cur + 2)) + 1;
      off = rd32(base + 8 + 4 * n + 4 * cur);
    }
  }
  __shared__ int bidx[kSegRBitmaps], nbm;
  constexpr int kPer = 4;  // array elements in flight per lane (8 costs a quarter of the workgroups per CU)
  for (int chunk = c0; chunk < c1; ++chunk) {
    for (int i = tid; i < nl * 2048; i += kSegRThreads) lmask[i] = 0u;
    if (tid == 0) ncont = 0;
    // LDS-only barriers: the container-field prefetches and the previous chunk's mask stores stay in flight
    seg_lds_barrier();
    if (key == chunk) {
      const int slot = atomicAdd(&ncont, 1);
      cptr[slot] = base + off;
      ccard[slot] = card;
      cleaf[slot] = leaf;
      // advance the cursor and prefetch the next container's fields (consumed at a later chunk)
      ++cur;
      if (cur < n) {
        key = static_cast<int>(rd16(base + 8 + 4 * cur));
        card = static_cast<int>(rd16(base + 8 + 4 * cur + 2)) + 1;
        off = rd32(base + 8 + 4 * n + 4 * cur);
      } else {
        key = 1 << 30;
      }
    }
    seg_lds_barrier();
    const int nc = ncont;
    if (tid < 64) {  // exclusive prefix of the array containers' cardinalities (8 per lane); bitmap containers listed
      int v[8], x = 0, nb = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = tid * 8 + q;
        const bool in = k < nc;
        v[q] = (in && ccard[k] <= 4096) ? ccard[k] : 0;
        nb += (in && ccard[k] > 4096) ? 1 : 0;
        x += v[q];
      }
      int incl = x, binc = nb;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        const int z = __shfl_up(binc, d, 64);
        if (tid >= d) {
          incl += y;
          binc += z;
        }
      }
      int e = incl - x, b = binc - nb;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = tid * 8 + q;
        if (k < kSegRBitmaps) cpre[k] = e;
        e += v[q];
        if (k < nc && ccard[k] > 4096) bidx[b++] = k;
      }
      if (tid == 63) {
        cpre[kSegRBitmaps] = incl;
        nbm = binc;
      }
    }
    seg_lds_barrier();
    const int ne = cpre[kSegRBitmaps];
    const int nbc = nbm;
    // the first bitmap container's words are requested before the array elements, so both round trips overlap
    constexpr int kWords = 2048 / kSegRThreads;
    uint32_t bw[kWords];
    if (nbc > 0) {
      const uint8_t* c = cptr[bidx[0]];
#pragma unroll
      for (int q = 0; q < kWords; ++q) bw[q] = rd32(c + 4 * (q * kSegRThreads + tid));
    }
    for (int e0 = 0; e0 < ne; e0 += kPer * kSegRThreads) {
      uint32_t val[kPer];
      int dst[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int e = e0 + q * kSegRThreads + tid;
        dst[q] = -1;
        if (e < ne) {
          int lo = 0, hi = nc - 1;
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (cpre[mid] <= e) lo = mid; else hi = mid - 1;
          }
          val[q] = rd16(cptr[lo] + 2 * (e - cpre[lo]));
          dst[q] = cleaf[lo] * 2048;
        }
      }
#pragma unroll
      for (int q = 0; q < kPer; ++q)
        if (dst[q] >= 0) atomicOr(&lmask[dst[q] + (val[q] >> 5)], 1u << (val[q] & 31u));
    }
    for (int i = 0; i < nbc; ++i) {  // bitmap containers: all words in flight, then the ORs
      const int k = bidx[i];
      if (i > 0) {
        const uint8_t* c = cptr[k];
#pragma unroll
        for (int q = 0; q < kWords; ++q) bw[q] = rd32(c + 4 * (q * kSegRThreads + tid));
      }
      uint32_t* m = lmask + cleaf[k] * 2048;
#pragma unroll
      for (int q = 0; q < kWords; ++q)
        if (bw[q]) atomicOr(&m[q * kSegRThreads + tid], bw[q]);
    }
    seg_lds_barrier();
    const int64_t doc0 = static_cast<int64_t>(chunk) << 16;
    uint32_t* out = P.mask + static_cast<size_t>(chunk) * 2048;
    for (int w = tid; w < 2048; w += kSegRThreads) {
      uint32_t st[kRProgStack + 4];
      int sp = 0, lf = 0;
      const int64_t d = doc0 + 32 * w;
      const uint32_t keep = d >= P.num_docs ? 0u : (d + 32 > P.num_docs ? (1u << (P.num_docs - d)) - 1u : 0xFFFFFFFFu);
      for (int i = 0; i < P.nops; ++i) {
        const int op = P.op[i];
        if (op == RP_LEAF) {
          st[sp++] = lmask[lf * 2048 + w];
          ++lf;
        } else if (op == RP_NOT) {
          st[sp - 1] = ~st[sp - 1] & keep;
        } else {
          st[sp - 2] = op == RP_AND ? (st[sp - 2] & st[sp - 1]) : (st[sp - 2] | st[sp - 1]);
          --sp;
        }
      }
      out[w] = st[0];
    }
    seg_lds_barrier();  // lmask is zeroed for the next chunk
  }
}

// Wave-per-chunk form of the bitmap programs: every wavefront walks its own range of one segment's chunks with its own
// LDS masks, and the workgroup never synchronises (the workgroup kernel above spends most of a chunk waiting at five
// barriers for its slowest wave).  Lane b owns bitmap b of the program (<= 64 bitmaps) and its container cursor.
// Leaves share mask "slots" while the slot's operand is still "pure" (an OR of leaves, nothing applied to it yet):
//   * a leaf directly followed by OR is ORed into the pure top operand's slot (phase 0);
//   * a leaf directly followed by NOT, AND is cleared out of the pure top operand's slot (phase 1: AND-NOT, after
//     every phase-0 container of the chunk), which leaves the slot impure.
// C5's (f1 IN .. OR f2 = 7) AND NOT f3 = 3 thus needs ONE 8 KiB slot per wave.  The rest of the postfix program is
// evaluated over the slots and the chunk's mask written.  The plan is a walk of the program with a 4-bit-per-entry
// stack in one 64-bit word (slot in bits 0-2, "pure" in bit 3); the host applies the same rule (rprog_slots).
#ifndef PGX_WAVE_ELEMS
#define PGX_WAVE_ELEMS 16  // array elements per lane in flight (C5: 16 -> 0.75 ms, 8 -> 0.79, 32 with per-element searches slower)
#endif
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Fusion of the leaf at op i into the top operand: 0 none, 1 OR (skips op i + 1), 2 AND-NOT (skips ops i + 1, i + 2).
__device__ __forceinline__ int rprog_fusion(const RProg& P, int i, uint64_t stk) {
  if (!(stk & 8u)) return 0;
  if (i + 1 < P.nops && P.op[i + 1] == RP_OR) return 1;
  if (i + 2 < P.nops && P.op[i + 1] == RP_NOT && P.op[i + 2] == RP_AND) return 2;
  return 0;
}

template <int NS, int WPB, int MINW>
__global__ void __launch_bounds__(64 * WPB, MINW) pgx_roaring_program_wave(const RProg* __restrict__ progs,
                                                                          const RDesc* __restrict__ descs, int nprogs,
                                                                          int parts) {
  extern __shared__ uint32_t wmask[];  // [wave][NS][2048]
  __shared__ int wpre[WPB][65];
  __shared__ const uint8_t* wptr[WPB][64];
  __shared__ int wslot[WPB][64];
  const int lane = static_cast<int>(threadIdx.x) & 63, wv = static_cast<int>(threadIdx.x) >> 6;
  const int gw = static_cast<int>(blockIdx.x) * WPB + wv;
  const int pi = gw / parts;
  if (pi >= nprogs) return;  // per wave: nothing below synchronises the workgroup
  const RProg& P = progs[pi];
  const int per = (P.nchunks + parts - 1) / parts;
  const int c0 = (gw % parts) * per;
  const int c1 = min(P.nchunks, c0 + per);
  if (c0 >= c1) return;
  uint32_t* sm = wmask + wv * NS * 2048;
  int* pre = wpre[wv];
  const uint8_t** ptrs = wptr[wv];
  int* slots = wslot[wv];
  // slot plan: this lane's bitmap, its leaf's slot and phase
  int my_desc = -1, my_first = 0, my_slot = 0, my_phase = 0;
  bool any_andnot = false;
  {
    uint64_t stk = 0;
    int ns = 0, tot = 0;
    for (int i = 0; i < P.nops; ++i) {
      const int op = P.op[i];
      if (op == RP_LEAF) {
        const int a = P.arg[i];
        const int nb = a >= 0 ? descs[a].nb : 0;
        const int f = rprog_fusion(P, i, stk);
        const int slot = f ? static_cast<int>(stk & 7u) : ns;
        if (!f) {
          stk = (stk << 4) | 8u | static_cast<uint64_t>(ns);
          ++ns;
        }
        if (lane >= tot && lane < tot + nb) {
          my_desc = a;
          my_first = tot;
          my_slot = slot;
          my_phase = f == 2 ? 1 : 0;
        }
        tot += nb;
        if (f == 2) {
          stk &= ~uint64_t(8);
          any_andnot = true;
        }
        i += f;  // the fused OR / NOT, AND are done by the expansion itself
      } else if (op == RP_NOT) {
        stk &= ~uint64_t(8);
      } else {
        stk >>= 4;  // drop the right operand; the left one holds the result, no longer pure
        stk &= ~uint64_t(8);
      }
    }
  }
  const uint8_t* base = nullptr;
  int n = 0, cur = 0, key = 1 << 30, card = 0;
  uint32_t off = 0;
  if (my_desc >= 0) {
    const RDesc& D = descs[my_desc];
    base = rbitmap(D, lane - my_first);
    n = static_cast<int>(rd32(base + 4));
    if (c0 > 0 && n > 0) {
      if (n > c0 && static_cast<int>(rd16(base + 8 + 4 * c0)) == c0) {
        cur = c0;
      } else {
        int lo = 0, hi = n;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (static_cast<int>(rd16(base + 8 + 4 * mid)) < c0) lo = mid + 1; else hi = mid;
        }
        cur = lo;
      }
    }
    if (cur < n) {
      key = static_cast<int>(rd16(base + 8 + 4 * cur));
      card = static_cast<int>(rd16(base + 8 + 4 * cur + 2)) + 1;
      off = rd32(base + 8 + 4 * n + 4 * cur);
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s)
    for (int j = 0; j < 32; ++j) sm[s * 2048 + j * 64 + lane] = 0u;
  for (int chunk = c0; chunk < c1; ++chunk) {
    const bool act = key == chunk;
    const uint8_t* cptr = base + off;
    const int ccard = card;
    if (act) {  // advance the cursor now; the next container's fields are consumed at a later chunk
      ++cur;
      if (cur < n) {
        key = static_cast<int>(rd16(base + 8 + 4 * cur));
        card = static_cast<int>(rd16(base + 8 + 4 * cur + 2)) + 1;
        off = rd32(base + 8 + 4 * n + 4 * cur);
      } else {
        key = 1 << 30;
      }
    }
    for (int ph = 0; ph < (any_andnot ? 2 : 1); ++ph) {
      const bool mine = act && my_phase == ph;
      const bool arr = mine && ccard <= 4096;
      const int v = arr ? ccard : 0;
      int incl = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      const int total = __shfl(incl, 63, 64);
      pre[lane] = incl - v;
      if (lane == 63) pre[64] = incl;
      ptrs[lane] = mine ? cptr : nullptr;
      slots[lane] = my_slot;
      uint64_t bm = __ballot(mine && ccard > 4096);
      wave_lds_sync();
      // array containers: element e of the chunk's concatenated containers, container k with pre[k] <= e < pre[k + 1];
      // the lane's first element by one search, later ones (64 apart) by stepping forward (about one step each)
      if (total > 0) {
        int k = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
          if (pre[k + step] <= lane) k += step;  // largest k <= 63 with pre[k] <= lane
        int kend = pre[k + 1], kbeg = pre[k];
        const uint8_t* kp = ptrs[k];
        int ks = slots[k];
        constexpr int B = PGX_WAVE_ELEMS;
        for (int e0 = lane; e0 < total; e0 += 64 * B) {
          uint32_t val[B];
          int dst[B];
#pragma unroll
          for (int q = 0; q < B; ++q) {
            const int e = e0 + 64 * q;
            dst[q] = -1;
            if (e < total) {
              while (kend <= e) {
                ++k;
                kbeg = kend;
                kend = pre[k + 1];
                kp = ptrs[k];
                ks = slots[k];
              }
              val[q] = rd16(kp + 2 * (e - kbeg));
              dst[q] = ks * 2048;
            }
          }
#pragma unroll
          for (int q = 0; q < B; ++q)
            if (dst[q] >= 0) {
              if (ph == 0) atomicOr(&sm[dst[q] + (val[q] >> 5)], 1u << (val[q] & 31u));
              else atomicAnd(&sm[dst[q] + (val[q] >> 5)], ~(1u << (val[q] & 31u)));
            }
        }
      }
      // bitmap containers: 16 words per lane in flight at a time, ORed into (or cleared out of) the leaf's slot
      while (bm) {
        const int src = __builtin_ctzll(bm);
        bm &= bm - 1;
        const uint8_t* c = ptrs[src];
        uint32_t* m = sm + slots[src] * 2048;
        const bool al = (reinterpret_cast<uintptr_t>(c) & 3u) == 0;
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {
          uint32_t x[16];
          if (al) {
            const PGX_GLOBAL uint32_t* c32 = (const PGX_GLOBAL uint32_t*)(c);
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = c32[(h * 16 + j) * 64 + lane];
          } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = rd32(c + 4 * ((h * 16 + j) * 64 + lane));
          }
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (x[j]) {
              if (ph == 0) atomicOr(&m[(h * 16 + j) * 64 + lane], x[j]);
              else atomicAnd(&m[(h * 16 + j) * 64 + lane], ~x[j]);
            }
        }
      }
      wave_lds_sync();
    }
    // the rest of the program over the slots (same walk as the plan), word j * 64 + lane; result written, slots cleared
    const int64_t doc0 = static_cast<int64_t>(chunk) << 16;
    uint32_t* out = P.mask + static_cast<size_t>(chunk) * 2048;
    uint64_t stk = 0;
    int ns = 0;
    for (int i = 0; i < P.nops; ++i) {
      const int op = P.op[i];
      if (op == RP_LEAF) {
        const int f = rprog_fusion(P, i, stk);
        if (!f) {
          stk = (stk << 4) | 8u | static_cast<uint64_t>(ns);
          ++ns;
        }
        if (f == 2) stk &= ~uint64_t(8);
        i += f;
      } else if (op == RP_NOT) {
        uint32_t* a = sm + static_cast<int>(stk & 7u) * 2048;
#pragma unroll 4
        for (int j = 0; j < 32; ++j) {
          const int w = j * 64 + lane;
          const int64_t d = doc0 + 32 * w;
          const uint32_t keep =
              d >= P.num_docs ? 0u : (d + 32 > P.num_docs ? (1u << (P.num_docs - d)) - 1u : 0xFFFFFFFFu);
          a[w] = ~a[w] & keep;
        }
        stk &= ~uint64_t(8);
      } else {
        const uint32_t* b = sm + static_cast<int>(stk & 7u) * 2048;
        stk >>= 4;
        uint32_t* a = sm + static_cast<int>(stk & 7u) * 2048;
        if (op == RP_AND) {
#pragma unroll 8
          for (int j = 0; j < 32; ++j) a[j * 64 + lane] &= b[j * 64 + lane];
        } else {
#pragma unroll 8
          for (int j = 0; j < 32; ++j) a[j * 64 + lane] |= b[j * 64 + lane];
        }
        stk &= ~uint64_t(8);
      }
    }
    const uint32_t* r = sm + static_cast<int>(stk & 7u) * 2048;
#pragma unroll 8
    for (int j = 0; j < 32; ++j) out[j * 64 + lane] = r[j * 64 + lane];
    for (int s = 0; s < NS; ++s)
#pragma unroll 8
      for (int j = 0; j < 32; ++j) sm[s * 2048 + j * 64 + lane] = 0u;
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------------------------------------
// Multi-value columns.  One thread owns 32 consecutive docs (one mask word); their values are consecutive in the raw
// section, so neighbouring threads read neighbouring bytes.  A value is cut out of the big-endian bit stream with one
// 64-bit window (two byte-swapped dwords; the staged buffer is padded past the last value).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mv_value(const uint32_t* __restrict__ vals, int64_t i, int bits) {
  const int64_t o = i * bits;
  const PGX_GLOBAL uint32_t* w = (const PGX_GLOBAL uint32_t*)(vals) + (o >> 5);
  const uint64_t x = (static_cast<uint64_t>(__builtin_bswap32(w[0])) << 32) | __builtin_bswap32(w[1]);
  return static_cast<uint32_t>(x >> (64 - (o & 31) - bits)) & (bits == 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u));
}

__global__ void __launch_bounds__(256) pgx_mv_leaf_mask(const MvLeaf* __restrict__ items, int nitems, int max_words) {
  const int it = static_cast<int>(blockIdx.y);
  if (it >= nitems) return;
  const MvLeaf& L = items[it];
  const int w = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x);
  const int words = (L.num_docs + 31) >> 5;
  if (w >= words) return;
  (void)max_words;
  uint32_t out = 0u;
  const int d0 = w * 32;
  const int dn = min(32, L.num_docs - d0);
  for (int k = 0; k < dn; ++k) {
    const int s = L.start[d0 + k], e = L.start[d0 + k + 1];
    bool hit = false;  // any value in the matching set (EQ / IN / RANGE) or outside it (NEQ / NOT_IN)
    for (int i = s; i < e && !hit; ++i) {
      const uint32_t v = mv_value(L.vals, i, L.bits);
      const bool in = L.bitset ? ((L.bitset[v >> 5] >> (v & 31u)) & 1u) : (v - L.lo <= L.span);
      hit = in != (L.neg != 0);
    }
    if (hit != (L.neg != 0)) out |= 1u << k;
  }
  L.mask[w] = out;
}

__device__ __forceinline__ uint64_t mv_ord_i64(int64_t x) { return static_cast<uint64_t>(x) ^ 0x8000000000000000ull; }
__device__ __forceinline__ uint64_t mv_ord_f64(double d) {
  const uint64_t b = static_cast<uint64_t>(__double_as_longlong(d));
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

__global__ void __launch_bounds__(256) pgx_mv_aggregate(const MvAgg* __restrict__ items, int nitems) {
  const int it = static_cast<int>(blockIdx.y);
  if (it >= nitems) return;
  const MvAgg& A = items[it];
  const int w = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x);
  const int words = (A.num_docs + 31) >> 5;
  uint64_t cnt = 0;
  int64_t isum = 0;
  double dsum = 0.0;
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;  // dictIds: numeric dictionaries are sorted (SegmentDictionaryCreator)
  if (w < words) {
    uint32_t sel = A.sel[w];
    const int d0 = w * 32;
    if (d0 + 32 > A.num_docs) sel &= (1u << (A.num_docs - d0)) - 1u;
    while (sel) {
      const int k = __builtin_ctz(sel);
      sel &= sel - 1u;
      const int s = A.start[d0 + k], e = A.start[d0 + k + 1];
      for (int i = s; i < e; ++i) {
        const uint32_t v = mv_value(A.vals, i, A.bits);
        ++cnt;
        if (A.fp) dsum += ((const PGX_GLOBAL double*)A.dict)[v];
        else isum += ((const PGX_GLOBAL int64_t*)A.dict)[v];
        mn = min(mn, v);
        mx = max(mx, v);
      }
    }
  }
  uint64_t omin = ~0ull, omax = 0ull;
  if (cnt) {
    omin = A.fp ? mv_ord_f64(((const PGX_GLOBAL double*)A.dict)[mn])
                : mv_ord_i64(((const PGX_GLOBAL int64_t*)A.dict)[mn]);
    omax = A.fp ? mv_ord_f64(((const PGX_GLOBAL double*)A.dict)[mx])
                : mv_ord_i64(((const PGX_GLOBAL int64_t*)A.dict)[mx]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    cnt += __shfl_xor(cnt, off);
    isum += __shfl_xor(isum, off);
    dsum += __shfl_xor(dsum, off);
    const uint64_t a = __shfl_xor(omin, off), b = __shfl_xor(omax, off);
    omin = a < omin ? a : omin;
    omax = b > omax ? b : omax;
  }
  if ((threadIdx.x & 63) == 0 && cnt) {
    atomicAdd(A.out, static_cast<unsigned long long>(cnt));
    if (A.fp) atomicAdd(reinterpret_cast<double*>(A.out + 1), dsum);
    else atomicAdd(A.out + 1, static_cast<unsigned long long>(isum));
    atomicMin(A.out + 2, static_cast<unsigned long long>(omin));
    atomicMax(A.out + 3, static_cast<unsigned long long>(omax));
  }
}

// ---------------------------------------------------------------------------------------------
// Group-by over multi-value group columns and/or with multi-value functions (DefaultGroupKeyGenerator.java:475-608,
// DefaultGroupByExecutor.java:154-196).  One thread per selected doc: the doc's contribution to every function is
// folded once (SV: its value; COUNTMV: its value count; SUMMV / AVGMV: sum and count of its values), then every key of
// the doc -- one per combination of its group columns' values, duplicates included, as generateKeysForDocId* builds
// them -- receives it (COUNT: 1 per key, CountAggregationFunction.java:81-90; Sum/Min/Max/Avg.aggregateGroupByMV).
// Keys follow the single-value layouts: dense slot = sum gid_g * mul_g, hash keys gid_g << shift_g.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t mv_slot64(unsigned long long* keys, uint64_t cap, uint64_t key) {
  const uint64_t mask = cap - 1;
  const uint64_t lim = cap < kGlobalMaxProbes ? cap : kGlobalMaxProbes;
  uint64_t h = mix64(key) & mask;
  for (uint64_t probe = 0; probe < lim; ++probe) {
    const unsigned long long prev = atomicCAS(keys + h, kEmptyKey, static_cast<unsigned long long>(key));
    if (prev == kEmptyKey || prev == key) return static_cast<int64_t>(h);
    h = (h + 1) & mask;
  }
  return -1;
}

__device__ __forceinline__ int64_t mv_slot128(unsigned long long* keys, unsigned int* key_state, uint64_t cap,
                                              uint64_t klo, uint64_t khi) {
  const uint64_t mask = cap - 1;
  const uint64_t lim = cap < kGlobalMaxProbes ? cap : kGlobalMaxProbes;
  uint64_t h = mix64(klo ^ mix64(khi)) & mask;
  uint64_t probes = 0;
  while (probes < lim) {
    const unsigned int st = atomicCAS(key_state + h, 0u, 1u);
    if (st == 0u) {
      __hip_atomic_store(keys + 2 * h, klo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(keys + 2 * h + 1, khi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
      atomicExch(key_state + h, 2u);
      return static_cast<int64_t>(h);
    }
    if (st == 2u) {
      const unsigned long long a = __hip_atomic_load(keys + 2 * h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long b = __hip_atomic_load(keys + 2 * h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a == klo && b == khi) return static_cast<int64_t>(h);
      h = (h + 1) & mask;
      ++probes;
    }
  }
  return -1;
}


// The doc's group keys, in generateKeysForDocId* combination order, one callback per key: f(dense slot or packed lo,
// packed hi).  Returns false when a multi-value group column holds no value (no key).
template <typename F>
__device__ __forceinline__ bool mv_for_each_key(const MvGroupArgs& A, const MvGroupSeg& S, int d, F&& f) {
  int nv[kMaxGroupCols], base[kMaxGroupCols], idx[kMaxGroupCols];
  uint32_t sv[kMaxGroupCols];
#pragma unroll
  for (int g = 0; g < kMaxGroupCols; ++g) {
    nv[g] = 1;
    base[g] = 0;
    idx[g] = 0;
    sv[g] = 0;
    if (g >= A.ngcols) continue;
    const MvGCol& c = S.g[g];
    if (c.start) {
      base[g] = c.start[d];
      nv[g] = c.start[d + 1] - base[g];
      if (nv[g] <= 0) return false;
    } else {
      sv[g] = mv_value(c.vals, d, c.bits);
    }
  }
  for (;;) {
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int g = 0; g < kMaxGroupCols; ++g) {
      if (g >= A.ngcols) continue;
      const MvGCol& c = S.g[g];
      uint32_t id = c.start ? mv_value(c.vals, base[g] + idx[g], c.bits) : sv[g];
      if (c.remap) id = static_cast<uint32_t>(c.remap[id]);
      if (A.group_mode == G_DENSE_GLOBAL) lo += static_cast<uint64_t>(id) * A.gmul[g];
      else if (A.ghi[g]) hi |= static_cast<uint64_t>(id) << A.gshift[g];
      else lo |= static_cast<uint64_t>(id) << A.gshift[g];
    }
    f(lo, hi);
    int g = 0;  // odometer over the multi-value columns, column 0 fastest
    for (; g < A.ngcols; ++g) {
      if (++idx[g] < nv[g]) break;
      idx[g] = 0;
    }
    if (g == A.ngcols) return true;
  }
}

__global__ void __launch_bounds__(256) pgx_mv_group(const MvGroupArgs* __restrict__ Ap) {
  const MvGroupArgs& A = *Ap;
  const int s = static_cast<int>(blockIdx.y);
  if (s >= A.nsegs) return;
  const MvGroupSeg& S = A.segs[s];
  const int d = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x);
  if (d >= S.num_docs || !((S.sel[d >> 5] >> (d & 31)) & 1u)) return;
  // the doc's contribution per function: enc (plane encoding) and cnt (AVGMV value count)
  unsigned long long enc[kMaxAggs];
  long long cnt[kMaxAggs];
#pragma unroll
  for (int a = 0; a < kMaxAggs; ++a) {
    enc[a] = 0;
    cnt[a] = 0;
    if (a >= A.naggs) continue;
    const MvGCol& c = S.a[a];
    const int fn = A.fn[a];
    const bool fp = A.fp[a] != 0;
    if (fn == MVF_COUNT || fn == MVF_MINMV || fn == MVF_MAXMV) continue;  // MINMV / MAXMV: pgx_mv_group_ordered
    if (fn <= MVF_AVG) {  // single-value column: the doc's value
      const uint32_t id = mv_value(c.vals, d, c.bits);
      if (fp) {
        const double v = static_cast<const double*>(c.dict)[id];
        enc[a] = (fn == MVF_MIN || fn == MVF_MAX) ? ord_f64(v) : static_cast<unsigned long long>(__double_as_longlong(v));
      } else {
        const int64_t v = static_cast<const int64_t*>(c.dict)[id];
        enc[a] = (fn == MVF_MIN || fn == MVF_MAX) ? ord_i64(v) : static_cast<unsigned long long>(v);
      }
      continue;
    }
    const int b0 = c.start[d], b1 = c.start[d + 1];
    cnt[a] = b1 - b0;
    if (fn == MVF_COUNTMV) {
      enc[a] = static_cast<unsigned long long>(b1 - b0);
      continue;
    }
    double ds = 0.0;  // SUMMV / AVGMV: the doc's values in order (SumMVAggregationFunction.java:98-112)
    int64_t is = 0;
    for (int i = b0; i < b1; ++i) {
      const uint32_t id = mv_value(c.vals, i, c.bits);
      if (fp) ds += static_cast<const double*>(c.dict)[id];
      else is += static_cast<const int64_t*>(c.dict)[id];
    }
    enc[a] = fp ? static_cast<unsigned long long>(__double_as_longlong(ds)) : static_cast<unsigned long long>(is);
  }
  mv_for_each_key(A, S, d, [&](uint64_t lo, uint64_t hi) {
    int64_t slot;
    if (A.group_mode == G_DENSE_GLOBAL) slot = static_cast<int64_t>(lo);
    else if (A.group_mode == G_HASH64) slot = mv_slot64(A.keys, A.slots, lo);
    else slot = mv_slot128(A.keys, A.key_state, A.slots, lo, hi);
    if (slot < 0) {
      atomicAdd(A.overflow, 1ull);
      return;
    }
    atomicAdd(A.table + slot, 1ull);  // plane 0: (doc, key) pairs = COUNT
#pragma unroll
    for (int a = 0; a < kMaxAggs; ++a) {
      if (a >= A.naggs) continue;
      const int fn = A.fn[a];
      unsigned long long* p = A.table + static_cast<uint64_t>(a + 1) * A.slots + slot;
      const bool fp = A.fp[a] != 0;
      switch (fn) {
        case MVF_SUM: case MVF_AVG: case MVF_SUMMV: case MVF_AVGMV:
          if (fp) atomicAdd(reinterpret_cast<double*>(p), __longlong_as_double(static_cast<long long>(enc[a])));
          else atomicAdd(p, enc[a]);
          if (fn == MVF_AVGMV)
            atomicAdd(A.table + static_cast<uint64_t>(A.cnt_plane[a]) * A.slots + slot,
                      static_cast<unsigned long long>(cnt[a]));
          break;
        case MVF_COUNTMV: atomicAdd(p, enc[a]); break;
        case MVF_MIN: atomicMin(p, enc[a]); break;
        case MVF_MAX: atomicMax(p, enc[a]); break;
        default: break;
      }
    }
  });
}

// Slot of a key pgx_mv_group already inserted (read-only probe; -1 if absent).
__device__ __forceinline__ int64_t mv_find(const MvGroupArgs& A, uint64_t lo, uint64_t hi) {
  const uint64_t mask = A.slots - 1;
  if (A.group_mode == G_HASH64) {
    uint64_t h = mix64(lo) & mask;
    for (uint64_t probe = 0; probe < A.slots; ++probe) {
      const unsigned long long k = A.keys[h];
      if (k == lo) return static_cast<int64_t>(h);
      if (k == kEmptyKey) return -1;
      h = (h + 1) & mask;
    }
    return -1;
  }
  uint64_t h = mix64(lo ^ mix64(hi)) & mask;
  for (uint64_t probe = 0; probe < A.slots; ++probe) {
    if (A.key_state[h] != 2u) return -1;
    if (A.keys[2 * h] == lo && A.keys[2 * h + 1] == hi) return static_cast<int64_t>(h);
    h = (h + 1) & mask;
  }
  return -1;
}

// MINMV / MAXMV under GROUP BY (MinMVAggregationFunction.java:76-91 aggregateGroupBySV, :103-119 aggregateGroupByMV;
// MaxMV alike): the holder's value is read ONCE per (doc, key) and every value of the doc below (above) it replaces the
// holder, so a doc leaves the LAST such value in its value order -- an order-dependent fold, not a minimum.  One
// workgroup walks one segment's selected docs in doc order; thread t owns the keys whose dense slot s has
// s % 256 == t (hash key spaces: whose key hash has that residue; the owner finds the key's slot in the table
// pgx_mv_group filled) and applies the fold to them only, so every key sees its docs in order with no atomics.  Holders
// are that segment's dictIds (sorted dictionaries: dictId order = value order); the per-segment results merge into the
// table with the combine's min / max (combineTwoValues).
__global__ void __launch_bounds__(256) pgx_mv_group_ordered(const MvGroupArgs* __restrict__ Ap) {
  const MvGroupArgs& A = *Ap;
  const int s = static_cast<int>(blockIdx.x);
  if (s >= A.nsegs) return;
  const MvGroupSeg& S = A.segs[s];
  const int tid = static_cast<int>(threadIdx.x);
  int64_t* hold = reinterpret_cast<int64_t*>(A.ord) + static_cast<uint64_t>(s) * A.naggs * A.slots;
  for (uint64_t sl = tid; sl < A.slots; sl += 256)
    for (int a = 0; a < A.naggs; ++a) hold[a * A.slots + sl] = A.fn[a] == MVF_MINMV ? INT64_MAX : -1;
  __syncthreads();  // hash key spaces: a slot's owner is not the thread that initialised it
  for (int d = 0; d < S.num_docs; ++d) {
    if (!((S.sel[d >> 5] >> (d & 31)) & 1u)) continue;
    mv_for_each_key(A, S, d, [&](uint64_t lo, uint64_t hi) {
      uint64_t sl = lo;
      if (A.group_mode == G_DENSE_GLOBAL) {
        if (static_cast<int>(lo & 255u) != tid) return;
      } else {
        const uint64_t own = A.group_mode == G_HASH64 ? mix64(lo) : mix64(lo ^ mix64(hi));
        if (static_cast<int>((own >> 40) & 255u) != tid) return;
        const int64_t f = mv_find(A, lo, hi);
        if (f < 0) {
          atomicAdd(A.overflow, 1ull);
          return;
        }
        sl = static_cast<uint64_t>(f);
      }
      for (int a = 0; a < A.naggs; ++a) {
        const int fn = A.fn[a];
        if (fn != MVF_MINMV && fn != MVF_MAXMV) continue;
        const MvGCol& c = S.a[a];
        int64_t* h = hold + a * A.slots + sl;
        const int64_t old = *h;
        for (int i = c.start[d]; i < c.start[d + 1]; ++i) {
          const int64_t id = mv_value(c.vals, i, c.bits);
          if (fn == MVF_MINMV ? id < old : id > old) *h = id;
        }
      }
    });
  }
  __syncthreads();  // ... nor the thread that flushes it
  for (uint64_t sl = tid; sl < A.slots; sl += 256)
    for (int a = 0; a < A.naggs; ++a) {
      const int fn = A.fn[a];
      if (fn != MVF_MINMV && fn != MVF_MAXMV) continue;
      const int64_t id = hold[a * A.slots + sl];
      if (id == INT64_MAX || id < 0) continue;
      const MvGCol& c = S.a[a];
      const unsigned long long e = A.fp[a] ? ord_f64(static_cast<const double*>(c.dict)[id])
                                           : ord_i64(static_cast<const int64_t*>(c.dict)[id]);
      unsigned long long* p = A.table + static_cast<uint64_t>(a + 1) * A.slots + sl;
      if (fn == MVF_MINMV) atomicMin(p, e);
      else atomicMax(p, e);
    }
}

// ---------------------------------------------------------------------------------------------
// High-cardinality group-by (LONG_MAP semantics, DefaultGroupKeyGenerator.java:239-246 / :429-441): the reference
// probes a Long2IntOpenHashMap per doc; at 10^7 groups a device-wide hash table turns every row into random HBM atomics.
// Instead the generated scan kernel emits one packed record per selected row (key | value << keybits), two radix
// passes split the records into 64 x 128 partitions by hash bits, and one workgroup per partition aggregates it in an
// LDS hash table, then appends its groups to compact output arrays.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t part_mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

constexpr int kPartThreads = 1024;
constexpr int kPartPer = 8;                             // records per thread, held in registers
constexpr int kPartChunk = kPartThreads * kPartPer;     // records per partitioning workgroup (64 KiB LDS staging)
constexpr uint64_t kNoRecord = ~0ull;

constexpr int kPartMaxBuckets = 256;

// Exclusive scan of hist[0, nb) (nb <= 256) by wave 0, four buckets per lane: offs[b] = sum of hist[< b]; *total = sum
// of all.
__device__ __forceinline__ void part_scan256(const int* hist, int* offs, int* total, int nb, int tid) {
  if (tid >= 64) return;
  int h[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) h[k] = 4 * tid + k < nb ? hist[4 * tid + k] : 0;
  const int own = h[0] + h[1] + h[2] + h[3];
  int x = own;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (tid >= d) x += y;
  }
  int run = x - own;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (4 * tid + k < nb) offs[4 * tid + k] = run;
    run += h[k];
  }
  if (tid == 63) *total = x;
}

// Records of region r live at in + in_off[r] (in_off null: r * in_cap), in_cnt[r * in_cstride] of them (in_cnt null:
// in_cap; else typically the previous pass's cursors, read on the device, so passes chain without a host round trip);
// regions come in groups of reg_div (the scan's per-workgroup slabs of one bucket), and group q's partition b goes to
// out + (q * nb + b) * cap, appended at cursor[(q * nb + b) * cstride] (cursors spread over separate cache lines: every
// workgroup of a pass reserves its runs there).
__global__ void __launch_bounds__(kPartThreads) pgx_partition(const uint64_t* __restrict__ in,
                                                              const int64_t* __restrict__ in_off,
                                                              const unsigned long long* __restrict__ in_cnt,
                                                              int in_cstride, int nreg, int reg_div,
                                                              int64_t in_cap, int chunks_per_reg, uint64_t keymask,
                                                              int shift, int nbits, uint64_t* __restrict__ out,
                                                              int64_t cap, unsigned long long* __restrict__ cursor,
                                                              int cstride, unsigned long long* __restrict__ overflow) {
  const int r = static_cast<int>(blockIdx.x / chunks_per_reg);
  const int64_t chunk = static_cast<int64_t>(blockIdx.x % chunks_per_reg);
  if (r >= nreg) return;
  const int64_t n = in_cnt ? min(static_cast<int64_t>(in_cnt[static_cast<int64_t>(r) * in_cstride]), in_cap) : in_cap;
  const int q = r / reg_div;
  const int64_t c0 = chunk * kPartChunk;
  if (c0 >= n) return;
  const int cn = static_cast<int>(min<int64_t>(kPartChunk, n - c0));
  const int nb = 1 << nbits;
  __shared__ uint64_t stage[kPartChunk];
  __shared__ int hist[kPartMaxBuckets], offs[kPartMaxBuckets], total;
  __shared__ unsigned long long gpos[kPartMaxBuckets];
  const int tid = threadIdx.x;
  const uint64_t bmask = static_cast<uint64_t>(nb - 1);
  for (int i = tid; i < nb; i += kPartThreads) hist[i] = 0;
  const PGX_GLOBAL uint64_t* src = (const PGX_GLOBAL uint64_t*)(in) +
                                   (in_off ? in_off[r] : static_cast<int64_t>(r) * in_cap) + c0;
  uint64_t rec[kPartPer];
#pragma unroll
  for (int k = 0; k < kPartPer; ++k) {
    const int i = k * kPartThreads + tid;
    rec[k] = i < cn ? __builtin_nontemporal_load(src + i) : kNoRecord;
  }
  __syncthreads();
  // the histogram atomic returns the record's rank within its bucket, so staging needs no second atomic
  int bk[kPartPer], rk[kPartPer];
#pragma unroll
  for (int k = 0; k < kPartPer; ++k) {
    bk[k] = rec[k] == kNoRecord ? -1 : static_cast<int>((part_mix(rec[k] & keymask) >> shift) & bmask);
    rk[k] = bk[k] >= 0 ? atomicAdd(&hist[bk[k]], 1) : 0;
  }
  __syncthreads();
  part_scan256(hist, offs, &total, nb, tid);
  if (tid < nb && hist[tid]) {
    const unsigned long long g = atomicAdd(&cursor[(static_cast<int64_t>(q) * nb + tid) * cstride],
                                           static_cast<unsigned long long>(hist[tid]));
    gpos[tid] = g;
    if (g + hist[tid] > static_cast<unsigned long long>(cap)) atomicAdd(overflow, 1ull);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPartPer; ++k) {
    if (bk[k] >= 0) stage[offs[bk[k]] + rk[k]] = rec[k];
  }
  __syncthreads();
  // copy out bucket runs: consecutive staged records of one bucket go to consecutive output words
  PGX_GLOBAL uint64_t* dst = (PGX_GLOBAL uint64_t*)(out);
  const int tot = total;
  for (int i = tid; i < tot; i += kPartThreads) {
    const uint64_t v = stage[i];
    const int b = static_cast<int>((part_mix(v & keymask) >> shift) & bmask);  // recomputed: cheaper than an LDS byte array
    const unsigned long long p = gpos[b] + static_cast<unsigned long long>(i - offs[b]);
    // plain (not streaming) stores: a bucket run's first and last lines are completed by other workgroups' runs,
    // which L2 merges before write-back
    if (p < static_cast<unsigned long long>(cap)) dst[(static_cast<int64_t>(q) * nb + b) * cap + static_cast<int64_t>(p)] = v;
  }
}

// One workgroup aggregates one partition in an LDS hash table and appends its groups to the output: okey[g] = packed
// key, oplane[p * ocap + g] = plane p (count, int64 sum, ordered min, ordered max).  The table is bucketised: a key
// hashes to a bucket of 4 slots (32 contiguous bytes, read with two 16-byte LDS loads and compared in registers), so a
// lookup is straight-line code; a full bucket continues in the next one (rare at the planned load <= 1/3).
// PACK: count and sum share one 64-bit LDS add ((1 << pack_shift) + value; the host checks that a partition's value
// sum stays below bit pack_shift and its count below bit 64 - pack_shift).
constexpr int kAggWays = 4;
constexpr int kAggBuckets = 512;
constexpr int kAggSlots = kAggBuckets * kAggWays;
constexpr int kAggThreads = 1024;
constexpr int kAggPer = 8;

template <bool PACK, bool MN, bool MX>
__global__ void __launch_bounds__(kAggThreads) pgx_part_aggregate(const uint64_t* __restrict__ in,
                                                                  const unsigned long long* __restrict__ in_cnt,
                                                                  int cstride, int64_t cap, uint64_t keymask,
                                                                  int keybits, int64_t vbase, int pack_shift,
                                                                  uint64_t* __restrict__ okey,
                                                                  uint64_t* __restrict__ oplane, int64_t ocap,
                                                                  unsigned long long* __restrict__ ocount,
                                                                  unsigned long long* __restrict__ overflow) {
  __shared__ __attribute__((aligned(16))) uint64_t tkey[kAggSlots];
  __shared__ unsigned long long tsum[kAggSlots];   // sum, or (count << pack_shift) + sum
  __shared__ unsigned int tcnt[PACK ? 1 : kAggSlots];
  __shared__ unsigned int tmin[MN ? kAggSlots : 1], tmax[MX ? kAggSlots : 1];
  __shared__ int nfound;
  __shared__ unsigned long long obase;
  const int tid = threadIdx.x;
  const int part = blockIdx.x;
  for (int i = tid; i < kAggSlots; i += kAggThreads) {
    tkey[i] = kNoRecord;
    tsum[i] = 0ull;
    if (!PACK) tcnt[i] = 0u;
    if (MN) tmin[i] = 0xFFFFFFFFu;
    if (MX) tmax[i] = 0u;
  }
  if (tid == 0) nfound = 0;
  __syncthreads();
  const int64_t n = min(static_cast<int64_t>(in_cnt[static_cast<int64_t>(part) * cstride]), cap);
  const PGX_GLOBAL uint64_t* src = (const PGX_GLOBAL uint64_t*)(in) + static_cast<int64_t>(part) * cap;
  const unsigned long long one = PACK ? (1ull << pack_shift) : 0ull;
  bool lost = false;
  for (int64_t base = 0; base < n; base += kAggThreads * kAggPer) {
    uint64_t rec[kAggPer];
#pragma unroll
    for (int k = 0; k < kAggPer; ++k) {
      const int64_t i = base + k * kAggThreads + tid;
      rec[k] = i < n ? __builtin_nontemporal_load(src + i) : kNoRecord;
    }
    unsigned int sv[kAggPer];  // the values to sum: the records' offsets
#pragma unroll
    for (int k = 0; k < kAggPer; ++k) sv[k] = static_cast<unsigned int>(rec[k] >> keybits);
#pragma unroll
    for (int k = 0; k < kAggPer; ++k) {
      if (rec[k] == kNoRecord) continue;
      const uint64_t key = rec[k] & keymask;
      const unsigned int v = static_cast<unsigned int>(rec[k] >> keybits);  // value offset
      unsigned int bk = static_cast<unsigned int>(part_mix(key)) & (kAggBuckets - 1);
      int slot = -1;
      for (int t = 0; t < kAggBuckets;) {
        const ulonglong2* bp = reinterpret_cast<const ulonglong2*>(&tkey[bk * kAggWays]);
        const ulonglong2 a = bp[0], c = bp[1];
        const int m = a.x == key ? 0 : a.y == key ? 1 : c.x == key ? 2 : c.y == key ? 3 : -1;
        if (m >= 0) { slot = static_cast<int>(bk) * kAggWays + m; break; }
        const int e = a.x == kNoRecord ? 0 : a.y == kNoRecord ? 1 : c.x == kNoRecord ? 2 : c.y == kNoRecord ? 3 : -1;
        if (e >= 0) {
          const int cand = static_cast<int>(bk) * kAggWays + e;
          const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&tkey[cand]), kNoRecord, key);
          if (prev == kNoRecord || prev == key) { slot = cand; break; }
          continue;  // another key took that slot first: re-read this bucket
        }
        bk = (bk + 1) & (kAggBuckets - 1);
        ++t;
      }
      if (slot < 0) { lost = true; continue; }
      if (PACK) {
        atomicAdd(&tsum[slot], one + sv[k]);
      } else {
        atomicAdd(&tcnt[slot], 1u);
        atomicAdd(&tsum[slot], static_cast<unsigned long long>(sv[k]));
      }
      if (MN) atomicMin(&tmin[slot], v);
      if (MX) atomicMax(&tmax[slot], v);
    }
  }
  if (lost) atomicAdd(overflow, 1ull);
  __syncthreads();
  // compact: count, reserve once, write
  int mine = 0;
  for (int i = tid; i < kAggSlots; i += kAggThreads) mine += tkey[i] != kNoRecord;
  const int before = atomicAdd(&nfound, mine);
  __syncthreads();
  if (tid == 0) obase = atomicAdd(ocount, static_cast<unsigned long long>(nfound));
  __syncthreads();
  unsigned long long o = obase + static_cast<unsigned long long>(before);
  const unsigned long long smask = PACK ? (1ull << pack_shift) - 1ull : ~0ull;
  for (int i = tid; i < kAggSlots; i += kAggThreads) {
    if (tkey[i] == kNoRecord) continue;
    if (o >= static_cast<unsigned long long>(ocap)) { atomicAdd(overflow, 1ull); continue; }
    okey[o] = tkey[i];
    const unsigned long long c = PACK ? (tsum[i] >> pack_shift) : tcnt[i];
    const unsigned long long sm = tsum[i] & smask;
    const unsigned int lo = MN ? tmin[i] : 0u, hi = MX ? tmax[i] : 0u;
    oplane[o] = c;  // plane 0: doc count
    // planes 1..3: sum (int64 incl. vbase * count), min, max (ordered encodings of the int64 value)
    oplane[ocap + o] = static_cast<unsigned long long>(static_cast<int64_t>(sm) + static_cast<int64_t>(c) * vbase);
    const int64_t vlo = vbase + static_cast<int64_t>(lo);
    const int64_t vhi = vbase + static_cast<int64_t>(hi);
    oplane[2 * ocap + o] = static_cast<unsigned long long>(vlo) ^ 0x8000000000000000ull;
    oplane[3 * ocap + o] = static_cast<unsigned long long>(vhi) ^ 0x8000000000000000ull;
    ++o;
  }
}


// FLOAT / DOUBLE value column (SumAggregationFunction / Min / Max over a double dictionary): the record's value field
// is an index into the query's concatenation of the segments' dictionaries (fdict, each segment's records rebased to
// its dictionary's place by the scan), looked up here -- the dictionaries are small and L2-resident.  Per slot: count,
// f64 sum (LDS f64 add), ordered-u64 min / max of the value (64-bit LDS min / max).  Planes as pgx_part_aggregate's
// with the sum as f64 bits and the ordered encodings of doubles.
template <bool MN, bool MX>
__global__ void __launch_bounds__(kAggThreads) pgx_part_aggregate_f64(const uint64_t* __restrict__ in,
                                                                      const unsigned long long* __restrict__ in_cnt,
                                                                      int cstride, int64_t cap, uint64_t keymask,
                                                                      int keybits, const double* __restrict__ fdict,
                                                                      uint64_t* __restrict__ okey,
                                                                      uint64_t* __restrict__ oplane, int64_t ocap,
                                                                      unsigned long long* __restrict__ ocount,
                                                                      unsigned long long* __restrict__ overflow) {
  __shared__ __attribute__((aligned(16))) uint64_t tkey[kAggSlots];
  __shared__ double tsum[kAggSlots];
  __shared__ unsigned int tcnt[kAggSlots];
  __shared__ unsigned long long tmin[MN ? kAggSlots : 1], tmax[MX ? kAggSlots : 1];
  __shared__ int nfound;
  __shared__ unsigned long long obase;
  const int tid = threadIdx.x;
  const int part = blockIdx.x;
  for (int i = tid; i < kAggSlots; i += kAggThreads) {
    tkey[i] = kNoRecord;
    tsum[i] = 0.0;
    tcnt[i] = 0u;
    if (MN) tmin[i] = ~0ull;
    if (MX) tmax[i] = 0ull;
  }
  if (tid == 0) nfound = 0;
  __syncthreads();
  const int64_t n = min(static_cast<int64_t>(in_cnt[static_cast<int64_t>(part) * cstride]), cap);
  const PGX_GLOBAL uint64_t* src = (const PGX_GLOBAL uint64_t*)(in) + static_cast<int64_t>(part) * cap;
  const PGX_GLOBAL double* fd = (const PGX_GLOBAL double*)fdict;
  bool lost = false;
  for (int64_t base = 0; base < n; base += kAggThreads * kAggPer) {
    uint64_t rec[kAggPer];
#pragma unroll
    for (int k = 0; k < kAggPer; ++k) {
      const int64_t i = base + k * kAggThreads + tid;
      rec[k] = i < n ? __builtin_nontemporal_load(src + i) : kNoRecord;
    }
    double val[kAggPer];
#pragma unroll
    for (int k = 0; k < kAggPer; ++k) val[k] = rec[k] != kNoRecord ? fd[rec[k] >> keybits] : 0.0;
#pragma unroll
    for (int k = 0; k < kAggPer; ++k) {
      if (rec[k] == kNoRecord) continue;
      const uint64_t key = rec[k] & keymask;
      unsigned int bk = static_cast<unsigned int>(part_mix(key)) & (kAggBuckets - 1);
      int slot = -1;
      for (int t = 0; t < kAggBuckets;) {
        const ulonglong2* bp = reinterpret_cast<const ulonglong2*>(&tkey[bk * kAggWays]);
        const ulonglong2 a = bp[0], c = bp[1];
        const int m = a.x == key ? 0 : a.y == key ? 1 : c.x == key ? 2 : c.y == key ? 3 : -1;
        if (m >= 0) { slot = static_cast<int>(bk) * kAggWays + m; break; }
        const int e = a.x == kNoRecord ? 0 : a.y == kNoRecord ? 1 : c.x == kNoRecord ? 2 : c.y == kNoRecord ? 3 : -1;
        if (e >= 0) {
          const int cand = static_cast<int>(bk) * kAggWays + e;
          const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&tkey[cand]), kNoRecord, key);
          if (prev == kNoRecord || prev == key) { slot = cand; break; }
          continue;
        }
        bk = (bk + 1) & (kAggBuckets - 1);
        ++t;
      }
      if (slot < 0) { lost = true; continue; }
      atomicAdd(&tcnt[slot], 1u);
      atomicAdd(&tsum[slot], val[k]);
      if (MN || MX) {
        const uint64_t b = static_cast<uint64_t>(__double_as_longlong(val[k]));
        const unsigned long long o = (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
        if (MN) atomicMin(&tmin[slot], o);
        if (MX) atomicMax(&tmax[slot], o);
      }
    }
  }
  if (lost) atomicAdd(overflow, 1ull);
  __syncthreads();
  int mine = 0;
  for (int i = tid; i < kAggSlots; i += kAggThreads) mine += tkey[i] != kNoRecord;
  const int before = atomicAdd(&nfound, mine);
  __syncthreads();
  if (tid == 0) obase = atomicAdd(ocount, static_cast<unsigned long long>(nfound));
  __syncthreads();
  unsigned long long o = obase + static_cast<unsigned long long>(before);
  for (int i = tid; i < kAggSlots; i += kAggThreads) {
    if (tkey[i] == kNoRecord) continue;
    if (o >= static_cast<unsigned long long>(ocap)) { atomicAdd(overflow, 1ull); continue; }
    okey[o] = tkey[i];
    oplane[o] = tcnt[i];
    oplane[ocap + o] = static_cast<unsigned long long>(__double_as_longlong(tsum[i]));
    oplane[2 * ocap + o] = MN ? tmin[i] : ~0ull;
    oplane[3 * ocap + o] = MX ? tmax[i] : 0ull;
    ++o;
  }
}

// ---------------------------------------------------------------------------------------------
// Synthetic forward-index generator (benchmarks): dictId(row) = splitmix64(seed ^ row*golden) % card, packed
// MSB-first big-endian.  One thread writes one 32-bit big-endian word = the 32 rows' bits that fall in it.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint32_t synth_value(uint64_t seed, int64_t row, uint32_t card) {
  return static_cast<uint32_t>(splitmix64(seed ^ (static_cast<uint64_t>(row) * 0x9E3779B97F4A7C15ull)) % card);
}

// npairs > 0: the row first draws a pair index from pair_seed, and the value is a function of that index, so two
// columns generated with the same pair_seed / npairs take their values jointly from npairs fixed combinations.
__global__ void pgx_synth_kernel(uint32_t* out_words, int64_t n_rows, int bits, uint32_t card, uint64_t seed,
                                 int64_t n_words, uint64_t pair_seed, uint32_t npairs) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < n_words; w += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bit0 = w * 32;
    const int64_t r_first = bit0 / bits;
    const int64_t r_last = (bit0 + 31) / bits;
    uint32_t word = 0;
    for (int64_t r = r_first; r <= r_last; ++r) {
      if (r >= n_rows) break;
      const int64_t src = npairs ? static_cast<int64_t>(synth_value(pair_seed, r, npairs)) : r;
      const uint64_t v = synth_value(seed, src, card);
      // bits of row r occupy [r*bits, r*bits+bits); MSB-first.
      const int64_t rs = r * bits;
      // position of row's MSB relative to word start
      const int64_t off = rs - bit0;  // may be negative
      // shift so that the row's bits land in the word (bit 31 = first bit of the word)
      const int64_t sh = 32 - off - bits;  // left shift amount (may be negative)
      uint64_t placed;
      if (sh >= 0) placed = v << sh;
      else placed = v >> (-sh);
      word |= static_cast<uint32_t>(placed & 0xFFFFFFFFull);
    }
    out_words[w] = bswap32(word);
  }
}


// Realtime snapshot (pgx_mutable_snapshot): the fixed-bit forward index of dictIds remap[ids[r]] (arrival-order ids
// through the arrival -> sorted map; remap null: ids as they are), packed MSB-first big-endian like pgx_synth_kernel:
// one thread per 32-bit word, the rows that overlap it.
__global__ void pgx_pack_remap_kernel(uint32_t* out_words, const int32_t* __restrict__ ids,
                                      const int32_t* __restrict__ remap, int64_t n_rows, int bits, int64_t n_words) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < n_words; w += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bit0 = w * 32;
    const int64_t r_first = bit0 / bits;
    const int64_t r_last = (bit0 + 31) / bits;
    uint32_t word = 0;
    for (int64_t r = r_first; r <= r_last && r < n_rows; ++r) {
      const int32_t a = ids[r];
      const uint64_t v = static_cast<uint32_t>(remap ? remap[a] : a);
      const int64_t sh = 32 - (r * bits - bit0) - bits;
      word |= static_cast<uint32_t>((sh >= 0 ? v << sh : v >> (-sh)) & 0xFFFFFFFFull);
    }
    out_words[w] = bswap32(word);
  }
}

// ---------------------------------------------------------------------------------------------
// numEntriesScannedInFilter automaton (pgx_stats.cpp): the reference's iterator algebra restated as a finite automaton
// over each row's leaf-membership bits.  Pass 1: one thread per (1024-row chunk, start state) runs the chunk; pass 2:
// per segment, the chunk transitions are composed (threads over chunk ranges x start states, then one lane walks the
// range results from the initial state) and the total is added to stats[1].
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) pgx_fsm_chunks(const FsmSeg* __restrict__ segs, int nsegs,
                                                      const uint32_t* __restrict__ table, int S, int L,
                                                      int64_t total_chunks, uint32_t* __restrict__ out_count,
                                                      uint16_t* __restrict__ out_state) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gid >= total_chunks * S) return;
  const int64_t chunk = gid / S;
  uint32_t state = static_cast<uint32_t>(gid - chunk * S);
  int lo = 0, hi = nsegs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].chunk0 <= chunk) lo = mid; else hi = mid - 1;
  }
  const FsmSeg& G = segs[lo];
  const int32_t r0 = static_cast<int32_t>((chunk - G.chunk0) * kFsmChunkRows);
  const int32_t r1 = min(r0 + kFsmChunkRows, G.num_docs);
  int iv = 0;
  while (iv + 1 < G.nint && G.ibeg[iv + 1] <= r0) ++iv;
  int32_t cut = iv + 1 < G.nint ? G.ibeg[iv + 1] : 0x7FFFFFFF;
  const uint32_t* tab = table + (static_cast<uint64_t>(G.itab[iv]) * S << L);
  uint32_t count = 0;
  for (int32_t w = r0 >> 5; (w << 5) < r1; ++w) {
    uint32_t m[kFsmMaxLeaves];
#pragma unroll
    for (int l = 0; l < kFsmMaxLeaves; ++l) m[l] = l < L ? G.lmask[l * G.words + w] : 0u;
    const int jn = min(32, r1 - (w << 5));
    for (int j = 0; j < jn; ++j) {
      const int32_t r = (w << 5) + j;
      if (r >= cut) {
        ++iv;
        cut = iv + 1 < G.nint ? G.ibeg[iv + 1] : 0x7FFFFFFF;
        tab = table + (static_cast<uint64_t>(G.itab[iv]) * S << L);
      }
      uint32_t in = 0;
#pragma unroll
      for (int l = 0; l < kFsmMaxLeaves; ++l) in |= ((m[l] >> j) & 1u) << l;
      const uint32_t e = tab[(static_cast<uint64_t>(state) << L) | in];
      count += e & 0xFFFFu;
      state = e >> 16;
    }
  }
  out_count[gid] = count;
  out_state[gid] = static_cast<uint16_t>(state);
}

__global__ void __launch_bounds__(256) pgx_fsm_compose(const FsmSeg* __restrict__ segs, int S, int T,
                                                       const uint32_t* __restrict__ cnt,
                                                       const uint16_t* __restrict__ stv,
                                                       unsigned long long* __restrict__ pcount,
                                                       uint16_t* __restrict__ pstate,
                                                       unsigned long long* __restrict__ stats) {
  const FsmSeg& G = segs[blockIdx.x];
  const int64_t nch = (static_cast<int64_t>(G.num_docs) + kFsmChunkRows - 1) / kFsmChunkRows;
  const int64_t per = (nch + T - 1) / T;
  unsigned long long* pc = pcount + static_cast<int64_t>(blockIdx.x) * T * S;
  uint16_t* ps = pstate + static_cast<int64_t>(blockIdx.x) * T * S;
  for (int i = threadIdx.x; i < T * S; i += blockDim.x) {
    const int t = i / S;
    uint32_t q = static_cast<uint32_t>(i - t * S);
    unsigned long long c = 0;
    const int64_t c0 = t * per, c1 = min(nch, c0 + per);
    for (int64_t ch = c0; ch < c1; ++ch) {
      const int64_t e = (G.chunk0 + ch) * S + q;
      c += cnt[e];
      q = stv[e];
    }
    pc[i] = c;
    ps[i] = static_cast<uint16_t>(q);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long total = 0;
    uint32_t q = 0;  // the initial state: every iterator idle, the root's first next() pending
    for (int t = 0; t < T; ++t) {
      total += pc[t * S + q];
      q = ps[t * S + q];
    }
    if (total) atomicAdd(stats + 1, total);
  }
}

}  // namespace pgx

// ---------------------------------------------------------------------------------------------
// Host-side launchers (called from pgx_host.cpp)
// ---------------------------------------------------------------------------------------------
extern "C" hipError_t pgx_launch_scan(const pgx::KQuery* q, int grid, int64_t tiles_per_wg, size_t lds_bytes,
                                      hipStream_t stream) {
  switch (q->group_mode) {
    case pgx::G_NONE:
      hipLaunchKernelGGL(pgx::pgx_scan_kernel<pgx::G_NONE>, dim3(grid), dim3(pgx::kBlock), lds_bytes, stream, *q,
                         tiles_per_wg);
      break;
    case pgx::G_DENSE_LDS:
      hipLaunchKernelGGL(pgx::pgx_scan_kernel<pgx::G_DENSE_LDS>, dim3(grid), dim3(pgx::kBlock), lds_bytes, stream, *q,
                         tiles_per_wg);
      break;
    case pgx::G_DENSE_GLOBAL:
      hipLaunchKernelGGL(pgx::pgx_scan_kernel<pgx::G_DENSE_GLOBAL>, dim3(grid), dim3(pgx::kBlock), lds_bytes, stream,
                         *q, tiles_per_wg);
      break;
    case pgx::G_HASH64:
      hipLaunchKernelGGL(pgx::pgx_scan_kernel<pgx::G_HASH64>, dim3(grid), dim3(pgx::kBlock), lds_bytes, stream, *q,
                         tiles_per_wg);
      break;
    case pgx::G_HASH128:
      hipLaunchKernelGGL(pgx::pgx_scan_kernel<pgx::G_HASH128>, dim3(grid), dim3(pgx::kBlock), lds_bytes, stream, *q,
                         tiles_per_wg);
      break;
    case pgx::G_HASHW:
      if (q->key_words < 3 || q->key_words > pgx::kMaxKeyWords) return hipErrorInvalidValue;
      hipLaunchKernelGGL(pgx::pgx_scan_kernel<pgx::G_HASHW>, dim3(grid), dim3(pgx::kBlock), lds_bytes, stream, *q,
                         tiles_per_wg);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_init_planes(unsigned long long* table, uint64_t slots, int num_planes,
                                             const pgx::KQuery* q, unsigned long long* keys, uint64_t key_words,
                                             unsigned int* key_state, hipStream_t stream) {
  uint64_t n = slots * num_planes;
  if (key_words > n) n = key_words;
  int grid = static_cast<int>(std::min<uint64_t>((n + 255) / 256, 8192));
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(pgx::pgx_init_planes, dim3(grid), dim3(256), 0, stream, table, slots, num_planes, *q, keys,
                     key_words, key_state);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_compact(unsigned long long* table, uint64_t slots, int num_planes,
                                         unsigned long long* counter, int64_t* out_slot,
                                         unsigned long long* out_planes, uint64_t cap_out, int reset,
                                         uint32_t min_mask, hipStream_t stream) {
  if (reset && (slots > (uint64_t(1) << 20) || cap_out < slots || num_planes > 32)) return hipErrorInvalidValue;
  if (slots <= (uint64_t(1) << 20)) {
    const int grid = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>((slots + 255) / 256, 4096)));
    hipLaunchKernelGGL(pgx::pgx_compact_wave, dim3(grid), dim3(256), 0, stream, table, slots, num_planes, counter,
                       out_slot, out_planes, cap_out, reset, min_mask);
    return hipGetLastError();
  }
  int grid = static_cast<int>(std::min<uint64_t>((slots + 4095) / 4096, 4096));
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(pgx::pgx_compact, dim3(grid), dim3(256), 0, stream, table, slots, num_planes, counter, out_slot,
                     out_planes, cap_out);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_synth(uint32_t* out_words, int64_t n_rows, int bits, uint32_t card, uint64_t seed,
                                       int64_t n_words, uint64_t pair_seed, uint32_t npairs, hipStream_t stream) {
  int grid = static_cast<int>(std::min<int64_t>((n_words + 255) / 256, 65536));
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(pgx::pgx_synth_kernel, dim3(grid), dim3(256), 0, stream, out_words, n_rows, bits, card, seed,
                     n_words, pair_seed, npairs);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_pack_remap(uint32_t* out_words, const int32_t* ids, const int32_t* remap,
                                            int64_t n_rows, int bits, int64_t n_words, hipStream_t stream) {
  if (n_words <= 0) return hipSuccess;
  if (bits < 1 || bits > 32 || !out_words || (n_rows > 0 && !ids)) return hipErrorInvalidValue;
  const int grid = static_cast<int>(std::min<int64_t>((n_words + 255) / 256, 65536));
  hipLaunchKernelGGL(pgx::pgx_pack_remap_kernel, dim3(grid), dim3(256), 0, stream, out_words, ids, remap, n_rows, bits,
                     n_words);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_roaring(const pgx::RDesc* descs, int npairs, int maxchunks, hipStream_t stream) {
  if (npairs <= 0 || maxchunks <= 0) return hipSuccess;
  const long long blocks = static_cast<long long>(npairs) * maxchunks;
  if (blocks > 0x7FFFFFFFll) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pgx::pgx_roaring_expand, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, descs, npairs,
                     maxchunks);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_partition(const uint64_t* in, const int64_t* in_off, const unsigned long long* in_cnt,
                                           int in_cstride, int nreg, int reg_div, int64_t in_cap, int chunks_per_reg,
                                           uint64_t keymask, int shift, int nbits, uint64_t* out, int64_t cap,
                                           unsigned long long* cursor, int cstride, unsigned long long* overflow,
                                           hipStream_t stream) {
  const long long blocks = static_cast<long long>(nreg) * chunks_per_reg;
  if (blocks <= 0) return hipSuccess;
  // nbits 0: one partition per region group (gathers the scan's slabs of a bucket into one contiguous run)
  if (blocks > 0x7FFFFFFFll || nbits > 8 || nbits < 0 || reg_div < 1 || shift < 1 || shift > 63) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pgx::pgx_partition, dim3(static_cast<unsigned>(blocks)), dim3(pgx::kPartThreads), 0, stream, in,
                     in_off, in_cnt, in_cstride, nreg, reg_div, in_cap, chunks_per_reg, keymask, shift, nbits, out, cap,
                     cursor, cstride, overflow);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_part_aggregate(const uint64_t* in, const unsigned long long* in_cnt, int cstride,
                                                int nparts, int64_t cap, uint64_t keymask, int keybits, int64_t vbase,
                                                int need_sum, int need_min, int need_max, int pack_shift,
                                                uint64_t* okey, uint64_t* oplane, int64_t ocap,
                                                unsigned long long* ocount, unsigned long long* overflow,
                                                hipStream_t stream) {
  (void)need_sum;  // sums are always accumulated (one add)
  if (nparts <= 0) return hipSuccess;
  const int sel = (pack_shift ? 4 : 0) | (need_min ? 2 : 0) | (need_max ? 1 : 0);
#define PGX_AGG_CASE(K, A, B, C)                                                                                    \
  case K:                                                                                                            \
    hipLaunchKernelGGL((pgx::pgx_part_aggregate<A, B, C>), dim3(nparts), dim3(pgx::kAggThreads), 0, stream, in,     \
                       in_cnt, cstride, cap, keymask, keybits, vbase, pack_shift, okey, oplane, ocap, ocount,       \
                       overflow);                                                                                   \
    break;
  switch (sel) {
    PGX_AGG_CASE(0, false, false, false)
    PGX_AGG_CASE(1, false, false, true)
    PGX_AGG_CASE(2, false, true, false)
    PGX_AGG_CASE(3, false, true, true)
    PGX_AGG_CASE(4, true, false, false)
    PGX_AGG_CASE(5, true, false, true)
    PGX_AGG_CASE(6, true, true, false)
    PGX_AGG_CASE(7, true, true, true)
  }
#undef PGX_AGG_CASE
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_part_aggregate_f64(const uint64_t* in, const unsigned long long* in_cnt, int cstride,
                                                    int nparts, int64_t cap, uint64_t keymask, int keybits,
                                                    const double* fdict, int need_min, int need_max, uint64_t* okey,
                                                    uint64_t* oplane, int64_t ocap, unsigned long long* ocount,
                                                    unsigned long long* overflow, hipStream_t stream) {
  if (nparts <= 0) return hipSuccess;
  if (!fdict || keybits < 1 || keybits > 63) return hipErrorInvalidValue;
  const int sel = (need_min ? 2 : 0) | (need_max ? 1 : 0);
#define PGX_AGGF_CASE(K, B, C)                                                                                      \
  case K:                                                                                                            \
    hipLaunchKernelGGL((pgx::pgx_part_aggregate_f64<B, C>), dim3(nparts), dim3(pgx::kAggThreads), 0, stream, in,    \
                       in_cnt, cstride, cap, keymask, keybits, fdict, okey, oplane, ocap, ocount, overflow);         \
    break;
  switch (sel) {
    PGX_AGGF_CASE(0, false, false)
    PGX_AGGF_CASE(1, false, true)
    PGX_AGGF_CASE(2, true, false)
    PGX_AGGF_CASE(3, true, true)
  }
#undef PGX_AGGF_CASE
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_fsm(const pgx::FsmSeg* segs, int nsegs, const uint32_t* table, int S, int L,
                                     int64_t total_chunks, uint32_t* cnt, uint16_t* stv, unsigned long long* pcount,
                                     uint16_t* pstate, int T, unsigned long long* stats, hipStream_t stream) {
  const int64_t threads = total_chunks * S;
  if (threads > 0) {
    const unsigned grid = static_cast<unsigned>((threads + 255) / 256);
    hipLaunchKernelGGL(pgx::pgx_fsm_chunks, dim3(grid), dim3(256), 0, stream, segs, nsegs, table, S, L, total_chunks,
                       cnt, stv);
  }
  if (nsegs > 0)
    hipLaunchKernelGGL(pgx::pgx_fsm_compose, dim3(nsegs), dim3(256), 0, stream, segs, S, T, cnt, stv, pcount, pstate,
                       stats);
  return hipGetLastError();
}

// Wave-per-chunk bitmap programs (host: every program <= 64 bitmaps and <= 3 slots).
extern "C" hipError_t pgx_launch_roaring_program_wave(const pgx::RProg* progs, const pgx::RDesc* descs, int nprogs,
                                                      int maxchunks, int nslots, hipStream_t stream) {
  if (nprogs <= 0 || maxchunks <= 0) return hipSuccess;
  // ~8192 waves (four rounds of 256 CUs x 8 resident), at most one per chunk
  int parts = std::max(1, std::min(maxchunks, (8192 + nprogs - 1) / nprogs));
  const long long waves = static_cast<long long>(nprogs) * parts;
  // waves per SIMD the LDS allows (NS x 8 KiB per wave) bound the registers: 1 slot -> 4, 2 -> 2, 3 -> 1
#define PGX_WAVE_LAUNCH(NS, WPB, MINW)                                                                             \
  hipLaunchKernelGGL((pgx::pgx_roaring_program_wave<NS, WPB, MINW>),                                              \
                     dim3(static_cast<unsigned>((waves + WPB - 1) / WPB)), dim3(64 * WPB),                        \
                     static_cast<size_t>(NS) * WPB * 2048 * 4, stream, progs, descs, nprogs, parts)
  if (nslots <= 1) PGX_WAVE_LAUNCH(1, 4, 4);
  else if (nslots == 2) PGX_WAVE_LAUNCH(2, 2, 2);
  else PGX_WAVE_LAUNCH(3, 2, 1);
#undef PGX_WAVE_LAUNCH
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_roaring_program(const pgx::RProg* progs, const pgx::RDesc* descs, int nprogs,
                                                 int maxchunks, int maxleaves, hipStream_t stream) {
  if (nprogs <= 0 || maxchunks <= 0) return hipSuccess;
  const long long blocks = static_cast<long long>(nprogs) * maxchunks;
  if (maxleaves < 0 && -maxleaves <= pgx::kRProgMaxLeaves) {  // per-segment walk (host: every program <= 512 bitmaps)
    // at least ~2048 workgroups (two full rounds at 4 resident per CU on 256 CUs), at most 8 parts per segment
    int parts = std::max(1, std::min(std::min(maxchunks, 8), (2048 + nprogs - 1) / nprogs));
      hipLaunchKernelGGL(pgx::pgx_roaring_program_seg, dim3(static_cast<unsigned>(nprogs * parts)),
                       dim3(pgx::kSegRThreads), static_cast<size_t>(-maxleaves) * 2048 * 4, stream, progs, descs,
                       nprogs, parts);
    return hipGetLastError();
  }
  if (maxleaves >= 1 && maxleaves <= pgx::kRProgMaxLeaves) {
    hipLaunchKernelGGL(pgx::pgx_roaring_program_wide, dim3(static_cast<unsigned>(blocks)), dim3(256),
                       static_cast<size_t>(maxleaves) * 2048 * 4, stream, progs, descs, nprogs, maxchunks);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(pgx::pgx_roaring_program, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, progs, descs,
                     nprogs, maxchunks);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_mv_leaf_mask(const pgx::MvLeaf* items, int nitems, int max_words, hipStream_t stream) {
  if (nitems <= 0 || max_words <= 0) return hipSuccess;
  hipLaunchKernelGGL(pgx::pgx_mv_leaf_mask, dim3(static_cast<unsigned>((max_words + 255) / 256),
                                                   static_cast<unsigned>(nitems)),
                     dim3(256), 0, stream, items, nitems, max_words);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_mv_aggregate(const pgx::MvAgg* items, int nitems, int max_words, hipStream_t stream) {
  if (nitems <= 0 || max_words <= 0) return hipSuccess;
  hipLaunchKernelGGL(pgx::pgx_mv_aggregate, dim3(static_cast<unsigned>((max_words + 255) / 256),
                                                   static_cast<unsigned>(nitems)),
                     dim3(256), 0, stream, items, nitems);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_mv_group(const pgx::MvGroupArgs* args, int nsegs, int max_docs, int ordered,
                                          hipStream_t stream) {
  if (nsegs <= 0 || max_docs <= 0) return hipSuccess;
  hipLaunchKernelGGL(pgx::pgx_mv_group, dim3(static_cast<unsigned>((max_docs + 255) / 256), static_cast<unsigned>(nsegs)),
                     dim3(256), 0, stream, args);
  if (ordered) hipLaunchKernelGGL(pgx::pgx_mv_group_ordered, dim3(static_cast<unsigned>(nsegs)), dim3(256), 0, stream, args);
  return hipGetLastError();
}
