// Narrow partitioned group-by: the second split and the aggregation (pgx_part.cpp run_narrow).
//
// Sparse group keys (LONG_MAP_BASED, DefaultGroupKeyGenerator.java:239-246 / :429-441: the packed raw key probes a
// Long2IntOpenHashMap per doc; SumAggregationFunction.aggregateGroupBySV, MinAggregationFunction / Max... per doc) are
// aggregated without a device-wide hash table and without 8-byte records:
//   1. the generated scan kernel (pgx_jit.cpp, part_narrow) mixes each selected row's key with a bijection of [0, 2^K)
//      (NarrowMix), splits the rows 256 ways on the mix's top 8 bits inside its LDS and appends to its own slab of each
//      bucket: K - 8 bits of the mix + the value's dictId, as a u32 (+ a u16 when wider than 32 bits);
//   2. pgx_narrow_split: one workgroup per bucket reads the bucket's slabs and splits them 2^k2 ways on the next bits of
//      the mix into partitions of u32 records (the remaining mix bits + the dictId, <= 32 bits by construction);
//   3. pgx_narrow_aggregate: every wavefront owns a small LDS hash table and aggregates one partition at a time (count
//      and value sum in one 64-bit LDS add, MIN / MAX over dictIds: numeric dictionaries are sorted, so the extreme
//      dictId is the extreme value), with the value column's image (FOR16 / U32) in the workgroup's LDS; then rebuilds
//      each group's packed key from the partition index and the record bits (the mix's inverse) and appends the group.
// Record bytes per row: 6 written + 6 read + 4 written + 4 read, against 8 B through two radix passes (40 B) before.
// The output layout (packed key + count / int64 sum / ordered min / ordered max planes) is pgx_part_aggregate's, so the
// trim, gather, decode and cross-device merges are shared.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "pgx_internal.h"

#define PGX_GLOBAL __attribute__((address_space(1)))

namespace pgx {
namespace {

__device__ __forceinline__ void n_lds_barrier() {  // LDS-only ordering: loads in flight are not drained
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---------------------------------------------------------------------------------------------------------------------
// Second split.  Bucket b's records: slab w (one per scan workgroup) holds cnt1[b * nwg + w] records (u32 at
// lo[(b * nwg + w) * cap1 + i], bits 32.. at hi[same] when hi != null).  A record is r1 | d << rb1 (r1: the mix's low
// rb1 bits, d: the value's dictId); sub-bucket = r1's top k2 bits; the output record is (r1's low rb1 - k2 bits) |
// d << (rb1 - k2), appended to partition (b << k2 | sub) at out[part * cap2 + i], its count in cnt2[part].
// ---------------------------------------------------------------------------------------------------------------------
typedef unsigned int na_u32x4 __attribute__((ext_vector_type(4)));
constexpr int kN2Threads = 1024;
constexpr int kN2Waves = kN2Threads / 64;
constexpr int kN2Per = 8;
constexpr int kN2Chunk = kN2Threads * kN2Per;  // records per round
constexpr int kN2MaxSub = 1 << kNarrowMaxBits2;
constexpr int kN2MaxSlabs = 1024;
constexpr int kN2RingWords = 32768;             // 128 KiB of LDS rings: 32768 >> k2 records per sub-bucket
constexpr int kN2Unit = 16;                     // records per unit: one 64-byte line segment
constexpr int kN2ListCap = kN2Chunk / kN2Unit + kN2MaxSub;  // units that can complete in one round

// Software write combining, as in the scan (pgx_jit.cpp narrow sub-step): sub-bucket s's records take consecutive
// positions of partition (b << k2 | s) (an LDS cursor per sub-bucket: the atomic returns the position) and wait in the
// sub-bucket's LDS ring (position mod ring) until their 16-record unit is complete; whole units leave as 64 contiguous
// bytes written by 16 consecutive lanes.  Partial-unit stores would leave as separate partial-line writes.
// Rounds walk the bucket's slabs in order: round (w, c0) holds records [c0, c0 + kN2Chunk) of slab w, so a record's
// address is plain arithmetic; the loads of the next two rounds are in flight.  Per round:
//   split fields, positions (LDS atomics)
//   | A | owner lanes (one per sub-bucket) list the units that complete (one LDS atomic per wavefront reserves list
//   space), every lane writes its records into the rings (a record past its ring -- key skew -- goes straight out)
//   | B | the listed units are written out, four per wavefront instruction.
// U (first unflushed position, a unit boundary) and V (ring-valid-from: positions below it were stored straight out)
// are double-buffered so the owners write the next round's while this round's are read.
// W: u32 words per output record -- 1, or 2 when the remaining key bits and the value field need more than 32 bits
// (value offsets of per-segment dictionaries, c3d): the rings then hold kN2RingWords / 2 records and a 64-byte unit 8.
template <int W>
__global__ void __launch_bounds__(kN2Threads) pgx_narrow_split(const uint32_t* __restrict__ lo,
                                                               const uint16_t* __restrict__ hi,
                                                               const unsigned long long* __restrict__ cnt1, int nwg,
                                                               int64_t cap1, int rb1, int k2,
                                                               uint32_t* __restrict__ out, int64_t cap2,
                                                               unsigned int* __restrict__ cnt2,
                                                               unsigned long long* __restrict__ ovf) {
  __shared__ __attribute__((aligned(16))) uint32_t ring[kN2RingWords];
  __shared__ uint32_t cur[kN2MaxSub], Ub[2][kN2MaxSub], Vb[2][kN2MaxSub];
  __shared__ uint16_t lsub[kN2ListCap];
  __shared__ uint32_t lpos[kN2ListCap];
  __shared__ uint32_t lcnt[2];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nsub = 1 << k2;
  const int rb2 = rb1 - k2;
  constexpr int UR = kN2Unit / W;  // records per 64-byte unit
  const int rlog = (W == 2 ? 14 : 15) - k2;  // ring records per sub-bucket: 2^rlog
  const uint32_t rmask = (1u << rlog) - 1u;
  const uint64_t m2 = (uint64_t(1) << rb2) - 1u;
  const uint32_t ucap = static_cast<uint32_t>(cap2 < 0xFFFFFFFFll ? cap2 : 0xFFFFFFFFll);
  for (int i = tid; i < nsub; i += kN2Threads) {
    cur[i] = 0u;
    Ub[0][i] = 0u;
    Vb[0][i] = 0u;
  }
  if (tid < 2) lcnt[tid] = 0u;
  __syncthreads();
  const unsigned long long* const c1 = cnt1 + static_cast<int64_t>(b) * nwg;
  auto scount = [&](int w) -> uint32_t {  // records of slab w (uniform)
    const unsigned long long c = c1[w];
    return static_cast<uint32_t>(c < static_cast<unsigned long long>(cap1) ? c : static_cast<unsigned long long>(cap1));
  };
  const PGX_GLOBAL uint32_t* glo = (const PGX_GLOBAL uint32_t*)lo + static_cast<int64_t>(b) * nwg * cap1;
  const PGX_GLOBAL uint16_t* ghi = hi ? (const PGX_GLOBAL uint16_t*)hi + static_cast<int64_t>(b) * nwg * cap1 : nullptr;
  PGX_GLOBAL uint32_t* gout = (PGX_GLOBAL uint32_t*)out + static_cast<int64_t>(b) * nsub * cap2 * W;
  // record i of sub-bucket sb: words [(sb * cap2 + i) * W, + W) of gout; ring slot (sb << rlog) + (i & rmask) likewise
  auto put_out = [&](uint32_t sb, uint32_t i, uint64_t r) {
    const int64_t at = (static_cast<int64_t>(sb) * cap2 + i) * W;
    if (W == 2) *(PGX_GLOBAL uint64_t*)(gout + at) = r;
    else gout[at] = static_cast<uint32_t>(r);
  };
  auto put_ring = [&](uint32_t slot, uint64_t r) {
    if (W == 2) *reinterpret_cast<uint64_t*>(ring + 2 * slot) = r;
    else ring[slot] = static_cast<uint32_t>(r);
  };
  auto get_ring = [&](uint32_t slot) -> uint64_t {
    return W == 2 ? *reinterpret_cast<const uint64_t*>(ring + 2 * slot) : static_cast<uint64_t>(ring[slot]);
  };
  struct Rd {
    int w;
    uint32_t c0, n;
  };
  // the round after r (or the first at or after (w, 0)): slabs with no records left are skipped
  auto advance = [&](Rd r) -> Rd {
    r.c0 += kN2Chunk;
    while (r.w < nwg && r.c0 >= r.n) {
      ++r.w;
      r.c0 = 0u;
      r.n = r.w < nwg ? scount(r.w) : 0u;
    }
    return r;
  };
  auto load = [&](Rd r, uint32_t (&xl)[kN2Per], uint32_t (&xh)[kN2Per]) {
    const PGX_GLOBAL uint32_t* sl = glo + static_cast<int64_t>(r.w) * cap1;
#pragma unroll
    for (int k = 0; k < kN2Per; ++k) {
      const uint32_t pos = r.c0 + static_cast<uint32_t>(k * kN2Threads + tid);
      xl[k] = pos < r.n ? __builtin_nontemporal_load(sl + pos) : 0u;
      xh[k] = (ghi && pos < r.n) ? __builtin_nontemporal_load(ghi + static_cast<int64_t>(r.w) * cap1 + pos) : 0u;
    }
  };
  uint32_t l0[kN2Per], h0[kN2Per], l1[kN2Per], h1[kN2Per], l2[kN2Per], h2[kN2Per];
  Rd r0{0, 0u - static_cast<uint32_t>(kN2Chunk), nwg > 0 ? scount(0) : 0u};
  r0 = advance(r0);
  if (r0.w < nwg) load(r0, l0, h0);
  Rd r1 = advance(r0);
  if (r1.w < nwg) load(r1, l1, h1);
  int par = 0;
  while (r0.w < nwg) {
    const Rd r2n = advance(r1);
    if (r2n.w < nwg) load(r2n, l2, h2);
    // split fields and positions
    uint64_t rec[kN2Per];
    uint32_t sbp[kN2Per];  // sbp: sub-bucket | valid << 31
    uint32_t pp[kN2Per];
#pragma unroll
    for (int k = 0; k < kN2Per; ++k) {
      const uint32_t pos = r0.c0 + static_cast<uint32_t>(k * kN2Threads + tid);
      const uint64_t x = static_cast<uint64_t>(l0[k]) | (static_cast<uint64_t>(h0[k]) << 32);
      rec[k] = (x & m2) | ((x >> rb1) << rb2);
      const uint32_t sb = static_cast<uint32_t>(x >> rb2) & static_cast<uint32_t>(nsub - 1);
      sbp[k] = pos < r0.n ? (sb | 0x80000000u) : 0u;
      pp[k] = pos < r0.n ? atomicAdd(&cur[sb], 1u) : 0u;
    }
    n_lds_barrier();  // A
    const uint32_t* const Uc = Ub[par];
    const uint32_t* const Vc = Vb[par];
    if (wave * 64 < nsub) {  // owner lanes: sub-bucket tid
      uint32_t nu = 0u, en = 0u, u0 = 0u, v0 = 0u;
      if (tid < nsub) {
        en = cur[tid];
        u0 = Uc[tid];
        v0 = Vc[tid];
        const uint32_t lim = u0 + (1u << rlog);
        nu = ((en < lim ? en : lim) - u0) / UR;
        Ub[par ^ 1][tid] = en & ~static_cast<uint32_t>(UR - 1);
        Vb[par ^ 1][tid] = en > lim ? en : v0;
      }
      uint32_t incl = nu;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      const uint32_t tot = __shfl(incl, 63, 64);
      uint32_t base = 0u;
      if (lane == 0 && tot) base = atomicAdd(&lcnt[par], tot);
      base = __shfl(base, 0, 64);
      for (uint32_t q = 0, k = base + incl - nu; q < nu; ++q, ++k) {
        lsub[k] = static_cast<uint16_t>(tid);
        lpos[k] = u0 + q * UR;
      }
    }
    if (tid == 0) lcnt[par ^ 1] = 0u;  // the next round's list (its reservations follow barrier B)
#pragma unroll
    for (int k = 0; k < kN2Per; ++k) {
      if (!sbp[k]) continue;
      const uint32_t sb = sbp[k] & 0x7FFFFFFFu;
      const uint32_t pos = pp[k];
      if (pos < Uc[sb] + (1u << rlog)) put_ring((sb << rlog) + (pos & rmask), rec[k]);
      else if (pos < ucap) put_out(sb, pos, rec[k]);  // past the ring: straight out
    }
    n_lds_barrier();  // B
    {  // four lanes per unit, 16 bytes each; a unit holding positions below V goes record by record
      const uint32_t n = lcnt[par];
      const int g = lane & 3;
      for (uint32_t u = static_cast<uint32_t>(wave * 16 + (lane >> 2)); u < n; u += kN2Waves * 16) {
        const uint32_t sb = lsub[u];
        const uint32_t p0 = lpos[u];
        if (p0 >= ucap) continue;
        PGX_GLOBAL uint32_t* const dst = gout + (static_cast<int64_t>(sb) * cap2 + p0) * W + 4 * g;
        const uint32_t* const rs = ring + ((sb << rlog) + (p0 & rmask)) * W + 4 * g;
        if (p0 >= Vc[sb]) {
          *(PGX_GLOBAL na_u32x4*)dst = *(const na_u32x4*)rs;
        } else {  // this lane's 4 / W records, each only if it was not stored straight out
          for (int q = 0; q < 4 / W; ++q)
            if (p0 + (4 / W) * g + q >= Vc[sb])
              for (int w = 0; w < W; ++w) dst[q * W + w] = rs[q * W + w];
        }
      }
    }
    par ^= 1;
#pragma unroll
    for (int k = 0; k < kN2Per; ++k) {
      l0[k] = l1[k];
      h0[k] = h1[k];
      l1[k] = l2[k];
      h1[k] = h2[k];
    }
    r0 = r1;
    r1 = r2n;
  }
  __syncthreads();
  // the rings' last partial units, then the partition fills (every record, also past cap2)
  for (int x = tid; x < nsub * UR; x += kN2Threads) {
    const int sb = x / UR;
    const uint32_t i = Ub[par][sb] + static_cast<uint32_t>(x % UR);
    if (i < cur[sb] && i >= Vb[par][sb] && i < ucap) put_out(sb, i, get_ring((sb << rlog) + (i & rmask)));
  }
  for (int sb = tid; sb < nsub; sb += kN2Threads) {
    cnt2[static_cast<int64_t>(b) * nsub + sb] = cur[sb];
    if (cur[sb] > ucap) atomicAdd(ovf, 1ull);
  }
}

// ---------------------------------------------------------------------------------------------------------------------
// Aggregation.  Wavefront-private open-addressing tables of kNABuckets 4-way buckets (16 contiguous bytes of keys,
// read with ONE ds_read_b128): key bits, count << cshift | value sum, min dictId, max dictId.  A wavefront takes
// partitions p = its global index, + all wavefronts, ...; the next 1024 records (of this partition or the next) are
// loaded while the current ones are aggregated.  Records are resolved 8 at a time: the 8 home buckets and the 8 values
// are read back to back (one LDS round trip for all), a key found in its home bucket -- every record of a group but
// its first, unless the bucket overflowed -- goes straight to the fire-and-forget LDS atomics, and only the others take
// the probing loop (insert by CAS, then neighbouring buckets).  The record's value field is a dictId whose value the
// workgroup's LDS image holds (IMG 1: u32 value - vbase per dictId, 2: FOR16 = 64 u32 block bases + u16 offset per
// dictId), or the dictId of a MIN / MAX-only column looked up in vdict at the flush (IMG 0), or the value offset itself
// (IMG 3: value - vbase; no image, so the LDS holds only the tables and more wavefronts fit a CU), or the value's index
// in a table of the query's distinct dictionaries in global memory (L2-resident; segments with their own dictionaries,
// c3d / c3f): IMG 5 gathers value - vbase (u32) and then aggregates as IMG 3, IMG 6 gathers the double and keeps count,
// f64 sum (LDS f64 add) and ordered-f64 min / max per slot (pgx_part_aggregate_f64's planes).  The gathers of batch i + 1
// are issued while batch i is aggregated.
// ctr: [0] groups appended, [3] overflow (a table filled up, or more groups than ocap).
// ---------------------------------------------------------------------------------------------------------------------
constexpr int kNAWays = 4;
constexpr int kNABuckets = 48;
constexpr int kNASlots = kNABuckets * kNAWays;  // 192
constexpr int kNAImgWords = 64 + 65536 / 2;
// IMG 4 (packed frame of reference): 1024-thread workgroups, so 16 wavefront tables (60 KiB) sit beside the image
constexpr int kNAImg4Words = (160 * 1024 - 16 * kNASlots * 20 - 1024) / 4;
constexpr uint32_t kNAEmpty = 0xFFFFFFFFu;
template <int IMG>
constexpr int na_threads() {
  return IMG == 4 ? 1024 : 512;
}

__device__ __forceinline__ unsigned long long oplane_sum_key(int64_t sum) {  // trim_key(SUM)
  return static_cast<unsigned long long>(sum) ^ 0x8000000000000000ull;
}

// IMG 4: img_sh packs the block shift (bits 0-4), the offset width b (bits 5-9) and the number of block bases (bits
// 10..): the image is nblk u32 bases, then the b-bit offsets packed LSB-first into dwords (plus one pad dword).
template <int IMG>
__device__ __forceinline__ uint32_t na_img(const uint32_t* simg, int img_sh, uint32_t d) {
  if (IMG == 1) return simg[d];
  if (IMG == 2) return simg[d >> img_sh] + static_cast<uint32_t>(reinterpret_cast<const uint16_t*>(simg + 64)[d]);
  if (IMG == 3 || IMG == 5) return d;
  if (IMG == 4) {
    const int sh = img_sh & 31, b = (img_sh >> 5) & 31, nb = img_sh >> 10;
    const uint32_t bp = d * static_cast<uint32_t>(b);
    const uint32_t* pk = simg + nb + (bp >> 5);
    const uint32_t off = __builtin_amdgcn_alignbit(pk[1], pk[0], bp & 31u) & ((1u << b) - 1u);
    return simg[d >> sh] + off;
  }
  return 0u;
}

__device__ __forceinline__ int na_way(const na_u32x4 k, uint32_t key) {
  return k.x == key ? 0 : k.y == key ? 1 : k.z == key ? 2 : k.w == key ? 3 : -1;
}

// W: u32 words per record (pgx_narrow_split<W>); W = 2 carries value offsets wider than the 32-bit record leaves room
// for (IMG 3 only): 512 records per batch instead of 1024, the same 4 KiB per wavefront.
template <int IMG, bool SUM, bool MN, bool MX, int W>
__global__ void __launch_bounds__(na_threads<IMG>()) __attribute__((amdgpu_waves_per_eu(IMG >= 5 ? 2 : (IMG >= 3 ? 4 : 1))))
pgx_narrow_aggregate(
    const uint32_t* __restrict__ in, const unsigned int* __restrict__ cnt2, int64_t cap2, int nparts, int rb2,
    uint64_t kmask, uint64_t ic1, int ms, int64_t vbase, const uint32_t* __restrict__ img, int img_words,
    int img_sh, const int64_t* __restrict__ vdict, int cshift, uint64_t* __restrict__ rkey,
    uint64_t* __restrict__ rplane, int64_t wcap, int64_t rstride, unsigned long long* __restrict__ wcount,
    unsigned long long* __restrict__ ctr, unsigned long long* __restrict__ prange) {
  constexpr int kNAThreads = na_threads<IMG>();
  constexpr int kNAWaves = kNAThreads / 64;
  constexpr bool LIMG = IMG == 1 || IMG == 2 || IMG == 4;  // an image in LDS
  constexpr bool BIG = IMG == 1 || IMG == 2;               // 512 threads, two waves per SIMD: wider batches
  constexpr bool GATHER = IMG >= 5;                         // values gathered from a global table (img)
  constexpr bool F64 = IMG == 6;                            // ... doubles: count, f64 sum, ordered-f64 min / max
  constexpr bool PIPE3 = BIG || GATHER;                     // three batches in registers
  constexpr int LQ = 4;                                    // 16-byte loads per lane per batch (GATHER in half
                                                           // batches at four waves per SIMD measured slower)
  constexpr int BW = 4 * LQ;                               // u32 words per lane per batch
  constexpr int NR = BW / W;                               // records per lane per batch
  constexpr uint32_t BATCH = 64u * NR;
  typedef typename std::conditional<F64, unsigned long long, uint32_t>::type MT;  // min / max slot type
  typedef typename std::conditional<F64, double, uint32_t>::type GT;              // gathered value type
  __shared__ __attribute__((aligned(16))) uint32_t simg[LIMG ? (IMG == 4 ? kNAImg4Words : kNAImgWords) : 1];
  __shared__ __attribute__((aligned(16))) uint32_t tkey[kNAWaves * kNASlots];
  __shared__ unsigned long long tsc[kNAWaves * kNASlots];
  __shared__ uint32_t tcn[F64 ? kNAWaves * kNASlots : 1];
  __shared__ MT tmn[MN ? kNAWaves * kNASlots : 1], tmx[MX ? kNAWaves * kNASlots : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (LIMG) {
    const PGX_GLOBAL uint32_t* gi = (const PGX_GLOBAL uint32_t*)img;
    for (int i = tid; i < img_words; i += kNAThreads) simg[i] = gi[i];
  }
  for (int i = tid; i < kNAWaves * kNASlots; i += kNAThreads) {
    tkey[i] = kNAEmpty;
    tsc[i] = 0ull;  // (F64: the bits of 0.0)
    if (F64) tcn[i] = 0u;
    if (MN) tmn[i] = static_cast<MT>(~0ull);
    if (MX) tmx[i] = static_cast<MT>(0);
  }
  __syncthreads();  // the only workgroup barrier: wavefronts run independently from here on
  uint32_t* K = tkey + wave * kNASlots;
  unsigned long long* S = tsc + wave * kNASlots;
  MT* N = tmn + (MN ? wave * kNASlots : 0);
  MT* X = tmx + (MX ? wave * kNASlots : 0);
  uint32_t* C = tcn + (F64 ? wave * kNASlots : 0);
  const PGX_GLOBAL GT* gtab = (const PGX_GLOBAL GT*)img;  // GATHER: the value table
  const uint32_t rmask = rb2 >= 32 ? 0xFFFFFFFFu : (1u << rb2) - 1u;
  // home bucket of key bits r2 < 2^rb2: (r2 * kNABuckets) >> rb2, as one 32-bit high multiply
  const int hsh = rb2 >= 1 ? 32 - rb2 : 31;
  auto home = [&](uint32_t r2) -> uint32_t {
    return rb2 >= 1 ? __umulhi(r2 << hsh, static_cast<uint32_t>(kNABuckets)) : 0u;
  };
  const unsigned long long one = 1ull << cshift;
  const unsigned long long smask = one - 1ull;
  const int nw = gridDim.x * kNAWaves;
  const PGX_GLOBAL na_u32x4* src = (const PGX_GLOBAL na_u32x4*)in;
  const PGX_GLOBAL int64_t* vd = (const PGX_GLOBAL int64_t*)vdict;
  bool lost = false;

  auto load = [&](int pp, uint32_t i0, uint32_t nn, uint32_t (&buf)[BW]) {
    const int64_t base = ((static_cast<int64_t>(pp) * cap2 + i0) * W) >> 2;  // cap2 and i0 are multiples of 4
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
      const uint32_t e = static_cast<uint32_t>(q * (256 / W) + lane * (4 / W));
      na_u32x4 x = {0u, 0u, 0u, 0u};
      if (i0 + e < nn) x = __builtin_nontemporal_load(src + base + q * 64 + lane);
      buf[4 * q] = x.x;
      buf[4 * q + 1] = x.y;
      buf[4 * q + 2] = x.z;
      buf[4 * q + 3] = x.w;
    }
  };
  // slot of key r2 whose home bucket b did not hold it: empty ways are claimed by CAS, then the next buckets
  auto probe = [&](uint32_t r2, uint32_t b) -> int {
    for (int t = 0; t < kNABuckets;) {
      const na_u32x4 k = *reinterpret_cast<const na_u32x4*>(K + b * kNAWays);
      const int m = na_way(k, r2);
      if (m >= 0) return static_cast<int>(b) * kNAWays + m;
      const int e = k.x == kNAEmpty ? 0 : k.y == kNAEmpty ? 1 : k.z == kNAEmpty ? 2 : k.w == kNAEmpty ? 3 : -1;
      if (e >= 0) {
        const uint32_t prev = atomicCAS(&K[b * kNAWays + e], kNAEmpty, r2);
        if (prev == kNAEmpty || prev == r2) return static_cast<int>(b) * kNAWays + e;
        continue;  // another lane took that way first: look at the bucket again
      }
      b = b + 1u == static_cast<uint32_t>(kNABuckets) ? 0u : b + 1u;
      ++t;
    }
    return -1;
  };
  // A finished partition: its groups move to registers (<= 3 slots per lane) and the table is cleared; the rows are
  // written at the NEXT partition's end (flush_end), into this wavefront's own region of the scratch output (wcap rows:
  // its partitions times the table size, so it cannot run over).  No output row is reserved with a device atomic: one
  // counter for every partition's reservation serialised 2^18 atomics at C3 (~11 ns each at one L2 address, ~2.9 ms);
  // pgx_narrow_compact packs the regions afterwards.
  constexpr int Q = kNASlots / 64;
  uint32_t fk[Q], fcn[F64 ? Q : 1], fhas = 0, fexcl = 0;
  MT fn_[Q], fx[Q];
  unsigned long long fbase = 0ull, cursor = 0ull;  // (wave-uniform) rows this wavefront has written
  unsigned long long fsc[Q];
  int fp = -1;
  const int64_t gw = static_cast<int64_t>(blockIdx.x) * kNAWaves + wave;
  uint64_t* const wkey = rkey + gw * wcap;
  uint64_t* const wpl = rplane + gw * wcap;
  // trim-key ranges of the written groups (pgx_trim.hip trim_key: COUNT, SUM, MIN, MAX), so the trim skips its range
  // pass: [kind] smallest, [4 + kind] largest
  unsigned long long rlo[4] = {~0ull, ~0ull, ~0ull, ~0ull}, rhi[4] = {0ull, 0ull, 0ull, 0ull};
  auto note = [&](int k, unsigned long long x) {
    rlo[k] = x < rlo[k] ? x : rlo[k];
    rhi[k] = x > rhi[k] ? x : rhi[k];
  };
  auto flush_end = [&]() {
    if (fp < 0) return;
    unsigned long long o = fbase + fexcl;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (!((fhas >> q) & 1u)) continue;
      if (o < static_cast<unsigned long long>(wcap)) {
        uint64_t y = (static_cast<uint64_t>(fp) << rb2) | fk[q];
        y ^= y >> ms;
        wkey[o] = (y * ic1) & kmask;
        if constexpr (F64) {  // planes as pgx_part_aggregate_f64: count, f64 sum bits, ordered min / max
          wpl[o] = fcn[q];
          wpl[rstride + o] = fsc[q];
          wpl[2 * rstride + o] = MN ? static_cast<uint64_t>(fn_[q]) : ~0ull;
          wpl[3 * rstride + o] = MX ? static_cast<uint64_t>(fx[q]) : 0ull;
          ++o;
          continue;
        }
        const uint64_t c = fsc[q] >> cshift;
        wpl[o] = c;  // plane 0: doc count; planes 1..3: int64 sum, ordered min, ordered max (pgx_part_aggregate)
        wpl[rstride + o] = static_cast<uint64_t>(static_cast<int64_t>(fsc[q] & smask) + static_cast<int64_t>(c) * vbase);
        int64_t vlo = 0, vhi = 0;
        if (MN) vlo = IMG ? vbase + static_cast<int64_t>(na_img<IMG>(simg, img_sh, static_cast<uint32_t>(fn_[q])))
                          : vd[static_cast<uint32_t>(fn_[q])];
        if (MX) vhi = IMG ? vbase + static_cast<int64_t>(na_img<IMG>(simg, img_sh, static_cast<uint32_t>(fx[q])))
                          : vd[static_cast<uint32_t>(fx[q])];
        wpl[2 * rstride + o] = static_cast<uint64_t>(vlo) ^ 0x8000000000000000ull;
        wpl[3 * rstride + o] = static_cast<uint64_t>(vhi) ^ 0x8000000000000000ull;
        note(0, c);
        note(1, oplane_sum_key(static_cast<int64_t>(fsc[q] & smask) + static_cast<int64_t>(c) * vbase));
        note(2, ~(static_cast<uint64_t>(vlo) ^ 0x8000000000000000ull));
        note(3, static_cast<uint64_t>(vhi) ^ 0x8000000000000000ull);
      } else {
        lost = true;
      }
      ++o;
    }
    fp = -1;
  };
  auto flush_begin = [&](int pp) {
    fhas = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int s = q * 64 + lane;
      fk[q] = K[s];
      fsc[q] = S[s];
      if constexpr (F64) {
        fcn[q] = C[s];
        C[s] = 0u;
      }
      fn_[q] = MN ? N[s] : static_cast<MT>(0);
      fx[q] = MX ? X[s] : static_cast<MT>(0);
      fhas |= (fk[q] != kNAEmpty ? 1u : 0u) << q;
      K[s] = kNAEmpty;
      S[s] = 0ull;
      if (MN) N[s] = static_cast<MT>(~0ull);
      if (MX) X[s] = static_cast<MT>(0);
    }
    const uint32_t mine = __popc(fhas);
    uint32_t incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    const uint32_t tot = __shfl(incl, 63, 64);
    fexcl = incl - mine;
    fbase = cursor;
    cursor += tot;
    fp = pp;
  };

  // three batches of 1024 records in registers: the one being aggregated and the next two, loaded ahead
  struct Pos {
    int p;
    uint32_t i0, n;
  };
  auto count = [&](int pp) { return pp < nparts ? min(cnt2[pp], static_cast<unsigned int>(cap2)) : 0u; };
  auto advance = [&](Pos a) -> Pos {
    if (a.i0 + BATCH < a.n) return Pos{a.p, a.i0 + BATCH, a.n};
    const int np = a.p + nw;
    return Pos{np, 0u, count(np)};
  };
  // (four waves per SIMD -- no image, or the packed image of 1024-thread workgroups: two batches and groups of 4
  // records, so 128 VGPRs hold a wavefront)
  constexpr int HB = BIG ? 8 : 4;  // records resolved together
  uint32_t b0[BW], b1[BW], b2[PIPE3 ? BW : 1];
  GT g0[GATHER ? NR : 1], g1[GATHER ? NR : 1];  // GATHER: the values of batches b0 and b1
  auto field = [&](uint64_t R) -> uint32_t {  // the value field: dictId, value offset or table index
    return rb2 >= 32 && W == 1 ? 0u : static_cast<uint32_t>(R >> rb2);
  };
  auto recb = [&](const uint32_t (&buf)[BW], int jj) -> uint64_t {
    return W == 1 ? static_cast<uint64_t>(buf[jj])
                  : static_cast<uint64_t>(buf[2 * jj]) | (static_cast<uint64_t>(buf[2 * jj + 1]) << 32);
  };
  auto gather = [&](const uint32_t (&buf)[BW], GT (&g)[GATHER ? NR : 1]) {
    if constexpr (GATHER) {
#pragma unroll
      for (int jj = 0; jj < NR; ++jj) {
        // a batch's last 16-byte load may hold up to three stale words past the partition's records: their index is
        // clamped into the table (the records themselves are never aggregated)
        const uint32_t ix = field(recb(buf, jj));
        g[jj] = gtab[ix < static_cast<uint32_t>(img_words) ? ix : 0u];
      }
    }
  };
  Pos c{static_cast<int>(blockIdx.x) * kNAWaves + wave, 0u, 0u};
  c.n = count(c.p);
  if (c.p < nparts) load(c.p, c.i0, c.n, b0);
  Pos d = advance(c);
  if constexpr (PIPE3) {
    if (d.p < nparts) load(d.p, d.i0, d.n, b1);
  }
  if (c.p < nparts) gather(b0, g0);
  while (c.p < nparts) {
    const Pos e = advance(d);
    if constexpr (PIPE3) {
      if (e.p < nparts) load(e.p, e.i0, e.n, b2);
    } else {
      if (d.p < nparts) load(d.p, d.i0, d.n, b1);
    }
    if (d.p < nparts) gather(b1, g1);
    const bool full = c.i0 + BATCH <= c.n;  // every record of the batch is the partition's
    auto rec = [&](int jj) -> uint64_t { return recb(b0, jj); };  // record jj of this lane's batch
    // one record into slot: count (+ value), min / max
    auto accumulate = [&](int slot, uint32_t v, uint32_t dd, GT gv) {
      if constexpr (F64) {
        atomicAdd(&C[slot], 1u);
        if (SUM) atomicAdd(reinterpret_cast<double*>(&S[slot]), gv);
        if (MN || MX) {
          const uint64_t b = static_cast<uint64_t>(__double_as_longlong(gv));
          const unsigned long long o = (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
          if (MN) atomicMin(&N[slot], o);
          if (MX) atomicMax(&X[slot], o);
        }
      } else {
        atomicAdd(&S[slot], SUM ? one + v : one);
        if (MN) atomicMin(&N[slot], dd);
        if (MX) atomicMax(&X[slot], dd);
      }
    };
#pragma unroll
    for (int h = 0; h < NR / HB; ++h) {  // groups of HB records: home buckets and values read back to back
      na_u32x4 kb[HB];
      uint32_t val[HB];
#pragma unroll
      for (int j = 0; j < HB; ++j) {
        const int jj = h * HB + j;
        const uint64_t R = rec(jj);
        const uint32_t r2 = static_cast<uint32_t>(R) & rmask;
        const uint32_t b = home(r2);
        kb[j] = *reinterpret_cast<const na_u32x4*>(K + b * kNAWays);
        if constexpr (GATHER && !F64) val[j] = g0[jj];
        else if constexpr (!GATHER) val[j] = SUM ? na_img<IMG>(simg, img_sh, field(R)) : 0u;
        else val[j] = 0u;
      }
      uint32_t miss = 0u;  // records of this group whose key is not in its home bucket (yet)
#pragma unroll
      for (int j = 0; j < HB; ++j) {
        const int jj = h * HB + j;
        const uint32_t ei = W == 1 ? static_cast<uint32_t>((jj >> 2) * 256 + lane * 4 + (jj & 3))
                                   : static_cast<uint32_t>((jj >> 1) * 128 + lane * 2 + (jj & 1));
        const bool valid = full || c.i0 + ei < c.n;  // (full: a wave-uniform flag, no per-record compare)
        const uint64_t R = rec(jj);
        const uint32_t r2 = static_cast<uint32_t>(R) & rmask;
        const uint32_t dd = GATHER && !F64 ? val[j] : field(R);
        const uint32_t b = home(r2);
        const int m = na_way(kb[j], r2);
        if (valid && m < 0) miss |= 1u << j;
        if (!valid || m < 0) continue;
        accumulate(static_cast<int>(b) * kNAWays + m, val[j], dd, g0[GATHER ? jj : 0]);
      }
      // The misses (a group's first record, ~1 in 60 at C3: some lane of the wave misses at most j) probe together:
      // each pass resolves every lane's next missed record, so the wave pays one probe chain per pass instead of
      // one per j that any lane missed.
      while (__ballot(miss != 0u)) {
        if (!miss) continue;
        const int js = __builtin_ctz(miss);
        miss &= miss - 1u;
        uint64_t R = 0u;
        uint32_t v = 0u;
        GT gv = GT(0);
#pragma unroll
        for (int j = 0; j < HB; ++j)
          if (j == js) {
            R = rec(h * HB + j);
            v = val[j];
            gv = g0[GATHER ? h * HB + j : 0];
          }
        const uint32_t r2 = static_cast<uint32_t>(R) & rmask;
        const uint32_t dd = GATHER && !F64 ? v : field(R);
        const int slot = probe(r2, home(r2));
        if (slot < 0) {
          lost = true;
          continue;
        }
        accumulate(slot, v, dd, gv);
      }
    }
    if (d.p != c.p) {  // partition c.p is complete
      flush_end();
      flush_begin(c.p);
    }
#pragma unroll
    for (int j = 0; j < BW; ++j) {
      b0[j] = b1[j];
      if constexpr (PIPE3) b1[j] = b2[j];
    }
    if constexpr (GATHER) {
#pragma unroll
      for (int j = 0; j < NR; ++j) g0[j] = g1[j];
    }
    c = d;
    d = e;
  }
  flush_end();
  if (lane == 0) wcount[gw] = cursor;
  if (lost) atomicAdd(ctr + 3, 1ull);
  if (prange) {  // wavefront minimum / maximum, then one atomic per wavefront and kind
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      unsigned long long a = rlo[k], b = rhi[k];
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long x = __shfl_xor(a, d, 64), y = __shfl_xor(b, d, 64);
        a = x < a ? x : a;
        b = y > b ? y : b;
      }
      if (lane == 0 && a <= b) {
        atomicMin(prange + k, a);
        atomicMax(prange + 4 + k, b);
      }
    }
  }
}

// The wavefronts' output regions -> one compact group list (okey, oplane[p * ocap + i]).  Workgroup w copies region w to
// the rows after every earlier region's (an exclusive sum over wcount, recomputed by each workgroup: nw <= 8192 reads);
// workgroup 0 publishes the total in ctr[0] and counts an overflow of ocap in ctr[3].
__global__ void __launch_bounds__(256) pgx_narrow_compact(const uint64_t* __restrict__ rkey,
                                                          const uint64_t* __restrict__ rplane, int64_t wcap,
                                                          int64_t rstride, const unsigned long long* __restrict__ wcount,
                                                          int nw, uint64_t* __restrict__ okey,
                                                          uint64_t* __restrict__ oplane, int64_t ocap,
                                                          unsigned long long* __restrict__ ctr) {
  __shared__ unsigned long long part[256];
  const int w = blockIdx.x, tid = threadIdx.x;
  const int upto = w == 0 ? nw : w;  // workgroup 0 sums every region (the total), the others the earlier ones
  unsigned long long s = 0;
  for (int i = tid; i < upto; i += 256) s += wcount[i];
  part[tid] = s;
  __syncthreads();
  for (int d = 128; d > 0; d >>= 1) {
    if (tid < d) part[tid] += part[tid + d];
    __syncthreads();
  }
  const unsigned long long sum = part[0];
  __syncthreads();
  unsigned long long off = 0;
  if (w == 0) {
    if (tid == 0) {
      ctr[0] = sum;
      if (sum > static_cast<unsigned long long>(ocap)) atomicAdd(ctr + 3, 1ull);
    }
  } else {
    off = sum;
  }
  const unsigned long long n = wcount[w];
  const uint64_t* sk = rkey + static_cast<int64_t>(w) * wcap;
  const uint64_t* sp = rplane + static_cast<int64_t>(w) * wcap;
  for (unsigned long long i = tid; i < n; i += 256) {
    const unsigned long long o = off + i;
    if (o >= static_cast<unsigned long long>(ocap)) break;
    okey[o] = sk[i];
#pragma unroll
    for (int p = 0; p < 4; ++p) oplane[p * ocap + static_cast<int64_t>(o)] = sp[p * rstride + static_cast<int64_t>(i)];
  }
}

}  // namespace
}  // namespace pgx

// Scratch of the narrow aggregation (pgx_launch_narrow_aggregate): per wavefront, an output region of its partitions x
// the table size (key + 4 planes), and its row count.
extern "C" int64_t pgx_narrow_scratch_words(int nparts, int img_kind, int grid) {
  const int64_t nw = int64_t(grid) * (img_kind == 4 ? 16 : 8);
  const int64_t wcap = (int64_t(nparts) + nw - 1) / nw * pgx::kNASlots;
  return nw * wcap * 5 + nw;
}

extern "C" hipError_t pgx_launch_narrow_split(const uint32_t* lo, const uint16_t* hi, const unsigned long long* cnt1,
                                              int nbuckets, int nwg, int64_t cap1, int rb1, int k2, uint32_t* out,
                                              int64_t cap2, unsigned int* cnt2, unsigned long long* ovf, int wide,
                                              hipStream_t stream) {
  if (nbuckets <= 0) return hipSuccess;
  if (nwg < 1 || nwg > pgx::kN2MaxSlabs || k2 < 0 || k2 > pgx::kNarrowMaxBits2 || rb1 - k2 < 0 || rb1 > 48 ||
      cap1 < 1 || cap1 * nwg >= (int64_t(1) << 32) || cap2 < 1 || cap2 >= (int64_t(1) << 32) || !lo || !out || !cnt1 ||
      !cnt2 || !ovf)
    return hipErrorInvalidValue;
  if (wide)
    hipLaunchKernelGGL(pgx::pgx_narrow_split<2>, dim3(nbuckets), dim3(pgx::kN2Threads), 0, stream, lo, hi, cnt1, nwg,
                       cap1, rb1, k2, out, cap2, cnt2, ovf);
  else
    hipLaunchKernelGGL(pgx::pgx_narrow_split<1>, dim3(nbuckets), dim3(pgx::kN2Threads), 0, stream, lo, hi, cnt1, nwg,
                       cap1, rb1, k2, out, cap2, cnt2, ovf);
  return hipGetLastError();
}

extern "C" hipError_t pgx_launch_narrow_aggregate(const uint32_t* in, const unsigned int* cnt2, int64_t cap2,
                                                  int nparts, int rb2, int keybits, int64_t vbase, int img_kind,
                                                  const uint32_t* img, int img_words, int img_sh, const int64_t* vdict,
                                                  int need_sum, int need_min, int need_max, int cshift, uint64_t* okey,
                                                  uint64_t* oplane, int64_t ocap, unsigned long long* ctr,
                                                  unsigned long long* prange, int grid, uint64_t* scratch,
                                                  int64_t scratch_words, int wide, hipStream_t stream) {
  if (nparts <= 0) return hipSuccess;
  if (!scratch || scratch_words < pgx_narrow_scratch_words(nparts, img_kind, grid)) return hipErrorInvalidValue;
  const int nw = grid * (img_kind == 4 ? 16 : 8);
  const int64_t wcap = (int64_t(nparts) + nw - 1) / nw * pgx::kNASlots;
  const int64_t rstride = int64_t(nw) * wcap;
  uint64_t* rkey = scratch;
  uint64_t* rplane = scratch + rstride;
  unsigned long long* wcount = reinterpret_cast<unsigned long long*>(scratch + 5 * rstride);
  if (rb2 < 0 || rb2 > 31 || keybits < 1 || keybits > 64 || cap2 < 4 || (cap2 & 3) || cshift < 1 || cshift > 63 ||
      grid < 1 || !in || !cnt2 || !okey || !oplane || !ctr || img_kind < 0 || img_kind > 6 ||
      ((img_kind == 1 || img_kind == 2) && (!img || img_words < 1 || img_words > pgx::kNAImgWords)) ||
      (img_kind == 4 && (!img || img_words < 1 || img_words > pgx::kNAImg4Words)) ||
      (img_kind >= 5 && (!img || img_words < 1)) || (need_sum && !img_kind) ||
      ((need_min || need_max) && !img_kind && !vdict) || (wide && img_kind != 3 && img_kind < 5) ||
      (img_kind == 6 && prange))
    return hipErrorInvalidValue;
  const pgx::NarrowMix m = pgx::narrow_mix(keybits);
  // kernel: image kinds 0-4 (32-bit records), 5 = IMG 3 on 64-bit records, 6 / 7 = IMG 5 on 32 / 64-bit records,
  // 8 / 9 = IMG 6 on 32 / 64-bit records
  const int kk = img_kind <= 4 ? (wide ? 5 : img_kind) : (img_kind == 5 ? 6 : 8) + (wide ? 1 : 0);
  const int sel = kk * 8 + (need_sum ? 4 : 0) + (need_min ? 2 : 0) + (need_max ? 1 : 0);
#define PGX_NA_CASE(C, I, A, B, D)                                                                                   \
  case C:                                                                                                            \
    hipLaunchKernelGGL((pgx::pgx_narrow_aggregate<I, A, B, D, 1>), dim3(grid), dim3(pgx::na_threads<I>()), 0, stream, in, \
                       cnt2,                                                                                          \
                       cap2, nparts, rb2, m.mask, m.ic1, m.s, vbase, img, img_words, img_sh, vdict, cshift,   \
                       rkey, rplane, wcap, rstride, wcount, ctr, prange);                                            \
    break;
#define PGX_NA_CASES(I)                       \
  PGX_NA_CASE(I * 8 + 0, I, false, false, false) \
  PGX_NA_CASE(I * 8 + 1, I, false, false, true)  \
  PGX_NA_CASE(I * 8 + 2, I, false, true, false)  \
  PGX_NA_CASE(I * 8 + 3, I, false, true, true)   \
  PGX_NA_CASE(I * 8 + 4, I, true, false, false)  \
  PGX_NA_CASE(I * 8 + 5, I, true, false, true)   \
  PGX_NA_CASE(I * 8 + 6, I, true, true, false)   \
  PGX_NA_CASE(I * 8 + 7, I, true, true, true)
  switch (sel) {
    PGX_NA_CASES(0)
    PGX_NA_CASES(1)
    PGX_NA_CASES(2)
    PGX_NA_CASES(3)
    PGX_NA_CASES(4)
#define PGX_NA_CASE_IW(C, I, Wd, A, B, D)                                                                            \
  case C:                                                                                                            \
    hipLaunchKernelGGL((pgx::pgx_narrow_aggregate<I, A, B, D, Wd>), dim3(grid), dim3(pgx::na_threads<I>()), 0, stream, \
                       in, cnt2, cap2, nparts, rb2, m.mask, m.ic1, m.s, vbase, img, img_words, img_sh, vdict, cshift,  \
                       rkey, rplane, wcap, rstride, wcount, ctr, prange);                                            \
    break;
#define PGX_NA_CASES_IW(K, I, Wd)                          \
  PGX_NA_CASE_IW(K * 8 + 0, I, Wd, false, false, false) \
  PGX_NA_CASE_IW(K * 8 + 1, I, Wd, false, false, true)  \
  PGX_NA_CASE_IW(K * 8 + 2, I, Wd, false, true, false)  \
  PGX_NA_CASE_IW(K * 8 + 3, I, Wd, false, true, true)   \
  PGX_NA_CASE_IW(K * 8 + 4, I, Wd, true, false, false)  \
  PGX_NA_CASE_IW(K * 8 + 5, I, Wd, true, false, true)   \
  PGX_NA_CASE_IW(K * 8 + 6, I, Wd, true, true, false)   \
  PGX_NA_CASE_IW(K * 8 + 7, I, Wd, true, true, true)
    PGX_NA_CASES_IW(5, 3, 2)
    PGX_NA_CASES_IW(6, 5, 1)
    PGX_NA_CASES_IW(7, 5, 2)
    PGX_NA_CASES_IW(8, 6, 1)
    PGX_NA_CASES_IW(9, 6, 2)
#undef PGX_NA_CASES_IW
#undef PGX_NA_CASE_IW
    default:
      return hipErrorInvalidValue;
  }
#undef PGX_NA_CASES
#undef PGX_NA_CASE
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pgx::pgx_narrow_compact, dim3(nw), dim3(256), 0, stream, rkey, rplane, wcap, rstride, wcount, nw,
                     okey, oplane, ocap, ctr);
  return hipGetLastError();
}
