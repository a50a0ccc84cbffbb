// libpgx: partitioned sparse group-by runtime (LONG_MAP / ARRAY_MAP group keys) and the
// device-resident results it produces.  The query kernels (pgx_jit.cpp) emit records; this file sizes, allocates and
// drives the splits and aggregations (pgx_kernels.hip pgx_partition / pgx_part_aggregate, pgx_narrow.hip), retries on
// capacity overflows, replays kept plans, and trims / decodes the resulting group planes (pgx_trim.hip).
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#include "pgx_host.h"

namespace pgxh {

// -------------------------------------------------------------------------------------------------
// Partitioned group-by (DESIGN.md "Sparse group-by").  The query kernel writes one 8-byte record per scanned row,
// key | (value - vbase) << keybits (~0: row not selected).  Two radix passes on independent bits of a 64-bit mix of
// the key (128 buckets, then 2^nbits2 per bucket) split the records into partitions whose groups fit one workgroup's
// LDS hash table; pgx_part_aggregate aggregates each partition and appends its groups.  Each pass reads the previous
// pass's cursors on the device, so the chain runs without a host round trip until the final counters.
// Replaces, for sparse keys, the reference's per-segment MAP-based group-key holders
// (DefaultGroupKeyGenerator.java:239-343 LONG_MAP / ARRAY_MAP) with a layout that streams HBM instead of probing it.
// -------------------------------------------------------------------------------------------------

// PGX_DEBUG=part_small (tests): start from undersized buckets and one pass, and allow at most one refinement, so the
// resize, re-split and hash-table fallback branches run at small row counts.
bool part_debug(const ExecPlan& P) { return P.kn.part_small; }

// second-pass split bits: up to 128 ways
int part_max_bits2(const ExecPlan&) { return 7; }

void part_size(const ExecPlan& P, PartBuffers& PB) {
  const int64_t N = P.rec_total;
  double ub = double(N);  // groups: at most the rows and the product of the key cardinalities
  double prod = 1;
  for (const auto& g : P.gdicts) prod *= double(g.card);
  ub = std::min(ub, prod);
  PB.nbits2 = 0;
  while (PB.nbits2 < part_max_bits2(P) && double(int64_t(1) << (kPart1Bits + PB.nbits2)) * kPartGroupsPerWg < ub)
    ++PB.nbits2;
  PB.cap1 = N / kPart1N + N / 512 + 65536;
  const int64_t np = PB.nparts();
  PB.cap2 = N / np + N / np / 4 + 16384;
  if (part_debug(P)) {
    PB.nbits2 = 0;
    PB.cap1 = N / 256 + 1;
    PB.cap2 = 1;
  }
}

bool part_alloc(pgx_ctx* ctx, const ExecPlan& P, PartBuffers& PB) {
  const int64_t np = PB.nparts();
  PB.ocap = std::max<int64_t>(1, std::min<int64_t>(P.rec_total, np * 4096));
  const uint64_t bytes = uint64_t(PB.out1_recs()) * 8 + (PB.pass2() ? uint64_t(np) * PB.cap2 * 8 : 0) + uint64_t(PB.ocap) * 40;
  if (bytes > kPartMaxBytes) return false;
  PB.out1 = DevBuf(ctx, size_t(std::max<int64_t>(PB.out1_recs(), 1)) * 8);
  if (PB.pass2()) PB.out2 = DevBuf(ctx, size_t(np) * PB.cap2 * 8);
  PB.okey = DevBuf(ctx, size_t(PB.ocap) * 8);
  PB.oplane = DevBuf(ctx, size_t(PB.ocap) * 4 * 8);
  PB.ctr = DevBuf(ctx, PB.ctr_words() * 8);
  return true;
}

// Before the scan: zero the cursors and counters (the scan writes row-order records into the plan's record array).
void part_prepare(ExecPlan& P, PartBuffers& PB, hipStream_t st) {
  unsigned long long* ctr = devp(PB.ctr);
  hip_check(hipMemsetAsync(ctr, 0, PB.ctr_words() * 8, st), "partition counters");
  P.part_cursor = nullptr;
  P.part_overflow = nullptr;
  P.part_cap = PB.cap1;
}

// After the scan: first pass, second pass, aggregation.
void part_enqueue(const ExecPlan& P, PartBuffers& PB, hipStream_t st) {
  const int64_t N = P.rec_total;
  unsigned long long* ctr = devp(PB.ctr);
  const int64_t np = PB.nparts();
  unsigned long long* c1 = ctr;
  unsigned long long* c2 = ctr + kPart1N * kCursorStride;
  unsigned long long* tail = ctr + PB.ctr_words() - 4;  // ocount, overflow[3]
  if (N == 0) return;
  const uint64_t keymask = (uint64_t(1) << P.part_keybits) - 1u;
  {
    const uint64_t* recs = reinterpret_cast<const uint64_t*>(P.kq.table);
    const int64_t chunks1 = (N + kPartChunkRecs - 1) / kPartChunkRecs;
    if (chunks1 > 0x7FFFFFFF) fail(PGX_ERR_UNSUPPORTED, "too many rows for one partitioned group-by");
    PGX_LAUNCH(st, "pgx_partition", pgx_launch_partition(recs, nullptr, nullptr, 1, 1, 1, N, int(chunks1), keymask,
                                   64 - kPart1Bits, kPart1Bits, PB.out1.as<uint64_t>(), PB.cap1, c1, kCursorStride,
                                   tail + 1, st),
              "partition pass 1");
  }
  const uint64_t* ain = PB.out1.as<uint64_t>();
  const unsigned long long* acnt = c1;
  int64_t acap = PB.cap1;
  int aparts = kPart1N;
  if (PB.pass2()) {
    const int64_t nreg = kPart1N;
    const int64_t chunks2 = (PB.cap1 + kPartChunkRecs - 1) / kPartChunkRecs;
    if (chunks2 * nreg > 0x7FFFFFFF) fail(PGX_ERR_UNSUPPORTED, "too many rows for one partitioned group-by");
    PGX_LAUNCH(st, "pgx_partition", pgx_launch_partition(PB.out1.as<uint64_t>(), nullptr, c1, kCursorStride, int(nreg),
                                   1, PB.cap1,
                                   int(chunks2), keymask, 64 - kPart1Bits - PB.nbits2, PB.nbits2,
                                   PB.out2.as<uint64_t>(), PB.cap2, c2, kCursorStride, tail + 2, st),
              "partition pass 2");
    ain = PB.out2.as<uint64_t>();
    acnt = c2;
    acap = PB.cap2;
    aparts = int(np);
  }
  // count and sum share one LDS add when a partition's count and value sum both fit their bit fields
  const int cbits = bits_for(acap + 1);
  const int pack_shift = (2 * cbits + P.part_vbits <= 64) ? 64 - cbits : 0;
  if (P.part_fp)
    PGX_LAUNCH(st, "pgx_part_aggregate_f64",
               pgx_launch_part_aggregate_f64(ain, acnt, kCursorStride, aparts, acap, keymask, P.part_keybits,
                                             P.part_fdict, P.part_min, P.part_max, PB.okey.as<uint64_t>(),
                                             PB.oplane.as<uint64_t>(), PB.ocap, tail, tail + 3, st),
               "partition aggregate (f64)");
  else
    PGX_LAUNCH(st, "pgx_part_aggregate", pgx_launch_part_aggregate(ain, acnt, kCursorStride, aparts, acap, keymask, P.part_keybits, P.part_vbase,
                                        P.part_sum, P.part_min, P.part_max,
                                        pack_shift, PB.okey.as<uint64_t>(), PB.oplane.as<uint64_t>(), PB.ocap, tail,
                                        tail + 3, st),
              "partition aggregate");
}

// Scan (records), partition passes and aggregation; grows the buffers to the measured bucket sizes when a pass
// overflowed.  False: the groups do not fit the partitioned layout (the caller uses the global hash table).
bool run_partitioned(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, PartBuffers& PB, hipStream_t st) {
  alloc_outputs(ctx, P, B, nullptr, 0);
  part_size(P, PB);
  for (int attempt = 0; attempt < 12; ++attempt) {
    if (!part_alloc(ctx, P, PB)) return false;
    part_prepare(P, PB, st);
    if (attempt == 0) {
      reset_outputs(P, B, st);
      launch_scan(P, st);
    }
    part_enqueue(P, PB, st);
    unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
    hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "outputs D2H");
    unsigned long long* tail = outs + 28;  // spare words of the outputs block
    hip_check(hipMemcpyAsync(tail, devp(PB.ctr) + PB.ctr_words() - 4, 32, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    if (!tail[1] && !tail[2] && !tail[3]) return true;
    std::vector<unsigned long long> c(PB.ctr_words());
    hip_check(hipMemcpy(c.data(), PB.ctr.p, c.size() * 8, hipMemcpyDeviceToHost), "counters D2H");
    auto max_cursor = [&](size_t first, int64_t count) {
      unsigned long long m = 0;
      for (int64_t i = 0; i < count; ++i) m = std::max(m, c[first + size_t(i) * kCursorStride]);
      return int64_t(m);
    };
    if (tail[1]) {  // a first-pass bucket overflowed: size to the largest (cursors count every record)
      PB.cap1 = max_cursor(0, kPart1N) + 1024;
      continue;
    }
    if (tail[2]) {
      PB.cap2 = max_cursor(kPart1N * kCursorStride, PB.nparts()) + 1024;
      continue;
    }
    if (PB.nbits2 == (part_debug(P) ? 1 : part_max_bits2(P))) return false;  // an LDS table overflowed at the finest split
    ++PB.nbits2;
    const int64_t np = PB.nparts();
    PB.cap2 = P.rec_total / np + P.rec_total / np / 4 + (part_debug(P) ? 1 : 16384);
  }
  return false;
}

// -------------------------------------------------------------------------------------------------
// Narrow partitioned group-by (pgx_narrow.hip): the scan's 256-way split into per-workgroup slabs of u32 (+ u16)
// dictId records, pgx_narrow_split into 2^(8 + k2) partitions of u32 records, pgx_narrow_aggregate with wavefront-
// private LDS tables and the value image.  Capacities are sized from the row counts with an 8-sigma margin over the
// binomial bucket sizes a uniform mix gives; a skewed key distribution that overflows one falls back to the 8-byte
// radix path (run_partitioned), which sizes from measured counts.
// -------------------------------------------------------------------------------------------------

// mean + 8 sigma (binomial, p small) + slack, a multiple of 32: slabs then start on 128-byte lines (u32 records) and
// 64-byte lines (u16), so the scan's whole 32-record units are whole lines
int64_t narrow_cap(double m, int64_t slack) {
  const int64_t c = int64_t(m + 8.0 * std::sqrt(std::max(m, 1.0))) + slack;
  return (c + 31) & ~int64_t(31);
}

bool narrow_size(const ExecPlan& P, NarrowBuffers& NB) {
  const int K = P.part_keybits;
  NB.rb1 = K - kNarrow1Bits;
  NB.hib = NB.rb1 + P.narrow_vd > 32;
  NB.nwg = P.part_nwg;
  if (NB.nwg < 1 || NB.nwg > kNarrowMaxWg) return false;
  // second split: what the record width needs, finer while partitions would average more than 64 groups
  double ub = double(P.rec_total), prod = 1;
  for (const auto& g : P.gdicts) prod *= double(g.card);
  ub = std::min(ub, prod);
  NB.k2 = P.narrow_k2min;
  while (NB.k2 < kNarrowMaxBits2 && NB.k2 < NB.rb1 && ub / double(int64_t(1) << (kNarrow1Bits + NB.k2)) > 64.0) ++NB.k2;
  if (P.kn.narrow_k2 >= 0)  // tests (PGX_DEBUG=narrow_k2=N): coarser partitions, to drive the table-overflow fallback
    NB.k2 = std::max(P.narrow_k2min, std::min(P.kn.narrow_k2, std::min(kNarrowMaxBits2, NB.rb1)));
  if (NB.k2 > kNarrowMaxBits2 || NB.k2 > NB.rb1) return false;
  NB.rb2 = NB.rb1 - NB.k2;
  NB.w2 = P.narrow_wide ? 2 : 1;
  if (NB.rb2 + P.narrow_vd > 32 * NB.w2 || NB.rb2 > 31) return false;
  NB.nparts = int64_t(1) << (kNarrow1Bits + NB.k2);
  NB.cap1 = narrow_cap(double(P.part_wg_rows) / (1 << kNarrow1Bits), 64);
  // a partition holds whole groups, so its record count varies more than a binomial: start at 1.5x the mean (C3: ~6
  // sigma of the group-clumped spread) and resize from the measured fills if that is not enough (run_narrow)
  NB.cap2 = narrow_cap(1.5 * double(P.rec_total) / double(NB.nparts), 64);
  if (NB.cap1 * NB.nwg >= (int64_t(1) << 32) || NB.cap2 >= (int64_t(1) << 31)) return false;
  // count and value-offset sum of one group in one u64: count < 2^cb (a partition holds <= cap2 records)
  const int cb = bits_for(NB.cap2 + 1);
  const long double smax = (long double)NB.cap2 * (long double)P.narrow_vrange;
  int sb = 1;
  while (sb < 64 && std::ldexp(1.0L, sb) <= smax) ++sb;
  if (cb + sb > 64 || cb > 62) return false;
  NB.cshift = 64 - cb;
  NB.ocap = std::max<int64_t>(1, std::min<int64_t>(P.rec_total, NB.nparts * kNarrowSlots));
  const uint64_t bytes = uint64_t(kNarrow1Bits == 8 ? 256 : (1 << kNarrow1Bits)) * NB.nwg * NB.cap1 * (NB.hib ? 6 : 4) +
                         uint64_t(NB.nparts) * NB.cap2 * 4 * NB.w2 + uint64_t(NB.ocap) * 40 +
                         // the aggregation's per-wavefront output regions (pgx_narrow_scratch_words; wavefront
                         // rounding bounded by 4096 wavefronts' tables)
                         (uint64_t(NB.nparts) + 4096) * kNarrowSlots * 40;
  return bytes <= kPartMaxBytes;
}

void narrow_alloc(pgx_ctx* ctx, NarrowBuffers& NB) {
  const int64_t slabs = int64_t(1 << kNarrow1Bits) * NB.nwg;
  NB.lo1 = DevBuf(ctx, size_t(slabs * NB.cap1) * 4);
  if (NB.hib) NB.hi1 = DevBuf(ctx, size_t(slabs * NB.cap1) * 2);
  NB.cnt1 = DevBuf(ctx, size_t(slabs) * 8);
  NB.rec2 = DevBuf(ctx, size_t(NB.nparts * NB.cap2) * 4 * NB.w2);
  NB.cnt2 = DevBuf(ctx, size_t(NB.nparts) * 4);
  NB.okey = DevBuf(ctx, size_t(NB.ocap) * 8);
  NB.oplane = DevBuf(ctx, size_t(NB.ocap) * 4 * 8);
  NB.ctr = DevBuf(ctx, 4 * 8);
  NB.prange = DevBuf(ctx, 8 * 8);
}

// Before the scan: zero the slab fills (workgroups without tiles publish none) and the counters; point the scan's
// record outputs at the slabs.
void narrow_prepare(ExecPlan& P, NarrowBuffers& NB, hipStream_t st) {
  hip_check(hipMemsetAsync(NB.cnt1.p, 0, size_t(int64_t(1 << kNarrow1Bits) * NB.nwg) * 8, st), "slab counters");
  hip_check(hipMemsetAsync(NB.ctr.p, 0, 32, st), "narrow counters");
  P.kq.table = reinterpret_cast<unsigned long long*>(NB.lo1.p);
  P.part_hi = NB.hib ? NB.hi1.as<unsigned short>() : nullptr;
  P.part_cursor = devp(NB.cnt1);
  P.part_overflow = devp(NB.ctr) + 1;
  P.part_cap = NB.cap1;
}

// After the scan: the second split and the aggregation.
void narrow_enqueue(pgx_ctx* ctx, const ExecPlan& P, NarrowBuffers& NB, hipStream_t st) {
  if (P.rec_total == 0) return;
  if (P.narrow_img == 6) NB.prange = DevBuf();  // f64 planes: the trim finds its key ranges itself
  if (NB.prange.p) {
    hip_check(hipMemsetAsync(NB.prange.p, 0xFF, 32, st), "range minima");
    hip_check(hipMemsetAsync(static_cast<uint8_t*>(NB.prange.p) + 32, 0, 32, st), "range maxima");
  }
  unsigned long long* ctr = devp(NB.ctr);
  // an LDS image allows one workgroup per CU (512 threads; 1024 for the packed image), the tables alone four (gathered
  // values: one, two waves per SIMD for the registers of three batches and their values in flight)
  const int agg_grid = ctx->num_cus * (P.narrow_img == 3 ? 4 : 1);
  const int64_t sw = pgx_narrow_scratch_words(int(NB.nparts), P.narrow_img, agg_grid);
  if (NB.agg_scratch_words < sw) {
    NB.agg_scratch = DevBuf(ctx, size_t(sw) * 8);
    NB.agg_scratch_words = sw;
  }
  PGX_LAUNCH(st, "pgx_narrow_split",
             pgx_launch_narrow_split(NB.lo1.as<uint32_t>(), NB.hib ? NB.hi1.as<uint16_t>() : nullptr, devp(NB.cnt1),
                                     1 << kNarrow1Bits, int(NB.nwg), NB.cap1, NB.rb1, NB.k2, NB.rec2.as<uint32_t>(),
                                     NB.cap2, NB.cnt2.as<unsigned int>(), ctr + 2, NB.w2 == 2, st),
             "narrow split");
  PGX_LAUNCH(st, "pgx_narrow_aggregate",
             pgx_launch_narrow_aggregate(NB.rec2.as<uint32_t>(), NB.cnt2.as<unsigned int>(), NB.cap2, int(NB.nparts),
                                         NB.rb2, P.part_keybits, P.part_vbase, P.narrow_img, P.narrow_imgp,
                                         P.narrow_img_words, P.narrow_img_sh, P.part_vdict, P.part_sum, P.part_min,
                                         P.part_max, NB.cshift, NB.okey.as<uint64_t>(), NB.oplane.as<uint64_t>(),
                                         NB.ocap, ctr, NB.prange.p ? devp(NB.prange) : nullptr, agg_grid, NB.agg_scratch.as<uint64_t>(),
                                         NB.agg_scratch_words, NB.w2 == 2, st),
             "narrow aggregate");
}

// Scan, split and aggregation once.  False (nothing usable produced): a capacity ran over, or the plan does not fit the
// narrow layout; the caller re-plans the query kernels for the radix path.
bool run_narrow(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, NarrowBuffers& NB, hipStream_t st) {
  alloc_outputs(ctx, P, B, nullptr, 0);
  if (!narrow_size(P, NB)) {
    if (P.kn.narrow_log)
      std::fprintf(stderr, "[pgx narrow] layout does not fit: nwg=%lld keybits=%d vd=%d k2=%d cap1=%lld cap2=%lld\n",
                   (long long)NB.nwg, P.part_keybits, P.narrow_vd, NB.k2, (long long)NB.cap1, (long long)NB.cap2);
    return false;
  }
  narrow_alloc(ctx, NB);
  unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
  unsigned long long* tail = outs + 28;  // spare words of the outputs block: ocount, overflows (part_result reads [28])
  bool scan = true, ok = false;
  int attempt = 0;
  for (; attempt < 4 && !ok; ++attempt) {
    if (scan) {
      narrow_prepare(P, NB, st);
      reset_outputs(P, B, st);
      launch_scan(P, st);
    } else {
      hip_check(hipMemsetAsync(NB.ctr.p, 0, 8, st), "group counter");
      hip_check(hipMemsetAsync(devp(NB.ctr) + 2, 0, 16, st), "overflow counters");
    }
    narrow_enqueue(ctx, P, NB, st);
    hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "outputs D2H");
    hip_check(hipMemcpyAsync(tail, NB.ctr.p, 32, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    ok = !tail[1] && !tail[2] && !tail[3];
    if (ok || (tail[3] && !tail[1] && !tail[2])) break;  // done, or a wavefront table overflowed: no resize helps
    // a capacity ran over (keys clump: a partition holds whole groups): resize to the measured fills and rerun what
    // depends on it -- the split and the aggregation, and the scan only if a slab overflowed
    if (tail[1]) {
      std::vector<unsigned long long> c(size_t(1 << kNarrow1Bits) * NB.nwg);
      hip_check(hipMemcpy(c.data(), NB.cnt1.p, c.size() * 8, hipMemcpyDeviceToHost), "slab fills D2H");
      NB.cap1 = narrow_cap(double(*std::max_element(c.begin(), c.end())), 64);
      const int64_t slabs = int64_t(1 << kNarrow1Bits) * NB.nwg;
      if (NB.cap1 * NB.nwg >= (int64_t(1) << 32) || uint64_t(slabs) * NB.cap1 * 6 > kPartMaxBytes) break;
      NB.lo1 = DevBuf(ctx, size_t(slabs * NB.cap1) * 4);
      if (NB.hib) NB.hi1 = DevBuf(ctx, size_t(slabs * NB.cap1) * 2);
      scan = true;
      continue;  // the split's fills are void: it read truncated slabs
    }
    std::vector<unsigned int> c2(size_t(NB.nparts));
    hip_check(hipMemcpy(c2.data(), NB.cnt2.p, c2.size() * 4, hipMemcpyDeviceToHost), "partition fills D2H");
    NB.cap2 = narrow_cap(double(*std::max_element(c2.begin(), c2.end())), 64);
    if (NB.cap2 >= (int64_t(1) << 31) || uint64_t(NB.nparts) * NB.cap2 * 4 * NB.w2 > kPartMaxBytes) break;
    const int cb = bits_for(NB.cap2 + 1);
    const long double smax = (long double)NB.cap2 * (long double)P.narrow_vrange;
    int sb = 1;
    while (sb < 64 && std::ldexp(1.0L, sb) <= smax) ++sb;
    if (cb + sb > 64 || cb > 62) break;
    NB.cshift = 64 - cb;
    NB.rec2 = DevBuf(ctx, size_t(NB.nparts * NB.cap2) * 4 * NB.w2);
    scan = false;
  }
  if (P.kn.narrow_log)  // tests (PGX_DEBUG=narrow_log): which path ran
    std::fprintf(stderr, "[pgx narrow] nwg=%lld cap1=%lld k2=%d cap2=%lld groups=%llu ovf=%llu/%llu/%llu attempts=%d ok=%d\n",
                 (long long)NB.nwg, (long long)NB.cap1, NB.k2, (long long)NB.cap2, tail[0], tail[1], tail[2], tail[3],
                 attempt + (ok ? 1 : 0), int(ok));
  return ok;
}

// A kept narrow plan again (plan cache): the slabs and partitions are the first run's, the group outputs (handed to
// that run's result) are allocated anew.  False if a capacity ran over (the caller plans afresh).
bool replay_narrow(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, NarrowBuffers& NB, hipStream_t st) {
  alloc_outputs(ctx, P, B, nullptr, 0);
  NB.okey = DevBuf(ctx, size_t(NB.ocap) * 8);
  NB.oplane = DevBuf(ctx, size_t(NB.ocap) * 4 * 8);
  NB.prange = DevBuf(ctx, 8 * 8);
  narrow_prepare(P, NB, st);
  reset_outputs(P, B, st);
  launch_scan(P, st);
  narrow_enqueue(ctx, P, NB, st);
  unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
  unsigned long long* tail = outs + 28;
  hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "outputs D2H");
  hip_check(hipMemcpyAsync(tail, NB.ctr.p, 32, hipMemcpyDeviceToHost, st), "D2H");
  hip_check(hipStreamSynchronize(st), "sync");
  return !tail[1] && !tail[2] && !tail[3];
}

// A kept radix plan again (plan cache): buckets and partitions as the first run sized them, the group outputs anew.
bool replay_part(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, PartBuffers& PB, hipStream_t st) {
  alloc_outputs(ctx, P, B, nullptr, 0);
  PB.okey = DevBuf(ctx, size_t(PB.ocap) * 8);
  PB.oplane = DevBuf(ctx, size_t(PB.ocap) * 4 * 8);
  part_prepare(P, PB, st);
  reset_outputs(P, B, st);
  launch_scan(P, st);
  part_enqueue(P, PB, st);
  unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
  unsigned long long* tail = outs + 28;
  hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "outputs D2H");
  hip_check(hipMemcpyAsync(tail, devp(PB.ctr) + PB.ctr_words() - 4, 32, hipMemcpyDeviceToHost, st), "D2H");
  hip_check(hipStreamSynchronize(st), "sync");
  return !tail[1] && !tail[2] && !tail[3];
}

// The radix path's plan after a narrow attempt gave up: row-order 8-byte value records.
void narrow_fallback(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, ExecPlan& P, ExecBuffers& B) {
  P.part_narrow = false;
  P.part_slab = false;
  P.part_dictid = P.part_fp;  // FLOAT / DOUBLE radix records carry the value's index too
  P.part_hi = nullptr;
  plan_jit(ctx, q, segs, n, P, B);
}

void part_result(pgx_ctx* ctx, const pgx_query& q, ExecPlan& P, ExecBuffers& B, PartBuffers& PB, pgx_result* R) {
  const unsigned long long* outs = reinterpret_cast<const unsigned long long*>(B.host.bytes() + B.off_outs);
  const unsigned long long* stats = outs + 16;
  const KQuery& K = P.kq;
  R->stats[0] = int64_t(stats[0]);
  R->stats[1] = int64_t(stats[1]) + P.host_entries;
  R->stats[2] = int64_t(stats[0]) * P.n_proj;
  R->stats[3] = P.total_raw;
  R->num_aggs = K.num_aggs;
  R->agg_fn = q.agg_fn;
  R->top_n = q.top_n;
  R->group_by = true;
  R->mode = P.mode_ref;
  R->num_groups = int64_t(std::min<unsigned long long>(outs[28], uint64_t(PB.ocap)));
  auto L = std::make_unique<pgx_result::Lazy>();
  L->okey = std::move(PB.okey);
  L->oplane = std::move(PB.oplane);
  L->prange = std::move(PB.prange);
  L->ocap = PB.ocap;
  if (!P.lazy_rep_seg) {  // the key tables move to shared storage once (a kept plan's replays share them)
    auto rs = std::make_shared<std::vector<std::vector<int32_t>>>();
    auto ri = std::make_shared<std::vector<std::vector<int32_t>>>();
    for (int g = 0; g < K.num_gcols; ++g) {
      rs->push_back(std::move(P.gdicts[g].rep_seg));
      ri->push_back(std::move(P.gdicts[g].rep_id));
    }
    P.lazy_rep_seg = std::move(rs);
    P.lazy_rep_id = std::move(ri);
  }
  for (int g = 0; g < K.num_gcols; ++g) {
    L->gshift.push_back(K.gshift[g]);
    L->gbits.push_back(P.gbits[g]);
  }
  L->rep_seg = P.lazy_rep_seg;
  L->rep_id = P.lazy_rep_id;
  for (int a = 0; a < K.num_aggs; ++a) L->agg_kind.push_back(K.agg_kind[a]);
  // planes: count, then sum / min / max per value column in part_cols order (one column: the kernels' own layout)
  L->nplanes = 1 + 3 * std::max<int>(1, int(P.part_cols.size()));
  for (int a = 0; a < K.num_aggs; ++a) {
    const int k = K.agg_kind[a];
    int c = 0;
    for (size_t i = 0; i < P.part_cols.size(); ++i)
      if (P.part_cols[i].vcol == K.agg_col[a]) c = int(i);
    L->agg_plane.push_back(k == A_COUNT ? 0 : 1 + 3 * c + (k == A_MIN ? 1 : (k == A_MAX ? 2 : 0)));
    L->agg_fp.push_back(k != A_COUNT && K.agg_fp[a]);
  }
  ctx->refs.fetch_add(1);
  L->ctx = ctx;
  R->lazy = std::move(L);
}

// A partitioned plan over several value columns (SELECT SUM(a), MAX(b) ... GROUP BY sparse keys): the pipeline runs
// once per column -- the emitted value and its record layout re-planned between passes (plan_jit), the key columns and
// the filter the same -- and every later pass's sum / min / max planes are joined into the first pass's group order by
// key on the device (pgx_merge.hip pgx_join_*).  The result carries 1 + 3 x columns planes.  False: a pass could not
// run partitioned (the caller takes the global hash table for the whole query).
bool run_value_columns(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, ExecPlan& P, ExecBuffers& B,
                       hipStream_t st, pgx_result* R) {
  const int V = int(P.part_cols.size());
  const int NP = 1 + 3 * V;
  DevBuf okey0, comb, tkey, tidx, miss(ctx, 64);
  int64_t ng0 = 0, ccap = 1;
  uint64_t tcap = 1024;
  hip_check(hipMemsetAsync(miss.p, 0, 8, st), "join miss counter");
  for (int v = 0; v < V; ++v) {
    if (v > 0) {
      P.load_part_col(P.part_cols[size_t(v)]);
      plan_jit(ctx, q, segs, n, P, B);
    }
    PartBuffers PB;
    bool ok = false;
    if (P.part_narrow) {
      NarrowBuffers NB;
      if (run_narrow(ctx, P, B, NB, st)) {
        PB.okey = std::move(NB.okey);
        PB.oplane = std::move(NB.oplane);
        PB.ocap = NB.ocap;
        ok = true;
      } else {
        narrow_fallback(ctx, q, segs, n, P, B);
      }
    }
    if (!ok && !run_partitioned(ctx, P, B, PB, st)) {
      if (v > 0) P.load_part_col(P.part_cols[0]);  // the caller's global-hash fallback plans from column 0's state
      return false;
    }
    const unsigned long long* outs = reinterpret_cast<const unsigned long long*>(B.host.bytes() + B.off_outs);
    const int64_t ng = int64_t(std::min<unsigned long long>(outs[28], uint64_t(PB.ocap)));
    if (v == 0) {
      ng0 = ng;
      ccap = std::max<int64_t>(ng0, 1);
      okey0 = std::move(PB.okey);
      comb = DevBuf(ctx, size_t(ccap) * NP * 8);
      for (int p = 0; p < 4; ++p)
        if (ng0)
          hip_check(hipMemcpyAsync(comb.as<uint64_t>() + p * ccap, PB.oplane.as<uint64_t>() + p * PB.ocap, ng0 * 8,
                                   hipMemcpyDeviceToDevice, st),
                    "first pass planes");
      while (tcap < uint64_t(ng0) * 2) tcap <<= 1;
      tkey = DevBuf(ctx, tcap * 8);
      tidx = DevBuf(ctx, tcap * 8);
      hip_check(hipMemsetAsync(tkey.p, 0xFF, tcap * 8, st), "join table");
      PGX_LAUNCH(st, "pgx_join", pgx_launch_join(okey0.as<uint64_t>(), ng0, nullptr, nullptr, 0, 0, devp(tkey),
                                                 tidx.as<int64_t>(), tcap, nullptr, 0, 0, nullptr, st),
                 "join build");
    } else {
      if (ng != ng0) fail(PGX_ERR_INTERNAL, "value-column passes found different group counts");
      PGX_LAUNCH(st, "pgx_join", pgx_launch_join(nullptr, 0, PB.okey.as<uint64_t>(), PB.oplane.as<uint64_t>(), PB.ocap,
                                                 ng, devp(tkey), tidx.as<int64_t>(), tcap, comb.as<uint64_t>(), ccap,
                                                 1 + 3 * v, devp(miss), st),
                 "join scatter");
      hip_check(hipStreamSynchronize(st), "sync");  // PB's buffers go out of scope: the scatter has read them
    }
  }
  unsigned long long nmiss = 0;
  hip_check(hipMemcpyAsync(&nmiss, miss.p, 8, hipMemcpyDeviceToHost, st), "D2H");
  hip_check(hipStreamSynchronize(st), "sync");
  if (nmiss) fail(PGX_ERR_INTERNAL, "value-column passes found different groups");
  unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
  outs[28] = uint64_t(ng0);
  PartBuffers PR;
  PR.okey = std::move(okey0);
  PR.oplane = std::move(comb);
  PR.ocap = ccap;
  P.load_part_col(P.part_cols[0]);
  part_result(ctx, q, P, B, PR, R);
  return true;
}

}  // namespace pgxh

// Decode n groups of a device-resident result (packed keys; planes p at planes[p * n], p = 0 count, 1 int64 sum,
// 2 ordered min, 3 ordered max: pgx_part_aggregate) into column / function-major outputs of stride out_stride.
void pgx_result::decode_lazy(const uint64_t* keys, const uint64_t* planes, int64_t n, int64_t out_stride,
                             int32_t* seg_index, int32_t* dict_id, double* value, int64_t* count) const {
  const Lazy& L = *lazy;
  const int ncols = int(L.gshift.size());
  for (int g = 0; g < ncols; ++g) {
    const uint64_t mask = (uint64_t(1) << L.gbits[g]) - 1u;
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t gid = (keys[i] >> L.gshift[g]) & mask;
      if (seg_index) seg_index[g * out_stride + i] = (*L.rep_seg)[g][gid];
      if (dict_id) dict_id[g * out_stride + i] = (*L.rep_id)[g][gid];
    }
  }
  for (int a = 0; a < int(L.agg_kind.size()); ++a) {
    const int k = L.agg_kind[a];
    const int p = L.agg_plane[size_t(a)];
    const bool fp = !L.agg_fp.empty() && L.agg_fp[size_t(a)];
    const int op = k == A_MIN ? P_MIN_ORD : (k == A_MAX ? P_MAX_ORD : (fp ? P_ADD_F64 : P_ADD_I64));
    for (int64_t i = 0; i < n; ++i) {
      if (count) count[a * out_stride + i] = int64_t(planes[i]);
      if (value) value[a * out_stride + i] = decode_plane(op, fp, planes[size_t(p) * n + i], k);
    }
  }
}

// Read the partitioned group-by's groups back and decode them into the columnar host result.
void pgx_result::materialize() {
  if (!lazy) return;
  const int64_t ng = num_groups;
  hip_check(hipSetDevice(lazy->ctx->device), "hipSetDevice");
  std::vector<uint64_t> keys(ng), pl(size_t(lazy->nplanes) * ng);
  if (ng) {
    hip_check(hipMemcpy(keys.data(), lazy->okey.p, ng * 8, hipMemcpyDeviceToHost), "group keys D2H");
    for (int p = 0; p < lazy->nplanes; ++p)
      hip_check(hipMemcpy(pl.data() + p * ng, lazy->oplane.as<uint64_t>() + p * lazy->ocap, ng * 8,
                          hipMemcpyDeviceToHost),
                "group planes D2H");
  }
  const int ncols = int(lazy->gshift.size()), na = int(lazy->agg_kind.size());
  std::vector<int32_t> seg(size_t(ncols) * ng), id(size_t(ncols) * ng);
  std::vector<double> val(size_t(na) * ng);
  std::vector<int64_t> cnt(size_t(na) * ng);
  decode_lazy(keys.data(), pl.data(), ng, ng, seg.data(), id.data(), val.data(), cnt.data());
  key_seg.assign(ncols, {});
  key_id.assign(ncols, {});
  for (int g = 0; g < ncols; ++g) {
    key_seg[g].assign(seg.begin() + g * ng, seg.begin() + (g + 1) * ng);
    key_id[g].assign(id.begin() + g * ng, id.begin() + (g + 1) * ng);
  }
  g_value.assign(na, {});
  g_count.assign(na, {});
  for (int a = 0; a < na; ++a) {
    g_value[a].assign(val.begin() + a * ng, val.begin() + (a + 1) * ng);
    g_count[a].assign(cnt.begin() + a * ng, cnt.begin() + (a + 1) * ng);
  }
  lazy.reset();
}

// Combine trim of a device-resident result (pgx_trim.hip): indices of the `size` best groups for function fn, best
// first (ties in index order).  The first call selects for EVERY function of the result in one set of launches (one
// range pass, <= 8 histogram passes, one select, all functions side by side) and keeps the selections.
const std::vector<int64_t>& pgx_result::device_trim(int fn, int64_t size) {
  Lazy& L = *lazy;
  const int nf = int(L.agg_kind.size());
  if (int(L.trims.size()) < nf) L.trims.resize(nf);
  if (!L.trims[fn].empty() && L.trim_size == size) return L.trims[fn];
  hip_check(hipSetDevice(L.ctx->device), "hipSetDevice");
  hipStream_t st = L.ctx->stream;
  std::vector<int> kinds(nf), planes(nf);
  for (int f = 0; f < nf; ++f) {
    const int k = L.agg_kind[f];
    const bool fp = !L.agg_fp.empty() && L.agg_fp[size_t(f)];
    kinds[f] = k == A_COUNT ? 0 : k == A_SUM ? (fp ? 5 : 1) : k == A_MIN ? 2 : k == A_MAX ? 3 : (fp ? 6 : 4);
    planes[f] = L.agg_plane[size_t(f)];
  }
  const size_t sb = pgx_trim_state_bytes();
  std::vector<uint8_t> init(sb * nf, 0);
  const int64_t want = size;
  const uint64_t kmin0 = ~0ull;
  for (int f = 0; f < nf; ++f) {
    std::memcpy(init.data() + f * sb + 16, &want, 8);   // TrimState.k
    std::memcpy(init.data() + f * sb + 48, &kmin0, 8);  // TrimState.kmin
  }
  DevBuf state(L.ctx, sb * nf), idx(L.ctx, size_t(size) * 8 * nf), keys(L.ctx, size_t(size) * 8 * nf);
  hip_check(hipMemcpyAsync(state.p, init.data(), init.size(), hipMemcpyHostToDevice, st), "trim state H2D");
  const int grid = int(std::max<int64_t>(1, std::min<int64_t>((num_groups + 255) / 256, int64_t(L.ctx->num_cus) * 8)));
  // candidate lists after the first digit (pgx_trim_cand): room for 32x the groups wanted, at least 1M (a MAX
  // threshold's bin at C3 holds a few 100k groups), at most every group
  const int64_t ccap = std::min<int64_t>(num_groups, std::max<int64_t>(int64_t(1) << 20, 32 * size));
  DevBuf cidx(L.ctx, size_t(std::max<int64_t>(ccap, 1)) * 8 * nf), ckey(L.ctx, size_t(std::max<int64_t>(ccap, 1)) * 8 * nf);
  PGX_LAUNCH(st, "pgx_trim", pgx_launch_trim(L.oplane.as<uint64_t>(), L.ocap, num_groups, kinds.data(), planes.data(), nf, state.p,
                            idx.as<int64_t>(), keys.as<uint64_t>(), size, grid,
                            L.prange.p ? devp(L.prange) : nullptr, cidx.as<int64_t>(), ckey.as<uint64_t>(), ccap, st),
            "trim launch");
  std::vector<int64_t> ix(size_t(size) * nf);
  std::vector<uint64_t> ky(size_t(size) * nf);
  hip_check(hipMemcpyAsync(ix.data(), idx.p, ix.size() * 8, hipMemcpyDeviceToHost, st), "trim D2H");
  hip_check(hipMemcpyAsync(ky.data(), keys.p, ky.size() * 8, hipMemcpyDeviceToHost, st), "trim D2H");
  hip_check(hipStreamSynchronize(st), "sync");
  L.trim_size = size;
  for (int f = 0; f < nf; ++f) {
    const int64_t* fi = ix.data() + size_t(f) * size;
    const uint64_t* fk = ky.data() + size_t(f) * size;
    std::vector<int64_t> order(size);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(),
              [&](int64_t a, int64_t b) { return fk[a] != fk[b] ? fk[a] > fk[b] : fi[a] < fi[b]; });
    std::vector<int64_t>& out = L.trims[f];
    out.resize(size);
    for (int64_t i = 0; i < size; ++i) out[i] = fi[order[i]];
  }
  return L.trims[fn];
}

