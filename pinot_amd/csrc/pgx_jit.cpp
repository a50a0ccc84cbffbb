// Query compiler of libpgx: generates one HIP kernel per query SHAPE and compiles it for gfx950 with hiprtc.
//
// The reference interprets every query through a tree of virtual iterators (operator/dociditerators/*,
// operator/aggregation/*Executor.java): per doc a chain of next()/apply()/readInt() calls.  Here the operator tree
// of one query over one group of segments (plan/maker/InstancePlanMakerImplV2.java:72-109) is flattened into a
// single fused kernel whose loops are specialised to the query's shape:
//   * the bit width of every column (fixed-bit decode, util/PinotDataCustomBitSet.java:122-155) is a constant, so the
//     unpack of a lane's rows is straight-line shifts / byte-permutes on registers;
//   * the physical filter program (plan/FilterPlanNode.java:77-170, AndBlockDocIdSet / OrBlockDocIdSet) becomes
//     bitwise logic on per-lane doc-mask words;
//   * the aggregation list (operator/aggregation/DefaultAggregationExecutor.java, DefaultGroupByExecutor.java)
//     becomes per-lane register accumulators (aggregation-only) or LDS / global atomics (dense group-by);
//   * SUM/AVG values are read from an LDS-resident image of the column's dictionary (Dictionary.readDoubleValues,
//     segment/index/readers/ImmutableDictionaryReader.java:107-155) instead of HBM/L2 gathers.
// Everything else (segment pointers, dictId intervals, bitsets, doc ranges) is a kernel argument, so one compiled
// kernel serves every query and segment set with the same shape.  Results use the same accumulator planes as the
// generic interpreter kernel (pgx_kernels.hip), so the host decodes them identically.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "pgx_internal.h"

extern "C" int pgx_jit_compile_check(const char* source, char* log, unsigned long log_cap);

namespace pgx {

namespace {

const char* kAbiSrc =
#include "pgx_jit_abi.inc"
    ;
const char* kDevSrc =
#include "pgx_jit_device.inc"
    ;

struct Emitter {
  std::ostringstream o;
  int ind = 0;
  template <typename... Ts>
  Emitter& ln(Ts&&... xs) {
    for (int i = 0; i < ind; ++i) o << "  ";
    (o << ... << xs);
    o << "\n";
    return *this;
  }
};

// Words a lane loads per sub-step: R * bits / 32, or for frac columns the words covering R * bits bits that start at
// any multiple of gcd(R * bits, 32) inside the first word.
int dwords_per(const JitShape& s, int c) {
  const int rb = s.R * s.cols[c].bits;
  if (!s.cols[c].frac) return rb / 32;
  int g = 32;
  while (rb % g) g >>= 1;
  return (rb + 32 - g + 31) / 32;
}
bool is_docmask(int mode) { return mode == LEAF_DOCMASK || mode == LEAF_DOCMASK_NOT; }

std::string plane_atomic(int op, const std::string& ptr, const std::string& val) {
  switch (op) {
    case P_ADD_I64: return "atomicAdd(" + ptr + ", " + val + ");";
    case P_ADD_F64: return "atomicAdd((double*)(" + ptr + "), pgx_bits_f64(" + val + "));";
    case P_MIN_ORD: return "atomicMin(" + ptr + ", " + val + ");";
    default: return "atomicMax(" + ptr + ", " + val + ");";
  }
}

// Expression (u32) for the value image of column c at dictId expression v, relative to vbase.
std::string img_value(const JitShape& s, int c, const std::vector<int>& img_off, const std::string& v) {
  const JitCol& C = s.cols[c];
  const int off = img_off[c];  // byte offset in lds
  if (C.img == IMG_U32) return "lds[" + std::to_string(off / 4) + " + " + v + "]";
  // FOR16: bases first (64 x u32), then u16 offsets
  return "(lds[" + std::to_string(off / 4) + " + (" + v + " >> " + std::to_string(C.img_sh) + ")] + (u32)lds16[" +
         std::to_string((off + 4 * kImgFor16Blocks) / 2) + " + " + v + "])";
}

}  // namespace

std::string jit_source(const JitShape& s, int* lds_bytes_out) {
  const int ncols = int(s.cols.size());
  const int U = s.TL / s.R;
  const bool emit = s.group_mode == G_EMIT;
  const bool hashm = s.group_mode == G_HASH64 || s.group_mode == G_HASH128;
  const bool h128 = s.group_mode == G_HASH128;
  // packed count + value-offset add in the LDS hash table (flushed per segment into the global table): one plane
  const bool hpack = s.dense_pack > 0 && hashm && s.num_planes == 2 && s.agg_kind.size() == 1 &&
                     (s.agg_kind[0] == A_SUM || s.agg_kind[0] == A_AVG) && !s.cols[s.agg_col[0]].fp &&
                     s.cols[s.agg_col[0]].img != IMG_NONE;
  const int htp = hpack ? 1 : s.num_planes;  // LDS hash planes
  const bool grouped = s.group_mode == G_DENSE_LDS || s.group_mode == G_DENSE_GLOBAL || emit || hashm;
  // ---- LDS layout: images, then the dense group table ----
  std::vector<int> img_off(ncols, -1);
  int lds = 0;
  for (int c = 0; c < ncols; ++c) {
    if (s.cols[c].img == IMG_NONE) continue;
    img_off[c] = lds;
    lds += ((s.cols[c].img_words * 4 + 15) / 16) * 16;
  }
  int tab_off = -1;
  if (s.group_mode == G_DENSE_LDS) {
    tab_off = lds;
    lds += int(s.dense_slots) * s.num_planes * 8;
  }
  // hash group-by: LDS keys (1 or 2 words per slot), 128-bit key states, planes x hash_slots
  int hk_off = -1, hst_off = -1, ht_off = -1;
  const int HS = s.hash_slots;
  if (hashm) {
    lds = (lds + 15) & ~15;
    hk_off = lds;
    lds += HS * 8 * (h128 ? 2 : 1);
    if (h128) {
      hst_off = lds;
      lds += HS * 4;
    }
    lds = (lds + 15) & ~15;
    ht_off = lds;
    lds += HS * htp * 8;
  }
  // G_EMIT: per-wave LDS staging of the records, so that they leave as 64 lanes x 8 contiguous bytes per store
  // instead of R-strided 8-byte stores (each lane owns R consecutive rows).  A lane's R records sit at a pitch of
  // R + 2 words (conflict-free 16-byte LDS writes); rounds of stg_recs records when the budget is tight.
  int stg_off = -1, stg_recs = 0;
  const int stg_pitch = s.R + 2;
  // G_EMIT with part_bits (narrow records only: part_slab and part_narrow): the sub-step's records are split
  // 2^part_bits ways into this workgroup's slab of each bucket, a u32 array and a u16 array (records wider than 32
  // bits), written through per-bucket LDS rings so that only whole 32-record units leave (128-B u32 / 64-B u16 lines,
  // see the sub-step below).  Without part_bits the records leave in row order (the 8-byte radix path).
  const bool epart = emit && s.part_bits > 0;
  const bool enarrow = epart && s.part_slab && s.part_narrow;
  const int nrb1 = s.keybits - s.part_bits;  // narrow: bits of the key's mix left in the record
  const bool nhib = enarrow && nrb1 + s.narrow_vbits > 32;
  const int pnb = 1 << s.part_bits;
  const int NU = s.narrow_unit, NRG = 2 * s.narrow_unit;  // narrow: records per unit, ring records per bucket
  // (narrow: pnb = 256 and T a multiple of 256 -- plan_jit's choices; four owner wavefronts hold one bucket per lane)
  int nring_off = -1, nringb_off = -1, nst_off = -1;
  if (enarrow) {
    lds = (lds + 15) & ~15;  // 16-byte ring reads and writes
    nring_off = lds;
    lds += pnb * NRG * 4;
    nringb_off = lds;
    if (nhib) lds += pnb * NRG * 2;
    // cursors[256], unflushed-unit starts[2][256], ring-valid-from[2][256], unit lists (u16 bucket, u32 position)
    // [4][128] each, list counts[4]
    nst_off = lds;
    lds += pnb * 4 * 5 + 4 * 128 * 2 + 4 * 128 * 4 + 16;
  }
  if (emit && !epart) {
    const int waves = s.T / 64;
    for (int r = 64 * s.R; r >= std::max(64, s.R); r /= 2)
      if (lds + (r / s.R) * stg_pitch * 8 * waves <= kLdsBudget) {
        stg_recs = r;
        break;
      }
    if (stg_recs) {
      stg_off = lds;
      lds += (stg_recs / s.R) * stg_pitch * 8 * waves;
    }
  }
  // LEAF_RCHUNK: one 2048-word mask per leaf of each bitmap program, plus the container-search scratch
  const int nleaves_all = int(s.leaf_col.size());
  std::vector<int> rch_off(nleaves_all, -1), rch_nl(nleaves_all, 0);
  int scr_off = -1;
  {
    size_t k = 0;
    for (int l = 0; l < nleaves_all; ++l) {
      if (s.leaf_mode[l] != LEAF_RCHUNK) continue;
      const std::vector<int>& ops = s.rprog_ops.at(k++);
      for (int op : ops) rch_nl[l] += op == RP_LEAF;
      rch_off[l] = lds;
      lds += rch_nl[l] * 2048 * 4;
    }
    if (k) {
      scr_off = lds;
      lds += (int(sizeof(void*)) * 256 + 3 * 4 * 256 + 16 + 15) / 16 * 16;
    }
  }
  // compact: the selected rows of a sub-step are packed into consecutive lanes (wave prefix of the per-lane selection
  // counts, the rows' dictIds staged in LDS) before values are looked up and aggregated, so a selective filter costs
  // one gather / atomic wave-instruction per 64 SELECTED rows instead of PR mostly-idle ones per sub-step
  std::vector<int> ccols;  // columns whose dictIds are staged: group columns, then aggregated value columns
  int cst_off = -1;
  const bool compact = s.compact && !emit && s.group_mode != G_HASH64 && s.group_mode != G_HASH128;
  if (compact) {
    if (grouped)
      for (int c : s.gcol)
        if (std::find(ccols.begin(), ccols.end(), c) == ccols.end()) ccols.push_back(c);
    for (size_t a = 0; a < s.agg_kind.size(); ++a)
      if (s.agg_kind[a] != A_COUNT && std::find(ccols.begin(), ccols.end(), s.agg_col[a]) == ccols.end())
        ccols.push_back(s.agg_col[a]);
    cst_off = lds;
    lds += (s.T / 64) * 64 * std::max<int>(1, int(ccols.size())) * 4;
  }
  if (lds_bytes_out) *lds_bytes_out = lds;
  const bool any_img = lds > 0 && (tab_off != 0 || s.group_mode != G_DENSE_LDS);

  Emitter e;
  e.o << kAbiSrc << "\n" << kDevSrc << "\n";
  e.ln("#define PT ", s.T);
  e.ln("#define PR ", s.R);
  e.ln("#define PTL ", s.TL);
  e.ln("extern \"C\" __global__ void __launch_bounds__(PT) pgxq(const JArgs A) {");
  e.ind = 1;
  if (lds > 0) {
    e.ln("__shared__ __attribute__((aligned(16))) u32 lds[", (lds + 3) / 4, "];");
    e.ln("const unsigned short* lds16 = (const unsigned short*)lds;");
    e.ln("(void)lds16;");
  }
  e.ln("__shared__ u64 s_acc[", s.num_planes, "];");
  e.ln("const int tid = threadIdx.x;");
  e.ln("const int lane = tid & 63;");
  e.ln("const long long tb = A.tile_base + (long long)blockIdx.x * A.tiles_per_wg;");
  e.ln("const long long te = (tb + A.tiles_per_wg < A.total_tiles) ? tb + A.tiles_per_wg : A.total_tiles;");
  e.ln("if (tb >= te) return;");
  // accumulator init
  {
    std::string init = "0ull";
    e.ln("if (tid < ", s.num_planes, ") {");
    e.ind++;
    e.ln("u64 z = 0ull;");
    for (int p = 1; p < s.num_planes; ++p)
      if (s.plane_op[p] == P_MIN_ORD) e.ln("if (tid == ", p, ") z = ~0ull;");
    e.ln("s_acc[tid] = z;");
    e.ind--;
    e.ln("}");
  }
  if (s.group_mode == G_DENSE_LDS) {
    e.ln("{");
    e.ind++;
    e.ln("u64* tab = (u64*)(lds + ", tab_off / 4, ");");
    e.ln("for (int i = tid; i < ", s.dense_slots * s.num_planes, "; i += PT) {");
    e.ind++;
    e.ln("const int p = i / ", s.dense_slots, ";");
    e.ln("u64 z = 0ull;");
    for (int p = 1; p < s.num_planes; ++p)
      if (s.plane_op[p] == P_MIN_ORD) e.ln("if (p == ", p, ") z = ~0ull;");
    e.ln("tab[i] = z;");
    e.ind--;
    e.ln("}");
    e.ind--;
    e.ln("}");
  }
  if (hashm) {
    e.ln("u64* const hk = (u64*)(lds + ", hk_off / 4, ");");
    if (h128) e.ln("u32* const hst = lds + ", hst_off / 4, ";");
    e.ln("u64* const ht = (u64*)(lds + ", ht_off / 4, ");");
    e.ln("for (int i = tid; i < ", HS * (h128 ? 2 : 1), "; i += PT) hk[i] = ~0ull;");
    if (h128) e.ln("for (int i = tid; i < ", HS, "; i += PT) hst[i] = 0u;");
    e.ln("for (int i = tid; i < ", HS * htp, "; i += PT) {");
    e.ln("  u64 z = 0ull;");
    for (int p = 1; p < s.num_planes; ++p)
      if (s.plane_op[p] == P_MIN_ORD) e.ln("  if (i / ", HS, " == ", p, ") z = ~0ull;");
    e.ln("  ht[i] = z;");
    e.ln("}");
  }
  e.ln("__syncthreads();");
  if (s.group_mode == G_DENSE_LDS) e.ln("u64* const tab = (u64*)(lds + ", tab_off / 4, ");");
  if (s.group_mode == G_DENSE_GLOBAL) e.ln("u64* const tab = A.table;");
  if (scr_off >= 0) e.ln("PgxRScratch& rscr = *(PgxRScratch*)(lds + ", scr_off / 4, ");");
  if (compact) e.ln("u32* const cstg = lds + ", cst_off / 4, " + (tid >> 6) * ", 64 * std::max<size_t>(1, ccols.size()), ";");
  if (enarrow) {
    e.ln("u32* const ringA = lds + ", nring_off / 4, ";");
    if (nhib) e.ln("unsigned short* const ringB = (unsigned short*)(lds + ", nringb_off / 4, ");");
    e.ln("u32* const ncur = lds + ", nst_off / 4, ";");
    e.ln("u32* const nU = ncur + 256;");
    e.ln("u32* const nV = ncur + 768;");
    e.ln("unsigned short* const nlb = (unsigned short*)(ncur + 1280);");
    e.ln("u32* const nlp = ncur + 1536;");
    e.ln("u32* const nlc = ncur + 2048;");
    e.ln("for (int i = tid; i < 1280; i += PT) ncur[i] = 0u;");
    e.ln("int npar = 0;");
    e.ln("PGX_G u32* const poutA = (PGX_G u32*)A.table;");
    if (nhib) e.ln("PGX_G unsigned short* const poutB = (PGX_G unsigned short*)A.part_hi;");
    e.ln("const long long wsl = A.part_wg_base + (long long)blockIdx.x;");
    e.ln("__syncthreads();");
  }
  e.ln("u64 st_docs = 0, st_ent = 0;");
  // value images already in LDS (segments sharing one dictionary share one image: not restaged per segment)
  for (int c = 0; c < ncols; ++c)
    if (s.cols[c].img != IMG_NONE) e.ln("const void* imgp", c, " = nullptr;");
  e.ln("int seg = __builtin_amdgcn_readfirstlane(pgx_find_seg(A.segs, A.num_segs, tb));  // workgroup-uniform");
  e.ln("long long t = tb;");
  e.ln("while (t < te) {");
  e.ind = 2;
  e.ln("const JSeg* __restrict__ S = A.segs + seg;");
  e.ln("const long long tse = (seg + 1 < A.num_segs) ? A.segs[seg + 1].tile_begin : A.total_tiles;");
  e.ln("const long long t2 = (te < tse) ? te : tse;");
  e.ln("const int nd = S->num_docs;");
  e.ln("const long long tile0 = S->tile_begin;");
  e.ln("const PGX_G int* __restrict__ tl = (const PGX_G int*)S->tiles;  // tile skipping (star-tree ranges)");
  // stage this segment's value images into LDS (emitted after the first tile's loads are in flight, below): four
  // 16-byte loads per thread are issued before their LDS stores, so a 128 KiB image costs two load latencies, not eight
  bool has_img = false;
  for (int c = 0; c < ncols; ++c) has_img |= s.cols[c].img != IMG_NONE;
  (void)any_img;
  auto emit_images = [&]() {
    if (!has_img) return;
    // uniform: every thread reads the same segment descriptor
    std::string same;
    for (int c = 0; c < ncols; ++c)
      if (s.cols[c].img != IMG_NONE) same += std::string(same.empty() ? "" : " && ") + "S->img[" + std::to_string(c) +
                                             "] == imgp" + std::to_string(c);
    e.ln("if (!(", same, ")) {");
    e.ind++;
    e.ln("pgx_lds_barrier();");
    for (int c = 0; c < ncols; ++c) {
      if (s.cols[c].img == IMG_NONE) continue;
      e.ln("imgp", c, " = S->img[", c, "];");
      e.ln("{");
      e.ind++;
      e.ln("const PGX_G pgx_u32x4* __restrict__ src = (const PGX_G pgx_u32x4*)S->img[", c, "];");
      e.ln("pgx_u32x4* dst = (pgx_u32x4*)(lds + ", img_off[c] / 4, ");");
      e.ln("const int nq = (S->img_words[", c, "] + 3) >> 2;");
      e.ln("for (int i0 = 0; i0 < nq; i0 += 4 * PT) {");
      e.ln("  pgx_u32x4 x[4];");
      e.ln("  #pragma unroll");
      e.ln("  for (int k = 0; k < 4; ++k) if (i0 + k * PT + tid < nq) x[k] = src[i0 + k * PT + tid];");
      e.ln("  #pragma unroll");
      e.ln("  for (int k = 0; k < 4; ++k) if (i0 + k * PT + tid < nq) dst[i0 + k * PT + tid] = x[k];");
      e.ln("}");
      e.ind--;
      e.ln("}");
    }
    e.ln("pgx_lds_barrier();");
    e.ind--;
    e.ln("}");
  };
  // per-segment pointers and leaf parameters
  for (int c = 0; c < ncols; ++c)
    if (s.cols[c].decode) e.ln("const u32* __restrict__ f", c, " = pgx_sgpr(S->fwd[", c, "]);");
  const int nleaves = int(s.leaf_col.size());
  for (int l = 0; l < nleaves; ++l) {
    switch (s.leaf_mode[l]) {
      case LEAF_SCAN_INTERVAL:
        e.ln("const u32 lo", l, " = S->llo[", l, "], sp", l, " = S->lspan[", l, "];");
        break;
      case LEAF_SCAN_BITSET:
        e.ln("const PGX_G u32* __restrict__ bs", l, " = (const PGX_G u32*)S->lbits[", l, "];");
        break;
      case LEAF_DOCMASK:
      case LEAF_DOCMASK_NOT:
        e.ln("const PGX_G u32* __restrict__ dm", l, " = (const PGX_G u32*)S->lbits[", l, "];");
        break;
      case LEAF_RCHUNK:
        e.ln("const PGX_G JRProg* __restrict__ rp", l, " = (const PGX_G JRProg*)S->lbits[", l, "];");
        e.ln("u32* const rlm", l, " = lds + ", rch_off[l] / 4, ";");
        break;
      case LEAF_RANGES:
        e.ln("const PGX_G int* __restrict__ rg", l, " = (const PGX_G int*)S->lranges[", l, "];");
        e.ln("const int nr", l, " = S->lnr[", l, "];");
        e.ln("int cur", l, " = pgx_ranges_seek(rg", l, ", nr", l, ", (int)((tl ? (long long)tl[t - tile0] : (t - tile0)) * (PT * PTL)));");
        break;
      default:
        break;
    }
  }
  // group columns: remap tables
  if (grouped)
    for (size_t g = 0; g < s.gcol.size(); ++g)
      if (s.cols[s.gcol[g]].remap) e.ln("const PGX_G int* __restrict__ rm", g, " = (const PGX_G int*)S->remap[", s.gcol[g], "];");
  // value bases / dictionaries used by the aggregations
  const int naggs = int(s.agg_kind.size());
  std::vector<bool> need_vb(ncols, false), need_dict(ncols, false);
  for (int a = 0; a < naggs; ++a) {
    const int k = s.agg_kind[a];
    if (k == A_COUNT) continue;
    const int c = s.agg_col[a];
    const JitCol& C = s.cols[c];
    if (!grouped) {
      if (k == A_SUM || k == A_AVG) {
        if (C.img == IMG_U32 || C.img == IMG_FOR16) need_vb[c] = true;
        else if (C.img == IMG_NONE) need_dict[c] = true;
      } else {
        need_dict[c] = true;  // MIN/MAX: one value lookup per lane at flush
      }
    } else {
      if (C.img == IMG_U32 || C.img == IMG_FOR16) need_vb[c] = true;
      else if (C.img == IMG_NONE) need_dict[c] = true;
    }
  }
  // Values gathered per selected row (no LDS image: HBM/L2 dictionary; group-key remaps): the row loop is split into a
  // filter pass (selection bits), a gather pass that issues every selected row's loads back to back, and the
  // aggregation pass; a gather inside the filtered row loop would wait for its load before the next row's.
  std::vector<bool> gcolv(ncols, false), gremap(s.gcol.size(), false);
  bool split = compact;
  if (!emit) {
    for (int c = 0; c < ncols; ++c)
      if (need_dict[c]) {
        bool summed = false;
        for (int a = 0; a < naggs; ++a)
          if (s.agg_col[a] == c && (grouped || s.agg_kind[a] == A_SUM || s.agg_kind[a] == A_AVG)) summed = true;
        if (summed) gcolv[c] = split = true;
      }
    if (grouped)
      for (size_t g = 0; g < s.gcol.size(); ++g)
        if (s.cols[s.gcol[g]].remap) gremap[g] = split = true;
  }
  const bool pack = s.dense_pack > 0 && s.group_mode == G_DENSE_LDS && s.num_planes == 2 && naggs == 1 &&
                    (s.agg_kind[0] == A_SUM || s.agg_kind[0] == A_AVG) && !s.cols[s.agg_col[0]].fp &&
                    s.cols[s.agg_col[0]].img != IMG_NONE && !emit;
  // (hpack: the same packed count + value-offset add in the LDS hash table, decided above)
  for (int c = 0; c < ncols; ++c) {
    if (need_vb[c]) e.ln("const i64 vb", c, " = S->vbase[", c, "];");
    if (need_dict[c]) {
      if (s.cols[c].fp) e.ln("const PGX_G double* __restrict__ dd", c, " = (const PGX_G double*)S->dict[", c, "];");
      else e.ln("const PGX_G i64* __restrict__ di", c, " = (const PGX_G i64*)S->dict[", c, "];");
    }
  }
  if (scr_off >= 0) e.ln("int rc_cur = -1;  // chunk whose bitmap-program masks are in LDS");
  // lane accumulators (aggregation-only)
  e.ln("u64 wcnt = 0;  // selected rows of this wave in this segment (wave-uniform)");
  if (!grouped) {
    for (int a = 0; a < naggs; ++a) {
      const int k = s.agg_kind[a];
      const int c = s.agg_col[a];
      if (k == A_SUM || k == A_AVG) {
        if (s.cols[c].fp) e.ln("double acc", a, " = 0.0;");
        else if (s.cols[c].img == IMG_NONE) e.ln("i64 acc", a, " = 0;");
        else e.ln("u64 acc", a, " = 0;");
      } else if (k == A_MIN) {
        e.ln("u32 mn", a, " = 0xFFFFFFFFu;");
      } else if (k == A_MAX) {
        e.ln("u32 mx", a, " = 0u;");
      }
    }
  }
  // Mask-gated loads: when every filter leaf is a doc-mask leaf (a bitmap program's mask, an MV leaf's mask: no scan
  // leaf reads a column) and the program selects only rows whose mask bit `gate` is set, a row with a clear bit is
  // never selected and its forward-index words matter to nothing (not the filter, not the statistics, not any group or
  // value).  The gate leaf's mask words then load one tile earlier than the columns, and a lane whose rows are all
  // clear does not load their words: the row-selective read of the reference's projection
  // (DataFetcher.fetchSingleDictIds over the filtered docIds), at the granularity of a lane's dwords.
  int gate = -1;
  {
    bool all_masks = !s.prog_op.empty();
    for (size_t pc = 0; pc < s.prog_op.size() && all_masks; ++pc)
      if (s.prog_op[pc] == OP_LEAF && !is_docmask(s.leaf_mode[s.prog_arg[pc]])) all_masks = false;
    std::vector<std::vector<int>> impl;  // per stack entry: the doc-mask leaves every selected row has set
    for (size_t pc = 0; pc < s.prog_op.size() && all_masks; ++pc) {
      const int op = s.prog_op[pc], arg = s.prog_arg[pc];
      if (op == OP_LEAF) {
        impl.push_back(s.leaf_mode[arg] == LEAF_DOCMASK ? std::vector<int>{arg} : std::vector<int>{});
      } else if (op == OP_AND || op == OP_OR) {
        std::vector<int> acc = impl.back();
        impl.pop_back();
        for (int k = 1; k < arg; ++k) {
          std::vector<int> x = impl.back(), y;
          impl.pop_back();
          if (op == OP_AND) {
            y = acc;
            y.insert(y.end(), x.begin(), x.end());
          } else {
            for (int l : acc)
              if (std::find(x.begin(), x.end(), l) != x.end()) y.push_back(l);
          }
          acc = y;
        }
        impl.push_back(acc);
      } else if (op == OP_TRUE) {
        impl.push_back({});
      }
    }
    if (all_masks && impl.size() == 1 && !impl[0].empty() && !compact) gate = impl[0][0];
  }
  auto gate_bits = [&](const std::string& w) {  // the lane's PR bits of gate word w (r0 in scope)
    return s.R == 32 ? w : "((" + w + " >> (r0 & 31)) & " + std::to_string((1u << s.R) - 1u) + "u)";
  };
  // software-pipelined tile loop: raw words of tile tt+1 are loaded while tile tt is computed
  auto emit_loads = [&](const std::string& tile, const std::string& dst, const std::string& rbv = "rbn") {
    e.ln("{");
    e.ind++;
    e.ln(rbv, " = (int)((tl ? (long long)tl[", tile, " - tile0] : (", tile, " - tile0)) * (PT * PTL));");
    e.ln("const int rb = ", rbv, ";");
    e.ln("const bool full = rb + PT * PTL <= nd;");
    for (int u = 0; u < U; ++u) {
      e.ln("{");
      e.ind++;
      e.ln("const int r0 = rb + ", u * s.R, " * PT + tid * PR;");
      const std::string cond =
          gate >= 0 ? "(full || r0 < nd) && " + gate_bits("ga[" + std::to_string(u) + "]") + " != 0u" : "full || r0 < nd";
      for (int c = 0; c < ncols; ++c) {
        if (!s.cols[c].decode) continue;
        const int D = dwords_per(s, c);
        if (s.cols[c].frac)
          e.ln("if (", cond, ") pgx_ld_u<", D, ">(f", c, " + (((long long)r0 * ", s.cols[c].bits, ") >> 5), &", dst,
               c, "[", u * D, "]); else pgx_zero<", D, ">(&", dst, c, "[", u * D, "]);");
        else
        e.ln("if (", cond, ") pgx_ld<", D, ">(f", c, " + (long long)(r0 / PR) * ", D, ", &", dst, c, "[", u * D,
             "]); else pgx_zero<", D, ">(&", dst, c, "[", u * D, "]);");
      }
      for (int l = 0; l < nleaves; ++l)
        if (l == gate) e.ln(dst, "q", l, "[", u, "] = ga[", u, "];");
        else if (is_docmask(s.leaf_mode[l]))
          e.ln(dst, "q", l, "[", u, "] = (full || r0 < nd) ? dm", l, "[r0 >> 5] : 0u;");
      e.ind--;
      e.ln("}");
    }
    e.ind--;
    e.ln("}");
  };
  // gate words of one tile (gate >= 0): into ga for the tile whose columns load next, gn for the one after
  auto emit_gate_loads = [&](const std::string& tile, const std::string& dst) {
    e.ln("{");
    e.ind++;
    e.ln("const int rb = (int)((tl ? (long long)tl[", tile, " - tile0] : (", tile, " - tile0)) * (PT * PTL));");
    e.ln("const bool full = rb + PT * PTL <= nd;");
    for (int u = 0; u < U; ++u)
      e.ln("{ const int r0 = rb + ", u * s.R, " * PT + tid * PR; ", dst, "[", u, "] = (full || r0 < nd) ? dm", gate,
           "[r0 >> 5] : 0u; }");
    e.ind--;
    e.ln("}");
  };
  // (prefetch2, no gate leaf: a second buffer set m* holds tile tt+2)
  const bool pf2 = s.prefetch2 && gate < 0;
  for (int c = 0; c < ncols; ++c)
    if (s.cols[c].decode) {
      e.ln("u32 n", c, "[", U * dwords_per(s, c), "];");
      if (pf2) e.ln("u32 m", c, "[", U * dwords_per(s, c), "];");
    }
  for (int l = 0; l < nleaves; ++l)
    if (is_docmask(s.leaf_mode[l])) {
      e.ln("u32 nq", l, "[", U, "];");
      if (pf2) e.ln("u32 mq", l, "[", U, "];");
    }
  // first row of the tile whose raw words are in flight: carried into the next iteration, so the loop body never
  // reloads the tile list after issuing the prefetch (that load's wait would also wait for the prefetch)
  e.ln("int rbn;");
  if (gate >= 0) {
    e.ln("u32 ga[", U, "], gn[", U, "];");
    emit_gate_loads("t", "ga");
  }
  emit_loads("t", "n");
  if (pf2) {
    e.ln("int rbm = 0;");
    e.ln("if (t + 1 < t2)");
    emit_loads("t + 1", "m", "rbm");
  }
  if (gate >= 0) {
    e.ln("if (t + 1 < t2)");
    emit_gate_loads("t + 1", "gn");
  }
  emit_images();
  e.ln("for (long long tt = t; tt < t2; ++tt) {");
  e.ind = 3;
  for (int c = 0; c < ncols; ++c) {
    if (!s.cols[c].decode) continue;
    const int n = U * dwords_per(s, c);
    e.ln("u32 c", c, "[", n, "];");
    e.ln("#pragma unroll");
    e.ln("for (int i = 0; i < ", n, "; ++i) c", c, "[i] = n", c, "[i];");
  }
  for (int l = 0; l < nleaves; ++l)
    if (is_docmask(s.leaf_mode[l])) {
      e.ln("u32 cq", l, "[", U, "];");
      e.ln("#pragma unroll");
      e.ln("for (int i = 0; i < ", U, "; ++i) cq", l, "[i] = nq", l, "[i];");
    }
  e.ln("const int rb = rbn;");
  if (gate >= 0) {  // the next tile's gate words arrived during the previous tile; the one after that's load now
    e.ln("if (tt + 1 < t2) {");
    e.ind++;
    e.ln("#pragma unroll");
    e.ln("for (int i = 0; i < ", U, "; ++i) ga[i] = gn[i];");
    emit_loads("tt + 1", "n");
    e.ln("if (tt + 2 < t2)");
    emit_gate_loads("tt + 2", "gn");
    e.ind--;
    e.ln("}");
  } else if (pf2) {  // tile tt+1's words moved up; tile tt+2's load now
    for (int c = 0; c < ncols; ++c) {
      if (!s.cols[c].decode) continue;
      e.ln("#pragma unroll");
      e.ln("for (int i = 0; i < ", U * dwords_per(s, c), "; ++i) n", c, "[i] = m", c, "[i];");
    }
    for (int l = 0; l < nleaves; ++l)
      if (is_docmask(s.leaf_mode[l])) {
        e.ln("#pragma unroll");
        e.ln("for (int i = 0; i < ", U, "; ++i) nq", l, "[i] = mq", l, "[i];");
      }
    e.ln("rbn = rbm;");
    e.ln("if (tt + 2 < t2) ");
    emit_loads("tt + 2", "m", "rbm");
  } else {
    e.ln("if (tt + 1 < t2) ");
    emit_loads("tt + 1", "n");
  }
  if (scr_off >= 0) {
    // a tile (PT * PTL rows) lies inside one 65536-doc chunk: build that chunk's program masks when it changes (the next
    // tile's forward-index loads are already in flight)
    e.ln("if ((rb >> 16) != rc_cur) {");
    e.ln("  rc_cur = rb >> 16;");
    e.ln("  pgx_lds_barrier();");
    size_t k = 0;
    for (int l = 0; l < nleaves_all; ++l) {
      if (s.leaf_mode[l] != LEAF_RCHUNK) continue;
      const std::vector<int>& ops = s.rprog_ops[k++];
      e.ln("  pgx_rchunk_leaves<PT, ", rch_nl[l], ">(rp", l, ", (const PGX_G JRDesc*)A.rdesc, rc_cur, rlm", l, ", rscr);");
      e.ln("  pgx_lds_barrier();");
      bool has_not = false;
      for (int op : ops) has_not |= op == RP_NOT;
      e.ln("  for (int w = tid; w < 2048; w += PT) {");
      if (has_not) {
        e.ln("    const long long dw = ((long long)rc_cur << 16) + 32 * w;");
        e.ln("    const u32 keep = dw >= nd ? 0u : (dw + 32 > nd ? (1u << (nd - dw)) - 1u : 0xFFFFFFFFu);");
      }
      std::vector<std::string> st;
      int leaf = 0, tmp = 0;
      for (int op : ops) {
        const std::string X = "y" + std::to_string(tmp++);
        if (op == RP_LEAF) {
          e.ln("    const u32 ", X, " = rlm", l, "[", leaf++ * 2048, " + w];");
        } else if (op == RP_NOT) {
          e.ln("    const u32 ", X, " = ~", st.back(), " & keep;");
          st.pop_back();
        } else {
          const std::string b = st.back();
          st.pop_back();
          const std::string a = st.back();
          st.pop_back();
          e.ln("    const u32 ", X, " = ", a, op == RP_AND ? " & " : " | ", b, ";");
        }
        st.push_back(X);
      }
      e.ln("    rlm", l, "[w] = ", st.empty() ? std::string("0u") : st.back(), ";");
      e.ln("  }");
    }
    e.ln("  pgx_lds_barrier();");
    e.ln("}");
  }
  // The tile body is instantiated twice: for whole tiles (no per-row bound check) and for a segment's last tile.
  e.ln("auto body = [&](auto FT) {");
  e.ind = 4;
  e.ln("constexpr bool FULL = decltype(FT)::value;");
  for (int u = 0; u < U; ++u) {
    e.ln("{");
    e.ind = 5;
    e.ln("const int r0 = rb + ", u * s.R, " * PT + tid * PR;");
    for (int c = 0; c < ncols; ++c) {
      if (!s.cols[c].decode) continue;
      e.ln("u32 v", c, "[PR];");
      if (s.cols[c].frac)
        e.ln("pgx_unpack_frac<", s.cols[c].bits, ", PR, ", dwords_per(s, c), ">(&c", c, "[", u * dwords_per(s, c),
             "], (u32)(((long long)r0 * ", s.cols[c].bits, ") & 31), v", c, ");");
      else
        e.ln("pgx_unpack<", s.cols[c].bits, ", PR>(&c", c, "[", u * dwords_per(s, c), "], v", c, ");");
    }
    for (int l = 0; l < nleaves; ++l) {
      if (s.leaf_mode[l] == LEAF_RANGES) e.ln("const u32 W", l, " = pgx_ranges_bits(rg", l, ", nr", l, ", cur", l, ", r0, PR);");
      if (is_docmask(s.leaf_mode[l])) e.ln("const u32 W", l, " = cq", l, "[", u, "] >> (r0 & 31);");
      if (s.leaf_mode[l] == LEAF_RCHUNK) e.ln("const u32 W", l, " = rlm", l, "[(r0 & 0xFFFF) >> 5] >> (r0 & 31);");
    }
    // per-aggregation sub-step partials
    if (!grouped)
      for (int a = 0; a < naggs; ++a) {
        const int k = s.agg_kind[a];
        if ((k == A_SUM || k == A_AVG) && !s.cols[s.agg_col[a]].fp && s.cols[s.agg_col[a]].img != IMG_NONE &&
            s.cols[s.agg_col[a]].acc32)
          e.ln("u32 p", a, " = 0u;");
      }
    if (emit) e.ln("u64 recs[PR];");
    if (split) e.ln("u32 msk = 0u;");
    if (s.selmask) e.ln("u32 smk = 0u;");
    if (s.leafmask)
      for (int l = 0; l < nleaves; ++l) e.ln("u32 lw", l, " = 0u;");
    e.ln("#pragma unroll");
    e.ln("for (int j = 0; j < PR; ++j) {");
    e.ind = 6;
    e.ln("const bool vj = FULL || (r0 + j < nd);");
    // filter program over per-row predicates (lane masks: AND/OR become scalar ops on the wave's masks)
    std::vector<std::string> st;
    int tmp = 0;
    for (size_t pc = 0; pc < s.prog_op.size(); ++pc) {
      const int op = s.prog_op[pc], arg = s.prog_arg[pc];
      if (op == OP_LEAF) {
        const int l = arg, c = s.leaf_col[l];
        const std::string B = "b" + std::to_string(tmp++);
        const std::string v = "v" + std::to_string(c) + "[j]";
        switch (s.leaf_mode[l]) {
          case LEAF_SCAN_INTERVAL:
            e.ln("const bool ", B, " = vj && ((", v, " - lo", l, ") <= sp", l, ");");
            break;
          case LEAF_SCAN_BITSET:
            e.ln("const bool ", B, " = vj && ((bs", l, "[", v, " >> 5] >> (", v, " & 31u)) & 1u);");
            break;
          case LEAF_RANGES:
          case LEAF_DOCMASK:
          case LEAF_RCHUNK:
            e.ln("const bool ", B, " = vj && ((W", l, " >> j) & 1u);");
            break;
          case LEAF_DOCMASK_NOT:  // BitmapBasedFilterOperator NEQ / NOT_IN: flip of the OR of the non-matching bitmaps
            e.ln("const bool ", B, " = vj && !((W", l, " >> j) & 1u);");
            break;
          default:
            e.ln("const bool ", B, " = false;");
            break;
        }
        if (s.leafmask) e.ln("lw", l, " |= (u32)", B, " << j;");
        st.push_back(B);
      } else if (op == OP_AND || op == OP_OR) {
        for (int k = 1; k < arg; ++k) {
          const std::string b = st.back();
          st.pop_back();
          const std::string a = st.back();
          st.pop_back();
          const std::string X = "x" + std::to_string(tmp++);
          e.ln("const bool ", X, " = ", a, op == OP_AND ? " & " : " | ", b, ";");
          st.push_back(X);
        }
      } else if (op == OP_STAT) {
        e.ln("st_ent += __popcll(__ballot(", st.back(), "));");
      } else if (op == OP_TRUE) {
        st.push_back("vj");
      }
    }
    e.ln("const bool m = ", st.empty() ? std::string("vj") : st.back(), ";");
    e.ln("wcnt += __popcll(__ballot(m));");
    if (s.selmask) e.ln("smk |= (u32)m << j;");
    if (compact) {
      const int ncw = int(std::max<size_t>(1, ccols.size()));
      e.ln("msk |= (u32)m << j;");
      e.ind = 5;
      e.ln("}");
      e.ln("const u32 ccnt = __popc(msk);");
      e.ln("u32 cinc = ccnt;");
      e.ln("#pragma unroll");
      e.ln("for (int d = 1; d < 64; d <<= 1) { const u32 y = __shfl_up(cinc, d, 64); if (lane >= d) cinc += y; }");
      e.ln("const u32 cexc = cinc - ccnt;");
      e.ln("const u32 ctot = __shfl(cinc, 63, 64);");
      e.ln("for (u32 cb = 0; cb < ctot; cb += 64) {");
      e.ind = 6;
      e.ln("u32 ck = cexc;");
      e.ln("#pragma unroll");
      e.ln("for (int j = 0; j < PR; ++j)");
      e.ln("  if ((msk >> j) & 1u) {");
      e.ln("    const u32 sl = ck - cb;");
      e.ln("    if (sl < 64u) {");
      for (size_t i = 0; i < ccols.size(); ++i) e.ln("      cstg[sl * ", ncw, " + ", i, "] = v", ccols[i], "[j];");
      e.ln("    }");
      e.ln("    ++ck;");
      e.ln("  }");
      e.ln("pgx_wave_lds_sync();");
      e.ln("const bool m = (u32)lane < ((ctot - cb) < 64u ? (ctot - cb) : 64u);");
      e.ln("{");
      e.ind = 7;
      e.ln("const int j = 0;");
      for (size_t i = 0; i < ccols.size(); ++i)
        e.ln("u32 v", ccols[i], "[1] = {m ? cstg[lane * ", ncw, " + ", i, "] : 0u};");
      for (int c = 0; c < ncols; ++c)
        if (gcolv[c]) e.ln(s.cols[c].fp ? "double" : "i64", " gv", c, "[1] = {m ? ", s.cols[c].fp ? "dd" : "di", c,
                           "[v", c, "[0]] : 0};");
      for (size_t g = 0; g < s.gcol.size(); ++g)
        if (gremap[g]) e.ln("u32 gr", g, "[1] = {m ? (u32)rm", g, "[v", s.gcol[g], "[0]] : 0u};");
    } else if (split) {
      e.ln("msk |= (u32)m << j;");
      e.ind = 5;
      e.ln("}");
      for (int c = 0; c < ncols; ++c)
        if (gcolv[c]) {
          const bool fp = s.cols[c].fp;
          e.ln(fp ? "double" : "i64", " gv", c, "[PR];");
          e.ln("#pragma unroll");
          e.ln("for (int j = 0; j < PR; ++j) gv", c, "[j] = ((msk >> j) & 1u) ? ", fp ? "dd" : "di", c, "[v", c,
               "[j]] : 0;");
        }
      for (size_t g = 0; g < s.gcol.size(); ++g)
        if (gremap[g]) {
          const int c = s.gcol[g];
          e.ln("u32 gr", g, "[PR];");
          e.ln("#pragma unroll");
          e.ln("for (int j = 0; j < PR; ++j) gr", g, "[j] = ((msk >> j) & 1u) ? (u32)rm", g, "[v", c, "[j]] : 0u;");
        }
      e.ln("#pragma unroll");
      e.ln("for (int j = 0; j < PR; ++j) {");
      e.ind = 6;
      e.ln("const bool m = (msk >> j) & 1u;");
    }
    // dense group-by update of the row (j, m) in scope
    auto emit_dense = [&]() {
      // dense group-by: key = sum_g id_g * mul_g (column 0 least significant, DefaultGroupKeyGenerator.java:230-237)
      e.ln("if (m) {");
      e.ind = 7;
      std::string key;
      for (size_t g = 0; g < s.gcol.size(); ++g) {
        const int c = s.gcol[g];
        std::string id = "v" + std::to_string(c) + "[j]";
        if (s.cols[c].remap) id = gremap[g] ? "gr" + std::to_string(g) + "[j]" : "(u32)rm" + std::to_string(g) + "[" + id + "]";
        if (!key.empty()) key += " + ";
        key += id + " * " + std::to_string(s.gmul[g]) + "u";
      }
      e.ln("const u32 key = ", key.empty() ? "0u" : key, ";");
      if (pack) {  // count and value offset in one add (the segment flush splits them and adds count * vbase)
        const int c = s.agg_col[0];
        e.ln("atomicAdd(&tab[key], (1ull << ", s.dense_pack, ") + (u64)", img_value(s, c, img_off, "v" + std::to_string(c) + "[j]"),
             ");");
        e.ind = 6;
        e.ln("}");
        return;
      }
      e.ln("atomicAdd(&tab[key], 1ull);");
      for (int a = 0; a < naggs; ++a) {
        const int k = s.agg_kind[a];
        if (k == A_COUNT) continue;
        const int c = s.agg_col[a];
        const JitCol& C = s.cols[c];
        const std::string id = "v" + std::to_string(c) + "[j]";
        std::string val;  // i64 or double expression
        if (C.fp) val = (C.img == IMG_F64) ? "((const double*)lds)[" + std::to_string(img_off[c] / 8) + " + " + id + "]"
                                            : (gcolv[c] ? "gv" + std::to_string(c) + "[j]" : "dd" + std::to_string(c) + "[" + id + "]");
        else if (C.img == IMG_NONE) val = gcolv[c] ? "gv" + std::to_string(c) + "[j]" : "di" + std::to_string(c) + "[" + id + "]";
        else val = "(vb" + std::to_string(c) + " + (i64)" + img_value(s, c, img_off, id) + ")";
        std::string enc;
        if (k == A_MIN || k == A_MAX) enc = C.fp ? "pgx_ord_f64(" + val + ")" : "pgx_ord_i64(" + val + ")";
        else enc = C.fp ? "pgx_f64_bits(" + val + ")" : "(u64)" + val;
        e.ln(plane_atomic(s.plane_op[a + 1], "&tab[" + std::to_string((a + 1) * s.dense_slots) + " + key]", enc));
      }
      e.ind = 6;
      e.ln("}");
    };
    // hash group-by: the packed raw key (LONG_MAP / ARRAY_MAP, DefaultGroupKeyGenerator.java:239-246), a slot of the
    // workgroup's LDS table, or of the global table when the LDS one has no room for it
    auto emit_hash = [&]() {
      e.ln("if (m) {");
      e.ind = 7;
      std::string klo = "0ull", khi = "0ull";
      for (size_t g = 0; g < s.gcol.size(); ++g) {
        const int c = s.gcol[g];
        std::string id = "v" + std::to_string(c) + "[j]";
        if (s.cols[c].remap) id = gremap[g] ? "gr" + std::to_string(g) + "[j]" : "(u32)rm" + std::to_string(g) + "[" + id + "]";
        const std::string part = " | ((u64)" + id + " << " + std::to_string(s.gshift[g]) + ")";
        if (h128 && s.ghi[g]) khi += part;
        else klo += part;
      }
      e.ln("const u64 klo = ", klo, ";");
      if (h128) e.ln("const u64 khi = ", khi, ";");
      std::vector<std::string> encs(naggs);
      for (int a = 0; a < naggs; ++a) {
        const int k = s.agg_kind[a];
        if (k == A_COUNT) continue;
        const int c = s.agg_col[a];
        const JitCol& C = s.cols[c];
        const std::string id = "v" + std::to_string(c) + "[j]";
        std::string val;
        if (C.fp) val = (C.img == IMG_F64) ? "((const double*)lds)[" + std::to_string(img_off[c] / 8) + " + " + id + "]"
                                            : (gcolv[c] ? "gv" + std::to_string(c) + "[j]" : "dd" + std::to_string(c) + "[" + id + "]");
        else if (C.img == IMG_NONE) val = gcolv[c] ? "gv" + std::to_string(c) + "[j]" : "di" + std::to_string(c) + "[" + id + "]";
        else val = "(vb" + std::to_string(c) + " + (i64)" + img_value(s, c, img_off, id) + ")";
        if (k == A_MIN || k == A_MAX) encs[a] = C.fp ? "pgx_ord_f64(" + val + ")" : "pgx_ord_i64(" + val + ")";
        else encs[a] = C.fp ? "pgx_f64_bits(" + val + ")" : "(u64)" + val;
      }
      // the values (LDS image reads) are read before the probe, so their round trip overlaps the probe's
      for (int a = 0; a < naggs; ++a)
        if (s.agg_kind[a] != A_COUNT) {
          e.ln("const u64 ev", a, " = ", encs[a], ";");
          encs[a] = "ev" + std::to_string(a);
        }
      if (hpack) {
        const int c = s.agg_col[0];
        e.ln("const u64 hv = (1ull << ", s.dense_pack, ") + (u64)", img_value(s, c, img_off, "v" + std::to_string(c) + "[j]"),
             ";");
      }
      e.ln("const int ls = ", h128 ? "pgx_lhash128(hk, hst, " + std::to_string(HS) + ", klo, khi)"
                                   : "pgx_lhash64(hk, " + std::to_string(HS) + ", klo)", ";");
      e.ln("if (ls >= 0) {");
      if (hpack) {
        e.ln("  atomicAdd(&ht[ls], hv);");
      } else {
        e.ln("  atomicAdd(&ht[ls], 1ull);");
        for (int a = 0; a < naggs; ++a)
          if (s.agg_kind[a] != A_COUNT)
            e.ln("  ", plane_atomic(s.plane_op[a + 1], "&ht[" + std::to_string((a + 1) * HS) + " + ls]", encs[a]));
      }
      e.ln("} else {");
      e.ln("  const long long gs = ", h128 ? "pgx_ghash128((PGX_G unsigned long long*)A.hkeys, (PGX_G unsigned int*)A.hstate, A.hash_cap, klo, khi, A.overflow)"
                                           : "pgx_ghash64((PGX_G unsigned long long*)A.hkeys, A.hash_cap, klo, A.overflow)", ";");
      e.ln("  if (gs < 0) {");
      e.ln("    atomicAdd(A.overflow, 1ull);");
      e.ln("  } else {");
      e.ln("    atomicAdd(A.table + gs, 1ull);");
      for (int a = 0; a < naggs; ++a)
        if (s.agg_kind[a] != A_COUNT)
          e.ln("    ", plane_atomic(s.plane_op[a + 1], "A.table + " + std::to_string(a + 1) + " * A.hash_cap + gs", encs[a]));
      e.ln("  }");
      e.ln("}");
      e.ind = 6;
      e.ln("}");
    };
    if (!grouped) {
      for (int a = 0; a < naggs; ++a) {
        const int k = s.agg_kind[a];
        if (k == A_COUNT) continue;
        const int c = s.agg_col[a];
        const JitCol& C = s.cols[c];
        const std::string v = "v" + std::to_string(c) + "[j]";
        if (k == A_MIN) {
          e.ln("mn", a, " = min(mn", a, ", m ? ", v, " : 0xFFFFFFFFu);");
        } else if (k == A_MAX) {
          e.ln("mx", a, " = max(mx", a, ", m ? ", v, " : 0u);");
        } else if (C.fp) {
          const std::string val = (C.img == IMG_F64)
                                      ? "((const double*)lds)[" + std::to_string(img_off[c] / 8) + " + " + v + "]"
                                      : (gcolv[c] ? "gv" + std::to_string(c) + "[j]" : "dd" + std::to_string(c) + "[" + v + "]");
          e.ln("if (m) acc", a, " += ", val, ";");
        } else if (C.img == IMG_NONE) {
          if (gcolv[c]) e.ln("acc", a, " += gv", c, "[j];");  // 0 for unselected rows
          else e.ln("if (m) acc", a, " += di", c, "[", v, "];");
        } else if (C.acc32) {
          e.ln("{ const u32 x = ", img_value(s, c, img_off, v), "; p", a, " += m ? x : 0u; }");
        } else {
          e.ln("{ const u32 x = ", img_value(s, c, img_off, v), "; acc", a, " += m ? (u64)x : 0ull; }");
        }
      }
    } else {
      if (emit) {
        // partitioned group-by: one record per row (~0 = not selected); key packing as the LONG_MAP raw key
        // (DefaultGroupKeyGenerator.java:239-246: dictIds at fixed bit offsets)
        e.ln("u64 rec = ~0ull;");
        e.ln("if (m) {");
        std::string key = "0ull";
        for (size_t g = 0; g < s.gcol.size(); ++g) {
          const int c = s.gcol[g];
          std::string id = "v" + std::to_string(c) + "[j]";
          if (s.cols[c].remap) id = "(u32)rm" + std::to_string(g) + "[" + id + "]";
          key += " | ((u64)" + id + " << " + std::to_string(s.gshift[g]) + ")";
        }
        std::string x = "0u";
        if (s.emit_col >= 0) {
          const std::string ec = std::to_string(s.emit_col);
          // the value's dictId, looked up at aggregation (narrow: the sorted dictionary, rebase 0; FLOAT / DOUBLE: the
          // segment's place in the concatenated dictionaries)
          if (s.emit_dictid) x = "(u32)(v" + ec + "[j] + (u32)S->emit_rebase)";
          else x = s.cols[s.emit_col].img != IMG_NONE
                       ? "(u32)(" + img_value(s, s.emit_col, img_off, "v" + ec + "[j]") + " + (u32)S->emit_rebase)"
                       : "(u32)(di" + ec + "[v" + ec + "[j]] - S->vbase[" + ec + "] + S->emit_rebase)";
        }
        if (enarrow) {  // mix the key (NarrowMix), bucket = top part_bits of the mix (bits 56.. of rec), record below
          const NarrowMix mx = narrow_mix(s.keybits);
          const std::string M = std::to_string(mx.mask) + "ull";
          e.ln("  u64 h = ((", key, ") * ", mx.c1, "ull) & ", M, ";");
          e.ln("  h ^= h >> ", mx.s, ";");
          e.ln("  rec = ((h >> ", nrb1, ") << 56) | (h & ", (uint64_t(1) << nrb1) - 1u, "ull) | ((u64)(", x, ") << ", nrb1,
               ");");
        } else {
          e.ln("  rec = (", key, ") | ((u64)(", x, ") << ", s.keybits, ");");
        }
        e.ln("}");
        e.ln("recs[j] = rec;");
      } else if (hashm) {
        emit_hash();
      } else {
        emit_dense();
      }
    }
    e.ind = 5;
    e.ln("}");
    if (compact) {
      e.ln("  pgx_wave_lds_sync();");
      e.ln("}");
    }
    if (!grouped)
      for (int a = 0; a < naggs; ++a) {
        const int k = s.agg_kind[a];
        if ((k == A_SUM || k == A_AVG) && !s.cols[s.agg_col[a]].fp && s.cols[s.agg_col[a]].img != IMG_NONE &&
            s.cols[s.agg_col[a]].acc32)
          e.ln("acc", a, " += p", a, ";");
      }
    if (s.selmask) {  // the lane's PR selection bits (r0 is a multiple of PR, PR divides 32)
      const char* ty = s.R == 8 ? "unsigned char" : (s.R == 16 ? "unsigned short" : "unsigned int");
      e.ln("if (FULL || r0 < nd) ((PGX_G ", ty, "*)S->selmask)[r0 / PR] = (", ty, ")smk;");
    }
    if (s.leafmask) {
      // the lane's PR rows are PR consecutive bits of the leaf's mask (r0 is a multiple of PR, PR divides 32)
      const char* ty = s.R == 8 ? "unsigned char" : (s.R == 16 ? "unsigned short" : "unsigned int");
      e.ln("if (FULL || r0 < nd) {");
      for (int l = 0; l < nleaves; ++l)
        e.ln("  ((PGX_G ", ty, "*)(S->lmask + ", l, " * S->lmask_words))[r0 / PR] = (", ty, ")lw", l, ";");
      e.ln("}");
    }
    if (enarrow) {
      // Narrow split of this sub-step's records 256 ways through per-bucket LDS rings (software write combining).
      // Bucket b's records go to this workgroup's slab of b at consecutive positions (an LDS cursor per bucket: the
      // atomic returns the position); a record is held in the ring slot (position mod kNarrowRing) until its 32-record
      // unit is complete, and whole units leave as one 128-B u32 line (+ one 64-B u16 line) each, written by 32
      // consecutive lanes.  Stores of partial units would leave as separate partial-line writes (the L2 does not
      // merge them across sub-steps).  Per sub-step: positions (atomics) | A | four owner wavefronts (a bucket per
      // lane) list the units that complete, every lane writes its records into the rings | B | every wavefront
      // writes listed units.  The ring holds positions [U, U + kNarrowRing) (U: first unflushed unit); a record
      // beyond that (a key-skewed sub-step) is stored straight to the slab, and the ring's copy of positions below V
      // (ring-valid-from) is ignored.  Two buffers of U and V: the owners write the next sub-step's while this one's
      // are read.
      const std::string NR = std::to_string(NRG), NUs = std::to_string(NU);
      e.ln("{");
      e.ln("  u32 pp[PR];");
      e.ln("  #pragma unroll");
      e.ln("  for (int j = 0; j < PR; ++j) pp[j] = recs[j] != ~0ull ? atomicAdd(&ncur[(u32)(recs[j] >> 56)], 1u) : 0u;");
      e.ln("  pgx_lds_barrier();");
      e.ln("  const u32* const Ucur = nU + npar * 256;");
      e.ln("  const u32* const Vcur = nV + npar * 256;");
      e.ln("  if (tid < 256) {");
      e.ln("    const u32 en = ncur[tid], u0 = Ucur[tid], v0 = Vcur[tid];");
      e.ln("    const u32 lim = u0 + ", NR, "u;");
      e.ln("    const u32 nu = (((en < lim) ? en : lim) - u0) / ", NUs, "u;");
      e.ln("    nU[(npar ^ 1) * 256 + tid] = en & ~", NU - 1, "u;");
      e.ln("    nV[(npar ^ 1) * 256 + tid] = en > lim ? en : v0;");
      e.ln("    u32 incl = nu;");
      e.ln("    #pragma unroll");
      e.ln("    for (int d = 1; d < 64; d <<= 1) {");
      e.ln("      const u32 y = __shfl_up(incl, d, 64);");
      e.ln("      if (lane >= d) incl += y;");
      e.ln("    }");
      e.ln("    const int w = tid >> 6;");
      e.ln("    for (u32 q = 0, k = incl - nu; q < nu; ++q, ++k) {");
      e.ln("      nlb[w * 128 + k] = (unsigned short)tid;");
      e.ln("      nlp[w * 128 + k] = u0 + ", NUs, "u * q;");
      e.ln("    }");
      e.ln("    if (lane == 63) nlc[w] = incl;");
      e.ln("  }");
      e.ln("  #pragma unroll");
      e.ln("  for (int j = 0; j < PR; ++j)");
      e.ln("    if (recs[j] != ~0ull) {");
      e.ln("      const u32 b = (u32)(recs[j] >> 56);");
      e.ln("      const u32 pos = pp[j];");
      e.ln("      if (pos < Ucur[b] + ", NR, "u) {");
      e.ln("        ringA[b * ", NR, "u + (pos & ", NRG - 1, "u)] = (u32)recs[j];");
      if (nhib) e.ln("        ringB[b * ", NR, "u + (pos & ", NRG - 1, "u)] = (unsigned short)(recs[j] >> 32);");
      e.ln("      } else if (pos < (u32)A.part_cap) {  // past the ring (key skew): straight to the slab");
      e.ln("        const long long o = ((long long)b * A.part_nwg + wsl) * A.part_cap + (long long)pos;");
      e.ln("        poutA[o] = (u32)recs[j];");
      if (nhib) e.ln("        poutB[o] = (unsigned short)(recs[j] >> 32);");
      e.ln("      }");
      e.ln("    }");
      e.ln("  pgx_lds_barrier();");
      // NU / 4 lanes per unit, 16 bytes each (u32: 4 records per lane; u16: the first NU / 8 lanes x 8 records); a
      // unit holding positions below V (after a skewed sub-step) goes record by record
      const int LPU = NU / 4, UPW = 64 / LPU;  // lanes per unit, units per wavefront instruction
      e.ln("  {");
      e.ln("    const int w = tid >> 6, l = w & 3, g = lane & ", LPU - 1, ";");
      e.ln("    const int cnt = (int)nlc[l];");
      e.ln("    for (int k = (w >> 2) * ", UPW, " + (lane / ", LPU, "); k < cnt; k += ", UPW, " * (PT / 256)) {");
      e.ln("      const u32 b = nlb[l * 128 + k];");
      e.ln("      const u32 u = nlp[l * 128 + k];");
      e.ln("      if (u >= (u32)A.part_cap) continue;");
      e.ln("      const long long o = ((long long)b * A.part_nwg + wsl) * A.part_cap + (long long)u;");
      e.ln("      const u32 rs = b * ", NR, "u + (u & ", NRG - 1, "u);");
      e.ln("      if (u >= Vcur[b]) {");
      e.ln("        *(PGX_G pgx_u32x4*)(poutA + o + 4 * g) = *(const pgx_u32x4*)(ringA + rs + 4 * g);");
      if (nhib)
        e.ln("        if (g < ", NU / 8, ") *(PGX_G pgx_u32x4*)(poutB + o + 8 * g) = *(const pgx_u32x4*)(ringB + rs + 8 * g);");
      e.ln("      } else {");
      e.ln("        for (int q = 0; q < 4; ++q) {");
      e.ln("          const u32 x = 4 * g + q;");
      e.ln("          if (u + x < Vcur[b]) continue;");
      e.ln("          poutA[o + x] = ringA[rs + x];");
      if (nhib) e.ln("          poutB[o + x] = ringB[rs + x];");
      e.ln("        }");
      e.ln("      }");
      e.ln("    }");
      e.ln("  }");
      e.ln("  npar ^= 1;");
      e.ln("}");
    } else if (emit && stg_recs) {
      const int L = stg_recs / s.R;  // lanes whose records fill one round
      int lg = 0;
      while ((1 << lg) < L) ++lg;
      e.ln("{");
      e.ln("  u64* stg = (u64*)(lds + ", stg_off / 4, ") + (tid >> 6) * ", L * stg_pitch, ";");
      e.ln("  const int w0 = r0 - lane * PR;  // first row of this wave's slice");
      e.ln("  PGX_G u64* out = (PGX_G u64*)A.table + S->rec_base + w0;");
      e.ln("  #pragma unroll");
      e.ln("  for (int rd = 0; rd < ", 64 * s.R / stg_recs, "; ++rd) {");
      e.ln("    if ((lane >> ", lg, ") == rd) {");
      e.ln("      u64* d = stg + (lane & ", L - 1, ") * ", stg_pitch, ";");
      e.ln("      #pragma unroll");
      e.ln("      for (int j = 0; j < PR; ++j) d[j] = recs[j];");
      e.ln("    }");
      e.ln("    __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");");
      e.ln("    __builtin_amdgcn_wave_barrier();");
      e.ln("    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");");
      e.ln("    #pragma unroll");
      e.ln("    for (int k = 0; k < ", stg_recs / 64, "; ++k) {");
      e.ln("      const int i = k * 64 + lane;");
      e.ln("      const int row = rd * ", stg_recs, " + i;");
      e.ln("      if (FULL || w0 + row < nd) __builtin_nontemporal_store(stg[(i / PR) * ", stg_pitch, " + (i % PR)], out + row);");
      e.ln("    }");
      e.ln("    __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");");
      e.ln("    __builtin_amdgcn_wave_barrier();");
      e.ln("    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");");
      e.ln("  }");
      e.ln("}");
    } else if (emit) {
      e.ln("#pragma unroll");
      e.ln("for (int j = 0; j < PR; ++j) if (FULL || r0 + j < nd) A.table[S->rec_base + r0 + j] = recs[j];");
    }
    e.ind = 4;
    e.ln("}");
  }
  e.ind = 3;
  e.ln("};");
  e.ln("if (rb + PT * PTL <= nd) body(pgx_bool<true>{}); else body(pgx_bool<false>{});");
  e.ind = 2;
  e.ln("}");
  // per-segment flush of the lane accumulators (values depend on this segment's dictionaries)
  e.ln("st_docs += wcnt;");
  if (!grouped) {
    for (int a = 0; a < naggs; ++a) {
      const int k = s.agg_kind[a];
      if (k == A_COUNT) continue;
      const int c = s.agg_col[a];
      const JitCol& C = s.cols[c];
      e.ln("{");
      e.ind++;
      if (k == A_SUM || k == A_AVG) {
        if (C.fp) {
          e.ln("const double x = pgx_wsum_f64(acc", a, ");");
          e.ln("if (lane == 0) atomicAdd((double*)&s_acc[", a + 1, "], x);");
        } else if (C.img == IMG_NONE) {
          e.ln("const u64 x = pgx_wsum_u64((u64)acc", a, ");");
          e.ln("if (lane == 0) atomicAdd(&s_acc[", a + 1, "], x);");
        } else {
          e.ln("const u64 x = pgx_wsum_u64(acc", a, ");");
          e.ln("if (lane == 0) atomicAdd(&s_acc[", a + 1, "], x + wcnt * (u64)vb", c, ");");
        }
      } else {
        const bool mn = k == A_MIN;
        const std::string id = (mn ? "mn" : "mx") + std::to_string(a);
        const std::string v = C.fp ? "pgx_ord_f64(dd" + std::to_string(c) + "[" + id + "])"
                                   : "pgx_ord_i64(di" + std::to_string(c) + "[" + id + "])";
        e.ln("u64 x = ", mn ? "~0ull" : "0ull", ";");
        e.ln("if (", mn ? "mn" + std::to_string(a) + " != 0xFFFFFFFFu" : std::string("wcnt"), ") x = ", v, ";");
        e.ln("x = ", mn ? "pgx_wmin_u64(x)" : "pgx_wmax_u64(x)", ";");
        e.ln("if (lane == 0) ", mn ? "atomicMin" : "atomicMax", "(&s_acc[", a + 1, "], x);");
      }
      e.ind--;
      e.ln("}");
    }
  }
  if (hpack) {  // per-segment flush of the packed LDS hash planes into the global table (the keys stay)
    const int c = s.agg_col[0];
    const std::string mask = std::to_string((1ull << s.dense_pack) - 1ull) + "ull";
    e.ln("__syncthreads();");
    e.ln("for (int i = tid; i < ", HS, "; i += PT) {");
    e.ln("  const u64 x = ht[i];");
    e.ln("  if (x == 0ull) continue;");
    e.ln("  const long long gs = ", h128 ? "pgx_ghash128((PGX_G unsigned long long*)A.hkeys, (PGX_G unsigned int*)A.hstate, A.hash_cap, hk[2 * i], hk[2 * i + 1], A.overflow)"
                                         : "pgx_ghash64((PGX_G unsigned long long*)A.hkeys, A.hash_cap, hk[i], A.overflow)", ";");
    e.ln("  const u64 cnt = x >> ", s.dense_pack, ";");
    e.ln("  if (gs < 0) {");
    e.ln("    atomicAdd(A.overflow, cnt);");
    e.ln("  } else {");
    e.ln("    atomicAdd(A.table + gs, cnt);");
    e.ln("    atomicAdd(A.table + A.hash_cap + gs, (x & ", mask, ") + cnt * (u64)vb", c, ");");
    e.ln("  }");
    e.ln("  ht[i] = 0ull;");
    e.ln("}");
    e.ln("__syncthreads();");
  }
  if (pack) {  // per-segment flush of the packed table: counts and sums (offset sums + count * this segment's vbase)
    const int c = s.agg_col[0];
    const std::string mask = std::to_string((1ull << s.dense_pack) - 1ull) + "ull";
    e.ln("__syncthreads();");
    e.ln("for (int i = tid; i < ", s.dense_slots, "; i += PT) {");
    e.ln("  const u64 x = tab[i];");
    e.ln("  if (x == 0ull) continue;");
    e.ln("  const u64 cnt = x >> ", s.dense_pack, ";");
    e.ln("  atomicAdd(A.table + i, cnt);");
    e.ln("  atomicAdd(A.table + ", s.dense_slots, " + i, (x & ", mask, ") + cnt * (u64)vb", c, ");");
    e.ln("  tab[i] = 0ull;");
    e.ln("}");
    e.ln("__syncthreads();");
  }
  e.ln("t = t2;");
  e.ln("++seg;");
  e.ind = 1;
  e.ln("}");
  e.ln("{");
  e.ln("  const u64 d = st_docs, x = st_ent;  // wave-uniform counts");
  e.ln("  if (lane == 0) {");
  e.ln("    if (d) atomicAdd(A.stats, d);");
  e.ln("    if (x) atomicAdd(A.stats + 1, x);");
  if (!grouped) e.ln("    if (d) atomicAdd(&s_acc[0], d);");
  e.ln("  }");
  e.ln("}");
  e.ln("__syncthreads();");
  if (hashm && !hpack) {  // the workgroup's LDS table into the global one (identity planes merge harmlessly)
    e.ln("for (int i = tid; i < ", HS, "; i += PT) {");
    if (h128) {
      e.ln("  if (hst[i] != 2u) continue;");
      e.ln("  const long long gs = pgx_ghash128((PGX_G unsigned long long*)A.hkeys, (PGX_G unsigned int*)A.hstate, A.hash_cap, hk[2 * i], hk[2 * i + 1], A.overflow);");
    } else {
      e.ln("  if (hk[i] == ~0ull) continue;");
      e.ln("  const long long gs = pgx_ghash64((PGX_G unsigned long long*)A.hkeys, A.hash_cap, hk[i], A.overflow);");
    }
    e.ln("  if (gs < 0) {");
    e.ln("    atomicAdd(A.overflow, ht[i]);");
    e.ln("    continue;");
    e.ln("  }");
    e.ln("  atomicAdd(A.table + gs, ht[i]);");
    for (int a = 0; a < naggs; ++a)
      if (s.agg_kind[a] != A_COUNT)
        e.ln("  ", plane_atomic(s.plane_op[a + 1], "A.table + " + std::to_string(a + 1) + " * A.hash_cap + gs",
                               "ht[" + std::to_string((a + 1) * HS) + " + i]"));
    e.ln("}");
  }
  if (enarrow) {  // the rings' last partial units, then the slab fills (every record, also past part_cap)
    const std::string NR = std::to_string(NRG);
    e.ln("for (int x = tid; x < 256 * ", NU, "; x += PT) {");
    e.ln("  const u32 b = (u32)x / ", NU, "u;");
    e.ln("  const u32 i = nU[npar * 256 + b] + ((u32)x & ", NU - 1, "u);");
    e.ln("  if (i < ncur[b] && i >= nV[npar * 256 + b] && i < (u32)A.part_cap) {");
    e.ln("    const long long o = ((long long)b * A.part_nwg + wsl) * A.part_cap + (long long)i;");
    e.ln("    poutA[o] = ringA[b * ", NR, "u + (i & ", NRG - 1, "u)];");
    if (nhib) e.ln("    poutB[o] = ringB[b * ", NR, "u + (i & ", NRG - 1, "u)];");
    e.ln("  }");
    e.ln("}");
    e.ln("for (int i = tid; i < 256; i += PT) {");
    e.ln("  const u32 h = ncur[i];");
    e.ln("  A.part_cursor[((long long)i * A.part_nwg + wsl) * A.part_cstride] = h;");
    e.ln("  if (h > (u32)A.part_cap) atomicAdd(A.part_overflow, 1ull);");
    e.ln("}");
  }
  if (!grouped) {
    e.ln("if (tid < ", s.num_planes, ") {");
    e.ind++;
    for (int p = 0; p < s.num_planes; ++p) {
      if (p > 0 && s.agg_kind[p - 1] == A_COUNT) continue;
      const int op = p == 0 ? P_ADD_I64 : s.plane_op[p];
      e.ln("if (tid == ", p, ") ", plane_atomic(op, "A.agg_out + " + std::to_string(p), "s_acc[" + std::to_string(p) + "]"));
    }
    e.ind--;
    e.ln("}");
  }
  if (s.group_mode == G_DENSE_LDS && !pack) {
    e.ln("for (int i = tid; i < ", s.dense_slots * s.num_planes, "; i += PT) {");
    e.ind++;
    e.ln("const int p = i / ", s.dense_slots, ";");
    e.ln("const int sl = i - p * ", s.dense_slots, ";");
    e.ln("if (tab[sl] == 0ull) continue;");
    e.ln("u64* g = A.table + i;");
    e.ln("const u64 x = tab[i];");
    for (int p = 0; p < s.num_planes; ++p)
      e.ln("if (p == ", p, ") ", plane_atomic(p == 0 ? P_ADD_I64 : s.plane_op[p], "g", "x"));
    e.ind--;
    e.ln("}");
  }
  e.ind = 0;
  e.ln("}");
  return e.o.str();
}

namespace {

struct JitEntry {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  int lds = 0;
};

std::mutex g_jit_mu;
std::map<std::pair<int, std::string>, JitEntry> g_jit_cache;

}  // namespace

// Every field of a shape that the generated source depends on, flattened: the per-query lookup key (generating the
// source text to find a cached kernel cost ~14 us per query).
std::vector<int64_t> shape_key(const JitShape& s, int device) {
  std::vector<int64_t> k{device, s.T, s.R, s.TL, s.group_mode, int64_t(s.dense_slots), s.num_planes, s.keybits, s.emit_col,
                         int64_t(s.cols.size()), s.leafmask};
  for (const JitCol& c : s.cols)
    k.insert(k.end(), {c.bits, c.decode, c.img, c.img_sh, c.img_words, c.acc32, c.fp, c.remap, c.frac});
  auto add = [&](const auto& v) {
    k.push_back(-int64_t(v.size()) - 1);
    for (auto x : v) k.push_back(int64_t(x));
  };
  add(s.leaf_col);
  add(s.leaf_mode);
  add(s.prog_op);
  add(s.prog_arg);
  add(s.agg_kind);
  add(s.agg_col);
  add(s.plane_op);
  add(s.gcol);
  add(s.gmul);
  add(s.gshift);
  for (const auto& ops : s.rprog_ops) add(ops);
  k.push_back(s.part_bits);
  k.push_back(s.emit_dictid);
  k.push_back(s.part_slab);
  k.push_back(s.dense_pack);
  k.push_back(s.compact);
  k.push_back(s.selmask);
  k.push_back(s.part_narrow);
  k.push_back(s.narrow_vbits);
  k.push_back(s.narrow_unit);
  k.push_back(s.prefetch2);
  add(s.ghi);
  k.push_back(s.hash_slots);
  return k;
}

std::map<std::vector<int64_t>, JitEntry> g_jit_shapes;  // shape key -> compiled entry (same entries as g_jit_cache)

// Persistent code-object cache (opt-in): with PGX_JIT_CACHE=<directory> a server restart (or a new process on the same
// host) reuses the kernels earlier processes compiled instead of paying hiprtc (~0.4 s per new query shape).  Unset:
// no file is read or written.  File name: FNV-1a of the source and the compile options; the file starts with a second,
// independent hash of the same text, checked on load.
constexpr const char* kJitOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};

std::string jit_cache_dir() {
  const char* d = std::getenv("PGX_JIT_CACHE");
  return d && *d ? d : "";
}

uint64_t text_hash(const std::string& t, uint64_t h, uint64_t mul) {
  for (unsigned char c : t) {
    h ^= c;
    h *= mul;
  }
  return h;
}

std::string cache_text(const std::string& src) {
  std::string t = src;
  for (const char* o : kJitOpts) t += std::string("\n//") + o;
  return t;
}

std::string cache_path(const std::string& dir, const std::string& text) {
  char name[64];
  std::snprintf(name, sizeof name, "/pgxq_%016llx.co",
                static_cast<unsigned long long>(text_hash(text, 1469598103934665603ull, 1099511628211ull)));
  return dir + name;
}

bool cache_load(const std::string& src, std::string* code) {
  const std::string dir = jit_cache_dir();
  if (dir.empty()) return false;
  const std::string text = cache_text(src);
  FILE* f = std::fopen(cache_path(dir, text).c_str(), "rb");
  if (!f) return false;
  uint64_t check = 0;
  bool ok = std::fread(&check, 8, 1, f) == 1 && check == text_hash(text, 0x9E3779B97F4A7C15ull, 0x100000001B3ull);
  if (ok) {
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f) - 8;
    ok = n > 0;
    if (ok) {
      code->resize(size_t(n));
      std::fseek(f, 8, SEEK_SET);
      ok = std::fread(&(*code)[0], 1, size_t(n), f) == size_t(n);
    }
  }
  std::fclose(f);
  return ok;
}

void cache_store(const std::string& src, const std::string& code) {
  const std::string dir = jit_cache_dir();
  if (dir.empty()) return;
  std::string cmd_dir = dir;  // create the directory chain
  for (size_t i = 1; i <= cmd_dir.size(); ++i)
    if (i == cmd_dir.size() || cmd_dir[i] == '/') mkdir(cmd_dir.substr(0, i).c_str(), 0755);
  const std::string text = cache_text(src);
  const std::string path = cache_path(dir, text);
  const std::string tmp = path + ".tmp" + std::to_string(getpid());
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;
  const uint64_t check = text_hash(text, 0x9E3779B97F4A7C15ull, 0x100000001B3ull);
  const bool ok = std::fwrite(&check, 8, 1, f) == 1 && std::fwrite(code.data(), 1, code.size(), f) == code.size();
  std::fclose(f);
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());
}

void* jit_function(const JitShape& s, int device, int* lds_bytes, std::string* err) {
  const std::vector<int64_t> skey = shape_key(s, device);
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    auto it = g_jit_shapes.find(skey);
    if (it != g_jit_shapes.end()) {
      if (lds_bytes) *lds_bytes = it->second.lds;
      return it->second.fn;
    }
  }
  int lds = 0;
  const std::string src = jit_source(s, &lds);
  if (lds_bytes) *lds_bytes = lds;
  std::lock_guard<std::mutex> g(g_jit_mu);
  auto key = std::make_pair(device, src);
  auto it = g_jit_cache.find(key);
  if (it != g_jit_cache.end()) {
    g_jit_shapes.emplace(skey, it->second);
    return it->second.fn;
  }
  if (const char* dump = std::getenv("PGX_JIT_DUMP")) {  // debugging: keep every generated kernel's source
    const std::string path = std::string(dump) + "/pgxq_" + std::to_string(g_jit_cache.size()) + ".hip";
    if (FILE* f = std::fopen(path.c_str(), "w")) {
      std::fputs(src.c_str(), f);
      std::fclose(f);
    }
  }
  std::string code;
  if (!cache_load(src, &code)) {
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "pgx_query.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
      if (err) *err = "hiprtcCreateProgram failed";
      return nullptr;
    }
    const hiprtcResult rc = hiprtcCompileProgram(prog, 3, const_cast<const char**>(pgx::kJitOpts));
    if (rc != HIPRTC_SUCCESS) {
      size_t n = 0;
      hiprtcGetProgramLogSize(prog, &n);
      std::string log(n, '\0');
      if (n) hiprtcGetProgramLog(prog, &log[0]);
      hiprtcDestroyProgram(&prog);
      if (err) *err = "hiprtc compile failed: " + log.substr(0, 4000);
      return nullptr;
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(prog, &code_size);
    code.assign(code_size, '\0');
    hiprtcGetCode(prog, &code[0]);
    hiprtcDestroyProgram(&prog);
    cache_store(src, code);
  }
  JitEntry ent;
  ent.lds = lds;
  if (hipModuleLoadData(&ent.mod, code.data()) != hipSuccess ||
      hipModuleGetFunction(&ent.fn, ent.mod, "pgxq") != hipSuccess) {
    if (err) *err = "hipModuleLoadData / hipModuleGetFunction failed";
    return nullptr;
  }
  g_jit_cache.emplace(key, ent);
  g_jit_shapes.emplace(skey, ent);
  return ent.fn;
}

}  // namespace pgx

// Debug / build-check entry: compile the kernel source of a shape without a device (declared in include/pgx.h).
extern "C" int pgx_jit_compile_check(const char* source, char* log, unsigned long log_cap) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, source, "pgx_query.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) return -1;
  const hiprtcResult rc = hiprtcCompileProgram(prog, 3, const_cast<const char**>(pgx::kJitOpts));
  size_t n = 0;
  hiprtcGetProgramLogSize(prog, &n);
  if (log && log_cap) {
    std::string l(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &l[0]);
    std::snprintf(log, log_cap, "%s", l.c_str());
  }
  // debugging: with PGX_JIT_DUMP=<dir>, <dir>/last_check.co keeps the code object of the last compile (llvm-objdump)
  if (rc == HIPRTC_SUCCESS)
    if (const char* dir = std::getenv("PGX_JIT_DUMP")) {
      size_t cs = 0;
      hiprtcGetCodeSize(prog, &cs);
      std::string code(cs, '\0');
      hiprtcGetCode(prog, &code[0]);
      if (FILE* f = std::fopen((std::string(dir) + "/last_check.co").c_str(), "wb")) {
        std::fwrite(code.data(), 1, cs, f);
        std::fclose(f);
      }
    }
  hiprtcDestroyProgram(&prog);
  return rc == HIPRTC_SUCCESS ? 0 : 1;
}

// Build check without a device: generate and compile a representative set of query shapes (every bit width, every
// leaf kind, AND/OR/STAT programs, every aggregation, dense LDS / global group-by, every value-image kind).
// Returns the number of shapes that failed; *n_total receives the number tried.  Declared in include/pgx.h.
extern "C" int pgx_jit_selftest(int* n_total, char* log, unsigned long log_cap) {
  using namespace pgx;
  std::vector<JitShape> shapes;
  auto base = [](int bits_f, int bits_m, int img, int sh) {
    JitShape s;
    s.cols.resize(2);
    s.cols[0].bits = bits_f;
    s.cols[0].decode = true;
    s.cols[1].bits = bits_m;
    s.cols[1].decode = true;
    s.cols[1].img = img;
    s.cols[1].img_sh = sh;
    s.cols[1].img_words = img == IMG_FOR16 ? kImgFor16Blocks + (1 << 15) : (img == IMG_NONE ? 0 : 1024);
    s.cols[1].acc32 = true;
    int R = 8;
    for (int b : {bits_f, bits_m}) {
      int g = 1;
      while (g < 32 && b % (g * 2) == 0) g *= 2;
      R = std::max(R, 32 / g);
    }
    s.R = R;
    s.T = img == IMG_FOR16 ? 1024 : 256;
    s.leaf_col = {0};
    s.leaf_mode = {LEAF_SCAN_INTERVAL};
    s.prog_op = {OP_LEAF};
    s.prog_arg = {0};
    s.agg_kind = {A_COUNT, A_SUM, A_MIN, A_MAX, A_AVG};
    s.agg_col = {-1, 1, 1, 1, 1};
    s.plane_op = {P_ADD_I64, P_ADD_I64, P_ADD_I64, P_MIN_ORD, P_MAX_ORD, P_ADD_I64};
    s.num_planes = 6;
    return s;
  };
  for (int b = 1; b <= 32; b += 3) shapes.push_back(base(b, 33 - b, IMG_U32, 0));
  shapes.push_back(base(8, 16, IMG_FOR16, 11));
  {  // the C2 benchmark shape: COUNT(*), SUM(m) WHERE dA BETWEEN lo AND hi
    JitShape s = base(8, 16, IMG_FOR16, 11);
    s.agg_kind = {A_COUNT, A_SUM};
    s.agg_col = {-1, 1};
    s.plane_op = {P_ADD_I64, P_ADD_I64, P_ADD_I64};
    s.num_planes = 3;
    shapes.push_back(s);
  }
  {  // the C5 benchmark shape: SUM(m) over the bitmap program's doc mask GROUP BY gk (card 1000, dense LDS table)
    JitShape s = base(10, 16, IMG_FOR16, 11);
    s.cols.resize(5);
    s.cols[4] = s.cols[0];                 // gk, 10 bits
    s.cols[3] = s.cols[1];                 // m, 16 bits, FOR16 image
    s.cols[0] = s.cols[1] = s.cols[2] = JitCol{};
    s.cols[0].bits = 10;                   // f1, f2, f3: bitmap leaves, not decoded
    s.cols[1].bits = 7;
    s.cols[2].bits = 4;
    s.leaf_col = {0, 1, 2, -1};
    s.leaf_mode = {LEAF_NONE, LEAF_NONE, LEAF_NONE, LEAF_DOCMASK};
    s.prog_op = {OP_LEAF, OP_STAT};
    s.prog_arg = {3, 0};
    s.agg_kind = {A_SUM};
    s.agg_col = {3};
    s.plane_op = {P_ADD_I64, P_ADD_I64};
    s.num_planes = 2;
    s.group_mode = G_DENSE_LDS;
    s.gcol = {4};
    s.gmul = {1};
    s.dense_slots = 1000;
    s.R = 16;
    s.T = 1024;
    shapes.push_back(s);
    s.R = 8;  // m's words contiguous per load; gk's 80 bits start mid-dword (frac)
    s.cols[4].frac = true;
    shapes.push_back(s);
    s.R = 16;  // count and sum in one 64-bit LDS add, flushed per segment
    s.cols[4].frac = false;
    s.dense_pack = 40;
    shapes.push_back(s);
  }
  shapes.push_back(base(8, 16, IMG_NONE, 0));
  {
    JitShape s = base(10, 16, IMG_F64, 0);
    s.cols[1].fp = true;
    s.plane_op = {P_ADD_I64, P_ADD_I64, P_ADD_F64, P_MIN_ORD, P_MAX_ORD, P_ADD_F64};
    s.leaf_mode = {LEAF_SCAN_BITSET};
    shapes.push_back(s);
  }
  {
    JitShape s = base(7, 12, IMG_U32, 0);
    s.cols.push_back(JitCol{});
    s.cols[2].bits = 4;
    s.cols[2].decode = false;
    s.leaf_col = {0, 2, 0};
    s.leaf_mode = {LEAF_SCAN_INTERVAL, LEAF_RANGES, LEAF_NONE};
    s.prog_op = {OP_LEAF, OP_STAT, OP_LEAF, OP_AND, OP_LEAF, OP_OR};
    s.prog_arg = {1, 0, 0, 2, 2, 2};
    s.cols[1].acc32 = false;
    shapes.push_back(s);
  }
  {  // bitmap inverted-index leaves (doc masks), one of them negated, OR / AND with a scan leaf
    JitShape s = base(10, 16, IMG_FOR16, 11);
    s.cols[0].decode = true;
    s.leaf_col = {0, 0, 0};
    s.leaf_mode = {LEAF_DOCMASK, LEAF_DOCMASK_NOT, LEAF_SCAN_INTERVAL};
    s.prog_op = {OP_LEAF, OP_LEAF, OP_OR, OP_LEAF, OP_AND};
    s.prog_arg = {0, 1, 2, 2, 2};
    s.R = 16;
    shapes.push_back(s);
  }
  {  // C5 shape: (L0 OR L1) AND NOT L2 over bitmap leaves evaluated per chunk in LDS, dense LDS group-by, no image
    JitShape s = base(10, 16, IMG_NONE, 0);
    s.cols.push_back(JitCol{});
    s.cols[2].bits = 10;
    s.cols[2].decode = false;
    s.leaf_col = {2, 2, 2, -1};
    s.leaf_mode = {LEAF_NONE, LEAF_NONE, LEAF_NONE, LEAF_RCHUNK};
    s.prog_op = {OP_LEAF, OP_STAT};
    s.prog_arg = {3, 0};
    s.rprog_ops = {{RP_LEAF, RP_LEAF, RP_OR, RP_LEAF, RP_NOT, RP_AND}};
    s.R = 16;
    s.T = 512;
    s.group_mode = G_DENSE_LDS;
    s.gcol = {0};
    s.gmul = {1};
    s.dense_slots = 1000;
    s.agg_kind = {A_SUM};
    s.agg_col = {1};
    s.plane_op = {P_ADD_I64, P_ADD_I64};
    s.num_planes = 2;
    shapes.push_back(s);
    s.compact = true;  // selected rows packed into consecutive lanes before the gathers and atomics
    shapes.push_back(s);
    s.group_mode = G_NONE;  // aggregation-only, compacted, every function
    s.gcol.clear();
    s.gmul.clear();
    s.agg_kind = {A_COUNT, A_SUM, A_MIN, A_MAX, A_AVG};
    s.agg_col = {-1, 1, 1, 1, 1};
    s.plane_op = {P_ADD_I64, P_ADD_I64, P_ADD_I64, P_MIN_ORD, P_MAX_ORD, P_ADD_I64};
    s.num_planes = 6;
    shapes.push_back(s);
    s.cols[1].img = IMG_U32;  // ... with a value image
    s.cols[1].img_words = 1024;
    shapes.push_back(s);
    s.compact = false;  // selection bits written for the multi-value aggregation pass
    s.selmask = true;
    shapes.push_back(s);
  }
  {  // the C5 bench shape: the bitmap program's doc mask as one leaf, dense LDS group-by of gk, packed COUNT + SUM(m)
     // through the FOR16 image
    JitShape s = base(10, 16, IMG_FOR16, 11);
    s.cols[1].img_words = 64 + 32768;
    s.cols.push_back(JitCol{});
    s.cols[2].bits = 10;
    s.cols[2].decode = false;
    s.leaf_col = {2, 2, 2, -1};
    s.leaf_mode = {LEAF_NONE, LEAF_NONE, LEAF_NONE, LEAF_DOCMASK};
    s.prog_op = {OP_LEAF, OP_STAT};
    s.prog_arg = {3, 0};
    s.R = 16;
    s.T = 1024;
    s.group_mode = G_DENSE_LDS;
    s.gcol = {0};
    s.gmul = {1};
    s.dense_slots = 1000;
    s.agg_kind = {A_SUM};
    s.agg_col = {1};
    s.plane_op = {P_ADD_I64, P_ADD_I64};
    s.num_planes = 2;
    s.dense_pack = 40;
    shapes.push_back(s);
  }
  for (int R : {8, 16, 32}) {  // statistics automaton input: every leaf's predicate bits written per lane
    JitShape s = base(R == 8 ? 8 : (R == 16 ? 10 : 7), 16, IMG_FOR16, 11);
    s.cols.push_back(JitCol{});
    s.cols[2].bits = 4;
    s.leaf_col = {0, 2, 0};
    s.leaf_mode = {LEAF_SCAN_INTERVAL, LEAF_RANGES, LEAF_DOCMASK_NOT};
    s.prog_op = {OP_LEAF, OP_LEAF, OP_LEAF, OP_OR, OP_AND};
    s.prog_arg = {0, 1, 2, 2, 2};
    s.R = R;
    s.leafmask = true;
    shapes.push_back(s);
  }
  {  // partitioned group-by records (C3 shape: g1 14 bits, g2 20 bits, value offsets of m)
    JitShape s = base(14, 16, IMG_FOR16, 11);
    s.cols.push_back(JitCol{});
    s.cols[2].bits = 20;
    s.cols[2].decode = true;
    s.leaf_col.clear();
    s.leaf_mode.clear();
    s.prog_op.clear();
    s.prog_arg.clear();
    s.R = 16;
    s.T = 512;
    s.group_mode = G_EMIT;
    s.gcol = {0, 2};
    s.gshift = {0, 14};
    s.keybits = 34;
    s.emit_col = 1;
    s.agg_kind = {A_SUM, A_MIN, A_MAX};
    s.agg_col = {1, 1, 1};
    s.plane_op = {P_ADD_I64, P_ADD_I64, P_MIN_ORD, P_MAX_ORD};
    s.num_planes = 4;
    shapes.push_back(s);
    s.cols[1].img = IMG_NONE;  // value image demoted (LDS budget): values from the HBM dictionary
    s.cols[2].remap = true;
    shapes.push_back(s);
    s.emit_dictid = true;       // narrow records: 26 bits of the key's mix + a 16-bit dictId (u32 + u16 arrays)
    s.cols[2].remap = false;
    s.part_slab = true;
    s.part_bits = kNarrow1Bits;
    s.part_narrow = true;
    s.narrow_vbits = 16;
    shapes.push_back(s);
    {  // eight rows per lane (fractional loads of the 14-bit column), 1024 threads: the same records per sub-step
      JitShape t = s;
      t.R = 8;
      t.T = 1024;
      for (JitCol& C : t.cols) C.frac = C.decode && (8 * C.bits) % 32 != 0;
      shapes.push_back(t);
      t.TL = 16;  // half tiles: half the raw words in flight per lane
      shapes.push_back(t);
      t.T = 512;
      shapes.push_back(t);
    }
    s.emit_col = -1;            // COUNT only: 26-bit records, one u32 array
    s.narrow_vbits = 0;
    shapes.push_back(s);
  }
  {  // twelve columns (the C6 "wide" shape): ten filter leaves ANDed, a 10-bit dense group column, SUM of a 16-bit one
    JitShape s = base(8, 16, IMG_U32, 0);
    for (int c = 2; c < 12; ++c) {
      JitCol C;
      C.bits = c == 11 ? 10 : 8 + 2 * (c % 3);
      C.decode = true;
      s.cols.push_back(C);
    }
    s.leaf_col.clear();
    s.leaf_mode.clear();
    s.prog_op.clear();
    s.prog_arg.clear();
    for (int l = 0; l < 10; ++l) {
      s.leaf_col.push_back(l == 0 ? 0 : l + 1);
      s.leaf_mode.push_back(LEAF_SCAN_INTERVAL);
      s.prog_op.push_back(OP_LEAF);
      s.prog_arg.push_back(l);
      if (l) {
        s.prog_op.push_back(OP_AND);
        s.prog_arg.push_back(0);
      }
    }
    s.R = 16;
    s.group_mode = G_DENSE_LDS;
    s.gcol = {11};
    s.gmul = {1};
    s.dense_slots = 1024;
    s.agg_kind = {A_SUM};
    s.agg_col = {1};
    s.plane_op = {P_ADD_I64, P_ADD_I64};
    s.num_planes = 2;
    shapes.push_back(s);
  }
  for (int gm : {G_HASH64, G_HASH128}) {  // hash group-by: LDS table + global overflow, remapped group ids
    JitShape s = base(8, 16, IMG_U32, 0);
    for (int c = 2; c < 5; ++c) {
      JitCol C;
      C.bits = 14;
      C.decode = true;
      C.remap = c == 3;
      s.cols.push_back(C);
    }
    s.R = 16;
    s.group_mode = gm;
    s.gcol = {2, 3, 4, 0};
    s.gmul = {1, 1, 1, 1};
    s.gshift = gm == G_HASH128 ? std::vector<int>{0, 14, 28, 0} : std::vector<int>{0, 14, 28, 42};
    s.ghi = gm == G_HASH128 ? std::vector<int>{0, 0, 0, 1} : std::vector<int>{0, 0, 0, 0};
    s.hash_slots = 1024;
    s.agg_kind = {A_SUM, A_MIN, A_MAX, A_COUNT};
    s.agg_col = {1, 1, 1, -1};
    s.plane_op = {P_ADD_I64, P_ADD_I64, P_MIN_ORD, P_MAX_ORD, P_ADD_I64};
    s.num_planes = 5;
    shapes.push_back(s);
    s.agg_kind = {A_SUM};  // packed count + value offset in one LDS add, flushed per segment
    s.agg_col = {1};
    s.plane_op = {P_ADD_I64, P_ADD_I64};
    s.num_planes = 2;
    s.dense_pack = 40;
    shapes.push_back(s);
  }
  for (int gm : {G_DENSE_LDS, G_DENSE_GLOBAL}) {
    JitShape s = base(8, 16, IMG_U32, 0);
    s.cols.push_back(JitCol{});
    s.cols[2].bits = 10;
    s.cols[2].decode = true;
    s.cols[2].remap = gm == G_DENSE_GLOBAL;
    s.R = 16;
    s.group_mode = gm;
    s.gcol = {2, 0};
    s.gmul = {1, 1000};
    s.dense_slots = gm == G_DENSE_LDS ? 1000 : 256000;
    s.agg_kind = {A_SUM, A_MIN, A_MAX, A_COUNT};
    s.agg_col = {1, 1, 1, -1};
    s.plane_op = {P_ADD_I64, P_ADD_I64, P_MIN_ORD, P_MAX_ORD, P_ADD_I64};
    s.num_planes = 5;
    shapes.push_back(s);
  }
  {
    JitShape s = base(8, 16, IMG_U32, 0);
    s.prog_op.clear();
    s.prog_arg.clear();
    s.leaf_col.clear();
    s.leaf_mode.clear();
    s.agg_kind = {A_COUNT};
    s.agg_col = {-1};
    s.plane_op = {P_ADD_I64, P_ADD_I64};
    s.num_planes = 2;
    s.cols[1].decode = false;
    s.cols[1].img = IMG_NONE;
    shapes.push_back(s);
  }
  int failed = 0;
  std::string all;
  for (size_t i = 0; i < shapes.size(); ++i) {
    const std::string src = jit_source(shapes[i], nullptr);
    if (const char* dump = std::getenv("PGX_JIT_DUMP")) {
      const std::string path = std::string(dump) + "/selftest_" + std::to_string(i) + ".hip";
      if (FILE* f = std::fopen(path.c_str(), "w")) {
        std::fputs(src.c_str(), f);
        std::fclose(f);
      }
    }
    char buf[4096];
    if (pgx_jit_compile_check(src.c_str(), buf, sizeof(buf)) != 0) {
      ++failed;
      all += "shape " + std::to_string(i) + ": " + buf + "\n";
    }
  }
  if (n_total) *n_total = int(shapes.size());
  if (log && log_cap) std::snprintf(log, log_cap, "%s", all.c_str());
  return failed;
}

