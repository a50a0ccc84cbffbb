// Internal host/device structures of libpgx (not part of the ABI).
#pragma once
#include <stdint.h>

#include "pgx_jit_abi.h"

namespace pgx {

constexpr int kTileRows = 8192;        // rows per workgroup tile = 256 lanes x 32 rows
constexpr int kLaneRows = 32;          // rows owned by one lane: exactly one 32-bit mask word
constexpr int kBlock = 256;            // threads per workgroup
constexpr int kMaxQCols = 16;          // distinct columns a query touches
constexpr int kMaxLeaves = 16;
constexpr int kMaxAggs = 8;
constexpr int kMaxGroupCols = 16;
constexpr int kMaxProg = 64;
constexpr int kStackDepth = 8;
constexpr uint64_t kEmptyKey = ~0ull;

enum LeafMode : int8_t {
  LEAF_SCAN_INTERVAL = 0,  // decode + lo <= id <= hi
  LEAF_SCAN_BITSET = 1,    // decode + bitset lookup
  LEAF_RANGES = 2,         // sorted doc ranges
  LEAF_NONE = 3,           // always false (empty binding)
  LEAF_DOCMASK = 4,        // query kernels: bitmap inverted-index leaf expanded to a per-segment doc mask
  LEAF_DOCMASK_NOT = 5,    // ... NEQ / NOT_IN: OR of the non-matching bitmaps, flipped (BitmapBasedFilterOperator)
  LEAF_RCHUNK = 6,         // query kernels: a bitmap program evaluated per 65536-doc chunk into LDS by the kernel
};

// Bitmap inverted-index expansion (pgx_kernels.hip pgx_roaring_expand): one descriptor per (segment, leaf).  The
// layout is shared with the generated query kernels (pgx_jit_abi.h JRDesc), which evaluate bitmap programs per chunk
// themselves (LEAF_RCHUNK).
//   mask: nchunks x 2048 words: bit (doc & 31) of word (doc >> 5); inv: device copy of <col>.bitmap.inv;
//   offs: byte offsets (into inv) of the roaring bitmaps to OR; nb: their number; nchunks: ceil(total_docs / 65536)
using RDesc = ::JRDesc;

// A sub-tree of the filter whose leaves are all bitmap inverted-index leaves, evaluated per 65536-doc chunk into ONE
// doc mask: by pgx_roaring_program into HBM, or inside the query kernel into LDS (LEAF_RCHUNK).  pgx_jit_abi.h JRProg.
constexpr int kMaxRProg = PGX_J_MAX_RPROG;
enum RProgOp : int8_t { RP_LEAF = 0, RP_AND = 1, RP_OR = 2, RP_NOT = 3 };
using RProg = ::JRProg;

enum ProgOp : int8_t { OP_LEAF = 0, OP_AND = 1, OP_OR = 2, OP_STAT = 3, OP_TRUE = 4 };

// Multi-value columns (pgx_kernels.hip).  Values are the .mv.fwd raw section (value i at bits [i*B, i*B+B), MSB-first
// big-endian, like a single-value forward index over value positions); doc d owns values [start[d], start[d+1]).
// MV scan leaf (MVScanDocIdIterator + the evaluators' apply(int[]), operator/filter/predicate/*PredicateEvaluator
// .java): a doc matches when ANY value is in the matching set (EQ / IN / RANGE), or, for NEQ / NOT_IN, when NO value is
// outside it; one output bit per doc.
struct MvLeaf {
  const uint32_t* vals;
  const int32_t* start;        // num_docs + 1
  const uint32_t* bitset;      // matching dictIds (null: lo <= id <= lo + span)
  uint32_t* mask;              // out: bit (d & 31) of word d >> 5
  int32_t bits;
  int32_t num_docs;
  uint32_t lo, span;
  int32_t neg;
  int32_t pad;
};
// MV aggregation (Count/Sum/Min/Max/AvgMVAggregationFunction): every value of every selected doc of one segment.
struct MvAgg {
  const uint32_t* vals;
  const int32_t* start;
  const uint32_t* sel;         // selected docs: bit (d & 31) of word d >> 5 (written by the query kernel)
  const void* dict;            // int64 or double per dictId
  unsigned long long* out;     // [count, sum (int64 or f64 bits), ordered min, ordered max]
  int32_t bits;
  int32_t num_docs;
  int32_t fp;
  int32_t pad;
};

// Group-by with multi-value group columns and/or multi-value functions (DefaultGroupKeyGenerator.java:475-608
// generateKeysForDocId*, DefaultGroupByExecutor.java:154-196 aggregateGroupByMV): per selected doc, one group key per
// combination of its group columns' values; every key receives the doc's contribution of every function.
struct MvGCol {                // one group-by or aggregated column of one segment
  const uint32_t* vals;        // single-value forward index, or the multi-value values section
  const int32_t* start;        // multi-value: doc starts (num_docs + 1); null for single-value
  const int32_t* remap;        // group column: segment dictId -> global id (null: identity)
  const void* dict;            // aggregated column: int64 / double per dictId
  int32_t bits;
  int32_t pad;
};
struct MvGroupSeg {
  const uint32_t* sel;         // selected docs (query kernel selection bits, bit d & 31 of word d >> 5)
  int32_t num_docs;
  int32_t pad;
  MvGCol g[kMaxGroupCols];
  MvGCol a[kMaxAggs];
};
enum MvFnKind : int8_t { MVF_COUNT = 0, MVF_SUM = 1, MVF_MIN = 2, MVF_MAX = 3, MVF_AVG = 4, MVF_COUNTMV = 5,
                         MVF_SUMMV = 6, MVF_MINMV = 7, MVF_MAXMV = 8, MVF_AVGMV = 9 };
struct MvGroupArgs {
  const MvGroupSeg* segs;
  int32_t nsegs;
  int32_t ngcols, naggs;
  int32_t group_mode;          // G_DENSE_GLOBAL, G_HASH64 or G_HASH128
  int8_t fn[kMaxAggs];         // MvFnKind
  int8_t fp[kMaxAggs];         // FLOAT / DOUBLE values
  int8_t cnt_plane[kMaxAggs];  // AVGMV: the plane of its value count (else -1)
  uint64_t gmul[kMaxGroupCols];
  int32_t gshift[kMaxGroupCols];
  int32_t ghi[kMaxGroupCols];
  uint64_t slots;              // dense slots or hash capacity (power of two)
  unsigned long long* table;   // planes x slots
  unsigned long long* keys;    // hash keys (64-bit, or lo / hi pairs)
  unsigned int* key_state;     // hash128 slot states
  unsigned long long* overflow;
  unsigned long long* ord;     // MINMV / MAXMV per-segment holders: [seg][agg][slot] (ordered encodings)
};

// Statistics automaton over one segment's leaf masks (pgx_kernels.hip pgx_fsm_chunks / pgx_fsm_compose).
struct FsmSeg {
  const uint32_t* lmask;       // leaf l, row r: bit (r & 31) of word [l * words + (r >> 5)]
  int64_t words;               // words per leaf
  int32_t num_docs;
  int32_t nint;                // intervals of constant range position
  int64_t chunk0;              // first chunk of this segment in the launch
  int32_t ibeg[3 * 10 + 2];    // interval first rows (ascending, ibeg[0] = 0)
  int32_t itab[3 * 10 + 2];    // interval transition table
};

enum AggKind : int8_t { A_COUNT = 0, A_SUM = 1, A_MIN = 2, A_MAX = 3, A_AVG = 4 };

// Accumulator plane ops (pgx.h pgx_query_dense_plane_op)
enum PlaneOp : int8_t { P_ADD_I64 = 0, P_ADD_F64 = 1, P_MIN_ORD = 2, P_MAX_ORD = 3 };

enum GroupMode : int8_t { G_NONE = 0, G_DENSE_LDS = 1, G_DENSE_GLOBAL = 2, G_HASH64 = 3, G_HASH128 = 4,
                          G_EMIT = 5 /* query kernels: emit key|value records for the partitioned group-by */,
                          G_HASHW = 6 /* keys of 3-4 64-bit words (ARRAY_MAP keys over 126 bits): generic kernel */ };
constexpr int kMaxKeyWords = 4;
inline bool hash_mode(int gm) { return gm == G_HASH64 || gm == G_HASH128 || gm == G_HASHW; }

struct KLeaf {
  int32_t lo, hi;
  const uint32_t* bitset;      // device, ceil(card/32) words (LEAF_SCAN_BITSET)
  const int32_t* ranges;       // device, 2*nranges inclusive [a,b] pairs, sorted (LEAF_RANGES)
  int32_t nranges;
  int8_t mode;
  int8_t pad[3];
};

struct KSeg {
  int64_t tile_begin;          // global tile index of this segment's first tile
  int32_t num_docs;            // rows scanned: [0, num_docs)
  int32_t num_tiles;
  const uint32_t* fwd[kMaxQCols];     // packed big-endian fixed-bit forward index (padded)
  const void* dict[kMaxQCols];        // value columns: int64 (INT/LONG) or double (FLOAT/DOUBLE) per dictId
  const int32_t* remap[kMaxQCols];    // group columns: dictId -> global id (nullptr = identity)
  int8_t bits[kMaxQCols];
  KLeaf leaf[kMaxLeaves];
  uint32_t* lmask;                    // statistics automaton input: leaf l, row r -> bit (r & 31) of
  int64_t lmask_words;                // word [l * lmask_words + (r >> 5)] (nullptr: not requested)
};

struct KQuery {
  const KSeg* segs;
  int32_t num_segs;
  int32_t num_qcols;
  int64_t total_tiles;
  // filter program (postfix, stack machine)
  int32_t prog_len;
  int8_t prog_op[kMaxProg];
  int8_t prog_arg[kMaxProg];
  int8_t leaf_col[kMaxLeaves];
  // value columns decoded for aggregation (distinct), and aggs
  int32_t num_aggs;
  int8_t agg_kind[kMaxAggs];
  int8_t agg_col[kMaxAggs];      // query-column slot (-1 for COUNT)
  int8_t agg_fp[kMaxAggs];       // value column is FLOAT/DOUBLE
  int8_t plane_op[kMaxAggs + 1]; // plane 0 = count
  int32_t num_planes;            // 1 + num_aggs
  // group-by
  int8_t group_mode;
  int32_t num_gcols;
  int8_t gcol[kMaxGroupCols];
  uint64_t gmul[kMaxGroupCols];  // dense: mixed-radix multiplier; hash: bit shift
  int32_t gshift[kMaxGroupCols];
  int32_t ghi[kMaxGroupCols];    // 128-bit / wide keys: the 64-bit word the field goes to (0 = low)
  int32_t key_words;             // hash keys: 64-bit words per key (1, 2, or up to kMaxKeyWords for G_HASHW)
  uint64_t dense_slots;          // dense key space
  uint64_t hash_cap;             // power of two
  // outputs
  unsigned long long* agg_out;   // aggregation-only: num_planes accumulators (plane encodings)
  unsigned long long* stats;     // [0] docs matched, [1] entries scanned in filter (kernel part)
  unsigned long long* table;     // dense: planes x dense_slots ; hash: planes x hash_cap
  unsigned long long* keys;      // hash: key_words * hash_cap (word w of slot s at keys[s * key_words + w])
  unsigned int* key_state;       // hash128 / wide: 0 empty, 1 busy, 2 ready
  unsigned long long* overflow;  // hash insert failures (table full) -> host retries bigger
};

}  // namespace pgx

// =================================================================================================
// Query-specialised kernels (pgx_jit.cpp): the shape of one launch group, from which a kernel is generated and
// compiled by hiprtc once per distinct shape (cached per process and device).
// =================================================================================================
#include <string>
#include <vector>

namespace pgx {

// Value images staged in LDS for aggregated columns (built once per column at staging time, pgx_stage.cpp).
enum ImgKind : int8_t {
  IMG_NONE = 0,   // no image: values are gathered from the HBM value table (int64 / double per dictId)
  IMG_U32 = 1,    // u32 (value - vbase) per dictId
  IMG_FOR16 = 2,  // 64 x u32 block bases (relative to vbase) then u16 offset per dictId; block = 1 << sh dictIds
  IMG_F64 = 3,    // double per dictId
};
constexpr int kImgFor16Blocks = 64;
constexpr int kLdsBudget = 160 * 1024 - 256;  // static LDS of one workgroup, minus the per-plane accumulators

// Narrow partitioned group-by (pgx_part.cpp run_narrow): the packed K-bit group key is mixed by a bijection of
// [0, 2^K), h = ((key * c1) & M) ^ (that >> s) with s = ceil(K / 2) (so the xor-shift inverts itself), and the
// partitions are h's top bits (the multiply carries every key bit into them); the xor-shift folds those well-mixed top
// bits into the low bits that choose a record's slot in the aggregation tables.  h's remaining bits travel in the
// records and the aggregation rebuilds the key with the inverse.  c1 has 32 bits: the scan's multiply of a key of up
// to 64 bits is three 32-bit multiplies (round 4 used two full 64-bit multiplies, eight, for the same partitions).
// Shared by the generated scan (pgx_jit.cpp), the split / aggregation kernels and the host.
constexpr uint64_t kNarrowC1 = 0x9E3779B1ull;
constexpr int kNarrow1Bits = 8;      // first split (inside the scan): 256 buckets
constexpr int kNarrowRing = 64;      // scan: per-bucket LDS ring of records (two 32-record units; the largest ring)
constexpr int kNarrowMaxBits2 = 10;  // second split (pgx_narrow_split): up to 1024 sub-buckets per bucket
// Environment knobs (A/B switches and test hooks), read ONCE per query by pgx_query_compile and kept with the query:
// planning and execution read them from there, never from the environment (no per-query walk of environ, no race
// with a setenv on another thread).  The whole set:
//   PGX_JIT=0          the generic interpreter kernel instead of the generated (hiprtc) kernels, everywhere (A/B)
//   PGX_PART_NARROW=0  sparse group-by through the 8-byte radix path instead of the narrow records; =direct: narrow
//                      records carry value offsets wherever they fit (default: dictIds + LDS image when there is one);
//                      =gather: integer records carry the dictId's index in a global value table (IMG 5, tests)
//   PGX_RCHUNK=0|1     bitmap programs evaluated by the separate pass / inside the query kernels (default: planner)
//   PGX_RPROG=off|wave|seg|chunk|stack   bitmap-program kernel (off: no program fusion; default: planner)
//   PGX_BATCH_SEGS=N   segments per batch of a long segment list on its first execution (0: one launch)
//   PGX_DEBUG=opt,...  part_small (radix buckets start undersized), narrow_k2=N (coarser narrow partitions),
//                      narrow_log (which sparse path ran, hash-table regrowth; on stderr), host_profile (planning phases
//                      on stderr); A/B switches measured slower and kept off: nunit=16 (16-record narrow
//                      scan units), pf2 (narrow scans load two tiles ahead), noimg (no LDS value images in the query
//                      kernels), head=N (a lone replay's first part is 1/N of the segments)
// and, outside the query: PGX_PLAN_CACHE=0 (process-wide), PGX_JIT_CACHE=<dir> / PGX_JIT_DUMP=<dir> (the compiler).
enum RProgKind { RPROG_AUTO = -1, RPROG_OFF = 0, RPROG_WAVE = 1, RPROG_SEG = 2, RPROG_CHUNK = 3, RPROG_STACK = 4 };
struct Knobs {
  bool jit = true;
  bool narrow = true;
  bool narrow_direct = false;  // PGX_PART_NARROW=direct
  bool narrow_gather = false;  // PGX_PART_NARROW=gather (tests): value-table records (IMG 5) where they fit
  int rchunk = -1;          // -1: planner's choice
  int rprog = RPROG_AUTO;
  int batch_segs = -1;      // -1: default (512; 0 with PGX_X_THROUGHPUT)
  bool no_img = false;      // PGX_DEBUG noimg: query kernels gather values from the dictionaries, no LDS images (A/B)
  bool prefetch2 = false;   // PGX_DEBUG pf2: narrow scans load two tiles ahead (A/B)
  int narrow_unit = 32;     // PGX_DEBUG nunit=16: 16-record units (32-record rings: two scan workgroups per CU)
  int lone_head = 2;        // PGX_DEBUG head=N: a lone replay's first part is 1/N of the segments (A/B)
  bool part_small = false;  // PGX_DEBUG part_small
  int narrow_k2 = -1;       // PGX_DEBUG narrow_k2=N
  bool narrow_log = false;  // PGX_DEBUG narrow_log
  bool host_profile = false;
};
Knobs read_knobs();

struct NarrowMix {
  uint64_t mask = 0, c1 = kNarrowC1, ic1 = 0;
  int s = 0;
};
inline uint64_t narrow_inverse(uint64_t c) {  // c odd: c * inverse == 1 (mod 2^64), Newton iteration
  uint64_t x = c;
  for (int i = 0; i < 6; ++i) x *= 2 - c * x;
  return x;
}
inline NarrowMix narrow_mix(int keybits) {
  NarrowMix m;
  m.mask = keybits >= 64 ? ~0ull : (uint64_t(1) << keybits) - 1u;
  m.s = (keybits + 1) / 2;
  m.ic1 = narrow_inverse(m.c1);
  return m;
}

struct JitCol {
  int bits = 0;
  bool decode = false;   // read by a scan leaf, an aggregation or a group key
  int img = IMG_NONE;    // value image kind (aggregated columns)
  int img_sh = 0;        // IMG_FOR16 block shift
  int img_words = 0;     // LDS dwords reserved for the image (max over the group's segments)
  bool acc32 = false;    // R rows of (value - vbase) always fit a u32 partial sum
  bool fp = false;       // FLOAT/DOUBLE values
  bool remap = false;    // group column with a local->global dictId remap table
  bool frac = false;     // R * bits is not a multiple of 32: a lane's rows start mid-dword (dword-aligned load of
                         // the covering words, then a funnel shift by (first row * bits) % 32)
};

struct JitShape {
  int T = 256;           // threads per workgroup
  int R = 8;             // rows per lane per sub-step (R * bits % 32 == 0 for every decoded column without frac)
  int TL = 32;           // rows per lane per tile (a multiple of R): the rows whose raw words are loaded one tile ahead
  std::vector<JitCol> cols;
  std::vector<int> leaf_col, leaf_mode;   // leaf_col -1: doc-range leaf with no column (star-tree node ranges)
  std::vector<int> prog_op, prog_arg;
  std::vector<int> agg_kind, agg_col, plane_op;
  int group_mode = G_NONE;
  std::vector<int> gcol;
  std::vector<uint64_t> gmul;
  uint64_t dense_slots = 0;
  int num_planes = 1;
  // G_EMIT: record = key (group ids at gshift) | value offset << keybits; emit_col = value column (-1: none)
  std::vector<int> gshift;
  int keybits = 0;
  int emit_col = -1;
  // G_HASH64 / G_HASH128: group ids at gshift of the low (ghi 0) or high (ghi 1) key word; hash_slots LDS slots
  std::vector<int> ghi;
  int hash_slots = 0;
  bool leafmask = false;  // write every leaf's per-row predicate bit (statistics automaton input, pgx_stats.cpp)
  // LEAF_RCHUNK leaves, in leaf order: the bitmap program's postfix ops (RP_*), identical for the group's segments
  std::vector<std::vector<int>> rprog_ops;
  // G_EMIT: records split 2^part_bits ways inside the kernel (first radix pass fused; 0 = row-order records), and the
  // record's value field is the value column's dictId (sorted dictionary) instead of its offset from vbase
  int part_bits = 0;
  bool emit_dictid = false;
  // with part_bits: each workgroup appends to its own region ("slab") per bucket through LDS cursors, no staging and no
  // global cursor per sub-step (slab (b, w) at table + (b * part_nwg + part_wg_base + w) * part_cap)
  bool part_slab = false;
  // dense LDS group-by of COUNT + one integer SUM / AVG with a value image: both planes in ONE 64-bit LDS add, the
  // row count above bit dense_pack (the value offset below), flushed per segment (0: two adds per row)
  int dense_pack = 0;
  bool compact = false;   // pack each sub-step's selected rows into consecutive lanes before aggregating (selective)
  bool selmask = false;   // write every row's selection bit (multi-value aggregations read it)
  // with part_slab: narrow records (run_narrow).  The key is mixed (NarrowMix), its top part_bits choose the bucket and
  // the record is the rest of the mix | value dictId << (keybits - part_bits), narrow_vbits wide; it leaves as a u32
  // (the record's low half) plus, when it is wider than 32 bits, a u16 (bits 32..47) in a second array
  bool part_narrow = false;
  int narrow_vbits = 0;
  int narrow_unit = 32;   // records per unit that leaves the scan's rings (ring: two units per bucket)
  bool prefetch2 = false; // raw words of tiles tt+1 AND tt+2 in flight (no gate leaf): twice the bytes in flight
};

// ----- numEntriesScannedInFilter automaton (pgx_stats.cpp builds it, pgx_kernels.hip pgx_fsm_* runs it) -----
constexpr int kFsmMaxLeaves = 10;                // transition tables are indexed by every leaf's membership bit
constexpr int kFsmMaxStates = 4096;
constexpr uint64_t kFsmMaxTable = 1ull << 22;    // u32 entries over all tables
constexpr int kFsmChunkRows = 1024;              // rows one thread runs from every start state
constexpr int kFsmMaxIntervals = 3 * kFsmMaxLeaves + 2;

struct FsmTreeNode {             // the physical filter tree after FilterPlanNode.reorder
  int op = 0;                    // 0 leaf, 1 AND, 2 OR
  int leaf = -1;
  int phys = 3;                  // leaf: 0 sorted, 2 bitmap, 3 scan
  std::vector<FsmTreeNode> kids;
};
struct FsmSegInfo {
  int32_t num_docs = 0;
  std::vector<int64_t> sorted_first, sorted_last;  // per leaf: first / last doc of a sorted leaf's ranges (0, 0 empty)
  uint32_t always_false = 0;                       // scan leaves whose predicate evaluator is alwaysFalse
};
struct FsmPlan {
  int num_states = 0, num_leaves = 0, num_tables = 0;
  std::vector<uint32_t> table;   // [(t * S + q) << L | input] = next_state << 16 | entries counted
  std::vector<std::vector<std::pair<int32_t, int32_t>>> seg_intervals;  // per segment: (first row, table)
};
bool fsm_build(const FsmTreeNode& tree, int num_leaves, const std::vector<FsmSegInfo>& segs, FsmPlan& out,
               std::string* err);

std::string jit_source(const JitShape& s, int* lds_bytes);
// Compile (or fetch from the cache) the kernel for shape s on the current device.  Returns the hipFunction_t as void*.
void* jit_function(const JitShape& s, int device, int* lds_bytes, std::string* err);

}  // namespace pgx
