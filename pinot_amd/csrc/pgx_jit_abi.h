// Argument block shared by the host (pgx_jit.cpp) and the query kernels it generates at run time (hiprtc).
// Plain builtin types only, no includes: this file is compiled by hipcc for the host AND pasted verbatim in front of
// every generated kernel, so both sides see the same layout.
#ifndef PGX_JIT_ABI_H_
#define PGX_JIT_ABI_H_

#define PGX_J_MAX_COLS 16    // distinct columns one generated kernel reads (== kMaxQCols)
#define PGX_J_MAX_LEAVES 16  // filter leaves (== kMaxLeaves)
#define PGX_J_MAX_AGGS 8     // aggregation functions (== kMaxAggs)

// Bitmap inverted-index leaf of one segment: the roaring bitmaps (byte offsets into the staged .bitmap.inv) whose OR
// is the leaf's doc set (BitmapBasedFilterOperator.java:62-92).  pgx::RDesc on the host side.
#define PGX_J_MAX_RPROG 24   // ops of one bitmap program (== kMaxRProg)
#define PGX_J_MAX_RLEAVES 8  // leaves of one bitmap program (== kRProgMaxLeaves)
struct JRDesc {
  unsigned int* mask;            // separate-expansion path only: nchunks x 2048 words
  const unsigned char* inv;      // device copy of <col>.bitmap.inv: (card + 1) big-endian int offsets, then the bitmaps
  const unsigned int* ids;       // dictIds of the roaring bitmaps to OR (bitmap id starts at inv + BE int at inv + 4 id;
                                 // shared by every segment with the same binding)
  int nb;                        // number of bitmaps
  int nchunks;                   // ceil(total_docs / 65536)
};
// A filter sub-tree whose leaves are all bitmap leaves (AND / OR / NOT, postfix), for one segment.  pgx::RProg.
struct JRProg {
  unsigned int* mask;            // separate-expansion path only: nchunks x 2048 words
  int nchunks;
  int num_docs;                  // NOT flips inside [0, num_docs) (BitmapDocIdSet: flip(startDocId, endDocId + 1))
  int nops;
  signed char op[PGX_J_MAX_RPROG];   // 0 leaf, 1 AND, 2 OR, 3 NOT
  short arg[PGX_J_MAX_RPROG];        // leaf: index into the JRDesc array (-1: empty leaf)
  short ldesc[PGX_J_MAX_RLEAVES];    // the leaves' arg values in program order (LEAF_RCHUNK)
};

// Per-segment arguments of one launch group (segments whose columns share bit widths and value-image kinds).
struct JSeg {
  long long tile_begin;                          // first tile of this segment inside the launch group
  int num_docs;                                  // rows scanned: [0, num_docs)
  int pad0;
  const unsigned int* fwd[PGX_J_MAX_COLS];       // packed big-endian fixed-bit forward index
  const void* img[PGX_J_MAX_COLS];               // value image (LDS-staged) of SUM/AVG columns
  const void* dict[PGX_J_MAX_COLS];              // full value table per dictId: int64 (INT/LONG) or double
  const int* remap[PGX_J_MAX_COLS];              // group columns: local dictId -> global id (0 = identity)
  long long vbase[PGX_J_MAX_COLS];               // integer images store value - vbase
  const unsigned int* lbits[PGX_J_MAX_LEAVES];   // scan-bitset leaves: ceil(card/32) words
  const int* lranges[PGX_J_MAX_LEAVES];          // sorted leaves: inclusive [a,b] doc ranges, ascending
  int lnr[PGX_J_MAX_LEAVES];                     // number of ranges
  unsigned int llo[PGX_J_MAX_LEAVES];            // scan-interval leaves: lo <= id <= lo + lspan
  unsigned int lspan[PGX_J_MAX_LEAVES];
  int img_words[PGX_J_MAX_COLS];                 // dwords of img to stage into LDS
  long long rec_base;                            // G_EMIT: index of this segment's row 0 in the record array
  const int* tiles;                              // optional: ascending local tile ids to visit (others hold no
                                                 // selected doc, e.g. outside every star-tree node range); 0 = all
  unsigned int* lmask;                           // statistics automaton: leaf l's predicate bit of row r goes to bit
  long long lmask_words;                         // (r & 31) of word [l * lmask_words + (r >> 5)]
  unsigned int* selmask;                         // selection bit of row r: bit (r & 31) of word r >> 5 (MV functions)
  long long emit_rebase;                         // G_EMIT value records: this segment's vbase - the query's vbase
};

struct JArgs {
  const struct JSeg* segs;
  int num_segs;
  int pad0;
  long long total_tiles;
  long long tiles_per_wg;
  unsigned long long* agg_out;   // aggregation-only: plane accumulators (plane 0 = matched docs)
  unsigned long long* stats;     // [0] docs matched, [1] entries scanned in filter
  unsigned long long* table;     // dense group-by: planes x slots
  const struct JRDesc* rdesc;    // LEAF_RCHUNK leaves: the bitmap descriptors their programs index
  unsigned long long* part_cursor;   // G_EMIT with part_bits: bucket b appends at part_cursor[b * part_cstride]
  unsigned long long* part_overflow; // ... counts buckets that ran past part_cap records
  long long part_cap;                // records per bucket; bucket b's records at table + b * part_cap
  long long part_cstride;
  long long part_wg_base;            // slab mode: this launch's first workgroup slab and the slabs per bucket; slab
  long long part_nwg;                // (b, w) holds records at table + (b * part_nwg + w) * part_cap, its count at
                                     // part_cursor[(b * part_nwg + w) * part_cstride]
  unsigned short* part_hi;           // narrow records wider than 32 bits: bits 32..47, same index as the u32 in table
  unsigned long long* hkeys;         // hash group-by: the global table's keys (1 or 2 words per slot),
  unsigned int* hstate;              // its 128-bit key states,
  long long hash_cap;                // its slots (a power of two; planes at table + p * hash_cap)
  unsigned long long* overflow;      // keys that found no global slot (the host grows the table and reruns)
  long long tile_base;               // first tile of this launch (a plan launched in two halves: the second half's)
};

#endif  // PGX_JIT_ABI_H_
