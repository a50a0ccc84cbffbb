/*
 * pgx.h -- C ABI of the MI355X-native pinot-core segment query path (libpgx.so).
 *
 * This is the drop-in boundary a JNI shim binds.  It replaces, for immutable
 * v1 segments and COUNT/SUM/MIN/MAX/AVG aggregation or group-by queries, the per-segment operator
 * tree the reference builds behind its plan-maker API and the in-JVM combine of the per-segment
 * results.  Reference interfaces replaced (pinot-core/src/main/java/com/linkedin/pinot/core/...):
 *
 *   pgx_segment_stage   <- segment/index/loader/Loaders.java:44-118 (Loaders.IndexSegment.load) +
 *                          segment/index/column/ColumnIndexContainer.java:45-139 (reader per column kind)
 *   pgx_execute         <- plan/maker/InstancePlanMakerImplV2.java:72-109 (makeInnerSegmentPlan /
 *                          makeInterSegmentPlan) -> plan/CombinePlanNode.java:66-124 ->
 *                          operator/MCombineOperator.java:84-199, operator/MCombineGroupByOperator.java:139-233
 *                          over per-segment operator/aggregation/AggregationOperator.java:77-104 and
 *                          operator/aggregation/groupby/AggregationGroupByOperator.java:81-106
 *   pgx_result_*        <- operator/blocks/IntermediateResultsBlock.java:65-233 (aggregation result list,
 *                          AggregationGroupByResult.getResultForKey, ExecutionStatistics)
 *   pgx_leaf_binding    <- operator/filter/predicate/PredicateEvaluator.getMatchingDictionaryIds (the caller's
 *                          PredicateEvaluatorProvider resolves each predicate to dictId space per segment)
 *
 * Conventions: every call returns pgx_status (0 = OK); no C++ exception crosses the ABI; on error
 * pgx_last_error() returns a thread-local message.  Plain pointers and sizes only.  A pgx_ctx is
 * bound to one device and is thread-safe; staged segments are immutable and may be shared by
 * concurrent queries.  Host buffers passed in are only read during the call.
 */
#ifndef PGX_H_
#define PGX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGX_ABI_VERSION 8  /* 7: pgx_mutable_* (realtime segments in place); 8: pgx_result_record_words, records of
                              * every device-resident layout (several value columns, f64 sums) */

typedef enum {
  PGX_OK = 0,
  PGX_ERR_INVALID_ARG = 1,
  PGX_ERR_UNSUPPORTED = 2, /* caller falls back to the Java operators */
  PGX_ERR_OOM = 3,
  PGX_ERR_DEVICE = 4,
  PGX_ERR_TIMEOUT = 5,
  PGX_ERR_INTERNAL = 6
} pgx_status;

typedef enum { PGX_INT = 0, PGX_LONG = 1, PGX_FLOAT = 2, PGX_DOUBLE = 3, PGX_STRING = 4 } pgx_data_type;

/* The *MV functions aggregate every value of a multi-value column in the selected docs
 * (operator/aggregation/function/{Count,Sum,Min,Max,Avg}MVAggregationFunction.java); aggregation-only queries. */
typedef enum { PGX_COUNT = 0, PGX_SUM = 1, PGX_MIN = 2, PGX_MAX = 3, PGX_AVG = 4,
               PGX_COUNTMV = 5, PGX_SUMMV = 6, PGX_MINMV = 7, PGX_MAXMV = 8, PGX_AVGMV = 9 } pgx_agg_fn;

/* Predicate kinds (common/Predicate.java Type); they select the physical filter operator exactly as
 * plan/FilterPlanNode.java:118-132 does and drive the numEntriesScannedInFilter statistic. */
typedef enum { PGX_PRED_EQ = 0, PGX_PRED_NEQ = 1, PGX_PRED_IN = 2, PGX_PRED_NOT_IN = 3, PGX_PRED_RANGE = 4 } pgx_pred_kind;

typedef enum { PGX_F_LEAF = 0, PGX_F_AND = 1, PGX_F_OR = 2 } pgx_filter_op;

typedef enum { PGX_MEM_HOST = 0, PGX_MEM_DEVICE = 1 } pgx_mem_kind;

typedef struct pgx_ctx pgx_ctx;
typedef struct pgx_segment pgx_segment;
typedef struct pgx_query pgx_query;
typedef struct pgx_result pgx_result;

typedef struct {
  int32_t device;          /* HIP device ordinal */
  uint32_t flags;          /* reserved, 0 */
} pgx_ctx_opts;

/* ---- context -------------------------------------------------------------------------------- */
pgx_status pgx_ctx_create(const pgx_ctx_opts* opts, pgx_ctx** out);
pgx_status pgx_ctx_destroy(pgx_ctx* ctx);
const char* pgx_last_error(void);
int32_t pgx_abi_version(void);

/* ---- segments (staging into HBM) ---------------------------------------------------------------
 * Buffers are the VERBATIM v1 file bytes (big-endian), see DESIGN.md "Data layout in HBM".
 * mem == PGX_MEM_DEVICE means fwd/dict/... already live in HBM on the context's device (e.g. produced
 * by pgx_synth_column); the library then references them without copying and the caller keeps them
 * alive until pgx_segment_release. */
typedef struct {
  const char* name;
  int32_t data_type;          /* pgx_data_type */
  int32_t cardinality;
  int32_t bits_per_element;   /* from metadata.properties, never recomputed */
  int32_t is_sorted;
  int32_t dict_width;         /* bytes per dictionary entry (lengthOfEachEntry for STRING) */
  const void* fwd;            /* <col>.sv.unsorted.fwd, ceil(total_docs*bits/8) bytes (NULL if sorted) */
  uint64_t fwd_len;
  const void* sorted_pairs;   /* <col>.sv.sorted.fwd, card x (int32 BE start, int32 BE end) (NULL if unsorted) */
  uint64_t sorted_len;
  const void* dict;           /* <col>.dict */
  uint64_t dict_len;
  const void* inv;            /* <col>.bitmap.inv (optional, host memory) */
  uint64_t inv_len;
  int32_t pad_char;           /* STRING padding byte: metadata "segment.padding.character" ('\0'), '%' when the key
                                 is absent (legacy segments, ColumnMetadata.java:93-98); StringDictionary.get cuts at
                                 its first occurrence (StringDictionary.java:53-66) */
  int32_t is_multi_value;     /* 1: fwd holds <col>.mv.fwd (io/writer/impl/v1/FixedBitMultiValueWriter.java: chunk
                                 offsets, doc-start bitset, fixed-bit values; ColumnIndexContainer.java:78) */
  int32_t total_entries;      /* metadata totalNumberOfEntries (multi-value columns) */
} pgx_column_desc;

typedef struct {
  const char* name;
  int32_t total_docs;
  int32_t total_raw_docs;
  int32_t num_columns;
  const pgx_column_desc* columns;
  const void* star_tree;      /* star-tree.bin in OFF_HEAP format (optional, host memory) */
  uint64_t star_tree_len;
  int32_t mem;                /* pgx_mem_kind of fwd/sorted_pairs/dict */
  int32_t num_star_skip_dims; /* metadata "star.tree.skip.materialization.for.dimensions": dimensions the star tree */
  const char* const* star_skip_dims;  /* does not materialise (RequestUtils.isFitForStarTreeIndex:149-163) */
} pgx_segment_desc;

pgx_status pgx_segment_stage(pgx_ctx* ctx, const pgx_segment_desc* desc, pgx_segment** out);
pgx_status pgx_segment_release(pgx_segment* seg);
/* HBM bytes held by the staged segment (forward indexes + dictionaries + inverted indexes). */
pgx_status pgx_segment_device_bytes(const pgx_segment* seg, uint64_t* out);

/* ---- realtime (consuming) segments, in place -----------------------------------------------------
 * RealtimeSegmentImpl.index (core/realtime/impl/RealtimeSegmentImpl.java:185-334) gives every column value an
 * arrival-order dictId in a mutable dictionary and appends one dictId per doc (a list per doc for multi-value columns).
 * A pgx_mutable keeps those dictIds in HBM: pgx_mutable_append sends only the new docs' ids.  The caller owns the
 * mutable dictionaries; whenever one grew it hands the column's current dictionary SORTED (v1 bytes, as
 * RealtimeSegmentConverter would write it) with the arrival -> sorted id map (pgx_mutable_set_dictionary, O(card)).
 * pgx_mutable_snapshot returns the docs indexed so far as a queryable pgx_segment: the forward indexes are re-packed
 * on the device through the maps (no row crosses PCIe again), unsorted (RealtimeColumnDataSource.isSorted() is false),
 * and columns with has_inverted keep bitmap-filter semantics (FilterPlanNode, numEntriesScannedInFilter) evaluated by
 * scanning the dictIds.  Release snapshots with pgx_segment_release; they stay valid after more appends. */
typedef struct pgx_mutable pgx_mutable;
typedef struct {
  const char* name;
  int32_t data_type;          /* pgx_data_type (multi-value: numeric only) */
  int32_t is_multi_value;
  int32_t has_inverted;       /* in the table's invertedIndexColumns */
} pgx_mutable_column;
pgx_status pgx_mutable_create(pgx_ctx* ctx, const char* name, int32_t capacity, int32_t num_columns,
                              const pgx_mutable_column* columns, pgx_mutable** out);
/* ndocs new docs.  ids[c]: column c's arrival-order dictIds, one per doc, or (multi-value) every value of the new docs
 * in doc order with counts[c][d] values for doc d (>= 1).  counts may be NULL when no column is multi-value. */
pgx_status pgx_mutable_append(pgx_mutable* m, int32_t ndocs, const int32_t* const* ids, const int32_t* const* counts);
pgx_status pgx_mutable_set_dictionary(pgx_mutable* m, int32_t column, int32_t cardinality, const void* dict,
                                      uint64_t dict_len, int32_t dict_width, int32_t pad_char,
                                      const int32_t* arrival_to_sorted);
pgx_status pgx_mutable_snapshot(pgx_mutable* m, pgx_segment** out);
pgx_status pgx_mutable_num_docs(const pgx_mutable* m, int32_t* out);
pgx_status pgx_mutable_release(pgx_mutable* m);

/* ---- query ---------------------------------------------------------------------------------- */
typedef struct {
  int32_t fn;                 /* pgx_agg_fn */
  const char* column;         /* NULL or "*" for COUNT(*) */
} pgx_agg;

/* Filter tree in postfix order.  LEAF: arg = leaf index.  AND / OR: arg = number of children popped. */
typedef struct {
  int32_t op;                 /* pgx_filter_op */
  int32_t arg;
} pgx_filter_node;

typedef struct {
  const char* column;
  int32_t kind;               /* pgx_pred_kind */
} pgx_leaf;

typedef struct {
  int32_t num_aggs;
  const pgx_agg* aggs;
  int32_t num_group_cols;     /* 0 => aggregation-only query */
  const char* const* group_cols;
  int32_t top_n;              /* GROUP BY ... TOP n (reference default 10) */
  int32_t num_filter_nodes;   /* 0 => MatchEntireSegment */
  const pgx_filter_node* filter;
  int32_t num_leaves;
  const pgx_leaf* leaves;
  uint32_t flags;             /* PGX_Q_* */
} pgx_query_desc;

#define PGX_Q_NO_STAR_TREE 0x1u /* debug option useStarTree=false (common/utils/request/RequestUtils.java:229-236) */

pgx_status pgx_query_compile(pgx_ctx* ctx, const pgx_query_desc* desc, pgx_query** out);
/* Cross-process key identity (SURVEY 8e "a host-side global dictionary per group-by column"; ABI 5): the key space of
 * group-by column group_col becomes the caller's sorted distinct values (type PGX_INT / PGX_LONG -> ivals, PGX_FLOAT /
 * PGX_DOUBLE -> dvals, PGX_STRING -> svals, compared bytewise) instead of the union of the executed segments'
 * dictionaries.  Processes that set the same domains plan the same dense slots / packed keys, so their partials merge
 * by slot (RCCL all-reduce) or by packed key (all-to-all + pgx_result_merge_groups) -- the value-keyed merge of
 * MCombineGroupByOperator.java:166-191 without shipping strings.  Results of such a query report seg_index -1 and
 * dict_id = the index into the domain for that column (pgx_result_group_keys / pgx_result_gather).  Every segment value
 * must be in the domain (PGX_ERR_INVALID_ARG otherwise).  num_values 0 clears it. */
pgx_status pgx_query_set_key_domain(pgx_query* q, int32_t group_col, int32_t type, int64_t num_values,
                                    const int64_t* ivals, const double* dvals, const char* const* svals);
pgx_status pgx_query_release(pgx_query* q);

/* Per-(segment, leaf) predicate in dictionary-id space, as produced by the caller's PredicateEvaluator:
 * a doc matches iff its dictId d satisfies  (words ? bit d of words : lo <= d <= hi).
 * For NEQ / NOT_IN the binding describes the MATCHING ids (the complement); the library derives the
 * non-matching list for bitmap exclusion itself.  words has ceil(card/32) little-endian uint32. */
typedef struct {
  int32_t lo;
  int32_t hi;
  const uint32_t* words;      /* host memory, optional */
} pgx_leaf_binding;

/* a-4 inside the library: resolve each leaf's raw predicate values against every segment's dictionary, as
 * PredicateEvaluatorProvider (operator/filter/predicate/PredicateEvaluatorProvider.java:31-54) and the Equals /
 * NotEquals / In / NotIn / RangeOffline evaluators do per segment; Dictionary.indexOf parses the value with the column's
 * type (Integer.parseInt, Long.parseLong, Float.parseFloat, Double.parseDouble; STRING padded with the padding char,
 * StringDictionary.java:37-51).  Segments whose dictionaries are byte-identical share one resolution. */
typedef struct {
  int32_t num_values;         /* EQ / NEQ 1, IN / NOT_IN n, RANGE 2 (lower, upper; "*" = unbounded) */
  const char* const* values;
  int32_t lower_inclusive;    /* RANGE only (RangePredicate.java:31-57) */
  int32_t upper_inclusive;
} pgx_predicate;

typedef struct pgx_bindings pgx_bindings;
/* preds[num_leaves] in the query's leaf order; the result holds bindings[n][num_leaves] for pgx_execute. */
pgx_status pgx_bind_predicates(const pgx_query* q, pgx_segment* const* segs, int32_t n, const pgx_predicate* preds,
                               pgx_bindings** out);
const pgx_leaf_binding* pgx_bindings_array(const pgx_bindings* b);
pgx_status pgx_bindings_release(pgx_bindings* b);

typedef struct {
  uint64_t stream;            /* hipStream_t (0 = the context's own stream) */
  void* dense_out;            /* optional device buffer for the dense group table (multi-GPU merge) */
  uint64_t dense_out_bytes;
  uint32_t flags;             /* PGX_X_* */
} pgx_exec_opts;

#define PGX_X_KEEP_DENSE_ON_DEVICE 0x1u /* leave the dense table in dense_out; do not compact to host */
#define PGX_X_FORCE_HASH 0x2u           /* testing: use the hash group-by path even for small key spaces */
#define PGX_X_NO_PARTITION 0x4u         /* testing: sparse group-by through the global hash table, not the partitioned
                                           record path (pgx_part.cpp run_partitioned) */
#define PGX_X_THROUGHPUT 0x8u           /* the caller keeps several queries in flight (pgx_execute_async): plan every
                                           segment into one launch per kernel instead of the batched pipeline, whose
                                           early start only shortens a lone query's latency (ABI 6) */

/* Execute the query over n segments on the context's device and merge the per-segment partials
 * (the combine).  bindings is [n][num_leaves].  Synchronous w.r.t. the returned result. */
pgx_status pgx_execute(pgx_ctx* ctx, const pgx_query* q, pgx_segment* const* segs, int32_t n,
                       const pgx_leaf_binding* bindings, const pgx_exec_opts* opts, pgx_result** out);
pgx_status pgx_result_release(pgx_result* r);  /* an async result waits for its execution first */

/* Asynchronous execute (SURVEY 8b "async on the stream, then pgx_result_wait"): returns at once with a pending result
 * while the query plans, launches on the context's stream (or opts->stream) and reads back on a library thread.  The
 * segment list, the bindings (including their bitsets) and opts are copied before the call returns; the query and the
 * segments must stay alive until the result is complete.  Every pgx_result_* accessor waits for completion first.
 * Replaces the per-query task the reference submits to its executor (query/executor/ServerQueryExecutorV1Impl.java:
 * 118-134 -> plan/CombinePlanNode.java:66-124 futures). */
pgx_status pgx_execute_async(pgx_ctx* ctx, const pgx_query* q, pgx_segment* const* segs, int32_t n,
                             const pgx_leaf_binding* bindings, const pgx_exec_opts* opts, pgx_result** out);
/* timeout_ms < 0: wait until done.  PGX_ERR_TIMEOUT if still running; otherwise the execution's own status. */
pgx_status pgx_result_wait(pgx_result* r, int64_t timeout_ms);

/* Multi-GPU in one process (SURVEY 8b/8e pgx_execute_multi): ctxs[k] is the context of one device; every segment runs
 * on the device it was staged on (segments never move per query).  The per-device executions run concurrently and
 * their partials merge on ctxs[0]'s device: one key space over ALL segments (the union dictionary per group-by
 * column), dense tables copied over xGMI (hipMemcpyPeerAsync) and reduced plane by plane, device-resident sparse groups
 * copied and merged by a device hash merge (pgx_merge.hip), the rest by key on the host.  Group keys of the result
 * index into THIS segs[] list.  opts: flags only (stream / dense_out must be 0).  Replaces the reference server's one
 * combine over all of its segments (operator/MCombineOperator.java:84-199, MCombineGroupByOperator.java:139-233). */
pgx_status pgx_execute_multi(pgx_ctx* const* ctxs, int32_t nctx, const pgx_query* q, pgx_segment* const* segs,
                             int32_t n, const pgx_leaf_binding* bindings, const pgx_exec_opts* opts, pgx_result** out);

/* Cross-process merge of sparse group-by results (one process per GPU; the caller exchanges the groups, e.g. an RCCL
 * all-to-all by key hash).  A group travels as a record of W uint64 (pgx_result_record_words: W = 1 + planes):
 * packed group key, doc count, then per value column sum, ordered min, ordered max (the layout of the partitioned
 * sparse group-by; an INT / LONG column's sum is int64, a FLOAT / DOUBLE column's the f64 bits).  One value column:
 * W = 5.  pgx_result_device_groups: *n = the number of groups of a result whose groups stay in device memory
 * (PGX_ERR_UNSUPPORTED otherwise) and, when records is non-NULL, the records written to that device buffer
 * (n x W x 8 bytes, on the result's device).  pgx_result_merge_groups: merge n records of like's layout (equal keys
 * combine: counts and integer sums add, f64 sums add in f64 -- in arbitrary order, so within rounding of the
 * reference's sequential order -- minima and maxima take the extreme) into a device-resident result decoded with
 * `like`'s key tables -- valid when every source planned the same key space (identical dictionaries on all ranks);
 * stats (may be NULL: like's) become the result's ExecutionStatistics.  Replaces the cross-server half of
 * MCombineGroupByOperator.java:139-233 (per-function combineTwoValues over equal keys). */
pgx_status pgx_result_device_groups(const pgx_result* r, int64_t* n, void* records);
pgx_status pgx_result_record_words(const pgx_result* r, int32_t* words);
pgx_status pgx_result_merge_groups(pgx_ctx* ctx, const pgx_result* like, const void* records, int64_t n,
                                   const int64_t stats[4], pgx_result** out);

/* ExecutionStatistics: numDocsScanned, numEntriesScannedInFilter, numEntriesScannedPostFilter, totalRawDocs
 * (operator/ExecutionStatistics.java:21-74). */
pgx_status pgx_result_stats(const pgx_result* r, int64_t out[4]);

/* Aggregation-only results.  COUNT: *count. SUM/MIN/MAX: *value. AVG: *value = sum, *count = count.
 * Empty input gives the reference defaults (MIN +inf, MAX -inf, AvgPair(0.0, 0)). */
pgx_status pgx_result_agg(const pgx_result* r, int32_t fn_index, double* value, int64_t* count);

/* Group-by results (combined over the segments, untrimmed). */
pgx_status pgx_result_num_groups(const pgx_result* r, int64_t* n);
/* For group-by column c: per group, the index (into the segs[] given to pgx_execute) of a segment that
 * holds the group's value and that segment's local dictId for it. */
pgx_status pgx_result_group_keys(const pgx_result* r, int32_t c, int32_t* seg_index, int32_t* dict_id);
/* Per group: value (SUM/MIN/MAX; AVG sum) and count (COUNT; AVG count; for SUM/MIN/MAX the group's doc count). */
pgx_status pgx_result_group_values(const pgx_result* r, int32_t fn_index, double* value, int64_t* count);
/* Storage mode the reference would pick for a single segment: 0 ARRAY_BASED, 1 LONG_MAP_BASED, 2 ARRAY_MAP_BASED
 * (operator/aggregation/groupby/DefaultGroupKeyGenerator.java:167-186). */
pgx_status pgx_result_group_mode(const pgx_result* r, int32_t* mode);
/* Combine trim (query/aggregation/groupby/AggregationGroupByOperatorService.java:59-77,284-361): if the number of
 * groups exceeds 20*max(top_n,1000), the indices of the top 5*max(top_n,1000) groups for function fn (MIN ascending,
 * AVG by sum/count, others descending), else all groups.  *n in: capacity, out: count written. */
pgx_status pgx_result_trim(const pgx_result* r, int32_t fn_index, int64_t* group_index, int64_t* n);
/* Keys and values of selected groups only (e.g. the indices pgx_result_trim returned): for group-by column c,
 * seg_index[c*n + j] / dict_id[c*n + j] as pgx_result_group_keys; for function f, value[f*n + j] / count[f*n + j] as
 * pgx_result_group_values.  Results that stay in device memory (sparse group-by) gather on the device and read back
 * only these n groups.  Any output may be NULL. */
pgx_status pgx_result_gather(const pgx_result* r, const int64_t* group_index, int64_t n, int32_t* seg_index,
                             int32_t* dict_id, double* value, int64_t* count);

/* Dense-table layout for PGX_X_KEEP_DENSE_ON_DEVICE (multi-GPU RCCL merge):
 * slots = product of group cardinalities; buffer = (1 + num_aggs) planes of slots x 8 bytes.
 * plane 0: int64 doc count; plane 1+i: function i in its accumulator encoding (pgx_result_dense_plane_op).
 * slots = -1: the query has no such table (GROUP BY a multi-value column, or multi-value functions under GROUP BY:
 * their partials merge by key, pgx_result_group_keys / _values, MCombineGroupByOperator.java:166-191). */
pgx_status pgx_query_dense_slots(const pgx_query* q, pgx_segment* const* segs, int32_t n, int64_t* slots);
/* For plane p: 0 = int64 add, 1 = double add, 2 = uint64 ordered-min, 3 = uint64 ordered-max. */
pgx_status pgx_query_dense_plane_op(const pgx_query* q, pgx_segment* const* segs, int32_t n, int32_t plane, int32_t* op);
/* Decode a (possibly RCCL-reduced) dense table living in device memory into a host-side result. */
pgx_status pgx_result_from_dense(pgx_ctx* ctx, const pgx_query* q, pgx_segment* const* segs, int32_t n,
                                 const void* dense_device, const int64_t stats[4], pgx_result** out);

/* ---- synthetic data (benchmarks) ------------------------------------------------------------
 * Fill a device buffer with the fixed-bit forward index of n rows whose dictId is
 * pgx_synth_value(seed, row) = splitmix64(seed ^ (row * 0x9E3779B97F4A7C15)) % card  (DESIGN.md). */
pgx_status pgx_synth_column(pgx_ctx* ctx, void* device_fwd, int64_t n_rows, int32_t bits, int32_t card,
                            uint64_t seed);
/* Joint columns: the row first draws pair = pgx_synth_value(pair_seed, row) % npairs, the dictId is then
 * pgx_synth_value(seed, pair) % card; columns sharing pair_seed / npairs take values from npairs fixed combinations. */
pgx_status pgx_synth_column_paired(pgx_ctx* ctx, void* device_fwd, int64_t n_rows, int32_t bits, int32_t card,
                                   uint64_t seed, uint64_t pair_seed, uint32_t npairs);
/* Host twin of pgx_synth_column's dictIds (int32 per row). */
pgx_status pgx_synth_dict_ids(uint64_t seed, int64_t n_rows, int32_t card, int32_t* out);
/* Segment creation: the <col>.bitmap.inv bytes of a column (HeapBitmapInvertedIndexCreator.java:42-81 layout, roaring
 * portable format).  out == NULL or cap too small: *len receives the size only. */
/* Segment creation: the <col>.sv.unsorted.fwd bytes of n dictIds at `bits` per value (FixedBitSingleValueWriter:
 * MSB-first, big-endian, values back to back); out holds ceil(n * bits / 8) bytes. */
pgx_status pgx_pack_fixed_bit(const int32_t* ids, int64_t n, int32_t bits, uint8_t* out);
pgx_status pgx_inverted_index_build(const int32_t* ids, int64_t n, int32_t card, uint8_t* out, uint64_t cap,
                                    uint64_t* len);
pgx_status pgx_device_alloc(pgx_ctx* ctx, uint64_t bytes, void** out);
pgx_status pgx_device_free(pgx_ctx* ctx, void* p);
pgx_status pgx_copy_to_device(pgx_ctx* ctx, void* dst, const void* src, uint64_t bytes);
pgx_status pgx_copy_to_host(pgx_ctx* ctx, void* dst, const void* src, uint64_t bytes);

/* ---- timing (bench) ---------------------------------------------------------------------------
 * Kernel time of whole executions (ABI 6): between pgx_timing_start and pgx_timing_stop every kernel the library
 * launches (on any stream: the context's, the side stream of batched plans, a caller's) is bracketed by HIP events on
 * its own stream.  pgx_timing_stop waits for the device and returns out[0] = the union of the launches' busy intervals
 * (concurrent kernels count once: the GPU time the executions cost), out[1] = the summed per-launch durations,
 * out[2] = the span from the first launch's start to the last one's end, all in ms; json (optional) receives the same
 * plus per kernel name [launches, summed ms].  One window at a time per process; no reference counterpart. */
pgx_status pgx_timing_start(pgx_ctx* ctx);
pgx_status pgx_timing_stop(pgx_ctx* ctx, double out[3], char* json, uint64_t json_cap);

/* Run the query `iters` times back to back as ONE plan over all n segments (one launch per kernel), returning the
 * average kernel time per iteration measured with HIP events on the stream it is launched on (diagnostics). */
pgx_status pgx_execute_timed(pgx_ctx* ctx, const pgx_query* q, pgx_segment* const* segs, int32_t n,
                             const pgx_leaf_binding* bindings, int32_t iters, double* total_ms,
                             double* kernel_ms, pgx_result** out);

/* ---- query compiler build checks (no device needed) ---------------------------------------------
 * The scan/aggregate kernels are generated per query shape and compiled by hiprtc for gfx950.
 * pgx_jit_compile_check compiles one generated source; pgx_jit_selftest generates and compiles a representative set
 * of shapes and returns the number that failed (*n_total = number tried), with the compiler log in log. */
int pgx_jit_compile_check(const char* source, char* log, unsigned long log_cap);
int pgx_jit_selftest(int* n_total, char* log, unsigned long log_cap);

#ifdef __cplusplus
}
#endif
#endif /* PGX_H_ */
