/*
 * CPU ORACLE (C twin) -- TEST INFRASTRUCTURE ONLY.  Used by tests/ (full-size spot checks) and by bench.py's
 * cpu_baseline leg; never linked into or called by the product path (libpgx / pinot_amd).
 *
 * A literal C restatement of the reference's per-segment aggregation path, keeping its execution STRUCTURE so that its
 * timing is a meaningful CPU baseline ("port"):
 *   - one thread per segment over a pool of worker threads   (operator/MCombineOperator.java:84-121,
 *                                                             operator/MCombineGroupByOperator.java:154-203)
 *   - per-row fixed-bit reads through readInt                (util/PinotDataCustomBitSet.java:122-155)
 *   - scan filter collecting <= 10000 / 5000 docIds per block (operator/dociditerators/SVScanDocIdIterator.java:102-118,
 *                                                             operator/BReusableFilteredDocIdSetOperator.java:68-93,
 *                                                             plan/DocIdSetPlanNode.java:33, plan/AggregationGroupByPlanNode.java:53)
 *   - projection: dictId gather at the block's docIds, then (double) dictionary values
 *                                                            (operator/aggregation/DataBlockCache.java:79-156)
 *   - block-local double SUM added to the holder; COUNT += block length
 *                                                            (operator/aggregation/function/SumAggregationFunction.java:45-56)
 *   - group-by: key = sum dictId_j * prod card_i (column 0 least significant), holder[key] += v in doc order
 *     (operator/aggregation/groupby/DefaultGroupKeyGenerator.java:214-262, SumAggregationFunction.java:70-81); the
 *     LONG_MAP mode uses an open-addressing long->int map in place of fastutil's Long2IntOpenHashMap.
 * Paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
 *
 * It also generates the synthetic forward indexes bit-identically to libpgx's device generator (pgx_synth_column).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MAX_DOC_PER_CALL 10000
#define GROUP_BY_BLOCK 5000

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

uint32_t pgo_synth_value(uint64_t seed, int64_t row, uint32_t card) {
  return (uint32_t)(splitmix64(seed ^ ((uint64_t)row * 0x9E3779B97F4A7C15ull)) % card);
}

/* Fixed-bit writer (io/writer/impl/FixedBitSingleValueMultiColWriter.java:86-130): MSB-first, big-endian.
   npairs > 0: the row's value is a function of a pair index drawn from pair_seed (libpgx pgx_synth_column_paired). */
void pgo_synth_fwd_paired(uint64_t seed, int64_t n, int bits, uint32_t card, uint8_t* out, int64_t out_len,
                          uint64_t pair_seed, uint32_t npairs) {
  memset(out, 0, (size_t)out_len);
  for (int64_t r = 0; r < n; ++r) {
    const int64_t src = npairs ? (int64_t)pgo_synth_value(pair_seed, r, npairs) : r;
    uint32_t v = pgo_synth_value(seed, src, card);
    int64_t bit = r * bits;
    for (int k = bits - 1; k >= 0; --k, ++bit)
      if ((v >> k) & 1u) out[bit >> 3] |= (uint8_t)(0x80u >> (bit & 7));
  }
}

void pgo_synth_fwd(uint64_t seed, int64_t n, int bits, uint32_t card, uint8_t* out, int64_t out_len) {
  pgo_synth_fwd_paired(seed, n, bits, card, out, out_len, 0, 0);
}

/* PinotDataCustomBitSet.readInt (util/PinotDataCustomBitSet.java:122-155), literal. */
static inline int32_t read_int(const uint8_t* buf, int64_t nr_bytes, int64_t start_bit, int64_t end_bit) {
  int32_t bit_length = (int32_t)(end_bit - start_bit);
  if (bit_length < 16 && end_bit + 32 < nr_bytes * 8) {
    int32_t byte_pos = (int32_t)(start_bit / 8);
    int32_t bit_off = (int32_t)(start_bit % 8);
    int32_t shift = 32 - (bit_off + bit_length);
    int32_t iv = (int32_t)(((uint32_t)buf[byte_pos] << 24) | ((uint32_t)buf[byte_pos + 1] << 16) |
                           ((uint32_t)buf[byte_pos + 2] << 8) | (uint32_t)buf[byte_pos + 3]);
    int32_t mask = (1 << bit_length) - 1;
    return (iv >> shift) & mask;
  }
  int64_t byte_pos = start_bit >> 3;
  int32_t start_off = (int32_t)(start_bit & 7);
  int32_t sum = start_off + bit_length;
  int32_t end_off = (8 - (sum & 7)) & 7;
  int32_t nbytes = (sum + 7) >> 3;
  int64_t number = 0;
  int i = -1;
  for (;;) {
    number |= buf[byte_pos] & 0xFF;
    i++;
    byte_pos++;
    if (i == nbytes - 1) break;
    number <<= 8;
  }
  number >>= end_off;
  number &= (int64_t)(0xFFFFFFFFu >> (32 - bit_length));
  return (int32_t)number;
}

typedef struct {
  const uint8_t* fwd;  /* packed forward index */
  int64_t nbytes;
  int bits;
  const double* dict; /* (double) dictionary values, or NULL */
  int32_t card;
} pgo_col;

typedef struct {
  int32_t num_docs;
  int32_t num_cols;
  const pgo_col* cols;
  /* filter: scan leaf on column filter_col, dictId in [lo, hi]; filter_col < 0 = match all */
  int32_t filter_col, lo, hi;
  /* or, when num_leaves > 0: a postfix program over leaves (prog[i] >= 0: leaf; -1: AND; -2: OR of the top two),
     leaf l matching a row iff the row's dictId of column leaf_col[l] has its bit set in leaf_bits[l] (the dictId
     sets the reference's predicate evaluators resolve, evaluated per row) */
  int32_t num_leaves;
  const int32_t* leaf_col;
  const uint32_t* const* leaf_bits;
  int32_t prog_len;
  const int32_t* prog;
  int32_t metric_col;       /* SUM / MIN / MAX (metric) */
  int32_t num_group_cols;   /* 0 = aggregation only */
  const int32_t* group_cols;
  /* outputs */
  int64_t count;
  double sum, vmin, vmax;
  int64_t entries_scanned;
  /* group-by output: dense table (if card product small) or hash map */
  int64_t num_groups;
  int64_t* g_keys;
  double* g_sums;
  int64_t* g_counts;
  double* g_mins;           /* optional, MIN / MAX per group (+inf / -inf defaults, MinAggregationFunction) */
  double* g_maxs;
  int64_t g_cap;
} pgo_segment_query;

static int row_matches(const pgo_segment_query* q, int64_t d) {
  int stack[32];
  int sp = 0;
  for (int i = 0; i < q->prog_len; ++i) {
    const int op = q->prog[i];
    if (op >= 0) {
      const int32_t id = read_int(q->cols[q->leaf_col[op]].fwd, q->cols[q->leaf_col[op]].nbytes,
                                  d * q->cols[q->leaf_col[op]].bits,
                                  d * q->cols[q->leaf_col[op]].bits + q->cols[q->leaf_col[op]].bits);
      stack[sp++] = (q->leaf_bits[op][id >> 5] >> (id & 31)) & 1u;
    } else {
      const int b = stack[--sp], a = stack[--sp];
      stack[sp++] = op == -1 ? (a & b) : (a | b);
    }
  }
  return sp ? stack[0] : 1;
}

static inline int32_t col_id(const pgo_col* c, int64_t row) {
  return read_int(c->fwd, c->nbytes, row * c->bits, row * c->bits + c->bits);
}

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

/* Long2IntOpenHashMap-like raw-key -> dense group id map (DefaultGroupKeyGenerator.updateRawKeyToGroupKeyMapping). */
typedef struct {
  int64_t* keys;
  int32_t* ids;
  int64_t cap, size;
} lmap;

static void lmap_init(lmap* m, int64_t cap) {
  m->cap = 16;
  while (m->cap < cap * 2) m->cap <<= 1;
  m->keys = (int64_t*)malloc(sizeof(int64_t) * m->cap);
  m->ids = (int32_t*)malloc(sizeof(int32_t) * m->cap);
  for (int64_t i = 0; i < m->cap; ++i) m->keys[i] = -1;
  m->size = 0;
}

static void lmap_grow(lmap* m);

static int32_t lmap_get_or_add(lmap* m, int64_t key) {
  if (m->size * 4 >= m->cap * 3) lmap_grow(m);
  int64_t h = (int64_t)(mix64((uint64_t)key) & (uint64_t)(m->cap - 1));
  for (;;) {
    if (m->keys[h] == key) return m->ids[h];
    if (m->keys[h] == -1) {
      m->keys[h] = key;
      m->ids[h] = (int32_t)m->size;
      return (int32_t)(m->size++);
    }
    h = (h + 1) & (m->cap - 1);
  }
}

static void lmap_grow(lmap* m) {
  lmap n;
  n.cap = m->cap * 2;
  n.keys = (int64_t*)malloc(sizeof(int64_t) * n.cap);
  n.ids = (int32_t*)malloc(sizeof(int32_t) * n.cap);
  for (int64_t i = 0; i < n.cap; ++i) n.keys[i] = -1;
  n.size = m->size;
  for (int64_t i = 0; i < m->cap; ++i) {
    if (m->keys[i] == -1) continue;
    int64_t h = (int64_t)(mix64((uint64_t)m->keys[i]) & (uint64_t)(n.cap - 1));
    while (n.keys[h] != -1) h = (h + 1) & (n.cap - 1);
    n.keys[h] = m->keys[i];
    n.ids[h] = m->ids[i];
  }
  free(m->keys);
  free(m->ids);
  *m = n;
}

static void run_segment(pgo_segment_query* q) {
  const int block = q->num_group_cols ? GROUP_BY_BLOCK : MAX_DOC_PER_CALL;
  int32_t* doc_ids = (int32_t*)malloc(sizeof(int32_t) * block);
  int32_t* dict_ids = (int32_t*)malloc(sizeof(int32_t) * block);
  double* values = (double*)malloc(sizeof(double) * block);
  int32_t* gkeys = (int32_t*)malloc(sizeof(int32_t) * block);
  const pgo_col* fc = q->filter_col >= 0 ? &q->cols[q->filter_col] : NULL;
  const pgo_col* mc = &q->cols[q->metric_col];
  double holder = 0.0, vmin = 1.0 / 0.0, vmax = -1.0 / 0.0;
  int64_t count = 0, scanned = 0;
  int64_t next = 0;
  /* group-by state */
  int64_t prod = 1;
  int overflow = 0;
  for (int g = 0; g < q->num_group_cols; ++g) {
    int64_t c = q->cols[q->group_cols[g]].card;
    if (prod > (int64_t)0x7FFFFFFFFFFFFFFFll / c) overflow = 1;
    else prod *= c;
  }
  const int array_based = q->num_group_cols && !overflow && prod <= 10000;
  double* dsum = NULL;
  int64_t* dcnt = NULL;
  double *dmin = NULL, *dmax = NULL, *mmin = NULL, *mmax = NULL;
  lmap map = {0};
  double* msum = NULL;
  int64_t* mcnt = NULL;
  int64_t mcap = 0;
  if (q->num_group_cols) {
    if (array_based) {
      dsum = (double*)calloc((size_t)prod, sizeof(double));
      dcnt = (int64_t*)calloc((size_t)prod, sizeof(int64_t));
      dmin = (double*)malloc(sizeof(double) * (size_t)prod);
      dmax = (double*)malloc(sizeof(double) * (size_t)prod);
      for (int64_t k = 0; k < prod; ++k) { dmin[k] = 1.0 / 0.0; dmax[k] = -1.0 / 0.0; }
    } else {
      lmap_init(&map, 1024);
      mcap = 1024;
      msum = (double*)calloc((size_t)mcap, sizeof(double));
      mcnt = (int64_t*)calloc((size_t)mcap, sizeof(int64_t));
      mmin = (double*)malloc(sizeof(double) * (size_t)mcap);
      mmax = (double*)malloc(sizeof(double) * (size_t)mcap);
      for (int64_t k = 0; k < mcap; ++k) { mmin[k] = 1.0 / 0.0; mmax[k] = -1.0 / 0.0; }
    }
  }
  for (;;) {
    /* BReusableFilteredDocIdSetOperator: collect up to `block` matching docIds via the scan iterator */
    int n = 0;
    while (n < block && next < q->num_docs) {
      int64_t d = next++;
      if (q->num_leaves > 0) {
        scanned += q->num_leaves;
        if (!row_matches(q, d)) continue;
      } else if (fc) {
        scanned++;
        int32_t id = col_id(fc, d);
        if (id < q->lo || id > q->hi) continue;
      }
      doc_ids[n++] = (int32_t)d;
    }
    if (n == 0) break;
    /* projection: dictId gather + dictionary decode (DataBlockCache) */
    for (int i = 0; i < n; ++i) dict_ids[i] = col_id(mc, doc_ids[i]);
    for (int i = 0; i < n; ++i) values[i] = mc->dict[dict_ids[i]];
    if (!q->num_group_cols) {
      double s = 0.0, lo = 1.0 / 0.0, hi = -1.0 / 0.0;
      for (int i = 0; i < n; ++i) {
        s += values[i];
        if (values[i] < lo) lo = values[i];
        if (values[i] > hi) hi = values[i];
      }
      holder += s;
      if (lo < vmin) vmin = lo;
      if (hi > vmax) vmax = hi;
      count += n;
    } else {
      for (int i = 0; i < n; ++i) {
        int64_t raw = 0;
        for (int g = q->num_group_cols - 1; g >= 0; --g) {
          const pgo_col* gc = &q->cols[q->group_cols[g]];
          raw = raw * gc->card + col_id(gc, doc_ids[i]);
        }
        if (array_based) {
          gkeys[i] = (int32_t)raw;
        } else {
          int32_t id = lmap_get_or_add(&map, raw);
          if (id >= mcap) {
            int64_t nc = mcap * 2;
            msum = (double*)realloc(msum, sizeof(double) * nc);
            mcnt = (int64_t*)realloc(mcnt, sizeof(int64_t) * nc);
            mmin = (double*)realloc(mmin, sizeof(double) * nc);
            mmax = (double*)realloc(mmax, sizeof(double) * nc);
            memset(msum + mcap, 0, sizeof(double) * (nc - mcap));
            memset(mcnt + mcap, 0, sizeof(int64_t) * (nc - mcap));
            for (int64_t k = mcap; k < nc; ++k) { mmin[k] = 1.0 / 0.0; mmax[k] = -1.0 / 0.0; }
            mcap = nc;
          }
          gkeys[i] = id;
        }
      }
      double* S_ = array_based ? dsum : msum;
      int64_t* C_ = array_based ? dcnt : mcnt;
      double* L_ = array_based ? dmin : mmin;
      double* H_ = array_based ? dmax : mmax;
      for (int i = 0; i < n; ++i) {  /* per doc in doc order (Sum/Min/MaxAggregationFunction.aggregateGroupBySV) */
        const int32_t k = gkeys[i];
        S_[k] += values[i];
        C_[k] += 1;
        if (values[i] < L_[k]) L_[k] = values[i];
        if (values[i] > H_[k]) H_[k] = values[i];
      }
      count += n;
    }
  }
  q->count = count;
  q->sum = holder;
  q->vmin = vmin;
  q->vmax = vmax;
  q->entries_scanned = scanned;
  q->num_groups = 0;
  if (q->num_group_cols) {
    int64_t ng = 0;
    if (array_based) {
      for (int64_t k = 0; k < prod; ++k) ng += dcnt[k] > 0;
    } else {
      ng = map.size;
    }
    q->num_groups = ng;
    if (q->g_keys && q->g_cap >= ng) {
      int64_t j = 0;
      if (array_based) {
        for (int64_t k = 0; k < prod; ++k)
          if (dcnt[k]) {
            q->g_keys[j] = k;
            q->g_sums[j] = dsum[k];
            q->g_counts[j] = dcnt[k];
            if (q->g_mins) q->g_mins[j] = dmin[k];
            if (q->g_maxs) q->g_maxs[j] = dmax[k];
            ++j;
          }
      } else {
        for (int64_t h = 0; h < map.cap; ++h)
          if (map.keys[h] != -1) {
            int32_t id = map.ids[h];
            q->g_keys[id] = map.keys[h];
            q->g_sums[id] = msum[id];
            q->g_counts[id] = mcnt[id];
            if (q->g_mins) q->g_mins[id] = mmin[id];
            if (q->g_maxs) q->g_maxs[id] = mmax[id];
          }
      }
    }
    if (array_based) { free(dsum); free(dcnt); free(dmin); free(dmax); }
    else { free(map.keys); free(map.ids); free(msum); free(mcnt); free(mmin); free(mmax); }
  }
  free(doc_ids);
  free(dict_ids);
  free(values);
  free(gkeys);
}

typedef struct {
  pgo_segment_query* qs;
  int n;
  int next;
  pthread_mutex_t mu;
} pool_t;

static void* worker(void* arg) {
  pool_t* p = (pool_t*)arg;
  for (;;) {
    pthread_mutex_lock(&p->mu);
    int i = p->next++;
    pthread_mutex_unlock(&p->mu);
    if (i >= p->n) break;
    run_segment(&p->qs[i]);
  }
  return NULL;
}

/* Run one query over n segments on `threads` worker threads (one segment per task). */
void pgo_run(pgo_segment_query* qs, int n, int threads) {
  pool_t p;
  p.qs = qs;
  p.n = n;
  p.next = 0;
  pthread_mutex_init(&p.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &p);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&p.mu);
}

int32_t pgo_read_int(const uint8_t* buf, int64_t nr_bytes, int64_t start_bit, int64_t end_bit) {
  return read_int(buf, nr_bytes, start_bit, end_bit);
}

int64_t pgo_segment_query_size(void) { return (int64_t)sizeof(pgo_segment_query); }
int64_t pgo_col_size(void) { return (int64_t)sizeof(pgo_col); }
