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
 *   - or, with inverted indexes, the bitmap filter: each leaf ORs the roaring bitmaps of its (non-)matching dictIds,
 *     flipped for NEQ / NOT_IN (operator/filter/BitmapBasedFilterOperator.java:62-92, docidsets/BitmapDocIdSet.java:60-98);
 *     an AND block ANDs its bitmap children and leapfrogs the rest (docidsets/AndBlockDocIdSet.java:146-229,
 *     dociditerators/AndDocIdIterator.java); an OR block ORs its bitmap children and merges iterators
 *     (docidsets/OrBlockDocIdSet.java:68-122, dociditerators/OrDocIdIterator.java:53-130, a min-scan over the children
 *     in place of the PriorityQueue); the matching docIds are pulled through the root iterator into the same blocks.
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

/* Rows [r0, r1) of the same stream into a zeroed buffer; r0 a multiple of 8, so ranges touch disjoint bytes and may be
   written by separate threads. */
void pgo_synth_fwd_range(uint64_t seed, int64_t r0, int64_t r1, int bits, uint32_t card, uint8_t* out,
                         uint64_t pair_seed, uint32_t npairs) {
  for (int64_t r = r0; r < r1; ++r) {
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
  /* bitmap filter: when leaf_inv != NULL every leaf reads its column's .bitmap.inv ((card+1) big-endian int32 offsets,
     then one portable roaring bitmap per dictId); leaf_excl[l] = 1 for NEQ / NOT_IN leaves */
  const uint8_t* const* leaf_inv;
  const int32_t* leaf_excl;
  /* test speed-up, not a reference structure: with key_parts > 1 a LONG_MAP group-by aggregates only the docs whose
     raw key hashes to key_part (mix64(key) >> 40 mod key_parts); the parts of one segment run as separate tasks and
     hold disjoint groups, each in doc order, so their union is the segment's group map */
  int32_t key_part, key_parts;
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


/* ---------------------------------------------------------------------------------------------------------------------
 * Roaring bitmaps (RoaringBitmap 0.5.x, no run containers): per 64K-doc key a sorted uint16 array (card <= 4096) or a
 * 1024-word bitmap.  Serialized containers are read in place, like ImmutableRoaringBitmap over the mapped index.
 * ------------------------------------------------------------------------------------------------------------------ */
#define RB_EOF INT32_MIN  /* Constants.EOF */

typedef struct {
  uint16_t key;
  int32_t card;
  uint16_t* arr;        /* owned array, or */
  uint64_t* words;      /* owned bitmap, or */
  const uint8_t* src;   /* serialized payload (immutable view) */
} rcont;

typedef struct {
  rcont* c;
  int n, cap;
} rbm;

static inline int rc_is_bitmap(const rcont* c) { return c->card > 4096; }
static inline uint16_t rc_at(const rcont* c, int i) {
  if (c->arr) return c->arr[i];
  uint16_t v;
  memcpy(&v, c->src + 2 * (size_t)i, 2);
  return v;
}
static inline uint64_t rc_word(const rcont* c, int w) {
  if (c->words) return c->words[w];
  uint64_t v;
  memcpy(&v, c->src + 8 * (size_t)w, 8);
  return v;
}

static void rbm_push(rbm* b, rcont c) {
  if (b->n == b->cap) {
    b->cap = b->cap ? b->cap * 2 : 8;
    b->c = (rcont*)realloc(b->c, sizeof(rcont) * (size_t)b->cap);
  }
  b->c[b->n++] = c;
}

static void rbm_free(rbm* b) {
  for (int i = 0; i < b->n; ++i) { free(b->c[i].arr); free(b->c[i].words); }
  free(b->c);
  b->c = NULL;
  b->n = b->cap = 0;
}

/* Portable deserialization view (cookie 12346: key / card-1 pairs, then int32 offsets, then payloads). */
static void rbm_view(rbm* b, const uint8_t* buf) {
  int32_t cookie, n;
  memcpy(&cookie, buf, 4);
  memcpy(&n, buf + 4, 4);
  memset(b, 0, sizeof(*b));
  if (cookie != 12346) return;
  for (int i = 0; i < n; ++i) {
    uint16_t k, cm1;
    int32_t off;
    memcpy(&k, buf + 8 + 4 * (size_t)i, 2);
    memcpy(&cm1, buf + 10 + 4 * (size_t)i, 2);
    memcpy(&off, buf + 8 + 4 * (size_t)n + 4 * (size_t)i, 4);
    rcont c = {k, (int32_t)cm1 + 1, NULL, NULL, buf + off};
    rbm_push(b, c);
  }
}

/* A container from a 1024-word scratch bitmap: array when card <= 4096 (the container type invariant). */
static rcont rc_from_words(uint16_t key, const uint64_t* w) {
  int32_t card = 0;
  for (int i = 0; i < 1024; ++i) card += __builtin_popcountll(w[i]);
  rcont c = {key, card, NULL, NULL, NULL};
  if (card > 4096) {
    c.words = (uint64_t*)malloc(8192);
    memcpy(c.words, w, 8192);
  } else if (card > 0) {
    c.arr = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)card);
    int j = 0;
    for (int i = 0; i < 1024; ++i)
      for (uint64_t x = w[i]; x; x &= x - 1) c.arr[j++] = (uint16_t)(i * 64 + __builtin_ctzll(x));
  }
  return c;
}

static void rc_or_into(uint64_t* w, const rcont* c) {
  if (rc_is_bitmap(c)) {
    for (int i = 0; i < 1024; ++i) w[i] |= rc_word(c, i);
  } else {
    for (int i = 0; i < c->card; ++i) { uint16_t v = rc_at(c, i); w[v >> 6] |= 1ull << (v & 63); }
  }
}

static rcont rc_clone(const rcont* c) {
  rcont o = {c->key, c->card, NULL, NULL, NULL};
  if (rc_is_bitmap(c)) {
    o.words = (uint64_t*)malloc(8192);
    for (int i = 0; i < 1024; ++i) o.words[i] = rc_word(c, i);
  } else {
    o.arr = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(c->card ? c->card : 1));
    for (int i = 0; i < c->card; ++i) o.arr[i] = rc_at(c, i);
  }
  return o;
}

/* MutableRoaringBitmap.or(bitmaps...) / answer.or(x): container-wise union over the keys of all inputs. */
static void rbm_or(rbm* out, rbm* const* in, int k) {
  memset(out, 0, sizeof(*out));
  int* pos = (int*)calloc((size_t)(k ? k : 1), sizeof(int));
  uint64_t* w = (uint64_t*)malloc(8192);
  for (;;) {
    int key = 65536, cnt = 0, only = -1;
    for (int i = 0; i < k; ++i)
      if (pos[i] < in[i]->n && in[i]->c[pos[i]].key < key) key = in[i]->c[pos[i]].key;
    if (key == 65536) break;
    for (int i = 0; i < k; ++i)
      if (pos[i] < in[i]->n && in[i]->c[pos[i]].key == key) { ++cnt; only = i; }
    if (cnt == 1) {
      rbm_push(out, rc_clone(&in[only]->c[pos[only]]));
      ++pos[only];
      continue;
    }
    memset(w, 0, 8192);
    for (int i = 0; i < k; ++i)
      if (pos[i] < in[i]->n && in[i]->c[pos[i]].key == key) rc_or_into(w, &in[i]->c[pos[i]++]);
    rbm_push(out, rc_from_words((uint16_t)key, w));
  }
  free(w);
  free(pos);
}

/* answer.and(x): container-wise intersection, in place (array & array by merge, array & bitmap by probe). */
static void rbm_and_inplace(rbm* a, const rbm* b) {
  rbm out = {0};
  int i = 0, j = 0;
  uint64_t* w = (uint64_t*)malloc(8192);
  while (i < a->n && j < b->n) {
    const rcont* x = &a->c[i];
    const rcont* y = &b->c[j];
    if (x->key < y->key) { ++i; continue; }
    if (y->key < x->key) { ++j; continue; }
    rcont r = {x->key, 0, NULL, NULL, NULL};
    if (rc_is_bitmap(x) && rc_is_bitmap(y)) {
      for (int t = 0; t < 1024; ++t) w[t] = rc_word(x, t) & rc_word(y, t);
      r = rc_from_words(x->key, w);
    } else if (!rc_is_bitmap(x) && !rc_is_bitmap(y)) {
      r.arr = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(x->card < y->card ? x->card : y->card) + 2);
      int p = 0, q = 0;
      while (p < x->card && q < y->card) {
        uint16_t u = rc_at(x, p), v = rc_at(y, q);
        if (u < v) ++p;
        else if (v < u) ++q;
        else { r.arr[r.card++] = u; ++p; ++q; }
      }
    } else {
      const rcont* ar = rc_is_bitmap(x) ? y : x;
      const rcont* bm = rc_is_bitmap(x) ? x : y;
      r.arr = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)ar->card + 2);
      for (int p = 0; p < ar->card; ++p) {
        uint16_t u = rc_at(ar, p);
        if ((rc_word(bm, u >> 6) >> (u & 63)) & 1u) r.arr[r.card++] = u;
      }
    }
    if (r.card) rbm_push(&out, r);
    else { free(r.arr); free(r.words); }
    ++i;
    ++j;
  }
  free(w);
  rbm_free(a);
  *a = out;
}

/* orBitmap.flip(start, end): complement over [start, end), end exclusive. */
static void rbm_flip(rbm* a, int64_t start, int64_t end) {
  if (end <= start) return;
  rbm out = {0};
  uint64_t* w = (uint64_t*)malloc(8192);
  const int klo = (int)(start >> 16), khi = (int)((end - 1) >> 16);
  int i = 0;
  while (i < a->n && a->c[i].key < klo) { rbm_push(&out, a->c[i]); a->c[i].arr = NULL; a->c[i].words = NULL; ++i; }
  for (int key = klo; key <= khi; ++key) {
    memset(w, 0, 8192);
    if (i < a->n && a->c[i].key == key) { rc_or_into(w, &a->c[i]); ++i; }
    const int64_t lo = key == klo ? (start & 0xFFFF) : 0, hi = key == khi ? ((end - 1) & 0xFFFF) : 65535;
    for (int64_t v = lo; v <= hi;) {
      if ((v & 63) == 0 && v + 63 <= hi) { w[v >> 6] = ~w[v >> 6]; v += 64; }
      else { w[v >> 6] ^= 1ull << (v & 63); ++v; }
    }
    rcont r = rc_from_words((uint16_t)key, w);
    if (r.card) rbm_push(&out, r);
  }
  while (i < a->n) { rbm_push(&out, a->c[i]); a->c[i].arr = NULL; a->c[i].words = NULL; ++i; }
  free(w);
  rbm_free(a);
  *a = out;
}

/* IntIterator over a bitmap (ascending). */
typedef struct {
  const rbm* b;
  int ci, pos;
  uint64_t word;
  int wi;
} rb_iter;

static void rbi_init(rb_iter* it, const rbm* b) {
  it->b = b;
  it->ci = 0;
  it->pos = 0;
  it->wi = -1;
  it->word = 0;
}

static int32_t rbi_next(rb_iter* it) { /* RB_EOF when exhausted (hasNext() false) */
  while (it->ci < it->b->n) {
    const rcont* c = &it->b->c[it->ci];
    if (!rc_is_bitmap(c)) {
      if (it->pos < c->card) return ((int32_t)c->key << 16) | rc_at(c, it->pos++);
    } else {
      for (;;) {
        if (it->word) {
          const int t = __builtin_ctzll(it->word);
          it->word &= it->word - 1;
          return ((int32_t)c->key << 16) | (it->wi * 64 + t);
        }
        if (++it->wi >= 1024) break;
        it->word = rc_word(c, it->wi);
      }
    }
    ++it->ci;
    it->pos = 0;
    it->wi = -1;
    it->word = 0;
  }
  return RB_EOF;
}

/* Block doc-id iterators: BitmapDocIdIterator (ranged) / RangelessBitmapDocIdIterator, AndDocIdIterator, OrDocIdIterator */
enum { DIT_BITMAP = 0, DIT_AND = 1, DIT_OR = 2 };
typedef struct dit {
  int kind;
  int32_t cur, lo, hi;   /* currentDocId, [startDocId, endDocId] (ranged bitmap / OR) */
  int ranged;
  rb_iter it;
  struct dit** ch;
  int nch;
  int32_t* ptr;          /* AND: docIdPointers; OR: queued value per child */
  int* inq;              /* OR: iteratorIsInQueue */
  int* has;              /* OR: child has an entry in the queue */
  int32_t cur_max;       /* AND */
} dit;

static int32_t dit_next(dit* d);

static int32_t dit_advance(dit* d, int32_t t) {
  if (d->kind == DIT_BITMAP) {  /* BitmapDocIdIterator.advance: equal -> stay, else step with next() */
    if (d->cur == t) return d->cur;
    int32_t c = dit_next(d);
    while (c < t && c != RB_EOF) c = dit_next(d);
    return c;
  }
  if (d->kind == DIT_AND) {     /* AndDocIdIterator.advance */
    if (d->cur == RB_EOF) return d->cur;
    if (d->cur >= t) return d->cur;
    d->cur_max = t - 1;
    return dit_next(d);
  }
  /* OrDocIdIterator.advance */
  if (d->cur == RB_EOF) return RB_EOF;
  if (t < d->lo) t = d->lo;
  else if (t > d->hi) return d->cur = RB_EOF;
  for (int i = 0; i < d->nch; ++i)
    if (d->has[i] && d->ptr[i] < t) { d->has[i] = 0; d->inq[i] = 0; }
  int32_t m = RB_EOF;
  for (int i = 0; i < d->nch; ++i) {
    if (!d->inq[i]) {
      const int32_t v = dit_advance(d->ch[i], t);
      if (v != RB_EOF) { d->ptr[i] = v; d->has[i] = 1; }
      d->inq[i] = 1;
    }
    if (d->has[i] && (m == RB_EOF || d->ptr[i] < m)) m = d->ptr[i];
  }
  return d->cur = m;
}

static int32_t dit_next(dit* d) {
  if (d->kind == DIT_BITMAP) {
    if (d->cur == RB_EOF) return RB_EOF;
    int32_t c = rbi_next(&d->it);
    if (c == RB_EOF) return d->cur = RB_EOF;
    if (d->ranged) {
      while (c < d->lo) { c = rbi_next(&d->it); if (c == RB_EOF) return d->cur = RB_EOF; }
      if (c > d->hi) c = RB_EOF;
    }
    return d->cur = c;
  }
  if (d->kind == DIT_AND) {     /* AndDocIdIterator.next: leapfrog to the next common docId */
    if (d->cur == RB_EOF) return d->cur;
    d->cur_max = d->cur_max + 1;
    for (int i = 0; i < d->nch; ++i) {
      d->ptr[i] = dit_advance(d->ch[i], d->cur_max);
      if (d->ptr[i] == RB_EOF) { d->cur_max = RB_EOF; break; }
      if (d->ptr[i] > d->cur_max) {
        d->cur_max = d->ptr[i];
        if (i > 0) i = -1;
      }
    }
    return d->cur = d->cur_max;
  }
  /* OrDocIdIterator.next */
  if (d->cur == RB_EOF) return RB_EOF;
  for (int i = 0; i < d->nch; ++i)
    if (d->has[i] && d->ptr[i] <= d->cur) { d->has[i] = 0; d->inq[i] = 0; }
  d->cur++;
  int32_t m = RB_EOF;
  for (int i = 0; i < d->nch; ++i) {
    if (!d->inq[i]) {
      const int32_t v = dit_advance(d->ch[i], d->cur);
      if (v != RB_EOF) { d->ptr[i] = v; d->has[i] = 1; }
      d->inq[i] = 1;
    }
    if (d->has[i] && (m == RB_EOF || d->ptr[i] < m)) m = d->ptr[i];
  }
  return d->cur = m;
}

static dit* dit_new(int kind, int nch) {
  dit* d = (dit*)calloc(1, sizeof(dit));
  d->kind = kind;
  d->cur = -1;
  d->cur_max = -1;
  d->nch = nch;
  if (nch) {
    d->ch = (dit**)calloc((size_t)nch, sizeof(dit*));
    d->ptr = (int32_t*)malloc(sizeof(int32_t) * (size_t)nch);
    d->inq = (int*)calloc((size_t)nch, sizeof(int));
    d->has = (int*)calloc((size_t)nch, sizeof(int));
    for (int i = 0; i < nch; ++i) d->ptr[i] = -1;
  }
  return d;
}

static void dit_free(dit* d) {
  if (!d) return;
  for (int i = 0; i < d->nch; ++i) dit_free(d->ch[i]);
  free(d->ch); free(d->ptr); free(d->inq); free(d->has);
  free(d);
}

/* Filter-tree node while building: a bitmap block (BitmapDocIdSet's answer) or a composite block (AND / OR) whose
   children are nodes; same-operator chains of the postfix program are flattened into one n-ary block, as the query's
   AND / OR lists are. */
typedef struct fnode {
  int op;                 /* 0 bitmap, -1 AND, -2 OR */
  rbm bm;                 /* op 0: the answer (owned, or an in-place view when owns == 0) */
  int owns;
  struct fnode** ch;
  int nch;
} fnode;

static fnode* fn_leaf(const pgo_segment_query* q, int l) {
  const pgo_col* c = &q->cols[q->leaf_col[l]];
  const uint8_t* inv = q->leaf_inv[l];
  const int excl = q->leaf_excl ? q->leaf_excl[l] : 0;
  fnode* f = (fnode*)calloc(1, sizeof(fnode));
  int nb = 0;
  rbm* views = (rbm*)calloc((size_t)c->card + 1, sizeof(rbm));
  rbm** ptrs = (rbm**)calloc((size_t)c->card + 1, sizeof(rbm*));
  for (int id = 0; id < c->card; ++id) {
    const int match = (q->leaf_bits[l][id >> 5] >> (id & 31)) & 1u;
    if (match == excl) continue;  /* matching ids, or the non-matching ones for NEQ / NOT_IN */
    int32_t off = (int32_t)(((uint32_t)inv[4 * id] << 24) | ((uint32_t)inv[4 * id + 1] << 16) |
                            ((uint32_t)inv[4 * id + 2] << 8) | (uint32_t)inv[4 * id + 3]);
    rbm_view(&views[nb], inv + off);
    ptrs[nb] = &views[nb];
    ++nb;
  }
  if (nb > 1 || excl) {           /* MutableRoaringBitmap.or(bitmaps), flipped over [start, end + 1) */
    rbm_or(&f->bm, ptrs, nb);
    if (excl) rbm_flip(&f->bm, 0, q->num_docs);
    f->owns = 1;
  } else if (nb == 1) {
    f->bm = views[0];             /* the index's own bitmap */
    views[0].c = NULL;
    f->owns = 2;                  /* container array owned, payloads in place */
  }
  for (int i = 0; i < nb; ++i) free(views[i].c);
  free(views);
  free(ptrs);
  return f;
}

static void fn_free(fnode* f) {
  if (!f) return;
  if (f->owns == 1) rbm_free(&f->bm);
  else free(f->bm.c);
  for (int i = 0; i < f->nch; ++i) fn_free(f->ch[i]);
  free(f->ch);
  free(f);
}

static dit* bitmap_iter(const rbm* b, int ranged, int32_t lo, int32_t hi) {
  dit* d = dit_new(DIT_BITMAP, 0);
  rbi_init(&d->it, b);
  d->ranged = ranged;
  d->lo = lo;
  d->hi = hi;
  return d;
}

/* Materialize a node's iterator (FilterBlockDocIdSet.iterator()); scratch bitmaps are kept in *keep for freeing. */
static dit* fn_iter(fnode* f, int32_t max_doc, rbm** keep, int* nkeep) {
  if (f->op == 0) return bitmap_iter(&f->bm, 1, 0, max_doc);
  int nbm = 0;
  for (int i = 0; i < f->nch; ++i) nbm += f->ch[i]->op == 0;
  if (f->op == -2) {              /* OrBlockDocIdSet.iterator */
    const int nit = (f->nch - nbm) + (nbm ? 1 : 0);
    dit* d = dit_new(DIT_OR, nit);
    d->lo = 0;
    d->hi = max_doc;
    int j = 0;
    for (int i = 0; i < f->nch; ++i)
      if (f->ch[i]->op != 0) d->ch[j++] = fn_iter(f->ch[i], max_doc, keep, nkeep);
    if (nbm) {                    /* answer = first.toMutableRoaringBitmap(); answer.or(each other) */
      rbm* ans = (rbm*)calloc(1, sizeof(rbm));
      rbm* first[1];
      int got = 0;
      for (int i = 0; i < f->nch; ++i) {
        if (f->ch[i]->op != 0) continue;
        if (!got) { first[0] = &f->ch[i]->bm; rbm_or(ans, first, 1); got = 1; continue; }
        rbm tmp;
        rbm* two[2] = {ans, &f->ch[i]->bm};
        rbm_or(&tmp, two, 2);
        rbm_free(ans);
        *ans = tmp;
      }
      keep[(*nkeep)++] = ans;
      d->ch[j++] = bitmap_iter(ans, 1, 0, max_doc);
    }
    return d;
  }
  /* AndBlockDocIdSet.fastIterator */
  if (nbm == 0) {
    dit* d = dit_new(DIT_AND, f->nch);
    for (int i = 0; i < f->nch; ++i) d->ch[i] = fn_iter(f->ch[i], max_doc, keep, nkeep);
    return d;
  }
  rbm* ans = (rbm*)calloc(1, sizeof(rbm));
  int got = 0;
  for (int i = 0; i < f->nch; ++i) {
    if (f->ch[i]->op != 0) continue;
    if (!got) { rbm* first[1] = {&f->ch[i]->bm}; rbm_or(ans, first, 1); got = 1; }
    else rbm_and_inplace(ans, &f->ch[i]->bm);
  }
  keep[(*nkeep)++] = ans;
  dit* a = bitmap_iter(ans, 0, 0, max_doc);  /* RangelessBitmapDocIdIterator */
  if (nbm == f->nch) return a;
  dit* d = dit_new(DIT_AND, f->nch - nbm + 1);
  d->ch[0] = a;
  int j = 1;
  for (int i = 0; i < f->nch; ++i)
    if (f->ch[i]->op != 0) d->ch[j++] = fn_iter(f->ch[i], max_doc, keep, nkeep);
  return d;
}

static fnode* fn_build(const pgo_segment_query* q) {
  fnode* stack[64];
  int sp = 0;
  for (int i = 0; i < q->prog_len; ++i) {
    const int op = q->prog[i];
    if (op >= 0) { stack[sp++] = fn_leaf(q, op); continue; }
    fnode* b = stack[--sp];
    fnode* a = stack[--sp];
    fnode* f = (fnode*)calloc(1, sizeof(fnode));
    f->op = op;
    f->ch = (fnode**)calloc((size_t)(a->nch + b->nch + 2), sizeof(fnode*));
    fnode* ab[2] = {a, b};
    for (int t = 0; t < 2; ++t) {
      if (ab[t]->op == op) {      /* flatten (x AND y) AND z into one block */
        for (int u = 0; u < ab[t]->nch; ++u) f->ch[f->nch++] = ab[t]->ch[u];
        ab[t]->nch = 0;
        fn_free(ab[t]);
      } else {
        f->ch[f->nch++] = ab[t];
      }
    }
    stack[sp++] = f;
  }
  return sp ? stack[0] : NULL;
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
  /* bitmap filter: the root block's iterator (numEntriesScannedInFilter stays 0 for bitmap blocks) */
  fnode* froot = NULL;
  dit* droot = NULL;
  rbm* keep[64];
  int nkeep = 0;
  if (q->leaf_inv && q->num_leaves > 0) {
    froot = fn_build(q);
    droot = fn_iter(froot, q->num_docs - 1, keep, &nkeep);
  }
  for (;;) {
    /* BReusableFilteredDocIdSetOperator: collect up to `block` matching docIds via the block's iterator */
    int n = 0;
    while (droot && n < block) {
      const int32_t d = dit_next(droot);
      if (d == RB_EOF) break;
      doc_ids[n++] = d;
    }
    while (!droot && n < block && next < q->num_docs) {
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
        } else if (q->key_parts > 1 && (int32_t)((mix64((uint64_t)raw) >> 40) % (uint64_t)q->key_parts) != q->key_part) {
          gkeys[i] = -1;
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
        if (k < 0) continue;
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
  if (droot) {
    dit_free(droot);
    fn_free(froot);
    for (int i = 0; i < nkeep; ++i) { rbm_free(keep[i]); free(keep[i]); }
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

/* Synthetic dictIds (pgo_synth_value per row, unpaired): the ids the forward index packs. */
void pgo_synth_ids(uint64_t seed, int64_t n, uint32_t card, int32_t* out) {
  for (int64_t r = 0; r < n; ++r) out[r] = (int32_t)pgo_synth_value(seed, r, card);
}

/* <col>.bitmap.inv writer (core/segment/creator/impl/inv/BitmapInvertedIndexCreator.java: one portable roaring bitmap
   per dictId behind (card + 1) big-endian int32 offsets).  Returns the file size; writes it when cap suffices. */
int64_t pgo_inverted_build(const int32_t* ids, int64_t n, int32_t card, uint8_t* out, int64_t cap) {
  int64_t* start = (int64_t*)calloc((size_t)card + 1, sizeof(int64_t));
  for (int64_t r = 0; r < n; ++r) start[ids[r] + 1]++;
  for (int32_t i = 0; i < card; ++i) start[i + 1] += start[i];
  int32_t* docs = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * ((size_t)card + 1));
  memcpy(fill, start, sizeof(int64_t) * ((size_t)card + 1));
  for (int64_t r = 0; r < n; ++r) docs[fill[ids[r]]++] = (int32_t)r;
  int64_t total = 4 * ((int64_t)card + 1);
  for (int pass = 0; pass < 2; ++pass) {
    int64_t pos = 4 * ((int64_t)card + 1);
    for (int32_t id = 0; id <= card; ++id) {
      if (pass && out) {
        out[4 * id] = (uint8_t)(pos >> 24); out[4 * id + 1] = (uint8_t)(pos >> 16);
        out[4 * id + 2] = (uint8_t)(pos >> 8); out[4 * id + 3] = (uint8_t)pos;
      }
      if (id == card) break;
      const int32_t* d = docs + start[id];
      const int64_t m = start[id + 1] - start[id];
      int32_t nk = 0;
      for (int64_t i = 0; i < m; ++i)
        if (i == 0 || (d[i] >> 16) != (d[i - 1] >> 16)) ++nk;
      const int64_t hdr = 8 + 8 * (int64_t)nk;
      int64_t body = 0;
      int64_t i = 0;
      uint8_t* o = (pass && out) ? out + pos : NULL;
      if (o) {
        const int32_t cookie = 12346;
        memcpy(o, &cookie, 4);
        memcpy(o + 4, &nk, 4);
      }
      for (int32_t k = 0; k < nk; ++k) {
        const int32_t key = d[i] >> 16;
        int64_t e = i;
        while (e < m && (d[e] >> 16) == key) ++e;
        const int32_t cc = (int32_t)(e - i);
        if (o) {
          const uint16_t kk = (uint16_t)key, cm1 = (uint16_t)(cc - 1);
          const int32_t off = (int32_t)(hdr + body);
          memcpy(o + 8 + 4 * k, &kk, 2);
          memcpy(o + 10 + 4 * k, &cm1, 2);
          memcpy(o + 8 + 4 * (int64_t)nk + 4 * k, &off, 4);
          uint8_t* p = o + hdr + body;
          if (cc <= 4096) {
            for (int64_t t = i; t < e; ++t) { const uint16_t lo = (uint16_t)(d[t] & 0xFFFF); memcpy(p + 2 * (t - i), &lo, 2); }
          } else {
            memset(p, 0, 8192);
            for (int64_t t = i; t < e; ++t) { const int lo = d[t] & 0xFFFF; p[lo >> 3] |= (uint8_t)(1u << (lo & 7)); }
          }
        }
        body += cc <= 4096 ? 2 * (int64_t)cc : 8192;
        i = e;
      }
      pos += hdr + body;
    }
    total = pos;
    if (!out || cap < total) break;
  }
  free(start);
  free(docs);
  free(fill);
  return total;
}
