// libpgx: multi-value columns -- MV aggregation functions and group-by on multi-value columns.
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#include "pgx_host.h"

namespace pgxh {

// Multi-value functions (Count/Sum/Min/Max/AvgMVAggregationFunction, operator/aggregation/function/*MV*.java),
// aggregation-only: the single-value part of the query (its filter and SV functions, or COUNT(*) alone) runs through
// the query kernels, which also write every scanned row's selection bit; pgx_mv_aggregate then folds every value of
// every selected doc of each MV column (count, int64 / f64 sum, min / max over the sorted dictionary's ids).
void run_mv(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
            uint32_t xflags, pgx_result* R, hipStream_t st) {
  if (!q.group_cols.empty()) fail(PGX_ERR_UNSUPPORTED, "multi-value functions with GROUP BY");
  if (!q.kn.jit) fail(PGX_ERR_UNSUPPORTED, "multi-value functions need the query kernels");
  pgx_query qs = q;
  qs.flags |= PGX_Q_NO_STAR_TREE;  // every raw row gets its selection bit
  qs.agg_fn.clear();
  qs.agg_col.clear();
  std::vector<int> sv_pos(q.agg_fn.size(), -1), mv_pos(q.agg_fn.size(), -1);
  std::vector<std::string> mv_cols;
  for (size_t a = 0; a < q.agg_fn.size(); ++a) {
    if (q.agg_fn[a] >= PGX_COUNTMV) {
      const std::string& c = q.agg_col[a];
      for (int s = 0; s < n; ++s) {
        const StagedColumn& col = segs[s]->col(c);
        if (!col.is_mv) fail(PGX_ERR_UNSUPPORTED, "multi-value function on single-value column " + c);
        if (col.data_type == PGX_STRING) fail(PGX_ERR_UNSUPPORTED, "numeric aggregation on STRING column " + c);
      }
      auto it = std::find(mv_cols.begin(), mv_cols.end(), c);
      mv_pos[a] = int(it - mv_cols.begin());
      if (it == mv_cols.end()) mv_cols.push_back(c);
    } else {
      sv_pos[a] = int(qs.agg_fn.size());
      qs.agg_fn.push_back(q.agg_fn[a]);
      qs.agg_col.push_back(q.agg_col[a]);
    }
  }
  if (qs.agg_fn.empty()) {
    qs.agg_fn.push_back(PGX_COUNT);
    qs.agg_col.push_back("");
  }
  ExecPlan P;
  P.want_selmask = true;
  plan_query(ctx, qs, segs, n, bindings, xflags, P);
  P.sel_off.assign(n, 0);
  int64_t words = 0;
  int max_words = 0;
  for (int s = 0; s < n; ++s) {
    P.sel_off[s] = words;
    const int w = (P.ksegs[s].num_docs + 31) / 32 + 1;
    words += w;
    max_words = std::max(max_words, w);
  }
  P.sel_buf = DevBuf(ctx, size_t(std::max<int64_t>(words, 1)) * 4);
  hip_check(hipMemsetAsync(P.sel_buf.p, 0, size_t(std::max<int64_t>(words, 1)) * 4, st), "selection masks");
  ExecBuffers B;
  upload_plan(ctx, P, B, st);
  plan_jit(ctx, qs, segs, n, P, B);
  if (P.jit.empty()) fail(PGX_ERR_UNSUPPORTED, "multi-value functions need the query kernels");
  alloc_outputs(ctx, P, B, nullptr, 0);
  reset_outputs(P, B, st);
  launch_scan(P, st);
  // one item per (segment, MV column); outputs [count, sum, ordered min, ordered max] per column
  std::vector<unsigned long long> init(mv_cols.size() * 4, 0ull);
  for (size_t k = 0; k < mv_cols.size(); ++k) init[4 * k + 2] = ~0ull;
  DevBuf outs(ctx, init.size() * 8);
  hip_check(hipMemcpy(outs.p, init.data(), init.size() * 8, hipMemcpyHostToDevice), "MV outputs init");
  std::vector<MvAgg> items;
  std::vector<int> fp(mv_cols.size(), 0);
  for (size_t k = 0; k < mv_cols.size(); ++k)
    for (int s = 0; s < n; ++s) {
      const StagedColumn& col = segs[s]->col(mv_cols[k]);
      fp[k] = col.data_type == PGX_FLOAT || col.data_type == PGX_DOUBLE;
      MvAgg m{};
      m.vals = col.fwd;
      m.start = col.mv_start.as<const int32_t>();
      m.sel = P.sel_buf.as<uint32_t>() + P.sel_off[s];
      m.dict = col.dict_dev;
      m.out = outs.as<unsigned long long>() + 4 * k;
      m.bits = col.bits;
      m.num_docs = P.ksegs[s].num_docs;
      m.fp = fp[k];
      items.push_back(m);
    }
  DevBuf idev(ctx, std::max<size_t>(1, items.size()) * sizeof(MvAgg));
  hip_check(hipMemcpy(idev.p, items.data(), items.size() * sizeof(MvAgg), hipMemcpyHostToDevice), "MV items H2D");
  PGX_LAUNCH(st, "pgx_mv_aggregate", pgx_launch_mv_aggregate(idev.as<MvAgg>(), int(items.size()), max_words, st), "multi-value aggregation");
  pgx_result Rs;
  finish_result(ctx, qs, P, B, segs, n, st, &Rs, nullptr);
  std::vector<unsigned long long> res(init.size());
  hip_check(hipMemcpy(res.data(), outs.p, res.size() * 8, hipMemcpyDeviceToHost), "MV outputs D2H");
  // assemble in the request's order; numEntriesScannedPostFilter counts the MV columns among the projected ones
  int extra = 0;
  for (const auto& c : mv_cols)
    if (std::find(qs.agg_col.begin(), qs.agg_col.end(), c) == qs.agg_col.end()) ++extra;
  for (int i = 0; i < 4; ++i) R->stats[i] = Rs.stats[i];
  R->stats[2] = Rs.stats[0] * (P.n_proj + extra);
  R->num_aggs = int(q.agg_fn.size());
  R->agg_fn = q.agg_fn;
  R->top_n = q.top_n;
  R->group_by = false;
  R->mode = Rs.mode;
  R->agg_value.assign(q.agg_fn.size(), 0.0);
  R->agg_count.assign(q.agg_fn.size(), 0);
  for (size_t a = 0; a < q.agg_fn.size(); ++a) {
    if (sv_pos[a] >= 0) {
      R->agg_value[a] = Rs.agg_value[sv_pos[a]];
      R->agg_count[a] = Rs.agg_count[sv_pos[a]];
      continue;
    }
    const int k = mv_pos[a];
    const unsigned long long* o = &res[4 * size_t(k)];
    const int64_t cnt = int64_t(o[0]);
    double sum;
    if (fp[k]) std::memcpy(&sum, &o[1], 8);
    else sum = double(int64_t(o[1]));
    R->agg_count[a] = cnt;
    switch (q.agg_fn[a]) {
      case PGX_COUNTMV: R->agg_value[a] = double(cnt); break;
      case PGX_MINMV: R->agg_value[a] = decode_plane(P_MIN_ORD, fp[k], o[2], PGX_MIN); break;
      case PGX_MAXMV: R->agg_value[a] = decode_plane(P_MAX_ORD, fp[k], o[3], PGX_MAX); break;
      default: R->agg_value[a] = sum; break;  // SUMMV; AVGMV: (sum, value count) like AvgPair
    }
  }
}

// Group-by over multi-value group columns and/or with multi-value functions (DefaultGroupKeyGenerator.java:268-608,
// DefaultGroupByExecutor.java:154-196).  The single-value part of the query (its filter) runs through the query kernels,
// which write every scanned row's selection bit; pgx_mv_group then expands each selected doc into its group keys (one
// per combination of its group columns' values) and applies every function's contribution to each; MINMV / MAXMV,
// whose reference fold depends on doc order, run in pgx_mv_group_ordered.  Key spaces and result decoding are the
// single-value ones (dense slots, or 64 / 128-bit hash keys), so finish_result decodes the table as usual.
void run_mv_group(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
                  uint32_t xflags, pgx_result* R, hipStream_t st, const Domain* dom) {
  if (!q.kn.jit) fail(PGX_ERR_UNSUPPORTED, "multi-value group-by needs the query kernels");
  const int na = int(q.agg_fn.size()), ng = int(q.group_cols.size());
  if (ng < 1 || ng > kMaxGroupCols) fail(PGX_ERR_UNSUPPORTED, "multi-value group-by: group column count");
  std::vector<int8_t> mvf(na), fpv(na, 0), cntp(na, -1);
  int extra = 0;
  bool ordered = false;
  for (int a = 0; a < na; ++a) {
    const int f = q.agg_fn[a];
    mvf[a] = int8_t(f);  // pgx_agg_fn and MvFnKind share their numbering
    if (f == PGX_COUNT) continue;
    const bool mvfn = f >= PGX_COUNTMV;
    for (int s = 0; s < n; ++s) {
      const StagedColumn& c = segs[s]->col(q.agg_col[a]);
      if (c.is_mv != mvfn)
        fail(PGX_ERR_UNSUPPORTED, std::string(mvfn ? "multi-value function on single-value column "
                                                   : "single-value aggregation on multi-value column ") + c.name);
      if (c.data_type == PGX_STRING) fail(PGX_ERR_UNSUPPORTED, "numeric aggregation on STRING column " + c.name);
    }
    const StagedColumn& c0 = segs[0]->col(q.agg_col[a]);
    fpv[a] = f != PGX_COUNTMV && (c0.data_type == PGX_FLOAT || c0.data_type == PGX_DOUBLE);
    if (f == PGX_AVGMV) cntp[a] = int8_t(1 + na + extra++);
    ordered = ordered || f == PGX_MINMV || f == PGX_MAXMV;
  }
  if (na + extra > kMaxAggs) fail(PGX_ERR_UNSUPPORTED, "too many functions for a multi-value group-by");

  // 1. selection bits of the single-value filter
  pgx_query qs = q;
  qs.flags |= PGX_Q_NO_STAR_TREE;
  qs.agg_fn.assign(1, PGX_COUNT);
  qs.agg_col.assign(1, "");
  qs.group_cols.clear();
  qs.key_domain.clear();
  ExecPlan P;
  P.want_selmask = true;
  plan_query(ctx, qs, segs, n, bindings, xflags, P);
  P.sel_off.assign(n, 0);
  int64_t words = 0;
  int max_docs = 0;
  for (int s = 0; s < n; ++s) {
    P.sel_off[s] = words;
    words += (P.ksegs[s].num_docs + 31) / 32 + 1;
    max_docs = std::max(max_docs, P.ksegs[s].num_docs);
  }
  P.sel_buf = DevBuf(ctx, size_t(std::max<int64_t>(words, 1)) * 4);
  hip_check(hipMemsetAsync(P.sel_buf.p, 0, size_t(std::max<int64_t>(words, 1)) * 4, st), "selection masks");
  ExecBuffers B;
  upload_plan(ctx, P, B, st);
  plan_jit(ctx, qs, segs, n, P, B);
  if (P.jit.empty() || !P.jit[0].fn) {
    bool empty = true;  // every segment empty: nothing scanned, no groups
    for (int s = 0; s < n; ++s) empty = empty && P.ksegs[s].num_docs == 0;
    if (!empty) fail(PGX_ERR_UNSUPPORTED, "multi-value group-by needs the query kernels");
  }
  alloc_outputs(ctx, P, B, nullptr, 0);
  reset_outputs(P, B, st);
  launch_scan(P, st);

  // 2. key space: global dictionaries per group column; dense slots, or packed 64 / 128-bit hash keys
  KQuery& K = P.kq;
  P.gdicts.clear();
  P.gbits.clear();
  uint64_t prod = 1;
  bool overflow = false;
  int total_bits = 0;
  for (int g = 0; g < ng; ++g) {
    P.gdicts.push_back(dom ? domain_dict(*dom, g, n) : group_dict(q, segs, n, g));
    const int64_t gc = std::max<int64_t>(1, P.gdicts.back().card);
    if (!overflow && prod > (uint64_t(1) << 62) / uint64_t(gc)) overflow = true;
    if (!overflow) prod *= uint64_t(gc);
    P.gbits.push_back(bits_for(gc));
    total_bits += P.gbits.back();
  }
  P.mode_ref = reference_mode(q, segs[0]);
  K.num_gcols = ng;
  const uint64_t kDenseMax = uint64_t(1) << 22;
  if (!overflow && prod <= kDenseMax && !(xflags & PGX_X_FORCE_HASH)) {
    uint64_t mul = 1;
    for (int g = 0; g < ng; ++g) {
      K.gmul[g] = mul;
      mul *= uint64_t(P.gdicts[g].card);
    }
    K.group_mode = G_DENSE_GLOBAL;
    P.dense_slots = prod;
  } else if (total_bits <= 126) {
    int sh = 0;
    bool hi = false;
    for (int g = 0; g < ng; ++g) {
      if (sh + P.gbits[g] > 63) {  // a field never straddles two words; each word keeps <= 63 bits
        if (hi) fail(PGX_ERR_UNSUPPORTED, "multi-value group-by: group key needs more than two 63-bit words");
        hi = true;
        sh = 0;
      }
      K.gshift[g] = sh;
      K.ghi[g] = hi;
      sh += P.gbits[g];
    }
    K.group_mode = hi ? G_HASH128 : G_HASH64;
    K.key_words = hi ? 2 : 1;
  } else {
    fail(PGX_ERR_UNSUPPORTED, "multi-value group-by: group key wider than 126 bits");
  }
  const bool dense = K.group_mode == G_DENSE_GLOBAL;
  K.num_aggs = na;
  K.num_planes = 1 + na + extra;
  K.plane_op[0] = P_ADD_I64;
  P.g_count_plane.assign(na, -1);
  for (int a = 0; a < na; ++a) {
    const int f = q.agg_fn[a];
    K.agg_fp[a] = fpv[a];
    K.agg_kind[a] = f == PGX_COUNT ? A_COUNT : (f == PGX_MIN || f == PGX_MINMV) ? A_MIN
                  : (f == PGX_MAX || f == PGX_MAXMV) ? A_MAX : (f == PGX_AVG || f == PGX_AVGMV) ? A_AVG : A_SUM;
    K.plane_op[a + 1] = K.agg_kind[a] == A_MIN ? P_MIN_ORD : K.agg_kind[a] == A_MAX ? P_MAX_ORD
                      : fpv[a] ? P_ADD_F64 : P_ADD_I64;
    if (f == PGX_COUNTMV) P.g_count_plane[a] = -2;
    if (f == PGX_AVGMV) P.g_count_plane[a] = cntp[a];
  }
  for (int p = 1 + na; p < K.num_planes; ++p) K.plane_op[p] = P_ADD_I64;
  std::vector<std::string> proj;  // numEntriesScannedPostFilter: docs x projected columns
  for (int a = 0; a < na; ++a)
    if (q.agg_fn[a] != PGX_COUNT && std::find(proj.begin(), proj.end(), q.agg_col[a]) == proj.end())
      proj.push_back(q.agg_col[a]);
  for (const auto& g : q.group_cols)
    if (std::find(proj.begin(), proj.end(), g) == proj.end()) proj.push_back(g);
  P.n_proj = int(proj.size());

  // 3. per-segment descriptors, remap tables (one device copy per distinct table)
  std::vector<int32_t> blob;
  std::map<const std::vector<int32_t>*, size_t> roff;
  for (int g = 0; g < ng; ++g)
    if (!P.gdicts[g].identity)
      for (int s = 0; s < n; ++s) {
        const std::vector<int32_t>* rm = P.gdicts[g].remap[s].get();
        if (rm && !roff.count(rm)) {
          roff[rm] = blob.size();
          blob.insert(blob.end(), rm->begin(), rm->end());
        }
      }
  DevBuf rdev(ctx, std::max<size_t>(1, blob.size()) * 4);
  if (!blob.empty())
    hip_check(hipMemcpyAsync(rdev.p, blob.data(), blob.size() * 4, hipMemcpyHostToDevice, st), "remap H2D");
  std::vector<MvGroupSeg> hs(n);
  for (int s = 0; s < n; ++s) {
    MvGroupSeg& m = hs[s];
    m = MvGroupSeg{};
    m.sel = P.sel_buf.as<uint32_t>() + P.sel_off[s];
    m.num_docs = P.ksegs[s].num_docs;
    for (int g = 0; g < ng; ++g) {
      const StagedColumn& c = segs[s]->col(q.group_cols[g]);
      m.g[g].vals = c.fwd;
      m.g[g].start = c.is_mv ? c.mv_start.as<const int32_t>() : nullptr;
      m.g[g].bits = c.bits;
      if (!P.gdicts[g].identity && P.gdicts[g].remap[s])
        m.g[g].remap = rdev.as<int32_t>() + roff[P.gdicts[g].remap[s].get()];
    }
    for (int a = 0; a < na; ++a) {
      if (q.agg_fn[a] == PGX_COUNT) continue;
      const StagedColumn& c = segs[s]->col(q.agg_col[a]);
      m.a[a].vals = c.fwd;
      m.a[a].start = c.is_mv ? c.mv_start.as<const int32_t>() : nullptr;
      m.a[a].dict = c.dict_dev;
      m.a[a].bits = c.bits;
    }
  }
  DevBuf sdev(ctx, std::max<size_t>(1, hs.size()) * sizeof(MvGroupSeg));
  hip_check(hipMemcpyAsync(sdev.p, hs.data(), hs.size() * sizeof(MvGroupSeg), hipMemcpyHostToDevice, st), "MV segs");

  // 4. table + launch (hash tables retried bigger on overflow)
  uint64_t slots = dense ? P.dense_slots : initial_hash_cap(segs, n, P);
  MvGroupArgs A{};
  DevBuf adev(ctx, sizeof(MvGroupArgs)), ovf(ctx, 64), ord;
  for (int attempt = 0;; ++attempt) {
    B.table = DevBuf(ctx, slots * K.num_planes * 8);
    K.table = devp(B.table);
    K.keys = nullptr;
    K.key_state = nullptr;
    uint64_t kw = 0;
    if (!dense) {
      K.hash_cap = slots;
      P.hash_cap = slots;
      kw = K.group_mode == G_HASH128 ? 2 * slots : slots;
      B.keys = DevBuf(ctx, kw * 8);
      K.keys = devp(B.keys);
      if (K.group_mode == G_HASH128) {
        B.key_state = DevBuf(ctx, slots * 4);
        K.key_state = B.key_state.as<unsigned int>();
      }
    } else {
      K.dense_slots = slots;
    }
    PGX_LAUNCH(st, "pgx_init_planes", pgx_launch_init_planes(K.table, slots, K.num_planes, &K, K.keys, kw, K.key_state,
                                                             st),
               "init planes");
    if (ordered) {
      const uint64_t bytes = uint64_t(n) * na * slots * 8;
      if (bytes > (uint64_t(1) << 30)) fail(PGX_ERR_UNSUPPORTED, "MINMV / MAXMV under GROUP BY: key space too large");
      ord = DevBuf(ctx, bytes);
    }
    A.segs = sdev.as<MvGroupSeg>();
    A.nsegs = n;
    A.ngcols = ng;
    A.naggs = na;
    A.group_mode = K.group_mode;
    for (int a = 0; a < na; ++a) {
      A.fn[a] = mvf[a];
      A.fp[a] = fpv[a];
      A.cnt_plane[a] = cntp[a];
    }
    for (int g = 0; g < ng; ++g) {
      A.gmul[g] = K.gmul[g];
      A.gshift[g] = K.gshift[g];
      A.ghi[g] = K.ghi[g];
    }
    A.slots = slots;
    A.table = K.table;
    A.keys = K.keys;
    A.key_state = K.key_state;
    A.overflow = devp(ovf);
    A.ord = ordered ? devp(ord) : nullptr;
    hip_check(hipMemsetAsync(ovf.p, 0, 8, st), "memset");
    hip_check(hipMemcpyAsync(adev.p, &A, sizeof A, hipMemcpyHostToDevice, st), "MV group args");
    PGX_LAUNCH(st, "pgx_mv_group", pgx_launch_mv_group(adev.as<MvGroupArgs>(), n, max_docs, ordered ? 1 : 0, st),
               "multi-value group-by");
    unsigned long long lost = 0;
    hip_check(hipMemcpyAsync(&lost, ovf.p, 8, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    if (!lost) break;
    if (dense || attempt >= 4 || slots >= (uint64_t(1) << 30)) fail(PGX_ERR_OOM, "multi-value group-by hash table");
    slots *= 4;
  }
  finish_result(ctx, q, P, B, segs, n, st, R, nullptr);
}

}  // namespace pgxh
