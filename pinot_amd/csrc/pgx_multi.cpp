// libpgx: group-by partials of several devices merged into one result (pgx_execute_multi and
// pgx_result_merge_groups).
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#include "pgx_host.h"

namespace pgxh {

// -------------------------------------------------------------------------------------------------
// Merging group-by partials of different devices (MCombineGroupByOperator.java:166-191 semantics: equal
// keys combine with each function's combineTwoValues).
// -------------------------------------------------------------------------------------------------
// The merge op of every plane of a device-resident result (count, then sum / min / max per value column): PlaneOp,
// 2 bits per plane.  A FLOAT / DOUBLE column's sum plane holds f64 bits (pgx_part_aggregate_f64), so it adds as f64.
uint64_t lazy_plane_ops(const pgx_result::Lazy& L) {
  uint64_t ops = uint64_t(P_ADD_I64);
  for (int p = 1; p < L.nplanes; ++p) {
    const int c = (p - 1) / 3, r = (p - 1) % 3;
    bool fp = false;
    for (size_t a = 0; a < L.agg_plane.size(); ++a)
      if (L.agg_plane[a] >= 1 + 3 * c && L.agg_plane[a] <= 3 + 3 * c && L.agg_fp[a]) fp = true;
    const int op = r == 0 ? (fp ? P_ADD_F64 : P_ADD_I64) : (r == 1 ? P_MIN_ORD : P_MAX_ORD);
    ops |= uint64_t(op) << (2 * p);
  }
  return ops;
}

// Sparse groups resident in device memory (packed keys; like.nplanes planes: group i key keys[i * es], plane p
// planes[p * ps + i * es]) -> one device-resident result of like's layout, decoded with `like`'s key tables
// (pgx_merge.hip).
void merge_device_groups(pgx_ctx* ctx, hipStream_t st, const uint64_t* keys, const uint64_t* planes, int64_t es,
                         int64_t ps, int64_t n, const pgx_result::Lazy& like, pgx_result* R) {
  const int NP = like.nplanes;
  const uint64_t ops = lazy_plane_ops(like);
  uint64_t cap = 1024;
  while (cap < uint64_t(std::max<int64_t>(n, 1)) * 2) cap <<= 1;
  DevBuf tkey(ctx, cap * 8), tpl(ctx, cap * NP * 8), ctr(ctx, 64);
  const int64_t ocap = std::max<int64_t>(n, 1);
  DevBuf okey(ctx, size_t(ocap) * 8), oplane(ctx, size_t(ocap) * NP * 8);
  unsigned long long* tp = tpl.as<unsigned long long>();
  hip_check(hipMemsetAsync(tkey.p, 0xFF, cap * 8, st), "merge table");
  for (int p = 0; p < NP; ++p)  // ordered-min planes start at the largest encoding, the others at 0 (0.0 for f64)
    hip_check(hipMemsetAsync(tp + p * cap, ((ops >> (2 * p)) & 3u) == P_MIN_ORD ? 0xFF : 0, cap * 8, st), "merge table");
  hip_check(hipMemsetAsync(ctr.p, 0, 16, st), "merge counters");
  unsigned long long* c = ctr.as<unsigned long long>();
  PGX_LAUNCH(st, "pgx_group_merge", pgx_launch_group_merge(keys, planes, es, ps, n, tkey.as<unsigned long long>(), tp, cap,
                                                           NP, ops, c + 1, st),
            "group merge");
  PGX_LAUNCH(st, "pgx_group_compact", pgx_launch_group_compact(tkey.as<unsigned long long>(), tp, cap, NP,
                                                               okey.as<uint64_t>(), oplane.as<uint64_t>(), ocap, c, st),
            "group compact");
  unsigned long long h[2] = {0, 0};
  hip_check(hipMemcpyAsync(h, c, 16, hipMemcpyDeviceToHost, st), "merge counters D2H");
  hip_check(hipStreamSynchronize(st), "sync");
  if (h[1]) fail(PGX_ERR_INTERNAL, "group merge table overflow");
  R->group_by = true;
  R->num_groups = int64_t(std::min<unsigned long long>(h[0], uint64_t(ocap)));
  auto L = std::make_unique<pgx_result::Lazy>();
  L->okey = std::move(okey);
  L->oplane = std::move(oplane);
  L->ocap = ocap;
  L->gshift = like.gshift;
  L->gbits = like.gbits;
  L->rep_seg = like.rep_seg;
  L->rep_id = like.rep_id;
  L->agg_kind = like.agg_kind;
  L->agg_plane = like.agg_plane;
  L->agg_fp = like.agg_fp;
  L->nplanes = NP;
  ctx->refs.fetch_add(1);
  L->ctx = ctx;
  R->lazy = std::move(L);
}

// Combine of one function's partial (value, count) into an accumulated one (the host-side combineTwoValues).
// A multi-value group column, or a multi-value function (run_mv / run_mv_group execute these).
bool query_is_mv(const pgx_query& q, pgx_segment* const* segs, int n) {
  for (int fn : q.agg_fn)
    if (fn >= PGX_COUNTMV) return true;
  for (const auto& g : q.group_cols)
    for (int s = 0; s < n; ++s)
      if (segs[s]->col(g).is_mv) return true;
  return false;
}

void combine_partial(int fn, double& v, int64_t& c, double v2, int64_t c2) {
  if (fn == PGX_MIN || fn == PGX_MINMV) v = std::min(v, v2);  // MinMVAggregationFunction.combineTwoValues: Math.min
  else if (fn == PGX_MAX || fn == PGX_MAXMV) v = std::max(v, v2);
  else if (fn == PGX_COUNT) v = double(c + c2);
  else v += v2;  // SUM, AVG sum; COUNTMV / SUMMV / AVGMV sums
  c += c2;
}

// Host merge of materialised group-by results whose keys come from one Domain (equal global ids <=> equal
// (rep segment, rep dictId) pairs, so the pairs key the merge).
void merge_host_groups(std::vector<std::unique_ptr<pgx_result>>& parts, pgx_result* R) {
  const int ncols = int(parts[0]->key_seg.size()), na = parts[0]->num_aggs;
  std::unordered_map<std::string, int64_t> where;
  R->key_seg.assign(ncols, {});
  R->key_id.assign(ncols, {});
  R->g_value.assign(na, {});
  R->g_count.assign(na, {});
  std::string k(size_t(ncols) * 8, '\0');
  for (auto& p : parts) {
    for (int64_t i = 0; i < p->num_groups; ++i) {
      for (int g = 0; g < ncols; ++g) {
        std::memcpy(&k[size_t(g) * 8], &p->key_seg[g][i], 4);
        std::memcpy(&k[size_t(g) * 8 + 4], &p->key_id[g][i], 4);
      }
      auto it = where.find(k);
      if (it == where.end()) {
        where.emplace(k, R->num_groups);
        for (int g = 0; g < ncols; ++g) {
          R->key_seg[g].push_back(p->key_seg[g][i]);
          R->key_id[g].push_back(p->key_id[g][i]);
        }
        for (int a = 0; a < na; ++a) {
          R->g_value[a].push_back(p->g_value[a][i]);
          R->g_count[a].push_back(p->g_count[a][i]);
        }
        ++R->num_groups;
      } else {
        for (int a = 0; a < na; ++a)
          combine_partial(R->agg_fn[a], R->g_value[a][it->second], R->g_count[a][it->second], p->g_value[a][i],
                          p->g_count[a][i]);
      }
    }
  }
}

// pgx_execute_multi: the segments run where they are staged (one thread per context, concurrently), then the partials
// merge on the first context's device: aggregation-only on the host; dense tables over the shared key space are copied
// to that device (hipMemcpyPeerAsync, xGMI between GPUs) and reduced plane by plane; sparse groups still in device
// memory are copied there and merged by pgx_group_merge; anything else merges on the host by key.
void run_multi(pgx_ctx* const* ctxs, int nctx, const pgx_query& q, pgx_segment* const* segs, int n,
               const pgx_leaf_binding* bindings, uint32_t xflags, pgx_result* R) {
  if (n < 1) fail(PGX_ERR_INVALID_ARG, "no segments");
  std::vector<std::vector<int>> part(nctx);
  for (int i = 0; i < n; ++i) {
    int k = 0;
    while (k < nctx && segs[i]->ctx != ctxs[k]) ++k;
    if (k == nctx) fail(PGX_ERR_INVALID_ARG, "segment " + segs[i]->name + " is not staged on any of the contexts");
    part[k].push_back(i);
  }
  std::vector<int> active;
  for (int k = 0; k < nctx; ++k)
    if (!part[k].empty()) active.push_back(k);
  const size_t L = q.leaf_col.size();
  std::vector<GlobalDict> gd;
  for (int g = 0; g < int(q.group_cols.size()); ++g) gd.push_back(group_dict(q, segs, n, g));
  uint64_t slots = 1;
  bool dense = !q.group_cols.empty() && !(xflags & PGX_X_FORCE_HASH) && !query_is_mv(q, segs, n);
  for (const auto& g : gd) {
    if (slots > (uint64_t(1) << 22) / uint64_t(std::max<int64_t>(g.card, 1))) dense = false;
    else slots *= uint64_t(g.card);
  }
  const int nplanes = 1 + int(q.agg_fn.size());
  const int na = int(q.agg_fn.size());
  uint64_t ops = 0;  // dense plane ops, 2 bits per plane (pgx_query_dense_plane_op)
  for (int a = 0; a < na; ++a) {
    const int fn = q.agg_fn[a];
    int op = P_ADD_I64;
    if (fn != PGX_COUNT) {
      const StagedColumn& c = segs[0]->col(q.agg_col[a]);
      const bool fp = c.data_type == PGX_FLOAT || c.data_type == PGX_DOUBLE;
      op = fn == PGX_MIN ? P_MIN_ORD : fn == PGX_MAX ? P_MAX_ORD : (fp ? P_ADD_F64 : P_ADD_I64);
    }
    ops |= uint64_t(op) << (2 * (a + 1));
  }
  const int na_ctx = int(active.size());
  std::vector<Domain> dom(na_ctx);
  std::vector<std::vector<pgx_segment*>> sub(na_ctx);
  std::vector<std::vector<pgx_leaf_binding>> sb(na_ctx);
  std::vector<std::unique_ptr<pgx_result>> res(na_ctx);
  std::vector<DevBuf> tables(na_ctx);
  std::vector<std::exception_ptr> errs(na_ctx);
  const uint64_t tbytes = slots * uint64_t(nplanes) * 8;
  for (int j = 0; j < na_ctx; ++j) {
    const int k = active[j];
    dom[j].g = &gd;
    dom[j].index = part[k];
    for (int i : part[k]) {
      sub[j].push_back(segs[i]);
      if (L) sb[j].insert(sb[j].end(), bindings + size_t(i) * L, bindings + size_t(i + 1) * L);
    }
    res[j] = std::make_unique<pgx_result>();
  }
  auto run_one = [&](int j) {
    pgx_ctx* c = ctxs[active[j]];
    hip_check(hipSetDevice(c->device), "hipSetDevice");
    pgx_exec_opts o{};
    o.flags = xflags & ~uint32_t(PGX_X_KEEP_DENSE_ON_DEVICE);
    if (dense) {
      tables[j] = DevBuf(c, tbytes);
      o.dense_out = tables[j].p;
      o.dense_out_bytes = tbytes;
      o.flags |= PGX_X_KEEP_DENSE_ON_DEVICE;
    }
    run_query(c, q, sub[j].data(), int(sub[j].size()), L ? sb[j].data() : nullptr, &o, res[j].get(), &dom[j]);
  };
  {
    std::vector<std::thread> th;
    for (int j = 1; j < na_ctx; ++j)
      th.emplace_back([&, j] {
        try {
          run_one(j);
        } catch (...) {
          errs[j] = std::current_exception();
        }
      });
    try {
      run_one(0);
    } catch (...) {
      errs[0] = std::current_exception();
    }
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
  }
  pgx_ctx* c0 = ctxs[active[0]];
  hip_check(hipSetDevice(c0->device), "hipSetDevice");
  hipStream_t st = c0->stream;
  int64_t stats[4] = {0, 0, 0, 0};
  for (auto& r : res)
    for (int i = 0; i < 4; ++i) stats[i] += r->stats[i];
  if (q.group_cols.empty()) {
    *R = std::move(*res[0]);
    for (int j = 1; j < na_ctx; ++j)
      for (int a = 0; a < na; ++a)
        combine_partial(q.agg_fn[a], R->agg_value[a], R->agg_count[a], res[j]->agg_value[a], res[j]->agg_count[a]);
  } else if (dense) {
    unsigned long long* t0 = tables[0].as<unsigned long long>();
    DevBuf stage;
    for (int j = 1; j < na_ctx; ++j) {
      const unsigned long long* src = tables[j].as<unsigned long long>();
      if (tables[j].ctx->device != c0->device) {
        if (!stage.p) stage = DevBuf(c0, tbytes);
        hip_check(hipMemcpyPeerAsync(stage.p, c0->device, tables[j].p, tables[j].ctx->device, tbytes, st),
                  "dense table peer copy");
        src = stage.as<unsigned long long>();
      }
      PGX_LAUNCH(st, "pgx_dense_reduce", pgx_launch_dense_reduce(t0, src, slots, nplanes, ops, st), "dense reduce");
    }
    std::vector<unsigned long long> host(slots * nplanes);
    hip_check(hipMemcpyAsync(host.data(), t0, tbytes, hipMemcpyDeviceToHost, st), "dense D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    ExecPlan P;
    std::vector<pgx_leaf_binding> none(sub[0].size() * L, pgx_leaf_binding{0, -1, nullptr});
    plan_query(c0, q, sub[0].data(), int(sub[0].size()), none.data(), xflags, P, &dom[0]);
    ExecBuffers B;
    B.host = PinnedBuf(c0, kOutsBytes);
    B.off_outs = 0;
    std::memset(B.host.p, 0, kOutsBytes);
    reinterpret_cast<unsigned long long*>(B.host.p)[16] = static_cast<unsigned long long>(stats[0]);
    finish_result(c0, q, P, B, sub[0].data(), int(sub[0].size()), st, R, host.data());
  } else {
    bool all_lazy = true;  // every context's groups in device memory, in one plane layout
    for (auto& r : res)
      all_lazy = all_lazy && r->lazy && r->lazy->nplanes == res[0]->lazy->nplanes &&
                 r->lazy->agg_plane == res[0]->lazy->agg_plane && r->lazy->agg_fp == res[0]->lazy->agg_fp;
    *R = pgx_result();
    R->num_aggs = na;
    R->agg_fn = q.agg_fn;
    R->group_by = true;
    if (all_lazy) {
      const int NP = res[0]->lazy->nplanes;
      int64_t total = 0;
      for (auto& r : res) total += r->num_groups;
      DevBuf keys(c0, size_t(std::max<int64_t>(total, 1)) * 8), pl(c0, size_t(std::max<int64_t>(total, 1)) * 8 * NP);
      int64_t off = 0;
      for (auto& r : res) {
        const auto& Lz = *r->lazy;
        const int64_t ng = r->num_groups;
        if (!ng) continue;
        hip_check(hipMemcpyPeerAsync(keys.as<uint64_t>() + off, c0->device, Lz.okey.p, Lz.ctx->device, ng * 8, st),
                  "group keys peer copy");
        for (int p = 0; p < NP; ++p)
          hip_check(hipMemcpyPeerAsync(pl.as<uint64_t>() + p * total + off, c0->device,
                                       Lz.oplane.as<uint64_t>() + p * Lz.ocap, Lz.ctx->device, ng * 8, st),
                    "group planes peer copy");
        off += ng;
      }
      merge_device_groups(c0, st, keys.as<uint64_t>(), pl.as<uint64_t>(), 1, total, total, *res[0]->lazy, R);
    } else {
      for (auto& r : res) r->materialize();
      merge_host_groups(res, R);
    }
  }
  for (int i = 0; i < 4; ++i) R->stats[i] = stats[i];
  R->num_aggs = na;
  R->agg_fn = q.agg_fn;
  R->top_n = q.top_n;
  R->group_by = !q.group_cols.empty();
  if (R->group_by) R->mode = reference_mode(q, segs[0]);
}

}  // namespace pgxh
