// libpgx: per-query physical planning -- the filter tree (FilterPlanNode's operator choice and reorder), bitmap
// programs fused from inverted-index leaves, predicate values to dictId ranges, group key spaces
// (DefaultGroupKeyGenerator), the partitioned-path choice, and the per-segment kernel descriptors (plan_query).
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#include <cstring>
#include "pgx_host.h"

namespace pgxh {

PNode build_tree(const pgx_query& q, const pgx_segment& seg0) {
  std::vector<PNode> st;
  for (const auto& n : q.filter) {
    if (n.op == PGX_F_LEAF) {
      if (n.arg < 0 || n.arg >= int(q.leaf_col.size())) fail(PGX_ERR_INVALID_ARG, "filter leaf index out of range");
      PNode p;
      p.op = PGX_F_LEAF;
      p.leaf = n.arg;
      const StagedColumn& c = seg0.col(q.leaf_col[n.arg]);
      if (c.has_inverted && q.leaf_kind[n.arg] != PGX_PRED_RANGE) p.phys = c.is_sorted ? PH_SORTED : PH_BITMAP;
      else p.phys = PH_SCAN;
      st.push_back(std::move(p));
    } else if (n.op == PGX_F_AND || n.op == PGX_F_OR) {
      if (n.arg < 1 || n.arg > int(st.size())) fail(PGX_ERR_INVALID_ARG, "filter node arity");
      PNode p;
      p.op = n.op;
      p.phys = n.op == PGX_F_AND ? PH_AND : PH_OR;
      p.kids.assign(std::make_move_iterator(st.end() - n.arg), std::make_move_iterator(st.end()));
      st.erase(st.end() - n.arg, st.end());
      std::stable_sort(p.kids.begin(), p.kids.end(), [](const PNode& a, const PNode& b) { return a.phys < b.phys; });
      st.push_back(std::move(p));
    } else {
      fail(PGX_ERR_INVALID_ARG, "bad filter op");
    }
  }
  if (st.size() != 1) fail(PGX_ERR_INVALID_ARG, "filter postfix does not reduce to one tree");
  return std::move(st.back());
}

// Emit the device program.  Evaluation order follows AndBlockDocIdSet.fastIterator (operator/docidsets/
// AndBlockDocIdSet.java:146-229): sorted ranges and bitmaps first, then every scan child tested against the running
// candidate set (applyAnd) -- an OP_STAT before each scan child records numEntriesScannedInFilter.  host_scan_leaves
// counts scan leaves whose entries equal the whole scan range (a root scan leaf; scan children of a root OR, which
// OrDocIdIterator advances doc by doc, operator/dociditerators/OrDocIdIterator.java:100-139).
void emit(const PNode& n, std::vector<int8_t>& op, std::vector<int8_t>& arg, bool root, bool stats_inside,
          int& host_scan_leaves) {
  if (n.op == PGX_F_LEAF) {
    op.push_back(OP_LEAF);
    arg.push_back(int8_t(n.leaf));
    if (root && n.phys == PH_SCAN) host_scan_leaves += 1;
    return;
  }
  if (n.op == PGX_F_OR) {
    for (size_t i = 0; i < n.kids.size(); ++i) {
      const PNode& k = n.kids[i];
      if (root && k.op == PGX_F_LEAF && k.phys == PH_SCAN) host_scan_leaves += 1;
      emit(k, op, arg, false, false, host_scan_leaves);
      if (i > 0) { op.push_back(OP_OR); arg.push_back(2); }
    }
    return;
  }
  // AND: index-based children first, then scans with statistics, then nested operators.
  int pushed = 0;
  auto fold = [&]() {
    if (pushed > 1) { op.push_back(OP_AND); arg.push_back(2); }
  };
  for (const PNode& k : n.kids)
    if (k.op == PGX_F_LEAF && (k.phys == PH_SORTED || k.phys == PH_BITMAP)) {
      emit(k, op, arg, false, false, host_scan_leaves);
      ++pushed;
      fold();
    }
  const bool fast = pushed > 0;
  for (const PNode& k : n.kids)
    if (k.op == PGX_F_LEAF && k.phys == PH_SCAN) {
      if (fast || pushed > 0) { op.push_back(OP_STAT); arg.push_back(0); }
      else if (root) host_scan_leaves += 1;  // first scan of an all-scan AND walks the whole range
      emit(k, op, arg, false, false, host_scan_leaves);
      ++pushed;
      fold();
    }
  for (const PNode& k : n.kids)
    if (k.op != PGX_F_LEAF) {
      emit(k, op, arg, false, stats_inside, host_scan_leaves);
      ++pushed;
      fold();
    }
}


double decode_plane(int op, bool fp, unsigned long long x, int fn) {
  if (op == P_ADD_I64) return double(int64_t(x));
  if (op == P_ADD_F64) {
    double d;
    std::memcpy(&d, &x, 8);
    return d;
  }
  // ordered min/max
  if (op == P_MIN_ORD && x == ~0ull) return std::numeric_limits<double>::infinity();
  if (op == P_MAX_ORD && x == 0ull) return -std::numeric_limits<double>::infinity();
  if (!fp) return double(int64_t(x ^ 0x8000000000000000ull));
  uint64_t b = (x & 0x8000000000000000ull) ? (x & ~0x8000000000000000ull) : ~x;
  double d;
  std::memcpy(&d, &b, 8);
  (void)fn;
  return d;
}


GlobalDict build_global_dict(pgx_segment* const* segs, int n, const std::string& col) {
  GlobalDict g;
  const StagedColumn& c0 = segs[0]->col(col);
  // every segment holds the same dictionary?  (long lists: chunks on the context's pool -- the loop is bound by cache
  // misses on the segments' column records, ~45 ns per segment)
  std::atomic<bool> same{true};
  auto check = [&](int lo, int hi) {
    for (int s = lo; s < hi && same.load(std::memory_order_relaxed); ++s) {
      const StagedColumn& c = segs[s]->col(col);
      if (!(c.dict_hash == c0.dict_hash && c.card == c0.card && c.data_type == c0.data_type)) same = false;
    }
  };
  constexpr int kChunk = 256;
  if (n >= 4 * kChunk) segs[0]->ctx->parallel_for((n + kChunk - 1) / kChunk, [&](int i) {
      check(std::max(1, i * kChunk), std::min(n, (i + 1) * kChunk));
    });
  else
    check(1, n);
  if (same) {
    g.card = c0.card;
    g.identity = true;
    g.rep_seg.assign(g.card, 0);
    g.rep_id.resize(g.card);
    std::iota(g.rep_id.begin(), g.rep_id.end(), 0);
    return g;
  }
  g.identity = false;
  g.remap.resize(n);
  // k-way merge of the sorted dictionaries by value, one representative segment per distinct dictionary
  struct Item { int seg; int id; };
  std::vector<Item> all;
  std::map<std::pair<uint64_t, int>, int> first;  // (dict hash, card) -> representative segment
  std::vector<int> rep(n);
  std::vector<std::vector<int32_t>> tabs(n);
  for (int s = 0; s < n; ++s) {
    const StagedColumn& c = segs[s]->col(col);
    if (c.data_type != c0.data_type) fail(PGX_ERR_INVALID_ARG, "column " + col + " has different types");
    auto it = first.emplace(std::make_pair(c.dict_hash, c.card), s).first;
    rep[s] = it->second;
    if (rep[s] != s) continue;
    tabs[s].resize(c.card);
    for (int i = 0; i < c.card; ++i) all.push_back({s, i});
  }
  auto less = [&](const Item& a, const Item& b) {
    const StagedColumn& ca = segs[a.seg]->col(col);
    const StagedColumn& cb = segs[b.seg]->col(col);
    if (c0.data_type == PGX_STRING) return ca.svals[a.id] < cb.svals[b.id];
    if (c0.data_type == PGX_INT || c0.data_type == PGX_LONG) return ca.ivals[a.id] < cb.ivals[b.id];
    return ca.dvals[a.id] < cb.dvals[b.id];
  };
  std::stable_sort(all.begin(), all.end(), less);
  int64_t gid = -1;
  for (size_t i = 0; i < all.size(); ++i) {
    if (i == 0 || less(all[i - 1], all[i])) {
      ++gid;
      g.rep_seg.push_back(all[i].seg);
      g.rep_id.push_back(all[i].id);
    }
    tabs[all[i].seg][all[i].id] = int32_t(gid);
  }
  std::vector<std::shared_ptr<const std::vector<int32_t>>> shared(n);
  for (int s = 0; s < n; ++s) {
    if (rep[s] == s) shared[s] = std::make_shared<const std::vector<int32_t>>(std::move(tabs[s]));
    g.remap[s] = shared[rep[s]];
  }
  g.card = gid + 1;
  return g;
}

// Key space from the caller's domain (pgx_query_set_key_domain): each distinct segment dictionary is remapped by value
// into the domain's sorted values; a value outside the domain is a caller error.
GlobalDict domain_global_dict(const KeyDomain& D, pgx_segment* const* segs, int n, const std::string& col) {
  GlobalDict g;
  g.card = D.size();
  g.identity = false;
  g.remap.resize(n);
  g.rep_seg.assign(size_t(g.card), -1);
  g.rep_id.resize(size_t(g.card));
  std::iota(g.rep_id.begin(), g.rep_id.end(), 0);
  std::map<std::pair<uint64_t, int>, std::shared_ptr<const std::vector<int32_t>>> memo;
  bool ident = true;
  for (int s = 0; s < n; ++s) {
    const StagedColumn& c = segs[s]->col(col);
    const bool str = c.data_type == PGX_STRING, integral = c.data_type == PGX_INT || c.data_type == PGX_LONG;
    if (str != (D.type == PGX_STRING) || integral != (D.type == PGX_INT || D.type == PGX_LONG))
      fail(PGX_ERR_INVALID_ARG, "key domain type differs from column " + col);
    auto& m = memo[std::make_pair(c.dict_hash, c.card)];
    if (!m) {
      std::vector<int32_t> t(c.card);
      for (int i = 0; i < c.card; ++i) {
        int64_t pos;
        if (str) pos = std::lower_bound(D.sv.begin(), D.sv.end(), c.svals[i]) - D.sv.begin();
        else if (integral) pos = std::lower_bound(D.iv.begin(), D.iv.end(), c.ivals[i]) - D.iv.begin();
        else pos = std::lower_bound(D.dv.begin(), D.dv.end(), c.dvals[i]) - D.dv.begin();
        const bool hit = pos < g.card && (str ? D.sv[pos] == c.svals[i]
                                              : integral ? D.iv[pos] == c.ivals[i] : D.dv[pos] == c.dvals[i]);
        if (!hit) fail(PGX_ERR_INVALID_ARG, "a value of column " + col + " is not in its key domain");
        t[i] = int32_t(pos);
        ident = ident && pos == i;
      }
      ident = ident && c.card == g.card;
      m = std::make_shared<const std::vector<int32_t>>(std::move(t));
    }
    g.remap[s] = m;
  }
  if (ident) {  // every segment holds exactly the domain: no remap tables (rep_seg stays -1: keys are domain indices)
    g.identity = true;
    g.remap.clear();
  }
  return g;
}

// The key space of group-by column g: the caller's domain when one is set, else the union of the segments' dictionaries.
GlobalDict group_dict(const pgx_query& q, pgx_segment* const* segs, int n, int g) {
  if (size_t(g) < q.key_domain.size() && q.key_domain[g].set)
    return domain_global_dict(q.key_domain[g], segs, n, q.group_cols[g]);
  return build_global_dict(segs, n, q.group_cols[g]);
}

// Reference storage mode of a single segment (DefaultGroupKeyGenerator.java:167-186): 0 ARRAY_BASED, 1 LONG_MAP_BASED,
// 2 ARRAY_MAP_BASED.
int reference_mode(const pgx_query& q, const pgx_segment* seg) {
  int64_t p1 = 1;
  bool ov = false;
  for (const auto& g : q.group_cols) {
    const int64_t cc = seg->col(g).card;
    if (!ov && p1 > std::numeric_limits<int64_t>::max() / cc) ov = true;
    else if (!ov) p1 *= cc;
  }
  return ov ? 2 : (p1 > 10000 ? 1 : 0);
}


GlobalDict domain_dict(const Domain& d, int col, int n) {
  const GlobalDict& full = (*d.g)[col];
  GlobalDict r;
  r.card = full.card;
  r.identity = full.identity;
  r.rep_seg = full.rep_seg;  // positions in the FULL segment list: the merged result is decoded against it
  r.rep_id = full.rep_id;
  if (!full.identity) {
    r.remap.resize(n);
    for (int s = 0; s < n; ++s) r.remap[s] = full.remap[d.index[s]];
  }
  return r;
}




}  // namespace pgxh

Knobs pgx::read_knobs() {
  Knobs k;
  auto env = [](const char* name) -> std::string {
    const char* e = std::getenv(name);
    return e ? std::string(e) : std::string();
  };
  const std::string jit = env("PGX_JIT"), nar = env("PGX_PART_NARROW"), rc = env("PGX_RCHUNK"), rp = env("PGX_RPROG");
  const std::string bs = env("PGX_BATCH_SEGS"), dbg = env("PGX_DEBUG");
  k.jit = !(jit.size() && jit[0] == '0');
  k.narrow = !(nar.size() && nar[0] == '0');
  k.narrow_direct = nar == "direct";
  k.narrow_gather = nar == "gather";
  if (rc.size()) k.rchunk = rc[0] == '1' ? 1 : 0;
  if (rp == "off") k.rprog = RPROG_OFF;
  else if (rp == "wave") k.rprog = RPROG_WAVE;
  else if (rp == "seg") k.rprog = RPROG_SEG;
  else if (rp == "chunk") k.rprog = RPROG_CHUNK;
  else if (rp == "stack") k.rprog = RPROG_STACK;
  if (bs.size()) k.batch_segs = std::atoi(bs.c_str());
  size_t i = 0;
  while (i < dbg.size()) {
    size_t j = dbg.find(',', i);
    if (j == std::string::npos) j = dbg.size();
    const std::string o = dbg.substr(i, j - i);
    if (o == "part_small") k.part_small = true;
    else if (o == "narrow_log") k.narrow_log = true;
    else if (o == "host_profile") k.host_profile = true;
    else if (o.rfind("narrow_k2=", 0) == 0) k.narrow_k2 = std::atoi(o.c_str() + 10);
    else if (o == "nunit=16") k.narrow_unit = 16;
    else if (o == "pf2") k.prefetch2 = true;
    else if (o == "noimg") k.no_img = true;
    else if (o.rfind("head=", 0) == 0) k.lone_head = std::max(2, std::atoi(o.c_str() + 5));
    i = j + 1;
  }
  return k;
}

namespace pgxh {

int qslot(ExecPlan& P, const std::string& name) {
  for (size_t i = 0; i < P.qcols.size(); ++i)
    if (P.qcols[i] == name) return int(i);
  if (P.qcols.size() >= size_t(kMaxQCols)) fail(PGX_ERR_UNSUPPORTED, "query touches too many columns");
  P.qcols.push_back(name);
  return int(P.qcols.size() - 1);
}

// RequestUtils.isFitForStarTreeIndex (pinot-common/.../common/utils/request/RequestUtils.java:128-220): aggregations
// only SUM, filter a single predicate or an AND of predicates on distinct star-tree dimensions.
bool star_fit(const pgx_query& q, const pgx_segment& seg) {
  if (!seg.st_ok || (q.flags & PGX_Q_NO_STAR_TREE) || q.agg_fn.empty()) return false;
  // group-by and predicate columns must be materialised (:149-163, :195-198, :209-211): a skipped dimension holds the
  // star value in every aggregated doc, so only a raw scan answers for it
  auto skipped = [&](const std::string& c) {
    return std::find(seg.st_skip.begin(), seg.st_skip.end(), c) != seg.st_skip.end();
  };
  for (const auto& g : q.group_cols)
    if (skipped(g)) return false;
  for (const auto& c : q.leaf_col)
    if (skipped(c)) return false;
  for (int fn : q.agg_fn)
    if (fn != PGX_SUM) return false;
  const size_t nl = q.leaf_col.size();
  if (!q.filter.empty()) {
    if (q.filter.size() == 1) {
      if (q.filter[0].op != PGX_F_LEAF) return false;
    } else {
      if (q.filter.back().op != PGX_F_AND || q.filter.back().arg != int(nl) || q.filter.size() != nl + 1) return false;
      for (size_t i = 0; i + 1 < q.filter.size(); ++i)
        if (q.filter[i].op != PGX_F_LEAF) return false;
    }
  }
  for (size_t i = 0; i < nl; ++i) {
    if (std::find(seg.st_dim_name.begin(), seg.st_dim_name.end(), q.leaf_col[i]) == seg.st_dim_name.end()) return false;
    for (size_t j = 0; j < i; ++j)
      if (q.leaf_col[j] == q.leaf_col[i]) return false;
  }
  return true;
}

// StarTreeIndexOperator (operator/filter/StarTreeIndexOperator.java:134-478) for one segment: BFS from the root; at a
// node splitting on a predicate column follow the children of the matching dictIds; on a group-by column (or with no
// star child) follow every non-star child; otherwise take the star child.  An entry matches at a leaf, or once no
// predicate / group-by column remains and the node has an aggregated doc.  Matched entries become: the aggregated doc
// (nothing left to apply), the node's doc range, or the range AND the remaining predicates (createChildOperator).
// The result is expressed as a filter program: OR(exact ranges, range_m AND preds(m) for each remaining-set m).
void plan_star_segment(const pgx_query& q, const pgx_segment& seg, const KSeg& S, const pgx_leaf_binding* b,
                       const std::vector<int>& leaf_phys, std::vector<int32_t>& blob, ExecPlan::StarPlan& sp) {
  const auto& nodes = seg.st_nodes;
  const int nl = int(q.leaf_col.size());
  const int ng = int(q.group_cols.size());
  sp.on = true;
  sp.op.clear();
  sp.arg.clear();
  sp.ranges.clear();
  bool empty = false;
  for (int l = 0; l < nl; ++l)
    if (S.leaf[l].mode == LEAF_NONE) empty = true;  // PredicateEvaluator.alwaysFalse -> emptyResult
  std::map<uint32_t, std::vector<std::pair<int32_t, int32_t>>> groups;  // remaining-predicate mask -> [a, b] ranges
  std::vector<std::pair<int32_t, int32_t>>& exact = groups[0];
  if (!empty) {
    std::vector<int> dim_leaf(seg.st_dim_name.size(), -1), dim_group(seg.st_dim_name.size(), -1);
    for (size_t d = 0; d < seg.st_dim_name.size(); ++d) {
      for (int l = 0; l < nl; ++l)
        if (q.leaf_col[l] == seg.st_dim_name[d]) dim_leaf[d] = l;
      for (int g = 0; g < ng; ++g)
        if (q.group_cols[g] == seg.st_dim_name[d]) dim_group[d] = g;
    }
    auto matches = [&](int l, int id) -> bool {
      const pgx_leaf_binding& x = b[l];
      if (x.words) return (x.words[id >> 5] >> (id & 31)) & 1u;
      return id >= x.lo && id <= x.hi;
    };
    struct Entry { int node; uint32_t pred, gb; };
    std::deque<Entry> queue;
    queue.push_back({0, nl ? (uint32_t(1) << nl) - 1u : 0u, ng ? (uint32_t(1) << ng) - 1u : 0u});
    const int32_t num_raw = seg.total_raw_docs;
    while (!queue.empty()) {
      const Entry e = queue.front();
      queue.pop_front();
      const auto& cur = nodes[e.node];
      const bool leaf = cur.cbeg == -1;
      if (leaf || (e.pred == 0 && e.gb == 0 && cur.agg >= num_raw)) {
        const bool agg_ok = cur.agg >= num_raw;
        if (e.pred == 0) {
          if (agg_ok && e.gb == 0) exact.push_back({cur.agg, cur.agg});
          else if (cur.end > cur.start) exact.push_back({cur.start, cur.end - 1});
        } else if (cur.end > cur.start) {
          groups[e.pred].push_back({cur.start, cur.end - 1});
        }
        continue;
      }
      const int cdim = nodes[cur.cbeg].dim;  // StarTreeIndexNodeOffHeap.getChildDimensionName: first child's dimension
      const int l = (cdim >= 0 && cdim < int(dim_leaf.size())) ? dim_leaf[cdim] : -1;
      const int g = (cdim >= 0 && cdim < int(dim_group.size())) ? dim_group[cdim] : -1;
      Entry ne{0, e.pred, e.gb};
      if (l >= 0) {
        ne.pred &= ~(uint32_t(1) << l);
        if (g >= 0) ne.gb &= ~(uint32_t(1) << g);
        // children sorted by value: each matching dictId is a binary search (getChildForDimensionValue)
        const int card = seg.col(q.leaf_col[l]).card;
        for (int id = 0; id < card; ++id) {
          if (!matches(l, id)) continue;
          int lo = cur.cbeg, hi = cur.cend;
          while (lo <= hi) {
            const int mid = lo + ((hi - lo) >> 1);
            if (nodes[mid].value == id) { ne.node = mid; queue.push_back(ne); break; }
            if (nodes[mid].value < id) lo = mid + 1; else hi = mid - 1;
          }
        }
      } else {
        const bool has_star = nodes[cur.cbeg].value == -1;
        if (g >= 0 || !has_star) {
          for (int c = cur.cbeg; c <= cur.cend; ++c) {
            if (nodes[c].value == -1) continue;
            if (g >= 0) ne.gb &= ~(uint32_t(1) << g);
            ne.node = c;
            queue.push_back(ne);
          }
        } else {
          ne.node = cur.cbeg;
          queue.push_back(ne);
        }
      }
    }
  }
  // ranges -> blob (sorted, merged), program
  auto put_ranges = [&](std::vector<std::pair<int32_t, int32_t>>& r) {
    std::sort(r.begin(), r.end());
    std::vector<int32_t> m;
    for (const auto& x : r) {
      if (!m.empty() && x.first <= m.back() + 1) m.back() = std::max(m.back(), x.second);
      else { m.push_back(x.first); m.push_back(x.second); }
    }
    sp.ranges.push_back({blob.size(), int(m.size() / 2)});
    blob.insert(blob.end(), m.begin(), m.end());
    return nl + int(sp.ranges.size()) - 1;  // leaf index of this range leaf
  };
  int terms = 0;
  for (auto& kv : groups) {
    if (kv.second.empty()) continue;
    const int rl = put_ranges(kv.second);
    sp.op.push_back(OP_LEAF);
    sp.arg.push_back(rl);
    for (int pass = 0; pass < 2; ++pass)  // index-based children first, then scans (AndBlockDocIdSet)
      for (int l = 0; l < nl; ++l) {
        if (!((kv.first >> l) & 1u)) continue;
        const bool scan = leaf_phys[l] == PH_SCAN;
        if (scan != (pass == 1)) continue;
        if (scan) { sp.op.push_back(OP_STAT); sp.arg.push_back(0); }
        sp.op.push_back(OP_LEAF);
        sp.arg.push_back(l);
        sp.op.push_back(OP_AND);
        sp.arg.push_back(2);
      }
    ++terms;
  }
  if (terms == 0) {
    std::vector<std::pair<int32_t, int32_t>> none;
    const int rl = put_ranges(none);
    sp.op.push_back(OP_LEAF);
    sp.arg.push_back(rl);
    terms = 1;
  }
  if (terms > 1) { sp.op.push_back(OP_OR); sp.arg.push_back(terms); }
}

// Does numEntriesScannedInFilter have a closed form the query kernels compute on the fly?  Yes for: no scan leaf at
// all (0); a root scan leaf or a root OR of leaves (SVScanDocIdIterator.next walks its whole [start, end] range,
// OrDocIdIterator.next re-targets a child right after each of its matches); a root AND of leaves with at least one
// sorted / bitmap leaf (AndBlockDocIdSet.fastIterator: each scan's applyAnd tests the running answer -- OP_STAT
// popcounts -- unless its evaluator is alwaysFalse, SVScanDocIdIterator.java:133-135).  Every other tree goes through
// the statistics automaton (pgx_stats.cpp).
bool has_scan_leaf(const PNode& n) {
  if (n.op == PGX_F_LEAF) return n.phys == PH_SCAN;
  for (const PNode& k : n.kids)
    if (has_scan_leaf(k)) return true;
  return false;
}

bool binding_empty(const pgx_leaf_binding& b, int card) {
  if (b.words) {
    const int nw = (card + 31) / 32;
    for (int w = 0; w < nw; ++w)
      if (b.words[w]) return false;
    return true;
  }
  return b.hi < b.lo;
}

bool stats_closed_form(const PNode& root, const pgx_query& q, pgx_segment* const* segs, int n,
                       const pgx_leaf_binding* bindings) {
  if (!has_scan_leaf(root)) return true;
  if (root.op == PGX_F_LEAF) return true;
  for (const PNode& k : root.kids)
    if (k.op != PGX_F_LEAF) return false;
  if (root.op == PGX_F_OR) return true;
  bool index = false;
  for (const PNode& k : root.kids) index |= k.phys == PH_SORTED || k.phys == PH_BITMAP;
  if (!index) return false;
  const size_t L = q.leaf_col.size();
  for (const PNode& k : root.kids)
    if (k.phys == PH_SCAN)
      for (int s = 0; s < n; ++s)
        if (binding_empty(bindings[size_t(s) * L + k.leaf], segs[s]->col(q.leaf_col[k.leaf]).card)) return false;
  return true;
}

// Bitmap sub-trees: a node whose leaves are all bitmap inverted-index leaves (and the bitmap / all-bitmap children of
// any AND / OR) is evaluated per 65536-doc chunk by pgx_roaring_program into ONE doc mask.
struct FusePlan {
  std::map<const PNode*, int> full;   // node evaluated whole by program k
  std::map<const PNode*, int> group;  // AND / OR whose all-bitmap children are program k
  std::vector<ExecPlan::DmProg> progs;
};

bool all_bitmap(const PNode& n) {
  if (n.op == PGX_F_LEAF) return n.phys == PH_BITMAP;
  for (const PNode& k : n.kids)
    if (!all_bitmap(k)) return false;
  return true;
}

void bitmap_prog(const PNode& n, const pgx_query& q, ExecPlan::DmProg& p) {
  if (n.op == PGX_F_LEAF) {
    p.op.push_back(RP_LEAF);
    p.arg.push_back(n.leaf);
    // BitmapBasedFilterOperator NEQ / NOT_IN: OR of the non-matching bitmaps, then flip (BitmapDocIdSet.java:60-73)
    if (q.leaf_kind[n.leaf] == PGX_PRED_NEQ || q.leaf_kind[n.leaf] == PGX_PRED_NOT_IN) {
      p.op.push_back(RP_NOT);
      p.arg.push_back(0);
    }
    return;
  }
  for (size_t i = 0; i < n.kids.size(); ++i) {
    bitmap_prog(n.kids[i], q, p);
    if (i > 0) {
      p.op.push_back(n.op == PGX_F_AND ? RP_AND : RP_OR);
      p.arg.push_back(0);
    }
  }
}

void plan_fuse(const PNode& n, const pgx_query& q, FusePlan& F) {
  if (n.op == PGX_F_LEAF) {
    if (n.phys == PH_BITMAP) {
      F.full[&n] = int(F.progs.size());
      F.progs.emplace_back();
      bitmap_prog(n, q, F.progs.back());
    }
    return;
  }
  if (all_bitmap(n)) {
    F.full[&n] = int(F.progs.size());
    F.progs.emplace_back();
    bitmap_prog(n, q, F.progs.back());
    return;
  }
  std::vector<const PNode*> fk;
  for (const PNode& k : n.kids) {
    if (all_bitmap(k)) fk.push_back(&k);
    else plan_fuse(k, q, F);
  }
  if (fk.empty()) return;
  ExecPlan::DmProg p;
  for (size_t i = 0; i < fk.size(); ++i) {
    bitmap_prog(*fk[i], q, p);
    if (i > 0) {
      p.op.push_back(n.op == PGX_F_AND ? RP_AND : RP_OR);
      p.arg.push_back(0);
    }
  }
  F.group[&n] = int(F.progs.size());
  F.progs.push_back(std::move(p));
}

int prog_depth(const ExecPlan::DmProg& p) {
  int d = 0, mx = 0;
  for (int op : p.op) {
    if (op == RP_LEAF) mx = std::max(mx, ++d);
    else if (op == RP_AND || op == RP_OR) --d;
  }
  return mx;
}

// emit() with bitmap programs: a fused node is one doc-mask leaf (query leaf L + k); an AND / OR puts its fused group
// where its bitmap children were (AND: after the sorted ranges, before the scan children and their OP_STATs).
void emit_fused(const PNode& n, const FusePlan& F, int L, std::vector<int8_t>& op, std::vector<int8_t>& arg, bool root,
                int& host_scan_leaves) {
  auto f = F.full.find(&n);
  if (f != F.full.end()) {
    op.push_back(OP_LEAF);
    arg.push_back(int8_t(L + f->second));
    return;
  }
  if (n.op == PGX_F_LEAF) {
    op.push_back(OP_LEAF);
    arg.push_back(int8_t(n.leaf));
    if (root && n.phys == PH_SCAN) host_scan_leaves += 1;
    return;
  }
  auto g = F.group.find(&n);
  int pushed = 0;
  auto fold = [&](int opc) {
    if (pushed > 1) { op.push_back(int8_t(opc)); arg.push_back(2); }
  };
  if (n.op == PGX_F_OR) {
    for (const PNode& k : n.kids) {
      if (all_bitmap(k)) continue;
      if (root && k.op == PGX_F_LEAF && k.phys == PH_SCAN) host_scan_leaves += 1;
      emit_fused(k, F, L, op, arg, false, host_scan_leaves);
      ++pushed;
      fold(OP_OR);
    }
    if (g != F.group.end()) {
      op.push_back(OP_LEAF);
      arg.push_back(int8_t(L + g->second));
      ++pushed;
      fold(OP_OR);
    }
    return;
  }
  for (const PNode& k : n.kids)
    if (k.op == PGX_F_LEAF && k.phys == PH_SORTED) {
      emit_fused(k, F, L, op, arg, false, host_scan_leaves);
      ++pushed;
      fold(OP_AND);
    }
  if (g != F.group.end()) {
    op.push_back(OP_LEAF);
    arg.push_back(int8_t(L + g->second));
    ++pushed;
    fold(OP_AND);
  }
  const bool fast = pushed > 0;
  for (const PNode& k : n.kids)
    if (k.op == PGX_F_LEAF && k.phys == PH_SCAN) {
      if (fast || pushed > 0) { op.push_back(OP_STAT); arg.push_back(0); }
      else if (root) host_scan_leaves += 1;
      emit_fused(k, F, L, op, arg, false, host_scan_leaves);
      ++pushed;
      fold(OP_AND);
    }
  for (const PNode& k : n.kids)
    if (k.op != PGX_F_LEAF && !all_bitmap(k)) {
      emit_fused(k, F, L, op, arg, false, host_scan_leaves);
      ++pushed;
      fold(OP_AND);
    }
}

FsmTreeNode fsm_tree(const PNode& n) {
  FsmTreeNode t;
  t.op = n.op == PGX_F_LEAF ? 0 : (n.op == PGX_F_AND ? 1 : 2);
  t.leaf = n.leaf;
  t.phys = n.phys;
  for (const PNode& k : n.kids) t.kids.push_back(fsm_tree(k));
  return t;
}


// ----- a-4: predicate values -> dictId space (per segment, memoised per distinct dictionary) -----


std::string trim_ws(const std::string& v) {
  size_t a = 0, b = v.size();
  while (a < b && (unsigned char)v[a] <= ' ') ++a;
  while (b > a && (unsigned char)v[b - 1] <= ' ') --b;
  return v.substr(a, b - a);
}

// Dictionary.indexOf (segment/index/readers/{Int,Long,Float,Double,String}Dictionary.java): binary search, -(insertion
// point) - 1 when absent.
int dict_index_of(const StagedColumn& c, const std::string& raw) {
  auto search = [&](auto less, auto eq) {
    int lo = 0, hi = c.card - 1;
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      if (eq(mid)) return mid;
      if (less(mid)) lo = mid + 1;
      else hi = mid - 1;
    }
    return -(lo + 1);
  };
  switch (c.data_type) {
    case PGX_INT:
    case PGX_LONG: {  // Integer.parseInt / Long.parseLong: optional sign, digits only
      const char* s = raw.c_str();
      char* end = nullptr;
      errno = 0;
      const long long v = std::strtoll(s, &end, 10);
      const bool ok = !raw.empty() && *end == '\0' && errno == 0 && !std::isspace((unsigned char)raw[0]) &&
                      (c.data_type == PGX_LONG || (v >= INT32_MIN && v <= INT32_MAX));
      if (!ok) fail(PGX_ERR_INVALID_ARG, "NumberFormatException: For input string: \"" + raw + "\"");
      return search([&](int i) { return c.ivals[i] < v; }, [&](int i) { return c.ivals[i] == v; });
    }
    case PGX_FLOAT:
    case PGX_DOUBLE: {  // Float.parseFloat / Double.parseDouble: surrounding whitespace and a trailing f/F/d/D allowed
      std::string t = trim_ws(raw);
      if (!t.empty() && std::strchr("fFdD", t.back())) t.pop_back();
      char* end = nullptr;
      const double d = c.data_type == PGX_FLOAT ? double(std::strtof(t.c_str(), &end)) : std::strtod(t.c_str(), &end);
      if (t.empty() || *end != '\0') fail(PGX_ERR_INVALID_ARG, "NumberFormatException: For input string: \"" + raw + "\"");
      return search([&](int i) { return c.dvals[i] < d; }, [&](int i) { return c.dvals[i] == d; });
    }
    default: {  // StringDictionary.indexOf: pad the lookup to the entry width unless it is at least that long
      const size_t w = size_t(c.dict_width);
      const char pad = char(c.pad_char);
      const std::string key = raw.size() >= w ? raw : raw + std::string(w - raw.size(), pad);
      auto entry = [&](int i) {
        const std::string& v = c.svals[i];
        return v.size() >= w ? v : v + std::string(w - v.size(), pad);
      };
      return search([&](int i) { return entry(i) < key; }, [&](int i) { return entry(i) == key; });
    }
  }
}

void resolve_binding(const StagedColumn& c, int kind, const pgx_predicate& p, int32_t& lo, int32_t& hi,
                     std::vector<uint32_t>& words) {
  const int card = c.card;
  auto val = [&](int i) { return std::string(p.values[i] ? p.values[i] : ""); };
  words.clear();
  lo = 0;
  hi = -1;
  if (kind == PGX_PRED_RANGE) {  // RangeOfflineDictionaryPredicateEvaluator.java:30-65
    if (p.num_values != 2) fail(PGX_ERR_INVALID_ARG, "RANGE needs (lower, upper)");
    const std::string a = val(0), b = val(1);
    int start = a == "*" ? 0 : dict_index_of(c, a);
    int end = b == "*" ? card - 1 : dict_index_of(c, b);
    if (start < 0) start = -(start + 1);
    else if (!p.lower_inclusive && a != "*") start += 1;
    if (end < 0) end = -(end + 1) - 1;
    else if (!p.upper_inclusive && b != "*") end -= 1;
    if (end >= start) {
      lo = start;
      hi = end;
    }
    return;
  }
  if (kind == PGX_PRED_EQ) {  // EqualsPredicateEvaluator.java:28-42
    if (p.num_values < 1) fail(PGX_ERR_INVALID_ARG, "EQ needs a value");
    const int i = dict_index_of(c, val(0));
    if (i >= 0) lo = hi = i;
    return;
  }
  std::vector<uint8_t> m(card, kind == PGX_PRED_IN ? 0 : 1);  // In / NotIn / NotEquals evaluators
  for (int k = 0; k < p.num_values; ++k) {
    const int i = dict_index_of(c, val(k));
    if (i >= 0) m[i] = kind == PGX_PRED_IN ? 1 : 0;
  }
  int first = -1, last = -1, cnt = 0;
  for (int i = 0; i < card; ++i)
    if (m[i]) {
      if (first < 0) first = i;
      last = i;
      ++cnt;
    }
  if (cnt == 0) return;
  if (last - first + 1 == cnt) {
    lo = first;
    hi = last;
    return;
  }
  words.assign((card + 31) / 32, 0u);
  for (int i = 0; i < card; ++i)
    if (m[i]) words[i >> 5] |= 1u << (i & 31);
}


// PGX_HOST_PROFILE=1: sub-phase marks of the planner (appended to the running pgx_execute's profile line).

void prof_mark(const char* what) {
  if (g_prof_mark) g_prof_mark(what);
}

void canon_rprog(std::vector<int>& op, std::vector<int>& arg);


void plan_query(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
                uint32_t xflags, ExecPlan& P, const Domain* dom) {
  if (n < 1) fail(PGX_ERR_INVALID_ARG, "no segments");
  if (q.agg_fn.size() > size_t(kMaxAggs)) fail(PGX_ERR_UNSUPPORTED, "too many aggregation functions");
  if (q.group_cols.size() > size_t(kMaxGroupCols)) fail(PGX_ERR_UNSUPPORTED, "too many group-by columns");
  if (q.leaf_col.size() > size_t(kMaxLeaves)) fail(PGX_ERR_UNSUPPORTED, "too many filter leaves");
  P.kn = q.kn;
  KQuery& K = P.kq;
  // query column slots
  for (size_t l = 0; l < q.leaf_col.size(); ++l) K.leaf_col[l] = int8_t(qslot(P, q.leaf_col[l]));
  K.num_aggs = int(q.agg_fn.size());
  K.num_planes = K.num_aggs + 1;
  K.plane_op[0] = P_ADD_I64;
  std::vector<std::string> proj;
  for (int a = 0; a < K.num_aggs; ++a) {
    const int fn = q.agg_fn[a];
    K.agg_kind[a] = int8_t(fn);
    if (fn == PGX_COUNT) {
      K.agg_col[a] = -1;
      K.agg_fp[a] = 0;
      K.plane_op[a + 1] = P_ADD_I64;
      continue;
    }
    const StagedColumn& c = segs[0]->col(q.agg_col[a]);
    if (c.data_type == PGX_STRING) fail(PGX_ERR_UNSUPPORTED, "numeric aggregation on STRING column " + c.name);
    if (fn >= PGX_COUNTMV) fail(PGX_ERR_INTERNAL, "multi-value function in the single-value plan");
    for (int s = 0; s < n; ++s)
      if (segs[s]->col(q.agg_col[a]).is_mv)
        fail(PGX_ERR_UNSUPPORTED, "single-value aggregation on multi-value column " + c.name);
    const bool fp = c.data_type == PGX_FLOAT || c.data_type == PGX_DOUBLE;
    K.agg_col[a] = int8_t(qslot(P, q.agg_col[a]));
    K.agg_fp[a] = fp;
    K.plane_op[a + 1] = (fn == PGX_MIN) ? P_MIN_ORD : (fn == PGX_MAX) ? P_MAX_ORD : (fp ? P_ADD_F64 : P_ADD_I64);
    if (std::find(proj.begin(), proj.end(), q.agg_col[a]) == proj.end()) proj.push_back(q.agg_col[a]);
  }
  for (const auto& g : q.group_cols)
    if (std::find(proj.begin(), proj.end(), g) == proj.end()) proj.push_back(g);
  P.n_proj = int(proj.size());

  // group-by key space
  K.num_gcols = int(q.group_cols.size());
  K.group_mode = G_NONE;
  if (K.num_gcols) {
    uint64_t prod = 1;
    bool overflow = false;
    int total_bits = 0;
    P.gdicts.clear();
    for (int g = 0; g < K.num_gcols; ++g) {
      for (int s = 0; s < n; ++s)
        if (segs[s]->col(q.group_cols[g]).is_mv)
          fail(PGX_ERR_UNSUPPORTED, "GROUP BY on multi-value column " + q.group_cols[g]);
      K.gcol[g] = int8_t(qslot(P, q.group_cols[g]));
      P.gdicts.push_back(dom ? domain_dict(*dom, g, n) : group_dict(q, segs, n, g));
      const int64_t gc = P.gdicts.back().card;
      if (!overflow && prod > (uint64_t(1) << 62) / uint64_t(gc)) overflow = true;
      if (!overflow) prod *= uint64_t(gc);
      P.gbits.push_back(bits_for(gc));
      total_bits += P.gbits.back();
    }
    P.mode_ref = reference_mode(q, segs[0]);
    const uint64_t kDenseMax = uint64_t(1) << 22;
    if (!overflow && prod <= kDenseMax && !(xflags & PGX_X_FORCE_HASH)) {
      uint64_t mul = 1;
      for (int g = 0; g < K.num_gcols; ++g) {  // column 0 least significant (DefaultGroupKeyGenerator.java:230-237)
        K.gmul[g] = mul;
        mul *= uint64_t(P.gdicts[g].card);
      }
      P.dense_slots = prod;
      const size_t lds = size_t(prod) * K.num_planes * 8;
      K.group_mode = (lds <= 48 * 1024) ? G_DENSE_LDS : G_DENSE_GLOBAL;
      if (K.group_mode == G_DENSE_LDS) P.lds_bytes = lds;
    } else {
      // LONG_MAP / ARRAY_MAP keys: the columns' id fields packed into 64-bit words, a field never straddling two
      // words (63 bits per word).  Wider than two words (DefaultGroupKeyGenerator.java:168-173: ARRAY_MAP takes any
      // key width): up to kMaxKeyWords words on the generic kernel (G_HASHW).
      int sh = 0, w = 0;
      for (int g = 0; g < K.num_gcols; ++g) {
        if (sh + P.gbits[g] > 63) {
          ++w;
          sh = 0;
        }
        K.gshift[g] = sh;
        K.ghi[g] = w;
        sh += P.gbits[g];
      }
      if (w + 1 > kMaxKeyWords) fail(PGX_ERR_UNSUPPORTED, "group key wider than 252 bits");
      K.key_words = w + 1;
      K.group_mode = w == 0 ? G_HASH64 : (w == 1 ? G_HASH128 : G_HASHW);
    }
  }
  K.num_qcols = int(P.qcols.size());
  prof_mark("p.keys");

  // Partitioned group-by: sparse 64-bit keys go through record-emitting query kernels, radix partitioning and LDS
  // aggregation (run_partitioned / run_narrow) instead of one global hash table.  Eligible when every non-COUNT function
  // reads an INT/LONG column (at most kPartMaxValueCols of them: one pipeline run per column, the passes' groups joined
  // by key) whose values span at most 32 bits, and key + value offset fit 63 bits.
  P.use_part = false;
  P.part_slab = P.part_dictid = P.part_narrow = false;
  P.part_hi = nullptr;
  P.part_cols.clear();
  if (K.group_mode == G_HASH64 && q.kn.jit && !(xflags & PGX_X_NO_PARTITION) &&
      K.num_qcols <= PGX_J_MAX_COLS) {
    std::vector<int> vcols;
    bool ok = true;
    for (int a = 0; a < K.num_aggs && ok; ++a) {
      if (K.agg_kind[a] == A_COUNT) continue;
      if (std::find(vcols.begin(), vcols.end(), K.agg_col[a]) == vcols.end()) vcols.push_back(K.agg_col[a]);
    }
    if (int(vcols.size()) > kPartMaxValueCols) ok = false;
    int keybits = 0;
    for (int g = 0; g < K.num_gcols; ++g) keybits = std::max(keybits, K.gshift[g] + P.gbits[g]);
    // one value column's settings into P (part_vcol ... narrow_vrange); false if the column does not qualify
    // narrow record widths (pgx_narrow.hip): the scan's records hold rb1 = keybits - 8 key bits + a vd-bit value field
    // (<= 48 bits); the second split's k2 bits leave rb1 - k2 key bits beside the field in 32 (or, wide, 64) bits
    const int rb1 = keybits - kNarrow1Bits;
    auto fits = [&](int vd, int& k2) {
      k2 = std::max(0, rb1 + vd - 32);
      if (rb1 - k2 > 31) k2 = rb1 - 31;
      return rb1 + vd <= 48 && k2 <= kNarrowMaxBits2;
    };
    auto fits_wide = [&](int vd, int& k2) {
      k2 = std::max(0, rb1 - 31);
      return rb1 + vd <= 48 && vd <= 32 && k2 <= kNarrowMaxBits2;
    };
    // narrow records whose value field indexes a table of the query's distinct dictionaries in global memory (IMG 5:
    // value - vbase as u32, IMG 6: doubles), gathered by the aggregation: per-segment dictionaries too large for the
    // scan's LDS beside its rings
    auto narrow_gather = [&](int img, int vd, const void* table, uint64_t entries) -> bool {
      if (!q.kn.narrow || keybits <= kNarrow1Bits) return false;
      int k2 = 0;
      bool wide = false;
      if (!fits(vd, k2)) {
        if (!fits_wide(vd, k2)) return false;
        wide = true;
      }
      P.part_narrow = true;
      P.part_slab = true;
      P.part_dictid = true;  // the scan emits dictId + the segment's place in the table (JSeg.emit_rebase)
      P.narrow_vd = vd;
      P.narrow_k2min = k2;
      P.narrow_img = img;
      P.narrow_wide = wide;
      P.narrow_imgp = static_cast<const uint32_t*>(table);
      P.narrow_img_words = int(std::min<uint64_t>(entries, 0x7FFFFFFF));
      P.narrow_img_sh = 0;
      return true;
    };
    auto config = [&](int vc) -> bool {
      P.part_slab = P.part_dictid = P.part_narrow = P.part_fp = false;
      P.narrow_img = 0;
      P.narrow_wide = false;
      P.part_fdict = nullptr;
      P.part_fbase.clear();
      bool need_sum = false, need_min = false, need_max = false;
      for (int a = 0; a < K.num_aggs; ++a) {
        if (K.agg_kind[a] == A_COUNT || K.agg_col[a] != vc) continue;
        need_sum |= K.agg_kind[a] == A_SUM || K.agg_kind[a] == A_AVG;
        need_min |= K.agg_kind[a] == A_MIN;
        need_max |= K.agg_kind[a] == A_MAX;
      }
      if (vc >= 0) {
        const StagedColumn& c0 = segs[0]->col(P.qcols[vc]);
        if (c0.data_type == PGX_FLOAT || c0.data_type == PGX_DOUBLE) {
          // FLOAT / DOUBLE: the records carry the value's index in the concatenation of the segments' dictionaries
          // (segments holding the same dictionary share one copy), 8-byte radix records, f64 aggregation
          // a dictionary is shared only when its values equal an earlier segment's (the hash picks the candidate);
          // the concatenation is sized before it is built, within the partition buffers' budget
          std::vector<double> all;
          std::vector<int64_t> fbase(size_t(n), 0);
          std::unordered_multimap<uint64_t, int> seen;  // dictionary hash -> first segment holding those values
          std::vector<int> first_of(size_t(n), -1);
          uint64_t total = 0;
          for (int s = 0; s < n; ++s) {
            const StagedColumn& c = segs[s]->col(P.qcols[vc]);
            if (c.data_type != c0.data_type || c.dvals.empty() || int64_t(c.dvals.size()) != int64_t(c.card)) return false;
            const uint64_t dk = c.dict_hash ^ (uint64_t(c.card) << 40);
            auto range = seen.equal_range(dk);
            for (auto it = range.first; it != range.second && first_of[size_t(s)] < 0; ++it) {
              const StagedColumn& o = segs[it->second]->col(P.qcols[vc]);
              if (o.dvals.size() == c.dvals.size() &&
                  std::memcmp(o.dvals.data(), c.dvals.data(), c.dvals.size() * sizeof(double)) == 0)
                first_of[size_t(s)] = it->second;
            }
            if (first_of[size_t(s)] >= 0) continue;
            first_of[size_t(s)] = s;
            seen.emplace(dk, s);
            total += c.dvals.size();
            if (total > (uint64_t(1) << 31) || total * 8 > kPartMaxBytes) return false;
          }
          all.reserve(size_t(total));
          for (int s = 0; s < n; ++s) {
            if (first_of[size_t(s)] != s) {
              fbase[size_t(s)] = fbase[size_t(first_of[size_t(s)])];
              continue;
            }
            const StagedColumn& c = segs[s]->col(P.qcols[vc]);
            fbase[size_t(s)] = int64_t(all.size());
            all.insert(all.end(), c.dvals.begin(), c.dvals.end());
          }
          const int vbits = bits_for(int64_t(all.size()));
          if (keybits + vbits > 63 || all.size() > (size_t(1) << 31)) return false;
          DevBuf buf(ctx, all.size() * 8);
          hip_check(hipMemcpy(buf.p, all.data(), all.size() * 8, hipMemcpyHostToDevice), "value dictionaries H2D");
          P.part_fp = true;
          P.part_fdict = buf.as<double>();
          P.part_fbase = std::move(fbase);
          P.part_fdict_bufs.push_back(std::move(buf));
          P.part_vcol = vc;
          P.part_keybits = keybits;
          P.part_vbits = vbits;
          P.part_vbase = 0;
          P.part_sum = need_sum;
          P.part_min = need_min;
          P.part_max = need_max;
          P.part_dictid = true;  // (the index, rebased per segment: JSeg.emit_rebase)
          P.part_vdict = nullptr;
          P.narrow_vrange = 0;
          narrow_gather(6, vbits, P.part_fdict, all.size());  // narrow records when they fit, else the radix path
          return true;
        }
      }
      bool cok = true;
      int vbits = 0;
      int64_t vbase = 0;
      uint64_t vrange = 0;
      bool same_dict = true;  // one dictionary in every segment: records may carry the dictId (narrow path)
      if (vc >= 0) {
        // Value records carry value - vbase with ONE query-wide vbase (the smallest value of any segment's
        // dictionary): each segment's records are rebased by (its image base - vbase) in the scan (JSeg.emit_rebase),
        // so segments with their own dictionaries (SegmentDictionaryCreator builds one per segment) share the path.
        const StagedColumn& c0 = segs[0]->col(P.qcols[vc]);
        int64_t vmin = 0, vmax = 0;
        for (int s = 0; s < n && cok; ++s) {
          const StagedColumn& c = segs[s]->col(P.qcols[vc]);
          cok = (c.data_type == PGX_INT || c.data_type == PGX_LONG) && !c.ivals.empty() && c.data_type == c0.data_type;
          if (!cok) break;
          const int64_t lo = *std::min_element(c.ivals.begin(), c.ivals.end());
          const int64_t hi = *std::max_element(c.ivals.begin(), c.ivals.end());
          vmin = s ? std::min(vmin, lo) : lo;
          vmax = s ? std::max(vmax, hi) : hi;
          same_dict = same_dict && c.dict_hash == c0.dict_hash && c.card == c0.card;
        }
        if (cok) {
          const uint64_t range = uint64_t(vmax) - uint64_t(vmin);
          cok = range <= 0xFFFFFFFFull;
          vbase = vmin;
          vrange = range;
          vbits = cok ? bits_for(int64_t(range) + 1) : 64;
        }
      }
      // The 8-byte radix path's records carry value offsets (round 3's dictId records with a fused first pass or
      // per-workgroup slabs measured slower at C3 and were removed in round 5)
      if (!cok || keybits + vbits > 63) return false;
      P.part_vcol = vc;
      P.part_keybits = keybits;
      P.part_vbits = vbits;
      P.part_vbase = vbase;
      P.part_sum = need_sum;
      P.part_min = need_min;
      P.part_max = need_max;
      P.part_vdict = nullptr;
      // Narrow records (default; PGX_PART_NARROW=0 keeps the 8-byte radix path): the value's dictId rides in a record of
      // keybits - 8 + dictId bits (<= 48) out of the scan's own 256-way split, then <= 32 bits after the second split,
      // and the aggregation looks values up in the column's image (FOR16 / U32) in LDS (run_narrow).  Needs a sorted
      // dictionary (MIN / MAX of dictIds) and, for SUM / AVG, an image that fits beside the aggregation tables.
      if (q.kn.narrow && keybits > kNarrow1Bits) {
        // Value field: the dictId looked up in an LDS image of the column (one sorted dictionary in every segment, an
        // image that fits the LDS), or the value offset itself (value - vbase, rebased per segment like the radix
        // records: per-segment dictionaries, no image, and no LDS spent on one -- PGX_PART_NARROW=direct prefers it)
        // (value offsets too wide for a 32-bit second-stage record take 64-bit ones: fits_wide)
        int vd = 0, imgk = 0, k2 = 0;
        bool nok = true, wide = false;
        if (vc >= 0) {
          const StagedColumn& c0 = segs[0]->col(P.qcols[vc]);
          nok = same_dict && c0.dict_dev != nullptr && std::is_sorted(c0.ivals.begin(), c0.ivals.end());
          vd = bits_for(c0.card);
          if (c0.img_dev && c0.img_kind == IMG_FOR16 && c0.img_words <= kImgFor16Blocks + 32768) imgk = 2;
          else if (c0.img_dev && c0.img_kind == IMG_U32 && c0.img_words <= kImgFor16Blocks + 32768) imgk = 1;
          if (need_sum && !imgk) nok = false;
          nok = nok && fits(vd, k2);
          int k2d = 0;
          const bool direct = vbits <= 32 && fits(vbits, k2d);
          // value-offset records are made in the scan, from the column's LDS image beside the scan's record rings
          // (256 buckets x kNarrowRing records x 6 B): a per-segment image larger than the rest of the LDS (c3d's
          // 128 KiB FOR16 images) keeps the 8-byte radix path
          int64_t scan_img = 0;
          for (int s = 0; s < n; ++s) {
            const StagedColumn& c = segs[s]->col(P.qcols[vc]);
            if (c.img_kind != IMG_NONE) scan_img = std::max<int64_t>(scan_img, int64_t(c.img_words) * 4);
          }
          const bool scan_fits =
              scan_img + (int64_t(1) << kNarrow1Bits) * (2 * q.kn.narrow_unit) * 6 + 16 * 1024 <= 160 * 1024;
          if (q.kn.narrow_gather) nok = false;
          if (!q.kn.narrow_gather && (!nok || q.kn.narrow_direct) && scan_fits &&
              (direct || (vbits <= 32 && fits_wide(vbits, k2d)))) {
            wide = !direct;
            nok = true;
            imgk = 3;
            vd = vbits;
            k2 = k2d;
            P.narrow_imgp = nullptr;
            P.narrow_img_words = 0;
            P.narrow_img_sh = 0;
            P.narrow_vrange = vrange;
          } else if (nok) {
            P.part_vdict = static_cast<const int64_t*>(c0.dict_dev);
            P.narrow_imgp = imgk ? static_cast<const uint32_t*>(c0.img_dev) : nullptr;
            P.narrow_img_words = imgk ? c0.img_words : 0;
            P.narrow_img_sh = c0.img_sh;
            P.narrow_vrange = c0.vrange;
            // the packed image, when it fits beside sixteen tables: 1024-thread aggregation workgroups (IMG 4)
            if (imgk && c0.shared && packed_value_image(ctx, *c0.shared, c0.ivals)) {
              imgk = 4;
              P.narrow_imgp = c0.shared->pk_img.as<uint32_t>();
              P.narrow_img_words = c0.shared->pk_words;
              P.narrow_img_sh = c0.shared->pk_sh;
            }
          } else if (vbits <= 32 && q.kn.narrow_gather) {
            // (measured at c3d: 13.98 ms per step against 13.83 on the 8-byte radix path, whose records carry the value
            // offsets the scan makes from each segment's image -- so the gather is the tests' option, not the default)
            // per-segment dictionaries whose value offsets the scan cannot make (no room for the image beside its
            // rings): the records carry the dictId's index in a u32 table of every distinct dictionary's value - vbase
            // (IMG 5), gathered by the aggregation from L2
            std::vector<uint32_t> all;
            std::vector<int64_t> fbase(size_t(n), 0);
            std::unordered_multimap<uint64_t, int> seen;
            std::vector<int> first_of(size_t(n), -1);
            uint64_t total = 0;
            bool tok = true;
            for (int s = 0; s < n && tok; ++s) {
              const StagedColumn& c = segs[s]->col(P.qcols[vc]);
              if (int64_t(c.ivals.size()) != int64_t(c.card)) tok = false;
              const uint64_t dk = c.dict_hash ^ (uint64_t(c.card) << 40);
              auto range = seen.equal_range(dk);
              for (auto it = range.first; it != range.second && first_of[size_t(s)] < 0; ++it)
                if (segs[it->second]->col(P.qcols[vc]).ivals == c.ivals) first_of[size_t(s)] = it->second;
              if (first_of[size_t(s)] >= 0) continue;
              first_of[size_t(s)] = s;
              seen.emplace(dk, s);
              total += c.ivals.size();
              if (total > (uint64_t(1) << 31) || total * 4 > kPartMaxBytes / 8) tok = false;
            }
            if (tok && total > 0) {
              all.reserve(size_t(total));
              for (int s = 0; s < n; ++s) {
                if (first_of[size_t(s)] != s) {
                  fbase[size_t(s)] = fbase[size_t(first_of[size_t(s)])];
                  continue;
                }
                fbase[size_t(s)] = int64_t(all.size());
                for (int64_t v : segs[s]->col(P.qcols[vc]).ivals) all.push_back(uint32_t(uint64_t(v) - uint64_t(vbase)));
              }
              DevBuf buf(ctx, all.size() * 4);
              hip_check(hipMemcpy(buf.p, all.data(), all.size() * 4, hipMemcpyHostToDevice), "value table H2D");
              if (narrow_gather(5, bits_for(int64_t(all.size())), buf.p, all.size())) {
                P.narrow_vrange = vrange;
                P.part_fbase = std::move(fbase);
                P.part_fdict_bufs.push_back(std::move(buf));
                return true;
              }
            }
          }
        } else {
          nok = fits(0, k2);
        }
        if (nok) {
          P.part_narrow = true;
          P.part_slab = true;
          P.part_dictid = vc >= 0 && imgk != 3;
          P.narrow_vd = vd;
          P.narrow_k2min = k2;
          P.narrow_img = imgk;
          P.narrow_wide = wide;
        }
      }
      return true;
    };
    if (vcols.empty()) vcols.push_back(-1);  // COUNT only
    for (size_t i = 0; i < vcols.size() && ok; ++i) {
      ok = config(vcols[i]);
      if (ok) P.part_cols.push_back(P.save_part_col());
    }
    if (ok) {
      P.use_part = true;
      P.load_part_col(P.part_cols[0]);
    } else {
      P.part_cols.clear();
      P.part_slab = P.part_dictid = P.part_narrow = P.part_fp = false;
    }
  }

  // filter program
  P.host_entries = 0;
  int host_scan_leaves = 0;
  std::vector<int8_t> pop, parg;
  PNode froot;
  P.fsm_on = false;
  P.rprog_on = false;
  P.dm_progs.clear();
  P.use_docmask = q.kn.jit && (K.group_mode == G_NONE || K.group_mode == G_DENSE_LDS ||
                                K.group_mode == G_DENSE_GLOBAL || K.group_mode == G_HASH64 ||
                                K.group_mode == G_HASH128 || P.use_part) && K.num_qcols <= PGX_J_MAX_COLS;
  // (G_HASHW keys stay on the generic kernel: the generated kernels hold two key words)
  if (!q.filter.empty()) {
    PNode root = build_tree(q, *segs[0]);
    const size_t L = q.leaf_col.size();
    bool fuse = P.use_docmask && stats_closed_form(root, q, segs, n, bindings) && q.kn.rprog != RPROG_OFF;
    for (int s = 0; s < n && fuse; ++s) {
      if (star_fit(q, *segs[s])) fuse = false;
      for (size_t l = 0; l < L && fuse; ++l) {
        const StagedColumn& c = segs[s]->col(q.leaf_col[l]);
        const bool bitmap = c.has_inverted && !c.is_sorted && q.leaf_kind[l] != PGX_PRED_RANGE;
        if (bitmap != (!segs[0]->col(q.leaf_col[l]).is_sorted && segs[0]->col(q.leaf_col[l]).has_inverted &&
                       q.leaf_kind[l] != PGX_PRED_RANGE))
          fuse = false;  // index kinds differ across segments
        else if (bitmap && !c.inv_dev.p && !binding_empty(bindings[size_t(s) * L + l], c.card))
          fuse = false;
      }
    }
    prof_mark("p.fusechk");
    FusePlan F;
    if (fuse) {
      plan_fuse(root, q, F);
      if (F.progs.empty() || L + F.progs.size() > size_t(PGX_J_MAX_LEAVES)) fuse = false;
      for (const auto& p : F.progs)
        if (prog_depth(p) > 4 || p.op.size() > size_t(kMaxRProg)) fuse = false;
    }
    if (fuse) {
      emit_fused(root, F, int(L), pop, parg, true, host_scan_leaves);
      P.rprog_on = true;
      P.dm_progs = F.progs;
      for (auto& p : P.dm_progs) canon_rprog(p.op, p.arg);
    } else {
      emit(root, pop, parg, true, false, host_scan_leaves);
    }
    if (!stats_closed_form(root, q, segs, n, bindings)) {
      // the automaton counts every entry: no OP_STAT popcounts, no whole-range host terms
      P.fsm_on = true;
      host_scan_leaves = 0;
      std::vector<int8_t> o2, a2;
      for (size_t i = 0; i < pop.size(); ++i)
        if (pop[i] != OP_STAT) {
          o2.push_back(pop[i]);
          a2.push_back(parg[i]);
        }
      pop.swap(o2);
      parg.swap(a2);
      froot = root;
    }
    P.leaf_phys.assign(q.leaf_col.size(), PH_SCAN);
    std::vector<const PNode*> todo{&root};
    while (!todo.empty()) {
      const PNode* x = todo.back();
      todo.pop_back();
      if (x->op == PGX_F_LEAF) P.leaf_phys[x->leaf] = x->phys;
      for (const PNode& k : x->kids) todo.push_back(&k);
    }
  }
  P.roar.clear();
  P.roar_index.assign(n, std::vector<int>(q.leaf_col.size(), -1));
  P.mask_words = 0;
  P.roar_maxchunks = 0;
  if (pop.size() > size_t(kMaxProg)) fail(PGX_ERR_UNSUPPORTED, "filter program too long");
  K.prog_len = int(pop.size());
  for (size_t i = 0; i < pop.size(); ++i) {
    K.prog_op[i] = pop[i];
    K.prog_arg[i] = parg[i];
  }

  prof_mark("p.head");
  // per-segment descriptors: planned in chunks of segments (in parallel for long segment lists); each chunk keeps its
  // blob words, pointer fixups and bitmap items with chunk-local offsets, concatenated in segment order afterwards.
  P.ksegs.assign(n, KSeg{});
  P.segcols.assign(n, {});
  P.sorted_span.assign(size_t(n) * q.leaf_col.size(), 0);
  // Per distinct (leaf, binding, cardinality) in a chunk: the leaf mode, ONE blob copy of its dictId bitset and ONE list
  // of the dictIds whose bitmaps a bitmap leaf ORs.  Segments sharing a dictionary share their bindings
  // (pgx_bind_predicates), so a chunk usually resolves each leaf once, whatever its segment count.
  struct LeafMemo {
    int8_t mode = LEAF_NONE;
    int64_t bits_off = -1;  // chunk blob offset of the bitset copy (LEAF_SCAN_BITSET)
    int64_t ids_off = -1;   // chunk blob offset of the dictId list (bitmap leaves), nb entries
    int nb = 0;
  };
  // keyed by whether the leaf reads the inverted index: a scan-only segment's entry carries no dictId list
  using LeafKey = std::tuple<size_t, const uint32_t*, int32_t, int32_t, int, bool>;
  struct ChunkOut {
    std::vector<int32_t> blob;
    std::map<const std::vector<int32_t>*, size_t> remap_off;
    std::map<LeafKey, LeafMemo> leaf_memo;
    std::vector<ExecPlan::Fix> fixes;
    std::vector<ExecPlan::RoarItem> roar;
    std::vector<ExecPlan::MvItem> mv;
    int64_t total_raw = 0, host_entries = 0;
    uint64_t mask_words = 0;
    int maxchunks = 0;
  };
  const int kSegsPerChunk = 64;
  const int nchunk = (n + kSegsPerChunk - 1) / kSegsPerChunk;
  std::vector<ChunkOut> chunks(nchunk);
  auto plan_chunk = [&](int ci) {
    ChunkOut& o = chunks[ci];
    for (int s = ci * kSegsPerChunk; s < std::min(n, (ci + 1) * kSegsPerChunk); ++s) {
      const pgx_segment& seg = *segs[s];
      KSeg& S = P.ksegs[s];
      S.num_docs = seg.total_raw_docs;  // MatchEntireSegment / FilterPlanNode scan range [0, totalRawDocs)
      S.num_tiles = int32_t((int64_t(S.num_docs) + kTileRows - 1) / kTileRows);
      o.total_raw += seg.total_raw_docs;
      o.host_entries += int64_t(host_scan_leaves) * seg.total_raw_docs;
      auto& segcols = P.segcols[s];
      segcols.resize(P.qcols.size());
      for (size_t c = 0; c < P.qcols.size(); ++c) {
        const StagedColumn& col = seg.col(P.qcols[c]);
        segcols[c] = &col;
        S.fwd[c] = col.fwd;
        S.bits[c] = int8_t(col.bits);
        S.dict[c] = col.dict_dev;
        S.remap[c] = nullptr;
      }
      for (int g = 0; g < K.num_gcols; ++g) {
        if (!P.gdicts[g].identity) {
          const std::vector<int32_t>* rm = P.gdicts[g].remap[s].get();
          auto it = o.remap_off.find(rm);  // one blob copy per distinct dictionary in this chunk
          if (it == o.remap_off.end()) {
            it = o.remap_off.emplace(rm, o.blob.size()).first;
            o.blob.insert(o.blob.end(), rm->begin(), rm->end());
          }
          o.fixes.push_back({size_t(s), 0, K.gcol[g], it->second});
        }
      }
      // leaves
      for (size_t l = 0; l < q.leaf_col.size(); ++l) {
        const StagedColumn& col = *segcols[K.leaf_col[l]];
        const pgx_leaf_binding& b = bindings[size_t(s) * q.leaf_col.size() + l];
        KLeaf& L = S.leaf[l];
        L.lo = b.lo;
        L.hi = b.hi;
        L.bitset = nullptr;
        L.ranges = nullptr;
        L.nranges = 0;
        // matching dictIds
        auto matches = [&](int id) -> bool {
          if (b.words) return (b.words[id >> 5] >> (id & 31)) & 1u;
          return id >= b.lo && id <= b.hi;
        };
        const bool bitmap_leaf = P.use_docmask && P.leaf_phys[l] == PH_BITMAP && col.inv_dev.p;
        if (col.is_sorted) {
          // SortedInvertedIndexBasedFilterOperator (additive ranges, merged), clipped to [0, totalRawDocs-1]
          std::vector<int32_t> r;
          for (int id = 0; id < col.card; ++id) {
            if (!matches(id)) continue;
            int32_t a = std::max(col.sorted_first[id], 0);
            int32_t e = std::min(col.sorted_last[id], seg.total_raw_docs - 1);
            if (e < a) continue;
            if (!r.empty() && a <= r.back() + 1) r.back() = std::max(r.back(), e);
            else { r.push_back(a); r.push_back(e); }
          }
          if (r.empty()) { L.mode = LEAF_NONE; continue; }
          P.sorted_span[size_t(s) * q.leaf_col.size() + l] = (int64_t(r.front()) << 32) | int64_t(uint32_t(r.back()));
          L.mode = LEAF_RANGES;
          L.nranges = int32_t(r.size() / 2);
          o.fixes.push_back({size_t(s), 1, int(l), o.blob.size()});
          o.blob.insert(o.blob.end(), r.begin(), r.end());
          continue;
        }
        const bool neg = q.leaf_kind[l] == PGX_PRED_NEQ || q.leaf_kind[l] == PGX_PRED_NOT_IN;
        auto mit = o.leaf_memo.find(LeafKey(l, b.words, b.lo, b.hi, col.card, bitmap_leaf));
        if (mit == o.leaf_memo.end()) {
          LeafMemo m;
          if (b.words) {
            bool any = false;
            const int nw = (col.card + 31) / 32;
            for (int w = 0; w < nw && !any; ++w) any = b.words[w] != 0;
            if (any) {
              m.mode = LEAF_SCAN_BITSET;
              m.bits_off = int64_t(o.blob.size());
              for (int w = 0; w < nw; ++w) o.blob.push_back(int32_t(b.words[w]));
            }
          } else {
            m.mode = (b.hi < b.lo) ? LEAF_NONE : LEAF_SCAN_INTERVAL;
          }
          if (bitmap_leaf && m.mode != LEAF_NONE) {
            // BitmapBasedFilterOperator (operator/filter/BitmapBasedFilterOperator.java:62-92): OR the roaring bitmaps
            // of the matching dictIds; NEQ / NOT_IN OR the NON-matching ones and flip over the scanned doc range.  The
            // list holds dictIds: the device reads each bitmap's offset from the staged file's own header.
            m.ids_off = int64_t(o.blob.size());
            auto take = [&](int id) {
              o.blob.push_back(int32_t(id));
              ++m.nb;
            };
            if (b.words) {  // walk the set (or, negated, the clear) bits of the dictId bitset
              const int nw = (col.card + 31) / 32;
              for (int w = 0; w < nw; ++w) {
                uint32_t x = neg ? ~b.words[w] : b.words[w];
                if (w == nw - 1 && (col.card & 31)) x &= (1u << (col.card & 31)) - 1u;
                while (x) {
                  take(w * 32 + __builtin_ctz(x));
                  x &= x - 1u;
                }
              }
            } else if (!neg) {
              for (int id = std::max(0, b.lo); id <= std::min(b.hi, col.card - 1); ++id) take(id);
            } else {
              for (int id = 0; id < col.card; ++id)
                if (id < b.lo || id > b.hi) take(id);
            }
          }
          mit = o.leaf_memo.emplace(LeafKey(l, b.words, b.lo, b.hi, col.card, bitmap_leaf), m).first;
        }
        const LeafMemo& m = mit->second;
        L.mode = m.mode;
        if (m.mode == LEAF_NONE) continue;
        if (m.mode == LEAF_SCAN_BITSET) o.fixes.push_back({size_t(s), 2, int(l), size_t(m.bits_off)});
        if (bitmap_leaf) {
          ExecPlan::RoarItem it{s, int(l), neg, size_t(m.ids_off), m.nb, int((int64_t(seg.total_docs) + 65535) >> 16),
                                o.mask_words, col.inv_dev.p};
          if (s == 0) {  // serialized bytes of the ORed bitmaps: segment 0's selectivity estimate only
            const int32_t* ids = o.blob.data() + m.ids_off;
            for (int k = 0; k < m.nb; ++k) it.bytes += col.inv_off[ids[k] + 1] - col.inv_off[ids[k]];
          }
          if (!P.rprog_on) o.mask_words += uint64_t(it.nchunks) * 2048;
          o.maxchunks = std::max(o.maxchunks, it.nchunks);
          o.roar.push_back(it);
        } else if (col.is_mv && L.mode != LEAF_NONE) {
          // MVScanDocIdIterator: the query kernel reads the doc mask pgx_mv_leaf_mask derives from the values
          if (!P.use_docmask) fail(PGX_ERR_UNSUPPORTED, "multi-value filter needs the query kernels");
          o.mv.push_back({s, int(l)});
        }
      }
    }
  };
  if (nchunk > 1 && !P.serial) ctx->parallel_for(nchunk, plan_chunk);
  else
    for (int ci = 0; ci < nchunk; ++ci) plan_chunk(ci);
  P.mv_items.clear();
  P.mv_index.assign(n, std::vector<int>(q.leaf_col.size(), -1));
  P.mv_neg.assign(q.leaf_col.size(), 0);
  for (size_t l = 0; l < q.leaf_col.size(); ++l)
    P.mv_neg[l] = q.leaf_kind[l] == PGX_PRED_NEQ || q.leaf_kind[l] == PGX_PRED_NOT_IN;
  for (ChunkOut& o : chunks)
    for (const auto& it : o.mv) {
      P.mv_index[it.seg][it.leaf] = int(P.mv_items.size());
      P.mv_items.push_back(it);
    }
  int64_t tiles = 0;
  P.total_raw = 0;
  for (int s = 0; s < n; ++s) {
    P.ksegs[s].tile_begin = tiles;
    tiles += P.ksegs[s].num_tiles;
  }
  prof_mark("p.chunks");
  for (ChunkOut& o : chunks) {
    const size_t base = P.blob32.size();
    const uint64_t mbase = P.mask_words;
    P.blob32.insert(P.blob32.end(), o.blob.begin(), o.blob.end());
    for (auto f : o.fixes) {
      f.off += base;
      P.fixes.push_back(f);
    }
    for (auto it : o.roar) {
      it.blob_off += base;
      it.mask_off += mbase;
      P.roar_index[it.seg][it.leaf] = int(P.roar.size());
      P.roar.push_back(it);
    }
    P.mask_words += o.mask_words;
    P.roar_maxchunks = std::max(P.roar_maxchunks, o.maxchunks);
    P.total_raw += o.total_raw;
    P.host_entries += o.host_entries;
  }
  // Bitmap programs inside the query kernels (LEAF_RCHUNK) when the filter is selective: the kernel then needs no
  // value image (selected rows gather their values from the dictionary in HBM/L2), leaving LDS for the chunk masks and
  // several workgroups per CU.  Selectivity estimate: segment 0's leaves, 2 serialized bytes per doc (array
  // containers), AND / OR / NOT as independent events.  PGX_RCHUNK=0/1 forces the choice.
  P.rchunk = false;
  if (P.rprog_on && !P.use_part) {
    double est = 1.0;
    const double nd0 = std::max(1, segs[0]->total_raw_docs);
    for (const auto& dp : P.dm_progs) {
      std::vector<double> st;
      for (size_t i = 0; i < dp.op.size(); ++i) {
        if (dp.op[i] == RP_LEAF) {
          const int ri = P.roar_index[0][dp.arg[i]];
          double f = ri >= 0 ? std::min(1.0, double(P.roar[ri].bytes) / 2.0 / nd0) : 0.0;
          if (ri >= 0 && P.roar[ri].neg) f = 1.0 - f;
          st.push_back(f);
        } else if (dp.op[i] == RP_NOT) {
          st.back() = 1.0 - st.back();
        } else {
          const double b = st.back();
          st.pop_back();
          st.back() = dp.op[i] == RP_AND ? st.back() * b : st.back() + b - st.back() * b;
        }
      }
      if (!st.empty()) est = std::min(est, st.back());  // the programs are ANDed or ORed into the tree: a bound
    }
    P.rchunk = est <= kRchunkMaxSel;
    if (q.kn.rchunk >= 0) P.rchunk = q.kn.rchunk == 1;
    for (int s = 0; s < n && P.rchunk; ++s)
      if (star_fit(q, *segs[s])) P.rchunk = false;
  }
  // per (segment, bitmap program): the program over that segment's leaf descriptors and its output mask
  P.rprogs.clear();
  P.rp_kind = -1;
  if (P.rprog_on) {
    const size_t np = P.dm_progs.size();
    P.rprogs.resize(size_t(n) * np);
    for (int s = 0; s < n; ++s) {
      const int nchunks = int((int64_t(segs[s]->total_docs) + 65535) >> 16);
      P.roar_maxchunks = std::max(P.roar_maxchunks, nchunks);
      for (size_t k = 0; k < np; ++k) {
        const auto& dp = P.dm_progs[k];
        RProg& r = P.rprogs[size_t(s) * np + k];
        r = RProg{};
        r.nchunks = nchunks;
        r.num_docs = P.ksegs[s].num_docs;
        r.mask = reinterpret_cast<uint32_t*>(uintptr_t(P.mask_words));  // word offset until the buffer exists
        if (!P.rchunk) P.mask_words += uint64_t(nchunks) * 2048;
        int o = 0, nl = 0;
        for (size_t i = 0; i < dp.op.size(); ++i) {
          if (dp.op[i] == RP_LEAF) {
            const int ri = P.roar_index[s][dp.arg[i]];
            r.op[o] = RP_LEAF;
            r.arg[o++] = int16_t(ri);
            if (nl < PGX_J_MAX_RLEAVES) r.ldesc[nl] = int16_t(ri);
            ++nl;
            // a leaf without matching dictIds (alwaysFalse) is empty, negated or not
            if (ri < 0 && i + 1 < dp.op.size() && dp.op[i + 1] == RP_NOT) ++i;
          } else {
            r.op[o] = int8_t(dp.op[i]);
            r.arg[o++] = 0;
          }
        }
        r.nops = o;
      }
    }
  }
  prof_mark("p.merge");
  // star-tree segments (query kernels only: the per-segment program needs the generated kernels)
  P.star.assign(n, ExecPlan::StarPlan{});
  if (P.use_docmask && !P.use_part && int(q.leaf_col.size()) + 8 <= PGX_J_MAX_LEAVES) {
    tiles = 0;
    for (int s = 0; s < n; ++s) {
      KSeg& S = P.ksegs[s];
      if (star_fit(q, *segs[s])) {
        plan_star_segment(q, *segs[s], S, bindings + size_t(s) * q.leaf_col.size(), P.leaf_phys, P.blob32, P.star[s]);
        if (int(q.leaf_col.size() + P.star[s].ranges.size()) > PGX_J_MAX_LEAVES) {
          P.star[s] = ExecPlan::StarPlan{};
        } else {
          // StarTreeIndexOperator reaches aggregated docs: scan [0, totalDocs); no root scan leaf
          P.host_entries -= int64_t(host_scan_leaves) * segs[s]->total_raw_docs;
          S.num_docs = segs[s]->total_docs;
        }
      }
      S.tile_begin = tiles;
      S.num_tiles = int32_t((int64_t(S.num_docs) + kTileRows - 1) / kTileRows);
      tiles += S.num_tiles;
    }
  }
  K.total_tiles = tiles;
  K.num_segs = n;
  P.lmask_off.assign(n, -1);
  P.lmask_words.assign(n, 0);
  P.lmask_total = 0;
  P.fsm_segs.clear();
  P.fsm_chunks = 0;
  if (P.fsm_on) {
    const int L = int(q.leaf_col.size());
    std::vector<FsmSegInfo> infos;
    std::vector<int> fsegs;
    for (int s = 0; s < n; ++s) {
      if (!P.star.empty() && P.star[s].on) continue;  // star-tree plans count their own statistic
      FsmSegInfo si;
      si.num_docs = P.ksegs[s].num_docs;
      si.sorted_first.assign(L, 0);
      si.sorted_last.assign(L, 0);
      for (int l = 0; l < L; ++l) {
        const int64_t sp = P.sorted_span[size_t(s) * L + l];
        if (sp) {
          si.sorted_first[l] = sp >> 32;
          si.sorted_last[l] = int32_t(uint32_t(sp));
        }
        if (P.ksegs[s].leaf[l].mode == LEAF_NONE && P.leaf_phys[l] == PH_SCAN) si.always_false |= 1u << l;
      }
      infos.push_back(std::move(si));
      fsegs.push_back(s);
    }
    std::string err;
    if (!fsegs.empty() && !fsm_build(fsm_tree(froot), L, infos, P.fsm, &err)) fail(PGX_ERR_UNSUPPORTED, err);
    for (size_t i = 0; i < fsegs.size(); ++i) {
      const int s = fsegs[i];
      const int64_t nd = P.ksegs[s].num_docs;
      P.lmask_words[s] = (nd + 31) / 32 + 1;
      P.lmask_off[s] = int64_t(P.lmask_total);
      P.lmask_total += uint64_t(P.lmask_words[s]) * L;
      FsmSeg g{};
      g.words = P.lmask_words[s];
      g.num_docs = int32_t(nd);
      g.chunk0 = P.fsm_chunks;
      P.fsm_chunks += (nd + kFsmChunkRows - 1) / kFsmChunkRows;
      const auto& iv = P.fsm.seg_intervals[i];
      if (iv.size() > size_t(kFsmMaxIntervals)) fail(PGX_ERR_INTERNAL, "statistics automaton intervals");
      g.nint = int32_t(iv.size());
      for (size_t k = 0; k < iv.size(); ++k) {
        g.ibeg[k] = iv[k].first;
        g.itab[k] = iv[k].second;
      }
      P.fsm_segs.push_back(g);
    }
    if (P.fsm_segs.empty()) P.fsm_on = false;
  }
  P.rec_base.assign(n, 0);
  P.rec_total = 0;
  for (int s = 0; s < n; ++s) {
    P.rec_base[s] = P.rec_total;
    P.rec_total += P.ksegs[s].num_docs;
  }

  // grid: persistent, contiguous tile ranges per workgroup
  const int cus = ctx->num_cus;
  const int wgs_per_cu = (K.group_mode == G_NONE) ? 8 : 4;
  const int64_t max_grid = int64_t(cus) * wgs_per_cu;
  P.tiles_per_wg = std::max<int64_t>(1, (tiles + max_grid - 1) / max_grid);
  P.grid = int(std::max<int64_t>(1, (tiles + P.tiles_per_wg - 1) / P.tiles_per_wg));
}

// Per-query device arguments live in ONE arena, written on the host into pinned memory and sent with ONE copy:
//   [blob (ranges / bitsets / remaps) | KSeg x n | JSeg x n | outputs (agg planes, stats, overflow)]

}  // namespace pgxh
