// numEntriesScannedInFilter as a finite automaton over rows (ExecutionStatistics, core/operator/ExecutionStatistics.java).
//
// The reference counts entries inside its doc-id iterators: SVScanDocIdIterator.next/advance count every row they scan
// forward from a target to the next match (core/operator/dociditerators/SVScanDocIdIterator.java:82-118), applyAnd
// counts every candidate doc it tests (:131-149), and which targets a scan receives depends on the leapfrog of
// AndDocIdIterator (AndDocIdIterator.java:86-122) and on OrDocIdIterator's queue (OrDocIdIterator.java:52-97), driven by
// BReusableFilteredDocIdSetOperator calling next() on the root (BReusableFilteredDocIdSetOperator.java:68-85).
//
// Every iterator only moves forward and answers advance(t) with the next member >= t of its doc set.  Sweeping the
// rows in increasing order, each iterator is idle (current doc behind the row) or searching (its current doc will be
// at or past the row); a target reaching an idle iterator starts a search at that row, a target reaching a searching
// one is a no-op, and a scan leaf counts each row it searches.  So the statistic is a finite automaton over each row's
// leaf-membership bits plus the row's position against each leaf's [start, end] range; this file builds its transition
// tables on the host (one per distinct range-position vector), pgx_kernels.hip runs them over the leaf masks the query
// kernels wrote.  tests/stats_fsm_model.py restates the same sweep in Python and checks it against the oracle's literal
// iterator algebra on random filter trees.
#include <algorithm>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <vector>

#include "pgx_internal.h"

namespace pgx {

namespace {

enum FKind { F_SCAN, F_INDEX, F_ANS, F_OR, F_AND };

struct FNode {
  int kind = F_SCAN;
  int leaf = -1;             // F_SCAN / F_INDEX
  std::vector<int> kids;     // F_OR / F_AND (iterator order)
  std::vector<int> idx;      // F_ANS: sorted / bitmap leaves (raw, unclipped)
  std::vector<int> scans;    // F_ANS: applyAnd scan leaves, in order
  int mult = 1;              // F_ANS: how many times iterator() runs on this AND
  bool fresh = false;        // F_ANS: a sorted child rebuilds the answer field on every call
  int done_off = -1;         // F_ANS: state bytes of the (pass, scan) applyAnd loop-ended flags
};

// FilterPlanNode reorder priorities (plan/FilterPlanNode.java:144-170)
enum { PH_SORTED = 0, PH_AND = 1, PH_BITMAP = 2, PH_SCAN = 3, PH_OR = 4 };

struct Builder {
  std::vector<FNode> nodes;
  int state_bytes = 0;
  int pending_off = 0;

  // BlockDocIdSet.iterator(): AndBlockDocIdSet.fastIterator (docidsets/AndBlockDocIdSet.java:146-229) turns an AND with
  // sorted / bitmap children into an eager answer (ranges, bitmaps, then each scan's applyAnd) and, if nested operators
  // remain, an AndDocIdIterator over [answer, rest...]; without index children every child becomes an iterator, and
  // iterator() runs twice on nested operators (the classification loop :166-168 and again :174-177).
  int build(const FsmTreeNode& x, int mult) {
    if (x.op == 0) {
      FNode f;
      f.kind = x.phys == PH_SCAN ? F_SCAN : F_INDEX;
      f.leaf = x.leaf;
      nodes.push_back(f);
      return int(nodes.size()) - 1;
    }
    if (x.op == 2) {
      std::vector<int> kids;
      for (const auto& k : x.kids) kids.push_back(build(k, mult));
      FNode f;
      f.kind = F_OR;
      f.kids = kids;
      nodes.push_back(f);
      return int(nodes.size()) - 1;
    }
    std::vector<int> idx, scans;
    bool fresh = false;
    for (const auto& k : x.kids)
      if (k.op == 0 && (k.phys == PH_SORTED || k.phys == PH_BITMAP)) {
        idx.push_back(k.leaf);
        fresh |= k.phys == PH_SORTED;
      }
    if (idx.empty()) {
      std::vector<int> kids;
      for (const auto& k : x.kids) kids.push_back(build(k, k.op == 0 ? mult : mult * 2));
      FNode f;
      f.kind = F_AND;
      f.kids = kids;
      nodes.push_back(f);
      return int(nodes.size()) - 1;
    }
    for (const auto& k : x.kids)
      if (k.op == 0 && k.phys == PH_SCAN) scans.push_back(k.leaf);
    FNode a;
    a.kind = F_ANS;
    a.idx = idx;
    a.scans = scans;
    a.mult = mult;
    a.fresh = fresh;
    nodes.push_back(a);
    const int ans = int(nodes.size()) - 1;
    std::vector<int> rest;
    for (const auto& k : x.kids)
      if (k.op != 0) rest.push_back(build(k, mult));
    if (rest.empty()) return ans;
    FNode f;
    f.kind = F_AND;
    f.kids.push_back(ans);
    f.kids.insert(f.kids.end(), rest.begin(), rest.end());
    nodes.push_back(f);
    return int(nodes.size()) - 1;
  }

  void layout() {
    state_bytes = int(nodes.size());  // one byte per node: leaf-like 0 idle / 1 searching; AND 0 idle / 1 + child
    pending_off = state_bytes++;
    for (auto& f : nodes)
      if (f.kind == F_ANS) {
        f.done_off = state_bytes;
        state_bytes += f.mult * int(f.scans.size());
      }
  }
};

// The row step: the reference's calls at one row, in the reference's order.
struct Step {
  const std::vector<FNode>& N;
  int root;
  int pending_off;
  // row inputs
  uint32_t raw = 0;                       // leaf predicate bits
  uint32_t ge_lo = 0, le_hi = 0, ge_hi = 0;  // row position against each leaf's [start, end]
  uint32_t always_false = 0;              // scan leaves whose evaluator is alwaysFalse
  // row memos
  std::vector<uint8_t> hit, proc, walked, ansb;
  std::vector<uint8_t> st;
  int count = 0;

  Step(const std::vector<FNode>& n, int r, int po) : N(n), root(r), pending_off(po) {}

  bool in_range(int l) const { return ((ge_lo & le_hi) >> l) & 1u; }
  bool bit(int l) const { return ((raw >> l) & 1u) && in_range(l); }

  bool member(int x) const { return N[x].kind == F_ANS ? ansb[x] : bit(N[x].leaf); }

  void protocol(int x) {
    const FNode& f = N[x];
    for (size_t i = 0; i < f.kids.size(); ++i)
      if (!visit(f.kids[i], true)) {
        st[x] = uint8_t(1 + i);
        return;
      }
    st[x] = 0;
    hit[x] = 1;
  }

  bool visit(int x, bool targeted) {
    const FNode& f = N[x];
    if (f.kind == F_SCAN || f.kind == F_INDEX || f.kind == F_ANS) {
      if (targeted && st[x] == 0 && !hit[x]) st[x] = 1;
      if (st[x] == 1 && !proc[x]) {
        proc[x] = 1;
        if (f.kind == F_SCAN && in_range(f.leaf)) ++count;
        if (member(x)) {
          st[x] = 0;
          hit[x] = 1;
        }
      }
      return hit[x];
    }
    if (f.kind == F_OR) {
      bool h = false;
      for (int k : f.kids) h |= visit(k, targeted);
      return h;
    }
    if (st[x] > 0 && !proc[x]) {
      proc[x] = 1;
      if (visit(f.kids[st[x] - 1], false)) protocol(x);
    }
    if (targeted && st[x] == 0 && !hit[x] && !walked[x]) {
      walked[x] = 1;
      protocol(x);
    }
    for (int k : f.kids) visit(k, false);
    return hit[x];
  }

  // state in -> state out (st holds the state bytes), returns the entries counted at this row
  int run(std::vector<uint8_t>& state) {
    st.swap(state);
    const size_t n = N.size();
    hit.assign(n, 0);
    proc.assign(n, 0);
    walked.assign(n, 0);
    ansb.assign(n, 0);
    count = 0;
    // eager applyAnd of every fast AND, `mult` passes (SVScanDocIdIterator.applyAnd :131-149: it walks the answer
    // while the previous doc < endDocId -- every doc up to the first one >= end -- and counts those >= start)
    for (size_t x = 0; x < n; ++x) {
      const FNode& f = N[x];
      if (f.kind != F_ANS) continue;
      bool idx = true;
      for (int l : f.idx) idx = idx && ((raw >> l) & 1u);
      bool run = idx;
      for (int p = 0; p < f.mult; ++p) {
        if (p == 0 || f.fresh) run = idx;
        for (size_t j = 0; j < f.scans.size(); ++j) {
          const int l = f.scans[j];
          uint8_t& done = st[f.done_off + p * int(f.scans.size()) + int(j)];
          if (!run) continue;
          if (((always_false >> l) & 1u) || done) {
            run = false;
            continue;
          }
          if ((ge_hi >> l) & 1u) done = 1;
          const bool lo_ok = (ge_lo >> l) & 1u;
          if (lo_ok) ++count;
          run = lo_ok && ((raw >> l) & 1u);
        }
      }
      ansb[x] = run;
    }
    const bool pending = st[pending_off];
    st[pending_off] = visit(root, pending) ? 1 : 0;
    state.swap(st);
    return count;
  }
};

}  // namespace

// Range propagation of AndBlockDocIdSet / OrBlockDocIdSet.updateMinMaxRange (docidsets/AndBlockDocIdSet.java:54-63,
// 247-257; OrBlockDocIdSet.java:47-56,131-140): scan and bitmap sets take the range they are assigned, sorted sets
// report their first / last pair (SortedDocIdSet.java:39-55) and ignore assignments.
namespace {
struct RNode {
  const FsmTreeNode* t;
  int64_t mn = 0, mx = 0;
  std::vector<RNode> kids;
};
void r_update(RNode& x);
void r_set_start(RNode& x, int64_t s) {
  if (x.t->op == 0) {
    if (x.t->phys != PH_SORTED) x.mn = s;
  } else if (x.t->op == 1) {
    x.mn = std::max(x.mn, s);
    r_update(x);
  } else {
    x.mn = std::min(x.mn, s);
    r_update(x);
  }
}
void r_set_end(RNode& x, int64_t e) {
  if (x.t->op == 0) {
    if (x.t->phys != PH_SORTED) x.mx = e;
  } else if (x.t->op == 1) {
    x.mx = std::min(x.mx, e);
    r_update(x);
  } else {
    x.mx = std::max(x.mx, e);
    r_update(x);
  }
}
void r_update(RNode& x) {
  for (auto& k : x.kids) {
    if (x.t->op == 1) {
      x.mn = std::max(x.mn, k.mn);
      x.mx = std::min(x.mx, k.mx);
    } else {
      x.mn = std::min(x.mn, k.mn);
      x.mx = std::max(x.mx, k.mx);
    }
  }
  for (auto& k : x.kids) {
    r_set_start(k, x.mn);
    r_set_end(k, x.mx);
  }
}
RNode r_build(const FsmTreeNode& t, const FsmSegInfo& si) {
  RNode x;
  x.t = &t;
  if (t.op == 0) {
    if (t.phys == PH_SORTED) {
      x.mn = si.sorted_first[t.leaf];
      x.mx = si.sorted_last[t.leaf];
    } else {
      x.mn = 0;
      x.mx = int64_t(si.num_docs) - 1;
    }
    return x;
  }
  for (const auto& k : t.kids) x.kids.push_back(r_build(k, si));
  if (t.op == 1) {
    x.mn = INT32_MIN;
    x.mx = INT32_MAX;
  } else {
    x.mn = INT32_MAX;
    x.mx = INT32_MIN;
  }
  r_update(x);
  return x;
}
void r_collect(const RNode& x, std::vector<int64_t>& lo, std::vector<int64_t>& hi) {
  if (x.t->op == 0) {
    lo[x.t->leaf] = x.mn;
    hi[x.t->leaf] = x.mx;
  }
  for (const auto& k : x.kids) r_collect(k, lo, hi);
}
}  // namespace

bool fsm_build(const FsmTreeNode& tree, int num_leaves, const std::vector<FsmSegInfo>& segs, FsmPlan& out,
               std::string* err) {
  out = FsmPlan{};
  const int L = num_leaves;
  if (L > kFsmMaxLeaves) {
    *err = "filter statistics automaton: more than " + std::to_string(kFsmMaxLeaves) + " leaves";
    return false;
  }
  Builder b;
  const int root = b.build(tree, 1);
  b.layout();
  // fast-AND index leaves read their raw bits: the eager answer is not clipped to the iterator ranges
  std::vector<bool> in_ans(L, false);
  for (const auto& f : b.nodes)
    if (f.kind == F_ANS) {
      for (int l : f.idx) in_ans[l] = true;
    }
  // per segment: leaf ranges, row intervals of constant range position, and their input key
  struct Key {
    uint32_t ge_lo, le_hi, ge_hi, af;
    bool operator<(const Key& o) const {
      return std::tie(ge_lo, le_hi, ge_hi, af) < std::tie(o.ge_lo, o.le_hi, o.ge_hi, o.af);
    }
  };
  std::map<Key, int> key_id;
  std::vector<Key> keys;
  out.seg_intervals.resize(segs.size());
  for (size_t s = 0; s < segs.size(); ++s) {
    const FsmSegInfo& si = segs[s];
    std::vector<int64_t> lo(L, 0), hi(L, int64_t(si.num_docs) - 1);
    RNode rt = r_build(tree, si);
    r_collect(rt, lo, hi);
    for (int l = 0; l < L; ++l)
      if (in_ans[l]) {
        lo[l] = 0;
        hi[l] = int64_t(si.num_docs) - 1;
      }
    std::vector<int64_t> cut{0, si.num_docs};
    for (int l = 0; l < L; ++l)
      for (int64_t c : {lo[l], hi[l], hi[l] + 1})
        if (c > 0 && c < si.num_docs) cut.push_back(c);
    std::sort(cut.begin(), cut.end());
    cut.erase(std::unique(cut.begin(), cut.end()), cut.end());
    for (size_t i = 0; i + 1 < cut.size(); ++i) {
      const int64_t r = cut[i];
      Key k{0, 0, 0, si.always_false};
      for (int l = 0; l < L; ++l) {
        if (r >= lo[l]) k.ge_lo |= 1u << l;
        if (r <= hi[l]) k.le_hi |= 1u << l;
        if (r >= hi[l]) k.ge_hi |= 1u << l;
      }
      auto it = key_id.find(k);
      if (it == key_id.end()) {
        it = key_id.emplace(k, int(keys.size())).first;
        keys.push_back(k);
      }
      out.seg_intervals[s].push_back({int32_t(r), it->second});
    }
  }
  // reachable states: BFS from the initial state (everything idle, the root's first next() pending) over every input
  // of every range-position key that occurs
  std::map<std::vector<uint8_t>, int> sid;
  std::vector<std::vector<uint8_t>> states;
  std::vector<uint8_t> s0(b.state_bytes, 0);
  s0[b.pending_off] = 1;
  sid[s0] = 0;
  states.push_back(s0);
  Step step(b.nodes, root, b.pending_off);
  const uint32_t ninputs = 1u << L;
  std::vector<std::vector<uint32_t>> next_of;  // [state][key * ninputs + input] -> (next << 16) | count
  for (size_t q = 0; q < states.size(); ++q) {
    std::vector<uint32_t> row(keys.size() * ninputs);
    for (size_t k = 0; k < keys.size(); ++k) {
      step.ge_lo = keys[k].ge_lo;
      step.le_hi = keys[k].le_hi;
      step.ge_hi = keys[k].ge_hi;
      step.always_false = keys[k].af;
      for (uint32_t in = 0; in < ninputs; ++in) {
        std::vector<uint8_t> st = states[q];
        step.raw = in;
        const int cnt = step.run(st);
        auto it = sid.find(st);
        if (it == sid.end()) {
          if (int(states.size()) >= kFsmMaxStates) {
            *err = "filter statistics automaton: more than " + std::to_string(kFsmMaxStates) + " states";
            return false;
          }
          it = sid.emplace(st, int(states.size())).first;
          states.push_back(st);
        }
        if (cnt > 0xFFFF) {
          *err = "filter statistics automaton: count overflow";
          return false;
        }
        row[k * ninputs + in] = (uint32_t(it->second) << 16) | uint32_t(cnt);
      }
    }
    next_of.push_back(std::move(row));
  }
  const int S = int(states.size());
  if (uint64_t(keys.size()) * uint64_t(S) * ninputs > kFsmMaxTable) {
    *err = "filter statistics automaton: transition tables too large";
    return false;
  }
  out.num_states = S;
  out.num_leaves = L;
  out.num_tables = int(keys.size());
  // device layout: table t, state q, input i -> [(t * S + q) << L | i]
  out.table.assign(size_t(keys.size()) * S * ninputs, 0);
  for (int q = 0; q < S; ++q)
    for (size_t k = 0; k < keys.size(); ++k)
      std::memcpy(&out.table[((k * S + q) << L)], &next_of[q][k * ninputs], ninputs * 4);
  return true;
}

}  // namespace pgx
