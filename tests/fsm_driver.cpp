// Test infrastructure (not part of libpgx): runs the statistics automaton that pgx_stats.cpp builds over host leaf masks,
// row by row, so tests/test_stats_fsm.py can check the table builder against the oracle's literal iterator algebra on
// a machine without a GPU.  libpgx runs the same tables on the device (pgx_kernels.hip pgx_fsm_*).
#include <cstdint>
#include <string>
#include <vector>

#include "../pinot_amd/csrc/pgx_internal.h"

using namespace pgx;

namespace {
// postfix: op 0 = leaf (arg = leaf index), 1 = AND, 2 = OR (arg = arity); phys[leaf]: 0 sorted, 2 bitmap, 3 scan
FsmTreeNode rebuild(const int32_t* op, const int32_t* arg, int n, const int32_t* phys) {
  std::vector<FsmTreeNode> st;
  for (int i = 0; i < n; ++i) {
    FsmTreeNode t;
    t.op = op[i];
    if (op[i] == 0) {
      t.leaf = arg[i];
      t.phys = phys[arg[i]];
    } else {
      t.kids.assign(st.end() - arg[i], st.end());
      st.erase(st.end() - arg[i], st.end());
    }
    st.push_back(t);
  }
  return st.back();
}
}  // namespace

extern "C" int64_t fsm_entries(const int32_t* op, const int32_t* arg, int n, const int32_t* phys, int L,
                               int32_t num_docs, const int64_t* sorted_first, const int64_t* sorted_last,
                               uint32_t always_false, const uint8_t* bits /* [L][num_docs] */, int32_t* num_states,
                               char* err, int errlen) {
  FsmSegInfo si;
  si.num_docs = num_docs;
  si.sorted_first.assign(sorted_first, sorted_first + L);
  si.sorted_last.assign(sorted_last, sorted_last + L);
  si.always_false = always_false;
  FsmPlan plan;
  std::string e;
  if (!fsm_build(rebuild(op, arg, n, phys), L, {si}, plan, &e)) {
    snprintf(err, errlen, "%s", e.c_str());
    return -1;
  }
  *num_states = plan.num_states;
  const auto& iv = plan.seg_intervals[0];
  int64_t total = 0;
  uint32_t q = 0;
  size_t k = 0;
  for (int32_t r = 0; r < num_docs; ++r) {
    while (k + 1 < iv.size() && iv[k + 1].first <= r) ++k;
    uint32_t in = 0;
    for (int l = 0; l < L; ++l) in |= uint32_t(bits[size_t(l) * num_docs + r] & 1) << l;
    const uint32_t e2 = plan.table[((uint64_t(iv[k].second) * plan.num_states + q) << L) | in];
    total += e2 & 0xFFFF;
    q = e2 >> 16;
  }
  return total;
}
