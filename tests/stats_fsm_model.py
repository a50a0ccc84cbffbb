"""Test infrastructure: the per-row "sweep" model of numEntriesScannedInFilter that libpgx's statistics automaton
(pgx_stats.cpp fsm_build, pgx_kernels.hip pgx_fsm_*) is built from, restated in Python so it can be checked against
the oracle's literal iterator algebra (oracle/pinot_oracle.py filter_docs) on random filter trees.

Every iterator of the reference filter algebra (SVScanDocIdIterator, Bitmap/Sorted/RangelessBitmapDocIdIterator,
OrDocIdIterator, AndDocIdIterator; AndBlockDocIdSet.fastIterator's eager applyAnd) only ever moves forward, and its
answer to advance(t) is the next member >= t of its doc set.  Processing rows in increasing order, each node is either
idle (its current doc is behind the row) or searching (a scan in progress: its current doc will be >= the row); a target
delivered to an idle node starts a search at that row, one delivered to a searching node is a no-op, and a scan leaf
counts every row it searches.  The state at a row boundary is finite, so the whole statistic is a finite automaton over
the rows' leaf-membership bits.
"""
from oracle import pinot_oracle as O

PRIO = {"sorted": 0, "and": 1, "bitmap": 2, "scan": 3, "or": 4}
INT_MIN, INT_MAX = -2 ** 31, 2 ** 31 - 1


def phys_tree(seg, tree):
    """FilterPlanNode.constructPhysicalOperator + reorder: nested dicts {kind, leaf|kids}; leaves numbered in order."""
    leaves = []

    def rec(t):
        if t["op"] in ("AND", "OR"):
            kids = sorted((rec(c) for c in t["children"]), key=lambda k: PRIO[k["kind"]])
            return {"kind": t["op"].lower(), "kids": kids}
        col = seg.columns[t["column"]]
        if col.has_inverted and t["op"] != "RANGE":
            kind = "sorted" if col.is_sorted else "bitmap"
        else:
            kind = "scan"
        leaves.append(t)
        return {"kind": kind, "leaf": len(leaves) - 1}

    return rec(tree), leaves


def leaf_ranges(seg, root, sorted_pairs):
    """min/max doc ids after the AndBlockDocIdSet / OrBlockDocIdSet updateMinMaxRange propagation (scan and bitmap sets
    take the assigned range; sorted sets report their first/last pair and ignore assignments)."""
    n = seg.total_raw_docs
    rng = {}

    def build(x):
        if "leaf" in x:
            if x["kind"] == "sorted":
                p = sorted_pairs[x["leaf"]]
                x["min"], x["max"] = (p[0][0], p[-1][1]) if p else (0, 0)
            else:
                x["min"], x["max"] = 0, n - 1
            return
        for k in x["kids"]:
            build(k)
        if x["kind"] == "and":
            x["min"], x["max"] = INT_MIN, INT_MAX
        else:
            x["min"], x["max"] = INT_MAX, INT_MIN
        update(x)

    def update(x):
        if x["kind"] == "and":
            for k in x["kids"]:
                x["min"] = max(x["min"], k["min"])
                x["max"] = min(x["max"], k["max"])
        else:
            for k in x["kids"]:
                x["min"] = min(x["min"], k["min"])
                x["max"] = max(x["max"], k["max"])
        for k in x["kids"]:
            set_start(k, x["min"])
            set_end(k, x["max"])

    def set_start(x, s):
        if "leaf" in x:
            if x["kind"] != "sorted":
                x["min"] = s
        elif x["kind"] == "and":
            x["min"] = max(x["min"], s)
            update(x)
        else:
            x["min"] = min(x["min"], s)
            update(x)

    def set_end(x, e):
        if "leaf" in x:
            if x["kind"] != "sorted":
                x["max"] = e
        elif x["kind"] == "and":
            x["max"] = min(x["max"], e)
            update(x)
        else:
            x["max"] = max(x["max"], e)
            update(x)

    build(root)

    def collect(x):
        if "leaf" in x:
            rng[x["leaf"]] = (x["min"], x["max"])
        else:
            for k in x["kids"]:
                collect(k)

    collect(root)
    return rng


def iterator_tree(root):
    """The iterator structure BlockDocIdSet.iterator() builds: fast ANDs (>= 1 sorted/bitmap child) become an eager
    answer ("ans": index leaves, applyAnd scans in order) followed, if nested operators remain, by an AndDocIdIterator
    over [answer, rest...].  `mult` = how many times iterator() runs on the node: an AND without index children calls
    iterator() twice on each nested operator child (AndBlockDocIdSet.java:166-178); every call of a fast AND repeats
    its applyAnd, re-using the answer field unless a sorted child rebuilds it (:182-203)."""
    def rec(x, mult):
        if "leaf" in x:
            return {"kind": "scan" if x["kind"] == "scan" else "index", "leaf": x["leaf"]}
        if x["kind"] == "or":
            return {"kind": "or", "kids": [rec(k, mult) for k in x["kids"]]}
        idx = [k["leaf"] for k in x["kids"] if "leaf" in k and k["kind"] in ("sorted", "bitmap")]
        if not idx:
            return {"kind": "and", "kids": [rec(k, mult * (1 if "leaf" in k else 2)) for k in x["kids"]]}
        scans = [k["leaf"] for k in x["kids"] if "leaf" in k and k["kind"] == "scan"]
        rest = [rec(k, mult) for k in x["kids"] if "leaf" not in k]
        ans = {"kind": "ans", "idx": idx, "scans": scans, "mult": mult,
               "fresh": any(k["kind"] == "sorted" for k in x["kids"] if "leaf" in k)}
        return ans if not rest else {"kind": "and", "kids": [ans] + rest}

    return rec(root, 1)


def entries_scanned(raw, ranges, it_root, n, always_false=()):
    """Sweep the rows; raw[l][r] = leaf l's predicate holds at row r, ranges[l] = leaf l's [start, end] (driven leaves
    only see docs inside it).  Returns numEntriesScannedInFilter."""
    bits = [[raw[l][r] and ranges[l][0] <= r <= ranges[l][1] for r in range(n)] for l in range(len(raw))]
    in_range = [[ranges[l][0] <= r <= ranges[l][1] for r in range(n)] for l in range(len(raw))]
    done = {}
    nodes = []

    def number(x):
        x["id"] = len(nodes)
        nodes.append(x)
        for k in x.get("kids", []):
            number(k)

    number(it_root)
    st = [0] * len(nodes)  # leaf-like: 0 idle / 1 searching; and: 0 idle / 1 + s searching child s
    count = 0
    pending = True
    for r in range(n):
        hit = [False] * len(nodes)
        proc = [False] * len(nodes)
        walked = [False] * len(nodes)
        ans_bit = {}
        cnt = [0]

        # eager applyAnd of every fast AND (AndBlockDocIdSet.fastIterator, at iterator-creation time), `mult` passes.
        # SVScanDocIdIterator.applyAnd (:131-149) walks the answer while the previous doc < endDocId: it processes
        # every answer doc up to the first one >= end (`done` once processed) and counts those >= start.
        for x in nodes:
            if x["kind"] == "ans":
                idx = all(raw[l][r] for l in x["idx"])  # raw bitmaps / sorted pairs: not clipped
                run = idx
                for p in range(x["mult"]):
                    if p == 0 or x["fresh"]:
                        run = idx
                    for j, l in enumerate(x["scans"]):
                        lo, hi = ranges[l]
                        key = (x["id"], p, j)
                        if not run:
                            continue
                        if l in always_false or done.get(key):  # applyAnd returns at once (:133-135) / loop ended
                            run = False
                            continue
                        if r >= hi:
                            done[key] = True
                        if r >= lo:
                            cnt[0] += 1
                        run = r >= lo and raw[l][r]
                ans_bit[x["id"]] = run

        def member(x):
            return ans_bit[x["id"]] if x["kind"] == "ans" else bits[x["leaf"]][r]

        def protocol(x):
            for i, k in enumerate(x["kids"]):
                if not visit(k, True):
                    st[x["id"]] = 1 + i
                    return
            st[x["id"]] = 0
            hit[x["id"]] = True

        def visit(x, targeted):
            i = x["id"]
            k = x["kind"]
            if k in ("scan", "index", "ans"):
                if targeted and st[i] == 0 and not hit[i]:
                    st[i] = 1
                if st[i] == 1 and not proc[i]:
                    proc[i] = True
                    if k == "scan" and in_range[x["leaf"]][r]:
                        cnt[0] += 1
                    if member(x):
                        st[i] = 0
                        hit[i] = True
                return hit[i]
            if k == "or":
                h = False
                for c in x["kids"]:
                    h |= visit(c, targeted)
                return h
            # and
            if st[i] > 0 and not proc[i]:
                proc[i] = True
                if visit(x["kids"][st[i] - 1], False):
                    protocol(x)
            if targeted and st[i] == 0 and not hit[i] and not walked[i]:
                walked[i] = True
                protocol(x)
            for c in x["kids"]:
                visit(c, False)
            return hit[i]

        pending = visit(it_root, pending)
        count += cnt[0]
    return count


def model_entries(seg, tree):
    """numEntriesScannedInFilter of `tree` on `seg` by the sweep model."""
    import numpy as np
    if tree is None:
        return 0
    root, leaves = phys_tree(seg, tree)
    n = seg.total_raw_docs
    pairs = {}
    for l, t in enumerate(leaves):
        col = seg.columns[t["column"]]
        if col.has_inverted and col.is_sorted and t["op"] != "RANGE":
            pairs[l] = O._SortedSet(col, O.make_evaluator(col, t), 0, n - 1).pairs
    rng = leaf_ranges(seg, root, pairs)
    it = iterator_tree(root)
    raw = [O.filter_mask_vectorized(seg, t).tolist() for t in leaves]
    af = {l for l, t in enumerate(leaves) if O.make_evaluator(seg.columns[t["column"]], t).always_false}
    return entries_scanned(raw, rng, it, n, af)
