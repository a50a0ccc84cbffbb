"""The C twin's bitmap filter (oracle/pinot_oracle_c.c: roaring containers, BitmapDocIdSet / AndBlockDocIdSet /
OrBlockDocIdSet iterators) -- it times C5's CPU baseline, so it is pinned here:
* its .bitmap.inv writer against pinot_amd.segment's (which the Java-written fixtures pin, test_segment_fixtures.py);
* its bitmap-iterated results against its own per-row dictId-set evaluation of the same filter tree, on filters that
  take every path: single-bitmap leaves (read in place), IN (OR of bitmaps), NEQ / NOT_IN (flip), AND of bitmaps,
  AND with an OR child (leapfrog), OR with composite children (iterator merge), nested blocks, empty results."""
import numpy as np
import pytest

from oracle import c_oracle
from pinot_amd import segment

ROWS = 150_000  # three 64K keys, the last partial


def bits(card, ids):
    w = np.zeros((card + 31) // 32, dtype=np.uint32)
    for i in ids:
        w[i >> 5] |= np.uint32(1 << (i & 31))
    return w


@pytest.fixture(scope="module")
def seg():
    rng = np.random.default_rng(5)
    cols, inv, ids = {}, {}, {}
    # a: card 4, skewed (bitmap containers); b: card 300 (array containers); c: card 12 with an empty dictId and one
    # dictId confined to the first key; m: the metric; g: the group key
    spec = {"a": 4, "b": 300, "c": 12, "g": 50, "m": 1000}
    for name, card in spec.items():
        if name == "a":
            x = rng.choice(4, ROWS, p=[0.7, 0.2, 0.08, 0.02]).astype(np.int32)
        elif name == "c":
            x = rng.integers(0, 11, ROWS).astype(np.int32)
            x[x == 5] = 6
            x[:3000][rng.random(3000) < 0.3] = 5  # dictId 5 only below doc 3000; dictId 11 never
        else:
            x = rng.integers(0, card, ROWS).astype(np.int32)
        bitsz = max(1, int(card - 1).bit_length())
        fwd = np.frombuffer(segment.pack_fixed_bit(x, bitsz) + b"\0" * 8, dtype=np.uint8)
        dv = np.arange(card, dtype=np.float64) * 1.5 + 1.0
        cols[name] = (fwd, bitsz, dv, card)
        ids[name] = x
        inv[name] = c_oracle.inverted_build(x, card)
    return c_oracle.Segment(ROWS, cols), inv, ids


def test_inverted_writer_matches_segment_writer(seg):
    _, inv, ids = seg
    for name, card in (("a", 4), ("b", 300), ("c", 12)):
        ref = segment.build_inverted_index(ids[name].astype(np.int64), card)
        assert bytes(inv[name]) == ref, name


def test_inverted_writer_empty_column():
    out = c_oracle.inverted_build(np.zeros(0, dtype=np.int32), 3)
    assert bytes(out) == segment.build_inverted_index(np.zeros(0, dtype=np.int64), 3)


LEAVES = {
    "a_eq0": ("a", [0], 0), "a_eq3": ("a", [3], 0), "a_in": ("a", [1, 3], 0), "a_neq0": ("a", [1, 2, 3], 1),
    "b_in": ("b", list(range(0, 300, 7)), 0), "b_eq": ("b", [42], 0), "b_notin": ("b", [i for i in range(300) if i % 3], 1),
    "c_eq5": ("c", [5], 0), "c_eq11": ("c", [11], 0), "c_neq6": ("c", [i for i in range(12) if i != 6], 1),
}

FILTERS = [
    (["a_eq0"], [0]),
    (["a_eq3"], [0]),
    (["c_eq11"], [0]),                                                  # empty bitmap
    (["a_neq0"], [0]),
    (["b_notin"], [0]),
    (["a_in", "b_eq"], [0, 1, -2]),                                     # OR of bitmaps
    (["a_eq0", "c_neq6"], [0, 1, -1]),                                  # AND of bitmaps
    (["b_in", "a_eq3", "c_neq6"], [0, 1, -2, 2, -1]),                   # C5's shape: (IN OR EQ) AND NEQ
    (["b_in", "a_eq3", "c_eq5"], [0, 1, -2, 2, -1]),                    # sparse AND side
    (["a_eq0", "b_in", "-", "c_eq5", "b_eq"], [0, 1, -1, 3, 4, -1, -2]),  # OR of two ANDs (iterator merge)
    (["a_in", "b_in", "c_neq6", "b_notin"], [0, 1, -1, 2, 3, -2, -1]),   # AND(AND(a,b), OR(c,b')) flattened
    (["c_eq5", "c_eq11"], [0, 1, -1]),                                  # empty AND
    (["a_eq0", "b_in", "c_neq6"], [0, 1, -1, 2, -1]),                   # flattened 3-way AND
]


@pytest.mark.parametrize("fi", range(len(FILTERS)))
@pytest.mark.parametrize("group", [False, True])
def test_bitmap_filter_matches_row_filter(seg, fi, group):
    s, inv, _ = seg
    names, prog = FILTERS[fi]
    used = [n for n in names if n != "-"]
    leaves, excl, remap = [], [], {}
    for n in used:
        col, vals, ex = LEAVES[n]
        remap[names.index(n)] = len(leaves)
        leaves.append((col, bits(s.columns[col][3], vals)))
        excl.append(ex)
    prog = [remap[p] if p >= 0 else p for p in prog]
    kw = dict(metric="m", leaves=leaves, prog=prog, collect_groups=group, group_cols=("g",) if group else ())
    rows = c_oracle.run([s], **kw)[0]
    bm = c_oracle.run([s], inverted=[inv], excl=excl, **kw)[0]
    assert bm["count"] == rows["count"]
    assert bm["sum"] == rows["sum"]
    assert bm["entries"] == 0 and rows["entries"] == ROWS * len(leaves)
    if group:
        assert bm["num_groups"] == rows["num_groups"]
        for a, b in zip(bm["groups"], rows["groups"]):
            np.testing.assert_array_equal(a, b)
    # and both against numpy
    ids = {c: c_oracle.dict_ids(s.columns[c][0], ROWS, s.columns[c][1]) for c in ("a", "b", "c", "m")}
    st = []
    for p in prog:
        if p >= 0:
            col, w = leaves[p]
            x = ids[col]
            st.append(((w[x >> 5] >> (x & 31)) & 1).astype(bool))
        else:
            y, x = st.pop(), st.pop()
            st.append(x & y if p == -1 else x | y)
    assert rows["count"] == int(st[0].sum())
