"""The C twin's test speed-ups (oracle/c_oracle.py): key-partitioned group-by tasks and threaded forward-index
generation give exactly the single-task answers."""
import ctypes as C

import numpy as np

from oracle import c_oracle
from pinot_amd import synth


def test_threaded_synth_fwd_is_bit_identical():
    n = (1 << 22) + 13
    got = c_oracle.synth_fwd(77, n, 13, 5000, pair_seed=5, npairs=1000)
    ref = np.zeros(len(got), np.uint8)
    c_oracle.lib().pgo_synth_fwd_paired(77, n, 13, 5000, ref.ctypes.data, len(ref), 5, 1000)
    assert np.array_equal(got, ref)


def _c3_like(rows, seg=0):
    wl = synth.WORKLOADS["c3"]
    cols = {}
    for ci, c in enumerate(wl.columns):
        pair = dict(pair_seed=synth.column_seed(wl.seed, seg, 99), npairs=wl.npairs) if c.paired else {}
        seed = synth.column_seed(wl.seed, 0 if c.paired else seg, ci)
        cols[c.name] = (c_oracle.synth_fwd(seed, rows, c.bits, c.card, **pair), c.bits,
                        synth.make_dictionary(c.dict_kind, c.card).astype(np.float64), c.card)
    return c_oracle.Segment(rows, cols)


def _sorted_groups(r):
    k, s, c, lo, hi = r["groups"]
    o = np.argsort(k)
    return k[o], s[o], c[o], lo[o], hi[o]


def test_key_parts_equal_one_task():
    segs = [_c3_like(300_000, s) for s in (0, 1)]
    kw = dict(metric="m", group_cols=("g1", "g2"), collect_groups=True)
    one = c_oracle.run(segs, **kw)
    parts = c_oracle.run(segs, threads=4, key_parts=5, **kw)
    for a, b in zip(one, parts):
        assert a["count"] == b["count"] and a["num_groups"] == b["num_groups"] > 200_000
        for x, y in zip(_sorted_groups(a), _sorted_groups(b)):
            assert np.array_equal(x, y)


def test_key_parts_overflowing_guess_reruns():
    """The rerun path of run(): a task whose group capacity is short reports num_groups > g_cap and writes nothing;
    rerun with the reported capacity it returns every group."""
    seg = _c3_like(50_000)
    L = c_oracle.lib()
    kw = dict(metric="m", group_cols=("g1", "g2"), collect_groups=True)
    ref = c_oracle.run([seg], **kw)[0]
    q = c_oracle.PgoSegQuery()
    cols = (c_oracle.PgoCol * len(seg.names))()
    for j, name in enumerate(seg.names):
        fwd, bits, dct, card = seg.columns[name]
        cols[j].fwd, cols[j].nbytes, cols[j].bits, cols[j].dict, cols[j].card = fwd.ctypes.data, len(fwd), bits, \
            dct.ctypes.data, card
    gc = (C.c_int32 * 2)(0, 1)
    q.num_docs, q.num_cols, q.cols, q.filter_col, q.metric_col = seg.num_docs, len(seg.names), cols, -1, 2
    q.num_group_cols, q.group_cols = 2, gc
    keep = []
    c_oracle._attach_groups(q, 10, keep)
    L.pgo_run(C.byref(q), 1, 1)
    assert q.num_groups == ref["num_groups"] > q.g_cap
    c_oracle._attach_groups(q, q.num_groups, keep)
    L.pgo_run(C.byref(q), 1, 1)
    got = np.ctypeslib.as_array(q.g_keys, shape=(q.num_groups,))
    assert np.array_equal(np.sort(got), np.sort(ref["groups"][0]))
