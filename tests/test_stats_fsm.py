"""numEntriesScannedInFilter automaton (pinot_amd/csrc/pgx_stats.cpp) against the oracle's literal iterator algebra.

The table builder is linked into a test-only library with tests/fsm_driver.cpp, which runs the tables row by row on the
host; libpgx runs the same tables on the GPU (tests/test_gpu_parity.py asserts the GPU statistic too).  Cases: the
reference's golden filter (BaseSingleValueQueriesTest.java:69-74: 84134 as the Java test loads the segment, 63064 with
the bitmap indexes loaded) and random filter trees over segments with sorted, bitmap-indexed and plain columns.
"""
import ctypes as C
import os
import random
import subprocess

import numpy as np
import pytest

from oracle import pinot_oracle as O
from pinot_amd import pql
from tests import helpers as H
from tests import stats_fsm_model as M

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PHYS = {"sorted": 0, "bitmap": 2, "scan": 3}


@pytest.fixture(scope="module")
def drv():
    out = os.path.join(HERE, "_build", "libfsmdrv.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", os.path.join(HERE, "fsm_driver.cpp"),
                           os.path.join(ROOT, "pinot_amd", "csrc", "pgx_stats.cpp"), "-o", out])
    lib = C.CDLL(out)
    lib.fsm_entries.restype = C.c_int64
    return lib


def automaton_entries(lib, seg, tree):
    root, leaves = M.phys_tree(seg, tree)
    op, arg = [], []

    def post(x):
        if "leaf" in x:
            op.append(0)
            arg.append(x["leaf"])
            return
        for k in x["kids"]:
            post(k)
        op.append(1 if x["kind"] == "and" else 2)
        arg.append(len(x["kids"]))

    post(root)
    L = len(leaves)
    n = seg.total_raw_docs
    phys = [3] * L

    def mark(x):
        if "leaf" in x:
            phys[x["leaf"]] = PHYS[x["kind"]]
        for k in x.get("kids", []):
            mark(k)

    mark(root)
    bits = np.zeros((L, n), dtype=np.uint8)
    first = np.zeros(L, dtype=np.int64)
    last = np.zeros(L, dtype=np.int64)
    af = 0
    for l, t in enumerate(leaves):
        m = O.filter_mask_vectorized(seg, t)
        bits[l] = m
        d = np.nonzero(m)[0]
        if phys[l] == 0 and len(d):
            first[l], last[l] = d[0], d[-1]
        if phys[l] == 3 and O.make_evaluator(seg.columns[t["column"]], t).always_false:
            af |= 1 << l
    ia = lambda v: (C.c_int32 * len(v))(*v)
    ns = C.c_int32()
    err = C.create_string_buffer(256)
    r = lib.fsm_entries(ia(op), ia(arg), len(op), ia(phys), L, n,
                        first.ctypes.data_as(C.POINTER(C.c_int64)), last.ctypes.data_as(C.POINTER(C.c_int64)),
                        C.c_uint32(af), bits.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(ns), err, 256)
    assert r >= 0, err.value
    return r, ns.value


@pytest.mark.parametrize("loaded", [False, True])
def test_golden_filter(drv, loaded):
    exp = H.load_expected()
    seg = O.OSegment.from_raw(H.sv_raw(), inverted=exp["inverted"] if loaded else exp["loaded_inverted"])
    q = pql.compile("SELECT COUNT(*) FROM testTable" + exp["filter"]["text"])
    got, _ = automaton_entries(drv, seg, q["filter"])
    assert got == (63064 if loaded else 84134)
    assert got == O.filter_docs(seg, q["filter"])[1]


def _rand_seg(rng, n):
    raw = {"s": np.sort(rng.integers(0, 20, n)), "a": rng.integers(0, 10, n), "b": rng.integers(0, 6, n),
           "c": rng.integers(0, 30, n), "d": rng.integers(0, 4, n)}
    inv = [c for c in "abcd" if rng.random() < 0.5] + ["s"]
    return O.OSegment.from_raw(raw, inverted=inv)


def _rand_leaf(r):
    col = r.choice("sabcd")
    k = r.random()
    if k < 0.3:
        return "%s = %d" % (col, r.randint(0, 8))
    if k < 0.5:
        return "%s <> %d" % (col, r.randint(0, 8))
    if k < 0.7:
        return "%s BETWEEN %d AND %d" % (col, r.randint(0, 4), r.randint(3, 12))
    if k < 0.85:
        return "%s IN (%d, %d, %d)" % (col, r.randint(0, 9), r.randint(0, 9), r.randint(0, 9))
    return "%s NOT IN (%d, %d)" % (col, r.randint(0, 9), r.randint(0, 9))


def _rand_tree(r, d, max_leaves):
    if d == 0 or r.random() < 0.3:
        return _rand_leaf(r)
    k = r.randint(2, 3)
    op = r.choice([" AND ", " OR "])
    return "(" + op.join(_rand_tree(r, d - 1, max_leaves) for _ in range(k)) + ")"


@pytest.mark.parametrize("seed", range(4))
def test_random_trees(drv, seed):
    r = random.Random(seed)
    rng = np.random.default_rng(seed)
    done = 0
    while done < 40:
        seg = _rand_seg(rng, r.choice([60, 300, 1500]))
        q = pql.compile("SELECT COUNT(*) FROM t WHERE " + _rand_tree(r, 3, 10))
        if len(M.phys_tree(seg, q["filter"])[1]) > 10:
            continue
        got, _ = automaton_entries(drv, seg, q["filter"])
        assert got == O.filter_docs(seg, q["filter"])[1], q["filter"]
        done += 1


def test_sweep_model_matches_oracle():
    """The Python restatement of the sweep (stats_fsm_model) on the golden filter, both index configurations."""
    exp = H.load_expected()
    for inv, want in ((exp["loaded_inverted"], 84134), (exp["inverted"], 63064)):
        seg = O.OSegment.from_raw(H.sv_raw(), inverted=inv)
        q = pql.compile("SELECT COUNT(*) FROM testTable" + exp["filter"]["text"])
        assert M.model_entries(seg, q["filter"]) == want
