"""ctypes wrapper of the oracle's C twin (oracle/pinot_oracle_c.c) -- TEST INFRASTRUCTURE ONLY (tests/, bench.py's
cpu_baseline leg)."""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libpgo.so")
_lib = None


class PgoCol(C.Structure):
    _fields_ = [("fwd", C.c_void_p), ("nbytes", C.c_int64), ("bits", C.c_int), ("dict", C.c_void_p),
                ("card", C.c_int32)]


class PgoSegQuery(C.Structure):
    _fields_ = [("num_docs", C.c_int32), ("num_cols", C.c_int32), ("cols", C.POINTER(PgoCol)),
                ("filter_col", C.c_int32), ("lo", C.c_int32), ("hi", C.c_int32), ("metric_col", C.c_int32),
                ("num_group_cols", C.c_int32), ("group_cols", C.POINTER(C.c_int32)),
                ("count", C.c_int64), ("sum", C.c_double), ("entries_scanned", C.c_int64),
                ("num_groups", C.c_int64), ("g_keys", C.POINTER(C.c_int64)), ("g_sums", C.POINTER(C.c_double)),
                ("g_counts", C.POINTER(C.c_int64)), ("g_cap", C.c_int64)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.check_call(["make", "-C", _HERE])
        L = C.CDLL(_LIB)
        L.pgo_synth_fwd.argtypes = [C.c_uint64, C.c_int64, C.c_int, C.c_uint32, C.c_void_p, C.c_int64]
        L.pgo_synth_value.argtypes = [C.c_uint64, C.c_int64, C.c_uint32]
        L.pgo_synth_value.restype = C.c_uint32
        L.pgo_run.argtypes = [C.POINTER(PgoSegQuery), C.c_int, C.c_int]
        L.pgo_read_int.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64]
        L.pgo_read_int.restype = C.c_int32
        L.pgo_segment_query_size.restype = C.c_int64
        assert L.pgo_segment_query_size() == C.sizeof(PgoSegQuery)
        _lib = L
    return _lib


def synth_fwd(seed, n, bits, card):
    """Packed fixed-bit forward index of synthetic dictIds (bit-identical to libpgx's pgx_synth_column)."""
    nbytes = (n * bits + 7) // 8 + 8
    out = np.zeros(nbytes, dtype=np.uint8)
    lib().pgo_synth_fwd(seed, n, bits, card, out.ctypes.data, nbytes)
    return out


class Segment:
    """Columns = {name: (fwd uint8 array, bits, dict float64 array or None, card)}."""

    def __init__(self, num_docs, columns):
        self.num_docs = num_docs
        self.names = list(columns)
        self.columns = columns


def run(segments, filter_col=None, lo=0, hi=-1, metric="m", group_cols=(), threads=1, collect_groups=False):
    L = lib()
    qs = (PgoSegQuery * len(segments))()
    keep = []
    for i, s in enumerate(segments):
        cols = (PgoCol * len(s.names))()
        for j, name in enumerate(s.names):
            fwd, bits, dct, card = s.columns[name]
            cols[j].fwd = fwd.ctypes.data
            cols[j].nbytes = len(fwd)
            cols[j].bits = bits
            cols[j].dict = dct.ctypes.data if dct is not None else None
            cols[j].card = card
        gc = (C.c_int32 * max(1, len(group_cols)))(*[s.names.index(g) for g in group_cols])
        keep += [cols, gc]
        q = qs[i]
        q.num_docs = s.num_docs
        q.num_cols = len(s.names)
        q.cols = cols
        q.filter_col = s.names.index(filter_col) if filter_col else -1
        q.lo, q.hi = lo, hi
        q.metric_col = s.names.index(metric)
        q.num_group_cols = len(group_cols)
        q.group_cols = gc
        if collect_groups:
            cap = s.num_docs
            arrs = (np.zeros(cap, np.int64), np.zeros(cap, np.float64), np.zeros(cap, np.int64))
            keep.append(arrs)
            q.g_keys = arrs[0].ctypes.data_as(C.POINTER(C.c_int64))
            q.g_sums = arrs[1].ctypes.data_as(C.POINTER(C.c_double))
            q.g_counts = arrs[2].ctypes.data_as(C.POINTER(C.c_int64))
            q.g_cap = cap
    L.pgo_run(qs, len(segments), threads)
    out = []
    for i in range(len(segments)):
        q = qs[i]
        r = {"count": q.count, "sum": q.sum, "entries": q.entries_scanned, "num_groups": q.num_groups}
        if collect_groups:
            ng = q.num_groups
            arrs = keep[-len(segments) + i] if False else None
            r["groups"] = (np.ctypeslib.as_array(q.g_keys, shape=(ng,)).copy(),
                           np.ctypeslib.as_array(q.g_sums, shape=(ng,)).copy(),
                           np.ctypeslib.as_array(q.g_counts, shape=(ng,)).copy())
        out.append(r)
    return out
