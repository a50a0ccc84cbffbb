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
                ("filter_col", C.c_int32), ("lo", C.c_int32), ("hi", C.c_int32),
                ("num_leaves", C.c_int32), ("leaf_col", C.POINTER(C.c_int32)),
                ("leaf_bits", C.POINTER(C.POINTER(C.c_uint32))), ("prog_len", C.c_int32),
                ("prog", C.POINTER(C.c_int32)), ("metric_col", C.c_int32),
                ("num_group_cols", C.c_int32), ("group_cols", C.POINTER(C.c_int32)),
                ("count", C.c_int64), ("sum", C.c_double), ("vmin", C.c_double), ("vmax", C.c_double),
                ("entries_scanned", C.c_int64),
                ("num_groups", C.c_int64), ("g_keys", C.POINTER(C.c_int64)), ("g_sums", C.POINTER(C.c_double)),
                ("g_counts", C.POINTER(C.c_int64)), ("g_mins", C.POINTER(C.c_double)),
                ("g_maxs", C.POINTER(C.c_double)), ("g_cap", C.c_int64),
                ("leaf_inv", C.POINTER(C.c_void_p)), ("leaf_excl", C.POINTER(C.c_int32)),
                ("key_part", C.c_int32), ("key_parts", C.c_int32)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.check_call(["make", "-C", _HERE])
        L = C.CDLL(_LIB)
        L.pgo_synth_fwd.argtypes = [C.c_uint64, C.c_int64, C.c_int, C.c_uint32, C.c_void_p, C.c_int64]
        L.pgo_synth_fwd_paired.argtypes = [C.c_uint64, C.c_int64, C.c_int, C.c_uint32, C.c_void_p, C.c_int64,
                                           C.c_uint64, C.c_uint32]
        L.pgo_synth_fwd_range.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int, C.c_uint32, C.c_void_p,
                                          C.c_uint64, C.c_uint32]
        L.pgo_synth_value.argtypes = [C.c_uint64, C.c_int64, C.c_uint32]
        L.pgo_synth_value.restype = C.c_uint32
        L.pgo_run.argtypes = [C.POINTER(PgoSegQuery), C.c_int, C.c_int]
        L.pgo_read_int.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64]
        L.pgo_read_int.restype = C.c_int32
        L.pgo_segment_query_size.restype = C.c_int64
        L.pgo_synth_ids.argtypes = [C.c_uint64, C.c_int64, C.c_uint32, C.c_void_p]
        L.pgo_inverted_build.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64]
        L.pgo_inverted_build.restype = C.c_int64
        assert L.pgo_segment_query_size() == C.sizeof(PgoSegQuery)
        _lib = L
    return _lib


def synth_fwd(seed, n, bits, card, pair_seed=0, npairs=0):
    """Packed fixed-bit forward index of synthetic dictIds (bit-identical to libpgx's pgx_synth_column, and with
    npairs > 0 to pgx_synth_column_paired)."""
    nbytes = (n * bits + 7) // 8 + 8
    out = np.zeros(nbytes, dtype=np.uint8)
    L = lib()
    if n < (1 << 22):
        L.pgo_synth_fwd_paired(seed, n, bits, card, out.ctypes.data, nbytes, pair_seed, npairs)
        return out
    from concurrent.futures import ThreadPoolExecutor  # row ranges of a multiple of 8 rows touch disjoint bytes
    T = test_threads()
    step = (n // T + 7) & ~7
    with ThreadPoolExecutor(T) as ex:
        list(ex.map(lambda r0: L.pgo_synth_fwd_range(seed, r0, min(n, r0 + step), bits, card, out.ctypes.data,
                                                     pair_seed, npairs), range(0, n, step)))
    return out


def synth_ids(seed, n, card):
    """The synthetic dictIds synth_fwd packs (unpaired columns)."""
    out = np.empty(n, dtype=np.int32)
    lib().pgo_synth_ids(seed, n, card, out.ctypes.data)
    return out


def inverted_build(ids, card):
    """<col>.bitmap.inv bytes of a dictId column (the C twin's writer; tests pin it to pinot_amd.segment's)."""
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    L = lib()
    n = L.pgo_inverted_build(ids.ctypes.data, len(ids), card, None, 0)
    out = np.empty(n, dtype=np.uint8)
    L.pgo_inverted_build(ids.ctypes.data, len(ids), card, out.ctypes.data, n)
    return out


def dict_ids(fwd, n, bits):
    """Decode a packed forward index (numpy, MSB-first big-endian; oracle decode_fixed_bit_fast)."""
    from oracle import pinot_oracle as O
    return O.decode_fixed_bit_fast(bytes(fwd), n, bits)


class Segment:
    """Columns = {name: (fwd uint8 array, bits, dict float64 array or None, card)}."""

    def __init__(self, num_docs, columns):
        self.num_docs = num_docs
        self.names = list(columns)
        self.columns = columns


def test_threads():
    """Host threads for the C twin in tests: the GPU box shows the whole machine's CPUs but grants 16."""
    return max(1, min(16, os.cpu_count() or 1))


def run(segments, filter_col=None, lo=0, hi=-1, metric="m", group_cols=(), threads=1, collect_groups=False,
        leaves=None, prog=None, inverted=None, excl=None, key_parts=1):
    """leaves = [(column, dictId bitset uint32 array)], prog = postfix ints (>= 0 leaf, -1 AND, -2 OR).
    inverted = {column: .bitmap.inv bytes (uint8 array)} per segment (a list, one dict per segment): every leaf is then
    evaluated on the bitmaps (BitmapBasedFilterOperator) instead of per row; excl[l] = 1 marks NEQ / NOT_IN leaves.
    key_parts > 1 (LONG_MAP group-by with collect_groups, tests only): every segment runs as key_parts tasks, each
    aggregating the groups of one hash part of the key space; the parts' groups are disjoint and are concatenated (in
    part order), and count / entries come from part 0 (every part scans every doc)."""
    L = lib()
    P = max(1, int(key_parts))
    qs = (PgoSegQuery * (len(segments) * P))()
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
        for part in range(P):
            q = qs[i * P + part]
            q.key_part, q.key_parts = part, P
            q.num_docs = s.num_docs
            q.num_cols = len(s.names)
            q.cols = cols
            q.filter_col = s.names.index(filter_col) if filter_col else -1
            q.lo, q.hi = lo, hi
            if leaves:
                lc = (C.c_int32 * len(leaves))(*[s.names.index(c) for c, _ in leaves])
                bits = [np.ascontiguousarray(b, dtype=np.uint32) for _, b in leaves]
                lb = (C.POINTER(C.c_uint32) * len(leaves))(*[b.ctypes.data_as(C.POINTER(C.c_uint32)) for b in bits])
                pg = (C.c_int32 * len(prog))(*prog)
                keep += [lc, bits, lb, pg]
                q.num_leaves = len(leaves)
                q.leaf_col = lc
                q.leaf_bits = lb
                q.prog_len = len(prog)
                q.prog = pg
                if inverted is not None:
                    invs = [np.ascontiguousarray(inverted[i][c], dtype=np.uint8) for c, _ in leaves]
                    li = (C.c_void_p * len(leaves))(*[a.ctypes.data for a in invs])
                    le = (C.c_int32 * len(leaves))(*(excl or [0] * len(leaves)))
                    keep += [invs, li, le]
                    q.leaf_inv = li
                    q.leaf_excl = le
            q.metric_col = s.names.index(metric)
            q.num_group_cols = len(group_cols)
            q.group_cols = gc
            if collect_groups:
                _attach_groups(q, s.num_docs if P == 1 else s.num_docs // P + s.num_docs // (4 * P) + 65536, keep)
    L.pgo_run(qs, len(qs), threads)
    if collect_groups and P > 1:  # a part whose groups overflowed its guess: rerun it alone with the exact capacity
        redo = [k for k in range(len(qs)) if qs[k].num_groups > qs[k].g_cap]
        for k in redo:
            _attach_groups(qs[k], qs[k].num_groups, keep)
            L.pgo_run(C.byref(qs[k]), 1, 1)
    out = []
    for i in range(len(segments)):
        q = qs[i * P]
        r = {"count": q.count, "sum": q.sum, "min": q.vmin, "max": q.vmax, "entries": q.entries_scanned,
             "num_groups": sum(qs[i * P + p].num_groups for p in range(P))}
        if collect_groups:
            parts = []
            for p in range(P):
                qp = qs[i * P + p]
                ng = qp.num_groups
                parts.append(tuple(np.ctypeslib.as_array(a, shape=(ng,)).copy() if ng else np.zeros(0, dt)
                                   for a, dt in zip((qp.g_keys, qp.g_sums, qp.g_counts, qp.g_mins, qp.g_maxs),
                                                    (np.int64, np.float64, np.int64, np.float64, np.float64))))
            r["groups"] = tuple(np.concatenate([pt[j] for pt in parts]) for j in range(5)) if P > 1 else parts[0]
        out.append(r)
    return out


def _attach_groups(q, cap, keep):
    arrs = (np.zeros(cap, np.int64), np.zeros(cap, np.float64), np.zeros(cap, np.int64),
            np.zeros(cap, np.float64), np.zeros(cap, np.float64))
    keep.append(arrs)
    q.g_keys = arrs[0].ctypes.data_as(C.POINTER(C.c_int64))
    q.g_sums = arrs[1].ctypes.data_as(C.POINTER(C.c_double))
    q.g_counts = arrs[2].ctypes.data_as(C.POINTER(C.c_int64))
    q.g_mins = arrs[3].ctypes.data_as(C.POINTER(C.c_double))
    q.g_maxs = arrs[4].ctypes.data_as(C.POINTER(C.c_double))
    q.g_cap = cap
