"""ctypes binding of libpgx.so (include/pgx.h).  Fails loudly when the HIP library is missing: there is no CPU
fallback on the product path."""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PGX_LIB", os.path.join(_HERE, "libpgx.so"))


PGX_ERR_INVALID_ARG = 1
PGX_ERR_UNSUPPORTED = 2  # pgx.h pgx_status: the caller falls back to the Java operators


class PgxError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("pgx error %d: %s" % (status, msg))
        self.status = status


PGX_INT, PGX_LONG, PGX_FLOAT, PGX_DOUBLE, PGX_STRING = range(5)
PGX_COUNT, PGX_SUM, PGX_MIN, PGX_MAX, PGX_AVG, PGX_COUNTMV, PGX_SUMMV, PGX_MINMV, PGX_MAXMV, PGX_AVGMV = range(10)
PGX_PRED = {"EQ": 0, "NEQ": 1, "IN": 2, "NOT_IN": 3, "RANGE": 4}
PGX_F_LEAF, PGX_F_AND, PGX_F_OR = 0, 1, 2
PGX_MEM_HOST, PGX_MEM_DEVICE = 0, 1
PGX_X_KEEP_DENSE_ON_DEVICE = 0x1
PGX_X_FORCE_HASH = 0x2
PGX_X_NO_PARTITION = 0x4
PGX_X_THROUGHPUT = 0x8
PGX_Q_NO_STAR_TREE = 0x1
ERR_UNSUPPORTED = 2
PGX_ERR_TIMEOUT = 5
PGX_ERR_INTERNAL = 6


class CtxOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("flags", C.c_uint32)]


class ColumnDesc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data_type", C.c_int32), ("cardinality", C.c_int32),
                ("bits_per_element", C.c_int32), ("is_sorted", C.c_int32), ("dict_width", C.c_int32),
                ("fwd", C.c_void_p), ("fwd_len", C.c_uint64), ("sorted_pairs", C.c_void_p), ("sorted_len", C.c_uint64),
                ("dict", C.c_void_p), ("dict_len", C.c_uint64), ("inv", C.c_void_p), ("inv_len", C.c_uint64),
                ("pad_char", C.c_int32), ("is_multi_value", C.c_int32), ("total_entries", C.c_int32)]


class SegmentDesc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("total_docs", C.c_int32), ("total_raw_docs", C.c_int32),
                ("num_columns", C.c_int32), ("columns", C.POINTER(ColumnDesc)), ("star_tree", C.c_void_p),
                ("star_tree_len", C.c_uint64), ("mem", C.c_int32), ("num_star_skip_dims", C.c_int32),
                ("star_skip_dims", C.POINTER(C.c_char_p))]


class Agg(C.Structure):
    _fields_ = [("fn", C.c_int32), ("column", C.c_char_p)]


class FilterNode(C.Structure):
    _fields_ = [("op", C.c_int32), ("arg", C.c_int32)]


class Leaf(C.Structure):
    _fields_ = [("column", C.c_char_p), ("kind", C.c_int32)]


class QueryDesc(C.Structure):
    _fields_ = [("num_aggs", C.c_int32), ("aggs", C.POINTER(Agg)), ("num_group_cols", C.c_int32),
                ("group_cols", C.POINTER(C.c_char_p)), ("top_n", C.c_int32), ("num_filter_nodes", C.c_int32),
                ("filter", C.POINTER(FilterNode)), ("num_leaves", C.c_int32), ("leaves", C.POINTER(Leaf)),
                ("flags", C.c_uint32)]


class LeafBinding(C.Structure):
    _fields_ = [("lo", C.c_int32), ("hi", C.c_int32), ("words", C.POINTER(C.c_uint32))]


class Predicate(C.Structure):
    _fields_ = [("num_values", C.c_int32), ("values", C.POINTER(C.c_char_p)), ("lower_inclusive", C.c_int32),
                ("upper_inclusive", C.c_int32)]


class MutableColumn(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data_type", C.c_int32), ("is_multi_value", C.c_int32),
                ("has_inverted", C.c_int32)]


class ExecOpts(C.Structure):
    _fields_ = [("stream", C.c_uint64), ("dense_out", C.c_void_p), ("dense_out_bytes", C.c_uint64),
                ("flags", C.c_uint32)]


_lib = None

EXPORTS = {
    "pgx_jit_compile_check": (C.c_int, [C.c_char_p, C.c_char_p, C.c_ulong]),
    "pgx_jit_selftest": (C.c_int, [C.POINTER(C.c_int), C.c_char_p, C.c_ulong]),
    "pgx_synth_column_paired": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_uint64,
                                          C.c_uint64, C.c_uint32]),
    "pgx_synth_dict_ids": (C.c_int, [C.c_uint64, C.c_int64, C.c_int32, C.c_void_p]),
    "pgx_pack_fixed_bit": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]),
    "pgx_inverted_index_build": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_uint64,
                                           C.POINTER(C.c_uint64)]),
    "pgx_last_error": (C.c_char_p, []),
    "pgx_abi_version": (C.c_int32, []),
    "pgx_ctx_create": (C.c_int, [C.POINTER(CtxOpts), C.POINTER(C.c_void_p)]),
    "pgx_ctx_destroy": (C.c_int, [C.c_void_p]),
    "pgx_segment_stage": (C.c_int, [C.c_void_p, C.POINTER(SegmentDesc), C.POINTER(C.c_void_p)]),
    "pgx_segment_release": (C.c_int, [C.c_void_p]),
    "pgx_segment_device_bytes": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "pgx_query_compile": (C.c_int, [C.c_void_p, C.POINTER(QueryDesc), C.POINTER(C.c_void_p)]),
    "pgx_query_release": (C.c_int, [C.c_void_p]),
    "pgx_query_set_key_domain": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_void_p, C.c_void_p,
                                           C.c_void_p]),
    "pgx_execute": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(LeafBinding),
                              C.POINTER(ExecOpts), C.POINTER(C.c_void_p)]),
    "pgx_result_release": (C.c_int, [C.c_void_p]),
    "pgx_result_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "pgx_result_agg": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "pgx_result_num_groups": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "pgx_result_group_keys": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "pgx_result_group_values": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "pgx_result_group_mode": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    "pgx_result_trim": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(C.c_int64)]),
    "pgx_result_gather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p]),
    "pgx_query_dense_slots": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(C.c_int64)]),
    "pgx_query_dense_plane_op": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.c_int32,
                                           C.POINTER(C.c_int32)]),
    "pgx_result_from_dense": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.c_void_p,
                                        C.POINTER(C.c_int64), C.POINTER(C.c_void_p)]),
    "pgx_synth_column": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_uint64]),
    "pgx_device_alloc": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "pgx_device_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pgx_copy_to_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "pgx_bind_predicates": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(Predicate),
                                      C.POINTER(C.c_void_p)]),
    "pgx_bindings_array": (C.POINTER(LeafBinding), [C.c_void_p]),
    "pgx_bindings_release": (C.c_int, [C.c_void_p]),
    "pgx_execute_async": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(LeafBinding),
                                    C.POINTER(ExecOpts), C.POINTER(C.c_void_p)]),
    "pgx_result_wait": (C.c_int, [C.c_void_p, C.c_int64]),
    "pgx_execute_multi": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                    C.POINTER(LeafBinding), C.POINTER(ExecOpts), C.POINTER(C.c_void_p)]),
    "pgx_result_device_groups": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_void_p]),
    "pgx_result_record_words": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    "pgx_result_merge_groups": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64),
                                          C.POINTER(C.c_void_p)]),
    "pgx_copy_to_host": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "pgx_execute_timed": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(LeafBinding),
                                    C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_void_p)]),
    "pgx_timing_start": (C.c_int, [C.c_void_p]),
    "pgx_mutable_create": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32, C.POINTER(MutableColumn),
                                     C.POINTER(C.c_void_p)]),
    "pgx_mutable_append": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "pgx_mutable_set_dictionary": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_uint64, C.c_int32,
                                             C.c_int32, C.c_void_p]),
    "pgx_mutable_snapshot": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "pgx_mutable_num_docs": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    "pgx_mutable_release": (C.c_int, [C.c_void_p]),
    "pgx_timing_stop": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_char_p, C.c_uint64]),
}


def lib():
    """Load libpgx.so.  Raises if it is missing -- the GPU path never silently falls back."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libpgx.so not built (%s): run `make` or __graft_entry__.build()" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(status):
    if status != 0:
        raise PgxError(status, lib().pgx_last_error().decode(errors="replace"))
