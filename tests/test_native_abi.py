"""CPU-side checks of the C-ABI boundary: libpgx.so loads and exports every symbol include/pgx.h declares
(no compute calls -- there is no GPU in the build container)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "pgx.h")
LIB = os.path.join(ROOT, "pinot_amd", "libpgx.so")


def declared_symbols():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pgx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("pgx_ctx_create", "pgx_segment_stage", "pgx_query_compile", "pgx_execute", "pgx_result_stats",
              "pgx_result_group_values", "pgx_result_trim", "pgx_last_error"):
        assert s in syms


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpgx.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    lib.pgx_abi_version.restype = ctypes.c_int32
    assert lib.pgx_abi_version() == 8


def test_binding_table_matches_header():
    from pinot_amd import native
    assert set(native.EXPORTS) <= set(declared_symbols())
    assert set(declared_symbols()) <= set(native.EXPORTS)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpgx.so not built")
def test_query_compiler_shapes_compile_for_gfx950():
    """The query compiler's generated kernels (every bit width, leaf kind, program op, aggregation, group mode and
    value-image kind) compile with hiprtc for gfx950 -- checked here without a device."""
    from pinot_amd import native
    n = ctypes.c_int()
    log = ctypes.create_string_buffer(1 << 16)
    failed = native.lib().pgx_jit_selftest(ctypes.byref(n), log, len(log))
    assert n.value >= 15
    assert failed == 0, log.value.decode(errors="replace")
