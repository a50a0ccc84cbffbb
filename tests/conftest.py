import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

_TIMES = os.environ.get("PGX_TEST_TIMES")  # optional: append "<elapsed>\t<seconds>\t<phase>\t<outcome>\t<id>" per phase
_T0 = time.time()
# The generated query kernels' persistent code-object cache (pgx_jit.cpp cache_load / cache_store: a file per FNV-1a of
# the generated source + compile options, checked by a second hash on load).  The GPU suite compiles ~500 distinct
# query shapes (~0.4 s of hiprtc each); tests/_jitcache holds the code objects an earlier run on the GPU box compiled
# from the same sources, so those shapes load instead of compiling.  A shape whose source changed misses and compiles.
os.environ.setdefault("PGX_JIT_CACHE", os.path.join(ROOT, "tests", "_jitcache"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


def pytest_runtest_logreport(report):
    if _TIMES:
        with open(_TIMES, "a") as f:
            f.write("%.2f\t%.2f\t%s\t%s\t%s\n" % (time.time() - _T0, report.duration, report.when, report.outcome,
                                                  report.nodeid))
