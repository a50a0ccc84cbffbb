"""The opt-in persistent code-object cache of the query compiler (pgx_jit.cpp, PGX_JIT_CACHE=<dir>): a first process
compiles the query's kernel with hiprtc and stores the code object; a second process with the same cache loads it from
disk (no new file, same result).  Without PGX_JIT_CACHE nothing is written."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, sys, time
import numpy as np
sys.path.insert(0, %(root)r)
from pinot_amd import engine as E, pql
from tests import helpers as H
rng = np.random.default_rng(3)
raw = {"a": rng.integers(0, 5000, 50000).astype(np.int32), "g": rng.integers(0, 37, 50000).astype(np.int32),
       "m": rng.integers(0, 1000, 50000).astype(np.int32)}
seg, _ = H.build_pair("jc", raw)
ctx = E.Context(0)
g = E.IndexSegment(ctx, seg)
q = pql.compile("SELECT SUM(m), COUNT(*) FROM t WHERE a > 1234 GROUP BY g")
t = time.time()
blk = E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan([g], q).execute()
dt = time.time() - t
print(json.dumps({"map": blk.get_aggregation_group_by_result().as_map(), "s": dt}))
"""


def _run(env):
    out = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT}], env=env, cwd=ROOT, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_persistent_code_object_cache(tmp_path):
    env = dict(os.environ)
    env["PGX_JIT_CACHE"] = str(tmp_path)
    first = _run(env)
    files = sorted(os.listdir(tmp_path))
    assert files and all(f.startswith("pgxq_") and f.endswith(".co") for f in files)
    second = _run(env)
    assert sorted(os.listdir(tmp_path)) == files  # loaded from disk: nothing new compiled
    assert second["map"] == first["map"]
    env.pop("PGX_JIT_CACHE")
    other = tmp_path / "unused"
    other.mkdir()
    env["HOME"] = str(other)
    assert _run(env)["map"] == first["map"]
    ours = [f for _, _, fs in os.walk(other) for f in fs if f.startswith("pgxq_")]
    assert not ours  # opt-in: no code object of ours written without PGX_JIT_CACHE (the runtime keeps its own caches)
