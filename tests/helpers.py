"""Shared test helpers: build the same segment for the oracle (logical columns) and for the GPU path (v1 bytes)."""
import json
import os

import numpy as np

from oracle import pinot_oracle as O
from pinot_amd import segment as S

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def load_expected():
    return json.load(open(os.path.join(GOLD, "expected_sv_queries.json")))


def sv_raw():
    return dict(np.load(os.path.join(GOLD, "test_data_sv.npz")))


def build_pair(name, raw, inverted=(), types=None, column_types=None):
    """(SegmentData for the GPU, OSegment for the oracle) from raw column values."""
    cols = []
    for c, vals in raw.items():
        dt = (types or {}).get(c)
        ct = (column_types or {}).get(c, "DIMENSION")
        cols.append(S.make_column(c, vals, data_type=dt, column_type=ct, inverted=c in inverted))
    seg = S.make_segment(name, cols)
    oseg = O.OSegment.from_raw(raw, inverted=inverted, dtypes=types)
    return seg, oseg


def oracle_answer(osegs, q, literal=False):
    """Combined oracle answer for a query over one or more segments."""
    if q.get("group_by"):
        parts = [O.run_group_by(s, q, literal_filter=literal) for s in osegs]
        if len(parts) == 1:
            p = parts[0]
            m = {p["string_key"](k): v for k, v in p["map"].items()}
            order = [p["string_key"](k) for k in p["order"]] if p["order"] is not None else None
            return {"map": m, "order": order, "mode": p["mode"], "stats": p["stats"]}
        c = O.combine_group_by(parts, q)
        return {"map": c["merged"], "order": None, "mode": None, "stats": c["stats"], "trimmed": c["trimmed"]}
    parts = [O.run_aggregation(s, q, literal_filter=literal) for s in osegs]
    c = O.combine_aggregation(parts, q)
    return {"results": c["results"], "stats": c["stats"]}


def assert_values_equal(got, exp, fns, rel=0.0):
    assert len(got) == len(exp)
    for g, e, f in zip(got, exp, fns):
        if f in ("avg", "avgmv"):
            assert g[1] == e[1], (g, e)
            _close(g[0], e[0], rel)
        elif f in ("count", "countmv"):
            assert int(g) == int(e), (g, e)
        else:
            _close(g, e, rel)


def _close(a, b, rel):
    if rel == 0.0 or not np.isfinite(b):
        assert a == b, (a, b)
    else:
        assert abs(a - b) <= rel * max(1.0, abs(b)), (a, b)


def literal_entries(osegs, q):
    """numEntriesScannedInFilter summed over segments, from the oracle's literal iterator algebra."""
    if not q.get("filter"):
        return 0
    return int(sum(O.filter_docs(s, q["filter"])[1] for s in osegs))
