"""QuantileDigest restatement (pinot_amd/qdigest.py; the reference vendors it as
core/query/aggregation/function/quantile/digest/QuantileDigest.java): the getQuantile rank-error contract at maxError
0.05, structural invariants (the reference's validate(): node weights sum to the count, node counts match), the
DataOutput byte layout and its round trip, merge, and the histogram construction the GPU path uses."""
import struct

import numpy as np
import pytest

from pinot_amd import qdigest as QD


def _rank_ok(values, x, q, err=0.05):
    n = len(values)
    lo, hi = np.searchsorted(values, x, side="left"), np.searchsorted(values, x, side="right")
    return lo - err * n - 1 <= q * n <= hi + err * n + 1


def _validate(d):
    nodes = d._post_order()
    assert abs(sum(n.w for n in nodes) - d.weighted_count) < 1e-5
    assert len(nodes) == d.total_nodes
    assert sum(n.w >= QD.ZERO_WEIGHT_THRESHOLD for n in nodes) == d.nonzero_nodes


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_quantiles_within_the_error_bound(seed):
    rng = np.random.default_rng(seed)
    vals = np.concatenate([rng.integers(-10 ** 6, 10 ** 6, 20000), rng.integers(0, 50, 5000)])
    d = QD.QuantileDigest()
    for v in vals.tolist():
        d.add(int(v))
    _validate(d)
    s = np.sort(vals)
    for q in (0.0, 0.5, 0.9, 0.95, 0.99, 1.0):
        assert _rank_ok(s, d.get_quantile(q), q)
    assert d.count == len(vals) and d.min == int(s[0]) and d.max == int(s[-1])


def test_histogram_digest_and_merge_within_bound():
    rng = np.random.default_rng(7)
    a = rng.integers(0, 3000, 40000)
    b = rng.integers(1000, 9000, 30000)
    ha = list(zip(*np.unique(a, return_counts=True)))
    hb = list(zip(*np.unique(b, return_counts=True)))
    da, db = QD.from_histogram(ha), QD.from_histogram(hb)
    _validate(da)
    m = QD.merge_all([da, db])
    _validate(m)
    s = np.sort(np.concatenate([a, b]))
    for q in (0.5, 0.9, 0.95, 0.99):
        assert _rank_ok(s, m.get_quantile(q), q)


def test_serialize_layout_and_round_trip():
    d = QD.QuantileDigest()
    for v in (5, 5, 7, -3, 1 << 40):
        d.add(v)
    b = d.serialize()
    max_error, alpha, landmark, mn, mx, total = struct.unpack_from(">ddqqqi", b, 0)
    assert (max_error, alpha, mn, mx, total) == (0.05, 0.0, -3, 1 << 40, d.total_nodes)
    assert len(b) == struct.calcsize(">ddqqqi") + total * 18  # flags, level, bits, weight per node
    e = QD.QuantileDigest.deserialize(b)
    assert e.serialize() == b
    for q in (0.1, 0.5, 0.99):
        assert e.get_quantile(q) == d.get_quantile(q)


def test_empty_digest_answers_its_max():
    # getQuantiles without nodes falls through to `max` (Long.MIN_VALUE for an empty digest)
    assert QD.QuantileDigest().get_quantile(0.5) == -(1 << 63)
