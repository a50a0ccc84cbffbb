"""CPU checks of the synthetic workloads bench.py measures (pinot_amd/synth.py): the dictionary kinds are what the
partitioned path and the C twin assume (sorted, distinct, exact), and the extra C3 shapes (c3d, c3m2, c3f) keep C3's
keys and rows so their bench lines compare with C3's."""
import numpy as np

from pinot_amd import synth


def test_metric_dictionaries_sorted_distinct():
    for kind in ("metric", "metric_seg"):
        for seg in (0, 1, 7):
            d = synth.make_dictionary(kind, 65536, seg)
            assert d.dtype == np.int64 and np.all(np.diff(d) > 0) and d[0] >= 0 and d[-1] < (1 << 20)
    assert not np.array_equal(synth.make_dictionary("metric_seg", 65536, 0),
                              synth.make_dictionary("metric_seg", 65536, 1))
    # the shared kind ignores the segment
    assert np.array_equal(synth.make_dictionary("metric", 4096, 0), synth.make_dictionary("metric", 4096, 5))


def test_double_metric_dictionary_exact():
    """metric_f64_seg = metric_seg / 8: sorted, distinct, exactly representable (multiples of 1/8 below 2^17), so sums
    of up to 2^36 of them are exact in any order (the c3f parity test compares exactly)."""
    for seg in (0, 3):
        d = synth.make_dictionary("metric_f64_seg", 65536, seg)
        i = synth.make_dictionary("metric_seg", 65536, seg)
        assert d.dtype == np.float64 and np.all(np.diff(d) > 0)
        assert np.array_equal(d * 8.0, i.astype(np.float64))
        assert d.max() < (1 << 17)


def test_c3_variants_share_c3_keys_and_rows():
    c3 = synth.WORKLOADS["c3"]
    for name, metric_kinds in (("c3d", ["metric_seg"]), ("c3m2", ["metric", "metric"]), ("c3f", ["metric_f64_seg"])):
        wl = synth.WORKLOADS[name]
        assert (wl.segments, wl.rows, wl.npairs, wl.seed) == (c3.segments, c3.rows, c3.npairs, c3.seed)
        assert [(c.name, c.card, c.paired) for c in wl.columns[:2]] == [(c.name, c.card, c.paired) for c in c3.columns[:2]]
        assert [c.dict_kind for c in wl.columns[2:]] == metric_kinds
        assert "GROUP BY g1, g2" in wl.query
