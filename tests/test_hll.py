"""DISTINCTCOUNTHLL host logic (pinot_amd/hll.py, vectorised) against the oracle's scalar per-offer restatement of
stream-lib 2.7.0 HyperLogLog(log2m = 8) / MurmurHash.hashLong, and the reference's own accuracy contract
(query/aggregation/DistinctCountHLLTest.java:145-171 with TestUtils.assertApproximation: relative error < 0.1 at
cardinalities >= 1000).  Parity of the hash itself is unpinned: stream-lib is a third-party jar absent from the
reference and no test there holds literal HLL registers or hashes."""
import numpy as np

from oracle import pinot_oracle as O
from pinot_amd import hll


def _oracle_regs(values):
    regs = [0] * 256
    for v in values:
        O.hll_offer(regs, int(v))
    return regs


def test_hash_matches_oracle_on_edge_and_random_ints():
    rng = np.random.default_rng(3)
    vals = [0, 1, -1, 2147483647, -2147483648, 12345, -54321] + rng.integers(-2**31, 2**31, 4000).tolist()
    got = hll.hash_long(np.array(vals, dtype=np.int64)).view(np.int32).tolist()
    assert got == [O.murmur_hash_long(v) for v in vals]


def test_registers_match_oracle_and_depend_only_on_the_set():
    rng = np.random.default_rng(4)
    for n in (0, 1, 7, 300, 5000):
        vals = rng.integers(-1000000, 1000000, n).tolist()
        exp = _oracle_regs(vals)  # per-doc offers, duplicates and order as drawn
        got = hll.from_ints(sorted(set(vals)))  # the distinct set, as the GPU histogram yields it
        assert list(got) == exp
        assert hll.cardinality(got) == O.hll_cardinality(exp)


def test_merge_is_union():
    a, b = list(range(0, 3000)), list(range(2000, 9000))
    assert list(hll.merge(hll.from_ints(a), hll.from_ints(b))) == list(hll.from_ints(a + b))
    assert O.combine_two("distinctcounthll", _oracle_regs(a), _oracle_regs(b)) == _oracle_regs(a + b)


def test_small_cardinalities_use_linear_counting():
    for n in (0, 1, 2, 10):
        assert hll.cardinality(hll.from_ints(range(n))) == n
    for n in (50, 200):  # m * ln(m / zeros): register collisions only
        assert abs(hll.cardinality(hll.from_ints(range(n))) - n) <= 0.05 * n


def test_accuracy_contract_of_the_reference():
    rng = np.random.default_rng(5)
    errs = []
    for _ in range(40):
        n = int(rng.integers(1000, 60000))
        xs = np.unique(rng.integers(-2**31, 2**31, n))
        errs.append(hll.cardinality(hll.from_ints(xs.tolist())) / len(xs) - 1.0)
    errs = np.abs(np.array(errs))
    assert np.mean(errs < 0.1) >= 0.8  # 1.04 / sqrt(256) = 6.5% standard error per estimate
    assert errs.mean() < 0.07


def test_java_hash_codes_known_answers():
    """Values the JDK defines: "a".hashCode() = 97, "hello".hashCode() = 99162322, "Aa" and "BB" collide (2112),
    Long.hashCode(1L << 32) = 1, Long.hashCode(-1L) = 0, Float.hashCode(1.0f) = 0x3f800000,
    Double.hashCode(1.0) = 0x3ff00000, Double.hashCode(-0.0) = 0x80000000 (as int)."""
    from pinot_amd.extended import java_hash_code as P
    cases = [("STRING", "a", 97), ("STRING", "hello", 99162322), ("STRING", "Aa", 2112), ("STRING", "BB", 2112),
             ("STRING", "", 0), ("LONG", 1 << 32, 1), ("LONG", -1, 0), ("INT", -5, -5),
             ("FLOAT", 1.0, 0x3F800000), ("DOUBLE", 1.0, 0x3FF00000), ("DOUBLE", -0.0, -0x80000000),
             ("FLOAT", float("nan"), 0x7FC00000)]
    for dt, v, h in cases:
        assert P(dt, v) == h, (dt, v)
        col = O.OColumn("c", dt, np.array([v], dtype=object if dt == "STRING" else None), np.zeros(1, np.int64),
                        True, False, 1)
        assert O.java_hash_code(col, 0) == h, (dt, v)


def test_serialized_form_size_and_round_trip():
    """HllFieldSizeTest: getBytes() of a log2m = 8 estimator is HllUtil.getHllFieldSizeFromLog2m(8) = 180 bytes; the
    STRING form (char = byte + 129) round-trips through the oracle's independent decoder."""
    rng = np.random.default_rng(6)
    for n in (0, 1, 50, 20000):
        regs = hll.from_ints(rng.integers(-2**31, 2**31, n).tolist())
        b = hll.to_bytes(regs)
        assert len(b) == 180 and b[:8] == bytes([0, 0, 0, 8, 0, 0, 0, 172])
        s = hll.to_string(regs)
        assert all(1 <= ord(c) <= 256 for c in s)
        assert list(hll.from_string(s)) == list(regs)
        assert O.hll_from_string(s) == list(regs)
