"""The on-disk format pinned against the reference's own Java-written fixtures and test vectors (CPU).

* starTreeSegment.tar.gz (pinot-core/src/test/resources/data): a v1 segment written by the Java creator.  Loaded with
  segment.load_segment: every dictId below its cardinality, sorted INT dictionaries, raw sum(m1) = 1634 and the
  aggregated doc (d1-v0, ALL, ALL) holding m1 = 1294 = raw sum(m1) where d1 = 'd1-v0' (SURVEY Appendix A).
* paddingOld / paddingPercent / paddingNull.tar.gz: string-dictionary padding, asserted exactly as
  LoadersTest.testPadding (core/segment/index/loader/LoadersTest.java:146-200) asserts it.
* SortedRangeIntersectionTest (core/util/SortedRangeIntersectionTest.java:45-80): the fixed vectors, on the oracle's
  restatement of SortedRangeIntersection.intersectSortedRangeSets.
"""
import json
import os
import tarfile

import numpy as np
import pytest

from oracle import pinot_oracle as O
from pinot_amd import engine as E
from pinot_amd import segment as S
from tests import helpers as H


def _untar(name, tmp_path):
    with tarfile.open(os.path.join(H.GOLD, name)) as t:
        t.extractall(tmp_path, filter="data")
    return str(tmp_path)


@pytest.fixture(scope="module")
def star_seg(tmp_path_factory):
    d = _untar("starTreeSegment.tar.gz", tmp_path_factory.mktemp("st"))
    return S.load_segment(os.path.join(d, "starTreeSegment"))


def test_star_tree_fixture_layout(star_seg):
    seg = star_seg
    assert seg.total_docs == 1031 and seg.total_raw_docs == 1000
    for c in seg.columns.values():
        ids = c.dict_ids()
        assert len(ids) == seg.total_docs
        assert ids.min() >= 0 and ids.max() < c.cardinality
        v = c.dictionary_values()
        if c.data_type == "INT":
            assert np.all(np.diff(np.asarray(v, dtype=np.int64)) > 0)
        else:
            assert list(v) == sorted(v)
    # '%' padding (no padding key in the metadata: legacy), the star value "ALL" in every star-tree dimension
    assert seg.columns["d1"].pad_char == "%" and seg.columns["d1"].dictionary_values()[0] == "ALL"


def test_star_tree_fixture_sums(star_seg):
    seg = star_seg
    m1 = seg.columns["m1"]
    vals = np.asarray(m1.dictionary_values(), dtype=np.int64)[m1.dict_ids()]
    assert vals[:seg.total_raw_docs].sum() == 1634
    dims = {n: np.asarray(seg.columns[n].dictionary_values(), dtype=object)[seg.columns[n].dict_ids()]
            for n in ("d1", "d2", "d3")}
    agg = [r for r in range(seg.total_raw_docs, seg.total_docs)
           if dims["d1"][r] == "d1-v0" and dims["d2"][r] == "ALL" and dims["d3"][r] == "ALL"]
    assert len(agg) == 1 and vals[agg[0]] == 1294
    raw = np.arange(seg.total_raw_docs)
    assert vals[raw[dims["d1"][:seg.total_raw_docs] == "d1-v0"]].sum() == 1294


def test_star_tree_fixture_roundtrip(star_seg, tmp_path):
    """Writing the loaded segment back gives byte-identical index files."""
    d = S.write_segment(star_seg, str(tmp_path))
    again = S.load_segment(d)
    for n, c in star_seg.columns.items():
        a = again.columns[n]
        assert a.dict_bytes == c.dict_bytes and a.fwd_bytes == c.fwd_bytes and a.sorted_bytes == c.sorted_bytes
        assert a.pad_char == c.pad_char


@pytest.mark.parametrize("name,pad,values,lookups", [
    ("paddingOld", "%", ["lynda 2.0", "lynda"], {"lynda%": 1, "lynda%%": 1}),
    ("paddingPercent", "%", ["lynda 2.0", "lynda"], {"lynda%": 1, "lynda%%": 1}),
    ("paddingNull", "\0", ["lynda", "lynda 2.0"], {"lynda\0": 0, "lynda\0\0": 0}),
])
def test_string_padding(tmp_path, name, pad, values, lookups):
    d = _untar(name + ".tar.gz", tmp_path)
    seg = S.load_segment(os.path.join(d, name))
    c = seg.columns["name"]
    assert c.pad_char == pad                       # ColumnMetadata.getPaddingCharacter
    raw = [c.dict_bytes[i * c.dict_width:(i + 1) * c.dict_width].decode() for i in range(c.cardinality)]
    assert raw[1 if pad == "%" else 0] == "lynda" + pad * 4  # StringDictionary.getStringValue
    assert c.dictionary_values() == values         # StringDictionary.get
    info = E._ColInfo(c, c.dictionary_values())
    for k, v in lookups.items():                   # StringDictionary.indexOf pads the lookup with the padding char
        assert info.index_of(k) == v


def test_writer_records_padding(tmp_path):
    for pad in ("\0", "%"):
        col = S.make_column("s", np.array(["ab", "abc", "b"]), pad=pad)
        seg = S.make_segment("p" + str(ord(pad)), [col])
        again = S.load_segment(S.write_segment(seg, str(tmp_path)))
        assert again.columns["s"].pad_char == pad
        assert again.columns["s"].dictionary_values() == col.dictionary_values()


def test_sorted_range_intersection_vectors():
    j = json.load(open(os.path.join(H.GOLD, "sorted_range_intersection.json")))
    assert O.intersect_sorted_range_sets(j["simple"]["sets"]) == j["simple"]["expected"]
    assert O.intersect_sorted_range_sets(j["complex"]["sets"]) == j["complex"]["expected"]
    # against the set-based brute force the reference test describes
    docs = set.intersection(*[{d for a, b in s for d in range(a, b + 1)} for s in j["complex"]["sets"]])
    got = {d for a, b in j["complex"]["expected"] for d in range(a, b + 1)}
    assert docs == got


def test_sorted_range_intersection_random():
    rng = np.random.default_rng(3)
    for _ in range(200):
        sets = []
        for _k in range(rng.integers(2, 5)):
            cuts = np.sort(rng.choice(400, size=2 * rng.integers(1, 8), replace=False))
            sets.append([[int(cuts[i]), int(cuts[i + 1])] for i in range(0, len(cuts), 2)])
        got = O.intersect_sorted_range_sets(sets)
        want = set.intersection(*[{d for a, b in s for d in range(a, b + 1)} for s in sets])
        assert {d for a, b in got for d in range(a, b + 1)} == want
