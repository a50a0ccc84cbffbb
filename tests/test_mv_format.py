"""Multi-value forward index (v1 <col>.mv.fwd, io/writer/impl/v1/FixedBitMultiValueWriter.java and the reader of the same
package): chunk-offset header, doc-start bitset, fixed-bit values.  CPU tests of the writer / reader restatement and
the oracle's MV semantics (MVScanDocIdIterator with the evaluators' apply(int[]), *MVAggregationFunction)."""
import struct

import numpy as np

from oracle import pinot_oracle as O
from pinot_amd import pql
from pinot_amd import segment as S


def test_docs_per_chunk_uses_the_integer_average():
    # float averageValuesPerDoc = totalNumValues / numDocs: 25 values over 10 docs average 2 (not 2.5)
    assert S.mv_docs_per_chunk(10, 25) == 1024
    assert S.mv_docs_per_chunk(10, 10) == 2048
    assert S.mv_docs_per_chunk(3, 30) == 205  # ceil(2048 / 10.0)


def test_layout_of_a_small_column():
    docs = [[1, 2], [3], [0, 1, 2, 3], [2]]
    buf = S.pack_mv_fwd(docs, 2)
    # 8 values / 4 docs -> average 2 -> 1024 docs per chunk -> one chunk offset (0)
    assert buf[:4] == struct.pack(">i", 0)
    # doc starts at value positions 0, 2, 3, 7: MSB-first bits of one byte
    assert buf[4] == 0b10110001
    # raw values 1,2,3,0,1,2,3,2 at 2 bits each, MSB-first
    assert buf[5:7] == bytes([0b01101100, 0b01101110])
    starts, off = S.mv_layout(buf, 4, 8)
    assert starts.tolist() == [0, 2, 3, 7, 8] and off == 5


def test_column_round_trip_through_a_segment_directory(tmp_path):
    rng = np.random.default_rng(3)
    docs = [rng.integers(-50, 50, rng.integers(1, 6)).tolist() for _ in range(3000)]
    col = S.make_mv_column("tags", docs, "INT", inverted=True)
    seg = S.make_segment("mv", [col, S.make_column("m", rng.integers(0, 9, 3000).astype(np.int32))])
    back = S.load_segment(S.write_segment(seg, str(tmp_path)))
    c = back.columns["tags"]
    assert c.is_mv and c.total_entries == sum(len(d) for d in docs) and c.max_mv == max(len(d) for d in docs)
    dictionary = c.dictionary_values()
    got = [dictionary[ids].tolist() for ids in c.mv_dict_ids()]
    assert got == docs
    for k in (0, 17, len(dictionary) - 1):  # inverted index: every doc holding the value
        exp = [d for d, v in enumerate(docs) if dictionary[k] in v]
        assert S.inverted_index_docs(c.inv_bytes, c.cardinality, k).tolist() == exp


def test_oracle_mv_predicates_and_functions():
    rng = np.random.default_rng(4)
    docs = [rng.integers(0, 9, rng.integers(1, 4)).tolist() for _ in range(400)]
    m = rng.integers(0, 100, 400).astype(np.int32)
    for inverted in ((), ("t",)):
        seg = O.OSegment.from_raw({"t": docs, "m": m}, inverted=inverted)
        r = O.run_aggregation(seg, pql.compile("SELECT COUNT(*) FROM x WHERE t <> 3"))
        assert r["results"][0] == sum(3 not in d for d in docs)  # NO value equals 3
        r = O.run_aggregation(seg, pql.compile("SELECT COUNT(*) FROM x WHERE t IN (3, 4)"))
        assert r["results"][0] == sum(bool({3, 4} & set(d)) for d in docs)  # ANY value in the set
        r = O.run_aggregation(seg, pql.compile("SELECT COUNTMV(t), SUMMV(t), MINMV(t), MAXMV(t), AVGMV(t) FROM x "
                                               "WHERE m > 50"))
        sel = [d for d, mm in zip(docs, m) if mm > 50]
        flat = [v for d in sel for v in d]
        assert r["results"] == [len(flat), float(sum(flat)), float(min(flat)), float(max(flat)),
                                (float(sum(flat)), len(flat))]
        # the MV scan leaf counts one entry per doc it visits (MVScanDocIdIterator.next)
        r = O.run_aggregation(seg, pql.compile("SELECT COUNT(*) FROM x WHERE t BETWEEN 2 AND 4"))
        assert r["stats"][1] == 400
