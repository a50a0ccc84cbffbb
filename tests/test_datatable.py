"""DataTable wire format (pinot_amd/datatable.py): the server -> broker bytes of
common/utils/DataTable.java:315-482 with the custom object ser/de of core/util/DataTableCustomSerDe.java.

Pinned by the layout rules of the reference's writer (52-byte header of (start, length) pairs, section order, DataSchema
type names, fixed cell widths, version-2 object type ids), JDK known answers (String.hashCode) and the reduce: the
BrokerReduceServiceTest goldens reproduce when every server response crosses the wire as DataTable bytes."""
import struct

import numpy as np
import pytest

from pinot_amd import broker as B
from pinot_amd import datatable as D
from pinot_amd import pql
from tests import helpers as H
from tests.test_broker import BASIC, GROUPED, MULTI, _by_fn, _oracle_response, osegs  # noqa: F401


def _header(b):
    return struct.unpack_from(">13i", b, 0)


def test_java_string_hash_known_answers():
    assert D.java_string_hash("") == 0
    assert D.java_string_hash("hello") == 99162322
    assert D.java_string_hash("Aa") == D.java_string_hash("BB") == 2112
    assert D.java_string_hash("polygenelubricants") == -2147483648  # Integer.MIN_VALUE
    assert D.java_string_hash("été") == 0xE9 * 961 + 0x74 * 31 + 0xE9


def test_hashmap_order_is_bucket_then_insertion():
    keys = ["k%d" % i for i in range(100)]
    order = D.java_hashmap_order(keys)
    assert sorted(order) == sorted(keys)
    cap = 256  # 100 entries > 0.75 * 128
    buckets = [((D.java_string_hash(k) & 0xFFFFFFFF) ^ ((D.java_string_hash(k) & 0xFFFFFFFF) >> 16)) & (cap - 1)
               for k in order]
    assert buckets == sorted(buckets)
    assert D.java_hashmap_order(["Aa", "BB"]) == ["Aa", "BB"] and D.java_hashmap_order(["BB", "Aa"]) == ["BB", "Aa"]


def test_exception_only_table_layout():
    """DataTable() + addException: no dictionary, no schema, no rows; metadata "Exception<code>" (DataTable.java:856-861)
    plus the four statistics attachMetadataToDataTable always writes (IntermediateResultsBlock.java:163-178), in
    HashMap order."""
    resp = B.InstanceResponse(exceptions={200: "boom"}, stats=[5, 6, 7, 8])
    b = D.response_to_datatable(pql.compile(BASIC), resp)
    h = _header(b)
    entries = {"numDocsScanned": "5", "numEntriesScannedInFilter": "6", "numEntriesScannedPostFilter": "7",
               "totalDocs": "8", "Exception200": "boom"}
    meta = struct.pack(">i", 5) + b"".join(struct.pack(">i", len(k)) + k.encode() + struct.pack(">i", len(entries[k]))
                                           + entries[k].encode() for k in D.java_hashmap_order(list(entries)))
    assert h == (2, 0, 0, 52, 0, 52, len(meta), 52 + len(meta), 0, 52 + len(meta), 0, 52 + len(meta), 0)
    assert b[52:] == meta
    back = D.datatable_to_response(pql.compile(BASIC), b)
    assert back.exceptions == {200: "boom"} and back.aggregation is None and back.group_by is None
    assert back.stats == [5, 6, 7, 8]


def test_mv_functions_use_their_base_functions_cells():
    """countmv / summv / minmv / maxmv / avgmv are the Count / Sum / Min / Max / Avg functions
    (AggregationFunctionRegistry.java:76-80): LONG, DOUBLE cells and an AvgPair object, read back as the same values."""
    q = pql.compile("SELECT COUNTMV(mv), SUMMV(mv), MINMV(mv), MAXMV(mv), AVGMV(mv) FROM t")
    resp = B.InstanceResponse(aggregation=[7, 21.0, 1.0, 6.0, (21.0, 7)], stats=[3, 0, 3, 10])
    b = D.response_to_datatable(q, resp)
    dt = D.DataTable.from_bytes(b)
    assert dt.types == ["LONG", "DOUBLE", "DOUBLE", "DOUBLE", "OBJECT"]
    back = D.datatable_to_response(q, b)
    assert back.aggregation == [7, 21.0, 1.0, 6.0, (21.0, 7)]
    assert isinstance(back.aggregation[0], int)
    red = B.BrokerReduceService().reduce_on_data_table(q, {"x": b, "y": b})
    assert red == B.BrokerReduceService().reduce_on_data_table(q, {"x": resp, "y": resp})


def test_aggregation_table_layout_and_values():
    q = pql.compile(BASIC)
    resp = B.InstanceResponse(aggregation=[3, 6.5, 3.25, -1.0, (6.5, 3)], stats=[3, 7, 12, 10])
    b = D.response_to_datatable(q, resp)
    h = _header(b)
    assert h[:3] == (2, 1, 5)
    ds, dl, ms, ml, ss, sl, fs, fl, vs, vl = h[3:]
    assert (ds, dl) == (52, 4) and b[52:56] == b"\0\0\0\0"  # empty reverse dictionary: its count only
    assert ms == 56 and ss == ms + ml and fs == ss + sl and vs == fs + fl and len(b) == vs + vl
    names = ["count_star", "sum_met", "max_met", "min_met", "avg_met"]
    types = ["LONG", "DOUBLE", "DOUBLE", "DOUBLE", "OBJECT"]
    schema = struct.pack(">i", 5) + b"".join(struct.pack(">i", len(n)) + n.encode() for n in names) + \
        b"".join(struct.pack(">i", len(t)) + t.encode() for t in types)
    assert b[ss:ss + sl] == schema
    assert fl == 40 and b[fs:fs + 32] == struct.pack(">qddd", 3, 6.5, 3.25, -1.0)
    assert struct.unpack_from(">ii", b, fs + 32) == (0, 16)  # (offset, length) of the AvgPair in the variable data
    assert b[vs:vs + vl] == struct.pack(">i", D.T_AVG_PAIR) + struct.pack(">dq", 6.5, 3)
    meta = D.DataTable.from_bytes(b).metadata
    assert meta == {"numDocsScanned": "3", "numEntriesScannedInFilter": "7", "numEntriesScannedPostFilter": "12",
                    "totalDocs": "10"}
    back = D.datatable_to_response(q, b)
    assert back.aggregation == [3, 6.5, 3.25, -1.0, (6.5, 3)] and back.stats == [3, 7, 12, 10]


def test_group_by_table_holds_function_names_and_maps(osegs):  # noqa: F811
    q = pql.compile(GROUPED)
    resp = _oracle_response(q, osegs)
    b = D.response_to_datatable(q, resp)
    dt = D.DataTable.from_bytes(b)
    assert dt.columns == ["functionName", "GroupByResultMap"] and dt.types == ["STRING", "OBJECT"]
    assert [r[0] for r in dt.rows] == ["sum_met", "count_star", "min_met", "avg_met"]
    back = D.datatable_to_response(q, b)
    assert len(back.group_by) == 4
    for a, m_in, m_out in zip(q["aggregations"], resp.group_by, back.group_by):
        assert set(m_in) == set(m_out)
        for k in m_in:
            exp = m_in[k]
            if a["fn"] == "avg":
                assert m_out[k] == (float(exp[0]), int(exp[1]))
            else:
                assert m_out[k] == float(exp)


def test_reduce_over_datatable_bytes_matches_reference_goldens(osegs):  # noqa: F811
    """BrokerReduceServiceTest (2 and 10 servers) with every response serialized and parsed back."""
    exp = H.load_expected()["broker_reduce"]
    q = pql.compile(MULTI)
    wire = D.response_to_datatable(q, _oracle_response(q, osegs))
    for n, key in ((2, "servers_2"), (10, "servers_10")):
        resp = B.BrokerReduceService().reduce_on_data_table(q, {"s%d" % i: wire for i in range(n)})
        got = _by_fn(resp)
        for fn, v in exp[key].items():
            assert float(got[fn]) == float(v), (fn, got[fn], v)
        assert resp.num_docs_scanned == n * 400002


def test_group_by_reduce_same_through_the_wire(osegs):  # noqa: F811
    q = pql.compile(GROUPED)
    obj = _oracle_response(q, osegs)
    wire = D.response_to_datatable(q, obj)
    a = B.BrokerReduceService().reduce_on_data_table(q, {"x": obj, "y": obj})
    b = B.BrokerReduceService().reduce_on_data_table(q, {"x": wire, "y": wire})
    assert a == b


@pytest.mark.parametrize("text", ["SELECT DISTINCTCOUNT(dim0), DISTINCTCOUNTHLL(dim0), MINMAXRANGE(met), "
                                  "PERCENTILE90(met) FROM midas",
                                  "SELECT DISTINCTCOUNT(dim1), MINMAXRANGE(met) FROM midas GROUP BY dim0 TOP 3",
                                  "SELECT PERCENTILEEST90(met), PERCENTILEEST50(met) FROM midas"])
def test_extended_intermediates_round_trip(osegs, text):  # noqa: F811
    """IntOpenHashSet, HyperLogLog (stream-lib bytes), MinMaxRangePair, DoubleArrayList and QuantileDigest objects."""
    q = pql.compile(text)
    obj = _oracle_response(q, osegs)
    wire = D.response_to_datatable(q, obj)
    a = B.BrokerReduceService().reduce_on_data_table(q, {"x": obj, "y": obj})
    b = B.BrokerReduceService().reduce_on_data_table(q, {"x": wire, "y": wire})
    assert a == b


def test_custom_serde_object_bytes():
    assert D.serialize_object(2.5) == struct.pack(">d", 2.5)
    assert D.serialize_object(D.MinMaxRangePair((1.0, 4.0))) == struct.pack(">dd", 1.0, 4.0)
    assert D.serialize_object([1.0, 2.0]) == struct.pack(">idd", 2, 1.0, 2.0)
    assert D.serialize_object({3, 1}) == struct.pack(">iii", 2, 1, 3)
    m = D.serialize_object({"a": 1.0})
    assert m == struct.pack(">iiii", 1, D.T_STRING, D.T_DOUBLE, 1) + b"a" + struct.pack(">i", 8) + struct.pack(">d", 1.0)
    assert D.deserialize_object(m, D.T_HASHMAP) == {"a": 1.0}
    assert D.deserialize_object(b"", D.T_HASHMAP) == {}
    with pytest.raises(ValueError):
        D.deserialize_object(b"\xac\xed", D.T_OBJECT)
