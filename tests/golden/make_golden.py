"""Generate the golden fixtures under tests/golden/ from the reference's own test data files.

This script runs ONLY in the build container (where /root/reference exists).  It reads the
reference's Avro fixtures as DATA (a tiny pure-Python Avro reader, codec "null"), converts the
columns the reference tests use into numpy arrays, and writes them as .npz fixtures next to a
JSON file holding the expected values asserted by the reference's own Java tests:

  * pinot-core/src/test/resources/data/test_data-sv.avro
      used by pinot-core/src/test/java/com/linkedin/pinot/queries/BaseSingleValueQueriesTest.java:62-110
      expected values: .../queries/AggregationSingleValueQueriesTest.java:43-221
  * pinot-core/src/test/resources/data/simpleData200001.avro
      used by .../query/executor/QueryExecutorTest.java:57,97-200 (2 segments)
      and     .../query/executor/BrokerReduceServiceTest.java:138-421
  * pinot-core/src/test/resources/data/starTreeSegment.tar.gz (Java-written v1 segment, bytes
      copied verbatim as a data fixture: it pins the on-disk format)

Null handling follows FieldSpec defaults (pinot-common/.../data/FieldSpec.java:37-47):
INT dimension/time null -> Integer.MIN_VALUE, INT metric null -> 0, STRING null -> "null".

Nothing here is imported by the product; the .npz / .json outputs are committed.
"""
import io
import json
import os
import shutil
import struct
import sys

import numpy as np

REF = "/root/reference/pinot-core/src/test/resources/data"
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------------------------
# Minimal Avro object-container reader (spec 1.7, codec "null" only)
# ----------------------------------------------------------------------------------------------
class _Buf:
    def __init__(self, data):
        self.d = data
        self.p = 0

    def long(self):
        shift = 0
        acc = 0
        while True:
            b = self.d[self.p]
            self.p += 1
            acc |= (b & 0x7F) << shift
            shift += 7
            if not (b & 0x80):
                break
        return (acc >> 1) ^ -(acc & 1)

    def bytes_(self):
        n = self.long()
        v = self.d[self.p:self.p + n]
        self.p += n
        return v

    def raw(self, n):
        v = self.d[self.p:self.p + n]
        self.p += n
        return v


def read_avro(path):
    data = open(path, "rb").read()
    b = _Buf(data)
    assert b.raw(4) == b"Obj\x01"
    meta = {}
    while True:
        n = b.long()
        if n == 0:
            break
        if n < 0:
            b.long()
            n = -n
        for _ in range(n):
            k = b.bytes_().decode()
            meta[k] = b.bytes_()
    codec = meta.get("avro.codec", b"null").decode()
    assert codec == "null", codec
    schema = json.loads(meta["avro.schema"])
    sync = b.raw(16)
    fields = []
    for f in schema["fields"]:
        t = f["type"]
        if isinstance(t, list):
            fields.append((f["name"], t))
        else:
            fields.append((f["name"], [t]))
    cols = {name: [] for name, _ in fields}
    while b.p < len(data):
        count = b.long()
        b.long()  # block size in bytes
        for _ in range(count):
            for name, types in fields:
                if len(types) > 1:
                    t = types[b.long()]
                else:
                    t = types[0]
                if t == "null":
                    v = None
                elif t in ("int", "long"):
                    v = b.long()
                elif t == "string":
                    v = b.bytes_().decode("utf-8")
                else:
                    raise ValueError(t)
                cols[name].append(v)
        assert b.raw(16) == sync
    return cols


INT_MIN = -(1 << 31)


def _int_col(vals, metric):
    null = 0 if metric else INT_MIN
    return np.array([null if v is None else v for v in vals], dtype=np.int32)


def _str_col(vals):
    return np.array([("null" if v is None else v).encode("utf-8") for v in vals])


def make_sv():
    cols = read_avro(os.path.join(REF, "test_data-sv.avro"))
    # Schema of BaseSingleValueQueriesTest.java:89-101
    metrics = ["column1", "column3", "column17", "column18"]
    ints = ["column6", "column7", "column9", "daysSinceEpoch"]
    strs = ["column5", "column11", "column12"]
    out = {}
    for c in metrics:
        out[c] = _int_col(cols[c], True)
    for c in ints:
        out[c] = _int_col(cols[c], False)
    for c in strs:
        out[c] = _str_col(cols[c])
    np.savez_compressed(os.path.join(OUT, "test_data_sv.npz"), **out)
    return out


def make_simple():
    cols = read_avro(os.path.join(REF, "simpleData200001.avro"))
    out = {c: _int_col(cols[c], c == "met") for c in ("dim0", "dim1", "met")}
    np.savez_compressed(os.path.join(OUT, "simple_data_200001.npz"), **out)
    return out


# Expected values, verbatim from the reference's Java test assertions.
EXPECTED = {
    "source": "pinot-core/src/test/java/com/linkedin/pinot/queries/AggregationSingleValueQueriesTest.java",
    "aggregation": " COUNT(*), SUM(column1), MAX(column3), MIN(column6), AVG(column7)",
    "filter": {
        "text": " WHERE column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000"
                " AND column5 = 'gFuH' AND (column6 < 500000000 OR column11 NOT IN ('t', 'P'))"
                " AND daysSinceEpoch = 126164076",
        "src": "BaseSingleValueQueriesTest.java:69-74",
    },
    # Inverted indexes are CREATED for these columns (BaseSingleValueQueriesTest.java:106-107) but the test loads the
    # segment with ColumnarSegmentLoader.load(dir, ReadMode.heap) (:121), i.e. without IndexLoadingConfigMetadata, so
    # ColumnIndexContainer.init (segment/index/column/ColumnIndexContainer.java:46-53) loads NO bitmap inverted index:
    # at query time only the sorted columns (column5, daysSinceEpoch) are index-based, every other leaf is a scan.  That
    # is what makes numEntriesScannedInFilter = 84134 (the nested OR holds two scan children).
    "inverted": ["column6", "column7", "column11", "column17", "column18"],
    "loaded_inverted": [],
    "aggregation_only": {
        "nofilter": {"stats": [30000, 0, 120000, 30000],
                     "result": [30000, 32317185437847, 2147419555, 1689277, [28175373944314, 30000]],
                     "line": "51-62"},
        "filter": {"stats": [6129, 84134, 24516, 30000],
                   "result": [6129, 6875947596072, 999813884, 1980174, [4699510391301, 6129]],
                   "line": "68-79"},
    },
    "group_by": {
        "small": {
            "columns": ["column9"], "mode": "ARRAY_BASED",
            "nofilter": {"stats": [30000, 0, 150000, 30000], "first_key": "11270",
                         "result": [1, 815409257, 1215316262, 1328642550, [788414092, 1]], "line": "92-106"},
            "filter": {"stats": [6129, 84134, 30645, 30000], "first_key": "242920",
                       "result": [3, 4348938306, 407993712, 296467636, [5803888725, 3]], "line": "112-125"},
        },
        "medium": {
            "columns": ["column9", "column11", "column12"], "mode": "LONG_MAP_BASED",
            "nofilter": {"stats": [30000, 0, 210000, 30000],
                         "first_key": "1577638897\tP\tKrNxpdycSiwoRohEiTIlLqDHnx",
                         "result": [5, 1211410535, 1720170285, 1585725369, [8398774425, 5]], "line": "138-152"},
            "filter": {"stats": [6129, 84134, 42903, 30000],
                       "first_key": "1096298724\tP\tKrNxpdycSiwoRohEiTIlLqDHnx",
                       "result": [7, 13531749490, 478007592, 394608493, [1229066783, 7]], "line": "158-172"},
        },
        "large": {
            "columns": ["column1", "column3", "column6", "column7", "column9", "column11", "column12",
                        "column17", "column18"], "mode": "ARRAY_MAP_BASED",
            "nofilter": {"stats": [30000, 0, 270000, 30000],
                         "first_key": "1784773968\t204243323\t628170461\t1985159279\t296467636\tP\tHEuxNvH\t402773817\t2047180536",
                         "result": [1, 1784773968, 204243323, 628170461, [1985159279, 1]], "line": "185-200"},
            "filter": {"stats": [6129, 84134, 55161, 30000],
                       "first_key": "1361199163\t178133991\t296467636\t788414092\t1719301234\tP\tMaztCmmxxgguBUxPti\t1284373442\t752388855",
                       "result": [1, 1361199163, 178133991, 296467636, [788414092, 1]], "line": "206-220"},
        },
    },
    "query_executor": {
        "source": "pinot-core/src/test/java/com/linkedin/pinot/query/executor/QueryExecutorTest.java",
        "segments": 2, "count": 400002, "sum_met": 40000200000.0, "max_met": 200000.0, "min_met": 0.0,
        "lines": "150,167,185,203",
    },
    "broker_reduce": {
        "source": "pinot-core/src/test/java/com/linkedin/pinot/query/executor/BrokerReduceServiceTest.java",
        "lines": "163,287,321,356,397-421",
        "servers_2": {"count_star": 800004, "avg_met": 100000.0, "distinctCount_dim0": 10, "distinctCount_dim1": 100},
        "servers_10": {"count_star": 4000020, "sum_met": 400002000000.0, "max_met": 200000.0, "min_met": 0.0,
                       "avg_met": 100000.0, "distinctCount_dim0": 10, "distinctCount_dim1": 100},
    },
}


def main():
    make_sv()
    make_simple()
    with open(os.path.join(OUT, "expected_sv_queries.json"), "w") as f:
        json.dump(EXPECTED, f, indent=1, sort_keys=True)
    shutil.copy(os.path.join(REF, "starTreeSegment.tar.gz"), os.path.join(OUT, "starTreeSegment.tar.gz"))
    for name in ("paddingOld", "paddingPercent", "paddingNull"):  # LoadersTest.testPadding fixtures (data files)
        shutil.copy(os.path.join(REF, name + ".tar.gz"), os.path.join(OUT, name + ".tar.gz"))
    make_sorted_range_vectors()
    print("wrote fixtures to", OUT)


def make_sorted_range_vectors():
    """The fixed range sets of SortedRangeIntersectionTest.testSimple / testComplex (:45-80), as JSON data."""
    import re
    src = open(os.path.join(REF, "..", "..", "java", "com", "linkedin", "pinot", "core", "util",
                            "SortedRangeIntersectionTest.java")).read()
    body = re.search(r"public void testComplex\(\)(.*?)\n  }\n", src, re.S).group(1)
    lit = lambda decl: json.loads("".join(re.findall(r'"(.*?)"', decl, re.S)))
    sets = [lit(x) for x in re.findall(r'String rangeSet\d = (".*?");', body, re.S)]
    exp = lit(re.search(r'String expectedOutputRangeSet = (".*?");', body, re.S).group(1))
    out = {"source": "pinot-core/src/test/java/com/linkedin/pinot/core/util/SortedRangeIntersectionTest.java:45-80",
           "simple": {"sets": [[[0, 4], [6, 10]], [[4, 7], [8, 14]]], "expected": [[4, 4], [6, 10]]},
           "complex": {"sets": sets, "expected": exp}}
    with open(os.path.join(OUT, "sorted_range_intersection.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    sys.exit(main())
