"""Pinot v1 segment format: writer, loader and the in-memory column model staged into HBM.

On-disk layout (verified byte-for-byte against the Java-written fixture tests/golden/starTreeSegment.tar.gz;
see SURVEY.md Appendix A).  Paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/:

  <col>.sv.unsorted.fwd  ceil(totalDocs*b/8) bytes, row r = bits [r*b, r*b+b) MSB-first, big-endian, no header
                         (io/writer/impl/FixedBitSingleValueMultiColWriter.java:86-130, util/PinotDataCustomBitSet.java)
  <col>.sv.sorted.fwd    card x (int32 BE start, int32 BE end), both inclusive
                         (segment/index/column/ColumnIndexContainer.java:112-121, io/reader/impl/SortedForwardIndexReader.java)
  <col>.dict             card x fixed width, sorted ascending; INT/FLOAT 4 B BE, LONG/DOUBLE 8 B BE, STRING padded to
                         lengthOfEachEntry with the padding char (segment/creator/impl/SegmentDictionaryCreator.java:187-301)
  <col>.bitmap.inv       (card+1) x int32 BE offsets then portable RoaringBitmap serialisations (cookie 12346, LE)
                         (segment/creator/impl/inv/HeapBitmapInvertedIndexCreator.java:42-81)
  metadata.properties    "key = value" (segment/creator/impl/SegmentColumnarIndexCreator.java:314,352)

bitsPerElement is always READ from metadata, never recomputed.
"""
from __future__ import annotations

import math
import os
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

DEFAULT_PAD = "\0"  # V1Constants.Str.DEFAULT_STRING_PAD_CHAR (segment/creator/impl/V1Constants.java:51)
LEGACY_PAD = "%"    # V1Constants.Str.LEGACY_STRING_PAD_CHAR (:52): segments whose metadata has no padding key
PAD_KEY = "segment.padding.character"  # V1Constants.MetadataKeys.Segment.SEGMENT_PADDING_CHARACTER (:127)


def java_escape(ch: str) -> str:
    """StringEscapeUtils.escapeJava of one char, as SegmentColumnarIndexCreator writes the padding key (:216-217)."""
    if ch == "\\":
        return "\\\\"
    if " " <= ch <= "~":
        return ch
    return "\\u%04X" % ord(ch)


def java_unescape(s: str) -> str:
    """StringEscapeUtils.unescapeJava (ColumnMetadata.java:93-98 takes charAt(0) of the result)."""
    out, i = [], 0
    while i < len(s):
        c = s[i]
        if c == "\\" and i + 1 < len(s):
            n = s[i + 1]
            if n == "u" and i + 6 <= len(s):
                out.append(chr(int(s[i + 2:i + 6], 16)))
                i += 6
                continue
            out.append({"t": "\t", "n": "\n", "r": "\r", "0": "\0", "\\": "\\"}.get(n, n))
            i += 2
            continue
        out.append(c)
        i += 1
    return "".join(out)
ROARING_COOKIE_NO_RUN = 12346
DTYPES = ("INT", "LONG", "FLOAT", "DOUBLE", "STRING")
_DICT_NP = {"INT": ">i4", "LONG": ">i8", "FLOAT": ">f4", "DOUBLE": ">f8"}


def num_bits(card: int) -> int:
    """SingleValueUnsortedForwardIndexCreator.getNumOfBits (segment/creator/impl/fwd/...:48-57)."""
    if card < 2:
        return 1
    r = int(math.ceil(math.log(card) / math.log(2)))
    return max(r, 1)


# ------------------------------------------------------------------------------------------------
# fixed-bit packing (MSB-first, big-endian)
# ------------------------------------------------------------------------------------------------
def pack_fixed_bit(values, bits: int) -> bytes:
    v = np.asarray(values, dtype=np.uint64)
    n = len(v)
    nbytes = (n * bits + 7) // 8
    if n == 0:
        return b""
    if bits == 8:
        return v.astype(np.uint8).tobytes()
    if bits == 16:
        return v.astype(">u2").tobytes()
    if bits == 32:
        return v.astype(">u4").tobytes()
    # Generic: expand to a bit matrix (n x bits, MSB first) and pack.
    shifts = np.arange(bits - 1, -1, -1, dtype=np.uint64)
    bitmat = ((v[:, None] >> shifts[None, :]) & np.uint64(1)).astype(np.uint8).reshape(-1)
    out = np.packbits(bitmat)  # MSB-first within each byte
    return out.tobytes()[:nbytes].ljust(nbytes, b"\0")


def _native_pack(v: np.ndarray, bits: int):
    """pgx_pack_fixed_bit (libpgx host code, no device needed); None when the library is not built."""
    import ctypes as C
    from . import native as N
    if not os.path.exists(N.LIB_PATH) or v.size == 0 or int(v.max()) >= (1 << 31) or int(v.min()) < 0:
        return None
    ids = np.ascontiguousarray(v, dtype=np.int32)
    out = np.zeros((len(ids) * bits + 7) // 8, dtype=np.uint8)
    N.check(N.lib().pgx_pack_fixed_bit(ids.ctypes.data, len(ids), bits, out.ctypes.data))
    return out.tobytes()


def pack_fixed_bit_chunked(values, bits: int, chunk: int = 1 << 22) -> bytes:
    """pack_fixed_bit for large arrays: the library's packer, else numpy chunked on byte boundaries (chunk rows a
    multiple of 8)."""
    v = np.asarray(values)
    if len(v) > 65536:
        out = _native_pack(v, bits)
        if out is not None:
            return out
    if len(v) <= chunk:
        return pack_fixed_bit(v, bits)
    assert chunk % 8 == 0
    parts = [pack_fixed_bit(v[i:i + chunk], bits) for i in range(0, len(v), chunk)]
    return b"".join(parts)


def unpack_fixed_bit(buf: bytes, n: int, bits: int) -> np.ndarray:
    a = np.frombuffer(bytes(buf) + b"\0" * 8, dtype=np.uint8)
    start = np.arange(n, dtype=np.int64) * bits
    byte = start >> 3
    w = np.zeros(n, dtype=np.uint64)
    for k in range(5):
        w = (w << np.uint64(8)) | a[byte + k].astype(np.uint64)
    shift = (40 - (start & 7) - bits).astype(np.uint64)
    return ((w >> shift) & np.uint64((1 << bits) - 1)).astype(np.int64)


# ------------------------------------------------------------------------------------------------
# RoaringBitmap portable serialisation (RoaringBitmap 0.5.10, no run containers)
# ------------------------------------------------------------------------------------------------
def roaring_serialize(docs: np.ndarray) -> bytes:
    docs = np.unique(np.asarray(docs, dtype=np.int64))
    keys = (docs >> 16).astype(np.int64)
    uk, starts = np.unique(keys, return_index=True)
    ends = list(starts[1:]) + [len(docs)]
    n = len(uk)
    header = struct.pack("<ii", ROARING_COOKIE_NO_RUN, n)
    desc = b""
    payloads = []
    for k, s, e in zip(uk, starts, ends):
        low = (docs[s:e] & 0xFFFF).astype(np.uint16)
        card = len(low)
        desc += struct.pack("<HH", int(k), card - 1)
        if card <= 4096:
            payloads.append(low.astype("<u2").tobytes())
        else:
            bm = np.zeros(65536, dtype=np.uint8)
            bm[low] = 1
            payloads.append(np.packbits(bm, bitorder="little").tobytes())  # 1024 x u64 LE
    off = len(header) + len(desc) + 4 * n
    offs = b""
    for p in payloads:
        offs += struct.pack("<i", off)
        off += len(p)
    return header + desc + offs + b"".join(payloads)


def roaring_deserialize(buf: bytes) -> np.ndarray:
    cookie, n = struct.unpack_from("<ii", buf, 0)
    if cookie != ROARING_COOKIE_NO_RUN:
        raise ValueError("unsupported roaring cookie %d (run containers are never written by the reference)" % cookie)
    pos = 8
    keys, cards = [], []
    for i in range(n):
        k, c = struct.unpack_from("<HH", buf, pos)
        keys.append(k)
        cards.append(c + 1)
        pos += 4
    offs = struct.unpack_from("<%di" % n, buf, pos) if n else ()
    out = []
    for k, c, o in zip(keys, cards, offs):
        if c <= 4096:
            low = np.frombuffer(buf, dtype="<u2", count=c, offset=o).astype(np.int64)
        else:
            bits = np.unpackbits(np.frombuffer(buf, dtype=np.uint8, count=8192, offset=o), bitorder="little")
            low = np.nonzero(bits)[0].astype(np.int64)
        out.append((k << 16) | low)
    return np.concatenate(out) if out else np.zeros(0, dtype=np.int64)


def build_inverted_index(dict_ids: np.ndarray, card: int) -> bytes:
    order = np.argsort(dict_ids, kind="stable")
    sorted_ids = dict_ids[order]
    bounds = np.searchsorted(sorted_ids, np.arange(card + 1))
    blobs = [roaring_serialize(order[bounds[i]:bounds[i + 1]]) for i in range(card)]
    offs = [4 * (card + 1)]
    for b in blobs:
        offs.append(offs[-1] + len(b))
    return struct.pack(">%di" % (card + 1), *offs) + b"".join(blobs)


def inverted_index_docs(inv: bytes, card: int, dict_id: int) -> np.ndarray:
    a, b = struct.unpack_from(">ii", inv, 4 * dict_id)
    return roaring_deserialize(inv[a:b])


# ------------------------------------------------------------------------------------------------
# Column / segment model
# ------------------------------------------------------------------------------------------------
@dataclass
class Column:
    name: str
    data_type: str
    column_type: str  # DIMENSION, METRIC, TIME
    cardinality: int
    bits: int
    total_docs: int
    total_raw_docs: int
    is_sorted: bool
    has_inverted: bool
    dict_bytes: bytes
    dict_width: int
    fwd_bytes: Optional[bytes]  # unsorted fixed-bit forward index
    sorted_bytes: Optional[bytes]  # sorted forward index pairs
    inv_bytes: Optional[bytes]  # bitmap inverted index
    pad_char: str = DEFAULT_PAD
    is_mv: bool = False          # multi-value column: fwd_bytes holds <col>.mv.fwd
    total_entries: int = 0       # totalNumberOfEntries
    max_mv: int = 0              # maxNumberOfMultiValues

    def dictionary_values(self):
        if self.data_type == "STRING":
            w = self.dict_width
            out = []
            for i in range(self.cardinality):
                raw = self.dict_bytes[i * w:(i + 1) * w]
                s = raw.decode("utf-8")
                p = s.find(self.pad_char)
                out.append(s if p < 0 else s[:p])  # StringDictionary.get (:53-66)
            return out
        return np.frombuffer(self.dict_bytes, dtype=_DICT_NP[self.data_type], count=self.cardinality)

    def dict_ids(self) -> np.ndarray:
        if self.is_mv:
            raise ValueError("multi-value column: use mv_dict_ids()")
        if self.is_sorted and self.sorted_bytes is not None:
            pairs = np.frombuffer(self.sorted_bytes, dtype=">i4").reshape(-1, 2)
            out = np.zeros(self.total_docs, dtype=np.int64)
            for d, (a, b) in enumerate(pairs):
                out[a:b + 1] = d
            return out
        return unpack_fixed_bit(self.fwd_bytes, self.total_docs, self.bits)


    def mv_dict_ids(self) -> List[np.ndarray]:
        """FixedBitMultiValueReader.getIntArray for every doc (io/reader/impl/v1/FixedBitMultiValueReader.java)."""
        starts, raw_off = mv_layout(self.fwd_bytes, self.total_docs, self.total_entries)
        vals = unpack_fixed_bit(self.fwd_bytes[raw_off:], self.total_entries, self.bits)
        return [vals[starts[d]:starts[d + 1]] for d in range(self.total_docs)]


def mv_docs_per_chunk(num_docs: int, total_values: int) -> int:
    """FixedBitMultiValueWriter: float averageValuesPerDoc = totalNumValues / numDocs (an INTEGER division, then
    widened); docsPerChunk = (int) Math.ceil(2048 / averageValuesPerDoc) in float arithmetic."""
    avg = np.float32(total_values // num_docs)
    return int(math.ceil(float(np.float32(2048) / avg)))


def pack_mv_fwd(doc_ids: Sequence[Sequence[int]], bits: int) -> bytes:
    """<col>.mv.fwd (io/writer/impl/v1/FixedBitMultiValueWriter.java): numChunks big-endian int chunk offsets (the
    value index of every docsPerChunk-th doc), a totalNumValues-bit MSB-first bitset with the first value of every doc
    set, then all values fixed-bit (MSB-first, as a single-value forward index over value positions)."""
    n = len(doc_ids)
    lens = np.array([len(v) for v in doc_ids], dtype=np.int64)
    assert n > 0 and lens.min() >= 1, "every doc holds at least one value"
    starts = np.concatenate([[0], np.cumsum(lens)])
    tv = int(starts[-1])
    dpc = mv_docs_per_chunk(n, tv)
    nchunks = (n + dpc - 1) // dpc
    head = starts[np.arange(nchunks) * dpc].astype(">i4").tobytes()
    bitset = np.zeros((tv + 7) // 8 * 8, dtype=np.uint8)
    bitset[starts[:-1]] = 1
    bs = np.packbits(bitset).tobytes()[:(tv + 7) // 8]
    flat = np.concatenate([np.asarray(v, dtype=np.int64) for v in doc_ids])
    raw = pack_fixed_bit(flat, bits)[:(tv * bits + 7) // 8]
    return head + bs + raw


def mv_layout(buf: bytes, num_docs: int, total_values: int):
    """(doc start offsets [num_docs + 1], byte offset of the raw values) of a <col>.mv.fwd."""
    dpc = mv_docs_per_chunk(num_docs, total_values)
    nchunks = (num_docs + dpc - 1) // dpc
    head = nchunks * 4
    nbs = (total_values + 7) // 8
    bits = np.unpackbits(np.frombuffer(buf, dtype=np.uint8, count=nbs, offset=head))[:total_values]
    starts = np.concatenate([np.nonzero(bits)[0], [total_values]]).astype(np.int64)
    assert len(starts) == num_docs + 1
    return starts, head + nbs


@dataclass
class SegmentData:
    name: str
    total_docs: int
    total_raw_docs: int
    columns: Dict[str, Column] = field(default_factory=dict)
    star_tree: Optional[bytes] = None
    metadata: Dict[str, str] = field(default_factory=dict)


def _java_string_sort(values: List[str], width: int, pad: str) -> List[str]:
    # SegmentDictionaryCreator sorts the PADDED strings (Arrays.sort(revised), :285-301) -- Java String.compareTo
    # compares UTF-16 code units; for the BMP that equals comparing code points.
    padded = [(v + pad * (width - len(v.encode("utf-8")))) if len(v) < width else v for v in values]
    order = sorted(range(len(values)), key=lambda i: [ord(ch) for ch in padded[i]])
    return [values[i] for i in order]


def make_column(name: str, values, data_type: str = None, column_type: str = "DIMENSION",
                inverted: bool = False, pad: str = DEFAULT_PAD, dictionary=None, dict_ids=None,
                force_unsorted: bool = False) -> Column:
    """Build a v1 column from raw values (SegmentDictionaryCreator + fwd-index creators).  Either raw `values`, or a
    pre-built sorted `dictionary` plus `dict_ids` (used by the synthetic generator).  force_unsorted: write a fixed-bit
    forward index even when the ids ascend (realtime snapshots: the realtime data source is never sorted)."""
    if dictionary is None:
        vals = np.asarray(values)
        if data_type is None:
            data_type = "STRING" if vals.dtype.kind in "SUO" else ("INT" if vals.dtype.kind in "iu" else "DOUBLE")
        if data_type == "STRING":
            sv = [v.decode() if isinstance(v, bytes) else str(v) for v in vals.tolist()]
            distinct = list(set(sv))
            width = max([1] + [len(s.encode("utf-8")) for s in distinct])
            dictionary = _java_string_sort(distinct, width, pad)
            lookup = {v: i for i, v in enumerate(dictionary)}
            dict_ids = np.array([lookup[v] for v in sv], dtype=np.int64)
        else:
            dictionary, dict_ids = np.unique(vals, return_inverse=True)
    n = len(dict_ids)
    card = len(dictionary)
    if data_type == "STRING":
        width = max([1] + [len(s.encode("utf-8")) for s in dictionary])
        dict_bytes = b"".join((s.encode("utf-8") + pad.encode() * (width - len(s.encode("utf-8")))) for s in dictionary)
    else:
        width = int(_DICT_NP[data_type][-1])
        dict_bytes = np.asarray(dictionary).astype(_DICT_NP[data_type]).tobytes()
    bits = num_bits(card)
    dict_ids = np.asarray(dict_ids, dtype=np.int64)
    is_sorted = not force_unsorted and bool(n <= 1 or np.all(np.diff(dict_ids) >= 0))
    fwd = sorted_b = None
    if is_sorted:
        first = np.searchsorted(dict_ids, np.arange(card), side="left")
        last = np.searchsorted(dict_ids, np.arange(card), side="right") - 1
        sorted_b = np.stack([first, last], axis=1).astype(">i4").tobytes()
    else:
        fwd = pack_fixed_bit_chunked(dict_ids, bits)
    inv = build_inverted_index(dict_ids, card) if (inverted and not is_sorted) else None
    return Column(name, data_type, column_type, card, bits, n, n, is_sorted, inverted or is_sorted,
                  dict_bytes, width, fwd, sorted_b, inv, pad)


def make_mv_column(name: str, doc_values: Sequence[Sequence], data_type: str = "INT", column_type: str = "DIMENSION",
                   inverted: bool = False) -> Column:
    """A v1 multi-value column from per-doc value lists (SegmentDictionaryCreator over all values; MV forward index;
    the inverted index holds every doc under each of its values, HeapBitmapInvertedIndexCreator.add(int, int[]))."""
    flat = np.concatenate([np.asarray(v) for v in doc_values])
    dictionary, ids = np.unique(flat.astype(_DICT_NP[data_type].replace(">", "<")), return_inverse=True)
    card = len(dictionary)
    bits = num_bits(card)
    lens = [len(v) for v in doc_values]
    starts = np.concatenate([[0], np.cumsum(lens)])
    doc_ids = [ids[starts[d]:starts[d + 1]] for d in range(len(doc_values))]
    fwd = pack_mv_fwd(doc_ids, bits)
    inv = None
    if inverted:
        docs = np.repeat(np.arange(len(doc_values)), lens)
        per = [np.unique(docs[ids == k]) for k in range(card)]
        blobs = [roaring_serialize(p) for p in per]
        offs = np.concatenate([[0], np.cumsum([len(b) for b in blobs])]) + 4 * (card + 1)
        inv = offs.astype(">i4").tobytes() + b"".join(blobs)
    width = int(_DICT_NP[data_type][-1])
    dict_bytes = np.asarray(dictionary).astype(_DICT_NP[data_type]).tobytes()
    n = len(doc_values)
    return Column(name, data_type, column_type, card, bits, n, n, False, inverted, dict_bytes, width, fwd, None, inv,
                  DEFAULT_PAD, True, int(starts[-1]), int(max(lens)))


def make_segment(name: str, columns: Sequence[Column]) -> SegmentData:
    n = columns[0].total_docs
    seg = SegmentData(name, n, n)
    for c in columns:
        assert c.total_docs == n
        seg.columns[c.name] = c
    return seg


# ------------------------------------------------------------------------------------------------
# Directory writer / loader (v1)
# ------------------------------------------------------------------------------------------------
def write_segment(seg: SegmentData, out_dir: str) -> str:
    d = os.path.join(out_dir, seg.name)
    os.makedirs(d, exist_ok=True)
    lines = ["segment.name = %s" % seg.name,
             "segment.total.raw.docs = %d" % seg.total_raw_docs,
             "segment.total.aggregate.docs = %d" % (seg.total_docs - seg.total_raw_docs),
             "segment.total.docs = %d" % seg.total_docs]
    if seg.star_tree is not None:
        lines.append("startree.enabled = true")
    pads = {c.pad_char for c in seg.columns.values() if c.data_type == "STRING"} or {DEFAULT_PAD}
    assert len(pads) == 1, "one padding character per segment"
    if PAD_KEY not in seg.metadata:
        lines.append("%s = %s" % (PAD_KEY, java_escape(pads.pop()).replace("\\", "\\\\")))
    for k, v in seg.metadata.items():
        lines.append("%s = %s" % (k, v))
    for c in seg.columns.values():
        p = "column.%s." % c.name
        lines += [p + "cardinality = %d" % c.cardinality, p + "totalDocs = %d" % c.total_docs,
                  p + "totalRawDocs = %d" % c.total_raw_docs,
                  p + "totalAggDocs = %d" % (c.total_docs - c.total_raw_docs),
                  p + "dataType = %s" % c.data_type, p + "bitsPerElement = %d" % c.bits,
                  p + "lengthOfEachEntry = %d" % (c.dict_width if c.data_type == "STRING" else 0),
                  p + "columnType = %s" % c.column_type, p + "isSorted = %s" % str(c.is_sorted).lower(),
                  p + "hasNullValue = false", p + "hasDictionary = true",
                  p + "hasInvertedIndex = %s" % str(c.has_inverted).lower(),
                  p + "isSingleValues = %s" % str(not c.is_mv).lower(),
                  p + "maxNumberOfMultiValues = %d" % c.max_mv, p + "totalNumberOfEntries = %d" % c.total_entries]
        with open(os.path.join(d, c.name + ".dict"), "wb") as f:
            f.write(c.dict_bytes)
        if c.is_mv:
            with open(os.path.join(d, c.name + ".mv.fwd"), "wb") as f:
                f.write(c.fwd_bytes)
        elif c.is_sorted:
            with open(os.path.join(d, c.name + ".sv.sorted.fwd"), "wb") as f:
                f.write(c.sorted_bytes)
        else:
            with open(os.path.join(d, c.name + ".sv.unsorted.fwd"), "wb") as f:
                f.write(c.fwd_bytes)
        if c.inv_bytes is not None:
            with open(os.path.join(d, c.name + ".bitmap.inv"), "wb") as f:
                f.write(c.inv_bytes)
    if seg.star_tree is not None:
        with open(os.path.join(d, "star-tree.bin"), "wb") as f:
            f.write(seg.star_tree)
    with open(os.path.join(d, "metadata.properties"), "w") as f:
        f.write("\n".join(lines) + "\n")
    return d


def _read_props(path):
    """metadata.properties as commons-configuration PropertiesConfiguration reads it: `key = value`, with the file's
    backslash escapes undone (the padding key is written as \\\\u0000, read back as the 6-char string \\u0000)."""
    props = {}
    for line in open(path, encoding="utf-8"):
        line = line.rstrip("\n")
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        props[k.strip()] = v.strip().replace("\\\\", "\\")
    return props


def load_segment(seg_dir: str) -> SegmentData:
    """Loaders.IndexSegment.load / ColumnIndexContainer.init for v1 SV columns (segment/index/loader/Loaders.java:44-118,
    segment/index/column/ColumnIndexContainer.java:45-139)."""
    props = _read_props(os.path.join(seg_dir, "metadata.properties"))
    name = props.get("segment.name", os.path.basename(seg_dir))
    total = int(props["segment.total.docs"])
    raw = int(props.get("segment.total.raw.docs", total))
    seg = SegmentData(name, total, raw, metadata=props)
    cols = sorted({k.split(".")[1] for k in props if k.startswith("column.")})
    for c in cols:
        p = "column.%s." % c

        def g(k, default=None):
            return props.get(p + k, default)

        dt = g("dataType")
        card = int(g("cardinality"))
        width = int(g("lengthOfEachEntry", "0")) if dt == "STRING" else int(_DICT_NP[dt][-1])
        is_sorted = g("isSorted") == "true"
        pad = java_unescape(props[PAD_KEY])[0] if PAD_KEY in props else LEGACY_PAD

        def rd(suffix):
            f = os.path.join(seg_dir, c + suffix)
            return open(f, "rb").read() if os.path.exists(f) else None

        mv = g("isSingleValues", "true") == "false"
        col = Column(c, dt, g("columnType"), card, int(g("bitsPerElement")), int(g("totalDocs")),
                     int(g("totalRawDocs", g("totalDocs"))), is_sorted, g("hasInvertedIndex") == "true",
                     rd(".dict"), width, rd(".mv.fwd") if mv else rd(".sv.unsorted.fwd"), rd(".sv.sorted.fwd"),
                     rd(".bitmap.inv"), pad, mv, int(g("totalNumberOfEntries", "0")),
                     int(g("maxNumberOfMultiValues", "0")))
        seg.columns[c] = col
    st = os.path.join(seg_dir, "star-tree.bin")
    if os.path.exists(st):
        seg.star_tree = open(st, "rb").read()
    return seg
