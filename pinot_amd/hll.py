"""DISTINCTCOUNTHLL / FASTHLL intermediates: HyperLogLog(log2m = 8) register sets, vectorised over numpy.

The hot path offers ``(int) hashCode`` of every selected doc's value (core/operator/aggregation/function/
DistinctCountHLLAggregationFunction.java:51-62 aggregate, :80-92 aggregateGroupBySV; log2m = HllConstants.DEFAULT_LOG2M,
core/startree/hll/HllConstants.java:19).  The HyperLogLog and its hash live in the third-party stream-lib
(com.clearspring.analytics:stream 2.7.0, pom.xml:525-527, not vendored in the reference); their published algorithm is
restated here:

* ``HyperLogLog.offer(Integer)`` -> ``MurmurHash.hash(Object)`` -> ``hashLong((long) i)`` (MurmurHash2, m = 0x5bd1e995,
  r = 24, over the low then the high 32-bit half);
* ``offerHashed(x)``: register ``j = x >>> 24``, rank ``numberOfLeadingZeros((x << 8) | (1 << 7) + 1) + 1``,
  ``updateIfGreater``;
* ``addAll``: register-wise max;
* ``cardinality()``: ``alphaMM / sum(2^-reg)`` with ``alphaMM = 0.7213 / (1 + 1.079 / m) * m * m``; at or below
  ``2.5 m`` the linear-counting estimate ``m * ln(m / zeros)``; ``Math.round`` of the result.

Registers depend only on the SET of offered ints (offer is an idempotent max), so the GPU's distinct-value histogram
(the DISTINCTCOUNT sub-query of extended.py) determines them exactly: no per-doc work is needed on the host.
"""
from __future__ import annotations

import math
from typing import Iterable

import numpy as np

LOG2M = 8
M = 1 << LOG2M
_MUL = np.uint32(0x5BD1E995)


def _u32(x) -> np.ndarray:
    return np.asarray(x, dtype=np.uint32)


def hash_long(values) -> np.ndarray:
    """MurmurHash.hashLong over an int64 array (Java int arithmetic as uint32 wraparound)."""
    v = np.asarray(values, dtype=np.int64).view(np.uint64)
    with np.errstate(over="ignore"):
        k = (v & np.uint64(0xFFFFFFFF)).astype(np.uint32) * _MUL
        k ^= k >> np.uint32(24)
        h = k * _MUL  # h = 0 ^ k * m
        k = (v >> np.uint64(32)).astype(np.uint32) * _MUL
        k ^= k >> np.uint32(24)
        h = h * _MUL
        h ^= k * _MUL
        h ^= h >> np.uint32(13)
        h = h * _MUL
        h ^= h >> np.uint32(15)
    return h


def _nlz32(x: np.ndarray) -> np.ndarray:
    """Integer.numberOfLeadingZeros for uint32 (x is never 0 here: bit 7 is forced on)."""
    x = _u32(x)
    n = np.zeros(x.shape, dtype=np.int32)
    for s in (16, 8, 4, 2, 1):
        m = x < (np.uint32(1) << np.uint32(32 - s))
        n += np.where(m, s, 0).astype(np.int32)
        x = np.where(m, x << np.uint32(s), x)
    return n


def empty() -> np.ndarray:
    return np.zeros(M, dtype=np.uint8)


def offer_ints(regs: np.ndarray, ints: Iterable[int]) -> np.ndarray:
    """offer((int) v) for every v (any order, duplicates irrelevant); returns the updated registers."""
    a = np.fromiter((int(i) for i in ints), dtype=np.int64)
    if a.size == 0:
        return regs
    h = hash_long(a)
    j = (h >> np.uint32(32 - LOG2M)).astype(np.int64)
    with np.errstate(over="ignore"):
        w = (h << np.uint32(LOG2M)) | np.uint32((1 << (LOG2M - 1)) + 1)
    r = (_nlz32(w) + 1).astype(np.uint8)
    np.maximum.at(regs, j, r)
    return regs


def from_ints(ints: Iterable[int]) -> np.ndarray:
    return offer_ints(empty(), ints)


def merge(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """HyperLogLog.addAll: register-wise max."""
    return np.maximum(a, b)


def cardinality(regs: np.ndarray) -> int:
    """HyperLogLog.cardinality() (stream-lib 2.7.0)."""
    reg_sum = 0.0
    zeros = 0.0
    for v in regs.tolist():  # sequential double sum, register order
        reg_sum += 1.0 / (1 << v)
        if v == 0:
            zeros += 1.0
    alpha_mm = (0.7213 / (1 + 1.079 / M)) * M * M
    estimate = alpha_mm * (1 / reg_sum)
    if estimate <= (5.0 / 2.0) * M:
        lc = M * math.log(M / zeros) if zeros > 0 else math.inf
        return _java_round(lc)
    return _java_round(estimate)


def _java_round(x: float) -> int:
    """Math.round(double): floor(x + 0.5), saturating (inf -> Long.MAX_VALUE)."""
    if x != x:
        return 0
    if x >= 9.223372036854775807e18:
        return (1 << 63) - 1
    return int(math.floor(x + 0.5))


# ---- serialized form (FASTHLL columns) --------------------------------------------------------------------------
# HyperLogLog.getBytes(): writeInt(log2m), writeInt(4 * words), then the RegisterSet words big-endian; a word holds 6
# registers of 5 bits (register i: word i / 6, shift 5 * (i % 6)); 2^8 registers -> 43 words -> 180 bytes
# (HllUtil.LOG2M_TO_SIZE_IN_BYTES, core/startree/hll/HllUtil.java:38-39).  The segment stores it as a STRING whose chars
# are byte + 129 (HllUtil.SerializationConverter, :146-175).
_PER_WORD = 6
_CHAR_OFFSET = 129


def _words_for(count: int) -> int:
    bits = count // _PER_WORD  # RegisterSet.getSizeForCount
    return 1 if bits == 0 else bits if bits % 32 == 0 else bits + 1


def to_bytes(regs: np.ndarray, log2m: int = LOG2M) -> bytes:
    n = 1 << log2m
    words = np.zeros(_words_for(n), dtype=np.uint32)
    pos = np.arange(n)
    np.bitwise_or.at(words, pos // _PER_WORD,
                     regs[:n].astype(np.uint32) << (5 * (pos % _PER_WORD)).astype(np.uint32))
    head = np.array([log2m, 4 * len(words)], dtype=">i4").tobytes()
    return head + words.astype(">u4").tobytes()


def from_bytes(b: bytes) -> np.ndarray:
    """HyperLogLog.Builder.build: the registers (log2m must be this module's: addAll of estimators of different sizes
    throws in the reference)."""
    log2m, nbytes = (int(x) for x in np.frombuffer(b[:8], dtype=">i4"))
    if log2m != LOG2M:
        raise ValueError("Cannot merge estimators of different sizes (log2m %d)" % log2m)
    words = np.frombuffer(b[8:8 + nbytes], dtype=">u4").astype(np.uint32)
    pos = np.arange(M)
    return ((words[pos // _PER_WORD] >> (5 * (pos % _PER_WORD)).astype(np.uint32)) & 0x1F).astype(np.uint8)


def to_string(regs: np.ndarray) -> str:
    """HllUtil.convertHllToString: one char per (signed) byte, char = byte + 129."""
    return "".join(chr(((x - 256) if x > 127 else x) + _CHAR_OFFSET) for x in to_bytes(regs))


def from_string(s: str) -> np.ndarray:
    """HllUtil.convertStringToHll: byte = (byte) (char - 129)."""
    return from_bytes(bytes(((ord(c) - _CHAR_OFFSET) & 0xFF) for c in s))
