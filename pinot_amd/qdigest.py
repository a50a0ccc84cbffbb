"""QuantileDigest for PERCENTILEEST50/90/95/99.

Restates the digest the reference vendors, core/query/aggregation/function/quantile/digest/QuantileDigest.java (an
airlift q-digest over the 64 bits of value ^ Long.MIN_VALUE: a binary trie whose nodes carry weights, compressed so
that at most 3 * compressionFactor nodes survive, compressionFactor = (root level + 1) / maxError), with maxError =
0.05 and alpha = 0 (no decay: every weight is exactly the count; the digests of one query never live the 50 s after
which the reference would rescale).  Operations: add(value, count) (:123-147, insert :525-560), compress (:449-494),
merge (:149-160, :596-640), getQuantile (:165-196, post-order traversal), serialize / deserialize (:283-360; the
DataTable object type 7 of DataTableCustomSerDe).

The GPU path computes, per segment, the column's value histogram under the filter (the same GROUP BY sub-query as
PERCENTILE); the host offers each distinct value once with its count, in ascending value order, and merges the
segments' digests in segment order.  The reference adds the values one doc at a time in doc order and merges segment
digests in combine-thread completion order, so its digest shape is not reproducible; both sides answer within the
digest's rank-error guarantee (maxError * count), which is the parity the tests assert.
"""
from __future__ import annotations

import struct
from typing import Iterable, List, Optional, Tuple

MAX_BITS = 64
MAX_SIZE_FACTOR = 1.5
ZERO_WEIGHT_THRESHOLD = 1e-5
DEFAULT_MAX_ERROR = 0.05
M64 = (1 << 64) - 1
SIGN = 1 << 63


def _long_to_bits(v: int) -> int:
    return (v & M64) ^ SIGN


def _bits_to_long(b: int) -> int:
    x = (b ^ SIGN) & M64
    return x - (1 << 64) if x & SIGN else x


def _s64(x: int) -> int:
    x &= M64
    return x - (1 << 64) if x & SIGN else x


def _nlz(x: int) -> int:
    return 64 - x.bit_length()


class _Node:
    __slots__ = ("bits", "level", "w", "left", "right")

    def __init__(self, bits: int, level: int, w: float):
        self.bits, self.level, self.w = bits, level, w
        self.left: Optional[_Node] = None
        self.right: Optional[_Node] = None

    def is_leaf(self):
        return self.left is None and self.right is None

    def single_child(self):
        return (self.left is None) != (self.right is None)

    def branch_mask(self):
        return 1 << (self.level - 1)

    def upper(self) -> int:
        mask = (M64 >> (MAX_BITS - self.level)) if self.level > 0 else 0
        return _bits_to_long(self.bits | mask)


def _same_subtree(a: int, b: int, level: int) -> bool:
    return level == MAX_BITS or (a >> level) == (b >> level)


class QuantileDigest:
    def __init__(self, max_error: float = DEFAULT_MAX_ERROR):
        self.max_error = max_error
        self.alpha = 0.0
        self.root: Optional[_Node] = None
        self.weighted_count = 0.0
        self.max = -(1 << 63)
        self.min = (1 << 63) - 1
        self.landmark = 0
        self.total_nodes = 0
        self.nonzero_nodes = 0

    # ---- add / insert ----
    def _compression_factor(self) -> int:
        if self.root is None:
            return 1
        return max(int((self.root.level + 1) / self.max_error), 1)

    def add(self, value: int, count: int = 1):
        if count <= 0:
            raise ValueError("count must be > 0")
        if self.nonzero_nodes > MAX_SIZE_FACTOR * (3 * self._compression_factor()):
            self.compress()
        w = float(count)  # weight(now) * count with alpha = 0
        self.max = max(self.max, value)
        self.min = min(self.min, value)
        self._insert(_long_to_bits(value), w)

    def _create(self, bits, level, w) -> _Node:
        self.weighted_count += w
        self.total_nodes += 1
        if w >= ZERO_WEIGHT_THRESHOLD:
            self.nonzero_nodes += 1
        return _Node(bits, level, w)

    def _set_child(self, parent, branch, child):
        if parent is None:
            self.root = child
        elif branch == 0:
            parent.left = child
        else:
            parent.right = child

    def _siblings(self, node: _Node, sib: _Node) -> _Node:
        level = MAX_BITS - _nlz(node.bits ^ sib.bits)
        parent = self._create(node.bits, level, 0.0)
        if sib.bits & parent.branch_mask() == 0:
            parent.left, parent.right = sib, node
        else:
            parent.left, parent.right = node, sib
        return parent

    def _insert(self, bits: int, w: float):
        last = 0
        parent = None
        cur = self.root
        while True:
            if cur is None:
                self._set_child(parent, last, self._create(bits, 0, w))
                return
            if not _same_subtree(bits, cur.bits, cur.level):
                self._set_child(parent, last, self._siblings(cur, self._create(bits, 0, w)))
                return
            if cur.level == 0 and cur.bits == bits:
                old = cur.w
                cur.w += w
                if cur.w >= ZERO_WEIGHT_THRESHOLD and old < ZERO_WEIGHT_THRESHOLD:
                    self.nonzero_nodes += 1
                self.weighted_count += w
                return
            branch = bits & cur.branch_mask()
            parent, last = cur, branch
            cur = cur.left if branch == 0 else cur.right

    # ---- compress ----
    def _try_remove(self, node: Optional[_Node]) -> Optional[_Node]:
        if node is None:
            return None
        if node.w >= ZERO_WEIGHT_THRESHOLD:
            self.nonzero_nodes -= 1
        self.weighted_count -= node.w
        if node.is_leaf():
            self.total_nodes -= 1
            return None
        if node.single_child():
            self.total_nodes -= 1
            return node.left if node.left is not None else node.right
        node.w = 0.0
        return node

    def compress(self):
        cf = self._compression_factor()

        def visit(node: _Node):
            if node.is_leaf():
                return
            lw = node.left.w if node.left is not None else 0.0
            rw = node.right.w if node.right is not None else 0.0
            should = node.w + lw + rw < int(self.weighted_count / cf)
            old = node.w
            if should or lw < ZERO_WEIGHT_THRESHOLD:
                node.left = self._try_remove(node.left)
                self.weighted_count += lw
                node.w += lw
            if should or rw < ZERO_WEIGHT_THRESHOLD:
                node.right = self._try_remove(node.right)
                self.weighted_count += rw
                node.w += rw
            if old < ZERO_WEIGHT_THRESHOLD <= node.w:
                self.nonzero_nodes += 1

        for n in self._post_order():
            visit(n)
        if self.root is not None and self.root.w < ZERO_WEIGHT_THRESHOLD:
            self.root = self._try_remove(self.root)

    def _post_order(self, reverse: bool = False) -> List[_Node]:
        """Post-order node list (left, right, node); the callbacks of the reference mutate children of the visited node
        only, which a precomputed order over the nodes still present reproduces."""
        out = []
        stack = [(self.root, False)] if self.root is not None else []
        while stack:
            n, done = stack.pop()
            if done:
                out.append(n)
                continue
            stack.append((n, True))
            a, b = (n.left, n.right) if not reverse else (n.right, n.left)
            if b is not None:
                stack.append((b, False))
            if a is not None:
                stack.append((a, False))
        return out

    # ---- merge ----
    def _copy(self, node: Optional[_Node]) -> Optional[_Node]:
        if node is None:
            return None
        r = self._create(node.bits, node.level, node.w)
        r.left = self._copy(node.left)
        r.right = self._copy(node.right)
        return r

    def _merge(self, node: Optional[_Node], other: Optional[_Node]) -> Optional[_Node]:
        if node is None:
            return self._copy(other)
        if other is None:
            return node
        if not _same_subtree(node.bits, other.bits, max(node.level, other.level)):
            return self._siblings(node, self._copy(other))
        if node.level > other.level:
            if other.bits & node.branch_mask() == 0:
                node.left = self._merge(node.left, other)
            else:
                node.right = self._merge(node.right, other)
            return node
        if node.level < other.level:
            r = self._create(other.bits, other.level, other.w)
            if node.bits & other.branch_mask() == 0:
                r.left = self._merge(node, other.left)
                r.right = self._copy(other.right)
            else:
                r.left = self._copy(other.left)
                r.right = self._merge(node, other.right)
            return r
        old = node.w
        self.weighted_count += other.w
        node.w = node.w + other.w
        node.left = self._merge(node.left, other.left)
        node.right = self._merge(node.right, other.right)
        if old < ZERO_WEIGHT_THRESHOLD <= node.w:
            self.nonzero_nodes += 1
        return node

    def merge(self, other: "QuantileDigest") -> "QuantileDigest":
        self.root = self._merge(self.root, other.root)
        self.max = max(self.max, other.max)
        self.min = min(self.min, other.min)
        self.compress()
        return self

    # ---- queries ----
    def get_quantile(self, q: float) -> int:
        s = 0.0
        for node in self._post_order():
            s += node.w
            if s > q * self.weighted_count:
                return min(node.upper(), self.max)
        return self.max

    @property
    def count(self) -> float:
        return self.weighted_count

    # ---- DataTable bytes (DataOutput, big-endian) ----
    def serialize(self) -> bytes:
        out = [struct.pack(">ddqqqi", self.max_error, self.alpha, self.landmark, self.min, self.max, self.total_nodes)]
        for n in self._post_order():
            flags = (1 if n.left is not None else 0) | (2 if n.right is not None else 0)  # Flags.HAS_LEFT / HAS_RIGHT
            out.append(struct.pack(">BBqd", flags, n.level, _s64(n.bits), n.w))
        return b"".join(out)

    @staticmethod
    def deserialize(b: bytes) -> "QuantileDigest":
        max_error, alpha, landmark, mn, mx, total = struct.unpack_from(">ddqqqi", b, 0)
        d = QuantileDigest(max_error)
        d.alpha, d.landmark, d.min, d.max, d.total_nodes = alpha, landmark, mn, mx, total
        p = struct.calcsize(">ddqqqi")
        stack: List[_Node] = []
        for _ in range(total):
            flags, level, bits, w = struct.unpack_from(">BBqd", b, p)
            p += struct.calcsize(">BBqd")
            node = _Node(bits & M64, level, w)
            if flags & 2:
                node.right = stack.pop()
            if flags & 1:
                node.left = stack.pop()
            stack.append(node)
            d.weighted_count += w
            if w >= ZERO_WEIGHT_THRESHOLD:
                d.nonzero_nodes += 1
        if stack:
            if len(stack) != 1:
                raise ValueError("Tree is corrupted. Expected a single root node")
            d.root = stack.pop()
        return d


def from_histogram(hist: Iterable[Tuple[float, int]], max_error: float = DEFAULT_MAX_ERROR) -> QuantileDigest:
    """The digest of a segment's selected values from their histogram: each distinct (long) value offered once with
    its count, ascending (PercentileestAggregationFunction.aggregate adds (long) value per doc)."""
    d = QuantileDigest(max_error)
    for v, c in sorted(hist):
        if int(c) > 0:
            d.add(int(v), int(c))
    return d


def merge_all(digests: Iterable[Optional[QuantileDigest]]) -> Optional[QuantileDigest]:
    """DigestAggregationFunction.combineTwoValues (:121-131) folded left; None sides yield the other."""
    acc = None
    for d in digests:
        if d is None:
            continue
        acc = d if acc is None else acc.merge(d)
    return acc
