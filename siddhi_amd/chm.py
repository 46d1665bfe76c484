"""Iteration order of a JDK 8 ``java.util.concurrent.ConcurrentHashMap`` built by successive ``put``s.

The reference iterates such maps where the order is observable in the output:
``PartitionRuntime.metaQueryRuntimeMap`` (a partition's queries by name,
``PartitionRuntime.java:81,177,270``) fixes the order of a key's junction receivers, and
``PartitionStreamReceiver.cachedStreamJunctionMap`` the fan-out order over keys
(``PartitionStreamReceiver.java:277-281``). The JDK is a dependency outside ``/root/reference``;
this restates its published algorithm for single-threaded puts of distinct keys: ``spread``,
``putVal`` (append to a list bin, prepend to a tree bin's ``first`` list), ``addCount``'s resize at
``sizeCtl`` (3/4 of the table), ``transfer``'s lastRun split of list bins, ``treeifyBin`` (tables
under 64 bins are presized instead) and ``untreeify`` of small split halves. The engine restates it
again in C++ (``csrc/chm_order.h``) and the oracle a third time; tests compare them.
"""
from __future__ import annotations

from typing import List, Sequence

HASH_BITS = 0x7FFFFFFF
TREEIFY_THRESHOLD = 8
UNTREEIFY_THRESHOLD = 6
MIN_TREEIFY_CAPACITY = 64


def spread(h: int) -> int:
    """``ConcurrentHashMap.spread``: (h ^ (h >>> 16)) & HASH_BITS on the 32-bit hash."""
    u = h & 0xFFFFFFFF
    return (u ^ (u >> 16)) & HASH_BITS


class _Bin:
    __slots__ = ("nodes", "tree")

    def __init__(self, nodes=None, tree=False):
        self.nodes = nodes if nodes is not None else []   # (spread hash, id), iteration order
        self.tree = tree


class ChmOrder:
    """Default-constructed map (16 bins, sizeCtl 12); ``put`` distinct keys by hash."""

    def __init__(self):
        self.table: List[_Bin] = [_Bin() for _ in range(16)]
        self.size_ctl = 12
        self.count = 0

    def _transfer(self):
        n = len(self.table)
        nxt = [_Bin() for _ in range(2 * n)]
        for i, b in enumerate(self.table):
            if not b.nodes:
                continue
            if b.tree:
                lo = [x for x in b.nodes if not x[0] & n]
                hi = [x for x in b.nodes if x[0] & n]
                nxt[i] = _Bin(lo, len(lo) > UNTREEIFY_THRESHOLD)
                nxt[i + n] = _Bin(hi, len(hi) > UNTREEIFY_THRESHOLD)
                continue
            # the trailing run whose nodes all go the same way moves as is; the nodes before it are
            # re-linked one by one at the head of their half (so they come out reversed)
            last = len(b.nodes) - 1
            bit = b.nodes[last][0] & n
            while last > 0 and (b.nodes[last - 1][0] & n) == bit:
                last -= 1
            halves = {0: [], n: []}
            halves[bit] = list(b.nodes[last:])
            for node in b.nodes[:last]:
                halves[node[0] & n].insert(0, node)
            nxt[i], nxt[i + n] = _Bin(halves[0]), _Bin(halves[n])
        self.table = nxt
        self.size_ctl = 2 * n - (n >> 1)

    def _presize(self, size: int):
        c = 1
        while c < size + (size >> 1) + 1:
            c <<= 1
        while c > self.size_ctl and len(self.table) < (1 << 30):
            self._transfer()

    def put(self, h: int, ident: int):
        hs = spread(h)
        b = self.table[hs & (len(self.table) - 1)]
        if b.tree:
            b.nodes.insert(0, (hs, ident))   # TreeBin.putTreeVal links the node at `first`
        else:
            was = len(b.nodes)
            b.nodes.append((hs, ident))
            if was >= TREEIFY_THRESHOLD:
                if len(self.table) < MIN_TREEIFY_CAPACITY:
                    self._presize(len(self.table) << 1)
                else:
                    b.tree = True
        self.count += 1
        while self.count >= self.size_ctl:
            self._transfer()

    def order(self) -> List[int]:
        """Ids in iteration order (``values()`` / ``keySet()`` traversal, bin by bin)."""
        return [ident for b in self.table for _, ident in b.nodes]


def iteration_order(hashes: Sequence[int]) -> List[int]:
    """Indices of ``hashes`` (keys put in this order) in the map's iteration order."""
    m = ChmOrder()
    for i, h in enumerate(hashes):
        m.put(int(h), i)
    return m.order()


def positions(hashes: Sequence[int]) -> List[int]:
    """Per key its iteration position."""
    pos = [0] * len(hashes)
    for r, i in enumerate(iteration_order(hashes)):
        pos[i] = r
    return pos
