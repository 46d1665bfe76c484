"""The reference runtime's ConcurrentHashMap iteration order (JDK 8; the fan-out order of
PartitionStreamReceiver.send(ComplexEvent), PartitionStreamReceiver.java:277-281), restated three
times independently: the engine's siddhi_amd/csrc/chm_order.h, the oracle's JavaCHM and the model
below (from the JDK 8 sources' published algorithm: putVal, addCount, transfer, treeifyBin,
tryPresize). No JVM is available, so this pins the three restatements to each other -- on random
keys and on colliding ones that drive bins into TreeBins and the pre-sizing path -- not to Java."""
import ctypes

import numpy as np
import pytest

from harness import oracle_lib
from kgen_host import lib as kgen_lib


def spread(h):
    return ((h & 0xFFFFFFFF) ^ ((h & 0xFFFFFFFF) >> 16)) & 0x7FFFFFFF


def jdk8_positions(hashes):
    tab = [[] for _ in range(16)]   # bins: lists of (spread, id); TreeBins keep their `first` order
    tree = [False] * 16
    size_ctl, count = 12, 0

    def transfer():
        nonlocal tab, tree, size_ctl
        n = len(tab)
        nt, ntree = [[] for _ in range(2 * n)], [False] * (2 * n)
        for i, b in enumerate(tab):
            if not b:
                continue
            if not tree[i]:
                run_bit, last = b[0][0] & n, 0
                for k in range(1, len(b)):
                    if (b[k][0] & n) != run_bit:
                        run_bit, last = b[k][0] & n, k
                lo = list(b[last:]) if run_bit == 0 else []
                hi = list(b[last:]) if run_bit != 0 else []
                for node in b[:last]:
                    (lo if (node[0] & n) == 0 else hi).insert(0, node)
                nt[i], nt[i + n] = lo, hi
            else:
                lo = [x for x in b if (x[0] & n) == 0]
                hi = [x for x in b if (x[0] & n) != 0]
                nt[i], nt[i + n] = lo, hi
                ntree[i], ntree[i + n] = len(lo) > 6, len(hi) > 6
        tab, tree = nt, ntree
        size_ctl = 2 * n - (n >> 1)

    for ident, h in enumerate(hashes):
        hs = spread(int(h))
        i = hs & (len(tab) - 1)
        bin_count = 0
        if not tab[i]:
            tab[i].append((hs, ident))
        elif tree[i]:
            tab[i].insert(0, (hs, ident))
            bin_count = 2
        else:
            bin_count = len(tab[i])
            tab[i].append((hs, ident))
            if bin_count >= 8:
                if len(tab) < 64:
                    size = len(tab) << 1
                    c = 1
                    while c < size + (size >> 1) + 1:
                        c <<= 1
                    while c > size_ctl:
                        transfer()
                else:
                    tree[i] = True
        count += 1
        while count >= size_ctl:
            transfer()
    pos = [0] * len(hashes)
    r = 0
    for b in tab:
        for _, ident in b:
            pos[ident] = r
            r += 1
    return pos


def _c_positions(fn, hashes):
    h = np.ascontiguousarray(hashes, dtype=np.int32)
    out = np.zeros(len(h), np.int32)
    fn(h.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(len(h)), out.ctypes.data_as(ctypes.c_void_p))
    return out.tolist()


def _colliding(n, rng, low_bits=6):
    """hashes whose spread values share their low `low_bits` bits (one bin until the table passes
    2^low_bits), distinct above"""
    out = []
    while len(out) < n:
        h = int(rng.integers(-2**31, 2**31))
        if spread(h) & ((1 << low_bits) - 1) == 0:
            out.append(h)
    return out


@pytest.mark.parametrize("case", ["random", "collide6", "collide4", "collide8", "mixed"])
@pytest.mark.parametrize("n", [1, 11, 12, 13, 47, 48, 49, 300, 2000])
def test_three_restatements_agree(case, n):
    rng = np.random.default_rng(n * 7 + len(case))
    if case == "random":
        hashes = rng.integers(-2**31, 2**31, n).tolist()
    elif case == "mixed":
        hashes = _colliding(n // 2, rng, 6) + rng.integers(-2**31, 2**31, n - n // 2).tolist()
        rng.shuffle(hashes)
    else:
        hashes = _colliding(n, rng, int(case[len("collide"):]))
    want = jdk8_positions(hashes)
    olib, klib = oracle_lib(), kgen_lib()
    assert _c_positions(olib.oracle_chm_positions, hashes) == want
    assert _c_positions(klib.kgh_chm_positions, hashes) == want
    assert sorted(want) == list(range(n))
