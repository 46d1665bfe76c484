"""The C host (tests/native/c1_abi.c): include/siddhi_hip.h + include/siddhi_hip_ir.h alone, no Python
binding -- a hand-built C1 blob, create, host pushes and polls on the GPU. Its delivered matches (count
and an order-dependent hash of every tuple) equal the oracle's over the same seeded stream, and over
1M events it reproduces the large_c1 golden's count."""
import subprocess

import numpy as np
import pytest

from harness import App
from large_golden import load
from test_abi import _c1_abi

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


def _fnv(matches):
    h = 1469598103934665603
    for q, k, ts, slots in matches:
        words = []
        for s in slots:
            words += [len(s)] + list(s)
        for w in [q, k, ts, len(words)] + words:
            h = ((h ^ (w & M64)) * 1099511628211) & M64
    return h


def _run(n, bs):
    out = subprocess.run([_c1_abi(), "run", str(n), str(bs)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    f = out.stdout.split()
    return int(f[1]), int(f[3])


def test_c_host_matches_equal_the_oracle():
    from siddhi_amd.workloads import c1_app, stock_events
    n = 60000
    o = App(c1_app())
    ts, sym, price, vol = stock_events(0, n)
    vals = np.stack([sym.astype(np.int64), price.view(np.uint32).astype(np.int64), vol.astype(np.int64)], 1)
    o.engine.send(0, ts, vals, None)
    want = o.engine.take_matches(lambda q: 2)
    got_n, got_h = _run(n, 4096)
    assert got_n == len(want) > 1000
    assert got_h == _fnv(want)


def test_c_host_reproduces_the_c1_golden_count():
    g = load("c1")
    got_n, _ = _run(g["events"], 1 << 16)
    assert got_n == g["n_matches"]
