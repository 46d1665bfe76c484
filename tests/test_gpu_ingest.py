"""Host-resident batches (sdh_batch.on_device = 0; north_star (2): SoA batches in pinned host
memory copied on a side stream): pageable and pinned host pushes reach HBM intact -- the same
matches as device-resident pushes of the same stream, with nulls -- and the copy is accounted."""
import numpy as np
import pytest

from harness import App

pytestmark = pytest.mark.gpu


def test_host_batches_pageable_and_pinned_equal_device_batches():
    import torch
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.workloads import c2_app, stock_events
    app = App(c2_app(64), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    dev_e, page_e, pin_e = (HipEngine(app.blob, stream_types=types) for _ in range(3))
    n = 1_100_000  # ts column 8.8 MB: three 4-MiB staging slices
    ts, sym, price, vol = stock_events(0, n)
    cols = [sym, price.view(np.uint32), vol]
    d = [torch.from_numpy(np.ascontiguousarray(x).view(np.int32) if x.dtype != np.int64 else x).cuda()
         for x in [ts] + cols]
    dev_e.push_device(0, n, d[0].data_ptr(), [c.data_ptr() for c in d[1:]])
    page_e.push_columns(0, ts, cols)
    assert page_e.stats().last_ingest_ms > 0
    pinned = [torch.from_numpy(np.ascontiguousarray(x)).pin_memory() for x in [ts] + cols]
    pin_e.push_columns(0, pinned[0].numpy(), [p.numpy() for p in pinned[1:]])
    assert pin_e.stats().ingest_bytes == page_e.stats().ingest_bytes >= n * 20
    a, b, c = dev_e.poll(), page_e.poll(), pin_e.poll()
    assert len(a[0]) > 1_000_000
    for x, y, z in zip(a, b, c):
        assert np.array_equal(x, y) and np.array_equal(x, z)


def test_host_batch_with_nulls_matches_oracle():
    from siddhi_amd.engine import HipEngine
    src = ("define stream S (k int, p float, v long); @info(name='q') from every e1=S[p > 50.0] -> "
           "e2=S[v > e1.v] within 40 milliseconds select e1.p as a insert into O;")
    o = App(src)
    g = App(src, engine_factory=lambda blob: None)
    g.engine = HipEngine(g.blob, stream_types=[s.attr_types for s in g.ir.streams])
    rng = np.random.default_rng(3)
    n = 50000
    ts = np.cumsum(rng.integers(0, 3, n)).astype(np.int64)
    vals = np.stack([rng.integers(0, 9, n), (rng.integers(0, 10000, n) / 100.0).astype(np.float32).view(np.uint32),
                     rng.integers(-1000, 1000, n)], 1).astype(np.int64)
    nl = (rng.random((n, 3)) < 0.05).astype(np.uint8)
    o.engine.send(0, ts, vals, nl)
    g.engine.send(0, ts, vals, nl)
    om = o.engine.take_matches(lambda q: 2)
    assert g.engine.take_matches(lambda q: 2) == om and len(om) > 10000
