"""sdh_engine_poll_compact: the R18-ordered matches as compact int32 rows.

Against sdh_engine_poll on a second engine fed the same pushes: the compact rows must be exactly
the poll tuples restated (query, trigger seq - seq_base, per slot trigger seq - the slot's event
seq, INT32_MIN for an empty slot), over placed windows (K_ratchet placement: the rows are handed
out as they are) and table windows (chain / K_gen matches: sorted, then converted). Matches the
form cannot express (count-state chains, partition keys) fail with SDH_E_UNSUPPORTED and stay
pending for sdh_engine_poll.
"""
import numpy as np
import pytest

from harness import App

pytestmark = pytest.mark.gpu

EMPTY = np.iinfo(np.int32).min


def restate(q, off, words, seq, width, seq_base):
    """poll tuples -> the compact rows sdh_engine_poll_compact promises (include/siddhi_hip.h)"""
    n = len(q)
    rows = np.full((n, width), EMPTY, np.int64)
    rows[:, 0] = q
    rows[:, 1] = seq - seq_base
    j = off[:-1].copy()
    w = np.append(words, 0)
    for slot in range(width - 2):
        live = j < off[1:]
        c = np.where(live, w[np.minimum(j, len(words))], 0)
        assert np.all(c <= 1)
        one = live & (c == 1)
        rows[one, 2 + slot] = seq[one] - w[j[one] + 1]
        j = np.where(live, j + 1 + c, j)
    assert np.array_equal(j, off[1:])
    return rows.astype(np.int32)


def _engines(src, **kw):
    from siddhi_amd.engine import HipEngine
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    return HipEngine(app.blob, stream_types=types, **kw), HipEngine(app.blob, stream_types=types, **kw)


MIXED = (" @info(name='x3') from every e1=StockStream[price > 90] -> e2=StockStream[price < 10] "
         "-> e3=StockStream[price > e1.price] within 1 sec select e1.price as a insert into O;"
         " @info(name='xl') from every e1=StockStream[price > 98] -> e2=StockStream[volume > 990] "
         "or e3=StockStream[price < 0.5] within 1 sec select e1.price as a insert into O;")


@pytest.mark.parametrize("mixed", [False, True])
def test_compact_equals_poll(mixed):
    from siddhi_amd.workloads import c2_app, stock_events
    a, b = _engines(c2_app(200) + (MIXED if mixed else ""))
    sizes = [700, 9000, 5, 1300, 40000, 1, 2500, 800, 800, 800, 6000, 300]
    polls = {0, 2, 4, 5, 9, 11}
    lo, total, seq_polled = 0, 0, 0
    for i, n in enumerate(sizes):
        ts, sym, price, vol = stock_events(lo, n)
        lo += n
        cols = [sym, price.view(np.uint32), vol]
        a.push_columns(0, ts, cols)
        b.push_columns(0, ts, cols)
        if i in polls:
            seq_base, rows = a.poll_compact()
            q, k, t, off, words, seq, tb = b.poll(with_seq=True)
            assert seq_base == seq_polled
            assert rows.shape == (len(q), 5 if mixed else 4)
            assert np.array_equal(rows, restate(q, off, words, seq, rows.shape[1], seq_base))
            total += len(q)
            seq_polled = lo
    assert total > 100000
    assert a.stats().placed_pushes > 0


def test_compact_device_rows():
    """device=1: the same rows left in HBM"""
    import ctypes
    from siddhi_amd.workloads import c2_app, stock_events
    a, b = _engines(c2_app(64) + MIXED)
    ts, sym, price, vol = stock_events(0, 20000)
    cols = [sym, price.view(np.uint32), vol]
    a.push_columns(0, ts, cols)
    b.push_columns(0, ts, cols)
    m = a.poll_compact(device=True)
    _, rows = b.poll_compact()
    assert m.n == len(rows) > 10000 and m.width == rows.shape[1]
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    got = np.zeros_like(rows)
    assert hip.hipMemcpy(got.ctypes.data, ctypes.cast(m.rows, ctypes.c_void_p).value, got.nbytes, 2) == 0
    assert np.array_equal(got, rows)


@pytest.mark.parametrize("kind", ["count", "partition"])
def test_compact_unsupported_keeps_window(kind):
    from siddhi_amd.engine import EngineError
    from siddhi_amd.workloads import STOCK_STREAM, c2_app, stock_events
    if kind == "count":
        src = c2_app(8) + (" @info(name='n1') from every e1=StockStream[price > 80] -> "
                           "e2=StockStream[price < 20]<2:4> -> e3=StockStream[price > 50] within 1 sec "
                           "select e1.price as a insert into O;")
    else:
        src = (STOCK_STREAM + " partition with (symbol of StockStream) begin "
               "@info(name='p1') from every e1=StockStream[price > 70] -> e2=StockStream[price < 30] "
               "within 1 sec select e1.price as a insert into O; end;")
    a, b = _engines(src)
    ts, sym, price, vol = stock_events(0, 20000)
    cols = [sym, price.view(np.uint32), vol]
    a.push_columns(0, ts, cols)
    b.push_columns(0, ts, cols)
    with pytest.raises(EngineError) as ex:
        a.poll_compact()
    assert ex.value.code == -2  # SDH_E_UNSUPPORTED
    ga, gb = a.poll(with_seq=True), b.poll(with_seq=True)
    assert len(ga[0]) > 0
    for x, y in zip(ga, gb):
        assert np.array_equal(x, y)


def test_compact_rows_when_lanes_walk_their_deques(monkeypatch):
    """Placed rows whose lane count comes from the deque walk: with 4 LDS entries per lane
    (SDH_RATCHET_ML=4) and falling runs of 12-40 prices every partial stays pending until one high
    price matches them all, so a lane pops past its first round's four compares, through the LDS ring
    into the spill ring. The placed rows must equal the table path's (SDH_NO_PLACE on the second
    engine), restated from its poll."""
    import os
    from siddhi_amd.workloads import TS0, c2_app
    monkeypatch.setenv("SDH_RATCHET_ML", "4")
    a, b = _engines(c2_app(64))
    monkeypatch.delenv("SDH_RATCHET_ML")
    rng = np.random.default_rng(7)
    price = []
    while len(price) < 30000:
        run = int(rng.integers(12, 41))
        top = float(rng.uniform(60.0, 99.0))
        price += list(np.linspace(top, top - rng.uniform(5, 40), run)) + [99.99]
    price = np.asarray(price[:30000], np.float32)
    n = len(price)
    ts = TS0 + np.arange(n, dtype=np.int64)
    cols = [np.zeros(n, np.int32), price.view(np.uint32), np.ones(n, np.int32)]
    seq_polled = 0
    for lo in range(0, n, 5000):
        sl = slice(lo, lo + 5000)
        part = [c[sl] for c in cols]
        a.push_columns(0, ts[sl], part)
        os.environ["SDH_NO_PLACE"] = "1"
        try:
            b.push_columns(0, ts[sl], part)
        finally:
            del os.environ["SDH_NO_PLACE"]
        seq_base, rows = a.poll_compact()
        q, k, t, off, words, seq, tb = b.poll(with_seq=True)
        assert seq_base == seq_polled
        assert len(q) > 1000
        assert np.array_equal(rows, restate(q, off, words, seq, rows.shape[1], seq_base))
        seq_polled = lo + 5000
    assert a.stats().placed_pushes == n // 5000
    assert b.stats().placed_pushes == 0
