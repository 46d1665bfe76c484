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


def test_compact_rows_when_lanes_walk_their_deques():
    """Placed rows whose lane count comes from the deque walk: with 4 LDS entries per lane
    (SDH_RATCHET_ML=4) and falling runs of 12-40 prices every partial stays pending until one high
    price matches them all, so a lane pops past its first round's four compares, through the LDS ring
    into the spill ring. The placed rows must equal the table path's (SDH_NO_PLACE on the second
    engine), restated from its poll."""
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.workloads import TS0, c2_app
    app = App(c2_app(64), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    a = HipEngine(app.blob, stream_types=types, debug={"SDH_RATCHET_ML": 4})
    b = HipEngine(app.blob, stream_types=types, debug={"SDH_RATCHET_ML": 4, "SDH_NO_PLACE": 1})
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
        b.push_columns(0, ts[sl], part)
        seq_base, rows = a.poll_compact()
        q, k, t, off, words, seq, tb = b.poll(with_seq=True)
        assert seq_base == seq_polled
        assert len(q) > 1000
        assert np.array_equal(rows, restate(q, off, words, seq, rows.shape[1], seq_base))
        seq_polled = lo + 5000
    assert a.stats().placed_pushes == n // 5000
    assert b.stats().placed_pushes == 0


def restate_ex(q, k, off, words, seq, tb, width, seq_base, with_key, with_tb):
    """poll tuples -> what sdh_engine_poll_compact_ex promises: rows with chains in a side array
    (include/siddhi_hip.h), keys and timer tiebreaks beside them"""
    rows = np.full((len(q), width), EMPTY, np.int64)
    chain = []
    for i in range(len(q)):
        rows[i, 0] = q[i]
        rows[i, 1] = seq[i] - seq_base
        w = words[off[i]:off[i + 1]]
        j, slot = 0, 0
        while j < len(w):
            c = int(w[j])
            if c == 1:
                rows[i, 2 + slot] = seq[i] - w[j + 1]
            elif c >= 2:
                rows[i, 2 + slot] = -(len(chain) + 1)
                chain += [c] + [int(seq[i] - x) for x in w[j + 1:j + 1 + c]]
            j += 1 + c
            slot += 1
    return rows.astype(np.int32), (np.asarray(k) if with_key else None), (np.asarray(tb) if with_tb else None), \
        np.asarray(chain, np.int32)


def _ex_equals_poll(a, b, with_key, with_tb):
    seq_base, rows, key, tb, chain = a.poll_compact_ex()
    q, k, t, off, words, seq, tbb = b.poll(with_seq=True)
    want = restate_ex(q, k, off, words, seq, tbb, rows.shape[1], seq_base, with_key, with_tb)
    assert np.array_equal(rows, want[0])
    assert (key is None) == (not with_key) and (tb is None) == (not with_tb)
    if with_key:
        assert np.array_equal(key, want[1])
    if with_tb:
        assert np.array_equal(tb, want[2])
    assert np.array_equal(chain, want[3])
    return len(q)


@pytest.mark.parametrize("family", ["c3", "c5"])
def test_compact_ex_equals_poll_partitioned_families(family):
    """Count chains and partition keys (C3: K_part count / and / or; C5: K_slab over four streams)."""
    from siddhi_amd.workloads import c3_app, c5_app, c5_events, stock_events
    src = c3_app(48) if family == "c3" else c5_app(64)
    a, b = _engines(src)
    total, lo = 0, 0
    for i in range(8):
        if family == "c3":
            ts, sym, price, vol = stock_events(lo, 3000, 12)
            cols = [(0, ts, [sym, price.view(np.uint32), vol])]
            lo += 3000
        else:
            cols = []
            for si in range(4):
                ts, acct, amt, code = c5_events(si, lo, 1500, 40)
                cols.append((si, ts, [acct, amt.view(np.uint32), code]))
            lo += 1500
        for si, ts, c in cols:
            a.push_columns(si, ts, c)
            b.push_columns(si, ts, c)
        if i % 2:
            total += _ex_equals_poll(a, b, True, False)
    assert total > 1000


def test_compact_ex_equals_poll_absent_apps():
    """Timer matches of absent states (tb beside the rows), on the absent-app timelines."""
    from dist_gpu_child import batches
    from siddhi_amd.events import encode_rows
    from siddhi_amd.engine import columns_from_words
    from test_dist import events, full_src
    app = App(full_src(absent=True), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    a, b = _engines(full_src(absent=True))
    evs = events()
    total = 0
    for i, (stream, rows, ts) in enumerate(batches(evs)):
        si = app.ir.stream_index(stream)
        vals, nulls = encode_rows(rows, types[si], app.dictionary)
        cols = columns_from_words(vals, types[si])
        a.push_columns(si, np.asarray(ts, np.int64), cols)
        b.push_columns(si, np.asarray(ts, np.int64), cols)
        if i % 4 == 3:
            total += _ex_equals_poll(a, b, True, True)
    a.advance_time(evs[-1][2] + 100)
    b.advance_time(evs[-1][2] + 100)
    total += _ex_equals_poll(a, b, True, True)
    assert total > 50


def test_compact_ex_placed_and_unpartitioned():
    """A program without partitions or absent states: no key / tb arrays; placed K_ratchet windows and
    chain windows (a count state in an unpartitioned query) both convert."""
    from siddhi_amd.workloads import c2_app, stock_events
    src = c2_app(64) + (" @info(name='n1') from every e1=StockStream[price > 80] -> "
                        "e2=StockStream[price < 20]<2:4> -> e3=StockStream[price > 50] within 1 sec "
                        "select e1.price as a insert into O;")
    for s in (c2_app(64), src):
        a, b = _engines(s)
        ts, sym, price, vol = stock_events(0, 20000)
        cols = [sym, price.view(np.uint32), vol]
        a.push_columns(0, ts, cols)
        b.push_columns(0, ts, cols)
        assert _ex_equals_poll(a, b, False, False) > 1000
