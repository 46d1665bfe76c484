"""GPU parity of the K_ratchet plan (2-state `every e1=S[f0] -> e2=S[a OP e1.a]`) against the CPU
oracle and against the general chain kernel (SDH_FLAG_NO_RATCHET), bit-exact match tuples."""
import numpy as np
import pytest

from harness import App
from siddhi_amd.workloads import c2_app, stock_events

pytestmark = pytest.mark.gpu

SDH_FLAG_NO_RATCHET = 2


def hip_app(src, **kw):
    from siddhi_amd.engine import HipEngine
    app = App(src, engine_factory=lambda blob: None)
    app.engine = HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], **kw)
    return app


def c2_columns(start, n):
    ts, sym, price, vol = stock_events(start, n)
    return ts, [sym, price.view(np.uint32), vol]


def words(cols):
    return np.stack([c.astype(np.int64) for c in cols], 1)


_ORACLE_CACHE = {}


def _c2_oracle_batches(n_pat, sizes):
    """The oracle's matches per batch of the C2 family (computed once per module: both chunk
    parametrisations check against the same run)."""
    key = (n_pat, sizes)
    if key not in _ORACLE_CACHE:
        o = App(c2_app(n_pat))
        out, start = [], 0
        for n in sizes:
            ts, cols = c2_columns(start, n)
            start += n
            o.engine.send(0, ts, words(cols), None)
            out.append(o.engine.take_matches(lambda q: 2))
        _ORACLE_CACHE[key] = out
    return _ORACLE_CACHE[key]


@pytest.mark.parametrize("chunk", [0, 512])
def test_c2_ratchet_vs_oracle_and_chain(chunk):
    src = c2_app(70)  # two wave groups, the second one partial
    sizes = (3000, 1, 7000, 777)
    want = _c2_oracle_batches(70, sizes)
    r = hip_app(src, chunk_events=chunk)
    c = hip_app(src, chunk_events=chunk, partials=256, flags=SDH_FLAG_NO_RATCHET)
    start = 0
    for bi, n in enumerate(sizes):
        ts, cols = c2_columns(start, n)
        start += n
        om = want[bi]
        r.engine.push_columns(0, ts, cols)
        rm = r.engine.take_matches(lambda q: 2)
        c.engine.push_columns(0, ts, cols)
        cm = c.engine.take_matches(lambda q: 2)
        assert rm == om
        assert cm == om
    assert r.engine.stats().matches > 50000


def test_c2_ratchet_vs_chain_large():
    """Full-shape differential check (both plans on the GPU, raw match arrays compared): 200
    patterns, 160K events in batches of uneven size, chunked so that the reverse-scan warm-up
    spans many chunks."""
    src = c2_app(200)
    r = hip_app(src, chunk_events=2048)
    c = hip_app(src, partials=256, flags=SDH_FLAG_NO_RATCHET)
    start, total = 0, 0
    for n in (60000, 17, 100000):
        ts, cols = c2_columns(start, n)
        start += n
        r.engine.push_columns(0, ts, cols)
        c.engine.push_columns(0, ts, cols)
        a, b = r.engine.poll(), c.engine.poll()
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
        total += len(a[0])
    assert total > 5_000_000


ORIENT = ["v > e1.v", "v >= e1.v", "v < e1.v", "v <= e1.v", "e1.v < v", "e1.v >= v"]


@pytest.mark.parametrize("typ", ["int", "long", "float", "double"])
def test_orientations_ties_nulls_nan(typ):
    qs = [f"define stream S (v {typ}, w int);"]
    for k, cond in enumerate(ORIENT):
        qs.append(f"@info(name='a{k}') from every e1=S[w > 2] -> e2=S[{cond}] within 40 milliseconds "
                  f"select e1.v as x insert into O;")
        qs.append(f"@info(name='b{k}') from every e1=S -> e2=S[{cond}] within 25 milliseconds "
                  f"select e1.v as x insert into O;")
    src = " ".join(qs)
    o = App(src)
    g = hip_app(src)
    rng = np.random.default_rng(5)
    vals = [0, 1, 2, 3, 3, 5, -1]
    if typ in ("float", "double"):
        vals += [float("nan"), -0.0, float("inf")]
    t = 0
    for k in range(1500):
        t += int(rng.integers(0, 4))
        v = vals[int(rng.integers(len(vals)))]
        if rng.random() < 0.04:
            v = None
        row = [v if v is None or typ in ("float", "double") else int(v), int(rng.integers(0, 6))]
        o.send("S", [row], [t])
        g.send("S", [row], [t])
    assert len(o.matches) > 2000
    assert g.matches == o.matches


def test_two_column_start_filter_and_batches():
    src = ("define stream S (a int, b float, c double); "
           "@info(name='q0') from every e1=S[a > 3 and b < c and c >= 2.5] -> e2=S[b > e1.b] within 30 "
           "milliseconds select e1.a as x insert into O; "
           "@info(name='q1') from every e1=S[b < c] -> e2=S[e1.b > b] within 90 milliseconds "
           "select e1.a as x insert into O;")
    o = App(src)
    g = hip_app(src, chunk_events=512)
    rng = np.random.default_rng(9)
    n = 20000
    ts = np.cumsum(rng.integers(0, 3, n)).astype(np.int64)
    a = rng.integers(0, 8, n).astype(np.int32)
    b = rng.integers(0, 50, n).astype(np.float32)
    c = rng.integers(0, 50, n).astype(np.float64)
    cols = [a, b.view(np.uint32), c.view(np.int64)]
    vals = np.stack([a.astype(np.int64), b.view(np.uint32).astype(np.int64), c.view(np.int64)], 1)
    for lo, hi in ((0, 3000), (3000, 3001), (3001, n)):
        o.engine.send(0, ts[lo:hi], vals[lo:hi], None)
        g.engine.push_columns(0, ts[lo:hi], [x[lo:hi] for x in cols])
        assert g.engine.take_matches(lambda q: 2) == o.engine.take_matches(lambda q: 2)


def test_deque_growth_to_10k_partials():
    """The reference's pending list is unbounded (StreamPreStateProcessor.java:298). A strictly
    decreasing run piles up every partial (no event matches any earlier one); the spill ring and the
    persisted deques double and the push re-runs exactly until 10K+ partials per pattern fit. The
    closing high value then matches all of them. Also chunked (reverse-scan warm-up over the pile)
    and through snapshot/restore into a fresh engine."""
    src = ("define stream S (v int); @info(name='q') from every e1=S -> e2=S[v > e1.v] select e1.v as a insert into O; "
           "@info(name='r') from every e1=S[v > 5000] -> e2=S[v > e1.v] select e1.v as a insert into O;")
    n = 12000
    ts = np.arange(n + 1, dtype=np.int64)
    v = np.concatenate([np.arange(n, 0, -1), [10 * n]]).astype(np.int32)
    o = App(src)  # (one oracle run for both chunk modes)
    o.engine.send(0, ts[:n], v[:n].astype(np.int64)[:, None], None)
    assert o.engine.take_matches(lambda q: 2) == []
    o.engine.send(0, ts[n:], v[n:].astype(np.int64)[:, None], None)
    want = o.engine.take_matches(lambda q: 2)
    for chunk in (0, 1024):
        g = hip_app(src, chunk_events=chunk)
        g.engine.push_columns(0, ts[:n], [v[:n]])
        assert g.engine.take_matches(lambda q: 2) == []
        assert g.engine.stats().live_partials == n + (n - 5000)
        g.engine.poll()
        snap = g.engine.snapshot()
        b = hip_app(src, chunk_events=chunk)
        b.engine.restore(snap)
        g.engine.push_columns(0, ts[n:], [v[n:]])
        b.engine.push_columns(0, ts[n:], [v[n:]])
        assert len(want) == n + (n - 5000)
        assert g.engine.take_matches(lambda q: 2) == want
        assert b.engine.take_matches(lambda q: 2) == want


def test_ratchet_unordered_timestamps_exact():
    src = c2_app(70)
    o = App(src)
    g = hip_app(src, chunk_events=1024)
    ts, cols = c2_columns(0, 12000)
    ts = ts.copy()
    ts[9000:9050] -= 20000
    o.engine.send(0, ts, words(cols), None)
    g.engine.push_columns(0, ts, cols)
    assert g.engine.take_matches(lambda q: 2) == o.engine.take_matches(lambda q: 2)
    ts2, cols2 = c2_columns(12000, 5000)
    o.engine.send(0, ts2, words(cols2), None)
    g.engine.push_columns(0, ts2, cols2)
    assert g.engine.take_matches(lambda q: 2) == o.engine.take_matches(lambda q: 2)


def test_ratchet_wide_timestamp_spans_and_windows():
    """The lazy forms compare deadlines in a 32-bit domain relative to each item's first timestamp
    (nfa_ratchet.hip rel_deadline): windows beyond 2^31 ms clamp to `never within this batch`,
    partials carried from far older batches clamp to `already expired`, and a batch spanning 2^31 ms
    or more runs in the FULL form. Timestamps far from 0, chunked and unchunked."""
    src = ("define stream S (v int); "
           "@info(name='a') from every e1=S[v > 2] -> e2=S[v > e1.v] within 35 days select e1.v as x insert into O; "
           "@info(name='b') from every e1=S -> e2=S[v < e1.v] within 3 sec select e1.v as x insert into O; "
           "@info(name='c') from every e1=S[v < 7] -> e2=S[v >= e1.v] within 40 milliseconds "
           "select e1.v as x insert into O;")
    rng = np.random.default_rng(21)
    base = 1 << 40
    batches = []
    t = base
    for n, step_hi in ((4000, 3), (3000, 2_000_000), (2500, 3), (2000, 5_000_000), (3000, 2)):
        ts = t + np.cumsum(rng.integers(0, step_hi, n)).astype(np.int64)
        t = int(ts[-1])
        batches.append((ts, rng.integers(0, 12, n).astype(np.int32)))
    # a gap of ~30 days between two batches and one batch whose own span is > 2^31 ms
    batches[2] = (batches[2][0] + 30 * 86_400_000, batches[2][1])
    t = int(batches[2][0][-1])
    batches[3] = (t + np.sort(rng.integers(0, 3 << 31, 2000)).astype(np.int64), batches[3][1])
    t = int(batches[3][0][-1])
    batches[4] = (t + np.cumsum(rng.integers(0, 2, 3000)).astype(np.int64), batches[4][1])
    for chunk in (0, 256):
        o = App(src)
        g = hip_app(src, chunk_events=chunk)
        for ts, v in batches:
            o.engine.send(0, ts, v.astype(np.int64)[:, None], None)
            g.engine.push_columns(0, ts, [v])
            assert g.engine.take_matches(lambda q: 2) == o.engine.take_matches(lambda q: 2)
        assert g.engine.stats().matches > 10000


def test_ratchet_snapshot_restore():
    src = c2_app(66)
    a = hip_app(src)
    ts, cols = c2_columns(0, 8000)
    a.engine.push_columns(0, ts, cols)
    a.engine.poll()
    snap = a.engine.snapshot()
    ts2, cols2 = c2_columns(8000, 6000)
    a.engine.push_columns(0, ts2, cols2)
    ref = a.engine.take_matches(lambda q: 2)
    b = hip_app(src)
    b.engine.restore(snap)
    b.engine.push_columns(0, ts2, cols2)
    assert b.engine.take_matches(lambda q: 2) == ref
    assert len(ref) > 1000


class _Hip:
    """Device buffers through the HIP runtime the engine library links (libamdhip64)."""

    def __init__(self):
        import ctypes
        self.c = ctypes
        self.rt = ctypes.CDLL("libamdhip64.so.7")
        self.bufs = []

    def put(self, arr):
        c = self.c
        arr = np.ascontiguousarray(arr)
        p = c.c_void_p()
        assert self.rt.hipMalloc(c.byref(p), c.c_size_t(max(1, arr.nbytes))) == 0
        assert self.rt.hipMemcpy(p, c.c_void_p(arr.ctypes.data), c.c_size_t(arr.nbytes), 1) == 0
        self.bufs.append(p)
        return p.value

    def fill(self, ptr, nbytes, byte):
        assert self.rt.hipMemset(self.c.c_void_p(ptr), byte, self.c.c_size_t(nbytes)) == 0
        assert self.rt.hipDeviceSynchronize() == 0

    def free(self):
        for p in self.bufs:
            self.rt.hipFree(p)


def test_device_batch_records_outlive_caller_buffer():
    """Records of a device-resident batch are decoded at poll time, after the caller has reused its
    buffers: the engine keeps its own copy of the batch's timestamps."""
    src = c2_app(40)
    a, b = hip_app(src), hip_app(src)
    ts, cols = c2_columns(0, 20000)
    h = _Hip()
    try:
        dts = h.put(ts)
        a.engine.push_device(0, len(ts), dts, [h.put(c) for c in cols])
        h.fill(dts, ts.nbytes, 0xFF)
        b.engine.push_columns(0, ts, cols)
        x, y = a.engine.poll(), b.engine.poll()
    finally:
        h.free()
    assert len(x[0]) > 10000
    for u, v in zip(x, y):
        assert np.array_equal(u, v)


def test_wide_records_for_batches_beyond_2_26_events():
    """A push of more than 2^26 events uses 16-B device records; the same events pushed as two
    smaller batches (8-B records) must give identical matches."""
    n = (1 << 26) + 4_000_000
    qs = ["define stream StockStream (symbol string, price float, volume int);"]
    for p in range(4):
        qs.append(f"@info(name='w{p}') from every e1=StockStream[price > {99.2 + p / 10}] -> "
                  f"e2=StockStream[price > e1.price] within {1 + p} sec select e1.price as p1 insert into O;")
    src = " ".join(qs)
    a, b = hip_app(src), hip_app(src)
    ts, cols = c2_columns(0, n)
    a.engine.push_columns(0, ts, cols)
    x = a.engine.poll()
    h = n // 2 + 12345
    b.engine.push_columns(0, ts[:h], [c[:h] for c in cols])
    y0 = b.engine.poll()
    b.engine.push_columns(0, ts[h:], [c[h:] for c in cols])
    y1 = b.engine.poll()
    assert len(x[0]) > 500_000
    for i in (0, 1, 2, 4):  # query, key, ts, slot words
        assert np.array_equal(x[i], np.concatenate([y0[i], y1[i]]))
    assert np.array_equal(x[3], np.concatenate([y0[3], y1[3][1:] + y0[3][-1]]))


def test_ring_rec4_distance_overflow_reruns_with_8b_records():
    """SDH_FLAG_DEVICE_MATCHES pushes write 4-B K_ratchet entries (an e1 distance below 2^26 and the
    lane) with one side entry per matching event (nfa_types.h rec4). A partial matched more than 2^26
    events after it opened sets err[4] and that push re-runs with 8-B records (its records come out as
    SDH_REC_8); the next push writes rec4 again. The device-record engine's record digest equals the
    normal-mode engine's in every push."""
    import torch
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES, SDH_REC_4, SDH_REC_8, HipEngine
    src = ("define stream S (v float); @info(name='q') from every e1=S[v > 2.0] -> e2=S[v > e1.v] "
           "select e1.v as a insert into O;")  # (SIM form; no `within`: one unchunked item per push)
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    normal = HipEngine(app.blob, stream_types=types)
    ring = HipEngine(app.blob, stream_types=types, flags=SDH_FLAG_DEVICE_MATCHES)
    dev = torch.device("cuda:0")
    n1 = 1 << 26  # (not past 2^26: the push keeps 8-B / rec4 records)
    fmts = []
    for lo, vals in ((0, None), (n1, [1, 1, 10]), (n1 + 3, [3, 20, 1])):
        n = n1 if vals is None else len(vals)
        ts = torch.arange(lo, lo + n, dtype=torch.int64, device=dev)
        if vals is None:
            v = torch.ones(n, dtype=torch.float32, device=dev)
            v[0] = 5
        else:
            v = torch.tensor(vals, dtype=torch.float32, device=dev)
        for e in (normal, ring):
            e.push_device(0, n, ts.data_ptr(), [v.data_ptr()])
        dn, dr = normal.debug_digest(), ring.debug_digest()
        assert dn == dr, f"push at {lo}: normal {dn} != ring {dr}"
        rec = ring.poll_records()
        assert rec.r_n == dn[0]
        fmts.append(rec.r_format)
        del ts, v
    # push 2: the partial of the first event, matched 2^26 + 2 events later -> the 8-B re-run;
    # push 3: two short-distance matches -> rec4 again
    assert fmts[1:] == [SDH_REC_8, SDH_REC_4]
    assert dn[0] == 2
    normal.close()
    ring.close()
