"""GPU parity of the K_gate plan (nfa_gate.hip): `every e1=S[f0] -> e2=S[cur.a OP e1.a and g]` with g
event-only conjuncts -- the pending keys are not monotone, so the lists are scanned -- against the CPU
oracle (oracle/oracle.cpp, the restatement of StreamPreStateProcessor.processAndReturn), bit-exact
match tuples in delivery order, over pushes that chunk (reverse-scan warm-up), lists that outgrow
LDS into the spill ring and the spill ring's exact re-run, out-of-order timestamps (the FULL form),
and the device-record mode."""
import numpy as np
import pytest

from harness import App

pytestmark = pytest.mark.gpu

ORIENT = ["v > e1.v", "v >= e1.v", "v < e1.v", "v <= e1.v", "e1.v < v", "e1.v >= v"]
GATES = ["w > 3", "w <= 4", "w != 2", "5 > w", "w >= 1 and w < 6", "u > 0.5"]


def hip_app(src, **kw):
    from siddhi_amd.engine import HipEngine
    app = App(src, engine_factory=lambda blob: None)
    app.engine = HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], **kw)
    return app


def gated_src(typ, seed, n=24):
    rng = np.random.default_rng(seed)
    qs = [f"define stream S (v {typ}, w int, u double);"]
    for k in range(n):
        cond = ORIENT[k % len(ORIENT)]
        gate = GATES[int(rng.integers(len(GATES)))]
        start = ["", "[w > 1]", "[v > 2]", "[u < 0.8 and w != 3]"][int(rng.integers(4))]
        within = [" within 40 milliseconds", " within 300 milliseconds", ""][int(rng.integers(3))]
        qs.append(f"@info(name='g{k}') from every e1=S{start} -> e2=S[{cond} and {gate}]{within} "
                  f"select e1.v as x insert into O;")
    return " ".join(qs)


def events(typ, n, seed, unordered=False):
    rng = np.random.default_rng(seed)
    ts = np.cumsum(rng.integers(0, 3, n)).astype(np.int64)
    if unordered:
        ts = ts + rng.integers(-2, 3, n) * (rng.random(n) < 0.05)
    if typ in ("float", "double"):
        v = rng.integers(0, 40, n).astype(np.float64)
        v[rng.random(n) < 0.01] = np.nan
    else:
        v = rng.integers(0, 40, n)
    w = rng.integers(0, 8, n).astype(np.int32)
    u = rng.random(n)
    vn = rng.random(n) < 0.02
    return ts, v, w, u, vn


def cols_vals(typ, v, w, u, vn):
    if typ == "float":
        vc = v.astype(np.float32).view(np.uint32)
        vw = vc.astype(np.int64)
    elif typ == "double":
        vc = v.astype(np.float64).view(np.int64)
        vw = vc
    elif typ == "int":
        vc = v.astype(np.int32)
        vw = vc.astype(np.int64)
    else:
        vc = v.astype(np.int64)
        vw = vc
    uc = u.astype(np.float64).view(np.int64)
    cols = [vc, w, uc]
    vals = np.stack([vw, w.astype(np.int64), uc], 1)
    nulls = np.zeros((len(v), 3), np.uint8)
    nulls[:, 0] = vn
    return cols, vals, nulls


@pytest.mark.parametrize("typ", ["int", "float"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gate_vs_oracle(typ, seed):
    src = gated_src(typ, seed)
    o = App(src)
    g = hip_app(src, chunk_events=256)
    st = g.engine.stats().plan_queries
    assert st[1] == 24 and st[0] == 0 and st[2] == 0, list(st)
    n = 12000
    ts, v, w, u, vn = events(typ, n, seed + 10)
    cols, vals, nulls = cols_vals(typ, v, w, u, vn)
    total = 0
    for lo, hi in ((0, 3000), (3000, 3001), (3001, 7000), (7000, n)):
        o.engine.send(0, ts[lo:hi], vals[lo:hi], nulls[lo:hi])
        g.engine.push_columns(0, ts[lo:hi], [c[lo:hi] for c in cols], [nulls[lo:hi, j] for j in range(3)])
        want = o.engine.take_matches(lambda q: 2)
        assert g.engine.take_matches(lambda q: 2) == want
        total += len(want)
    assert total > 8000


def test_gate_long_lists_spill_and_regrow():
    """A gate that almost never opens: each lane's list outgrows its 16 LDS entries into the spill
    ring, and the spill ring's 256 entries -- the push re-runs exactly with a larger ring."""
    src = ("define stream S (v int, w int); "
           "@info(name='a') from every e1=S -> e2=S[v > e1.v and w == 7] select e1.v as x insert into O; "
           "@info(name='b') from every e1=S[v > 10] -> e2=S[e1.v >= v and w > 6] within 2000 milliseconds "
           "select e1.v as x insert into O;")
    o = App(src)
    g = hip_app(src)
    rng = np.random.default_rng(4)
    n = 6000
    ts = np.arange(n, dtype=np.int64)
    v = rng.integers(0, 100000, n).astype(np.int32)
    w = np.where(rng.random(n) < 0.002, 7, 1).astype(np.int32)
    vals = np.stack([v.astype(np.int64), w.astype(np.int64)], 1)
    for lo, hi in ((0, 2500), (2500, n)):
        o.engine.send(0, ts[lo:hi], vals[lo:hi], None)
        g.engine.push_columns(0, ts[lo:hi], [v[lo:hi], w[lo:hi]])
        assert g.engine.take_matches(lambda q: 2) == o.engine.take_matches(lambda q: 2)
    assert g.engine.stats().live_partials > 1000


def test_gate_unordered_timestamps_full_form():
    src = gated_src("int", 7, n=12)
    o = App(src)
    g = hip_app(src, chunk_events=256)
    ts, v, w, u, vn = events("int", 12000, 17, unordered=True)
    cols, vals, nulls = cols_vals("int", v, w, u, vn)
    for lo, hi in ((0, 5000), (5000, 12000)):
        o.engine.send(0, ts[lo:hi], vals[lo:hi], nulls[lo:hi])
        g.engine.push_columns(0, ts[lo:hi], [c[lo:hi] for c in cols], [nulls[lo:hi, j] for j in range(3)])
        assert g.engine.take_matches(lambda q: 2) == o.engine.take_matches(lambda q: 2)


def test_gate_c2x_device_records_and_snapshot():
    """The C2x family (workloads.c2x_app) at 300 patterns: device-record pushes write the same
    records as normal-mode pushes (digest), and a snapshot restored into a fresh engine continues the
    stream exactly."""
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES
    from siddhi_amd.workloads import c2x_app, stock_events
    src = c2x_app(300)
    a = hip_app(src)
    b = hip_app(src, flags=SDH_FLAG_DEVICE_MATCHES)
    assert a.engine.stats().plan_queries[1] == 300
    lo = 0
    for n in (50000, 3, 70000):
        ts, sym, price, vol = stock_events(lo, n)
        lo += n
        cols = [sym, price.view(np.uint32), vol]
        a.engine.push_columns(0, ts, cols)
        b.engine.push_columns(0, ts, cols)
        da, db = a.engine.debug_digest(), b.engine.debug_digest()
        assert da == db and (n < 10 or da[0] > 10000)
        a.engine.poll()
    snap = a.engine.snapshot()
    c = hip_app(src)
    c.engine.restore(snap)
    ts, sym, price, vol = stock_events(lo, 40000)
    cols = [sym, price.view(np.uint32), vol]
    a.engine.push_columns(0, ts, cols)
    c.engine.push_columns(0, ts, cols)
    x, y = a.engine.poll(), c.engine.poll()
    assert len(x[0]) > 1000
    for p, q in zip(x, y):
        assert np.array_equal(p, q)
