"""GPU parity of K_part (nfa_part.hip): partitioned `every e1 -> e2 and|or e3` and
`every e1 -> e2<min:max> -> e3` patterns on compact partial tables, against the oracle -- random
thresholds, `within` windows, count bounds and e3 filters over e1 / e2[0] / e2[last], null
attributes, out-of-order timestamps, batched pushes, forced table growth (exact re-runs), snapshot /
restore, and the C3 family against K_gen."""
import numpy as np
import pytest

from harness import App

pytestmark = pytest.mark.gpu

SDH_FLAG_FORCE_GEN = 4
STREAM = "define stream S (k int, p float, v int, d double);"


def _hip_app(src, **kw):
    from siddhi_amd.engine import HipEngine
    app = App(src, engine_factory=lambda blob: None)
    app.engine = HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], **kw)
    return app


def _queries(seed, n=24):
    rng = np.random.default_rng(seed)
    qs = []
    for i in range(n):
        kind = i % 3
        t = int(rng.integers(10, 90))
        w = int(rng.choice([-1, 5, 20, 60]))
        within = f" within {w} milliseconds" if w > 0 else ""
        if kind == 0:
            lo = int(rng.integers(1, 4))
            hi = lo + int(rng.integers(0, 4))
            f3 = rng.choice(["p > e2[last].p", "p < e2[0].p", "v > e1.v", "p > e1.p and v < e2[last].v",
                             "d > e2[last].d", "e2[last].p > e1.p"])
            body = (f"every e1=S[p > {t}] -> e2=S[v > {int(rng.integers(0, 600))}] <{lo}:{hi}> -> e3=S[{f3}]{within} "
                    f"select e1.p as a, e2[0].v as b, e3.p as c")
        else:
            op = "and" if kind == 1 else "or"
            f2 = rng.choice([f"v > {int(rng.integers(0, 1000))}", f"d < {int(rng.integers(0, 100))}.5",
                             "v > 500 and not (d > 30.0)", f"p > {t} or v < 10"])
            f3 = rng.choice([f"p < {t}", f"v > {int(rng.integers(0, 1000))}", "d > 50.0"])
            body = f"every e1=S[p > {t}] -> e2=S[{f2}] {op} e3=S[{f3}]{within} select e1.p as a"
        qs.append(f"@info(name='q{i}') from {body} insert into O;")
    return f"{STREAM} partition with (k of S) begin {' '.join(qs)} end;"


def _events(seed, n, keys, nulls=True, unordered=False):
    rng = np.random.default_rng(seed + 1000)
    ts = np.cumsum(rng.integers(0, 4, n)).astype(np.int64)
    if unordered:
        ts = ts + rng.integers(-8, 9, n)
    k = rng.integers(0, keys, n).astype(np.int32)
    p = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    v = rng.integers(0, 1000, n).astype(np.int32)
    d = rng.integers(0, 10000, n) / 100.0
    nl = np.zeros((n, 4), np.uint8)
    if nulls:
        nl[:, 1] = rng.random(n) < 0.03
        nl[:, 3] = rng.random(n) < 0.03
    vals = np.stack([k.astype(np.int64), p.view(np.uint32).astype(np.int64), v.astype(np.int64),
                     d.view(np.int64)], 1)
    return ts, vals, nl


def _run_pair(src, ts, vals, nl, batch, **kw):
    o = App(src)
    g = _hip_app(src, **kw)
    items = 0
    for lo in range(0, len(ts), batch):
        sl = slice(lo, lo + batch)
        o.engine.send(0, ts[sl], vals[sl], nl[sl])
        g.engine.send(0, ts[sl], vals[sl], nl[sl])
        nq = lambda q: len(o.ir.queries[q].states)  # noqa: E731
        om, gm = o.engine.take_matches(nq), g.engine.take_matches(nq)
        assert gm == om, f"batch at {lo}: {len(gm)} vs {len(om)} matches"
        items = max(items, g.engine.stats().last_part_items)
    return o, g, items


@pytest.mark.parametrize("seed", range(8))
def test_kpart_random_apps(seed):
    src = _queries(seed)
    ts, vals, nl = _events(seed, 6000, keys=3 + seed % 5, unordered=seed % 4 == 3)
    _, g, items = _run_pair(src, ts, vals, nl, batch=[1, 7, 500, 6000][seed % 4])
    assert items > 0  # K_part ran
    assert g.engine.stats().matches > 100


@pytest.mark.parametrize("cap", [1, 2])
def test_kpart_table_growth_reruns_exactly(cap, monkeypatch):
    """Tiny initial tables (SDH_KPART_CAP): every overflow is undone and re-run with twice the
    room, in normal and in device-matches mode."""
    monkeypatch.setenv("SIDDHI_HIP_DEBUG", f"SDH_KPART_CAP={cap}")
    src = _queries(77, n=12)
    ts, vals, nl = _events(77, 5000, keys=2)
    _run_pair(src, ts, vals, nl, batch=1000)


def test_kpart_snapshot_restore():
    src = _queries(5, n=18)
    ts, vals, nl = _events(5, 4000, keys=4)
    o = App(src)
    a = _hip_app(src)
    nq = lambda q: len(o.ir.queries[q].states)  # noqa: E731
    o.engine.send(0, ts[:2000], vals[:2000], nl[:2000])
    a.engine.send(0, ts[:2000], vals[:2000], nl[:2000])
    assert a.engine.take_matches(nq) == o.engine.take_matches(nq)
    snap = a.engine.snapshot()
    b = _hip_app(src)
    b.engine.restore(snap)
    o.engine.send(0, ts[2000:], vals[2000:], nl[2000:])
    b.engine.send(0, ts[2000:], vals[2000:], nl[2000:])
    om = o.engine.take_matches(nq)
    assert b.engine.take_matches(nq) == om and len(om) > 100


def test_c3_family_kpart_equals_kgen():
    """The C3 bench family (count <2:5> mid-chain, logical and, logical or; 1000 keys) on K_part
    equals the general interpreter, match for match in R18 order."""
    from siddhi_amd.workloads import c3_app, stock_events
    src = c3_app(96)
    a = _hip_app(src)
    b = _hip_app(src, flags=SDH_FLAG_FORCE_GEN, gen_pool_states=64, gen_pool_nodes=256, gen_list_cap=64)
    for lo in (0, 20000, 20001):
        n = 20000 if lo != 20000 else 1
        ts, sym, price, vol = stock_events(lo, n, 1000)
        cols = [sym, price.view(np.uint32), vol]
        a.engine.push_columns(0, ts, cols)
        b.engine.push_columns(0, ts, cols)
        assert a.engine.stats().last_part_items > 0 and b.engine.stats().last_part_items == 0
        x, y = a.engine.poll(), b.engine.poll()
        for u, v in zip(x, y):
            assert np.array_equal(u, v)
    assert a.engine.stats().matches > 10000


def test_reserve_keys_presizes_and_keeps_results():
    """sdh_engine_reserve_keys sizes the per-key state up front (no growth copy inside later pushes);
    the matches equal an engine that grows as keys appear, K_gen (FORCE_GEN) and K_part alike, and a
    reservation beyond gen_max_keys is refused."""
    from siddhi_amd.engine import EngineError
    src = _queries(31, n=15)
    ts, vals, nl = _events(31, 5000, keys=300)
    o = App(src)
    nq = lambda q: len(o.ir.queries[q].states)  # noqa: E731
    o.engine.send(0, ts, vals, nl)
    want = o.engine.take_matches(nq)
    assert len(want) > 100
    for flags in (0, SDH_FLAG_FORCE_GEN):
        g = _hip_app(src, flags=flags, gen_max_keys=512)
        g.engine.reserve_keys(300)
        g.engine.reserve_keys(100)  # (smaller: no-op)
        with pytest.raises(EngineError):
            g.engine.reserve_keys(513)
        for lo in range(0, len(ts), 250):
            sl = slice(lo, lo + 250)
            g.engine.send(0, ts[sl], vals[sl], nl[sl])
        assert g.engine.take_matches(nq) == want
