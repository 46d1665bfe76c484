"""GPU parity of the chain NFA kernel against the CPU oracle (bit-exact match tuples)."""
import json
import os

import numpy as np
import pytest

from harness import App, OracleEngine, parse_literal
from siddhi_amd.ql import SiddhiAppCreationException
from siddhi_amd.workloads import c2_app, stock_events

pytestmark = pytest.mark.gpu

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))


def hip_app(src, **kw):
    app = App(src, engine_factory=lambda blob: None)
    from siddhi_amd.engine import HipEngine
    app.engine = HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], **kw)
    return app


def c2_columns(start, n):
    ts, sym, price, vol = stock_events(start, n)
    return ts, [sym, price.view(np.uint32), vol]


@pytest.mark.parametrize("chunk", [0, 1024])
def test_c2_synthetic_parity(chunk):
    src = c2_app(24)
    o = App(src)
    g = hip_app(src, chunk_events=chunk, partials=256)
    for start, n in ((0, 7000), (7000, 14000)):
        ts, cols = c2_columns(start, n)
        vals = np.stack([c.astype(np.int64) if c.dtype != np.uint32 else c.astype(np.int64) for c in cols], 1)
        o.engine.send(0, ts, vals, None)
        om = o.engine.take_matches(lambda q: 2)
        g.engine.push_columns(0, ts, cols)
        gm = g.engine.take_matches(lambda q: 2)
        assert len(om) > 1000
        assert gm == om


def test_lane_capacity_overflow_is_loud():
    from siddhi_amd.engine import EngineError
    src = ("define stream S (v int); @info(name='q') from every e1=S[v > 0] -> e2=S[v < 0] "
           "select e1.v as a insert into O;")
    g = hip_app(src, partials=64)
    ts = np.arange(200, dtype=np.int64)
    with pytest.raises(EngineError) as ei:
        g.engine.push_columns(0, ts, [np.ones(200, np.int32)])
    assert ei.value.code == -4


def test_snapshot_restore_roundtrip():
    src = c2_app(4)
    a = hip_app(src)
    ts, cols = c2_columns(0, 5000)
    a.engine.push_columns(0, ts, cols)
    a.engine.poll()
    snap = a.engine.snapshot()
    ts2, cols2 = c2_columns(5000, 5000)
    a.engine.push_columns(0, ts2, cols2)
    ref = a.engine.take_matches(lambda q: 2)
    b = hip_app(src)
    b.engine.restore(snap)
    b.engine.push_columns(0, ts2, cols2)
    assert b.engine.take_matches(lambda q: 2) == ref


TYPED_STREAM = "define stream T (i int, l long, f float, d double, b bool, s string);"
NUMERIC = ["i", "l", "f", "d"]
OPS = ["==", "!=", ">", ">=", "<", "<="]


def typed_events(n=400, seed=3):
    """Adversarial values for Java's typed compares: int->float and long->float/double rounding
    boundaries, signed zeros, NaN, infinities, extremes; some nulls."""
    rng = np.random.default_rng(seed)
    ints = [0, 1, -1, 16777216, 16777217, -16777217, 2**31 - 1, -2**31, 123456789, 7]
    longs = [0, 1, -1, 16777217, 2**53, 2**53 + 1, 2**62 + 1, -2**63, 2**63 - 1, 9007199254740993, 7]
    floats = [0.0, -0.0, 1.0, 16777216.0, 16777218.0, float("nan"), float("inf"), -float("inf"),
              3.4028235e38, 1e-45, 7.0, 0.1]
    doubles = [0.0, -0.0, 1.0, 16777217.0, 9007199254740992.0, 9007199254740994.0, float("nan"),
               float("inf"), 0.1, 7.0, 1e300]
    rows = []
    for k in range(n):
        row = [int(rng.choice(ints)), int(rng.choice(longs)), float(np.float32(rng.choice(floats))),
               float(rng.choice(doubles)), bool(rng.integers(2)), str(rng.choice(["a", "b", "c"]))]
        if rng.random() < 0.05:
            row[int(rng.integers(6))] = None
        rows.append(row)
    return rows


def test_typed_compare_semantics():
    qs = [TYPED_STREAM]
    n = 0
    for a in NUMERIC:
        for b in NUMERIC:
            for op in OPS:
                qs.append(f"@info(name='u{n}') from every e1=T[{a} {op} {b}] select e1.i as x insert into O;")
                qs.append(f"@info(name='x{n}') from every e1=T -> e2=T[{a} {op} e1.{b}] "
                          f"select e1.i as x insert into O;")
                n += 1
    for op in ("==", "!="):
        qs.append(f"@info(name='bb{op}') from every e1=T -> e2=T[b {op} e1.b] select e1.i as x insert into O;")
        qs.append(f"@info(name='ss{op}') from every e1=T -> e2=T[s {op} e1.s and s {op} 'b'] "
                  f"select e1.i as x insert into O;")
    qs.append("@info(name='flag') from every e1=T[b] select e1.i as x insert into O;")
    qs.append("@info(name='consts') from every e1=T[f > 16777216 and l < 3.0f and d >= 7L] "
              "select e1.i as x insert into O;")
    src = " ".join(qs)
    o = App(src)
    g = hip_app(src, partials=512)
    rows = typed_events()
    for k, row in enumerate(rows):
        o.send("T", [row], [1000 + k])
        g.send("T", [row], [1000 + k])
    assert len(o.matches) > 1000
    assert g.matches == o.matches


def test_multi_stream_chain_and_within():
    src = ("define stream A (v int, p float); define stream B (v int, p float); "
           "@info(name='q1') from every e1=A[p > 10] -> e2=B[p > e1.p] -> e3=A[v == e1.v] within 50 "
           "milliseconds select e1.v as a insert into O; "
           "@info(name='q2') from e1=A[p > 50] -> e2=B[p < e1.p] select e1.v as a insert into O;")
    o = App(src)
    g = hip_app(src)
    rng = np.random.default_rng(11)
    t = 0
    for k in range(600):
        t += int(rng.integers(0, 7))
        s = "A" if rng.random() < 0.5 else "B"
        row = [int(rng.integers(0, 5)), float(np.float32(rng.uniform(0, 100)))]
        o.send(s, [row], [t])
        g.send(s, [row], [t])
    assert len(o.matches) > 50
    assert g.matches == o.matches


def test_unordered_timestamps_fall_back_exactly():
    # out-of-order timestamps disable warm-up chunking; the result must still be exact
    src = c2_app(6)
    o = App(src)
    g = hip_app(src, chunk_events=512, partials=256)
    ts, cols = c2_columns(0, 20000)
    ts = ts.copy()
    ts[7000:7100] -= 5000
    vals = np.stack([c.astype(np.int64) for c in cols], 1)
    o.engine.send(0, ts, vals, None)
    g.engine.push_columns(0, ts, cols)
    assert g.engine.take_matches(lambda q: 2) == o.engine.take_matches(lambda q: 2)
