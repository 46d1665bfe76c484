"""GPU parity of absent patterns (`not S[..] for T`) against the CPU oracle: the
reference's own absent-suite timelines (tests/golden/reference_absent_kat.json), seeded random
absent apps over timelines of events and idle time, batched pushes (timers firing between the events
of one push), absent states inside partitions (per-key clones swept over every event), pool /
timer-queue growth and snapshot/restore of pending timers.

The device runs each absent state's scheduler inside K_gen (kgen.h fire_timers): the timers due by
an event fire before it, sdh_engine_advance_time fires those due by a time with no event, and the
timer matches are ordered by (trigger event, timer time, query, fire order) in the match table."""
import pytest

from fuzz_apps import random_absent_app, random_timeline
from harness import App, OracleError
from test_absent_kat import FIXTURES, check_absent_rows, out_of_scope, run_absent_fixture

pytestmark = pytest.mark.gpu

SDH_FLAG_FORCE_GEN = 4
SDH_FLAG_PLAYBACK = 8
IN_SCOPE = [f for f in FIXTURES if not out_of_scope(f)]


def hip_factory(src, **kw):
    probe = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in probe.ir.streams]
    flags = kw.pop("flags", 0) | (SDH_FLAG_PLAYBACK if probe.playback else 0)

    def make(blob):
        from siddhi_amd.engine import HipEngine
        return HipEngine(blob, stream_types=types, flags=flags, **kw)
    return make


@pytest.mark.parametrize("fx", IN_SCOPE, ids=[f["id"] for f in IN_SCOPE])
def test_absent_kat_on_gpu(fx):
    o, _, _ = run_absent_fixture(fx)
    g, rows, checks = run_absent_fixture(fx, engine_factory=hip_factory(fx["app"]))
    assert g.matches == o.matches
    check_absent_rows(fx, rows, checks)


def _timeline(src, seed, factory=None, batch=False):
    app = App(src, factory)
    app.start(0)
    tl = random_timeline(seed)
    i = 0
    while i < len(tl):
        stream, row, t = tl[i]
        if stream == "advance":
            app.advance_time(t)
            i += 1
            continue
        j = i + 1
        while batch and j < len(tl) and tl[j][0] == stream and j - i < 25:
            j += 1
        app.send(stream, [r for _, r, _ in tl[i:j]], [x for _, _, x in tl[i:j]])
        i = j
    return app


@pytest.mark.parametrize("batch", [False, True], ids=["per_event", "batched"])
@pytest.mark.parametrize("seed", range(30))
def test_absent_fuzz_on_gpu(seed, batch):
    src = random_absent_app(seed, partition=seed % 3 == 0)  # partitions run as timer sweeps
    try:
        o = _timeline(src, seed)
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    g = _timeline(src, seed, hip_factory(src), batch)
    assert g.matches == o.matches


@pytest.mark.parametrize("seed", [0, 3, 15])
def test_absent_timer_queues_grow(seed):
    """Lists and scheduler queues that start at 2 entries overflow: the push is undone, the queues
    double with the lists (gen_remap_kernel rewrites each FIFO ring from its head) and the push
    re-runs."""
    src = random_absent_app(seed)
    o = _timeline(src, seed)
    g = _timeline(src, seed, hip_factory(src, gen_pool_states=2, gen_pool_nodes=4, gen_list_cap=2))
    assert g.engine.stats().pool_regrows > 0
    assert g.matches == o.matches


def test_absent_snapshot_restore_keeps_pending_timers():
    """A snapshot taken while timers are pending (and after the runtime started) restores into a
    fresh engine that fires them exactly as the original."""
    src = ("define stream S1 (symbol string, price float, volume int); "
           "define stream S2 (symbol string, price float, volume int); "
           "@info(name='q1') from every e1=S1[price > 20] -> not S2[price > e1.price] for 100 milliseconds "
           "select e1.symbol as s insert into O; "
           "@info(name='q2') from not S1[price > 50] for 70 milliseconds -> e2=S2[price > 10] "
           "select e2.symbol as s insert into O;")
    t0 = 1_000_000
    first = [("S1", ["A", 30.0, 1], t0 + 10), ("S1", ["B", 25.0, 1], t0 + 40), ("S2", ["C", 35.0, 1], t0 + 60)]
    second = [("S2", ["D", 15.0, 1], t0 + 150), ("S1", ["E", 60.0, 1], t0 + 160)]
    o = App(src)
    a = App(src, hip_factory(src))
    for x in (o, a):
        x.start(t0)
        for s, r, t in first:
            x.send(s, [r], [t])
    a.engine.poll()
    snap = a.engine.snapshot()
    b = App(src, hip_factory(src))
    b.engine.restore(snap)
    o.matches.clear()
    for x in (o, b):
        for s, r, t in second:
            x.send(s, [r], [t])
        x.advance_time(t0 + 400)
    assert b.matches == o.matches and len(o.matches) >= 2


@pytest.mark.parametrize("seed", [0, 3, 6, 9, 12])
def test_absent_partition_indexed_sweep(seed):
    """Partitioned absent states over many keys and long ordered pushes take the indexed timer sweep
    (nfa_gen.hip: each key's clone walks its own routed events; a timer fires at the first batch event
    whose time reaches it, by binary search of the batch's time prefix max). Against the oracle, and
    equal to the whole-batch sweep (SDH_NO_TIMER_INDEX) push for push."""
    import numpy as np
    from fuzz_apps import random_events
    src = random_absent_app(seed, partition=True)
    rng = np.random.default_rng(seed)
    ev = [("A" if rng.random() < 0.9 else "B", row, t) for _, row, t in random_events(seed, n=3000, keys=60)]
    apps = [App(src), App(src, hip_factory(src)), App(src, hip_factory(src, debug={"SDH_NO_TIMER_INDEX": 1}))]
    try:
        for a in apps:
            a.start(0)
        i = 0
        while i < len(ev):
            j = i + 1
            while j < len(ev) and ev[j][0] == ev[i][0] and j - i < 500:
                j += 1
            rows, ts = [r for _, r, _ in ev[i:j]], [t for _, _, t in ev[i:j]]
            for a in apps:
                a.send(ev[i][0], rows, ts)
            i = j
        for a in apps:
            a.advance_time(ev[-1][2] + 50)
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    o, g, w = apps
    assert g.matches == w.matches
    assert g.matches == o.matches and len(o.matches) > 0
