"""GPU parity of chunk delivery (sdh_batch.chunk: one InputHandler.send(Event[]) per push) against
the oracle's chunk mode: every in-scope reference KAT app and 40 seeded random apps (partitions
included) with each run of same-stream events sent as one chunk, absent timelines (time moves once
per chunk), fan-out partitions, the K_ratchet plan, device-resident chunks, a chunk split by the
journal budget, and a poll window mixing single-event and chunk pushes.

Chunk order is parity-unpinned against the reference's suites (none sends an Event[] into a pattern
query); test_chunk_oracle.py pins the oracle's restatement on hand-checked cases."""
import numpy as np
import pytest

from fuzz_apps import fanout_app, fanout_events, random_absent_app, random_app, random_events, random_timeline
from harness import App, OracleError, parse_literal
from siddhi_amd.ql import SiddhiAppCreationException, SiddhiParserException
from test_oracle_reference_kat import KAT, OUT_OF_SCOPE

pytestmark = pytest.mark.gpu

SDH_FLAG_FORCE_GEN = 4
SDH_FLAG_PLAYBACK = 8
FIXTURES = [f for f in KAT["fixtures"] if f["id"] not in OUT_OF_SCOPE]


def hip_app(src, **kw):
    app = App(src, engine_factory=lambda blob: None)
    from siddhi_amd.engine import HipEngine
    flags = kw.pop("flags", 0) | (SDH_FLAG_PLAYBACK if app.playback else 0)
    app.engine = HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], flags=flags, **kw)
    return app


def send_runs(apps, ev, limit, as_chunk=True):
    """each run of consecutive same-stream events (at most `limit`) as one push"""
    i = 0
    while i < len(ev):
        j = i + 1
        while j < len(ev) and ev[j][0] == ev[i][0] and j - i < limit:
            j += 1
        for a in apps:
            a.send(ev[i][0], [r for _, r, _ in ev[i:j]], [t for _, _, t in ev[i:j]], as_chunk=as_chunk)
        i = j


@pytest.mark.parametrize("flags", [0, SDH_FLAG_FORCE_GEN], ids=["planned", "force_gen"])
@pytest.mark.parametrize("fx", FIXTURES, ids=[f["id"] for f in FIXTURES])
def test_reference_kat_apps_as_chunks(fx, flags):
    ev = [(e["stream"], [parse_literal(t) for t in e["data"]], e["ts"]) for e in fx["events"]]
    o = App(fx["app"])
    try:
        send_runs([o], ev, 1 << 30)
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    g = hip_app(fx["app"], flags=flags)
    send_runs([g], ev, 1 << 30)
    assert g.matches == o.matches


def _apps(src, **kw):
    try:
        return App(src), hip_app(src, **kw)
    except (SiddhiAppCreationException, SiddhiParserException):
        pytest.skip("app rejected by the planner")


@pytest.mark.parametrize("limit", [7, 40])
@pytest.mark.parametrize("seed", range(40))
def test_fuzz_apps_as_chunks(seed, limit):
    o, g = _apps(random_app(seed, partition=seed % 3 == 0))
    ev = random_events(seed)
    try:
        send_runs([o], ev, limit)
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    send_runs([g], ev, limit)
    assert g.matches == o.matches


@pytest.mark.parametrize("seed", range(12))
def test_absent_timelines_as_chunks(seed):
    src = random_absent_app(seed, partition=seed % 3 == 0)
    o, g = _apps(src)
    tl = random_timeline(seed)
    try:
        for a in (o, g):
            a.start(0)
            i = 0
            while i < len(tl):
                if tl[i][0] == "advance":
                    a.advance_time(tl[i][2])
                    i += 1
                    continue
                j = i + 1
                while j < len(tl) and tl[j][0] == tl[i][0] and j - i < 25:
                    j += 1
                a.send(tl[i][0], [r for _, r, _ in tl[i:j]], [t for _, _, t in tl[i:j]], as_chunk=True)
                i = j
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    assert g.matches == o.matches


@pytest.mark.parametrize("key_type", ["int", "bool", "string"])
@pytest.mark.parametrize("seed", range(4))
def test_fanout_as_chunks(seed, key_type):
    src = fanout_app(seed, key_type)
    o, g = _apps(src)
    send_runs([o, g], fanout_events(seed, keys=20 + 8 * seed, key_type=key_type), 64)
    assert len(o.matches) > 20
    assert g.matches == o.matches


def test_ratchet_chunk_goes_through_the_table():
    """K_ratchet matches of a chunk push take the match table (no direct placement): subscriber-major
    over the 16 patterns, not event-major."""
    from siddhi_amd.workloads import c2_app, stock_events
    src = c2_app(16)
    o, g = _apps(src)
    ts, sym, price, vol = stock_events(3, 3000)
    rows = [[f"s{int(a)}", float(p), int(v)] for a, p, v in zip(sym, price, vol)]
    for lo in range(0, 3000, 1000):
        for a in (o, g):
            a.send("StockStream", rows[lo:lo + 1000], ts[lo:lo + 1000].tolist(), as_chunk=True)
    assert len(o.matches) > 100
    assert g.matches == o.matches
    assert g.engine.stats().placed_pushes == 0


def test_device_resident_chunk_and_mixed_window():
    """A device-resident chunk (the run starts come from the key column copied back) and a poll
    window holding a single-event push, a chunk push and another single-event push."""
    import torch
    src = random_app(6, partition=True)
    o, g = _apps(src)
    ev = [e for e in random_events(6, n=600) if e[0] == "A"]
    ir = o.ir
    si = ir.stream_index("A")
    types = ir.streams[si].attr_types
    from siddhi_amd.events import encode_rows
    from siddhi_amd.engine import columns_from_words
    parts = [ev[:100], ev[100:400], ev[400:]]
    for k, part in enumerate(parts):
        rows, ts = [r for _, r, _ in part], [t for _, _, t in part]
        o.log.append(si, ts, *encode_rows(rows, types, o.dictionary))
        vals, nulls = encode_rows(rows, types, g.dictionary)
        o.engine.send(si, ts, *encode_rows(rows, types, o.dictionary), k == 1)
        if k == 1:
            if nulls is not None and nulls.any():
                pytest.skip("device pushes carry no null masks here")
            cols = columns_from_words(vals, types)
            dev = torch.device("cuda:0")
            t_ts = torch.tensor(ts, dtype=torch.int64, device=dev)
            t_cols = [torch.from_numpy(c.view(np.int32) if c.dtype == np.uint32 else c).to(dev) for c in cols]
            torch.cuda.synchronize()
            g.engine.push_device(si, len(ts), t_ts.data_ptr(), [c.data_ptr() for c in t_cols], chunk=True)
        else:
            g.engine.send(si, ts, vals, nulls)
    n_slots = lambda q: len(ir.queries[q].states)  # noqa: E731
    want = o.engine.take_matches(n_slots)
    got = g.engine.take_matches(n_slots)
    assert len(want) > 10
    assert got == want


def test_chunk_split_by_the_journal_budget(monkeypatch):
    """A chunk whose K_gen journal would pass SDH_JOURNAL_BUDGET is pushed as two halves that still
    act as one chunk (one time move, one run split, one subscriber order)."""
    monkeypatch.setenv("SIDDHI_HIP_DEBUG", "SDH_JOURNAL_BUDGET=1")
    src = random_absent_app(3, partition=True)
    o, g = _apps(src)
    ev = random_events(3, n=400)
    for a in (o, g):
        a.start(0)
    send_runs([o, g], ev, 200)
    assert g.matches == o.matches and len(o.matches) > 0
