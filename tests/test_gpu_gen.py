"""GPU parity of K_gen (the general per-instance interpreter) and of the plan selection as a whole,
against the CPU oracle: every in-scope reference KAT, seeded random apps (count, logical, sequences,
partitions, arithmetic, nulls), batched pushes through the device partition routing."""
import numpy as np
import pytest

from fuzz_apps import random_app, random_events, random_seq_app
from harness import App, OracleError
from siddhi_amd.ql import SiddhiAppCreationException, SiddhiParserException
from test_oracle_reference_kat import KAT, OUT_OF_SCOPE, check_rows, run_fixture

pytestmark = pytest.mark.gpu

SDH_FLAG_FORCE_GEN = 4
FIXTURES = [f for f in KAT["fixtures"] if f["id"] not in OUT_OF_SCOPE]


def hip_factory(**kw):
    def make(blob):
        from siddhi_amd.engine import HipEngine
        return HipEngine(blob, **kw)
    return make


def hip_app(src, **kw):
    app = App(src, engine_factory=lambda blob: None)
    from siddhi_amd.engine import HipEngine
    app.engine = HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], **kw)
    return app


def _types_factory(flags):
    def make_app(fx):
        a = App(fx["app"], engine_factory=lambda blob: None)
        from siddhi_amd.engine import HipEngine
        return HipEngine(a.blob, stream_types=[s.attr_types for s in a.ir.streams], flags=flags)
    return make_app


@pytest.mark.parametrize("flags", [0, SDH_FLAG_FORCE_GEN], ids=["planned", "force_gen"])
@pytest.mark.parametrize("fx", FIXTURES, ids=[f["id"] for f in FIXTURES])
def test_reference_kat_on_gpu(fx, flags):
    try:
        o, _ = run_fixture(fx)
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    probe = App(fx["app"], engine_factory=lambda blob: None)
    types = [s.attr_types for s in probe.ir.streams]
    g, grows = run_fixture(fx, engine_factory=hip_factory(stream_types=types, flags=flags))
    assert g.matches == o.matches
    check_rows(fx, grows)


def _fuzz(seed, flags, batch):
    src = random_app(seed, partition=seed % 3 == 0)
    try:
        o = App(src)
    except (SiddhiAppCreationException, SiddhiParserException):
        return None
    g = hip_app(src, flags=flags)
    ev = random_events(seed)
    by = {}
    try:
        if batch:
            # runs of same-stream events pushed as one batch (device routing + sort)
            i = 0
            while i < len(ev):
                j = i
                while j < len(ev) and ev[j][0] == ev[i][0] and j - i < 40:
                    j += 1
                rows = [r for _, r, _ in ev[i:j]]
                ts = [t for _, _, t in ev[i:j]]
                o.send(ev[i][0], rows, ts)
                g.send(ev[i][0], rows, ts)
                i = j
        else:
            for stream, row, t in ev:
                o.send(stream, [row], [t])
                g.send(stream, [row], [t])
    except OracleError:
        return None
    except Exception as ex:  # loud capacity errors are allowed, wrong answers are not
        from siddhi_amd.engine import EngineError
        if isinstance(ex, EngineError) and ex.code == -4:
            return "capacity"
        raise
    return o, g


@pytest.mark.parametrize("batch", [False, True], ids=["per_event", "batched"])
@pytest.mark.parametrize("seed", range(40))
def test_fuzz_apps_on_gpu(seed, batch):
    r = _fuzz(seed, 0, batch)
    if r is None:
        pytest.skip("app rejected by the planner or the reference would throw")
    assert r != "capacity", "K_gen pools grow on overflow: no capacity error is expected"
    o, g = r
    assert g.matches == o.matches


GROWTH_SEEDS = [7, 11, 12, 14, 30]  # streams that overflow the default pools (round-1 skips)


@pytest.mark.parametrize("batch", [False, True], ids=["per_event", "batched"])
@pytest.mark.parametrize("seed", GROWTH_SEEDS)
def test_pool_growth_reruns_exactly(seed, batch):
    """Pools that start tiny (2 StateEvents, 4 nodes, lists of 2) overflow on almost every push:
    each overflow undoes the push, doubles the limit that was hit, re-lays every arena on the device
    (gen_remap_kernel) and re-runs the push. The matches stay the oracle's."""
    src = random_app(seed, partition=seed % 3 == 0)
    o = App(src)
    g = hip_app(src, flags=SDH_FLAG_FORCE_GEN, gen_pool_states=2, gen_pool_nodes=4, gen_list_cap=2)
    ev = random_events(seed)
    step = 40 if batch else 1
    i = 0
    while i < len(ev):
        j = i + 1
        while batch and j < len(ev) and ev[j][0] == ev[i][0] and j - i < step:
            j += 1
        rows = [r for _, r, _ in ev[i:j]]
        ts = [t for _, _, t in ev[i:j]]
        o.send(ev[i][0], rows, ts)
        g.send(ev[i][0], rows, ts)
        i = j
    assert g.engine.stats().pool_regrows > 0
    assert g.matches == o.matches


def test_pool_growth_snapshot_restores_into_default_engine():
    """A snapshot taken after the pools grew carries their sizing: a fresh engine with the default
    pools restores it (re-laying its arenas to the snapshot's sizing) and continues exactly."""
    seed = 11
    src = random_app(seed, partition=seed % 3 == 0)
    ev = random_events(seed)
    half = len(ev) // 2
    o = App(src)
    a = hip_app(src, flags=SDH_FLAG_FORCE_GEN, gen_pool_states=2, gen_pool_nodes=4, gen_list_cap=2)
    for stream, row, t in ev[:half]:
        o.send(stream, [row], [t])
        a.send(stream, [row], [t])
    assert a.engine.stats().pool_regrows > 0
    a.engine.poll()
    snap = a.engine.snapshot()
    b = hip_app(src, flags=SDH_FLAG_FORCE_GEN)
    b.engine.restore(snap)
    o.matches.clear()
    for stream, row, t in ev[half:]:
        o.send(stream, [row], [t])
        b.send(stream, [row], [t])
    assert b.matches == o.matches


def test_partitioned_many_keys_batched():
    """count <2:4> and logical and/or over 700 partition keys, batches of 2000 events."""
    src = ("define stream S (sym int, price float, vol int); "
           "partition with (sym of S) begin "
           "@info(name='c') from every e1=S[price > 60] <2:4> -> e2=S[price > e1[last].price] within 40 "
           "milliseconds select e1[0].price as a, e2.price as b insert into O; "
           "@info(name='a') from every e1=S[price > 50] -> e2=S[vol > 500] and e3=S[price < 20] within 60 "
           "milliseconds select e1.price as a insert into O; "
           "@info(name='o') from every e1=S[vol < 100] -> e2=S[price > 90] or e3=S[vol > 990] within 30 "
           "milliseconds select e1.vol as a insert into O; "
           "@info(name='s') from every e1=S[price > 80], e2=S[price > e1.price] select e1.price as a insert into O; "
           "end;")
    o = App(src)
    g = hip_app(src, gen_pool_states=32, gen_pool_nodes=64, gen_list_cap=32)
    rng = np.random.default_rng(4)
    n = 20000
    ts = np.arange(n, dtype=np.int64) // 4
    sym = rng.integers(0, 700, n).astype(np.int32)
    price = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    vol = rng.integers(0, 1000, n).astype(np.int32)
    vals = np.stack([sym.astype(np.int64), price.view(np.uint32).astype(np.int64), vol.astype(np.int64)], 1)
    for lo in range(0, n, 2000):
        o.engine.send(0, ts[lo:lo + 2000], vals[lo:lo + 2000], None)
        g.engine.push_columns(0, ts[lo:lo + 2000], [sym[lo:lo + 2000], price[lo:lo + 2000].view(np.uint32),
                                                    vol[lo:lo + 2000]])
        om = o.engine.take_matches(lambda q: len(o.ir.queries[q].states))
        gm = g.engine.take_matches(lambda q: len(o.ir.queries[q].states))
        assert gm == om
    assert g.engine.stats().matches > 500


def test_force_gen_matches_chain_plans_on_c2():
    from siddhi_amd.workloads import c2_app, stock_events
    src = c2_app(40)
    r = hip_app(src)
    k = hip_app(src, flags=SDH_FLAG_FORCE_GEN)
    ts, sym, price, vol = stock_events(0, 6000)
    cols = [sym, price.view(np.uint32), vol]
    r.engine.push_columns(0, ts, cols)
    k.engine.push_columns(0, ts, cols)
    a, b = r.engine.poll(), k.engine.poll()
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert len(a[0]) > 10000


@pytest.mark.parametrize("world,absent", [(2, False), (3, False), (2, True), (3, True)])
def test_engine_shards_merge_to_single_engine(world, absent):
    """sdh_config.shard_rank/shard_world on the device: pattern-set sharding of the unpartitioned
    queries and key sharding of the partition (foreign keys dropped at routing); the union of the
    shards, merged by siddhi_amd.dist.merge_columns, equals one engine running every query (and the
    oracle). With absent states in the partition, timer matches of several ranks precede one event:
    the merge orders them by the exported tiebreak (sdh_matches.tb)."""
    from siddhi_amd import dist as sdist
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.ir import T_INT
    from test_dist import events, full_src
    o = App(full_src(absent))
    types = [s.attr_types for s in o.ir.streams]
    shards = [HipEngine(o.blob, stream_types=types, shard_rank=r, shard_world=world) for r in range(world)]
    log = sdist.StreamLog()
    from siddhi_amd.events import encode_rows
    evs = events()
    for stream, row, t in evs:
        o.send(stream, [row], [t])
        si = o.ir.stream_index(stream)
        log.push(si, 1)
        vals, nulls = encode_rows([row], o.ir.streams[si].attr_types, o.dictionary)
        for sh in shards:  # every rank sees the whole stream
            sh.send(si, [t], vals, nulls)
    o.advance_time(evs[-1][2] + 100)
    for sh in shards:
        sh.advance_time(evs[-1][2] + 100)
    per_rank = []
    for r, sh in enumerate(shards):
        q, k, ts, off, words, seq, tb = sh.poll(with_seq=True)
        cols = sdist.columns_from_arrays(q, k, ts, off, words, seq, tb)
        for qi, key in zip(q.tolist(), k.tolist()):
            if o.ir.queries[qi].partition_idx >= 0:
                assert sdist.key_shard(key, T_INT, world) == r
            else:
                assert qi % world == r
        per_rank.append(cols)
    merged = sdist.columns_to_tuples(sdist.merge_columns(o.ir, per_rank, log))
    assert merged == o.matches and len(merged) > 50


def test_gen_snapshot_restore_count_and_partition():
    """Snapshot/restore of K_gen arenas and the partition key table (the reference's persist() ->
    new runtime -> restoreLastRevision(), PersistenceTestCase.java:150-235): the restored engine
    continues exactly like the original."""
    src = ("define stream S (k int, v int, p float); "
           "@info(name='c') from every e1=S[v > 3] <2:4> -> e2=S[p > e1[last].p] select e1[0].v as a insert into O; "
           "partition with (k of S) begin "
           "@info(name='s') from every e1=S[v > 5], e2=S[v < e1.v]+ within 30 milliseconds select e1.v as a insert into O; "
           "@info(name='l') from every e1=S[p > 5] -> e2=S[v > 8] or e3=S[p < 1] select e1.v as a insert into O; "
           "end;")
    ev = random_events(17, n=600, keys=40)
    ev = [(s if s == "A" else "A", r[:3], t) for s, r, t in ev]
    a = hip_app(src.replace("S", "A"))
    o = App(src.replace("S", "A"))
    for stream, row, t in ev[:300]:
        a.send(stream, [row], [t])
        o.send(stream, [row], [t])
    a.engine.poll()
    snap = a.engine.snapshot()
    b = hip_app(src.replace("S", "A"))
    b.engine.restore(snap)
    o.matches.clear()
    a.matches.clear()
    for stream, row, t in ev[300:]:
        a.send(stream, [row], [t])
        b.send(stream, [row], [t])
        o.send(stream, [row], [t])
    assert a.matches == o.matches
    assert b.matches == o.matches and len(b.matches) > 20


# ---- event-chunked K_gen (kg::seq_lookback): every-start stream-state sequences ----

def _chunked_pair(src, chunk_len, monkeypatch):
    """Oracle + a K_gen-only engine (SDH_FLAG_FORCE_GEN keeps windowed sequences off K_seq)."""
    monkeypatch.setenv("SIDDHI_HIP_DEBUG", f"SDH_GEN_CHUNK_LEN={chunk_len}")
    return App(src), hip_app(src, flags=SDH_FLAG_FORCE_GEN)


@pytest.mark.parametrize("chunk_len", [1, 2, 3, 7])
@pytest.mark.parametrize("seed", range(8))
def test_chunked_random_sequences(seed, chunk_len, monkeypatch):
    src = random_seq_app(seed)
    o, g = _chunked_pair(src, chunk_len, monkeypatch)
    # runs of up to 60 same-stream events (one push each): chunks inside, state across pushes
    ev = [("AB"[(i // 60) % 2 if seed % 2 else 0], r, t) for i, (_, r, t) in enumerate(random_events(100 + seed, n=400))]
    i, items = 0, 0
    while i < len(ev):  # same-stream runs as one push: chunks inside, persisted state across pushes
        j = i
        while j < len(ev) and ev[j][0] == ev[i][0] and j - i < 90:
            j += 1
        rows = [r for _, r, _ in ev[i:j]]
        ts = [t for _, _, t in ev[i:j]]
        o.send(ev[i][0], rows, ts)
        g.send(ev[i][0], rows, ts)
        items = max(items, g.engine.stats().last_gen_items)
        i = j
    assert g.matches == o.matches
    assert items > 6  # event chunks engaged (6 queries = at most 6 groups unchunked)


@pytest.mark.parametrize("chunk_len", [2, 5, 256])
def test_chunked_c4_family(chunk_len, monkeypatch):
    """C4 fraud-rule sequences (float x double arithmetic compares) over 3 pushes of the Txn stream."""
    from siddhi_amd.workloads import c4_app, txn_events
    src = c4_app(96)
    o, g = _chunked_pair(src, chunk_len, monkeypatch)
    nq = len(o.ir.queries)
    n = 0
    for lo, hi in ((0, 3000), (3000, 3001), (3001, 9000)):
        ts, acc, amt, risk = txn_events(lo, hi - lo, n_accounts=500)
        vals = np.stack([acc.astype(np.int64), amt.view(np.uint32).astype(np.int64), risk.astype(np.int64)], 1)
        o.engine.send(0, ts, vals, None)
        g.engine.push_columns(0, ts, [acc, amt.view(np.uint32), risk])
        if hi - lo > 2 * chunk_len:
            assert g.engine.stats().last_gen_items > 2  # 96 same-shape queries = 2 groups, chunked
        om = o.engine.take_matches(lambda q: 3)
        gm = g.engine.take_matches(lambda q: 3)
        assert gm == om
        n += len(om)
    assert nq == 96 and n > 5000


# ---- K_seq (kg::seq_window): single-stream every-start sequences as windows of S events ----

def _push_runs(o, g, ev, max_run):
    i, items = 0, 0
    while i < len(ev):
        j = i
        while j < len(ev) and ev[j][0] == ev[i][0] and j - i < max_run(i):
            j += 1
        rows = [r for _, r, _ in ev[i:j]]
        ts = [t for _, _, t in ev[i:j]]
        o.send(ev[i][0], rows, ts)
        g.send(ev[i][0], rows, ts)
        items = max(items, g.engine.stats().last_seq_items)
        i = j
    return items


@pytest.mark.parametrize("seed", range(16))
def test_seq_windows_random(seed):
    """Planned path: even seeds are single-stream every-start sequences (K_seq); odd seeds read
    two streams and stay on K_gen. Pushes of 1-7 events exercise the carried tail."""
    src = random_seq_app(seed)
    o, g = App(src), hip_app(src)
    ev = [("AB"[(i // 60) % 2 if seed % 2 else 0], r, t) for i, (_, r, t) in
          enumerate(random_events(200 + seed, n=500))]
    items = _push_runs(o, g, ev, lambda i: 1 + (i % 7) if i < 250 else 200)
    assert g.matches == o.matches
    if seed % 2 == 0:
        assert items > 0


def test_seq_windows_c4_family():
    from siddhi_amd.workloads import c4_app, txn_events
    src = c4_app(200)
    o, g = App(src), hip_app(src)
    n = 0
    for lo, hi in ((0, 3000), (3000, 3001), (3001, 3003), (3003, 20000)):
        ts, acc, amt, risk = txn_events(lo, hi - lo, n_accounts=500)
        vals = np.stack([acc.astype(np.int64), amt.view(np.uint32).astype(np.int64), risk.astype(np.int64)], 1)
        o.engine.send(0, ts, vals, None)
        g.engine.push_columns(0, ts, [acc, amt.view(np.uint32), risk])
        assert g.engine.stats().last_seq_items > 0 and g.engine.stats().last_gen_items == 0
        om = o.engine.take_matches(lambda q: 3)
        assert g.engine.take_matches(lambda q: 3) == om
        n += len(om)
    assert n > 50000


def test_seq_windows_snapshot_restore():
    from siddhi_amd.workloads import c4_app, txn_events
    src = c4_app(64)
    o, a = App(src), hip_app(src)

    def batch(lo, hi):
        ts, acc, amt, risk = txn_events(lo, hi - lo, n_accounts=50)
        vals = np.stack([acc.astype(np.int64), amt.view(np.uint32).astype(np.int64), risk.astype(np.int64)], 1)
        return ts, vals, [acc, amt.view(np.uint32), risk]
    ts, vals, cols = batch(0, 1001)
    o.engine.send(0, ts, vals, None)
    a.engine.push_columns(0, ts, cols)
    o.engine.take_matches(lambda q: 3)
    a.engine.poll()
    snap = a.engine.snapshot()
    b = hip_app(src)
    b.engine.restore(snap)
    ts, vals, cols = batch(1001, 3000)
    o.engine.send(0, ts, vals, None)
    b.engine.push_columns(0, ts, cols)
    om = o.engine.take_matches(lambda q: 3)
    assert b.engine.take_matches(lambda q: 3) == om and len(om) > 100


@pytest.mark.gpu
def test_device_matches_ring_counts_every_record():
    """SDH_FLAG_DEVICE_MATCHES writes every K_gen record into the flat device-record buffer, which grows
    and re-runs the push when its records exceed it (no wrap); the records handed out
    (sdh_engine_poll_records) number the normal mode's matches over the same stream (pushed in
    batches small enough for the normal output buffer)."""
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES, HipEngine
    from siddhi_amd.workloads import c2_app, stock_events

    app = App(c2_app(64), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    ts, sym, price, vol = stock_events(0, 40_000)
    vals = np.stack([sym.astype(np.int64), price.view(np.uint32).astype(np.int64), vol.astype(np.int64)], 1)
    ring = HipEngine(app.blob, stream_types=types, flags=SDH_FLAG_FORCE_GEN | SDH_FLAG_DEVICE_MATCHES)
    ring.send(0, ts, vals, None)  # ~1.2M records x 11 words: past the initial 4M-word buffer
    rec = ring.poll_records()
    normal = HipEngine(app.blob, stream_types=types, flags=SDH_FLAG_FORCE_GEN)
    for b in range(0, len(ts), 10000):
        normal.send(0, ts[b:b + 10000], vals[b:b + 10000], None)
        normal.poll()
    n = ring.stats().matches
    assert n > 500_000
    assert n == normal.stats().matches == rec.f_n


def test_gen_output_overflow_reruns_exactly():
    """A push whose K_gen match records overflow the output buffer is undone (arena backup) and re-run
    with room for every record: no match is lost and later pushes continue exactly."""
    from siddhi_amd.workloads import c2_app, stock_events
    src = c2_app(64)
    o = App(src)
    g = hip_app(src, flags=SDH_FLAG_FORCE_GEN)
    for lo, hi in ((0, 12000), (12000, 16000)):  # the first push needs ~6M record words (4M buffer)
        ts, sym, price, vol = stock_events(lo, hi - lo)
        vals = np.stack([sym.astype(np.int64), price.view(np.uint32).astype(np.int64), vol.astype(np.int64)], 1)
        o.engine.send(0, ts, vals, None)
        g.engine.push_columns(0, ts, [sym, price.view(np.uint32), vol])
        om = o.engine.take_matches(lambda q: 2)
        gm = g.engine.take_matches(lambda q: 2)
        assert gm == om and len(om) > 50000


def test_journal_budget_splits_the_push_exactly():
    """The K_gen journal (the blocks a pass modifies, saved so that an overflow re-runs exactly) must
    fit a third of free HBM; a push whose bound does not is split into halves. With the budget forced
    to nothing (SDH_JOURNAL_BUDGET) every push of a partitioned K_gen app splits down to single
    events, and with tiny pools every one of those re-runs from the journal: the matches equal the
    oracle's."""
    from siddhi_amd.workloads import c3_app, stock_events
    src = c3_app(12)
    o = App(src)
    g = hip_app(src, flags=SDH_FLAG_FORCE_GEN, gen_pool_states=2, gen_pool_nodes=4, gen_list_cap=2,
                gen_max_keys=1024, debug={"SDH_JOURNAL_BUDGET": 1})
    if True:
        for lo, n in ((0, 700), (700, 1300)):
            ts, sym, price, vol = stock_events(lo, n, 40)
            vals = np.stack([sym.astype(np.int64), price.view(np.uint32).astype(np.int64), vol.astype(np.int64)], 1)
            o.engine.send(0, ts, vals, None)
            g.engine.push_columns(0, ts, [sym, price.view(np.uint32), vol])
            om = o.engine.take_matches(lambda q: 3)
            gm = g.engine.take_matches(lambda q: 3)
            assert gm == om and len(om) > 50
    assert g.engine.stats().pool_regrows > 0


def test_seq_windows_compiled_unclean_tiles():
    """The shape-compiled K_seq kernel (>= 2 waves of one shape) on tiles that are not clean
    (seq_body.h LdsWinT: a clean tile has no null, ordered timestamps and a span within every lane's
    `within`, and skips those tests): null amounts, windows of a few ms shorter than a tile's span,
    out-of-order timestamps, and clean tiles between them (the first wave's lanes wait an hour),
    against the oracle push by push."""
    from siddhi_amd.workloads import TXN_STREAM, txn_events
    qs = [TXN_STREAM]
    for p in range(130):
        w = "1 hour" if p < 64 else f"{(2, 3, 5)[p % 3]} milliseconds"
        qs.append(f"@info(name='s{p}') from every e1=Txn[amount > {100 + p % 700}], e2=Txn[amount > e1.amount * 1.05], "
                  f"e3=Txn[amount > e2.amount and risk > {p % 50}] within {w} select e1.amount as a1 insert into Alerts;")
    src = " ".join(qs)
    o, g = App(src), hip_app(src)
    st = g.engine.stats()
    assert st.spec_kernels > 0 and st.plan_queries[5] == 130  # (every query on K_seq, compiled)
    rng = np.random.default_rng(5)
    lo, t, total = 0, 1_000_000, 0
    for n, nullp, unord in ((4000, 0.0, False), (3000, 0.02, False), (5000, 0.0, True), (3000, 0.0, False)):
        _, acc, amt, risk = txn_events(lo, n, n_accounts=500)
        lo += n
        ts = t + np.cumsum(rng.integers(0, 3, n)).astype(np.int64)
        if unord:
            ts[1000:1010] -= 7
        t = int(ts.max())
        an = (rng.random(n) < nullp).astype(np.uint8)
        vals = np.stack([acc.astype(np.int64), amt.view(np.uint32).astype(np.int64), risk.astype(np.int64)], 1)
        nulls = np.zeros((n, 3), np.uint8)
        nulls[:, 1] = an
        o.engine.send(0, ts, vals, nulls)
        g.engine.push_columns(0, ts, [acc, amt.view(np.uint32), risk], [None, an, None])
        om = o.engine.take_matches(lambda q: 3)
        assert g.engine.take_matches(lambda q: 3) == om
        total += len(om)
    assert total > 5000
