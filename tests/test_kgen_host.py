"""The K_gen interpreter body (siddhi_amd/csrc/kgen.h), compiled for the host, against the CPU oracle
on every reference KAT stream (bit-exact match tuples, same delivery order) and on the KATs' expected
rows. This pins the device kernel's per-lane logic on machines without a GPU."""
import pytest

from harness import App, OracleError
from kgen_host import KGenHostEngine
from test_oracle_reference_kat import KAT, OUT_OF_SCOPE, check_rows, run_fixture

FIXTURES = [f for f in KAT["fixtures"] if f["id"] not in OUT_OF_SCOPE]


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["id"] for f in FIXTURES])
def test_kgen_host_matches_oracle(fx):
    try:
        o, orows = run_fixture(fx)
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    g, grows = run_fixture(fx, engine_factory=lambda blob: KGenHostEngine(blob))
    assert g.matches == o.matches
    check_rows(fx, grows)


def _fuzz_case(seed, partition, R=0, N=0):
    from fuzz_apps import random_app, random_events
    from siddhi_amd.ql import SiddhiAppCreationException, SiddhiParserException
    src = random_app(seed, partition=partition)
    try:
        o = App(src)
    except (SiddhiAppCreationException, SiddhiParserException):
        return None
    g = App(src, engine_factory=lambda blob: KGenHostEngine(blob, R=R, N=N))
    for stream, row, t in random_events(seed):
        try:
            o.send(stream, [row], [t])
        except OracleError:
            return None  # the reference would throw: out of the comparable domain
        try:
            g.send(stream, [row], [t])
        except RuntimeError as ex:
            if "capacity" in str(ex):
                return "capacity"
            raise
    return o, g


@pytest.mark.parametrize("seed", range(120))
def test_kgen_host_fuzz(seed):
    r = _fuzz_case(seed, partition=seed % 3 == 0)
    if r == "capacity":
        # the device engine grows its pools and re-runs the push; the host build runs the same
        # streams with big pools from the start (arena-resident bitmasks and GC marks, kgen.h)
        r = _fuzz_case(seed, partition=seed % 3 == 0, R=4096, N=4096)
    if r is None:
        pytest.skip("app rejected by the planner or the reference would throw")
    assert r != "capacity"
    o, g = r
    assert g.matches == o.matches


@pytest.mark.parametrize("seed", range(0, 120, 7))
def test_kgen_host_big_pools(seed):
    """Big-pool layouts (kgen.h: lay.big, bitmasks and GC marks in the arena) on streams the small
    pools also hold: the same matches as the oracle."""
    r = _fuzz_case(seed, partition=seed % 3 == 0, R=128, N=4096)
    if r is None:
        pytest.skip("app rejected by the planner or the reference would throw")
    o, g = r
    assert g.matches == o.matches


@pytest.mark.parametrize("chunk_len", [1, 2, 3, 7])
@pytest.mark.parametrize("seed", range(12))
def test_kgen_host_event_chunks(seed, chunk_len):
    """The look-back rule behind K_gen's event chunks (kg::seq_lookback): every-start stream-state
    sequences rebuilt from a fresh instance and S-1 replayed events give the oracle's matches."""
    from fuzz_apps import random_events, random_seq_app
    src = random_seq_app(seed)
    o = App(src)
    g = App(src, engine_factory=lambda blob: KGenHostEngine(blob, chunk_len=chunk_len))
    # runs of up to 60 same-stream events (one push each): chunks inside, state across pushes
    ev = [("AB"[(i // 60) % 2 if seed % 2 else 0], r, t) for i, (_, r, t) in enumerate(random_events(100 + seed, n=400))]
    i = 0
    while i < len(ev):
        j = i
        while j < len(ev) and ev[j][0] == ev[i][0] and j - i < 90:
            j += 1
        rows = [r for _, r, _ in ev[i:j]]
        ts = [t for _, _, t in ev[i:j]]
        o.send(ev[i][0], rows, ts)
        g.send(ev[i][0], rows, ts)
        i = j
    assert g.matches == o.matches


def test_kgen_host_event_chunks_c4():
    import numpy as np
    from siddhi_amd.workloads import c4_app, txn_events
    src = c4_app(40)
    o = App(src)
    g = App(src, engine_factory=lambda blob: KGenHostEngine(blob, R=8, N=32, LC=8, chunk_len=3))
    for lo, hi in ((0, 2000), (2000, 2001), (2001, 5000)):
        ts, acc, amt, risk = txn_events(lo, hi - lo, n_accounts=500)
        vals = np.stack([acc.astype(np.int64), amt.view(np.uint32).astype(np.int64), risk.astype(np.int64)], 1)
        o.engine.send(0, ts, vals, None)
        g.engine.send(0, ts, vals, None)
        assert g.engine.take_matches(lambda q: 3) == o.engine.take_matches(lambda q: 3)


@pytest.mark.parametrize("seed", range(16))
def test_kgen_host_seq_windows(seed):
    """The window rule behind K_seq (kg::seq_window / seq_match): a single-stream every-start
    stream-state sequence matches exactly the windows of S consecutive events whose states all
    pass in order, tails carried across pushes."""
    from fuzz_apps import random_events, random_seq_app
    src = random_seq_app(seed)
    o = App(src)
    g = App(src, engine_factory=lambda blob: KGenHostEngine(blob, window=True))
    ev = [("AB"[(i // 60) % 2 if seed % 2 else 0], r, t) for i, (_, r, t) in enumerate(random_events(200 + seed, n=400))]
    i = 0
    while i < len(ev):
        j = i
        while j < len(ev) and ev[j][0] == ev[i][0] and j - i < (1 + (i % 7)):
            j += 1
        rows = [r for _, r, _ in ev[i:j]]
        ts = [t for _, _, t in ev[i:j]]
        o.send(ev[i][0], rows, ts)
        g.send(ev[i][0], rows, ts)
        i = j
    assert g.matches == o.matches


def test_kgen_host_seq_windows_c4():
    import numpy as np
    from siddhi_amd.workloads import c4_app, txn_events
    src = c4_app(40)
    o = App(src)
    g = App(src, engine_factory=lambda blob: KGenHostEngine(blob, window=True))
    total = 0
    for lo, hi in ((0, 2000), (2000, 2001), (2001, 2003), (2003, 5000)):
        ts, acc, amt, risk = txn_events(lo, hi - lo, n_accounts=500)
        vals = np.stack([acc.astype(np.int64), amt.view(np.uint32).astype(np.int64), risk.astype(np.int64)], 1)
        o.engine.send(0, ts, vals, None)
        g.engine.send(0, ts, vals, None)
        om = o.engine.take_matches(lambda q: 3)
        assert g.engine.take_matches(lambda q: 3) == om
        total += len(om)
    assert total > 1000


# ---- absent patterns (kgen.h fire_timers / absent_timer) against the oracle ----
from test_absent_kat import FIXTURES as ABSENT_FIXTURES, check_absent_rows, out_of_scope, \
    run_absent_fixture  # noqa: E402

ABSENT_IN_SCOPE = [f for f in ABSENT_FIXTURES if not out_of_scope(f)]


@pytest.mark.parametrize("fx", ABSENT_IN_SCOPE, ids=[f["id"] for f in ABSENT_IN_SCOPE])
def test_kgen_host_absent_kat(fx):
    """The host build of the device interpreter runs the reference's absent-pattern timelines: the
    same match tuples as the oracle, in the same order, and the reference's asserted counts/rows."""
    o, _, _ = run_absent_fixture(fx)
    g, rows, checks = run_absent_fixture(fx, engine_factory=lambda blob: KGenHostEngine(blob))
    assert g.matches == o.matches
    check_absent_rows(fx, rows, checks)


def run_timeline(src, seed, engine_factory=None):
    from fuzz_apps import random_timeline
    app = App(src, engine_factory)
    app.start(0)
    for stream, row, t in random_timeline(seed):
        if stream == "advance":
            app.advance_time(t)
        else:
            app.send(stream, [row], [t])
    return app


@pytest.mark.parametrize("seed", range(200))
def test_kgen_host_absent_fuzz(seed):
    """Random absent patterns / sequences (any position, every, within, cross-references) over a
    random timeline of events and idle time: the host build of the device interpreter emits the
    oracle's matches in the oracle's order."""
    from fuzz_apps import random_absent_app
    src = random_absent_app(seed, partition=seed % 3 == 0)
    try:
        o = run_timeline(src, seed)
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    g = run_timeline(src, seed, engine_factory=lambda blob: KGenHostEngine(blob, R=4096, N=4096, LC=4096))
    assert g.matches == o.matches


def test_kgen_host_c5_family():
    """The C5 family (4 joined streams, one partition key, mixed 2-4-state patterns) on the host
    build of the K_gen interpreter equals the oracle."""
    from c5_family import run_c5
    o = run_c5(32, 200, 1500, 500)
    g = run_c5(32, 200, 1500, 500, engine_factory=lambda blob: KGenHostEngine(blob, R=4096, N=4096, LC=4096))
    assert g.matches == o.matches and len(o.matches) > 100


@pytest.mark.parametrize("key_type", ["int", "long", "bool"])
@pytest.mark.parametrize("seed", range(8))
def test_kgen_host_fanout(seed, key_type):
    """A stream the partition does not key reaches every key's instances in the order of the
    reference's ConcurrentHashMap of "streamId + key" (chm_order.h vs the oracle's own restatement):
    up to 60 keys, so the map resizes past 64 bins and bins collide."""
    from fuzz_apps import fanout_app, fanout_events
    src = fanout_app(seed, key_type)
    o, g = App(src), App(src, engine_factory=lambda blob: KGenHostEngine(blob, R=4096, N=4096, LC=4096))
    for stream, row, t in fanout_events(seed, keys=20 + 5 * seed, key_type=key_type):
        o.send(stream, [row], [t])
        g.send(stream, [row], [t])
    assert len(o.matches) > 20
    assert g.matches == o.matches


def test_fanout_plans_for_every_key_type():
    """The junction-map order needs String.valueOf of the key: int / long / bool text, a string's
    registered text (sdh_engine_set_strings), Java 8 Float / Double.toString (java_fmt.h): every key
    type plans for fan-out partitions."""
    from fuzz_apps import fanout_app
    from siddhi_amd.planner import compile_app
    for key_type in ("int", "long", "bool", "string", "float", "double"):
        assert compile_app(fanout_app(0, key_type)).partitions[0].fanout


def test_fanout_string_keys_on_the_oracle():
    """String keys: the oracle orders the fan-out by "A" + the key's text (its registered
    String.hashCode and UTF-16 length), so the order differs from the int ids'."""
    from fuzz_apps import fanout_app, fanout_events
    src = fanout_app(2, "string")
    o = App(src)
    for stream, row, t in fanout_events(2, keys=30, key_type="string"):
        o.send(stream, [row], [t])
    assert len(o.matches) > 20
