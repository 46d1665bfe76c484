"""GPU parity at each BASELINE config's full pattern count (SURVEY §8(c) large-stream golden vectors).

The HIP engine runs the whole pattern set of C1-C4 over the seeded synthetic stream, pushed from
HBM in large batches and polled through the C-ABI (sdh_engine_poll: the device R18 sort); the
R18-ordered match stream must reproduce the oracle's digest (tests/large_golden.py) and the
committed explicit samples exactly. The goldens were generated in the container by
tests/golden/make_large_golden.py (the oracle sharded by pattern set); nothing here runs the oracle.
"""
import ctypes

import numpy as np
import pytest

from harness import App
from large_golden import CONFIGS, Digest, app_source, events, load

pytestmark = pytest.mark.gpu

# push sizes on the device (the digest does not depend on how the stream is cut)
PUSH = {"c1": 1 << 18, "c2": 1 << 17, "c3": 1 << 16, "c4": 1 << 16, "c2x": 1 << 17}


def _engine(name, blob, types):
    from siddhi_amd.engine import HipEngine
    cfg = CONFIGS[name]
    if name == "c3":
        return HipEngine(blob, stream_types=types, gen_pool_states=32, gen_pool_nodes=128, gen_list_cap=32,
                         gen_max_keys=2 * cfg["keys"])
    return HipEngine(blob, stream_types=types)


def _run(name, n_events=None, check_every=None):
    import torch
    cfg = CONFIGS[name]
    g = load(name)
    app = App(app_source(name, cfg["patterns"]), engine_factory=lambda blob: None)
    eng = _engine(name, app.blob, [s.attr_types for s in app.ir.streams])
    dig = Digest(g["sample_stride"])
    dev = torch.device("cuda:0")
    n_events = n_events or cfg["events"]
    B = PUSH[name]
    for lo in range(0, n_events, B):
        n = min(B, n_events - lo)
        ts, cols, _ = events(name, lo, n)
        t_ts = torch.from_numpy(ts).to(dev)
        t_cols = [torch.from_numpy(np.ascontiguousarray(c).view(np.int32)).to(dev) for c in cols]
        eng.push_device(0, n, t_ts.data_ptr(), [c.data_ptr() for c in t_cols])
        dig.update(*eng.poll())
    return g, dig, eng


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4"])
def test_large_golden_full_config(name):
    g, dig, eng = _run(name)
    assert dig.n == g["n_matches"], f"{name}: {dig.n} matches, golden {g['n_matches']}"
    assert dig.first == g["sample_first"]
    assert dig.strided == g["sample_strided"]
    assert dig.n_words == g["n_words"]
    assert dig.hexdigest() == g["digest"]
    assert eng.stats().events == g["events"]


def _hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return lib


def _d2h(hip, ptr, first, n):
    out = np.zeros(n, np.int64)
    if n:
        addr = ctypes.cast(ptr, ctypes.c_void_p).value + first * 8
        assert hip.hipMemcpy(out.ctypes.data, addr, n * 8, 2) == 0  # hipMemcpyDeviceToHost
    return out


def _digest_device_matches(eng, dig, chunk=1 << 24):
    """sdh_engine_poll_device, then the R18-ordered tuples streamed to the host in slices into the
    running digest (the digest is independent of how the stream is cut)."""
    hip = _hip()
    m = eng.poll_device()
    for lo in range(0, m.n, chunk):
        n = min(chunk, m.n - lo)
        off = _d2h(hip, m.off, lo, n + 1)
        words = _d2h(hip, m.words, int(off[0]), int(off[-1] - off[0]))
        dig.update(_d2h(hip, m.query, lo, n), _d2h(hip, m.key, lo, n), _d2h(hip, m.ts, lo, n), off - off[0], words)
    return m.n


@pytest.mark.timeout(900)
def test_headline_config_golden():
    """The headline configuration itself (bench.py's default workload): 10,000 C2 patterns over 200K
    events (~860M matches), pushed from HBM in 100K-event batches, against the oracle's golden
    (tests/golden/large_c2h.json). The same pushes in SDH_FLAG_DEVICE_MATCHES mode (the bench's) write
    the same K_ratchet records: equal counts and equal order-independent record hashes
    (sdh_engine_debug_digest); and one 200K-event push in that mode produces the golden's count."""
    import torch
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES, HipEngine
    cfg = CONFIGS["c2h"]
    g = load("c2h")
    app = App(app_source("c2h", cfg["patterns"]), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    dev = torch.device("cuda:0")

    def batch(lo, n):
        ts, cols, _ = events("c2h", lo, n)
        t_ts = torch.from_numpy(ts).to(dev)
        t_cols = [torch.from_numpy(np.ascontiguousarray(c).view(np.int32)).to(dev) for c in cols]
        return t_ts, t_cols

    normal = HipEngine(app.blob, stream_types=types)
    ring = HipEngine(app.blob, stream_types=types, flags=SDH_FLAG_DEVICE_MATCHES)
    dig = Digest(g["sample_stride"])
    B = cfg["events"] // 2
    for lo in range(0, cfg["events"], B):
        t_ts, t_cols = batch(lo, B)
        for e in (normal, ring):
            e.push_device(0, B, t_ts.data_ptr(), [c.data_ptr() for c in t_cols])
        dn, dr = normal.debug_digest(), ring.debug_digest()
        assert dn == dr and dn[0] > 0, f"normal-mode records {dn} != device-match-mode records {dr}"
        assert ring.pending_matches() == dn[0]
        assert _digest_device_matches(normal, dig) == dn[0]
    ring.close()
    normal.close()
    assert dig.n == g["n_matches"]
    assert dig.first == g["sample_first"]
    assert dig.strided == g["sample_strided"]
    assert dig.n_words == g["n_words"]
    assert dig.hexdigest() == g["digest"]
    one = HipEngine(app.blob, stream_types=types, flags=SDH_FLAG_DEVICE_MATCHES)
    t_ts, t_cols = batch(0, cfg["events"])
    one.push_device(0, cfg["events"], t_ts.data_ptr(), [c.data_ptr() for c in t_cols])
    assert one.pending_matches() == g["n_matches"]
    assert one.debug_digest()[0] == g["n_matches"]


@pytest.mark.timeout(900)
def test_c2x_config_golden():
    """The C2x family (bench.py --workload c2x; workloads.c2x_app: C2 with an event-only conjunct
    `volume > V_p` on e2, off K_ratchet) at its 10,000 patterns over 200K events, on K_gate
    (nfa_gate.hip), against the oracle's golden (tests/golden/large_c2x.json): the R18-ordered
    tuples of every push (sdh_engine_poll_device) reproduce the golden digest and samples, and the
    same pushes in SDH_FLAG_DEVICE_MATCHES mode write the same records (count and hash)."""
    import os
    import torch
    from large_golden import golden_path
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES, HipEngine
    if not os.path.exists(golden_path("c2x")):
        pytest.skip("tests/golden/large_c2x.json not generated")
    cfg = CONFIGS["c2x"]
    g = load("c2x")
    app = App(app_source("c2x", cfg["patterns"]), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    dev = torch.device("cuda:0")
    normal = HipEngine(app.blob, stream_types=types)
    ring = HipEngine(app.blob, stream_types=types, flags=SDH_FLAG_DEVICE_MATCHES)
    assert normal.stats().plan_queries[1] == cfg["patterns"]  # (every query on K_gate)
    dig = Digest(g["sample_stride"])
    B = PUSH["c2x"]
    for lo in range(0, cfg["events"], B):
        n = min(B, cfg["events"] - lo)
        ts, cols, _ = events("c2x", lo, n)
        t_ts = torch.from_numpy(ts).to(dev)
        t_cols = [torch.from_numpy(np.ascontiguousarray(c).view(np.int32)).to(dev) for c in cols]
        for e in (normal, ring):
            e.push_device(0, n, t_ts.data_ptr(), [c.data_ptr() for c in t_cols])
        dn, dr = normal.debug_digest(), ring.debug_digest()
        assert dn == dr and dn[0] > 0, f"normal-mode records {dn} != device-match-mode records {dr}"
        assert _digest_device_matches(normal, dig) == dn[0]
    ring.close()
    normal.close()
    assert dig.n == g["n_matches"], f"c2x: {dig.n} matches, golden {g['n_matches']}"
    assert dig.first == g["sample_first"]
    assert dig.strided == g["sample_strided"]
    assert dig.n_words == g["n_words"]
    assert dig.hexdigest() == g["digest"]


@pytest.mark.timeout(600)
def test_bench_shape_one_push_equals_many():
    """The bench's exact timed configuration (bench.py's default line): one 8M-event push of the
    10K-pattern C2 family, from HBM, in SDH_FLAG_DEVICE_MATCHES mode writes every record (about 3.6e10,
    rec4 blocks that never wrap): its record digest -- count and order-independent hash of (e2 seq,
    query, e1 seq), sdh_engine_debug_digest -- equals the sum of the digests of the same events in 64
    normal-mode pushes of 128K (each placed at its R18 rows, the compact rows poll_compact hands out),
    and sdh_engine_poll_records hands out that many records."""
    import torch
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES, SDH_REC_4, HipEngine
    from siddhi_amd.workloads import c2_app, stock_events_torch
    app = App(c2_app(10000), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    dev = torch.device("cuda:0")
    B, parts = 1 << 23, 64
    ts, sym, price, vol = stock_events_torch(0, B, 100, dev)
    cols = [sym, price.view(torch.int32), vol]
    torch.cuda.synchronize()
    one = HipEngine(app.blob, stream_types=types, flags=SDH_FLAG_DEVICE_MATCHES)
    one.push_device(0, B, ts.data_ptr(), [c.data_ptr() for c in cols])
    d1 = one.debug_digest()
    rec = one.poll_records()
    assert rec.r_format == SDH_REC_4 and rec.n == rec.r_n == d1[0] and rec.r_bytes < 5 * rec.r_n
    one.close()
    normal = HipEngine(app.blob, stream_types=types)
    n, acc, hsum = B // parts, 0, 0
    for i in range(parts):
        ptrs = [c.data_ptr() + i * n * c.element_size() for c in cols]
        normal.push_device(0, n, ts.data_ptr() + i * n * 8, ptrs)
        dn = normal.debug_digest()
        acc += dn[0]
        hsum = (hsum + dn[1]) % (1 << 64)
        assert normal.poll_compact(device=True).n == dn[0]  # (drops the window)
    assert normal.stats().placed_pushes == parts
    normal.close()
    assert d1[0] > 3e10 and (acc, hsum) == d1


@pytest.mark.parametrize("mixed", [False, True])
def test_direct_placement_equals_sort(mixed):
    """Pushes whose matches all come from K_ratchet go straight to their R18 rows (nfa_ratchet.hip
    COUNT + scan + WRITE passes, compact rows; no sort at poll). Against the same pushes with
    placement off (SDH_NO_PLACE: match records, the device table + radix sort): identical poll
    output, over polls after one push and after several (placed windows), and -- `mixed` -- with
    chain / K_gen queries whose rare matches turn a placed window back into table rows
    (placed_to_table)."""
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.workloads import c2_app, stock_events
    src = c2_app(200)
    if mixed:
        src += (" @info(name='x3') from every e1=StockStream[price > 90] -> e2=StockStream[price < 10] "
                "-> e3=StockStream[price > e1.price] within 1 sec select e1.price as a insert into O;"
                " @info(name='xl') from every e1=StockStream[price > 98] -> e2=StockStream[volume > 990] "
                "or e3=StockStream[price < 0.5] within 1 sec select e1.price as a insert into O;")
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    a = HipEngine(app.blob, stream_types=types)
    b = HipEngine(app.blob, stream_types=types, debug={"SDH_NO_PLACE": 1})
    sizes = [700, 9000, 5, 1300, 40000, 1, 2500, 800, 800, 800, 6000, 300] * 2
    polls = {0, 2, 4, 5, 9, 10, 13, 17, 20, 23}
    lo, n_total, with_matches = 0, 0, 0
    for i, n in enumerate(sizes):
        ts, sym, price, vol = stock_events(lo, n)
        lo += n
        cols = [sym, price.view(np.uint32), vol]
        m0 = a.stats().matches
        a.push_columns(0, ts, cols)
        with_matches += a.stats().matches > m0
        b.push_columns(0, ts, cols)
        if i in polls:
            ga, gb = a.poll(with_seq=True), b.poll(with_seq=True)
            for x, y in zip(ga, gb):
                assert np.array_equal(x, y)
            n_total += len(ga[0])
    assert n_total > 100000
    placed = a.stats().placed_pushes
    assert b.stats().placed_pushes == 0
    # every push with a match is placed; a push without one (a 1-event push whose price closes no
    # pending partial) has nothing to place. mixed: pushes where the chain / K_gen queries match too
    # go through the table
    if mixed:
        assert 0 < placed < with_matches
    else:
        assert placed == with_matches and with_matches >= len(sizes) - 4


def test_poll_device_equals_poll():
    """sdh_engine_poll_device leaves the same R18-ordered tuples in HBM that sdh_engine_poll copies
    to the host (two engines over the same C2 stream: ratchet + chain + K_gen plans)."""
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.workloads import c2_app, stock_events
    src = c2_app(70) + (" @info(name='x3') from every e1=StockStream[price > 90] -> e2=StockStream[price < 10] "
                        "-> e3=StockStream[price > e1.price] within 1 sec select e1.price as a insert into O;"
                        " @info(name='xl') from every e1=StockStream[price > 95] -> e2=StockStream[volume > 900] "
                        "or e3=StockStream[price < 1] within 1 sec select e1.price as a insert into O;")
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    a, b = HipEngine(app.blob, stream_types=types), HipEngine(app.blob, stream_types=types)
    ts, sym, price, vol = stock_events(0, 30000)
    cols = [sym, price.view(np.uint32), vol]
    a.push_columns(0, ts, cols)
    b.push_columns(0, ts, cols)
    q, k, t, off, words = a.poll()
    m = b.poll_device()
    assert m.n == len(q) > 100000
    hip = _hip()
    D2H = 2
    for ptr, want in ((m.query, q), (m.key, k), (m.ts, t), (m.off, off), (m.words, words)):
        got = np.zeros(len(want), np.int64)
        addr = ctypes.cast(ptr, ctypes.c_void_p).value
        assert hip.hipMemcpy(got.ctypes.data, addr, got.nbytes, D2H) == 0
        assert np.array_equal(got, want)
    assert set(np.unique(q).tolist()) >= {70, 71}  # the chain and K_gen queries matched too
