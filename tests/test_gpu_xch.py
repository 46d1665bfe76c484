"""The multi-GPU exchange behind the C-ABI (include/siddhi_hip.h sdh_comm_*, sdh_engine_push_bcast,
sdh_engine_gather; csrc/comm.hip): every rank's engine runs its shard of one program
(sdh_config.shard_rank / shard_world), each batch reaches every rank through the library's broadcast,
and the library gathers every rank's R18-ordered matches to rank 0 and merges them on the device.

On this one-GPU box the ranks are engines of one process joined by a local communicator
(sdh_comm_create_local: the same protocol, buffers copied device-to-device); RCCL itself runs at
world 1 (ncclCommInitRank, broadcast and gather through it). The merged stream must equal one
unsharded engine and the oracle, tuple for tuple, in order: the absent app (timer matches of several
ranks before one event), the C3 family (key shards), the C4 family (pattern-set shards), chunk pushes
and the K_ratchet placed windows of the C2 family."""
import numpy as np
import pytest

from dist_gpu_child import batches
from harness import App
from test_dist import events, full_src

pytestmark = pytest.mark.gpu


def tuples(q, k, ts, off, words, *rest):
    out = []
    for i in range(len(q)):
        w = words[off[i]:off[i + 1]]
        slots, j = [], 0
        while j < len(w):
            c = int(w[j])
            slots.append(tuple(int(x) for x in w[j + 1:j + 1 + c]))
            j += 1 + c
        out.append((int(q[i]), int(k[i]), int(ts[i]), tuple(slots)))
    return out


class Sharded:
    """`world` engines of one program on this GPU, joined by a local communicator."""

    def __init__(self, blob, types, world, **kw):
        from siddhi_amd.engine import Comm, HipEngine
        self.comms = Comm.local(world)
        self.engs = [HipEngine(blob, shard_rank=r, shard_world=world, stream_types=types, **kw) for r in range(world)]
        for e, c in zip(self.engs, self.comms):
            e.set_comm(c)
        self.out = []
        self.sizes = [0] * world

    def push(self, si, ts, cols, chunk=False):
        self.engs[0].push_bcast_columns(si, ts, cols, root=0, chunk=chunk)
        for e in self.engs[1:]:
            e.push_bcast_recv(root=0)

    def push_device(self, si, n, ts_ptr, col_ptrs):
        self.engs[0].push_bcast_device(si, n, ts_ptr, col_ptrs, root=0)
        for e in self.engs[1:]:
            e.push_bcast_recv(root=0)

    def gather(self):
        for r in range(len(self.engs) - 1, 0, -1):  # (local communicator: rank 0 last)
            assert len(self.engs[r].gather()[0]) == 0
        self.out.extend(tuples(*self.engs[0].gather()))

    def advance_time(self, t):
        for e in self.engs:
            e.advance_time(t)

    def stats(self):
        return [e.stats() for e in self.engs]

    def close(self):
        for e in self.engs:
            e.close()


def _single(blob, types, **kw):
    from siddhi_amd.engine import HipEngine
    return HipEngine(blob, stream_types=types, **kw)


def _device_tuples(m, dev):
    """tuples of an sdh_matches whose pointers are in HBM"""
    import torch
    from siddhi_amd import dist as sdist
    hip = sdist._hip()
    t = {}
    for f, p, n in (("q", m.query, m.n), ("key", m.key, m.n), ("ts", m.ts, m.n), ("off", m.off, m.n + 1)):
        t[f] = torch.empty(n, dtype=torch.int64, device=dev)
        if n:
            sdist._d2d(hip, t[f].data_ptr(), p, n * 8)
    off = t["off"].cpu().numpy()
    words = torch.empty(int(off[-1]), dtype=torch.int64, device=dev)
    if words.numel():
        sdist._d2d(hip, words.data_ptr(), m.words, words.numel() * 8)
    return tuples(t["q"].cpu().numpy(), t["key"].cpu().numpy(), t["ts"].cpu().numpy(), off, words.cpu().numpy())


def _raw(cols, types):
    """native-width columns -> the raw attribute words the oracle engine takes"""
    from siddhi_amd.ir import T_FLOAT
    return np.stack([c.view(np.uint32).astype(np.int64) if t == T_FLOAT else c.astype(np.int64)
                     for c, t in zip(cols, types)], 1)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("chunk", [False, True], ids=["events", "chunks"])
def test_absent_app_gather_equals_single_engine_and_oracle(world, chunk):
    from siddhi_amd.engine import columns_from_words
    from siddhi_amd.events import encode_rows
    src = full_src(absent=True)
    oracle = App(src)
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    sh = Sharded(app.blob, types, world)
    evs = events()
    for i, (stream, rows, ts) in enumerate(batches(evs)):
        oracle.send(stream, rows, ts, as_chunk=chunk)
        si = app.ir.stream_index(stream)
        vals, nulls = encode_rows(rows, types[si], app.dictionary)
        sh.push(si, np.asarray(ts, np.int64), columns_from_words(vals, types[si]), chunk=chunk)
        if i % 3 == 2:
            sh.gather()
    oracle.advance_time(evs[-1][2] + 100)
    sh.advance_time(evs[-1][2] + 100)
    sh.gather()
    want = [tuple(m) for m in oracle.matches]
    assert len(want) > 50
    assert sh.out == want
    sh.close()


def _c_family(name, n_patterns, n_events, push, keys):
    from siddhi_amd.workloads import c3_app, c4_app, stock_events, txn_events
    src = c3_app(n_patterns) if name == "c3" else c4_app(n_patterns)
    gen = stock_events if name == "c3" else txn_events
    out = []
    for s in range(0, n_events, push):
        ts, a, b, c = gen(s, push, keys)
        out.append((ts, [a, b.view(np.uint32), c]))
    return src, out


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("family", ["c3", "c4"])
def test_c3_c4_gather_equals_single_engine_and_oracle(family, world):
    """C3: partitioned count / logical patterns, key shards; C4: sequences, pattern-set shards."""
    src, pushes = _c_family(family, 24, 3000, 500, 16 if family == "c3" else 40)
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    oracle = App(src)
    single = _single(app.blob, types)
    sh = Sharded(app.blob, types, world)
    want, got1 = [], []
    for i, (ts, cols) in enumerate(pushes):
        oracle.engine.send(0, ts, _raw(cols, types[0]), None)
        oracle._take()
        single.push_columns(0, ts, cols)
        got1.extend(tuples(*single.poll()))
        sh.push(0, ts, cols)
        if i % 2 == 1:
            sh.gather()
    sh.gather()
    want = [tuple(m) for m in oracle.matches]
    assert len(want) > 100
    assert got1 == want
    assert sh.out == want
    sh.close()
    single.close()


def test_c2_placed_windows_gather_from_device_batches():
    """C2: K_ratchet's placed windows (compact rows, no table) merge by their compact-row keys; the
    root's batches are device-resident (push_bcast_device) and gathered as HBM pointers too."""
    import torch
    from siddhi_amd.workloads import c2_app, stock_events_torch
    app = App(c2_app(100), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    single = _single(app.blob, types)
    sh = Sharded(app.blob, types, 2)
    dev = torch.device("cuda", 0)
    want, n_dev = [], 0
    for s in range(4):
        ts, sym, price, vol = stock_events_torch(s * 1024, 1024, 100, dev)
        cols = [sym, price.view(torch.int32), vol]
        torch.cuda.synchronize()
        single.push_device(0, 1024, ts.data_ptr(), [c.data_ptr() for c in cols])
        want.extend(tuples(*single.poll()))
        sh.push_device(0, 1024, ts.data_ptr(), [c.data_ptr() for c in cols])
        if s == 3:  # the last window gathered in HBM
            sh.engs[1].gather(device=True)
            m = sh.engs[0].gather(device=True)
            n_dev = m.n
            sh.out.extend(_device_tuples(m, dev))
        else:
            sh.gather()
    assert len(want) > 5000 and n_dev > 0
    assert sh.out == want
    assert all(st.placed_pushes > 0 for st in sh.stats())
    sh.close()
    single.close()


def test_rccl_world_one_broadcast_and_gather():
    """RCCL itself: ncclGetUniqueId, ncclCommInitRank at world 1, a broadcast push and a gather
    through it equal a plain engine's pushes and polls."""
    from siddhi_amd.engine import Comm, HipEngine
    src, pushes = _c_family("c3", 12, 1500, 500, 8)
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    comm = Comm.rccl(Comm.unique_id(), 0, 1, 0)
    eng = HipEngine(app.blob, shard_rank=0, shard_world=1, stream_types=types)
    eng.set_comm(comm)
    plain = _single(app.blob, types)
    got, want = [], []
    for ts, cols in pushes:
        eng.push_bcast_columns(0, ts, cols, root=0)
        plain.push_columns(0, ts, cols)
        got.extend(tuples(*eng.gather()))
        want.extend(tuples(*plain.poll()))
    assert len(want) > 50 and got == want
    eng.close()
    plain.close()
    comm.close()


def test_local_comm_misuse_is_invalid_and_recoverable():
    """Rank 0 gathering before the others, or a non-root receiving before the root pushed, fails with
    SDH_E_INVALID and changes nothing: the window stays pending and the collective then succeeds."""
    from siddhi_amd.engine import EngineError
    src, pushes = _c_family("c4", 12, 1000, 500, 30)
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    single = _single(app.blob, types)
    sh = Sharded(app.blob, types, 2)
    with pytest.raises(EngineError) as ei:
        sh.engs[1].push_bcast_recv(root=0)
    assert ei.value.code == -1
    want = []
    for ts, cols in pushes:
        single.push_columns(0, ts, cols)
        want.extend(tuples(*single.poll()))
        sh.push(0, ts, cols)
    with pytest.raises(EngineError) as ei:
        sh.engs[0].gather()
    assert ei.value.code == -1
    sh.gather()
    assert len(want) > 20 and sh.out == want
    sh.close()
    single.close()
