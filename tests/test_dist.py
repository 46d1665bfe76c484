"""The N>1 path on CPU (gloo, world_size 2): pattern-set sharding with the engine's shard rule, the
event stream delivered to every rank, per-rank engines, match gather to rank 0 and the R18 merge
(siddhi_amd/dist.py). The merged output must equal a single engine running every query.

Each rank runs the CPU oracle on its shard's sub-app (test infrastructure): what is under test
here is the sharding rule, the gather and the merge, which the multi-GPU bench path shares."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from siddhi_amd import dist as sdist

STREAMS = ("define stream A (k int, v int, p float); define stream B (k int, v int, p float);")
TOP = [
    "@info(name='t0') from every e1=A[v > 5] -> e2=B[p > e1.p] within 30 milliseconds select e1.v as a insert into O;",
    "@info(name='t1') from every e1=A[v < 3], e2=A[v > e1.v] select e1.v as a insert into O;",
    "@info(name='t2') from every e1=B[p > 4] <2:3> -> e2=A[v == 7] within 40 milliseconds select e1[0].v as a insert into O;",
    "@info(name='t3') from every e1=A[v > 1] -> e2=B[v > 8] or e3=A[p < 1] within 25 milliseconds select e1.v as a insert into O;",
]
PART = [
    "@info(name='p0') from every e1=A[v > 4] -> e2=A[p > e1.p] within 50 milliseconds select e1.v as a insert into O;",
    "@info(name='p1') from every e1=B[v > 2] -> e2=A[v > e1.v] and e3=B[p < 2] within 60 milliseconds select e1.v as a insert into O;",
]
# absent states inside the partition: timer matches of different keys fire before the same event
# (the merge must order them by (tb, query, key) across ranks)
PART_ABSENT = [
    "@info(name='p2') from every e1=A[v > 6] -> not B[p > 8] for 15 milliseconds select e1.v as a insert into O;",
    "@info(name='p3') from every e1=B[v > 7] -> not A[v < 2] for 9 milliseconds select e1.v as a insert into O;",
]


def full_src(absent=False):
    part = PART + (PART_ABSENT if absent else [])
    return " ".join([STREAMS, TOP[0], TOP[1], "partition with (k of A, k of B) begin", *part, "end;", TOP[2], TOP[3]])


def shard_src(ir, rank, world, absent=False):
    """Rank `rank`'s sub-app: its pattern shard of the unpartitioned queries plus the whole partition
    block (every rank runs the partition for the keys it owns)."""
    names = {ir.queries[q].name for q in range(len(ir.queries)) if sdist.shard_of(ir, q, world) in (rank, -1)}
    parts = [STREAMS] + [q for q in TOP[:2] if q.split("'")[1] in names]
    parts += ["partition with (k of A, k of B) begin", *PART, *(PART_ABSENT if absent else []), "end;"]
    parts += [q for q in TOP[2:] if q.split("'")[1] in names]
    return " ".join(parts), names


def events(seed=3, n=400):
    rng = np.random.default_rng(seed)
    t, out = 0, []
    for _ in range(n):
        t += int(rng.integers(0, 4))
        out.append(("A" if rng.random() < 0.5 else "B",
                    [int(rng.integers(0, 3)), int(rng.integers(0, 10)), float(np.float32(rng.integers(0, 20) / 2))], t))
    return out


def _worker(rank, world, port, results, absent=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from harness import App
    from siddhi_amd import ql
    from siddhi_amd.ir import T_INT
    from siddhi_amd.planner import plan
    ir = plan(ql.parse(full_src(absent)))
    src, names = shard_src(ir, rank, world, absent)
    local = App(src)
    log = sdist.StreamLog()
    evs = events()
    for stream, row, t in evs:  # every rank sees the whole stream (the broadcast)
        local.send(stream, [row], [t])
        log.push(ir.stream_index(stream), 1)
    local.advance_time(evs[-1][2] + 100)  # trailing timers fire (seq = one past the last event)
    rows, meta = [], []
    for m, mt in zip(local.matches, local.meta):
        gq = ir.query_index(local.ir.queries[m[0]].name)  # local query index -> global
        if ir.queries[gq].partition_idx >= 0 and sdist.key_shard(m[1], T_INT, world) != rank:
            continue  # another rank owns this key (the device drops its events at routing)
        rows.append((gq,) + tuple(m[1:]))
        meta.append(mt)
    q = [m[0] for m in rows]
    words, off = [], [0]
    for m in rows:
        for sl in m[3]:
            words += [len(sl), *sl]
        off.append(len(words))
    seq = [mt[0] for mt in meta]  # the event whose processing produced the match
    tb = [mt[1] for mt in meta]
    cols = sdist.columns_from_arrays(q, [m[1] for m in rows], [m[2] for m in rows], off, words, seq, tb)
    per_rank = sdist.gather_columns(cols)
    if rank == 0:
        full = App(full_src(absent))
        for stream, row, t in evs:
            full.send(stream, [row], [t])
        full.advance_time(evs[-1][2] + 100)
        merged = sdist.columns_to_tuples(sdist.merge_columns(ir, per_rank, log))
        results["timers"] = sum(1 for x in tb if x != sdist.TB_EVENT)
        results["ok"] = merged == full.matches
        results["n"] = len(full.matches)
        results["sizes"] = [int(c["q"].numel()) for c in per_rank]
        results["part_split"] = [int(sum(1 for x in c["q"].tolist() if ir.queries[x].partition_idx >= 0))
                                 for c in per_rank]
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,absent", [(2, False), (3, False), (2, True), (3, True)])
def test_sharded_gather_merge_equals_single_engine(world, absent):
    """Pattern-set + key sharding, the column gather (gloo) and the R18 merge reproduce one engine
    (with absent states in the partition: timer matches of several ranks before one event)."""
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), results, absent), nprocs=world, join=True)
    assert results["n"] > 50
    assert all(s > 0 for s in results["sizes"])
    assert sum(1 for x in results["part_split"] if x > 0) >= 2  # partition keys really split
    if absent:
        assert results["timers"] > 10
    assert results["ok"]


def test_merge_order_is_a_stable_kway_merge():
    """merge_order over sorted runs equals a stable sort of the concatenation (ties in run order)."""
    import torch
    g = torch.Generator().manual_seed(5)
    for _ in range(20):
        runs = [torch.sort(torch.randint(0, 40, (int(torch.randint(0, 30, (1,), generator=g)),), generator=g)).values
                for _ in range(int(torch.randint(1, 5, (1,), generator=g)))]
        pos = torch.cat(sdist.merge_order(runs))
        cat = torch.cat(runs)
        want = torch.sort(cat, stable=True).indices
        perm = torch.empty_like(pos)
        perm[pos] = torch.arange(cat.numel())
        assert torch.equal(perm, want)


def test_shard_rule():
    from siddhi_amd import ql
    from siddhi_amd.planner import plan
    ir = plan(ql.parse(full_src()))
    for world in (1, 2, 3, 8):
        owners = [sdist.shard_of(ir, q, world) for q in range(len(ir.queries))]
        for p in ir.partitions:
            assert all(owners[q] == -1 for q in p.query_idx)  # partitions run on every rank
        assert all(-1 <= o < world for o in owners)


def test_key_shard_is_the_reference_destination_rule():
    """|String.valueOf(key).hashCode() % N| (PartitionedDistributionStrategy.java:98-109)."""
    from siddhi_amd.ir import T_BOOL, T_INT, T_LONG
    assert sdist.java_string_hash("123") == 48690
    assert sdist.java_string_hash("-7") == 1450
    assert sdist.java_string_hash("true") == 3569038
    assert sdist.key_shard(123, T_INT, 8) == 48690 % 8
    assert sdist.key_shard(-7, T_INT, 4) == 1450 % 4
    assert sdist.key_shard((1 << 32) - 7, T_INT, 4) == 1450 % 4  # raw word of int -7
    big = -9223372036854775808
    h = sdist.java_string_hash(str(big))
    assert sdist.key_shard(big, T_LONG, 5) == abs(h) % 5
    assert sdist.key_shard(1, T_BOOL, 3) == 3569038 % 3
    counts = [0] * 4
    for k in range(1000):
        counts[sdist.key_shard(k, T_INT, 4)] += 1
    assert min(counts) > 150
