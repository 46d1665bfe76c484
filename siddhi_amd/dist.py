"""Multi-GPU sharding and match gather.

One process per GPU. State is private per (pattern, key), so the path shards with no data-path
collective: every rank sees the whole event stream (broadcast, or per-rank H2D from pinned host
memory), runs only its own query shard, and keeps its matches. The one exchange step is the match
gather to rank 0, where the per-rank match lists -- each already in the reference's delivery order
(R18) -- are merged into the single-engine order.

Shard rule (mirrors sdh_engine_create): query q runs on rank `shard_key(q) % world`, where
shard_key is q itself for an unpartitioned query and the partition's first query for a partitioned
one (a partition's queries share their per-key instances' routing, so they stay together).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

from .ir import R_MULTI, ProgramIR


def shard_key(ir: ProgramIR, q: int) -> int:
    pi = ir.queries[q].partition_idx
    return q if pi < 0 else ir.partitions[pi].query_idx[0]


def shard_of(ir: ProgramIR, q: int, world: int) -> int:
    return shard_key(ir, q) % max(1, world)


def output_ranks(ir: ProgramIR) -> Dict[Tuple[int, int], int]:
    """R18 order of the matches of one event across queries, per (query, stream): junction
    subscribers in definition order (a partition subscribes at its first query); inside a partition
    the multi-processor receivers emit while the event is delivered, the single-processor
    receivers' deferred selector calls follow (siddhi_amd/csrc/gen_lower.h output_ranks)."""
    nq, ns = len(ir.queries), len(ir.streams)
    rank: Dict[Tuple[int, int], int] = {}

    def multi(q, s):
        return any(r.stream_idx == s and r.kind == R_MULTI for r in ir.queries[q].receivers)

    for s in range(ns):
        done, r = set(), 0
        for q in range(nq):
            pi = ir.queries[q].partition_idx
            if pi < 0:
                rank[(q, s)] = r
                r += 1
                continue
            if pi in done:
                continue
            done.add(pi)
            for want_multi in (True, False):
                for pq in ir.partitions[pi].query_idx:
                    if multi(pq, s) == want_multi:
                        rank[(pq, s)] = r
                        r += 1
    return rank


def merge_matches(ir: ProgramIR, stream_of_seq, per_rank: Sequence[List[tuple]]) -> List[tuple]:
    """Merge per-rank match lists (each in R18 order) into the single-engine order.

    A match is (query, key, ts, slots); its triggering event is the newest event in its slots (the
    event being processed is copied into a slot before the selector runs)."""
    ranks = output_ranks(ir)
    keyed = []
    for r, lst in enumerate(per_rank):
        for i, m in enumerate(lst):
            seq = max(x for slot in m[3] for x in slot)
            keyed.append(((seq, ranks[(m[0], stream_of_seq(seq))], r, i), m))
    keyed.sort(key=lambda t: t[0])
    return [m for _, m in keyed]


def gather_matches(local: List[tuple], group=None) -> List[List[tuple]] | None:
    """Gather every rank's match list to rank 0 (torch.distributed; RCCL or gloo). Returns the
    per-rank lists on rank 0, None elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = [None] * world if dist.get_rank(group) == 0 else None
    dist.gather_object(local, out, dst=0, group=group)
    return out
