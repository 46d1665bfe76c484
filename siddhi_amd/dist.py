"""Multi-GPU sharding, event broadcast and match gather.

One process per GPU. State is private per (pattern, key), so the path shards with no data-path
collective but two exchange steps: every rank sees the whole event stream (an RCCL broadcast of each
batch from the ingest rank, or per-rank H2D from pinned host memory), runs only its share, and the
matches are gathered to rank 0, where the per-rank outputs -- each already in the reference's
delivery order (R18) -- are merged into the single-engine order.

Shard rule (mirrors sdh_engine_create and nfa_gen.hip key_shard):
* an unpartitioned query q runs on rank q % world (pattern-set sharding);
* a partition's queries run on every rank, and rank r owns the keys with
  |String.valueOf(key).hashCode() % world| == r -- the reference's PartitionedDistributionStrategy
  destination (stream/output/sink/distributed/PartitionedDistributionStrategy.java:98-109). Float /
  double keys and string dictionary ids hash their raw 64-bit word instead (key_shard below).

The gather moves device buffers: every rank's R18-sorted tuples stay in HBM
(sdh_engine_poll_device), counts are all-gathered and the columns are sent to rank 0 point-to-point
(RCCL over xGMI, or gloo on CPU tensors in the tests).

The merge. Every rank's stream is already in R18 order, i.e. sorted by the key (trigger sequence
number, receiver rank) -- with the global receiver ranks of the full program, since a shard keeps its
queries in definition order. A query's event matches for one event come from one rank (its pattern
shard, or the owner of the event's key), so keys never tie across ranks and the merge is a k-way
merge of sorted runs: each row's output position is its index in its own run plus, for every other
run, the number of rows with a smaller key (torch.searchsorted), then one scatter -- no sort.
Absent-state timer matches (tb != INT64_MIN) precede the event matches of their seq and are ordered
by (tb, query, partition key), then emission order (matches.hip); timers of different keys /
queries of one seq DO come from different ranks, so when any are present the merge is an exact
stable lexicographic sort on those keys instead.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

from .ir import T_BOOL, T_INT, T_LONG, ProgramIR

RANK_BITS = 20  # as nfa_types.h


def shard_of(ir: ProgramIR, q: int, world: int) -> int:
    """Rank of an unpartitioned query, -1 for a partitioned one (it runs on every rank)."""
    if ir.queries[q].partition_idx >= 0:
        return -1
    return q % max(1, world)


def _mix64(z: int) -> int:
    m = (1 << 64) - 1
    z &= m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def java_string_hash(s: str) -> int:
    h = 0
    for c in s:
        h = (31 * h + ord(c)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def key_shard(raw: int, attr_type: int, world: int) -> int:
    """Owner rank of a partition key (raw attribute word, as the engine sees it)."""
    if attr_type in (T_INT, T_LONG):
        v = raw
        if attr_type == T_INT:
            v = ((raw & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000
        h = java_string_hash(str(v))
    elif attr_type == T_BOOL:
        h = java_string_hash("true" if raw else "false")
    else:
        h = (_mix64(raw) >> 33) & 0xFFFFFFFF
        h = h - (1 << 32) if h >= (1 << 31) else h
    r = abs(h) % world  # |h % world| (Java remainder keeps the dividend's sign)
    return r


def output_ranks(ir: ProgramIR) -> Dict[Tuple[int, int], int]:
    """R18 order of the matches of one event across queries, per (query, stream): junction
    subscribers in definition order (a partition subscribes at its first query); inside a partition
    a key's junction holds the clones in the partition's query order (the planner emits
    ``query_idx`` in ``metaQueryRuntimeMap`` order), each emitting at the end of its own chunk
    (siddhi_amd/csrc/gen_lower.h output_ranks)."""
    nq, ns = len(ir.queries), len(ir.streams)
    rank: Dict[Tuple[int, int], int] = {}
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
            for pq in ir.partitions[pi].query_idx:
                rank[(pq, s)] = r
                r += 1
    return rank


class StreamLog:
    """Which stream each global sequence number belongs to (the host pushes the batches, so it
    knows): a list of (seq_base, n, stream) pushes."""

    def __init__(self):
        self.bases: List[int] = []
        self.streams: List[int] = []
        self.next = 0

    def push(self, stream: int, n: int):
        if self.streams and self.streams[-1] == stream:
            self.next += n
            return
        self.bases.append(self.next)
        self.streams.append(stream)
        self.next += n

    def stream_of(self, seq, ignore=None):
        """torch int64 tensor of seqs -> stream index tensor (0 where `ignore` is set: timer rows,
        whose seq may be one past the last push, or precede every push)."""
        import torch
        if not self.bases:
            return torch.zeros_like(seq)
        b = torch.tensor(self.bases, dtype=torch.int64, device=seq.device)
        s = torch.tensor(self.streams, dtype=torch.int64, device=seq.device)
        i = (torch.searchsorted(b, seq, right=True) - 1).clamp(min=0)
        out = s[i]
        return out if ignore is None else torch.where(ignore, torch.zeros_like(out), out)


FIELDS = ("q", "key", "ts", "seq", "tb", "len", "words")
TB_EVENT = -(1 << 63)  # tb of a match completed by an event (include/siddhi_hip.h sdh_matches.tb)


def columns_from_device(eng, device) -> Dict[str, "object"]:
    """This rank's R18-sorted matches since the last poll, left in HBM by sdh_engine_poll_device and
    copied device-to-device into torch tensors on `device`."""
    import torch
    m = eng.poll_device()
    n = m.n
    hip = _hip()
    out = {}
    for name, ptr in (("q", m.query), ("key", m.key), ("ts", m.ts), ("seq", m.seq), ("tb", m.tb), ("off", m.off)):
        t = torch.empty(n + 1 if name == "off" else n, dtype=torch.int64, device=device)
        if t.numel():
            _d2d(hip, t.data_ptr(), ptr, t.numel() * 8)
        out[name] = t
    nw = int(out["off"][-1].item()) if n else 0
    w = torch.empty(nw, dtype=torch.int64, device=device)
    if nw:
        _d2d(hip, w.data_ptr(), m.words, nw * 8)
    out["words"] = w
    out["len"] = out.pop("off").diff() if n else torch.empty(0, dtype=torch.int64, device=device)
    return out


def columns_from_arrays(q, key, ts, off, words, seq, tb=None, device="cpu"):
    import torch
    t = lambda a: torch.as_tensor(a, dtype=torch.int64).to(device)  # noqa: E731
    tb = t(tb) if tb is not None else torch.full((len(q),), TB_EVENT, dtype=torch.int64, device=device)
    return {"q": t(q), "key": t(key), "ts": t(ts), "seq": t(seq), "tb": tb, "len": t(off).diff(),
            "words": t(words)}


def gather_columns(cols, group=None) -> Optional[List[dict]]:
    """Gather every rank's match columns to rank 0 (torch.distributed: RCCL for device tensors, gloo
    for CPU ones): an all-gather of (matches, words), then point-to-point sends to rank 0. Returns
    the per-rank column dicts on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    dev = cols["q"].device
    cnt = torch.tensor([cols["q"].numel(), cols["words"].numel()], dtype=torch.int64, device=dev)
    allc = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(allc, cnt, group=group)
    if me != 0:
        for f in FIELDS:
            if cols[f].numel():
                dist.send(cols[f].contiguous(), dst=0, group=group)
        return None
    out = [cols]
    for r in range(1, world):
        n, nw = (int(x) for x in allc[r].tolist())
        got = {}
        for f in FIELDS:
            t = torch.empty(nw if f == "words" else n, dtype=torch.int64, device=dev)
            if t.numel():
                dist.recv(t, src=r, group=group)
            got[f] = t
        out.append(got)
    return out


def rank_table(ir: ProgramIR):
    """output_ranks as a [query * n_streams + stream] int64 tensor."""
    import torch
    ns = len(ir.streams)
    table = torch.zeros(len(ir.queries) * ns, dtype=torch.int64)
    for (q, s), r in output_ranks(ir).items():
        table[q * ns + s] = r
    return table


def merge_keys(cols, table, ns, stream_log: StreamLog, seq_ref: int = 0):
    """Primary merge key of each row: (trigger seq - seq_ref) << RANK_BITS | class, class 0 for a
    timer match and 1 + the global receiver rank of (query, stream) for an event match. seq_ref is
    the window's smallest trigger seq (as the engine's hi keys subtract its last poll's seq)."""
    import torch
    timer = cols["tb"] != TB_EVENT
    cls = table[cols["q"] * ns + stream_log.stream_of(cols["seq"], timer)] + 1
    rel = cols["seq"] - seq_ref
    if rel.numel() and (int(rel.min()) < 0 or int(rel.max()) >= 1 << (63 - RANK_BITS)):
        raise ValueError("trigger seqs outside the merge window")
    return (rel << RANK_BITS) | torch.where(timer, torch.zeros_like(cls), cls), timer


def merge_order(keys: Sequence["object"]):
    """k-way merge of sorted int64 runs: (run index, position in the output) for every row of every
    run. A row's position is its index in its run plus, per other run, the rows with a smaller key
    (and, for an earlier run, equal keys too: ties keep run order, like a stable sort of the
    concatenation)."""
    import torch
    pos = []
    for r, k in enumerate(keys):
        p = torch.arange(k.numel(), dtype=torch.int64, device=k.device)
        for r2, k2 in enumerate(keys):
            if r2 != r and k2.numel() and k.numel():
                p += torch.searchsorted(k2, k, right=r2 < r)
        pos.append(p)
    return pos


def merge_columns(ir: Optional[ProgramIR], per_rank: Sequence[dict], stream_log: StreamLog, table=None,
                  n_streams: int = 0) -> dict:
    """Per-rank R18-ordered columns -> the single-engine order: a k-way merge of the runs on (trigger
    seq, receiver rank), or, when absent-state timer matches are present, a stable lexicographic sort
    on (seq, class, tb, query, key) of the rank-major concatenation. `table` (rank_table) may be
    given instead of the program."""
    import torch
    dev = per_rank[0]["q"].device
    cat = {f: torch.cat([c[f] for c in per_rank]) for f in FIELDS}
    n = cat["q"].numel()
    if n == 0:
        return cat
    ns = n_streams or len(ir.streams)
    table = (rank_table(ir) if table is None else table).to(dev)
    seq_ref = min(int(c["seq"].min()) for c in per_rank if c["seq"].numel())
    keys, timers = zip(*(merge_keys(c, table, ns, stream_log, seq_ref) for c in per_rank))
    if not any(bool(t.any()) for t in timers):
        pos = torch.cat(merge_order(keys))
        perm = torch.empty_like(pos)
        perm[pos] = torch.arange(n, dtype=torch.int64, device=dev)
    else:  # LSD passes of a stable sort: key, query, tb (timer rows only), then the primary key
        key = torch.cat(keys)
        timer = torch.cat(timers)
        zero = torch.zeros_like(key)
        perm = torch.arange(n, dtype=torch.int64, device=dev)
        for k in (torch.where(timer, cat["key"], zero), torch.where(timer, cat["q"], zero),
                  torch.where(timer, cat["tb"], zero), key):
            perm = perm[torch.sort(k[perm], stable=True).indices]
    out = {f: cat[f][perm] for f in ("q", "key", "ts", "seq", "tb", "len")}
    starts = torch.cumsum(cat["len"], 0) - cat["len"]
    lens = out["len"]
    new_off = torch.cumsum(lens, 0) - lens
    src = torch.repeat_interleave(starts[perm] - new_off, lens) + torch.arange(int(lens.sum()), device=dev)
    out["words"] = cat["words"][src]
    return out


def columns_to_tuples(cols) -> List[tuple]:
    """(query, key, ts, slots) tuples (the harness' match form) from columns (n_slots from the words)."""
    q, k, ts, lens, words = (cols[f].cpu().tolist() for f in ("q", "key", "ts", "len", "words"))
    out, o = [], 0
    for i in range(len(q)):
        w = words[o:o + lens[i]]
        o += lens[i]
        slots, j = [], 0
        while j < len(w):
            c = w[j]
            slots.append(tuple(w[j + 1:j + 1 + c]))
            j += 1 + c
        out.append((q[i], k[i], ts[i], tuple(slots)))
    return out


_hip_lib = None


def _hip():
    global _hip_lib
    if _hip_lib is None:
        _hip_lib = ctypes.CDLL("libamdhip64.so")
        _hip_lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return _hip_lib


def _d2d(hip, dst: int, src_ptr, nbytes: int):
    src = ctypes.cast(src_ptr, ctypes.c_void_p).value
    if hip.hipMemcpy(dst, src, nbytes, 3) != 0:  # hipMemcpyDeviceToDevice
        raise RuntimeError("hipMemcpy device-to-device failed")
