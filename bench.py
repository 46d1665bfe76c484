#!/usr/bin/env python3
"""NFA-step throughput benchmark (BASELINE.json metric: events/s x active patterns, at 10K patterns).

Workload (default; BASELINE.json configs[1] at the metric's 10K patterns, SURVEY §8(d) C2 family):
P = 10,000 concurrent 2-state patterns per GPU
    every e1=StockStream[price > T_p] -> e2=StockStream[price > e1.price] within W_p
over the seeded synthetic StockStream (20 B/event SoA), generated on the device and resident in HBM
before the timed region. One step = one NFA-step pass (one sdh_engine_push) over a batch of B = 8M
events; every match record is written to HBM (SDH_FLAG_DEVICE_MATCHES: counted, not polled).
`--workload c3 | c4 | c5` runs the count/logical partitioned family, one GPU's shard of the fraud
sequences, or the C5 family (four joined streams, mixed 2-4-state patterns under one `partition with`
key, `within 1 hour`; one step = one batch per stream; reduced pattern / key counts)
instead.

Match expansion (`expansion` in the JSON line): a second engine in normal mode runs pushes of a
smaller batch followed by sdh_engine_poll_device -- the device R18 sort and the gather of the ABI
tuples (query, key, ts, off, words) in HBM -- and times both.

Multi-GPU (torchrun, one process per GPU): weak scaling by pattern set -- rank r runs patterns
r*P .. r*P+P-1 of the family. Rank 0 generates each batch and broadcasts it over RCCL (the event
broadcast of SURVEY §8(e)) inside the timed region; match counts are all-reduced. Timing: barrier +
device sync on both sides of the K timed steps, max over ranks.
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

DEFAULTS = {  # workload -> (patterns per GPU, events per step, keys)
    "c2": (10000, 1 << 23, 100),
    "c3": (1000, 1 << 20, 10000),
    "c4": (1250, 1 << 20, 100_000),
    "c5": (100_000, 1 << 16, 125_000),  # patterns, events per stream per GPU per step, accounts per GPU
}
C5_NODE = 8  # BASELINE configs[4] is one 8-GPU node: every rank is one of 8 key shards of 1M accounts


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=list(DEFAULTS), default="c2",
                    help="c2: BASELINE configs[1] at 10K patterns (headline); c3: configs[2] (count/logical, "
                         "partitioned); c4: configs[3] (fraud-rule sequences, one GPU's pattern-set shard)")
    ap.add_argument("--keys", type=int, default=0, help="partition keys / symbols (default per workload)")
    ap.add_argument("--patterns", type=int, default=0, help="patterns per GPU (default per workload)")
    ap.add_argument("--batch", type=int, default=0, help="events per step (default per workload; C2: 12 steps x 8M = 1.0e8 timed events)")
    ap.add_argument("--partials", type=int, default=128)
    ap.add_argument("--expansion-batch", type=int, default=1 << 16)
    ap.add_argument("--no-expansion", action="store_true")
    ap.add_argument("--no-ingest", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def app_source(workload, P, first):
    from siddhi_amd.workloads import c2_app, c3_app, c4_app, c5_app
    return {"c2": c2_app, "c3": c3_app, "c4": c4_app, "c5": c5_app}[workload](P, first=first)


def make_engine(workload, P, first, K, device, flags, partials, shard=(0, 1)):
    from siddhi_amd import ql
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.planner import plan
    blob = plan(ql.parse(app_source(workload, P, first))).serialize()
    if workload == "c4":
        # a sequence instance holds at most one partial per state (R8): small pools
        return HipEngine(blob, device=device, flags=flags, gen_pool_states=8, gen_pool_nodes=32, gen_list_cap=8)
    if workload == "c5":  # key sharding: every rank runs all patterns over its own accounts (K_slab)
        return HipEngine(blob, device=device, flags=flags, gen_max_keys=max(1024, 2 * K), shard_rank=shard[0],
                         shard_world=shard[1])
    if workload == "c3":
        pools = [int(x) for x in os.environ.get("SDH_C3_POOLS", "32,128,32").split(",")]
        return HipEngine(blob, device=device, flags=flags, gen_pool_states=pools[0], gen_pool_nodes=pools[1],
                         gen_list_cap=pools[2], gen_max_keys=max(1024, 2 * K))
    return HipEngine(blob, device=device, partials=partials, flags=flags)


def gen_batch(workload, start, n, K, dev):
    from siddhi_amd.workloads import c5_events_torch, stock_events_torch, txn_events_torch
    if workload == "c5":  # one batch per stream: [(ts, acct, amount bits, code)] x 4
        import torch
        out = []
        for si in range(4):
            ts, a, b, c = c5_events_torch(si, start, n, K, dev)
            out.append([ts, a, b.view(torch.int32), c])
        return out
    gen = txn_events_torch if workload == "c4" else stock_events_torch
    ts, a, b, c = gen(start, n, K, dev)
    return [ts, a, b.view(__import__("torch").int32), c]


def cpu_cores():
    """Cores this job may use: the affinity mask, capped by a cgroup CPU quota (the GPU box gives one
    GPU's job a share of the host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


def _oracle_shard(workload, shard, P, n_symbols, budget_s):
    """One CPU thread: the oracle on patterns shard*P .. shard*P+P-1 over consecutive batches of the
    stream until the time budget is spent. Matches are counted and dropped inside the library (no
    Python decoding), and ctypes releases the GIL, so shards run in parallel."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from harness import App
    from siddhi_amd.workloads import stock_events, txn_events
    from siddhi_amd.workloads import c5_events
    app = App(app_source(workload, P, shard * P))
    lib, h = app.engine.lib, app.engine.h
    gen = txn_events if workload == "c4" else stock_events
    done, start, n, matches = 0, 0, 20000, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        for si in range(4 if workload == "c5" else 1):  # C5: one batch per stream
            ts, sym, price, vol = c5_events(si, start, n, n_symbols) if workload == "c5" else gen(start, n, n_symbols)
            vals = np.stack([sym.astype(np.int64), price.view(np.uint32).astype(np.int64),
                             vol.astype(np.int64)], 1)
            app.engine.send(si, ts, vals, None)
            matches += lib.oracle_num_matches(h)
            lib.oracle_clear_matches(h)
            done += n
        start += n
    live = lib.oracle_live_partials(h)
    return done, time.perf_counter() - t0, matches, live


def cpu_baseline(workload, n_symbols, budget_s):
    """Reference-semantics C++ CPU engine (the oracle) on the host cores, on a
    bounded sample of the same workload: one thread, then N threads sharded by pattern set
    (N = the cores this job may use), 32 patterns per thread."""
    from concurrent.futures import ThreadPoolExecutor
    P = 32
    d1, t1, m1, _ = _oracle_shard(workload, 0, P, n_symbols, budget_s / 2)
    N = cpu_cores()
    with ThreadPoolExecutor(N) as ex:
        res = list(ex.map(lambda r: _oracle_shard(workload, r, P, n_symbols, budget_s / 2), range(N)))
    tn = max(r[1] for r in res)
    total = sum(r[0] for r in res) * P
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": total / tn, "unit": "pattern-events/s", "cores": N, "kind": "port",
            "single_thread_value": d1 * P / t1, "matches_per_s": sum(r[2] for r in res) / tn,
            "live_partials": int(sum(r[3] for r in res)), "host_cpus": os.cpu_count(), "cpu_model": model,
            "sample": f"{N} threads x {P} {workload.upper()} patterns (pattern-set shards, patterns 0..{N * P - 1}) "
                      f"over consecutive 20K-event batches for {budget_s / 2:.0f} s; 1 thread: {P} patterns x "
                      f"{d1} events (oracle/liboracle.so, matches counted in the library)"}


KERNEL_SOURCES = {  # what a kernel's code and launch configuration are built from
    "nfa_ratchet_kernel": ["nfa_ratchet.hip", "nfa_types.h", "engine.hip"],
    "nfa_gen_kernel": ["nfa_gen.hip", "kgen.h", "gen_lower.h", "nfa_types.h", "engine.hip"],
    "nfa_seq_kernel": ["nfa_gen.hip", "seq_body.h", "dev_common.h", "kgen.h", "gen_lower.h", "nfa_types.h",
                       "engine.hip"],
    "nfa_part_kernel": ["nfa_part.hip", "part_body.h", "dev_common.h", "kgen.h", "gen_lower.h", "nfa_types.h",
                        "engine.hip"],
    # shape-compiled kernels (spec.hip generates and compiles them with hiprtc at engine creation)
    "sdh_part_spec": ["spec.hip", "part_body.h", "dev_common.h", "kgen.h", "gen_lower.h", "nfa_types.h", "engine.hip"],
    "sdh_seq_spec": ["spec.hip", "seq_body.h", "dev_common.h", "kgen.h", "gen_lower.h", "nfa_types.h", "engine.hip"],
    "nfa_slab_kernel": ["nfa_slab.hip", "slab.h", "slab_lower.h", "dev_common.h", "kgen.h", "gen_lower.h",
                        "nfa_types.h", "engine.hip"],
}


def source_hash(kernel=None):
    """Hash of the sources `kernel` is built from (all kernel sources when None); a committed profile
    is attached to the bench line only at an equal hash."""
    names = KERNEL_SOURCES.get(kernel) or sorted({f for v in KERNEL_SOURCES.values() for f in v})
    h = hashlib.sha256()
    for name in names:
        f = os.path.join(ROOT, "siddhi_amd", "csrc", name)
        if os.path.exists(f):
            h.update(name.encode())
            h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def profiled(kernel, workload, patterns, batch):
    """The committed rocprofv3 profile of this same command at these sources (profiles/*/meta.json):
    HBM bytes per launch of `kernel` (FETCH_SIZE x2 gfx950 streaming-read correction + WRITE_SIZE,
    KiB) and the counter-derived issue / LDS figures."""
    src = source_hash(kernel)
    for meta_f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "meta.json"))):
        try:
            meta = json.load(open(meta_f))
        except (OSError, ValueError):
            continue
        if (meta.get("source_hash") != src or meta.get("workload") != workload or
                meta.get("patterns") != patterns or meta.get("batch") != batch):
            continue
        k = meta.get("kernels", {}).get(kernel)
        if k:
            return k, os.path.relpath(os.path.dirname(meta_f), ROOT)
    return None, None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # rehearsal knobs for a 1-GPU box (not used by the driver): every rank on one device, gloo
    backend = os.environ.get("SDH_BENCH_BACKEND", "nccl")
    if "SDH_BENCH_DEVICE" in os.environ:
        local = int(os.environ["SDH_BENCH_DEVICE"])
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # where the collectives run

    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES

    P0, B0, K0 = DEFAULTS[args.workload]
    P = args.patterns or P0
    B = args.batch or B0
    K = args.keys or K0
    c5 = args.workload == "c5"
    if c5:  # key sharding (weak scaling): rank r is shard r of the 8-GPU node's 1M accounts; every step
        # each stream carries the node's B * 8 events (generated by rank 0, broadcast) and a rank
        # evaluates the ~B of them whose account it owns against all P patterns
        if world > C5_NODE:
            raise SystemExit(f"--workload c5 models one {C5_NODE}-GPU node")
        t_build = time.perf_counter()
        eng = make_engine("c5", P, 0, K, local, SDH_FLAG_DEVICE_MATCHES, args.partials, shard=(rank, C5_NODE))
        t_build = time.perf_counter() - t_build
        B, K_gen = B * C5_NODE, K * C5_NODE
        # `within 1 hour` of event time: the untimed warm-up covers an hour (the state's steady size)
        args.warmup = max(args.warmup, -(-3_600_000 // B) + 1)
        args.no_expansion = args.no_ingest = True  # (single-stream helpers)
    else:
        eng = make_engine(args.workload, P, rank * P, K, local, SDH_FLAG_DEVICE_MATCHES, args.partials)
        K_gen = K

    n_batches = args.warmup + args.steps
    # synthetic batches generated on the device before the timed region (rank 0's copy is the
    # broadcast source in multi-GPU runs; the other ranks receive into their own buffers)
    batches = [gen_batch(args.workload, s * B, B, K_gen, dev) for s in range(n_batches)] if not c5 else None
    torch.cuda.synchronize()
    bcast = world > 1

    def bcast_into(t):
        if backend == "nccl":
            dist.broadcast(t, src=0)
        else:  # gloo rehearsal: the collective runs on a host copy, received back into t
            tc = t.cpu()
            dist.broadcast(tc, src=0)
            t.copy_(tc)

    if c5:
        # rank 0's batches of the timed steps are generated before the timed region; the other
        # ranks receive them into zeroed buffers (a missing broadcast shows as wrong matches)
        def c5_batch(i):
            cols = gen_batch("c5", i * B, B, K_gen, dev)
            return cols if rank == 0 or not bcast else [[torch.zeros_like(t) for t in c] for c in cols]
        c5_pre = [c5_batch(i) for i in range(args.warmup, n_batches)]

    def step(i):
        """One step: every stream's batch pushed once; returns (kernel ms, algorithmic bytes, matches)
        summed over the step's pushes."""
        per_stream = ((c5_batch(i) if i < args.warmup else c5_pre[i - args.warmup]) if c5 else [batches[i]])
        ms = by = 0.0
        nm = 0
        for si, cols in enumerate(per_stream):
            if bcast:
                for t in cols:
                    bcast_into(t)
            eng.push_device(si, B, cols[0].data_ptr(), [c.data_ptr() for c in cols[1:]])
            if len(per_stream) > 1 or i >= args.warmup:
                st = eng.stats()
                ms += st.last_kernel_ms
                by += st.last_kernel_bytes
                nm += eng.pending_matches()
        return ms, by, nm

    for i in range(args.warmup):
        step(i)
    kern_ms, kern_bytes, matches = [], [], 0
    pe0 = eng.stats().pattern_events
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, n_batches):
        ms, by, nm = step(i)
        kern_ms.append(ms)
        kern_bytes.append(by)
        matches += nm
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    live = eng.stats().live_partials
    # C5: (event, pattern) evaluations the engine performed (each rank's own accounts' events
    # against the patterns reading their stream)
    pe = float(eng.stats().pattern_events - pe0)
    if world > 1:
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        mt = torch.tensor([matches, live, pe], device=cdev, dtype=torch.float64)
        dist.all_reduce(mt)
        matches, live, pe = int(mt[0].item()), int(mt[1].item()), float(mt[2].item())
    del batches

    total_pe = pe if c5 else float(B) * args.steps * P * world
    value = total_pe / elapsed
    avg_ms = float(np.mean(kern_ms))
    avg_bytes = float(np.mean(kern_bytes))
    achieved = avg_bytes / (avg_ms * 1e-3) / 1e9
    peak = 8000.0
    if args.workload == "c2":
        wl = (f"C2 at the metric's 10K patterns: {P} concurrent 2-state filter+reference patterns per GPU "
              "(every e1[price>T_p] -> e2[price>e1.price] within W_p)")
        kernel = "nfa_ratchet_kernel"
    elif args.workload == "c3":
        wl = (f"C3: count <2:5> + logical and/or patterns, partition with (symbol) over {K} keys, "
              "within 10 sec")
        kernel = "sdh_part_spec"
    elif c5:
        wl = (f"C5: {P} mixed 2-4-state patterns (cross-stream reference, and, or, count) over 4 joined streams, "
              f"partition with (acct) over {K * C5_NODE} accounts, within 1 hour; this GPU is key shard(s) "
              f"{list(range(world))} of {C5_NODE} ({K} accounts each); {B} node events per stream per step")
        kernel = "nfa_slab_kernel"
    else:
        wl = ("C4: fraud-rule sequences every e1=Txn[..], e2=Txn[..e1.amount*M], e3=Txn[..] within 1 min "
              f"(strict contiguity), {K} accounts, pattern-set shard {rank * P}..{rank * P + P - 1}")
        kernel = "sdh_seq_spec"
    prof, prof_dir = profiled(kernel, args.workload, P, B)
    traffic = prof.get("traffic_bytes") if prof else None
    result = {
        "metric": "events/sec x active patterns (whole node) at 10K patterns; achieved HBM GB/s",
        "value": value,
        "unit": "pattern-events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded splitmix64 StockStream / Txn stream, SURVEY §8(d)), generated in HBM",
        "config": {"workload": wl, "patterns_per_gpu": P, "events_per_step": B * (4 if c5 else 1),
                   "timed_events": B * args.steps * (4 if c5 else 1),
                   "keys": K, "parallelism": (f"key shards x{world}" if c5 else f"pattern-set x{world}") +
                   (" (RCCL event broadcast)" if bcast else ""),
                   "matches": matches, "matches_per_s": matches / elapsed, "live_partials": live,
                   "source_hash": source_hash(kernel)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": traffic, "traffic_source": prof_dir,
                     "kernel": kernel, "kernel_ms": avg_ms,
                     # measured HBM rate (PMC traffic / live kernel time); below `achieved` when the
                     # device record is narrower than §8(d)'s 32-B match unit
                     # measured HBM rate: PMC bytes per launch / the profile's average launch time
                     "traffic_gbps": (traffic / (prof["kernel_ns_avg"] * 1e-9) / 1e9) if traffic else None},
    }
    if prof:
        result["roofline"]["counters"] = {k: v for k, v in prof.items() if k != "traffic_bytes"}
    if c5:  # the sparse state (K_slab): bytes per live partial, engine build time
        lb, rb, db = eng.state_bytes()
        result["config"].update({"state_live_bytes": lb, "state_slab_bytes": rb, "state_dir_bytes": db,
                                 "bytes_per_live_partial": (lb + db) / max(1, live),
                                 "engine_build_s": t_build, "warmup_event_hours": args.warmup * B / 3.6e6})
    if not args.no_expansion:
        result["expansion"] = expansion(args, P, rank, K, local, dev, world, cdev, dist)
    if not args.no_ingest and world == 1:
        result["host_ingest"] = host_ingest(args, eng, B, K, n_batches)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.workload, K, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_ingest(args, eng, B, K, first_step):
    """The same pushes with the batch in pinned HOST memory (sdh_batch.on_device = 0): the side-stream
    copy to HBM is inside the step (PCIe-inclusive rate), continuing the stream."""
    import torch
    steps = 2
    rows = []
    for s in range(steps):
        cols = gen_batch(args.workload, (first_step + s) * B, B, K, torch.device("cuda"))
        rows.append([c.cpu().pin_memory() for c in cols])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ing = 0.0
    for cols in rows:
        eng.push_columns(0, cols[0].numpy(), [c.numpy() for c in cols[1:]])
        ing += eng.stats().last_ingest_ms
    el = time.perf_counter() - t0
    nbytes = sum(c.numel() * c.element_size() for c in rows[0])
    return {"events_per_step": B, "steps": steps, "ms_per_step": el * 1e3 / steps, "h2d_ms_per_step": ing / steps,
            "h2d_gbps": nbytes / (ing / steps * 1e-3) / 1e9 if ing else None,
            "pattern_events_per_s": B * steps * eng_patterns(eng) / el}


def eng_patterns(eng):
    st = eng.stats()
    return st.pattern_events / max(1, st.events)


def expansion(args, P, rank, K, local, dev, world, cdev, dist):
    """Pushes of a smaller batch in normal mode, each followed by sdh_engine_poll_device (device R18
    sort + gather of the ABI tuples in HBM): the NFA step with every match expanded. With N GPUs the
    R18-sorted tuples are then gathered to rank 0 over RCCL and merged there (siddhi_amd/dist.py)."""
    import torch
    from siddhi_amd import dist as sdist
    # with N GPUs every rank's tuples are gathered to rank 0: at 10K patterns per rank a 64K-event
    # batch is ~280M matches per rank, so the multi-GPU gather runs on 2K-event batches
    E = args.expansion_batch if world == 1 else min(args.expansion_batch, 2048)
    eng = make_engine(args.workload, P, rank * P, K, local, 0, args.partials)
    steps, warm = 4, 1
    bs = [gen_batch(args.workload, s * E, E, K, dev) for s in range(steps + warm)]
    log = sdist.StreamLog()
    table = torch.arange(P * world, dtype=torch.int64)  # one stream, queries in definition order
    torch.cuda.synchronize()
    push_ms, gather_ms, matches, merged = 0.0, 0.0, 0, 0
    for i, cols in enumerate(bs):
        if i == warm:
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        t1 = time.perf_counter()
        eng.push_device(0, E, cols[0].data_ptr(), [c.data_ptr() for c in cols[1:]])
        log.push(0, E)
        t2 = time.perf_counter()
        if world > 1 and args.workload == "c2":
            mc = sdist.columns_from_device(eng, dev)
            mc["q"] += rank * P  # this rank's sub-app numbers its queries from 0
            if cdev.type != "cuda":  # gloo rehearsal: the collectives take host tensors
                mc = {k: v.to(cdev) for k, v in mc.items()}
            t3 = time.perf_counter()
            per_rank = sdist.gather_columns(mc)
            if rank == 0:
                out = sdist.merge_columns(None, per_rank, log, table=table, n_streams=1)
                merged += int(out["q"].numel())
            torch.cuda.synchronize()
            n_local = int(mc["q"].numel())
            t4 = time.perf_counter()
        else:
            n_local = eng.poll_device().n
            t3 = t4 = time.perf_counter()
        if i >= warm:
            push_ms += (t2 - t1) * 1e3
            gather_ms += (t4 - t3) * 1e3
            matches += n_local
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el, matches], device=cdev, dtype=torch.float64)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        mt = t[1:].clone()
        dist.all_reduce(mt)
        el, matches = float(t[0].item()), int(mt.item())
    eng.close()
    r = {"events_per_step": E, "steps": steps, "ms_per_step": el * 1e3 / steps,
         "push_ms_per_step": push_ms / steps, "matches_per_step": matches / steps,
         "pattern_events_per_s": E * steps * P * world / el, "matches_per_s": matches / el}
    if world > 1 and args.workload == "c2":
        r["rccl_gather_merge_ms_per_step"] = gather_ms / steps
        r["merged_matches_per_step_rank0"] = merged / steps
    return r


if __name__ == "__main__":
    main()
