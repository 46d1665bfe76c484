#!/usr/bin/env python3
"""NFA-step throughput benchmark (BASELINE.json metric: events/s x active patterns, whole node, at 10K
patterns).

Workload (default; BASELINE.json configs[1] at the metric's 10K patterns, SURVEY §8(d) C2 family):
P = 10,000 concurrent 2-state patterns in total
    every e1=StockStream[price > T_p] -> e2=StockStream[price > e1.price] within W_p
over the seeded synthetic StockStream (20 B/event SoA), generated on the device and resident in HBM
before the timed region. One step = one NFA-step pass (one sdh_engine_push per GPU) over a batch of
B = 8M events; every match is written to HBM as a device record (SDH_FLAG_DEVICE_MATCHES) and handed
out by sdh_engine_poll_records after each push (include/siddhi_hip.h documents the formats; a device
consumer reads them there -- tests/test_gpu_records.py decodes them). The NFA step's output is
therefore consumable, not discarded; the R18-ordered delivery is the `expansion` leg's figure.
`--workload c3 | c4 | c5` runs the count/logical partitioned family (1000 patterns x 10K keys), the
10K fraud-rule sequences, or the C5 family (100K mixed patterns over four joined streams under one
`partition with` key, `within 1 hour`; one step = one batch per stream; one GPU = one of the 8-GPU
node's key shards).

Multi-GPU: one process per GPU. `bench.py --gpus N` started without WORLD_SIZE launches its N ranks
itself (torch.distributed.run on 127.0.0.1, before any GPU call in the parent) and exits with their
status; under torchrun WORLD_SIZE must equal N. Fewer than N visible GPUs, or WORLD_SIZE != N, fail
non-zero (never a silent single-rank run). `--scaling strong` (default) measures the metric as
defined, the whole node at 10K patterns: every rank's engine runs the full program as its shard
(sdh_config.shard_rank / shard_world): the P patterns split by pattern set (rank r runs patterns r,
r+N, ...; c3: the partition keys are split instead, rank r owning |String.valueOf(key).hashCode() % N|
== r). `--scaling weak` gives every GPU P patterns of its own; a strong N>1 run appends that as a
second line (`weak_scaling`). The exchange is the library's (include/siddhi_hip.h): an RCCL
communicator (sdh_comm_create, its id handed out over torch.distributed's gloo control plane), rank
0's device batch broadcast to every rank by sdh_engine_push_bcast inside the timed region.
torch.distributed (gloo) carries only control: barriers, the max over ranks, the communicator id.
`value` = pattern-events summed over ranks / the max over ranks of the timed region (barrier + device
sync on both sides).

Match expansion (`expansion` in the JSON line): a second engine in normal mode runs pushes of a
smaller batch followed by sdh_engine_poll_device -- the device R18 sort and the gather of the ABI
tuples (query, key, ts, off, words) in HBM; with N GPUs sdh_engine_gather instead: every rank's
R18-ordered tuples go to rank 0 over RCCL and are merged there on the device, timed per step.
"""
import argparse
import glob
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

DEFAULTS = {  # workload -> (patterns, events per step, keys); patterns are the node total under strong
    # scaling and per GPU under weak scaling (c5: always per GPU, one of the 8-GPU node's key shards)
    "c2": (10000, 1 << 23, 100),
    "c2x": (10000, 1 << 22, 100),  # the C2 family with an event-only conjunct on e2 (workloads.c2x_app)
    "c3": (1000, 1 << 20, 10000),
    "c4": (10000, 1 << 20, 100_000),
    "c5": (100_000, 1 << 16, 125_000),  # patterns, events per stream per GPU per step, accounts per GPU
}
C5_NODE = 8  # BASELINE configs[4] is one 8-GPU node: every rank is one of 8 key shards of 1M accounts


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=list(DEFAULTS), default="c2",
                    help="c2: BASELINE configs[1] at the metric's 10K patterns (headline); c2x: the same family "
                         "with an event-only conjunct on e2 (off K_ratchet's plan); c3: configs[2] "
                         "(count/logical, partitioned); c4: configs[3] (10K fraud-rule sequences); c5: configs[4]")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong (default): the workload's patterns (c3: keys) are split over the N GPUs -- "
                         "the metric's 'whole node at 10K patterns'; weak: every GPU runs that many patterns")
    ap.add_argument("--no-weak-leg", action="store_true", help="N>1 strong runs: skip the weak-scaling line")
    ap.add_argument("--keys", type=int, default=0, help="partition keys / symbols (default per workload)")
    ap.add_argument("--patterns", type=int, default=0, help="patterns (default per workload)")
    ap.add_argument("--batch", type=int, default=0, help="events per step (default per workload; C2: 12 steps x 8M = 1.0e8 timed events)")
    ap.add_argument("--partials", type=int, default=128)
    ap.add_argument("--expansion-batch", type=int, default=1 << 16)
    ap.add_argument("--no-expansion", action="store_true")
    ap.add_argument("--no-ingest", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip the small-push latency leg")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU-baseline sample budget")
    ap.add_argument("--state-reserve-gb", type=float, default=140.0,
                    help="c5: HBM reserved up front for the sparse K_slab state (sdh_engine_reserve): the state "
                         "grows inside it with no device allocation during the run (the shard's steady state: "
                         "~72 GB live in ~125 GB of rings)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-calibrate", action="store_true", help="skip the HBM copy / read ceiling measurement")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch check: every rank prints {rank, local_rank, world_size} and exits (no GPU)")
    return ap.parse_args()


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` without WORLD_SIZE: start the N ranks (torch.distributed.run, one process per GPU) as
    child processes and return their exit status; None when this process is a rank itself. Nothing
    here touches the GPU (torch.cuda.device_count() counts devices without initialising HIP)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}")
        return None
    if args.gpus <= 1:
        return None
    if not args.dry_run:
        import torch
        n = torch.cuda.device_count()
        if n < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but {n} GPU(s) visible")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd)


def app_source(workload, n, first, step=1):
    from siddhi_amd.workloads import c2_app, c2x_app, c3_app, c4_app, c5_app
    return {"c2": c2_app, "c2x": c2x_app, "c3": c3_app, "c4": c4_app, "c5": c5_app}[workload](n, first=first, step=step)


class Shard:
    """This rank's share of a workload. The engine compiles patterns first, first+step, ... (n_prog of
    them) and runs the shard (rank, world) of that program (sdh_config.shard_rank / shard_world):
    patterns q % world == rank, and partition keys with |String.valueOf(key).hashCode() % world| ==
    rank. `n` = the patterns this GPU evaluates."""

    def __init__(self, workload, scaling, P, rank, world):
        self.keyed = (workload == "c5") or (workload == "c3" and scaling == "strong")
        self.first, self.step, self.n_prog = 0, 1, P
        if workload == "c5":
            self.n, self.key_shard = P, (rank, C5_NODE)
        elif scaling == "weak":
            self.first, self.n, self.key_shard = rank * P, P, (0, 1)
        elif workload == "c3":
            self.n, self.key_shard = P, (rank, world)
        else:  # pattern-set sharding by the engine's rule (strided: balances the threshold mix)
            self.n, self.key_shard = len(range(rank, P, world)), (rank, world)


def make_engine(workload, sh, K, device, flags, partials):
    from siddhi_amd import ql
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.planner import plan
    blob = plan(ql.parse(app_source(workload, sh.n_prog, sh.first, sh.step))).serialize()
    kr, kw = sh.key_shard
    if workload == "c4":
        # a sequence instance holds at most one partial per state (R8): small pools
        return HipEngine(blob, device=device, flags=flags, gen_pool_states=8, gen_pool_nodes=32, gen_list_cap=8,
                         shard_rank=kr, shard_world=kw)
    if workload == "c5":  # key sharding: every rank runs all patterns over its own accounts (K_slab)
        return HipEngine(blob, device=device, flags=flags, gen_max_keys=max(1024, 2 * K), shard_rank=kr,
                         shard_world=kw)
    if workload == "c3":
        pools = [int(x) for x in os.environ.get("SDH_C3_POOLS", "32,128,32").split(",")]
        return HipEngine(blob, device=device, flags=flags, gen_pool_states=pools[0], gen_pool_nodes=pools[1],
                         gen_list_cap=pools[2], gen_max_keys=max(1024, 2 * K), shard_rank=kr, shard_world=kw)
    return HipEngine(blob, device=device, partials=partials, flags=flags, shard_rank=kr, shard_world=kw)


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


T_START = time.time()


def log(msg):
    """progress on stderr (the JSON line stays alone on stdout)"""
    print(f"[bench {time.time() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


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


KERNEL_OF_PLAN = {"c2x": "nfa_gate_kernel"}  # workload -> the kernel its plan launches

KERNEL_SOURCES = {  # what a kernel's code and launch configuration are built from
    "nfa_chain_kernel": ["nfa_chain.hip", "nfa_types.h", "engine.hip"],
    "nfa_ratchet_kernel": ["nfa_ratchet.hip", "ratchet_common.h", "nfa_types.h", "engine.hip"],
    "nfa_gate_kernel": ["nfa_gate.hip", "ratchet_common.h", "nfa_types.h", "engine.hip"],
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


def build_provenance():
    """The source hash the loaded libsiddhi_hip.so was built from (sdh_build_info) against the hash of
    the tree's sources (siddhi_amd/csrc/src_hash.py): equal when the library matches this tree."""
    from siddhi_amd.engine import load_library
    sys.path.insert(0, os.path.join(ROOT, "siddhi_amd", "csrc"))
    from src_hash import src_hash
    info = load_library().sdh_build_info().decode()
    tree = src_hash(os.path.join(ROOT, "siddhi_amd", "csrc"))
    return {"lib": info, "tree_src_hash": tree, "lib_matches_tree": info.split()[1] == tree}


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


def timed_steps(eng, step, warmup, steps, world, dist):
    """W untimed steps, then K timed ones bracketed by barrier + device sync; returns (elapsed max over
    ranks, per-step kernel ms, per-step algorithmic bytes, matches, pattern-events summed over ranks)."""
    import torch
    for i in range(warmup):
        t = time.perf_counter()
        step(i)
        dt = time.perf_counter() - t
        mem = ""
        if torch.cuda.is_available():
            free, total = torch.cuda.mem_get_info()
            mem = f", HBM used {(total - free) / 1e9:.1f} GB"
            lb, rb, db = eng.state_bytes()
            if rb:
                mem += f" (slab live {lb / 1e9:.1f} GB, reserved {rb / 1e9:.1f} GB, directory {db / 1e9:.1f} GB)"
        log(f"warm-up step {i + 1}/{warmup}: {dt * 1e3:.1f} ms, last kernel "
            f"{eng.stats().last_kernel_ms:.1f} ms{mem}")
    kern_ms, kern_bytes, rec_bytes, matches = [], [], [], 0
    pe0 = eng.stats().pattern_events
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_wall = []  # (host clock per step call: a push returns once its step is done)
    for i in range(warmup, warmup + steps):
        ts = time.perf_counter()
        ms, by, nm, rb = step(i)
        step_wall.append((time.perf_counter() - ts) * 1e3)
        kern_ms.append(ms)
        kern_bytes.append(by)
        rec_bytes.append(rb)
        matches += nm
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    mem = ""
    if torch.cuda.is_available():
        free, total = torch.cuda.mem_get_info()
        lb, rb, db = eng.state_bytes()
        mem = f", HBM used {(total - free) / 1e9:.1f} GB" + (f" (slab live {lb / 1e9:.1f} GB, reserved {rb / 1e9:.1f} GB)" if rb else "")
    sw = sorted(step_wall)
    log(f"{steps} timed steps: {elapsed * 1e3 / steps:.2f} ms/step{mem}; per step: median "
        f"{sw[len(sw) // 2]:.1f} ms, max {sw[-1]:.1f} ms")
    # (event, pattern) evaluations the engine performed: B x patterns for pattern-set shards, each
    # rank's own keys' events x patterns for key shards (sdh_stats.pattern_events)
    pe = float(eng.stats().pattern_events - pe0)
    return elapsed, kern_ms, kern_bytes, rec_bytes, matches, pe


def reduce_run(elapsed, matches, pe, live, world, dist, cdev):
    import torch
    if world > 1:
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        mt = torch.tensor([matches, live, pe], device=cdev, dtype=torch.float64)
        dist.all_reduce(mt)
        matches, live, pe = int(mt[0].item()), int(mt[1].item()), float(mt[2].item())
    return elapsed, matches, pe, live


def launches_per_step(prof, prof_dir):
    """Launches of the profiled kernel per bench step: its rocprof call count over the pushes the
    profiled run made (warm-up included, as its own bench line recorded them in meta.json) plus the
    passes it re-ran (meta `reruns`: a push whose output or state outgrew its buffers is undone and
    launched again -- in the warm-up, as the buffers grow once), times the pushes per step (C5: one per
    stream). Older profiles: the recorded arguments, with bench.py's defaults and C5's forced warm-up."""
    if not prof:
        return 1
    try:
        meta = json.load(open(os.path.join(ROOT, prof_dir, "meta.json")))
        if meta.get("steps") is not None and meta.get("warmup") is not None:
            per = 4 if meta.get("workload") == "c5" else 1
            pushes = (int(meta["steps"]) + int(meta["warmup"])) * per
            return prof["calls"] * per / (pushes + int(meta.get("reruns", 0)))
        a = meta["bench_args"].split()
        steps = int(a[a.index("--steps") + 1]) if "--steps" in a else 12
        warm = int(a[a.index("--warmup") + 1]) if "--warmup" in a else 2
        if meta.get("workload") == "c5":
            warm = max(warm, -(-5_400_000 // meta["batch"]) + 1)  # (batch: node events per stream)
        return prof["calls"] / (steps + warm)
    except (OSError, ValueError, KeyError, IndexError):
        return 1


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        print(json.dumps({"rank": rank, "local_rank": local, "world_size": world, "gpus": args.gpus}), flush=True)
        return
    import torch
    if local >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local}, {torch.cuda.device_count()} visible")
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # control plane only (barriers, the max over ranks, the communicator id); the event broadcast
        # and the match gather run inside libsiddhi_hip.so over its own RCCL communicator
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu")  # where the control collectives run
    comm = None
    if world > 1:
        from siddhi_amd.engine import Comm
        uid = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm.rccl(uid[0], rank, world, local)

    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES

    P0, B0, K0 = DEFAULTS[args.workload]
    P = args.patterns or P0
    B = args.batch or B0
    K = args.keys or K0
    c5 = args.workload == "c5"
    scaling = "weak" if c5 else args.scaling
    sh = Shard(args.workload, scaling, P, rank, world)
    t_build = time.perf_counter()
    if c5:  # key sharding (weak scaling): rank r is shard r of the 8-GPU node's 1M accounts; every step
        # each stream carries the node's B * 8 events (generated by rank 0, broadcast) and a rank
        # evaluates the ~B of them whose account it owns against all P patterns
        if world > C5_NODE:
            raise SystemExit(f"--workload c5 models one {C5_NODE}-GPU node")
        B, K_gen = B * C5_NODE, K * C5_NODE
        # `within 1 hour` of event time: the untimed warm-up covers an hour and a half -- the hour of
        # partials plus the ones that expire lazily (at their key's next event) -- so the state and
        # its slab rings have reached their steady size when the timed steps start
        args.warmup = max(args.warmup, -(-5_400_000 // B) + 1)
        args.no_expansion = args.no_ingest = True  # (single-stream helpers)
    else:
        K_gen = K
    log(f"building the engine: {args.workload}, {sh.n} patterns on this GPU, {B} events per step")
    eng = make_engine(args.workload, sh, K, local, SDH_FLAG_DEVICE_MATCHES, args.partials)
    if comm is not None:
        eng.set_comm(comm)
    if c5 and args.state_reserve_gb > 0:
        eng.reserve(int(args.state_reserve_gb * 1e9))
    t_build = time.perf_counter() - t_build
    log(f"engine built in {t_build:.1f} s")

    n_batches = args.warmup + args.steps
    # synthetic batches generated on the device before the timed region; in multi-GPU runs only rank
    # 0 holds them (the broadcast source), the other ranks receive every batch through the library
    bcast = world > 1

    def local_batch(i):
        if bcast and rank != 0:
            return [None] * (4 if c5 else 1)
        cols = gen_batch(args.workload, i * B, B, K_gen, dev)
        return cols if c5 else [cols]

    pre = [local_batch(i) for i in range(args.warmup, n_batches)]
    torch.cuda.synchronize()

    def make_step(engine, batches):
        def step(i):
            """One step: every stream's batch pushed once (broadcast from rank 0 by the library in
            multi-GPU runs); returns (kernel ms, algorithmic bytes, matches) summed over the pushes."""
            if i < args.warmup:  # generated now (torch's stream): complete before the engine reads it
                per_stream = local_batch(i)
                torch.cuda.synchronize()
            else:
                per_stream = batches[i - args.warmup]
            ms = by = rb = 0.0
            nm = 0
            for si, cols in enumerate(per_stream):
                if not bcast:
                    engine.push_device(si, B, cols[0].data_ptr(), [c.data_ptr() for c in cols[1:]])
                elif rank == 0:
                    engine.push_bcast_device(si, B, cols[0].data_ptr(), [c.data_ptr() for c in cols[1:]], root=0)
                else:
                    engine.push_bcast_recv(root=0)
                # the push's device records go to their consumer (sdh_engine_poll_records: the
                # descriptor of the records in HBM; no device work)
                rec = engine.poll_records()
                if len(per_stream) > 1 or i >= args.warmup:
                    kms, kby = engine.push_stats()  # (no device work inside the timed steps)
                    ms += kms
                    by += kby
                    nm += rec.n
                    rb += rec.r_bytes + 8.0 * rec.f_words + 8.0 * rec.c_n * rec.c_words
            return ms, by, nm, rb
        return step

    elapsed, kern_ms, kern_bytes, rec_bytes, matches, pe = timed_steps(eng, make_step(eng, pre), args.warmup,
                                                                      args.steps, world, dist)
    live = eng.stats().live_partials
    elapsed, matches, pe, live = reduce_run(elapsed, matches, pe, live, world, dist, cdev)
    value = pe / elapsed
    avg_ms = float(np.mean(kern_ms))
    avg_bytes = float(np.mean(kern_bytes))  # SURVEY §8(d) accounting bytes per step (32 B per match)
    avg_rec = float(np.mean(rec_bytes))      # record bytes the kernels wrote per step (device records)
    peak = 8000.0
    per_gpu = "per GPU" if scaling == "weak" else f"in total over {world} GPU(s)"
    if args.workload == "c2":
        wl = (f"C2 at the metric's 10K patterns: {P} concurrent 2-state filter+reference patterns {per_gpu} "
              "(every e1[price>T_p] -> e2[price>e1.price] within W_p)")
        kernel = "nfa_ratchet_kernel"
    elif args.workload == "c2x":
        wl = (f"C2x: {P} C2 patterns {per_gpu} with an event-only conjunct on e2 "
              "(every e1[price>T_p] -> e2[price>e1.price and volume>V_p] within W_p)")
        kernel = KERNEL_OF_PLAN.get("c2x", "nfa_chain_kernel")
    elif args.workload == "c3":
        wl = (f"C3: {P} count <2:5> + logical and/or patterns, partition with (symbol) over {K} keys, "
              f"within 10 sec; " + (f"key shards x{world}" if sh.keyed else f"{P} patterns per GPU"))
        kernel = "sdh_part_spec"
    elif c5:
        wl = (f"C5: {P} mixed 2-4-state patterns (cross-stream reference, and, or, count) over 4 joined streams, "
              f"partition with (acct) over {K * C5_NODE} accounts, within 1 hour; this GPU is key shard(s) "
              f"{list(range(world))} of {C5_NODE} ({K} accounts each); {B} node events per stream per step")
        kernel = "nfa_slab_kernel"
    else:
        wl = (f"C4: {P} fraud-rule sequences {per_gpu}: every e1=Txn[..], e2=Txn[..e1.amount*M], e3=Txn[..] "
              f"within 1 min (strict contiguity), {K} accounts")
        kernel = "sdh_seq_spec"
    prof, prof_dir = profiled(kernel, args.workload, sh.n, B)
    traffic = prof.get("traffic_bytes") if prof else None
    launches = launches_per_step(prof, prof_dir)
    # Roofline. `achieved` is what the memory system moved: the committed rocprofv3 PMC
    # bytes per launch of this kernel at these sources (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) x
    # launches per step, over this run's kernel time per step (HIP events on the engine's stream).
    # Without a matching profile it falls back to the design's minimum bytes and says so.
    m_step = matches / max(1, args.steps * world)
    design = None
    if args.workload in ("c2", "c2x"):
        # the design's own minimum per step: every 64-pattern group streams the batch's ts + price
        # (the start filter reads the same column) once, plus the record bytes the kernel wrote
        # (rec4: 4 B per match + 8 B per matching event and wave) -- §8(d)'s accounting less its 32 B
        # per match, plus the records as written
        design = avg_bytes - 32.0 * m_step + avg_rec
    if traffic:
        moved, source = traffic * launches, "pmc"
    else:
        moved, source = (design if design is not None else avg_bytes), ("design" if design is not None else "accounting_8d")
    achieved = moved / (avg_ms * 1e-3) / 1e9
    result = {
        "metric": "events/sec x active patterns (whole node) at 10K patterns; achieved HBM GB/s",
        "value": value,
        "unit": "pattern-events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded splitmix64 StockStream / Txn / C5 streams, SURVEY §8(d)), generated in HBM",
        "config": {"workload": wl, "patterns_total": P * (world if scaling == "weak" else 1),
                   "patterns_per_gpu": sh.n, "events_per_step": B * (4 if c5 else 1),
                   "timed_events": B * args.steps * (4 if c5 else 1),
                   "keys": K, "parallelism": (f"key shards x{world}" if sh.keyed else f"pattern-set x{world}") +
                   (" (RCCL event broadcast)" if bcast else ""),
                   "output": "device records, every match written and handed out per push (sdh_engine_poll_records)",
                   "matches": matches, "matches_per_s": matches / elapsed, "live_partials": live,
                   "record_bytes_per_step": avg_rec, "record_bytes_per_match": avg_rec / max(1.0, m_step),
                   "source_hash": source_hash(kernel)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "achieved_source": source,
                     "traffic": traffic, "traffic_source": prof_dir,
                     "kernel": kernel, "kernel_ms": avg_ms,
                     "launches_per_step": launches,
                     "traffic_per_step": traffic * launches if traffic else None,
                     # the profiled run's own rate (its PMC bytes over its own launch time)
                     "traffic_gbps_profiled": (traffic / (prof["kernel_ns_avg"] * 1e-9) / 1e9) if traffic else None,
                     # SURVEY §8(d)'s work accounting (32 B per match: the tuple the reference hands over),
                     # not bytes the device moves -- the device record is ~4.6 B
                     "accounting_8d": {"bytes_per_step": avg_bytes, "per_kernel_second_gbps": avg_bytes / (avg_ms * 1e-3) / 1e9}},
    }
    if design is not None:
        result["roofline"]["design_bytes_per_step"] = design
        result["roofline"]["frac_design"] = design / (avg_ms * 1e-3) / 1e9 / peak
    if prof:
        result["roofline"]["counters"] = {k: v for k, v in prof.items() if k != "traffic_bytes"}
        # issue roofline: the profile's wave-instructions per step of this run's pattern-events, at
        # this run's kernel rate, against the issue capacity at the profile's clock (a wave64 VALU op
        # holds a SIMD32 for 2 cycles, 1024 SIMDs; one scalar issue per CU and cycle, 256 CUs;
        # profiles/summarize.py). The profile normalises one launch's instructions by patterns x batch;
        # a step runs `launches` of them and evaluates pe / steps pattern-events (routed events only
        # for key shards)
        pe_step = pe / max(1, args.steps) / max(1, world)
        to_run = float(sh.n) * float(B) * launches / max(1.0, pe_step)
        pe_kernel = pe / max(1e-12, sum(kern_ms) * 1e-3) / max(1, world)  # per GPU, per kernel-second
        clk = prof["clock_ghz"] * 1e9
        vpe, spe = prof["valu_insts_per_pe"] * to_run, prof["salu_insts_per_pe"] * to_run
        result["roofline"]["issue"] = {
            "valu_frac": vpe * pe_kernel * 2.0 / (1024.0 * clk), "salu_frac": spe * pe_kernel / (256.0 * clk),
            "valu_insts_per_pe": vpe, "salu_insts_per_pe": spe, "clock_ghz": prof["clock_ghz"],
            "profile_valu_frac": prof["valu_issue_frac"], "profile_salu_frac": prof["salu_issue_frac"]}
    if rank == 0 and not args.no_calibrate:
        from siddhi_amd.engine import calibrate_hbm
        copy_gbps, read_gbps = calibrate_hbm(local)
        rf = result["roofline"]
        rf["measured_peak"] = {"copy": copy_gbps, "read": read_gbps, "unit": "GB/s",
                               "how": "best of 5 streaming 4 GiB copies / reads (csrc/calib.hip)"}
        rf["frac_measured"] = achieved / copy_gbps
    if c5:  # the sparse state (K_slab): bytes per live partial, engine build time
        lb, rb, db = eng.state_bytes()
        result["config"].update({"state_live_bytes": lb, "state_slab_bytes": rb, "state_dir_bytes": db,
                                 "bytes_per_live_partial": (lb + db) / max(1, live),
                                 "engine_build_s": t_build, "warmup_event_hours": args.warmup * B / 3.6e6})
    del pre
    if world > 1 and scaling == "strong" and not args.no_weak_leg:
        # the second line: weak scaling, every GPU runs the workload's full pattern count
        eng.close()
        wsh = Shard(args.workload, "weak", P, rank, world)
        weng = make_engine(args.workload, wsh, K, local, SDH_FLAG_DEVICE_MATCHES, args.partials)
        weng.set_comm(comm)
        wsteps = max(2, args.steps // 3)
        wpre = [local_batch(i) for i in range(args.warmup, args.warmup + wsteps)]
        el, _, _, _, wm, wpe = timed_steps(weng, make_step(weng, wpre), args.warmup, wsteps, world, dist)
        el, wm, wpe, _ = reduce_run(el, wm, wpe, 0, world, dist, cdev)
        result["weak_scaling"] = {"value": wpe / el, "unit": "pattern-events/s", "patterns_per_gpu": wsh.n,
                                  "steps": wsteps, "ms_per_step": el * 1e3 / wsteps, "matches": wm}
        weng.close()
        del wpre
    if not args.no_expansion:
        log("expansion leg (normal mode + sdh_engine_poll_device)")
        result["expansion"] = expansion(args, sh, K, local, dev, world, cdev, dist, comm)
    if not args.no_ingest and world == 1:
        log("host-ingest leg")
        result["host_ingest"] = host_ingest(args, eng, B, K, n_batches)
    if not args.no_latency and world == 1 and not c5:
        log("push-latency leg")
        eng.close()
        result["push_latency"] = push_latency(args, sh, K, local)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline")
        result["cpu_baseline"] = cpu_baseline(args.workload, K, args.cpu_seconds)
    if rank == 0:
        result["build"] = build_provenance()
        print(json.dumps(result), flush=True)
    if world > 1:
        eng.close()
        comm.close()
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


def push_latency(args, sh, K, local):
    """Latency of one small push + poll, the JNI seam's granularity (StreamJunction.Receiver.receive(
    Event) / receive(Event[]) chunks, StreamJunction.java:376-389): host-resident events of 1, 64 and
    4,096, normal mode (every match polled to the host in R18 order). Median and p99 over 50 pushes
    after 5 warm-up pushes (64: 10; 4,096: 10 after 2; at 10K C2 patterns such a push carries ~17M matches),
    continuing one stream; keyed workloads reserve their K keys' state first
    (sdh_engine_reserve_keys). A second engine fed the same pushes polls the compact rows instead
    (sdh_engine_poll_compact_ex to the host: 16 B per C2 match instead of ~72; `compact_*`)."""
    from siddhi_amd.engine import EngineError
    from siddhi_amd.workloads import stock_events, txn_events
    eng = make_engine(args.workload, sh, K, local, 0, args.partials)
    ceng = make_engine(args.workload, sh, K, local, 0, args.partials)
    if args.workload in ("c3", "c5"):  # per-key state sized for the K keys up front (no growth copy
        for x in (eng, ceng):          # inside a push while new keys keep appearing)
            x.reserve_keys(K)
    gen = txn_events if args.workload == "c4" else stock_events
    out, lo = {}, 0
    compact_ok = True
    for bs in (1, 64, 4096):
        lat, plat, clat, nm = [], [], [], 0
        # (warm-up: the poll buffers grow to the push size's match counts -- C2's 64-event pushes carry
        # 0.2-0.4M matches each -- before the timed pushes)
        warm, reps = (5, 50) if bs == 1 else (10, 50) if bs < 4096 else (2, 10)
        for i in range(warm + reps):
            ts, a, b, c = gen(lo, bs, K)
            lo += bs
            cols = [a, b.view(np.uint32), c]
            t0 = time.perf_counter()
            eng.push_columns(0, ts, cols)
            t1 = time.perf_counter()
            m = eng.poll()
            t2 = time.perf_counter()
            if compact_ok:
                try:
                    ceng.push_columns(0, ts, cols)
                    _, rows, _, _, _ = ceng.poll_compact_ex()
                    if len(rows) != len(m[0]):
                        raise RuntimeError(f"poll_compact {len(rows)} rows, poll {len(m[0])} matches")
                except EngineError:
                    compact_ok = False
            t3 = time.perf_counter()
            if os.environ.get("BENCH_TRACE_PUSHES"):  # (diagnostics: one stderr line per push)
                log(f"latency push bs {bs} #{i}: push {(t1 - t0) * 1e3:.3f} ms, poll {(t2 - t1) * 1e3:.3f} ms")
            if i >= warm:
                lat.append((t2 - t0) * 1e3)
                plat.append((t1 - t0) * 1e3)
                clat.append((t3 - t2) * 1e3)
                nm += len(m[0])
        lat.sort()
        plat.sort()
        clat.sort()
        # push: host batch in, NFA step, matches placed in HBM in R18 order; poll: the tuples copied
        # to host arrays (PCIe and host copies, ~72 B per match)
        q = lambda v, f: v[min(len(v) - 1, int(len(v) * f))]
        out[str(bs)] = {"median_ms": q(lat, 0.5), "p99_ms": q(lat, 0.99), "push_median_ms": q(plat, 0.5),
                        "push_p99_ms": q(plat, 0.99), "matches_per_push": nm / len(lat),
                        "compact_median_ms": q(clat, 0.5) if compact_ok else None,
                        "compact_p99_ms": q(clat, 0.99) if compact_ok else None}
    eng.close()
    ceng.close()
    return out


def eng_patterns(eng):
    st = eng.stats()
    return st.pattern_events / max(1, st.events)


def expansion(args, sh, K, local, dev, world, cdev, dist, comm=None):
    """Pushes of a smaller batch in normal mode, each followed by sdh_engine_poll_device (device R18
    sort + gather of the ABI tuples in HBM): the NFA step with every match expanded. One GPU: 12 timed
    pushes after 3 warm-up pushes, keyed workloads with their K keys' state reserved first. With N GPUs the
    pushes are broadcast from rank 0 and every push is followed by sdh_engine_gather: every rank's
    R18-sorted tuples go to rank 0 over RCCL and are merged there on the device, timed per step."""
    import torch
    # with N GPUs every rank's tuples are gathered to rank 0: C2 at 10K patterns makes ~4,300 matches
    # per event, so the multi-GPU gather runs on 8K-event batches
    E = args.expansion_batch if world == 1 else min(args.expansion_batch, 8192)
    eng = make_engine(args.workload, sh, K, local, 0, args.partials)
    if args.workload in ("c3", "c5"):  # per-key state sized up front, as the latency leg does
        eng.reserve_keys(K)
    if comm is not None:
        eng.set_comm(comm)
    steps, warm = (12, 3) if world == 1 else (4, 1)
    root = world == 1 or dist.get_rank() == 0
    bs = [gen_batch(args.workload, s * E, E, K, dev) if root else None for s in range(steps + warm)]
    torch.cuda.synchronize()
    push_ms, gather_ms, matches, merged = 0.0, 0.0, 0, 0
    for i, cols in enumerate(bs):
        if i == warm:
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        t1 = time.perf_counter()
        if world == 1:
            eng.push_device(0, E, cols[0].data_ptr(), [c.data_ptr() for c in cols[1:]])
        elif root:
            eng.push_bcast_device(0, E, cols[0].data_ptr(), [c.data_ptr() for c in cols[1:]], root=0)
        else:
            eng.push_bcast_recv(root=0)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if world > 1:
            n_local = eng.pending_matches()  # this rank's window (one push)
            t3 = time.perf_counter()
            m = eng.gather(device=True)
            if root and i >= warm:  # (timed pushes only, as `matches`)
                merged += m.n
            t4 = time.perf_counter()
        else:
            n_local = eng.poll_device().n
            torch.cuda.synchronize()
            t3 = t4 = time.perf_counter()
        if i >= warm:
            push_ms += (t2 - t1) * 1e3
            gather_ms += (t4 - t3) * 1e3
            matches += n_local
        log(f"expansion push {i + 1}/{steps + warm}: {n_local} matches, push {(t2 - t1) * 1e3:.1f} ms, "
            f"poll/gather {(time.perf_counter() - t2) * 1e3:.1f} ms")
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el, matches], device=cdev, dtype=torch.float64)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        mt = t[1:].clone()
        dist.all_reduce(mt)
        el, matches = float(t[0].item()), int(mt.item())
    pe = eng.stats().pattern_events
    eng.close()
    if world > 1:
        x = torch.tensor([float(pe)], device=cdev, dtype=torch.float64)
        dist.all_reduce(x)
        pe = float(x.item())
    pe_timed = pe * steps / (steps + warm)
    r = {"events_per_step": E, "steps": steps, "ms_per_step": el * 1e3 / steps,
         "push_ms_per_step": push_ms / steps, "poll_ms_per_step": (el * 1e3 - push_ms - gather_ms) / steps,
         "matches_per_step": matches / steps, "pattern_events_per_s": pe_timed / el, "matches_per_s": matches / el}
    if world == 1:
        r["compact"] = compact_leg(args, sh, K, local, bs, E, warm, matches)
        r["compact"]["pattern_events_per_s"] = pe_timed / (r["compact"]["ms_per_step"] * 1e-3 * steps)
    if world > 1:
        if dist.get_rank() == 0 and merged != matches:
            raise RuntimeError(f"the gather merged {merged} matches, the ranks produced {matches}")
        r["rccl_gather_merge_ms_per_step"] = gather_ms / steps  # (sdh_engine_gather: sort, RCCL, merge)
        r["merged_matches_per_step_rank0"] = merged / steps
        r["gather_merge_ns_per_match"] = gather_ms * 1e6 / max(1, matches)
    return r


def compact_leg(args, sh, K, local, bs, E, warm, want):
    """The expansion pushes again on a fresh engine, each followed by sdh_engine_poll_compact_ex(device):
    the same R18-ordered matches as compact int32 rows (a window placed by K_ratchet is handed out as
    it is: no sort, no gather), count chains in a side array, partition keys / timer tiebreaks beside
    the rows when the program has them."""
    import torch
    eng = make_engine(args.workload, sh, K, local, 0, args.partials)
    if args.workload in ("c3", "c5"):
        eng.reserve_keys(K)
    matches, width, chain, extra = 0, 0, 0, 0
    try:
        for i, cols in enumerate(bs):
            if i == warm:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            eng.push_device(0, E, cols[0].data_ptr(), [c.data_ptr() for c in cols[1:]])
            m = eng.poll_compact_ex(device=True)
            if i >= warm:
                matches += m.n
                width = m.width
                chain += m.n_chain
                extra = 8 * (bool(m.key) + bool(m.tb))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    finally:
        eng.close()
    if matches != want:
        raise RuntimeError(f"poll_compact_ex delivered {matches} matches, sdh_engine_poll_device {want}")
    steps = len(bs) - warm
    log(f"compact leg: {matches} matches in {el * 1e3:.1f} ms (width {width})")
    return {"ms_per_step": el * 1e3 / steps, "matches_per_s": matches / el, "width": width,
            "pattern_events_per_s": None,
            "bytes_per_match": 4 * width + extra + (4.0 * chain / matches if matches else 0.0)}


if __name__ == "__main__":
    main()
