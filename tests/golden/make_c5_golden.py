#!/usr/bin/env python3
"""Generate tests/golden/large_c5.json and large_c5_deep.json with the CPU oracle (test infrastructure).

BASELINE configs[4] at its full size: 100,000 mixed patterns (workloads.c5_app) over four joined
streams in one `partition with (acct of ...)` over a 1,000,000-account key space, `within 1 hour`.

  c5       the unfiltered stream prefix: E events per stream over all 1M accounts (most keys are seen
           once or twice: the key-table / sparse-state scale case)
  c5deep   the same four streams restricted to the accounts with acct % 512 == 0 (1,954 accounts) over a
           long prefix, so every account sees tens of events per stream across several hours of event
           time (`within` expiry, count chains, logical partners, every re-arming)

The pushed stream is, per push, the four streams' next batches in the order Card, Login, Transfer,
Device (c5deep: each batch filtered to the account subset). Global sequence numbers count the pushed
events in that order.

The oracle restates one runtime per (query, key) (oracle/oracle.cpp); a partition's per-key clones are
independent (PartitionRuntime.java:257-306) and so are queries (StateInputStreamParser.java:90-143), so
the work is cut into (pattern shard x key class) tasks, each an oracle fed only its key class's events.
A task's match seqs are mapped back to global seqs, and the tasks' outputs merge into the one-engine
R18 order by a stable sort on (trigger seq, receiver rank): every slot event of a match precedes or is
its trigger (no absent states), so the trigger is the match's largest seq; all C5 receivers are single-
processor receivers, so the rank is the query's position in the partition's name map (chm.py); and one (event, query) pair's
matches all come from one task, in its emission order. Before the full run the merge is checked
against an unsharded oracle over a small pattern set (`--check`).

Usage: python tests/golden/make_c5_golden.py [c5 c5deep] [--threads 8]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from harness import App, OracleEngine  # noqa: E402
from large_golden import Digest, golden_path  # noqa: E402
from siddhi_amd.workloads import C5_STREAMS, c5_app, c5_events  # noqa: E402

ACCOUNTS = 1_000_000
C5_CONFIGS = {
    # prefix events per stream, push batch (prefix events per stream per push), account filter modulus
    "c5": dict(patterns=100_000, events=24_576, batch=8192, key_mod=1, key_classes=256, pattern_shards=16,
               sample_stride=50),
    "c5deep": dict(patterns=100_000, events=16_000_000, batch=1 << 20, key_mod=512, key_classes=32,
                   pattern_shards=8, sample_stride=200),
}


def pushes(cfg):
    """[(stream, ts, vals [n, 3])] of the pushed stream, in push order."""
    out = []
    for lo in range(0, cfg["events"], cfg["batch"]):
        n = min(cfg["batch"], cfg["events"] - lo)
        for si in range(len(C5_STREAMS)):
            ts, acct, amount, code = c5_events(si, lo, n, ACCOUNTS)
            keep = (acct % cfg["key_mod"]) == 0
            vals = np.stack([acct.astype(np.int64), amount.view(np.uint32).astype(np.int64), code.astype(np.int64)], 1)
            out.append((si, ts[keep], vals[keep]))
    return out


def key_class(acct, classes):
    return (acct.astype(np.int64) * 2654435761 >> 7) % classes


def oracle_matches(eng):
    lib, h = eng.lib, eng.h
    n = lib.oracle_num_matches(h)
    nw = lib.oracle_match_words(h)
    q, k, ts = (np.zeros(n, np.int64) for _ in range(3))
    off = np.zeros(n + 1, np.int64)
    words = np.zeros(max(nw, 1), np.int64)
    lib.oracle_get_matches(h, q.ctypes.data, k.ctypes.data, ts.ctypes.data, off.ctypes.data, words.ctypes.data)
    lib.oracle_clear_matches(h)
    return q, k, ts, off, words[:off[n]]


def run(cfg_name, threads, patterns=None, check=False, log=True):
    cfg = dict(C5_CONFIGS[cfg_name])
    P = patterns or cfg["patterns"]
    shards = 1 if check else min(cfg["pattern_shards"], P)
    classes = 1 if check else cfg["key_classes"]
    t0 = time.time()
    stream = pushes(cfg)
    g0s, g = [], 0
    for si, ts, vals in stream:
        g0s.append(g)
        g += len(ts)
    sp = list(zip(stream, g0s))
    cls = {(si, g0): key_class(vals[:, 0], classes) for (si, ts, vals), g0 in sp}
    bounds = [P * i // shards for i in range(shards + 1)]
    blobs = []
    for i in range(shards):
        app = App(c5_app(bounds[i + 1] - bounds[i], first=bounds[i]), engine_factory=lambda b: None)
        blobs.append(app.blob)
    if log:
        print(f"  {cfg_name}: {g} events pushed, {shards} pattern shards x {classes} key classes "
              f"(planned in {time.time() - t0:.0f} s)", flush=True)
    jobs = [(i, c) for i in range(shards) for c in range(classes)]
    done = [0]
    res = []
    with ThreadPoolExecutor(threads) as ex:
        futs = [ex.submit(task, blobs[i], bounds[i], sp, cls, c) for i, c in jobs]
        for k, f in enumerate(futs):
            res.append(f.result())
            done[0] += 1
            if log and done[0] % max(1, len(jobs) // 20) == 0:
                print(f"  {cfg_name}: {done[0]}/{len(jobs)} tasks, {time.time() - t0:.0f} s", flush=True)
    qs, ks, tss, lens, words, trig = [], [], [], [], [], []
    for r in res:
        for acc, part in zip((qs, ks, tss, lens, words, trig), r):
            acc.extend(part)
    if not qs:
        z = np.zeros(0, np.int64)
        return g, (z, z, z, np.zeros(1, np.int64), z)
    q = np.concatenate(qs)
    k = np.concatenate(ks)
    ts = np.concatenate(tss)
    ln = np.concatenate(lens)
    w = np.concatenate(words)
    tr = np.asarray(trig, np.int64)
    starts = np.concatenate([[0], np.cumsum(ln)[:-1]])
    # stable: trigger seq, then the receiver rank -- the query's position on a key's junction, the
    # order of PartitionRuntime.metaQueryRuntimeMap, a ConcurrentHashMap of the names c5p0 ..
    from siddhi_amd import chm
    from siddhi_amd.planner import java_string_hash
    rank = np.asarray(chm.positions([java_string_hash(f"c5p{p}") for p in range(P)]), np.int64)
    perm = np.lexsort((rank[q], tr))
    ln_s = ln[perm]
    off = np.concatenate([[0], np.cumsum(ln_s)])
    src = np.repeat(starts[perm] - off[:-1], ln_s) + np.arange(off[-1])
    return g, (q[perm], k[perm], ts[perm], off, w[src])


def task(blob, first, sp, cls, c):
    """One oracle over the events of key class c: its matches with global seqs and their triggers."""
    # slots per match = states of its query: kind p % 4 -> 2, 3, 3, 4 states (workloads.c5_query)
    eng = OracleEngine(blob)
    gmap, out = [], []
    for (si, ts, vals), g0 in sp:
        m = cls[(si, g0)] == c
        if not m.any():
            continue
        gmap.extend((g0 + np.nonzero(m)[0]).tolist())
        eng.send(si, ts[m], vals[m], None)
        out.append(oracle_matches(eng))
    del eng
    gmap = np.asarray(gmap, np.int64)
    qs, ks, tss, lens, words, trig = [], [], [], [], [], []
    for q, k, ts, off, w in out:
        if len(q) == 0:
            continue
        w = w.copy()
        for i in range(len(q)):
            S = (2, 3, 3, 4)[int(q[i] + first) % 4]
            p, tmax = off[i], -1
            for _ in range(S):
                cnt = int(w[p])
                if cnt:
                    seqs = gmap[w[p + 1:p + 1 + cnt]]
                    w[p + 1:p + 1 + cnt] = seqs
                    tmax = max(tmax, int(seqs.max()))
                p += 1 + cnt
            assert p == off[i + 1]
            trig.append(tmax)
        qs.append(q + first)
        ks.append(k)
        tss.append(ts)
        lens.append(np.diff(off))
        words.append(w)
    return qs, ks, tss, lens, words, trig


def digest(cols, stride):
    d = Digest(stride)
    d.update(*cols)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=list(C5_CONFIGS))
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--check-patterns", type=int, default=64)
    a = ap.parse_args()
    for name in a.configs:
        cfg = C5_CONFIGS[name]
        # merge check: the sharded run equals one unsharded oracle over a small pattern set
        _, one = run(name, 1, patterns=a.check_patterns, check=True, log=False)
        _, many = run(name, a.threads, patterns=a.check_patterns, log=False)
        d1, dT = digest(one, 7), digest(many, 7)
        assert d1.n > 0 and d1.hexdigest() == dT.hexdigest(), f"{name}: sharded merge differs from one engine"
        print(f"{name}: merge check ok ({a.check_patterns} patterns, {d1.n} matches)", flush=True)
        t0 = time.time()
        n_ev, cols = run(name, a.threads)
        d = digest(cols, cfg["sample_stride"])
        out = {"config": name, "event_seed": 42, "pattern_seed": 7, "patterns": cfg["patterns"],
               "accounts": ACCOUNTS, "key_mod": cfg["key_mod"], "prefix_events_per_stream": cfg["events"],
               "batch": cfg["batch"], "pushed_events": n_ev,
               "generator": "tests/golden/make_c5_golden.py (oracle/liboracle.so, pattern shards x key classes)",
               "oracle_seconds": round(time.time() - t0, 1)}
        out.update(d.summary())
        with open(golden_path(name), "w") as f:
            json.dump(out, f, separators=(",", ":"))
        print(f"{name}: {n_ev} events, {d.n} matches, digest {d.hexdigest()[:16]}, {time.time() - t0:.0f} s",
              flush=True)


if __name__ == "__main__":
    main()
