#!/usr/bin/env python3
"""Generate tests/golden/large_c{1,2,3,4}.json with the CPU oracle (test infrastructure).

The oracle restates the reference engine per query (oracle/oracle.cpp); queries are independent
(each has its own processor graph, StateInputStreamParser.java:90-143), so the pattern set is cut
into T shards that run in parallel threads (ctypes releases the GIL). Each batch's shard outputs are
merged into the one-engine R18 order: a stable sort by (match ts, receiver rank). The synthetic
streams have strictly increasing timestamps (1 event / ms), so a match's ts -- the timestamp of the
event that completed it -- identifies its triggering event, and a query's matches for one event all
come from one shard in their pending-list order. Before the full run, the merge is checked against
an unsharded oracle run over the stream's first events (`--check-events`).

Usage: python tests/golden/make_large_golden.py [c1 c2 c3 c4] [--threads 8]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from harness import App  # noqa: E402
from large_golden import CONFIGS, Digest, app_source, events, golden_path  # noqa: E402


def raw_matches(app):
    """The oracle's pending matches as ABI column arrays (no per-match Python decoding)."""
    lib, h = app.engine.lib, app.engine.h
    n = lib.oracle_num_matches(h)
    nw = lib.oracle_match_words(h)
    q = np.zeros(n, np.int64)
    k = np.zeros(n, np.int64)
    ts = np.zeros(n, np.int64)
    off = np.zeros(n + 1, np.int64)
    words = np.zeros(max(nw, 1), np.int64)
    lib.oracle_get_matches(h, q.ctypes.data, k.ctypes.data, ts.ctypes.data, off.ctypes.data, words.ctypes.data)
    lib.oracle_clear_matches(h)
    return q, k, ts, off, words


def receiver_ranks(cfg_name, P):
    """Per global query its receiver rank on the one stream (dist.output_ranks of the full app): the
    query index, except inside C3's partition, whose clones sit on a key's junction in the order of
    PartitionRuntime.metaQueryRuntimeMap (a ConcurrentHashMap of the names c3p0 .. c3p{P-1})."""
    from siddhi_amd import chm
    from siddhi_amd.planner import java_string_hash
    if cfg_name != "c3":
        return np.arange(P, dtype=np.int64)
    return np.asarray(chm.positions([java_string_hash(f"c3p{p}") for p in range(P)]), np.int64)


def merge(parts, firsts, rank):
    """Shard outputs of one batch -> one R18-ordered set of columns (query ids made global)."""
    qs, ks, tss, lens, words = [], [], [], [], []
    for (q, k, ts, off, w), first in zip(parts, firsts):
        qs.append(q + first)
        ks.append(k)
        tss.append(ts)
        lens.append(np.diff(off))
        words.append(w[:off[-1]])
    q = np.concatenate(qs)
    if len(q) == 0:
        return q, q, q, np.zeros(1, np.int64), q
    k = np.concatenate(ks)
    ts = np.concatenate(tss)
    ln = np.concatenate(lens)
    w = np.concatenate(words)
    starts = np.concatenate([[0], np.cumsum(ln)[:-1]])
    # receiver rank per query (receiver_ranks), checked by the unsharded comparison
    perm = np.lexsort((rank[q], ts))  # stable: primary ts, then rank; shard order kept within a query
    ln_s = ln[perm]
    off = np.concatenate([[0], np.cumsum(ln_s)])
    src = np.repeat(starts[perm] - off[:-1], ln_s) + np.arange(off[-1])
    return q[perm], k[perm], ts[perm], off, w[src]


def run(cfg_name, n_events, threads, stride, log=True):
    cfg = CONFIGS[cfg_name]
    P = cfg["patterns"]
    T = max(1, min(threads, P))
    bounds = [P * i // T for i in range(T + 1)]
    apps = [App(app_source(cfg_name, bounds[i + 1] - bounds[i], first=bounds[i])) if cfg_name != "c1"
            else App(app_source("c1", 1)) for i in range(T)]
    dig = Digest(stride)
    rank = receiver_ranks(cfg_name, P)
    B = cfg["batch"]
    t0 = time.time()
    with ThreadPoolExecutor(T) as ex:
        for lo in range(0, n_events, B):
            n = min(B, n_events - lo)
            ts, _, vals = events(cfg_name, lo, n)

            def one(i):
                apps[i].engine.send(0, ts, vals, None)
                return raw_matches(apps[i])
            parts = list(ex.map(one, range(T)))
            dig.update(*merge(parts, bounds[:T], rank))
            if log and (lo // B) % (1 if cfg_name == "c2x" else 4) == 0:
                print(f"  {cfg_name}: {lo + n}/{n_events} events, {dig.n} matches, {time.time() - t0:.0f} s",
                      flush=True)
    return dig


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=list(CONFIGS))
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--check-events", type=int, default=0, help="events of the unsharded merge check "
                    "(default: 3000, c3: 30000)")
    a = ap.parse_args()
    for name in a.configs:
        cfg = CONFIGS[name]
        chk = a.check_events or (30000 if name == "c3" else 3000)
        d1 = run(name, chk, 1, 7, log=False)
        dT = run(name, chk, a.threads, 7, log=False)
        assert d1.n > 0 and d1.hexdigest() == dT.hexdigest(), f"{name}: sharded merge differs from one engine"
        print(f"{name}: merge check ok over {chk} events ({d1.n} matches)", flush=True)
        t0 = time.time()
        d = run(name, cfg["events"], a.threads, cfg["sample_stride"])
        out = {"config": name, "event_seed": 42, "pattern_seed": 7, "patterns": cfg["patterns"],
               "events": cfg["events"], "keys": cfg["keys"], "stream": cfg["stream"],
               "generator": "tests/golden/make_large_golden.py (oracle/liboracle.so, sharded by pattern set)",
               "oracle_seconds": round(time.time() - t0, 1)}
        out.update(d.summary())
        with open(golden_path(name), "w") as f:
            json.dump(out, f, separators=(",", ":"))
        print(f"{name}: {d.n} matches, digest {d.hexdigest()[:16]}, {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
