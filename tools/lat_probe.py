"""Per-push latency trace of bench.py's push-latency leg for one workload: one line per push (push and
poll ms, matches). Run with SDH_ALLOC_TRACE=1 to interleave the library's buffer (re)allocations on
stderr, which is how a p99 spike is tied to its cause."""
import argparse
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3")
ap.add_argument("--bs", type=int, default=64)
ap.add_argument("--n", type=int, default=120)
ap.add_argument("--compact", action="store_true", help="poll compact_ex rows instead of tuples")
ap.add_argument("--reserve", action="store_true", help="sdh_engine_reserve_keys(K) before the first push")
a = ap.parse_args()
print("cmd: " + " ".join([sys.executable] + sys.argv), file=sys.stderr, flush=True)  # (the log names its run)

import torch  # noqa: E402,F401

from siddhi_amd.workloads import stock_events, txn_events  # noqa: E402

P0, B0, K0 = bench.DEFAULTS[a.workload]
sh = bench.Shard(a.workload, "strong", P0, 0, 1)
eng = bench.make_engine(a.workload, sh, K0, 0, 0, 128)
if a.reserve:
    eng.reserve_keys(K0)
gen = txn_events if a.workload == "c4" else stock_events
lo = 0
for i in range(a.n):
    ts, x, y, z = gen(lo, a.bs, K0)
    lo += a.bs
    cols = [x, y.view(np.uint32), z]
    t0 = time.perf_counter()
    eng.push_columns(0, ts, cols)
    t1 = time.perf_counter()
    if a.compact:
        _, rows, _, _, _ = eng.poll_compact_ex()
        nm = len(rows)
    else:
        nm = len(eng.poll()[0])
    t2 = time.perf_counter()
    print(f"push {i} push_ms {(t1 - t0) * 1e3:.3f} poll_ms {(t2 - t1) * 1e3:.3f} matches {nm}", file=sys.stderr, flush=True)
eng.close()
