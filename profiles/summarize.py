#!/usr/bin/env python3
"""Summarize a profiles/collect.sh run: kernel stats + per-kernel mean PMC counters.

usage: python profiles/summarize.py <collect-out-dir> <dest-dir>
Copies run_kernel_stats.csv and writes counters.json (mean per dispatch, per kernel, raw units:
FETCH_SIZE/WRITE_SIZE in KiB as rocprofv3 reports them; see DESIGN.md for the gfx950 corrections).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    out = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(float)
        n = collections.Counter()
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"], r["Counter_Name"])
            agg[k] += float(r["Counter_Value"])
            n[k] += 1
        for (kern, ctr), v in agg.items():
            out[kern][ctr] = v / n[(kern, ctr)]
    json.dump(out, open(os.path.join(dst, "counters.json"), "w"), indent=1, sort_keys=True)
    for kern, c in out.items():
        if c.get("SQ_WAVES", 0) > 0 or "FETCH_SIZE" in c:
            print(kern, json.dumps(c))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
