#!/usr/bin/env python3
"""Summarize a profiles/collect.sh run: kernel stats + per-kernel mean PMC counters + meta.json.

usage: python profiles/summarize.py <collect-out-dir> <dest-dir> <kernel-substring> <workload> <patterns> <batch>

Writes kernel_stats.csv (rocprofv3 --stats), counters.json (mean per dispatch, per kernel, raw units:
FETCH_SIZE / WRITE_SIZE in KiB as rocprofv3 reports them) and meta.json, which bench.py attaches to
its JSON line when the sources hash equal (bench.source_hash, recorded on the GPU box). Derived per
launch of the named kernel (MI355X_MICROARCH.md: HBM/rocprofv3 and PMC sections):
  traffic_bytes  = (2 x FETCH_SIZE + WRITE_SIZE) x 1024  (gfx950: FETCH_SIZE reports half of a
                   wide streaming read)
  clock_ghz      = GRBM_GUI_ACTIVE / 8 XCDs / kernel time
  valu_issue_frac= SQ_INSTS_VALU x 2 cycles (a wave64 VALU op on a SIMD32) / (1024 SIMDs x cycles)
  salu_issue_frac= SQ_INSTS_SALU / (256 CUs x cycles)  (one scalar issue per CU per cycle)
  *_per_pe       = wave-instructions per pattern-event (batch x patterns per launch)
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES, l2_hit = TCC_HIT / (TCC_HIT + TCC_MISS)
"""
import collections
import csv
import glob
import json
import re
import os
import shutil
import subprocess
import sys


def main(src, dst, kernel, workload, patterns, batch):
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
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(dst, "kernel_stats.csv")))}
    name = next(k for k in stats if kernel in k)
    c = next(v for k, v in out.items() if kernel in k)
    ns = float(stats[name]["AverageNs"])
    pe = float(patterns) * float(batch)
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    d = {"kernel_name": name, "kernel_ns_avg": ns, "calls": int(stats[name]["Calls"]),
         "traffic_bytes": (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0,
         "fetch_kib": c["FETCH_SIZE"], "write_kib": c["WRITE_SIZE"],
         "clock_ghz": cyc / ns,
         "valu_issue_frac": c["SQ_INSTS_VALU"] * 2.0 / (1024.0 * cyc),
         "salu_issue_frac": c["SQ_INSTS_SALU"] / (256.0 * cyc),
         "valu_insts_per_pe": c["SQ_INSTS_VALU"] / pe, "salu_insts_per_pe": c["SQ_INSTS_SALU"] / pe,
         "lds_insts_per_pe": c["SQ_INSTS_LDS"] / pe, "vmem_insts_per_pe": c["SQ_INSTS_VMEM"] / pe,
         "wait_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
         "l2_hit": c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])}
    if c.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    try:
        commit = subprocess.check_output(["git", "rev-parse", "--short=12", "HEAD"], text=True).strip()
    except (OSError, subprocess.CalledProcessError):
        commit = ""
    # the profiled run's own bench line: the steps and the warm-up it really ran (C5 forces a longer
    # warm-up than its arguments say), so bench.py divides the call count by the real step count
    # and the passes it re-ran (an output / capacity overflow undoes a pass and launches it again:
    # SDH_TRACE prints one line per attempt), so that re-run launches are not counted as per-step work
    line, reruns = {}, 0
    for ln in open(os.path.join(src, "trace.log"), errors="replace"):
        if ln.startswith('{"metric"'):
            line = json.loads(ln)
        elif re.match(r"\[sdh\] (ratchet|gen pass) .*attempt [1-9]", ln):
            reruns += 1
    meta = {"source_hash": open(os.path.join(src, "source_hash")).read().strip(),
            "steps": line.get("steps"), "warmup": line.get("warmup"), "reruns": reruns,
            "bench_args": open(os.path.join(src, "args")).read().strip(), "commit_base": commit,
            "workload": workload, "patterns": int(patterns), "batch": int(batch),
            "kernels": {kernel: d}}
    json.dump(meta, open(os.path.join(dst, "meta.json"), "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:7])
