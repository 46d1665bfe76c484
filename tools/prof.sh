#!/bin/bash
# Profiles at HEAD: rocprofv3 kernel trace + PMC passes (profiles/collect.sh) of the bench workloads,
# summarized by profiles/summarize.py into gpurun_out/${TAG}_<workload> (copy to profiles/ to commit).
# Usage: TAG=r4 tools/prof.sh [c2] [c3] [c4] [c5]
set -o pipefail
mkdir -p gpurun_out
for wl in "${@:-c2 c5}"; do
  case $wl in
    c2) args="--steps 2 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency"; kern=nfa_ratchet_kernel; pat=10000; batch=8388608 ;;
    c5) args="--workload c5 --steps 2 --no-cpu-baseline"; kern=nfa_slab_kernel; pat=100000; batch=524288 ;;
    c3) args="--workload c3 --steps 4 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency"; kern=sdh_part_spec; pat=1000; batch=1048576 ;;
    c4) args="--workload c4 --steps 4 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency"; kern=sdh_seq_spec; pat=10000; batch=1048576 ;;
  esac
  bash profiles/collect.sh gpurun_out/prof_$wl "$args" $kern > gpurun_out/prof_$wl.log 2>&1 || { tail -20 gpurun_out/prof_$wl.log; exit 1; }
  python3 profiles/summarize.py gpurun_out/prof_$wl gpurun_out/${TAG:-r4}_$wl $kern $wl $pat $batch > gpurun_out/sum_$wl.log 2>&1 || { tail -20 gpurun_out/sum_$wl.log; exit 1; }
  tail -25 gpurun_out/sum_$wl.log
  rm -rf gpurun_out/prof_$wl  # (raw traces: the summary is in gpurun_out/${TAG:-r4}_$wl; keeps the copy-back small)
done
