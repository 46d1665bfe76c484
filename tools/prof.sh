#!/bin/bash
# Round 3 profiles at HEAD: rocprofv3 kernel trace + PMC passes of C2 (10K patterns, 8M-event steps,
# K_ratchet SIM form) and C5 (100K patterns x 125K accounts, K_slab), summarized into profiles/r3_*
# Usage: tools/r3_prof.sh [c2] [c5]
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
  python3 profiles/summarize.py gpurun_out/prof_$wl gpurun_out/r3_$wl $kern $wl $pat $batch > gpurun_out/sum_$wl.log 2>&1 || { tail -20 gpurun_out/sum_$wl.log; exit 1; }
  tail -25 gpurun_out/sum_$wl.log
  rm -rf gpurun_out/prof_$wl  # (raw traces: the summary is in gpurun_out/r3_$wl; keeps the copy-back small)
done
