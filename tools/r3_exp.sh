#!/bin/bash
# expansion leg: direct placement vs the sort (SDH_NO_PLACE), and a kernel trace of the placement
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-ingest --no-latency --no-cpu-baseline > gpurun_out/exp_place.log 2> gpurun_out/exp_place.err || { tail -20 gpurun_out/exp_place.err; exit 1; }
grep expansion gpurun_out/exp_place.err
SDH_NO_PLACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-ingest --no-latency --no-cpu-baseline > gpurun_out/exp_sort.log 2> gpurun_out/exp_sort.err || { tail -20 gpurun_out/exp_sort.err; exit 1; }
grep expansion gpurun_out/exp_sort.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_exp -o run -- python -u bench.py --steps 1 --warmup 1 --no-ingest --no-latency --no-cpu-baseline > gpurun_out/prof_exp.log 2>&1 || { tail -20 gpurun_out/prof_exp.log; exit 1; }
f=$(find gpurun_out/prof_exp -name "*kernel_stats.csv" | head -1); head -14 "$f" | cut -c1-220
