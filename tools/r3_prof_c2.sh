#!/bin/bash
# Round 3: locate the C2 slowdown: kernel trace of a short C2 run (1M-event pushes)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2s -o run -- python3 bench.py --steps 2 --warmup 2 --batch 1048576 --no-expansion --no-ingest --no-cpu-baseline > gpurun_out/prof_c2s.log 2>&1 || { tail -30 gpurun_out/prof_c2s.log; exit 1; }
tail -12 gpurun_out/prof_c2s.log | cut -c1-400
find gpurun_out/prof_c2s -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof_c2s -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-200
