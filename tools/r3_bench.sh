#!/bin/bash
# Round 3: default bench (N=1) with progress on stderr, then the 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 6 --cpu-seconds 6 > gpurun_out/bench_c2.log 2> gpurun_out/bench_c2.err || { tail -30 gpurun_out/bench_c2.err; exit 1; }
tail -1 gpurun_out/bench_c2.log | cut -c1-2500
bash tools/r3_multi.sh c2 c4 c3
