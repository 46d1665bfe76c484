#!/bin/bash
# C5 shard bench line comparable to profiles/r3_runs/c5_full.log (4 steps after 8 warm-up steps), then
# its profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload c5 --steps 4 --warmup 8 --no-cpu-baseline > gpurun_out/c5_final.log 2> gpurun_out/c5_final.err || { tail -20 gpurun_out/c5_final.err; exit 1; }
tail -1 gpurun_out/c5_final.log | cut -c1-400
bash tools/r3_prof.sh c5
