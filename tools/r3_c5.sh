#!/bin/bash
# Round 3: C5 bench on K_slab (small pattern count first, then the config's 100K patterns)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c5 --patterns 4096 --steps 4 --no-cpu-baseline > gpurun_out/c5_small.log 2>&1 || { tail -30 gpurun_out/c5_small.log; exit 1; }
tail -1 gpurun_out/c5_small.log
timeout -k 10 800 python -u bench.py --workload c5 --steps 6 --no-cpu-baseline > gpurun_out/c5_full.log 2>&1 || { tail -30 gpurun_out/c5_full.log; exit 1; }
tail -1 gpurun_out/c5_full.log
