#!/bin/bash
# Round 3: K_slab tests after the per-ring restructure, then C5 bench at 4096 and 100K patterns
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/slab_tests.log 2>&1 || { tail -30 gpurun_out/slab_tests.log; exit 1; }
tail -2 gpurun_out/slab_tests.log
timeout -k 10 300 python -u bench.py --workload c5 --patterns 4096 --steps 4 --no-cpu-baseline > gpurun_out/c5_small.log 2>&1 || { tail -30 gpurun_out/c5_small.log; exit 1; }
tail -1 gpurun_out/c5_small.log
timeout -k 10 900 python -u bench.py --workload c5 --steps 4 --no-cpu-baseline > gpurun_out/c5_full.log 2>&1 || { tail -30 gpurun_out/c5_full.log; exit 1; }
tail -1 gpurun_out/c5_full.log
