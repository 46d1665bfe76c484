#!/bin/bash
# C5 deep golden, C3 / C4 bench lines at HEAD, then the C5 profile (trace + PMC passes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_c5_golden.py -m gpu -x -v -k "c5deep" --timeout 1000 --timeout-method thread > gpurun_out/c5deep_golden.log 2>&1 || { tail -30 gpurun_out/c5deep_golden.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/c5deep_golden.log
for wl in c3 c4; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$wl.log 2> gpurun_out/bench_$wl.err || { tail -20 gpurun_out/bench_$wl.err; exit 1; }
  tail -1 gpurun_out/bench_$wl.log | cut -c1-600
done
bash tools/r3_prof.sh c5
