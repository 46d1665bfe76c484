#!/bin/bash
# K_slab check + measure: its GPU tests, the C5 goldens, then the C5 bench line under a kernel trace
# (per-kernel time shares: nfa_slab_kernel vs slab_move_kernel). Usage: tools/c5_run.sh <out> [notests]
set -o pipefail
OUT=gpurun_out/${1:-c5run}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${2:-}" != notests ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_slab.py tests/test_gpu_c5.py tests/test_gpu_c5_golden.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload c5 --no-cpu-baseline --no-calibrate > $OUT/line.json 2> $OUT/line.err || { tail -20 $OUT/line.err; exit 1; }
grep -E "warm-up|timed" $OUT/line.err
head -6 $OUT/trace/run_kernel_stats.csv | cut -c1-150
