#!/bin/bash
# GPU box: full -m gpu suite, then the selected golden tests, then the default bench (no CPU leg).
set -o pipefail
OUT=gpurun_out/${1:-r2b}
SEL=${2:-"c1 or c3 or poll_device"}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_golden.py > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -v --timeout 400 --timeout-method thread -k "$SEL" > $OUT/golden.log 2>&1 || { tail -40 $OUT/golden.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/golden.log | tail -8
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
