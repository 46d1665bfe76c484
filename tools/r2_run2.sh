#!/bin/bash
# GPU box: K_part tests, full -m gpu suite, C3/C4 goldens, C3 and C4 bench lines
set -o pipefail
OUT=gpurun_out/${1:-r2f}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_part.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/part.log 2>&1 || { tail -60 $OUT/part.log; exit 1; }
tail -1 $OUT/part.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_golden.py --deselect tests/test_gpu_part.py > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -v --timeout 250 --timeout-method thread -k "c3 or c4" > $OUT/golden.log 2>&1 || { tail -40 $OUT/golden.log; exit 1; }
grep -E "PASS|FAIL" $OUT/golden.log | tail -3
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --no-expansion > $OUT/bench_c3.log 2>&1 || { tail -20 $OUT/bench_c3.log; exit 1; }
tail -1 $OUT/bench_c3.log
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --no-expansion > $OUT/bench_c4.log 2>&1 || { tail -20 $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log
