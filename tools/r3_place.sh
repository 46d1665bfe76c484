#!/bin/bash
# Round 3: direct R18 placement parity (vs the sort, and the C1-C4 goldens), the default bench,
# then the 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_gen.py -m gpu -x -v -k "not headline and (golden or placement or poll_device or journal or overflow or growth or shards or Query32 or Query33)" --timeout 600 --timeout-method thread > gpurun_out/place_tests.log 2>&1 || { tail -30 gpurun_out/place_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/place_tests.log | cut -c1-150
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5_golden.py -m gpu -x -v -k "c5 and not deep" --timeout 900 --timeout-method thread > gpurun_out/c5_golden.log 2>&1 || { tail -30 gpurun_out/c5_golden.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/c5_golden.log
timeout -k 10 600 python -u bench.py --steps 6 --cpu-seconds 6 > gpurun_out/bench_c2.log 2> gpurun_out/bench_c2.err || { tail -30 gpurun_out/bench_c2.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_c2.err | tail -12
tail -1 gpurun_out/bench_c2.log | cut -c1-3000
bash tools/r3_multi.sh c2 c4 c3
