#!/bin/bash
# expansion leg at HEAD, then the C2 profile (trace + PMC passes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -q -k "placement or poll_device or c2" --timeout 300 --timeout-method thread > gpurun_out/exp2_tests.log 2>&1 || { tail -30 gpurun_out/exp2_tests.log; exit 1; }
tail -1 gpurun_out/exp2_tests.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-ingest --no-latency --no-cpu-baseline > gpurun_out/exp2.log 2> gpurun_out/exp2.err || { tail -20 gpurun_out/exp2.err; exit 1; }
grep -E "expansion push 5" gpurun_out/exp2.err
bash tools/r3_prof.sh c2
