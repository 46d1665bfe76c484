#!/bin/bash
# Round 3: device shard-merge tests (timer rows across ranks), the default bench (N=1 strong), and the
# 2-rank gloo rehearsal of the strong-scaling / gather paths.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gen.py -k "shards_merge or poll_device" tests/test_gpu_golden.py -k "shards_merge or poll_device" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -30 gpurun_out/dist_tests.log; exit 1; }
tail -3 gpurun_out/dist_tests.log
timeout -k 10 600 python -u bench.py --steps 6 --cpu-seconds 6 > gpurun_out/bench_c2.log 2>&1 || { tail -30 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log | cut -c1-1500
bash tools/r3_multi.sh c2 c4 c3
