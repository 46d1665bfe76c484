#!/bin/bash
# K_slab: parity (slab suite, C5 family, the C5 golden), then the LDS staging sweep on the C5 shard
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_c5.py tests/test_gpu_c5_golden.py -m gpu -x -q -k "not c5deep" --timeout 800 --timeout-method thread > gpurun_out/slab_tests.log 2>&1 || { tail -30 gpurun_out/slab_tests.log; exit 1; }
tail -1 gpurun_out/slab_tests.log
b() {
  env "$1" timeout -k 10 400 python -u bench.py --workload c5 --steps 2 --warmup 4 --no-cpu-baseline > gpurun_out/c5s.log 2> gpurun_out/c5s.err || { tail -20 gpurun_out/c5s.err; exit 1; }
  echo "$1: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5s.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/c5s.log)"
}
b SDH_SLAB_LDS_WORDS=4096
b SDH_SLAB_LDS_WORDS=2048
b SDH_SLAB_LDS_WORDS=1024
