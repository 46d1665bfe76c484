#!/bin/bash
# Round 3: K_slab GPU parity (test_gpu_slab.py + the C5 family test), then a small C5 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_c5.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/slab_tests.log 2>&1
rc=$?
tail -15 gpurun_out/slab_tests.log
exit $rc
