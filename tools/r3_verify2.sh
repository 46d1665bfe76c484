#!/bin/bash
# indexed timer sweep (partitioned absent states): absent suite on the GPU, then the verification run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_absent.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/absent.log 2>&1 || { tail -30 gpurun_out/absent.log; exit 1; }
tail -2 gpurun_out/absent.log
bash tools/r3_verify.sh
