#!/bin/bash
# fan-out partitions (q30) + the K_gen / absent / persistence suites, then the placement run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fanout.py tests/test_gpu_gen.py tests/test_gpu_absent.py tests/test_gpu_persistence.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fanout_suite.log 2>&1 || { tail -40 gpurun_out/fanout_suite.log; exit 1; }
tail -2 gpurun_out/fanout_suite.log
bash tools/r3_place2.sh
