#!/bin/bash
# K_ratchet at 8 waves (SIM) and tile loads at tile start: ratchet / placement / golden parity,
# the headline-config golden, then the C2 profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ratchet.py tests/test_gpu_golden.py -m gpu -x -q -k "not headline" --timeout 600 --timeout-method thread > gpurun_out/v4_tests.log 2>&1 || { tail -30 gpurun_out/v4_tests.log; exit 1; }
tail -1 gpurun_out/v4_tests.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -q -k "headline" --timeout 900 --timeout-method thread > gpurun_out/v4_headline.log 2>&1 || { tail -30 gpurun_out/v4_headline.log; exit 1; }
tail -1 gpurun_out/v4_headline.log
bash tools/r3_prof.sh c2
