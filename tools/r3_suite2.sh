#!/bin/bash
# the full GPU suite at the final HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread > gpurun_out/suite2.log 2>&1 || { tail -40 gpurun_out/suite2.log; exit 1; }
tail -2 gpurun_out/suite2.log
