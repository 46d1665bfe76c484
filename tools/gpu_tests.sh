#!/bin/bash
# GPU tests on the box: tools/gpu_tests.sh <log name> <pytest targets...>
# (every GPU step under its own time limit; the log lands in gpurun_out/<log name>.log)
set -o pipefail
mkdir -p gpurun_out
NAME=$1
shift
timeout -k 10 1100 python -u -m pytest "$@" -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread --durations=60 \
  > gpurun_out/$NAME.log 2>&1
rc=$?
tail -30 gpurun_out/$NAME.log
exit $rc
