#!/bin/bash
# the full GPU suite at HEAD (what the driver runs at round end), then the C3 / C4 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread > gpurun_out/suite.log 2>&1 || { tail -40 gpurun_out/suite.log; exit 1; }
tail -2 gpurun_out/suite.log
for wl in c3 c4; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/s_$wl.log 2> gpurun_out/s_$wl.err || { tail -20 gpurun_out/s_$wl.err; exit 1; }
  tail -1 gpurun_out/s_$wl.log | cut -c1-300
done
