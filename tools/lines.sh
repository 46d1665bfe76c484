#!/bin/bash
# The bench lines of a round: the default (driver) command, then C3 / C4 / C2x (and C5 with `c5`)
# with their CPU baselines, each under its own time limit; logs in gpurun_out/line_<w>.log (copy to
# profiles/r6_runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/line_c2.log 2> gpurun_out/line_c2.err || { tail -20 gpurun_out/line_c2.err; exit 1; }
tail -1 gpurun_out/line_c2.log | cut -c1-300
for w in c3 c4 c2x; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/line_$w.log 2> gpurun_out/line_$w.err || { tail -20 gpurun_out/line_$w.err; exit 1; }
  tail -1 gpurun_out/line_$w.log | cut -c1-300
done
if [ "$1" = c5 ]; then
  timeout -k 10 900 python -u bench.py --workload c5 > gpurun_out/line_c5.log 2> gpurun_out/line_c5.err || { tail -20 gpurun_out/line_c5.err; exit 1; }
  tail -1 gpurun_out/line_c5.log | cut -c1-300
fi
