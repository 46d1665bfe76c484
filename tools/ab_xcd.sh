#!/bin/bash
# A/B of the per-XCD item ranges (SDH_XCD) on the partitioned / windowed workloads, then the default
# C2 bench line (with the HBM calibration). Logs: gpurun_out/ab_<wl>_<xcd>.log
set -o pipefail
mkdir -p gpurun_out
for wl in "$@"; do
  for x in 0 1; do
    SDH_XCD=$x timeout -k 10 300 python bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --no-expansion \
      --no-ingest --no-latency --no-calibrate > gpurun_out/ab_${wl}_$x.log 2>&1 || { tail -20 gpurun_out/ab_${wl}_$x.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${wl}_$x.log').read().strip().splitlines()[-1]); print('$wl xcd=$x', round(d['ms_per_step'],2), 'ms/step', '%.3g' % d['value'])"
  done
done
