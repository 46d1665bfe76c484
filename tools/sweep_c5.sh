#!/bin/bash
# C5 (K_slab) occupancy sweep: "wpe:small_rows" pairs, e.g. tools/sweep_c5.sh 4:1024 6:512
set -o pipefail
mkdir -p gpurun_out
for p in "$@"; do
  w=${p%%:*}; r=${p##*:}
  SDH_SLAB_WPE=$w SDH_SLAB_LDS_SMALL=$r timeout -k 10 300 python bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline \
    --no-expansion --no-ingest --no-latency --no-calibrate > gpurun_out/sw_c5_${w}_$r.log 2>&1 || { tail -5 gpurun_out/sw_c5_${w}_$r.log; exit 1; }
  echo "wpe $w rows $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw_c5_${w}_$r.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/sw_c5_${w}_$r.log)"
done
