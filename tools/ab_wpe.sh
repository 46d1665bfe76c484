#!/bin/bash
# A/B of the shape-compiled kernels' register budget (SDH_SEQ_WPE / SDH_PART_WPE) on C3 and C4
set -o pipefail
mkdir -p gpurun_out
export SDH_SPEC=require
for wl in c4 c3; do
  for w in 0 5 6 8; do
    if [ $wl = c4 ]; then export SDH_SEQ_WPE=$w; else export SDH_PART_WPE=$w; fi
    timeout -k 10 240 python bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest \
      > gpurun_out/wpe_${wl}_$w.log 2>&1 || { tail -5 gpurun_out/wpe_${wl}_$w.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), '%.3g' % d['value'], round(d['roofline']['kernel_ms'],2))" gpurun_out/wpe_${wl}_$w.log $wl $w
  done
  unset SDH_SEQ_WPE SDH_PART_WPE
done
