#!/bin/bash
# C3 K_part register-budget sweep: register-resident entries (logical / count) and waves per SIMD
set -o pipefail
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 300 python -u bench.py --workload c3 --steps 4 --warmup 1 --no-expansion --no-ingest --no-latency --no-cpu-baseline > gpurun_out/c3s.log 2> gpurun_out/c3s.err || { tail -20 gpurun_out/c3s.err; exit 1; }
  echo "$*: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c3s.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/c3s.log)"
}
run X=0
run SDH_KPART_REGS=4
run SDH_KPART_REGS=4 SDH_KPART_REGS_COUNT=2
run SDH_KPART_REGS=2 SDH_KPART_REGS_COUNT=1
run SDH_KPART_REGS=4 SDH_PART_WPE=4
run SDH_KPART_REGS=8 SDH_PART_WPE=4
run SDH_KPART_REGS=0 SDH_KPART_REGS_COUNT=0
