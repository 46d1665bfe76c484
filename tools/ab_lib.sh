#!/bin/bash
# A/B of alternative library builds on the C2 headline step: tools/ab_lib.sh ab/lib_x.so [ab/lib_y.so ...]
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-expansion --no-ingest --no-latency --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "$1: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab.log)"
}
run default
for lib in "$@"; do SIDDHI_HIP_LIB=$PWD/$lib run $lib; done
run default
