#!/bin/bash
# A/B of alternative library builds on the C2 expansion leg (64K-event pushes: normal-mode placement,
# poll_device and the compact leg): tools/ab_exp.sh ab/lib_x.so [...]
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-calibrate --no-cpu-baseline --no-ingest --no-latency ${AB_ARGS:-} > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "$1: $(python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); x=d['expansion']; print(round(x['push_ms_per_step'],3), round(x['poll_ms_per_step'],3), round(x['compact']['ms_per_step'],3))")"
}
run default
for lib in "$@"; do SIDDHI_HIP_LIB=$PWD/$lib run $lib; done
run default
