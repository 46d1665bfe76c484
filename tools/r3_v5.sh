#!/bin/bash
set -o pipefail
bash tools/r3_verify4.sh || exit 1
AB_ARGS="--workload c4" bash tools/ab_lib.sh ab/lib_seqnp.so || exit 1
mkdir -p gpurun_out/spec_c3 gpurun_out/spec_c4
SDH_SPEC_DUMP=gpurun_out/spec_c3 timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-expansion --no-ingest --no-latency --no-cpu-baseline > gpurun_out/c3dump.log 2>&1 || { tail -5 gpurun_out/c3dump.log; exit 1; }
SDH_SPEC_DUMP=gpurun_out/spec_c4 timeout -k 10 300 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-expansion --no-ingest --no-latency --no-cpu-baseline > gpurun_out/c4dump.log 2>&1 || { tail -5 gpurun_out/c4dump.log; exit 1; }
ls gpurun_out/spec_c3 gpurun_out/spec_c4 | head
