#!/bin/bash
# ratchet growth tests, then rocprofv3 kernel-trace + PMC passes of the C2-10K headline, C3 and C4
# bench commands at this tree (profiles/collect.sh), each summarized into gpurun_out/prof_*/summary
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_ratchet.py > gpurun_out/ratchet.log 2>&1 || { tail -30 gpurun_out/ratchet.log; exit 1; }
tail -2 gpurun_out/ratchet.log
COMMON="--steps 2 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest"
for spec in "c2:nfa_ratchet_kernel" "c3:sdh_part_spec" "c4:sdh_seq_spec"; do
  wl=${spec%%:*}; k=${spec##*:}
  bash profiles/collect.sh gpurun_out/prof_$wl "$COMMON --workload $wl" $k || exit 1
  echo "profiled $wl"
done
