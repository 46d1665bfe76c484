#!/bin/bash
# C3 write-traffic probe (run on the GPU box from the repo root): kernel trace (per-variant VGPRs,
# LDS, durations) and FETCH / WRITE per launch with and without match records
# (SDH_DEBUG_COUNT_ONLY=1: K_part counts its matches but writes no record). Usage: tools/c3_probe.sh <out>
set -u
OUT=${1:-gpurun_out/c3probe}
ARGS="--workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency --no-calibrate"
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
for mode in rec norec; do
  [ $mode = norec ] && export SDH_DEBUG_COUNT_ONLY=1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${mode}_$c" -o run -- python3 bench.py $ARGS > "$OUT/pmc_${mode}_$c.log" 2>&1 || { echo "pmc $mode $c failed"; exit 1; }
  done
done
echo probed
