#!/bin/bash
# K_part phase clocks (SDH_PART_PROF) on C3 and count-only
set -o pipefail
OUT=gpurun_out/${1:-pprof}
mkdir -p $OUT
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 1 --warmup 1 --workload c3"
SDH_PART_PROF=1 $B > $OUT/rec.log 2>&1 || { tail -5 $OUT/rec.log; exit 1; }
grep "part prof" $OUT/rec.log | tail -3
SDH_PART_PROF=1 SDH_DEBUG_COUNT_ONLY=1 $B > $OUT/cnt.log 2>&1 || { tail -5 $OUT/cnt.log; exit 1; }
grep "part prof" $OUT/cnt.log | tail -3
tail -1 $OUT/rec.log | cut -c1-300
