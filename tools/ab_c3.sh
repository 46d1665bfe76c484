#!/bin/bash
# C3 K_part experiments on one box
set -o pipefail
OUT=gpurun_out/${1:-abc3}
mkdir -p $OUT
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 3 --warmup 1 --workload c3"
run() { echo "== $1"; shift; env "$@" > $OUT/tmp.log 2>&1 || { tail -5 $OUT/tmp.log; exit 1; }; tail -1 $OUT/tmp.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.2f ms/step kernel %.2f ms matches/step %.3g" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["config"]["matches"]/d["steps"]))'; }
run "c3" $B
run "c3 count-only" SDH_DEBUG_COUNT_ONLY=1 $B
run "c3 count-only interp" SDH_DEBUG_COUNT_ONLY=1 SDH_SPEC=0 $B
run "c3 1k keys" $B --keys 1000
run "c3 100k keys" $B --keys 100000
