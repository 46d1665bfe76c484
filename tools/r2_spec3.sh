#!/bin/bash
# parity of the K_part / K_seq paths (every shape compiled) + C3 / C4 timing
set -o pipefail
OUT=gpurun_out/${1:-spec5}
mkdir -p $OUT
export SDH_SPEC=require
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_part.py tests/test_gpu_gen.py \
  -k "kpart or c3_family or seq_windows or chunked or reference_kat or partitioned or overflow or ring" > $OUT/gen.log 2>&1 || { tail -40 $OUT/gen.log; exit 1; }
tail -2 $OUT/gen.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_golden.py > $OUT/golden.log 2>&1 || { tail -30 $OUT/golden.log; exit 1; }
tail -2 $OUT/golden.log
unset SDH_SPEC
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 3 --warmup 1"
run() { echo "== $1"; shift; env "$@" > $OUT/tmp.log 2>&1 || { tail -5 $OUT/tmp.log; exit 1; }; tail -1 $OUT/tmp.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.2f ms/step kernel %.2f ms matches/step %.3g" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["config"]["matches"]/d["steps"]))'; }
run "c4" $B --workload c4
run "c4 10k" $B --workload c4 --patterns 10000
run "c3" $B --workload c3
run "c3 count-only" SDH_DEBUG_COUNT_ONLY=1 $B --workload c3
run "c2 10k" $B --workload c2
echo done
