#!/bin/bash
# K_part register-table sizes: parity at the default, phase clocks and timing per size
set -o pipefail
OUT=gpurun_out/${1:-regs}
mkdir -p $OUT
SDH_SPEC=require timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_part.py > $OUT/part.log 2>&1 || { tail -30 $OUT/part.log; exit 1; }
tail -1 $OUT/part.log
SDH_SPEC=require SDH_KPART_REGS=2 SDH_KPART_REGS_COUNT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_part.py > $OUT/part2.log 2>&1 || { tail -30 $OUT/part2.log; exit 1; }
tail -1 $OUT/part2.log
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 3 --warmup 1 --workload c3"
run() { echo "== $1"; shift; env "$@" > $OUT/tmp.log 2>&1 || { tail -5 $OUT/tmp.log; exit 1; }; grep "part prof" $OUT/tmp.log | tail -3; tail -1 $OUT/tmp.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.2f ms/step kernel %.2f ms matches/step %.3g" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["config"]["matches"]/d["steps"]))'; }
for rc in 0 2 3 4; do run "count regs $rc" SDH_PART_PROF=1 SDH_KPART_REGS_COUNT=$rc $B; done
for rl in 2 4 8; do run "logical regs $rl" SDH_KPART_REGS=$rl $B; done
run "default no prof" $B
echo done
