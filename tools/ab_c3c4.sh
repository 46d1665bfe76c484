#!/bin/bash
# A/B on one box: C3 (K_part LDS tables on/off, previous build) and C4 (current vs previous build)
set -o pipefail
OUT=gpurun_out/${1:-ab1}
mkdir -p $OUT
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 3 --warmup 1"
run() { echo "== $1"; shift; env "$@" > $OUT/tmp.log 2>&1 || { tail -5 $OUT/tmp.log; exit 1; }; tail -1 $OUT/tmp.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.2f ms/step kernel %.2f ms" % (d["ms_per_step"], d["roofline"]["kernel_ms"]))'; }
run "c3 cur lds" $B --workload c3
run "c3 cur nolds" SDH_KPART_LDS=0 $B --workload c3
run "c3 prev" SIDDHI_HIP_LIB=tools/ab/libsiddhi_prev.so $B --workload c3
run "c4 cur" $B --workload c4
run "c4 prev" SIDDHI_HIP_LIB=tools/ab/libsiddhi_prev.so $B --workload c4
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $OUT/pmc_c3 -o run -- python3 bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 1 --warmup 1 --workload c3 > $OUT/pmc_c3.log 2>&1 || { echo "pmc c3 failed"; tail -3 $OUT/pmc_c3.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $OUT/pmc_c4 -o run -- python3 bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 1 --warmup 1 --workload c4 > $OUT/pmc_c4.log 2>&1 || { echo "pmc c4 failed"; tail -3 $OUT/pmc_c4.log; exit 1; }
echo done
