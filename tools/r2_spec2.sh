#!/bin/bash
# Shape-compiled K_seq + K_part: parity with every shape compiled, then C3 / C4 A/B against the interpreter
set -o pipefail
OUT=gpurun_out/${1:-spec2}
mkdir -p $OUT
export SDH_SPEC=require
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_part.py tests/test_gpu_gen.py \
  -k "kpart or c3_family or seq_windows or chunked or reference_kat or partitioned or overflow or ring" > $OUT/gen.log 2>&1 || { tail -40 $OUT/gen.log; exit 1; }
tail -2 $OUT/gen.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_golden.py > $OUT/golden.log 2>&1 || { tail -30 $OUT/golden.log; exit 1; }
tail -2 $OUT/golden.log
unset SDH_SPEC
PYTHONPATH=. timeout -k 10 200 python -u tools/diag_pools.py > $OUT/pools.log 2>&1; tail -25 $OUT/pools.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_ingest.py > $OUT/ingest.log 2>&1 || { tail -30 $OUT/ingest.log; exit 1; }
tail -2 $OUT/ingest.log
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 3 --warmup 1"
run() { echo "== $1"; shift; env "$@" > $OUT/tmp.log 2>&1 || { tail -5 $OUT/tmp.log; exit 1; }; tail -1 $OUT/tmp.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.2f ms/step kernel %.2f ms" % (d["ms_per_step"], d["roofline"]["kernel_ms"]))'; }
run "c4 spec" $B --workload c4
run "c4 spec 10k" $B --workload c4 --patterns 10000
run "c3 spec" $B --workload c3
run "c3 interp" SDH_SPEC=0 $B --workload c3
run "c3 regs0" SDH_KPART_REGS=0 $B --workload c3
run "c3 regs2" SDH_KPART_REGS=2 $B --workload c3
export TMPDIR=/tmp
for w in c3 c4; do
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $OUT/pmc_$w -o run -- python3 bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 1 --warmup 1 --workload $w > $OUT/pmc_$w.log 2>&1 || { echo "pmc $w failed"; tail -3 $OUT/pmc_$w.log; exit 1; }
done
echo done
