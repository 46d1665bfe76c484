#!/bin/bash
# K_seq per-shape LDS rows: parity (K_seq fuzz + C4 golden), C4 bench; C3 register-entry sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gen.py tests/test_gpu_golden.py tests/test_gpu_part.py -m gpu -x -q -k "seq or chunked or c4 or c3 or part" --timeout 600 --timeout-method thread > gpurun_out/seqrow_tests.log 2>&1 || { tail -30 gpurun_out/seqrow_tests.log; exit 1; }
tail -1 gpurun_out/seqrow_tests.log
AB_ARGS="--workload c4" bash tools/ab_lib.sh || exit 1
for r in 3 5 6; do
  SDH_KPART_REGS=$r timeout -k 10 300 python -u bench.py --workload c3 --steps 4 --warmup 1 --no-expansion --no-ingest --no-latency --no-cpu-baseline > gpurun_out/c3s.log 2> gpurun_out/c3s.err || { tail -20 gpurun_out/c3s.err; exit 1; }
  echo "REGS=$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c3s.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/c3s.log)"
done
