#!/bin/bash
# K_part / K_seq LDS sizing: parity, then output-buffer sweeps on C3 / C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gen.py tests/test_gpu_golden.py tests/test_gpu_part.py -m gpu -x -q -k "seq or chunked or c4 or c3 or part" --timeout 600 --timeout-method thread > gpurun_out/outw_tests.log 2>&1 || { tail -30 gpurun_out/outw_tests.log; exit 1; }
tail -1 gpurun_out/outw_tests.log
b() {  # b <VAR=value> <workload>
  env "$1" timeout -k 10 300 python -u bench.py --workload $2 --steps 4 --warmup 1 --no-expansion --no-ingest --no-latency --no-cpu-baseline > gpurun_out/ow.log 2> gpurun_out/ow.err || { tail -20 gpurun_out/ow.err; exit 1; }
  echo "$1 $2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ow.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ow.log)"
}
for w in 1536 1024 768; do b SDH_KPART_OUTW=$w c3; done
for w in 1024 768 512; do b SDH_KSEQ_OUTW=$w c4; done
