#!/bin/bash
# HEAD: parity of the K_gen / K_seq / K_part / golden suites (ring-mode counts included), the bench
# lines of C2 (default run), C3, C4, then the C5 profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gen.py tests/test_gpu_golden.py tests/test_gpu_part.py -m gpu -x -q -k "not headline" --timeout 600 --timeout-method thread > gpurun_out/f1_tests.log 2>&1 || { tail -30 gpurun_out/f1_tests.log; exit 1; }
tail -1 gpurun_out/f1_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/f1_c2.log 2> gpurun_out/f1_c2.err || { tail -20 gpurun_out/f1_c2.err; exit 1; }
tail -1 gpurun_out/f1_c2.log | cut -c1-400
for wl in c3 c4; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/f1_$wl.log 2> gpurun_out/f1_$wl.err || { tail -20 gpurun_out/f1_$wl.err; exit 1; }
  tail -1 gpurun_out/f1_$wl.log | cut -c1-300
done
bash tools/r3_prof.sh c5
