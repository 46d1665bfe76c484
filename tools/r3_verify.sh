#!/bin/bash
# Round 3 verification at HEAD: K_ratchet (SIM form) + placement + journal + shard-merge + inner-stream
# KAT parity, the C1-C4 goldens, the C5 100K-pattern golden, then the C2 bench with and without the
# SIM form, then the 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ratchet.py tests/test_gpu_golden.py tests/test_gpu_gen.py -m gpu -x -v -k "not headline and (ratchet or golden or placement or poll_device or journal or overflow or growth or shards or Query32 or Query33)" --timeout 600 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || { tail -30 gpurun_out/verify_tests.log; exit 1; }
tail -2 gpurun_out/verify_tests.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5_golden.py -m gpu -x -v -k "c5 and not deep" --timeout 900 --timeout-method thread > gpurun_out/c5_golden.log 2>&1 || { tail -30 gpurun_out/c5_golden.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/c5_golden.log
timeout -k 10 600 python -u bench.py --steps 6 --cpu-seconds 6 > gpurun_out/bench_c2.log 2> gpurun_out/bench_c2.err || { tail -30 gpurun_out/bench_c2.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_c2.err | tail -14
tail -1 gpurun_out/bench_c2.log | cut -c1-3500
SDH_RATCHET_NO_SIM=1 timeout -k 10 300 python -u bench.py --steps 4 --no-expansion --no-ingest --no-latency --no-cpu-baseline > gpurun_out/bench_c2_nosim.log 2> gpurun_out/bench_c2_nosim.err || { tail -30 gpurun_out/bench_c2_nosim.err; exit 1; }
tail -1 gpurun_out/bench_c2_nosim.log | cut -c1-400
bash tools/r3_multi.sh c2 c4 c3
