#!/bin/bash
# direct placement from in-kernel (event, rank) counts: parity (placement == sort, goldens, headline
# config), then the expansion leg with placement and with the sort
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_ratchet.py -m gpu -x -v -k "placement or poll_device or c1 or c2 or ratchet" --timeout 600 --timeout-method thread > gpurun_out/place2_tests.log 2>&1 || { tail -30 gpurun_out/place2_tests.log; exit 1; }
tail -2 gpurun_out/place2_tests.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-ingest --no-cpu-baseline > gpurun_out/exp_place.log 2> gpurun_out/exp_place.err || { tail -20 gpurun_out/exp_place.err; exit 1; }
grep -E "expansion|timed" gpurun_out/exp_place.err
tail -1 gpurun_out/exp_place.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('expansion','push_latency')}))"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_exp2 -o run -- python -u bench.py --steps 1 --warmup 1 --no-ingest --no-latency --no-cpu-baseline > gpurun_out/prof_exp2.log 2>&1 || { tail -20 gpurun_out/prof_exp2.log; exit 1; }
f=$(find gpurun_out/prof_exp2 -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-200
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -v -k "headline" --timeout 900 --timeout-method thread > gpurun_out/headline_golden.log 2>&1 || { tail -30 gpurun_out/headline_golden.log; exit 1; }
tail -2 gpurun_out/headline_golden.log
