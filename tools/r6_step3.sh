# K_gate: its parity tests, then the C2x line (4M-event steps) and the records / ratchet tests again
set -o pipefail
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
echo "cmd: $T tests/test_gpu_gate.py tests/test_gpu_records.py" > gpurun_out/r6s3_tests.log
timeout -k 10 600 $T tests/test_gpu_gate.py tests/test_gpu_records.py >> gpurun_out/r6s3_tests.log 2>&1 || { tail -60 gpurun_out/r6s3_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6s3_tests.log
timeout -k 10 300 python -u bench.py --workload c2x --no-cpu-baseline --no-ingest --no-latency --no-expansion > gpurun_out/r6s3_c2x.json 2> gpurun_out/r6s3_c2x.err || { tail -20 gpurun_out/r6s3_c2x.err; exit 1; }
tail -3 gpurun_out/r6s3_c2x.err
