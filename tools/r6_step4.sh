# K_gate with worst-key eviction: parity tests, the C2x line; the C4 latency-probe sequence test
set -o pipefail
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
F="tests/test_gpu_gate.py tests/test_gpu_latency.py tests/test_gpu_gen.py::test_device_matches_ring_counts_every_record"
echo "cmd: $T $F" > gpurun_out/r6s7_tests.log
timeout -k 10 600 $T $F >> gpurun_out/r6s7_tests.log 2>&1 || { tail -60 gpurun_out/r6s7_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6s7_tests.log
timeout -k 10 300 python -u bench.py --workload c2x --no-cpu-baseline --no-ingest --no-latency --no-expansion > gpurun_out/r6s7_c2x.json 2> gpurun_out/r6s7_c2x.err || { tail -20 gpurun_out/r6s7_c2x.err; exit 1; }
tail -3 gpurun_out/r6s7_c2x.err
