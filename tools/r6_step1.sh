# Device records + RCCL world-1 + C host: the new tests, then the C2 line (device records) and a C2x line
set -o pipefail
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
F="tests/test_gpu_records.py tests/test_gpu_abi_c.py tests/test_gpu_xch.py tests/test_gpu_ratchet.py tests/test_gpu_compact.py"
echo "cmd: $T $F" > gpurun_out/r6s1_tests.log
timeout -k 10 700 $T $F >> gpurun_out/r6s1_tests.log 2>&1 || { tail -40 gpurun_out/r6s1_tests.log; exit 1; }
tail -3 gpurun_out/r6s1_tests.log
echo "cmd: $T tests/test_gpu_golden.py -k bench_shape" > gpurun_out/r6s1_shape.log
timeout -k 10 400 $T tests/test_gpu_golden.py -k bench_shape >> gpurun_out/r6s1_shape.log 2>&1 || { tail -40 gpurun_out/r6s1_shape.log; exit 1; }
tail -3 gpurun_out/r6s1_shape.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --no-latency --no-expansion > gpurun_out/r6s1_c2.json 2> gpurun_out/r6s1_c2.err || { tail -20 gpurun_out/r6s1_c2.err; exit 1; }
tail -4 gpurun_out/r6s1_c2.err
cat gpurun_out/r6s1_c2.json
timeout -k 10 300 python -u bench.py --workload c2x --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-latency --no-expansion > gpurun_out/r6s1_c2x.json 2> gpurun_out/r6s1_c2x.err || { tail -20 gpurun_out/r6s1_c2x.err; exit 1; }
tail -4 gpurun_out/r6s1_c2x.err
