# K_seq clean tiles (no null / expiry tests when a tile cannot fail them): K_seq / C4 parity, then the
# C4 line
set -o pipefail
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread --durations=8"
F="tests/test_gpu_gen.py tests/test_gpu_golden.py::test_large_golden_full_config tests/test_gpu_latency.py tests/test_gpu_records.py tests/test_gpu_compact.py tests/test_gpu_xch.py"
echo "cmd: $T $F" > gpurun_out/r6s12_tests.log
timeout -k 10 800 $T $F >> gpurun_out/r6s12_tests.log 2>&1 || { tail -60 gpurun_out/r6s12_tests.log; exit 1; }
tail -4 gpurun_out/r6s12_tests.log
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --no-ingest --no-latency --no-expansion --no-calibrate > gpurun_out/r6s12_c4.json 2> gpurun_out/r6s12_c4.err || { tail -20 gpurun_out/r6s12_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6s12_c4.json')); print('c4', d['ms_per_step'], d['roofline']['kernel_ms'])"
