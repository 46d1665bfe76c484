# K_gate spill swap-remove + K_slab exact record reservations: parity (gate, c2x golden, slab, C5
# goldens, records), then the c2x and C5 lines without legs
set -o pipefail
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread --durations=8"
F="tests/test_gpu_gate.py tests/test_gpu_golden.py::test_c2x_config_golden tests/test_gpu_slab.py tests/test_gpu_c5.py tests/test_gpu_c5_golden.py tests/test_gpu_records.py tests/test_gpu_compact.py"
echo "cmd: $T $F" > gpurun_out/r6s11_tests.log
timeout -k 10 800 $T $F >> gpurun_out/r6s11_tests.log 2>&1 || { tail -60 gpurun_out/r6s11_tests.log; exit 1; }
tail -12 gpurun_out/r6s11_tests.log
A="--no-cpu-baseline --no-ingest --no-latency --no-expansion --no-calibrate"
for w in c2x c5; do
  timeout -k 10 600 python -u bench.py --workload $w $A > gpurun_out/r6s11_$w.json 2> gpurun_out/r6s11_$w.err || { tail -20 gpurun_out/r6s11_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['record_bytes_per_match'])" gpurun_out/r6s11_$w.json $w
done
