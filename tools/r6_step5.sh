# trimmed slow tests (gate cases, rec4 overflow, C5 goldens sharing one plan) + the K_seq VGPR A/B on C4
set -o pipefail
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=15"
F="tests/test_gpu_gate.py tests/test_gpu_ratchet.py::test_ring_rec4_distance_overflow_reruns_with_8b_records tests/test_gpu_c5_golden.py"
echo "cmd: $T $F" > gpurun_out/r6s8_tests.log
timeout -k 10 700 $T $F >> gpurun_out/r6s8_tests.log 2>&1 || { tail -60 gpurun_out/r6s8_tests.log; exit 1; }
grep -E "passed|failed|s call" gpurun_out/r6s8_tests.log
bash tools/ab_knob.sh c4 "" "SDH_SEQ_VGPR=1"
