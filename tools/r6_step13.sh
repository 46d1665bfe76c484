# K_slab e1 items stage their first event tile while the directory word is in flight: parity (slab,
# C5 family, C5 goldens), then the C5 line with and without it
set -o pipefail
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
F="tests/test_gpu_slab.py tests/test_gpu_c5.py tests/test_gpu_c5_golden.py"
echo "cmd: $T $F" > gpurun_out/r6s13_tests.log
timeout -k 10 600 $T $F >> gpurun_out/r6s13_tests.log 2>&1 || { tail -40 gpurun_out/r6s13_tests.log; exit 1; }
tail -1 gpurun_out/r6s13_tests.log
bash tools/ab_knob.sh c5 "SDH_SLAB_HOIST=0" ""
