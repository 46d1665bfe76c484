# K_slab runs of groups per wave: slab / C5 parity (goldens included), then the C5 line A/B (one wave per
# item vs runs); the RCCL API calls of the world-1 exchange test (rccl trace)
set -o pipefail
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread --durations=10"
F="tests/test_gpu_slab.py tests/test_gpu_c5.py tests/test_gpu_c5_golden.py tests/test_gpu_compact.py tests/test_gpu_records.py"
echo "cmd: $T $F" > gpurun_out/r6s9_tests.log
timeout -k 10 700 $T $F >> gpurun_out/r6s9_tests.log 2>&1 || { tail -60 gpurun_out/r6s9_tests.log; exit 1; }
tail -14 gpurun_out/r6s9_tests.log
bash tools/ab_knob.sh c5 "SDH_SLAB_RUN=1" ""
mkdir -p gpurun_out/rccl2
timeout -k 10 300 rocprofv3 --rccl-trace --kernel-trace --stats --output-format csv -d gpurun_out/rccl2 -o run -- \
  python3 -m pytest -x -q tests/test_gpu_xch.py::test_rccl_world_one_broadcast_and_gather \
  > gpurun_out/rccl2/pytest.log 2>&1 || { tail -20 gpurun_out/rccl2/pytest.log; exit 1; }
ls gpurun_out/rccl2
