# RCCL kernels of the world-1 exchange test under a kernel trace; C3 64K-push phases + kernel timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rccl1 gpurun_out/c3small
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rccl1 -o run -- \
  python3 -m pytest -x -q tests/test_gpu_xch.py::test_rccl_world_one_broadcast_and_gather \
  > gpurun_out/rccl1/pytest.log 2>&1 || { tail -20 gpurun_out/rccl1/pytest.log; exit 1; }
tail -2 gpurun_out/rccl1/pytest.log
timeout -k 10 300 python3 -u tools/c3_small.py --pushes 20 > gpurun_out/c3small/plain.log 2>&1 || { tail -20 gpurun_out/c3small/plain.log; exit 1; }
tail -3 gpurun_out/c3small/plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3small/trace -o run -- \
  python3 -u tools/c3_small.py --pushes 12 > gpurun_out/c3small/traced.log 2>&1 || { tail -20 gpurun_out/c3small/traced.log; exit 1; }
tail -2 gpurun_out/c3small/traced.log
