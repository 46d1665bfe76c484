set -o pipefail
SDH_TRACE=1 timeout -k 10 300 python -u -m pytest -s -x -q --timeout 250 --timeout-method thread "tests/test_gpu_ratchet.py::test_ring_rec4_distance_overflow_reruns_with_8b_records" > gpurun_out/t_rec4b.log 2>&1 || { tail -30 gpurun_out/t_rec4b.log; exit 1; }
tail -1 gpurun_out/t_rec4b.log; grep -c "ratchet stream" gpurun_out/t_rec4b.log; grep "ratchet stream" gpurun_out/t_rec4b.log | tail -4
