set -o pipefail
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_part.py tests/test_gpu_gen.py tests/test_gpu_slab.py tests/test_gpu_golden.py tests/test_gpu_c5_golden.py > gpurun_out/t_lds.log 2>&1 || { tail -30 gpurun_out/t_lds.log; exit 1; }
tail -2 gpurun_out/t_lds.log
bash tools/r5_prof_c3.sh || exit 1
