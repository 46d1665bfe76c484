set -o pipefail
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_part.py tests/test_gpu_gen.py tests/test_gpu_slab.py > gpurun_out/t_swz.log 2>&1 || { tail -30 gpurun_out/t_swz.log; exit 1; }
tail -1 gpurun_out/t_swz.log
bash tools/r5_prof.sh c3 c4 || exit 1
