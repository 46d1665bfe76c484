set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_slab.py tests/test_gpu_c5_golden.py tests/test_gpu_golden.py::test_bench_shape_one_push_equals_many > gpurun_out/t_slab2.log 2>&1 || { tail -5 gpurun_out/t_slab2.log; exit 1; }
tail -2 gpurun_out/t_slab2.log
timeout -k 10 400 python -u bench.py --workload c3 --no-cpu-baseline > gpurun_out/l_c3.json 2> gpurun_out/l_c3.err || exit 1
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-ingest > gpurun_out/l_c2.json 2> gpurun_out/l_c2.err || exit 1
