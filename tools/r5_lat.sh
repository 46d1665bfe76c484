set -o pipefail
export SDH_ALLOC_TRACE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_part.py tests/test_abi.py > gpurun_out/t_part.log 2>&1 || { tail -30 gpurun_out/t_part.log; exit 1; }
tail -2 gpurun_out/t_part.log
timeout -k 10 200 python -u tools/lat_probe.py --workload c3 --bs 64 --n 150 --reserve > gpurun_out/lat_c3r.log 2>&1 || { tail gpurun_out/lat_c3r.log; exit 1; }
unset SDH_ALLOC_TRACE
timeout -k 10 400 python -u bench.py --workload c3 --no-cpu-baseline --no-ingest > gpurun_out/l_c3.json 2> gpurun_out/l_c3.err || exit 1
