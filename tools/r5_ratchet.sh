set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ratchet.py tests/test_gpu_chunk.py > gpurun_out/t_ratchet.log 2>&1 || { tail -30 gpurun_out/t_ratchet.log; exit 1; }
tail -2 gpurun_out/t_ratchet.log
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-ingest --no-expansion --no-latency > gpurun_out/l_c2r.json 2> gpurun_out/l_c2r.err || { tail gpurun_out/l_c2r.err; exit 1; }
cat gpurun_out/l_c2r.json
