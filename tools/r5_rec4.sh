set -o pipefail
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ratchet.py tests/test_gpu_golden.py "tests/test_gpu_gen.py::test_device_matches_ring_counts_every_record" tests/test_gpu_compact.py > gpurun_out/t_rec4.log 2>&1 || { tail -30 gpurun_out/t_rec4.log; exit 1; }
tail -1 gpurun_out/t_rec4.log
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-ingest --no-latency --no-expansion > gpurun_out/l_rec4.json 2> gpurun_out/l_rec4.err || { tail gpurun_out/l_rec4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/l_rec4.json')); print(d['ms_per_step'], d['value'], d['config']['matches'], d['roofline']['kernel_ms'])"
