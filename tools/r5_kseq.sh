set -o pipefail
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gen.py tests/test_gpu_compact.py tests/test_gpu_chunk.py tests/test_gpu_xch.py tests/test_gpu_golden.py > gpurun_out/t_kseq.log 2>&1 || { tail -30 gpurun_out/t_kseq.log; exit 1; }
tail -1 gpurun_out/t_kseq.log
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline > gpurun_out/l_c4.json 2> gpurun_out/l_c4.err || { tail gpurun_out/l_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/l_c4.json')); print(d['ms_per_step'], d['value'], d['expansion']['ms_per_step'], d['expansion']['compact']['ms_per_step'], d['push_latency'])"
