# K_seq per-tile emit (C4): K_seq tests + the C4 golden, the C4 line; C2x on K_chain at 256K-event pushes;
# the C2 profile at HEAD
set -o pipefail
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
echo "cmd: $T tests/test_gpu_gen.py -k seq_windows; tests/test_gpu_golden.py -k c4; tests/test_gpu_records.py" > gpurun_out/r6s2_tests.log
timeout -k 10 600 $T tests/test_gpu_gen.py -k seq_windows tests/test_gpu_records.py >> gpurun_out/r6s2_tests.log 2>&1 || { tail -40 gpurun_out/r6s2_tests.log; exit 1; }
timeout -k 10 600 $T tests/test_gpu_golden.py -k "full_config and c4" >> gpurun_out/r6s2_tests.log 2>&1 || { tail -40 gpurun_out/r6s2_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6s2_tests.log
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --no-ingest --no-latency --no-expansion > gpurun_out/r6s2_c4.json 2> gpurun_out/r6s2_c4.err || { tail -20 gpurun_out/r6s2_c4.err; exit 1; }
tail -2 gpurun_out/r6s2_c4.err
timeout -k 10 300 python -u bench.py --workload c2x --batch 262144 --steps 4 --warmup 1 --no-cpu-baseline --no-ingest --no-latency --no-expansion > gpurun_out/r6s2_c2x.json 2> gpurun_out/r6s2_c2x.err || { tail -20 gpurun_out/r6s2_c2x.err; exit 1; }
tail -2 gpurun_out/r6s2_c2x.err
bash tools/prof.sh r6 c2 || exit 1
