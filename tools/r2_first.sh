set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2a/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2a/gpu_tests.log
timeout -k 10 300 python bench.py --patterns 10000 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r2a/bench10k.log 2>&1 || { tail -20 gpurun_out/r2a/bench10k.log; exit 1; }
tail -1 gpurun_out/r2a/bench10k.log
