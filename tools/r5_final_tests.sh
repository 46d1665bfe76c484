set -o pipefail
bash tools/gpu_tests.sh gpu_suite tests --durations=15 > /dev/null || { tail -30 gpurun_out/gpu_suite.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_suite.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
