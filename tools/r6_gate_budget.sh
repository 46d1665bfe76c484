# K_gate chunk warm-up budget (SDH_GATE_BUDGET x the batch; 1e9 = the K_ratchet cap) on the C2x line
# with its 64K-push expansion leg; then the gate parity tests at the default
set -o pipefail
mkdir -p gpurun_out/gate_budget
for v in 1e9 4 1e9 4; do
  SIDDHI_HIP_DEBUG="SDH_GATE_BUDGET=$v" timeout -k 10 300 python -u bench.py --workload c2x --steps 4 --warmup 1 \
    --no-cpu-baseline --no-ingest --no-latency --no-calibrate > gpurun_out/gate_budget/$v.json 2> gpurun_out/gate_budget/$v.err || { tail -20 gpurun_out/gate_budget/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['expansion']; print(sys.argv[2], d['ms_per_step'], e['ms_per_step'], e['compact']['ms_per_step'])" gpurun_out/gate_budget/$v.json $v
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gate.py > gpurun_out/gate_budget/tests.log 2>&1 || { tail -30 gpurun_out/gate_budget/tests.log; exit 1; }
tail -1 gpurun_out/gate_budget/tests.log
