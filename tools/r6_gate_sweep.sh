# K_gate items per launch (SDH_RATCHET_WAVES via sdh_config.debug): is the reverse-scan warm-up the cost?
set -o pipefail
for w in 1024 4096 16384 65536; do
  SIDDHI_HIP_DEBUG="SDH_RATCHET_WAVES=$w" timeout -k 10 200 python -u bench.py --workload c2x --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-latency --no-expansion --no-calibrate > gpurun_out/gs_$w.json 2> gpurun_out/gs_$w.err || { tail -5 gpurun_out/gs_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/gs_$w.json')); print('$w', round(d['ms_per_step'],1), d['value'])"
done
C2X_KERNEL=nfa_gate_kernel bash tools/prof.sh r6 c2x || exit 1
