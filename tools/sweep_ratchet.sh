# K_ratchet resident-wave target (SDH_RATCHET_WAVES: items per launch ~ this) on the C2 line
set -o pipefail
for w in $*; do
  SDH_RATCHET_WAVES=$w timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency --no-calibrate > gpurun_out/rw_$w.json 2> gpurun_out/rw_$w.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/rw_$w.json')); print('$w', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
