# K_ratchet minimum chunk (SDH_RATCHET_MIN_CHUNK) on the C2 expansion legs (64K-event pushes)
set -o pipefail
for c in $*; do
  SDH_RATCHET_MIN_CHUNK=$c timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-latency --no-calibrate > gpurun_out/mc_$c.json 2> gpurun_out/mc_$c.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/mc_$c.json')); e=d['expansion']; print('$c', round(d['ms_per_step'],2), round(e['push_ms_per_step'],3), round(e['ms_per_step'],3), round(e['compact']['ms_per_step'],3))"
done
