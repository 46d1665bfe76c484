# K_seq items per launch (SDH_SEQ_WAVES) on the C4 line
set -o pipefail
for w in $*; do
  SDH_SEQ_WAVES=$w timeout -k 10 300 python -u bench.py --workload c4 --steps 6 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency --no-calibrate > gpurun_out/sq_$w.json 2> gpurun_out/sq_$w.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sq_$w.json')); print('$w', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
