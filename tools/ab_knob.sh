# A/B of two sdh_config.debug knob strings on one workload's bench line, alternated A B A B:
#   bash tools/ab_knob.sh <workload> "<knobs A>" "<knobs B>"     (an empty string = the defaults)
# each run's JSON line lands in gpurun_out/abk_<workload>_<run>.json; one summary line per run.
set -o pipefail
mkdir -p gpurun_out
W=$1; A=$2; B=$3
for run in a1 b1 a2 b2; do
  case $run in a*) K=$A ;; *) K=$B ;; esac
  SIDDHI_HIP_DEBUG="$K" timeout -k 10 300 python -u bench.py --workload $W --steps 8 --warmup 2 \
    --no-cpu-baseline --no-ingest --no-latency --no-expansion --no-calibrate \
    > gpurun_out/abk_${W}_$run.json 2> gpurun_out/abk_${W}_$run.err || { tail -20 gpurun_out/abk_${W}_$run.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], repr(sys.argv[3]), d['ms_per_step'], d['roofline']['kernel_ms'])" \
    gpurun_out/abk_${W}_$run.json $run "$K"
done
