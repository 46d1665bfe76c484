# round-5 tree (ab/r5, built from b1fbf31) against HEAD on one box: the C5 and C3 lines, alternated
set -o pipefail
mkdir -p gpurun_out/r5vs6
F="--steps 8 --warmup 2 --no-cpu-baseline --no-ingest --no-latency --no-expansion --no-calibrate"
for w in c5 c3; do
  for run in old1 new1 old2 new2; do
    case $run in old*) D=ab/r5 ;; *) D=. ;; esac
    (cd $D && timeout -k 10 300 python -u bench.py --workload $w $F) > gpurun_out/r5vs6/${w}_$run.json 2> gpurun_out/r5vs6/${w}_$run.err || { tail -20 gpurun_out/r5vs6/${w}_$run.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/r5vs6/${w}_$run.json $w $run
  done
done
bash tools/ab_knob.sh c5 "" "SDH_SLAB_PREFETCH=1"
