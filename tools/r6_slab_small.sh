# K_slab small LDS tier sweep (SDH_SLAB_LDS_SMALL rows; default 1024) on the C5 line, one run each
set -o pipefail
mkdir -p gpurun_out/slab_small
for v in 1024 1536 2048 768 1024; do
  SIDDHI_HIP_DEBUG="SDH_SLAB_LDS_SMALL=$v" timeout -k 10 300 python -u bench.py --workload c5 --steps 8 --warmup 2 \
    --no-cpu-baseline --no-ingest --no-latency --no-expansion --no-calibrate > gpurun_out/slab_small/$v.json 2> gpurun_out/slab_small/$v.err || { tail -20 gpurun_out/slab_small/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/slab_small/$v.json $v
done
