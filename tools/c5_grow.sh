# C5 ring growth factor sweep (SDH_SLAB_GROW_TO) under a kernel trace: slab_move share, reserved/live
set -o pipefail
export TMPDIR=/tmp
for g in $*; do
  OUT=gpurun_out/c5g_$g; mkdir -p $OUT
  SDH_SLAB_GROW_TO=$g timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload c5 --no-cpu-baseline --no-calibrate > $OUT/line.json 2> $OUT/line.err || { tail -5 $OUT/line.err; exit 1; }
  echo "grow_to $g"; grep -E "timed|warm-up step 12" $OUT/line.err; sed -n 2,3p $OUT/trace/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-20,80-200
done
