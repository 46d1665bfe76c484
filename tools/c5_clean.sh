# C5 ring policy sweep under a kernel trace: CLEAN_AT:SPAN[:GROW_TO] triples (SDH_SLAB_* env)
set -o pipefail
export TMPDIR=/tmp
for p in $*; do
  IFS=: read ca sp gt <<< "$p"; gt=${gt:-1.6}
  OUT=gpurun_out/c5c_${ca}_${sp}_${gt}; mkdir -p $OUT
  SDH_SLAB_CLEAN_AT=$ca SDH_SLAB_SPAN=$sp SDH_SLAB_GROW_TO=$gt timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload c5 --no-cpu-baseline --no-calibrate > $OUT/line.json 2> $OUT/line.err || { tail -5 $OUT/line.err; exit 1; }
  echo "policy $p"; grep -E "timed" $OUT/line.err
done
