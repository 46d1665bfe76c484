# C3 expansion leg (64K-event pushes + device poll) under a kernel trace, with buffer growth traced
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c3exp; mkdir -p $OUT
SDH_ALLOC_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --no-latency > $OUT/line.json 2> $OUT/line.err || { tail -5 $OUT/line.err; exit 1; }
grep -E "expansion|compact" $OUT/line.err | tail -12
