# C5 line with per-pass traces (re-runs, output words), HEAD vs the round-5 tree
set -o pipefail
mkdir -p gpurun_out/c5trace
F="--steps 4 --warmup 2 --no-cpu-baseline --no-ingest --no-latency --no-expansion --no-calibrate"
SIDDHI_HIP_DEBUG="SDH_TRACE=1;SDH_SLAB_TRACE=1" timeout -k 10 300 python -u bench.py --workload c5 $F > gpurun_out/c5trace/new.json 2> gpurun_out/c5trace/new.err || { tail -20 gpurun_out/c5trace/new.err; exit 1; }
(cd ab/r5 && SDH_TRACE=1 SDH_SLAB_TRACE=1 timeout -k 10 300 python -u bench.py --workload c5 $F) > gpurun_out/c5trace/old.json 2> gpurun_out/c5trace/old.err || { tail -20 gpurun_out/c5trace/old.err; exit 1; }
grep -c "gen pass" gpurun_out/c5trace/new.err
grep "attempt [1-9]" gpurun_out/c5trace/new.err | tail -5
tail -3 gpurun_out/c5trace/new.err gpurun_out/c5trace/old.err
