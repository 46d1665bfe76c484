# C5 kernel timelines: the round-5 tree vs HEAD with one wave per item (SDH_SLAB_RUN=1) and with runs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c5kt
F="--steps 3 --warmup 2 --no-cpu-baseline --no-ingest --no-latency --no-expansion --no-calibrate"
(cd ab/r5 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d ../../gpurun_out/c5kt/old -o run -- python3 -u bench.py --workload c5 $F) > gpurun_out/c5kt/old.json 2> gpurun_out/c5kt/old.err || { tail -20 gpurun_out/c5kt/old.err; exit 1; }
SIDDHI_HIP_DEBUG="SDH_SLAB_RUN=1" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5kt/new1 -o run -- python3 -u bench.py --workload c5 $F > gpurun_out/c5kt/new1.json 2> gpurun_out/c5kt/new1.err || { tail -20 gpurun_out/c5kt/new1.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5kt/new -o run -- python3 -u bench.py --workload c5 $F > gpurun_out/c5kt/new.json 2> gpurun_out/c5kt/new.err || { tail -20 gpurun_out/c5kt/new.err; exit 1; }
ls gpurun_out/c5kt/*
