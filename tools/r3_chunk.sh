#!/bin/bash
# ring-mode output reservations per SDH_RING_CHUNK buffers (C3 / C4 benches run in ring mode)
set -o pipefail
mkdir -p gpurun_out
b() {  # b <VAR=value> <workload>
  env "$1" timeout -k 10 300 python -u bench.py --workload $2 --steps 4 --warmup 1 --no-expansion --no-ingest --no-latency --no-cpu-baseline > gpurun_out/ch.log 2> gpurun_out/ch.err || { tail -20 gpurun_out/ch.err; exit 1; }
  echo "$1 $2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ch.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ch.log)"
}
for c in 1 4 16; do b SDH_RING_CHUNK=$c c3; done
for c in 1 4 16; do b SDH_RING_CHUNK=$c c4; done
b SDH_KPART_OUTW=1024 c3
env SDH_RING_CHUNK=16 SDH_KPART_OUTW=1024 true && b SDH_RING_CHUNK=16 c3
