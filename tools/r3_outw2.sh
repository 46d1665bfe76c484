#!/bin/bash
# output-buffer sizes with chunked ring reservations
set -o pipefail
mkdir -p gpurun_out
b() {  # b <VAR=value> <workload>
  env "$1" timeout -k 10 300 python -u bench.py --workload $2 --steps 4 --warmup 1 --no-expansion --no-ingest --no-latency --no-cpu-baseline > gpurun_out/ow.log 2> gpurun_out/ow.err || { tail -20 gpurun_out/ow.err; exit 1; }
  echo "$1 $2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ow.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ow.log)"
}
for w in 768 1024 1536 2048; do b SDH_KPART_OUTW=$w c3; done
for w in 512 768 1024 1536; do b SDH_KSEQ_OUTW=$w c4; done
