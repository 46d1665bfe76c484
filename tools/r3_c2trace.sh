#!/bin/bash
# Round 3: C2 at 8M-event pushes with the ratchet launch trace (SDH_TRACE) on stderr
set -o pipefail
mkdir -p gpurun_out
SDH_TRACE=1 timeout -k 10 240 python -u bench.py --steps 2 --warmup 2 --no-expansion --no-ingest --no-cpu-baseline > gpurun_out/c2trace.log 2> gpurun_out/c2trace.err
rc=$?
grep -v amdgpu.ids gpurun_out/c2trace.err | tail -20
tail -1 gpurun_out/c2trace.log | cut -c1-600
exit $rc
