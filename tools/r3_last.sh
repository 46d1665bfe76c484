#!/bin/bash
# what the driver runs at round end, at HEAD: smoke() then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last_smoke.log 2>&1 || { tail -20 gpurun_out/last_smoke.log; exit 1; }
tail -3 gpurun_out/last_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/last_bench.log 2> gpurun_out/last_bench.err || { tail -20 gpurun_out/last_bench.err; exit 1; }
tail -1 gpurun_out/last_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], json.dumps(d['roofline'])[:500])"
