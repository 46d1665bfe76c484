#!/bin/bash
# K_part check + measure: its GPU tests, the C3 golden, the C3 bench line, the traffic probe
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_part.py "tests/test_gpu_golden.py::test_large_golden_full_config[c3]" tests/test_gpu_chunk.py tests/test_gpu_xch.py tests/test_gpu_compact.py tests/test_gpu_persistence.py > gpurun_out/part_tests.log 2>&1 || { tail -30 gpurun_out/part_tests.log; exit 1; }
tail -2 gpurun_out/part_tests.log
timeout -k 10 300 python -u bench.py --workload c3 --steps 6 --warmup 2 --no-cpu-baseline --no-expansion --no-ingest --no-latency > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err || exit 1
grep timed gpurun_out/b_c3.err
tools/c3_probe.sh gpurun_out/${1:-c3probe}
