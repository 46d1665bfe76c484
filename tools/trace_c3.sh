#!/bin/bash
# kernel trace of one C3 / C4 bench run (per-kernel durations)
set -o pipefail
OUT=gpurun_out/${1:-trace}
mkdir -p $OUT
export TMPDIR=/tmp
for w in ${2:-c3}; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$w -o run -- python3 bench.py --no-cpu-baseline --no-expansion --no-ingest --steps 2 --warmup 1 --workload $w > $OUT/$w.log 2>&1 || { echo "trace $w failed"; tail -5 $OUT/$w.log; exit 1; }
python3 - $OUT/$w/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print("%-60s calls %6s avg_ms %8.3f tot_ms %9.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
done
