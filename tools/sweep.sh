#!/bin/bash
# K_ratchet tuning sweep (GPU box): LDS ring depth x waves per launch on the C2 bench.
# SDH_RATCHET_ML / SDH_RATCHET_WAVES override the engine's defaults (8 / CUs x occupancy).
for ml in ${MLS:-8 16}; do
  for w in ${WAVES:-0 4096 8192}; do
    r=$(SDH_RATCHET_ML=$ml SDH_RATCHET_WAVES=$w timeout -k 10 120 python bench.py --no-cpu-baseline --steps 4 2>/dev/null | tail -1) || { echo "fail ml=$ml w=$w"; exit 1; }
    echo "ml=$ml w=$w $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("%.3g %.3f ms" % (d["value"], d["roofline"]["kernel_ms"]))')"
  done
done
