#!/bin/bash
# rocprofv3 collection for the NFA-step kernel (run on the GPU box from the repo root).
# Kernel trace + stats, then one PMC pass per counter group (gfx950 slot limits: 8 SQ, 4 TCC), each
# pass its own run. Usage: profiles/collect.sh <out-dir> "<bench.py args>" <kernel name>
set -u
OUT=${1:-gpurun_out/prof}
ARGS=${2:-"--steps 2 --warmup 1 --no-cpu-baseline --no-expansion"}
KERNEL=${3:-nfa_ratchet_kernel}
export TMPDIR=/tmp
mkdir -p "$OUT"
python3 -c "import bench; print(bench.source_hash('$KERNEL'))" > "$OUT/source_hash"
echo "$ARGS" > "$OUT/args"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || { echo "trace run failed"; tail -5 "$OUT/trace.log"; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- python3 bench.py $ARGS > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc$i.log"; exit 1; }
done
echo collected
