#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: 2 ranks on device 0 over gloo (the driver's 8-GPU runs use
# RCCL, one rank per GPU). Strong scaling (the metric's 10K patterns split over the ranks) with the
# weak-scaling line, and the expansion leg's gather + k-way merge timed per matched tuple.
# Usage: tools/multi.sh [c2] [c3] [c4]
set -o pipefail
mkdir -p gpurun_out
export SDH_BENCH_BACKEND=gloo SDH_BENCH_DEVICE=0
port=29612
for wl in "${@:-c2 c4 c3}"; do
  case $wl in
    c2) extra="--batch 1048576" ;;
    c3) extra="--workload c3 --batch 262144" ;;
    c4) extra="--workload c4 --batch 262144" ;;
  esac
  port=$((port + 1))
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --expansion-batch 4096 $extra \
    > gpurun_out/multi_$wl.log 2> gpurun_out/multi_$wl.err || { tail -20 gpurun_out/multi_$wl.err; exit 1; }
  tail -1 gpurun_out/multi_$wl.log | cut -c1-900
done
