#!/bin/bash
# multi-rank rehearsal on a 1-GPU box: 2 ranks on device 0 over gloo (the driver's 8-GPU runs use
# RCCL, one rank per GPU). Usage: tools/r2_multi.sh [c2] [c5]
set -o pipefail
mkdir -p gpurun_out
export SDH_BENCH_BACKEND=gloo SDH_BENCH_DEVICE=0
port=29512
for wl in "${@:-c2 c5}"; do
  case $wl in
    c2) extra="--batch 1048576" ;;
    c5) extra="--workload c5 --batch 16384" ;;
  esac
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline $extra > gpurun_out/multi_$wl.log 2>&1 \
    || { tail -20 gpurun_out/multi_$wl.log; exit 1; }
  tail -1 gpurun_out/multi_$wl.log | cut -c1-700
done
