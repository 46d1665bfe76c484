#!/bin/bash
# multi-rank rehearsal on a 1-GPU box: 2 ranks on device 0 over gloo (the driver's 8-GPU runs use
# RCCL, one rank per GPU); C2 headline and the key-sharded C5 family
set -o pipefail
mkdir -p gpurun_out
export SDH_BENCH_BACKEND=gloo SDH_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --batch 1048576 > gpurun_out/multi_c2.log 2>&1 || { tail -20 gpurun_out/multi_c2.log; exit 1; }
tail -1 gpurun_out/multi_c2.log | cut -c1-600
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 2 --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --keys 20000 > gpurun_out/multi_c5.log 2>&1 || { tail -20 gpurun_out/multi_c5.log; exit 1; }
tail -1 gpurun_out/multi_c5.log | cut -c1-600
