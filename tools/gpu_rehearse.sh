#!/bin/bash
# 2 ranks on ONE GPU over gloo: exercises the multi-rank DDP / ZeRO-1 code paths with real GPU
# tensors and streams (not a performance measurement: both ranks share the device).
set -o pipefail
mkdir -p gpurun_out/rehearse
export KFAMD_DIST_BACKEND=gloo
for mode in --zero1 --no-zero1; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29631 bench.py --gpus 2 --steps 2 --warmup 1 --layers 2 --seq-len 2048 --micro-batch 1 $mode \
    > gpurun_out/rehearse/bench$mode.log 2>&1 || { tail -20 gpurun_out/rehearse/bench$mode.log; exit 1; }
  grep metric gpurun_out/rehearse/bench$mode.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$mode', d['config']['optimizer_sharding'], d['loss_first'], d['loss_last'])"
done
