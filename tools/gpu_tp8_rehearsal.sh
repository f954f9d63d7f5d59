#!/bin/bash
# 70B TP=8 code path on ONE GPU: 8 ranks share the card over gloo (RCCL refuses shared devices),
# 2 of the 80 layers (debug override), seq 2048 -- exercises every HIP kernel at the 70B TP=8
# shard shapes (8 q heads / 1 kv head per rank, FFN shard 3584, vocab shard 16032) plus the TP
# collectives.  Not a performance number.
set -o pipefail
export TMPDIR=/tmp KFAMD_DIST_BACKEND=gloo OMP_NUM_THREADS=2
mkdir -p gpurun_out/tp8
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 8 --model llama3-70b --tp 8 --layers 2 --seq-len 2048 --micro-batch 1 \
  --steps 2 --warmup 1 > gpurun_out/tp8/bench.log 2>&1
rc=$?; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/tp8/bench.log | tail -3; exit $rc
