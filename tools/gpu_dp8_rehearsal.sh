#!/bin/bash
# 8-rank ZeRO-1 data-parallel training on ONE GPU: 8 ranks share the card over gloo (RCCL refuses
# shared devices), 2 of the 32 Llama-3-8B layers (debug override), seq 2048 -- exercises the
# bucketed reduce-scatter / sharded AdamW / overlapped all-gather path with 8 ranks on the HIP
# kernels.  Not a performance number (the driver measures N = 1..8 over RCCL on an 8-GPU node).
set -o pipefail
export TMPDIR=/tmp KFAMD_DIST_BACKEND=gloo OMP_NUM_THREADS=2
mkdir -p gpurun_out/dp8
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29612 bench.py --gpus 8 --model llama3-8b --layers 2 --seq-len 2048 --micro-batch 1 \
  --steps 2 --warmup 1 > gpurun_out/dp8/bench.log 2>&1
rc=$?; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/dp8/bench.log | tail -3; exit $rc
