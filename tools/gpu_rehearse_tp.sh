#!/bin/bash
# Llama-3-70B TP=8 code path rehearsal: 8 ranks on ONE GPU over gloo, 2 layers, short sequence.
# Correctness/plumbing only (all ranks share one device) -- not a performance measurement.
set -o pipefail
mkdir -p gpurun_out/rehearse
export KFAMD_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29641 bench.py --gpus 8 --model llama3-70b --tp 8 --steps 2 --warmup 1 --layers 2 \
  --seq-len 1024 --micro-batch 1 > gpurun_out/rehearse/tp8.log 2>&1 || { tail -30 gpurun_out/rehearse/tp8.log; exit 1; }
grep metric gpurun_out/rehearse/tp8.log | cut -c1-400
