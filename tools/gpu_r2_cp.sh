#!/bin/bash
# Context parallelism on the GPU: the 2-rank one-GPU numerics test, then a long-context shape
# rehearsal -- Llama-3-8B layers at seq 32768 split over 2 gloo ranks sharing ONE MI355X (2 of
# 32 layers; gloo through the host, so the step time is not a performance number).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r2cp
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parallel_gpu.py -k context_parallel -x -v --timeout 300 --timeout-method thread > $O/cp_test.log 2>&1 && \
tail -3 $O/cp_test.log && \
KFAMD_DIST_BACKEND=gloo OMP_NUM_THREADS=4 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29615 bench.py --gpus 2 --cp --layers 2 --seq-len 32768 --micro-batch 1 \
  --steps 2 --warmup 1 > $O/cp2_32k.log 2>&1 && \
grep '^{' $O/cp2_32k.log | cut -c1-1400
