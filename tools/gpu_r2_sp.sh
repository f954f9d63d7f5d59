#!/bin/bash
# Sequence parallelism on the GPU: the TP=2 (+SP) one-GPU numerics test, then the 70B TP=8 shard
# shapes (8 gloo ranks sharing ONE MI355X, 2 of 80 layers, seq 4096) with and without --sp --
# per-rank peak memory and the SP collectives at the 70B shard shapes.  Not performance numbers.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r2sp
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parallel_gpu.py -k tensor_parallel -x -v --timeout 300 --timeout-method thread > $O/tp_test.log 2>&1 && \
tail -4 $O/tp_test.log && \
for v in nosp sp; do
  extra=""; [ $v = sp ] && extra="--sp"
  KFAMD_DIST_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 8 --model llama3-70b --tp 8 --layers 2 --seq-len 4096 \
    --micro-batch 1 --steps 2 --warmup 1 $extra > $O/tp8_$v.log 2>&1 || exit $?
  grep '^{' $O/tp8_$v.log | cut -c1-1200
done
