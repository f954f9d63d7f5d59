#!/bin/bash
# Full-size rehearsal of the N > 1 data-parallel path on one MI355X: Llama-3-8B, mb 4, seq 8192,
# the DP collectives forced on a one-rank RCCL group (bench.py --force-collectives): ZeRO-1 with the
# fp32 reduction (the N > 1 default), ZeRO-1 with bf16 reduce-scatter, and all-reduce DDP (fp32).
# Checks that the multi-GPU configuration fits in HBM at full size and what its collectives cost
# at world 1 (copies only), against the plain 1-GPU bench.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2rehearse
mkdir -p $O
run() {
  local name=$1; shift
  echo "== $name: $*"
  timeout -k 10 420 python -u bench.py --steps 5 --warmup 2 "$@" > $O/$name.log 2>&1
  local rc=$?
  grep '^{' $O/$name.log || tail -20 $O/$name.log
  return $rc
}
# At world 1 the ZeRO-1 fp32 shard buffer is the whole gradient in fp32 (30 GiB) while nothing
# is sharded, so that variant runs at micro-batch 2 next to a plain micro-batch-2 run: the
# difference is the path's extra memory, which shrinks as 1/N on N GPUs (see the log summary).
run plain_mb2 --micro-batch 2 && \
run zero1_fp32_mb2 --force-collectives --zero1 --grad-reduce fp32 --micro-batch 2 && \
run zero1_bf16_mb4 --force-collectives --zero1 --grad-reduce bf16 && \
run ddp_fp32_mb3 --force-collectives --no-zero1 --grad-reduce fp32 --micro-batch 3 && \
run plain_mb3 --micro-batch 3
