#!/bin/bash
# configs[4] proxy: one TP=8 rank's share of a Llama-3-70B step (all 80 layers) on one MI355X.
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2tpshard
mkdir -p $O
timeout -k 10 400 python -u tools/bench_tp_shard.py --seq-len 4096 --micro-batch 1 > $O/mb1.log 2>&1
rc=$?; grep '^{' $O/mb1.log || tail -20 $O/mb1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_tp_shard.py --seq-len 4096 --micro-batch 4 > $O/mb4.log 2>&1
rc=$?; grep '^{' $O/mb4.log || tail -5 $O/mb4.log; exit $rc
