#!/bin/bash
# Round 3: compute cost of the TP forward-overlap forms on one TP=8 rank's share of a Llama-3-70B
# step (tools/bench_tp_shard.py, one-rank group: the collectives are local copies, so this
# isolates what chunking / half-batch interleaving costs in GEMM efficiency).
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${TP_OUT:-r3tp2}
mkdir -p $O
for cfg in ${TP_CFGS:-"4 0" "4 1" "4 0" "4 1"}; do
  set -- $cfg
  echo "=== chunks=$1 dual=$2" >> $O/all.log
  timeout -k 10 300 python -u tools/bench_tp_shard.py --seq-len 4096 --micro-batch 4 --steps 4 --warmup 2 \
    --tp-comm-chunks $1 --tp-dual-batch $2 >> $O/all.log 2>&1 || { echo "rc=$? chunks=$1 dual=$2"; tail -20 $O/all.log; exit 1; }
  grep '^{' $O/all.log | tail -1
done
