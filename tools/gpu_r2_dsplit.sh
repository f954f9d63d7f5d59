#!/bin/bash
# Decode attention split count at large batches (B = 32, 64, 128, 256; ctx 1024, Lmax 2048)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2dsplit
mkdir -p $O
for B in 32 64 128 256; do
  for s in auto 3 4 6 8 12 16; do
    if [ $s = auto ]; then unset KFAMD_DECODE_SPLITS; else export KFAMD_DECODE_SPLITS=$s; fi
    timeout -k 10 120 python tools/bench_decode_splits.py $B 1024 2048 >> $O/sweep.jsonl 2> $O/err.log
    rc=$?; [ $rc -eq 0 ] || { cat $O/err.log; exit $rc; }
  done
done
cat $O/sweep.jsonl
