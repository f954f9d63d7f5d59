#!/bin/bash
# Round 3: attention ring depth A/B (tools/kbench fa_base / fa_n5, bench shape B4 S8192), then
# the GPU tests touched this round and the bench (tools/gpu_r3_b2.sh).
set -o pipefail
O=gpurun_out/r3b3
mkdir -p $O
for b in fa_base fa_n5 fa_base fa_n5; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|fwd\|dq \|dkdv\|total\|NUMERICS" $O/fa.txt
bash tools/gpu_r3_b2.sh
