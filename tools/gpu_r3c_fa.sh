#!/bin/bash
# Round 3 (cont.): pipelined dK/dV iteration A/B at the bench shape (B4 S8192 32/8, HBM-cold
# inputs), numerics vs float64 on sampled rows; then the GPU tier and the 1-GPU bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa
mkdir -p $O
for b in fa_old fa_pipe fa_kvonly fa_pa2 fa_old fa_pipe; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|fwd\|dq \|dkdv\|total\|NUMERICS" $O/fa.txt
grep -q "NUMERICS FAIL" $O/fa.txt && { echo "numerics failed"; exit 1; }
bash tools/gpu_r3c_tier.sh
