#!/bin/bash
# dK/dV workgroup of 4 vs 8 waves (128 vs 256 keys), B4 and B2 S8192 32/8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa5
mkdir -p $O
for b in fa_w4 fa_w8 fa_w8n fa_w4 fa_w8 fa_w8n; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dkdv\|dq \|NUMERICS" $O/fa.txt
