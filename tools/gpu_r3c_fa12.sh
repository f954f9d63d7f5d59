#!/bin/bash
# dK/dV persistent grid (static-stride item loop; 2 or 4 workgroups per CU) vs one workgroup per item.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa12
mkdir -p $O
for b in fa_ref fa_ps2 fa_ps4 fa_ref fa_ps2 fa_ps4; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dkdv\|NUMERICS" $O/fa.txt
