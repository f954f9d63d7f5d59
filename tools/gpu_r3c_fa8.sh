#!/bin/bash
# dK/dV: 32x32x16 (default) vs 16x16x32 MFMA form, B4 S8192 32/8; numerics vs float64.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa8
mkdir -p $O
for b in fa_m32 fa_m16 fa_m16p0 fa_m32 fa_m16 fa_m16p0; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dkdv\|err\|NUMERICS" $O/fa.txt
