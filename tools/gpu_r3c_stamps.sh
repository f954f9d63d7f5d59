#!/bin/bash
# dK/dV phase anatomy (diagnostic s_memtime build) at B4 S8192 32/8, next to the real kernel's time.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_stamps
mkdir -p $O
for b in fa_pipe fa_stamp; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dkdv\|NUMERICS" $O/fa.txt
