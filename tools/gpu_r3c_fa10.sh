#!/bin/bash
# dK/dV flush: LDS-only barriers (no vmcnt wait on the fp32 atomics) vs __syncthreads; stamp anatomy.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa10
mkdir -p $O
for b in fa_lb0 fa_lb1 fa_lb0 fa_lb1 fa_lb0 fa_lb1 fa_stamp; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dkdv\|NUMERICS" $O/fa.txt
