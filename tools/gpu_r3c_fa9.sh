#!/bin/bash
# attention forward: ping-pong wave roles (barrier after the S chain for waves 4-7) vs default, B4 and B2 S8192.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa9
mkdir -p $O
for b in fa_ref fa_pp fa_ref fa_pp fa_ref fa_pp; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
for b in fa_ref fa_pp; do
  echo "=== $b B2" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 2 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|fwd\|err\|NUMERICS" $O/fa.txt
