#!/bin/bash
# dK/dV kernel variants (microbench timings + numerics), optional PMC pass on the first
set -o pipefail
out=gpurun_out/${OUT:-r2fa64x}
mkdir -p $out
for b in "$@"; do
  echo "=== $b" >> $out/all.txt
  timeout -k 5 120 tools/kbench/bin/$b >> $out/all.txt 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "rc=$rc" >> $out/all.txt; cat $out/all.txt; exit $rc; fi
done
cat $out/all.txt
if [ -n "$PMC" ]; then bash tools/kbench/pmc.sh $out/pmc $1; fi
