#!/bin/bash
# dW GEMM microbench + PMC passes (tools/kbench/bin/gemm*)
set -o pipefail
O=gpurun_out/${OUT:-r2gemm}
mkdir -p $O
for b in "$@"; do
  echo "=== $b" >> $O/all.txt
  timeout -k 5 120 tools/kbench/bin/$b >> $O/all.txt 2>&1 || { echo "rc=$? on $b"; cat $O/all.txt; exit 1; }
done
cat $O/all.txt
if [ -n "$PMC" ]; then bash tools/kbench/pmc.sh $O/pmc $1 3; fi
