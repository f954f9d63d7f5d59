#!/bin/bash
# Round 3: dW GEMM variants (tools/kbench/bin/<names>), alternating; optional PMC of the first.
set -o pipefail
O=gpurun_out/${OUT:-r3gemm}
mkdir -p $O
for b in "$@"; do
  echo "=== $b" >> $O/all.txt
  timeout -k 5 120 tools/kbench/bin/$b 10 >> $O/all.txt 2>&1 || { echo "rc=$? on $b"; cat $O/all.txt; exit 1; }
done
cat $O/all.txt
if [ -n "$PMC" ]; then bash tools/kbench/pmc.sh $O/pmc $PMC 3; fi
