#!/bin/bash
# Round 3: dW GEMM anatomy (tools/kbench/bin/gemm_*: parts removed, numerics broken on purpose)
# + a 1-GPU bench of the current tree.
set -o pipefail
O=gpurun_out/r3anat
mkdir -p $O
for b in gemm_base gemm_nodma gemm_nobar gemm_noread gemm_nosync gemm_bare gemm_base; do
  echo "=== $b" >> $O/all.txt
  timeout -k 5 120 tools/kbench/bin/$b 10 >> $O/all.txt 2>&1 || { echo "rc=$? on $b"; cat $O/all.txt; exit 1; }
done
cat $O/all.txt
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -3 $O/bench.log
