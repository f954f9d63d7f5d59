#!/bin/bash
# Round 3: serving A/B of the batched-decode GEMM in the engine (KFAMD_BGEMM=1 vs 0), two rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3bgab
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    echo "## KFAMD_BGEMM=$v round $r" >> $O/ab.txt
    KFAMD_BGEMM=$v timeout -k 10 300 python -u tools/bench_serve.py --batches 32,64,128 --steps 32 > $O/serve_${v}_$r.log 2>&1 \
      || { echo "rc=$? v=$v"; tail -20 $O/serve_${v}_$r.log; exit 1; }
    grep '"decode"' $O/serve_${v}_$r.log >> $O/ab.txt
  done
done
cat $O/ab.txt
