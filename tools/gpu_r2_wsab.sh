#!/bin/bash
# hipBLASLt workspace size A/B on the training bench (default vs 256 MiB), alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2wsab
mkdir -p $O
for r in 1 2; do
  for ws in default 262144; do
    if [ $ws = default ]; then unset HIPBLASLT_WORKSPACE_SIZE; else export HIPBLASLT_WORKSPACE_SIZE=$ws; fi
    timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/bench_$ws.$r.log 2>&1
    rc=$?; echo "ws=$ws round $r: $(tail -1 $O/bench_$ws.$r.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
  done
done
