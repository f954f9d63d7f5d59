#!/bin/bash
# Decode at larger batches: skinny MFMA GEMM up to 64 rows vs hipBLASLt beyond 16 rows; kernel profile at B=128
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2serve
mkdir -p $O
for rows in 16 64 16 64; do
  KFAMD_SKINNY_MAX_ROWS=$rows timeout -k 10 300 python tools/bench_serve.py --batches 16,32,64 > $O/serve_rows$rows.log 2>&1
  rc=$?; echo "skinny_max_rows=$rows"; grep '"decode"' $O/serve_rows$rows.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_serve.py --batches 128 --steps 16 > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 tools/prof_summary.py $f 1 > $O/summary.md; head -40 $O/summary.md
