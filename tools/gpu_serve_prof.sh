#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/serve_prof
mkdir -p $OUT
timeout -k 10 400 python tools/bench_serve.py --batches 1,8,32,64,128 > $OUT/bench_full.log 2>&1 || { tail -5 $OUT/bench_full.log; exit 1; }
grep -v amdgpu $OUT/bench_full.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_serve.py --batches 1 --steps 16 > $OUT/bench.log 2>&1 || exit 1
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
head -25 $f | cut -c1-200
