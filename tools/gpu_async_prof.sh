#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/async_prof
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 3 --warmup 2 > $OUT/bench.log 2>&1 || exit 1
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python tools/overlap.py $f adamw
