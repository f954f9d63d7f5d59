#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/serve_prof2
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_serve.py --batches 1 --steps 16 > $OUT/bench.log 2>&1 || exit 1
grep decode $OUT/bench.log
