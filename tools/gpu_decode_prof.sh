#!/bin/bash
# decode check + B=1 decode bench + rocprofv3 kernel stats of a B=1 decode run
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/dec}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_serve.py --batches ${BATCHES:-1,8} > $OUT/bench.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_serve.py --batches 1 --steps 16 > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-5
