#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench; args passed through to bench.py
set -o pipefail
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py "$@" > $OUT/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -2 $OUT/bench.log
find $OUT -name "*kernel_stats.csv" | head -3
exit $rc
