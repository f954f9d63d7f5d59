#!/bin/bash
# Round-2 closing GPU session (re-entry session, row-tiled SwiGLU default): full GPU tier, smoke(), default bench, rocprofv3 step summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2final2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $O/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 tools/prof_summary.py $f 5 > $O/summary.md; head -16 $O/summary.md
