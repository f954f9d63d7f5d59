#!/bin/bash
# One GPU session: gpu tests -> 1-GPU bench -> rocprofv3 kernel stats + summary.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --steps 8 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
PROF_OUT=gpurun_out/prof_full bash tools/gpu_prof.sh --steps 3 --warmup 2 || exit 1
f=$(find gpurun_out/prof_full -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 5 > gpurun_out/prof_full/summary.md
head -20 gpurun_out/prof_full/summary.md
