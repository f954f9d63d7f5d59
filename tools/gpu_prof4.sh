#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
PROF_OUT=gpurun_out/s4/prof bash tools/gpu_prof.sh --steps 3 --warmup 2 || exit 1
f=$(find gpurun_out/s4/prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 5 > gpurun_out/s4/prof_summary.md
head -16 gpurun_out/s4/prof_summary.md
timeout -k 10 420 python bench.py --steps 10 --warmup 3 > gpurun_out/s4/bench.log 2>&1
rc=$?; tail -1 gpurun_out/s4/bench.log | cut -c1-300; exit $rc
