#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
timeout -k 10 420 python bench.py --steps 8 --warmup 3 > gpurun_out/s3/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s3/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_crd_to_step.py --jobs 5 --model llama3-8b --gpus 1 > gpurun_out/s3/crd2step_8b.log 2>&1
rc=$?; tail -6 gpurun_out/s3/crd2step_8b.log; [ $rc -eq 0 ] || exit $rc
PROF_OUT=gpurun_out/s3/prof bash tools/gpu_prof.sh --steps 3 --warmup 2 || exit 1
f=$(find gpurun_out/s3/prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 5 > gpurun_out/s3/prof_summary.md
head -14 gpurun_out/s3/prof_summary.md
