#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/mb
timeout -k 10 420 python bench.py --steps 6 --warmup 2 --micro-batch 3 > gpurun_out/mb/mb3.log 2>&1; rc=$?; tail -1 gpurun_out/mb/mb3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --steps 4 --warmup 2 --micro-batch 2 --grad-accum 2 > gpurun_out/mb/ga2.log 2>&1; rc=$?; tail -1 gpurun_out/mb/ga2.log; exit $rc
