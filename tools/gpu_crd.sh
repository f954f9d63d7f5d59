#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/crd
timeout -k 10 300 python tools/bench_crd_to_step.py --jobs 5 --model llama3-8b --gpus 1 > gpurun_out/crd/gap0.log 2>&1 || { tail -5 gpurun_out/crd/gap0.log; exit 1; }
tail -6 gpurun_out/crd/gap0.log
timeout -k 10 300 python tools/bench_crd_to_step.py --jobs 5 --model llama3-8b --gpus 1 --gap 2 > gpurun_out/crd/gap5.log 2>&1 || { tail -5 gpurun_out/crd/gap5.log; exit 1; }
tail -6 gpurun_out/crd/gap5.log
