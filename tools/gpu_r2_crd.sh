#!/bin/bash
# CRD-to-first-step on the GPU box: in-process control plane vs the platform as separate
# processes over HTTP (apiserver / controller-manager / kubelet), Llama-3-8B, 1 GPU
set -o pipefail
O=gpurun_out/r2crd
mkdir -p $O
timeout -k 10 400 python tools/bench_crd_to_step.py --processes --jobs 5 --model llama3-8b --gpus 1 --gap 2 > $O/processes.log 2>&1 || { tail -20 $O/processes.log; exit 1; }
tail -6 $O/processes.log
timeout -k 10 400 python tools/bench_crd_to_step.py --jobs 5 --model llama3-8b --gpus 1 --gap 2 > $O/inproc.log 2>&1 || { tail -20 $O/inproc.log; exit 1; }
tail -6 $O/inproc.log
