#!/bin/bash
# GPU tests -> 1-GPU training bench -> CRD-to-first-step (Llama-3-8B, 1 GPU) -> MNIST CPU plumbing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
timeout -k 10 420 python -m pytest tests -x -q -m gpu > gpurun_out/s2/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s2/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --steps 8 --warmup 3 > gpurun_out/s2/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/s2/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_crd_to_step.py --jobs 5 --model llama3-8b --gpus 1 > gpurun_out/s2/crd2step_8b.log 2>&1
rc=$?; echo "crd2step rc=$rc"; tail -6 gpurun_out/s2/crd2step_8b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_crd_to_step.py --jobs 3 --model mnist --gpus 0 --nodes 2 > gpurun_out/s2/crd2step_mnist.log 2>&1
rc=$?; tail -1 gpurun_out/s2/crd2step_mnist.log; exit $rc
