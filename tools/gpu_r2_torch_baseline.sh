#!/bin/bash
# Eager PyTorch-ROCm Llama-3-8B training step (tools/bench_torch_baseline.py) at micro-batch 1 and 2,
# next to the framework's bench at the same micro-batches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2torch
mkdir -p $O
timeout -k 10 400 python -u tools/bench_torch_baseline.py --micro-batch 1 --steps 4 --warmup 2 > $O/torch_mb1.log 2>&1
rc=$?; grep '^{' $O/torch_mb1.log || tail -5 $O/torch_mb1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_torch_baseline.py --micro-batch 2 --steps 4 --warmup 2 > $O/torch_mb2.log 2>&1
rc=$?; grep '^{' $O/torch_mb2.log || tail -3 $O/torch_mb2.log
timeout -k 10 300 python -u bench.py --micro-batch 1 --steps 6 --warmup 2 > $O/kfamd_mb1.log 2>&1 && grep '^{' $O/kfamd_mb1.log | cut -c1-400
