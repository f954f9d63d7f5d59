#!/bin/bash
# HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) A/B: decode B=1/8 and the training step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_kernarg
mkdir -p $O
for k in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 300 python -u tools/bench_serve.py --batches 1,8 --steps 48 > $O/serve_k$k.log 2>&1 || { echo "serve rc=$?"; tail -20 $O/serve_k$k.log; exit 1; }
  echo "kernarg=$k"; grep '"decode"' $O/serve_k$k.log | cut -c1-160
done
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --crd-jobs 0 > $O/bench_k$k.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_k$k.log; exit 1; }
  echo "kernarg=$k $(tail -1 $O/bench_k$k.log | cut -c1-170)"
done
