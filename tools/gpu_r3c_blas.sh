#!/bin/bash
# fwd/dX GEMM library A/B: hipBLASLt (default) vs rocBLAS (TORCH_BLAS_PREFER_HIPBLASLT=0), training step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_blas
mkdir -p $O
for k in 1 0 1 0; do
  TORCH_BLAS_PREFER_HIPBLASLT=$k timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --crd-jobs 0 > $O/bench_lt$k.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_lt$k.log; exit 1; }
  echo "hipblaslt=$k $(tail -1 $O/bench_lt$k.log | cut -c1-200)"
done
