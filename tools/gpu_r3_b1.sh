#!/bin/bash
# Round 3: dW ring-depth / stagger variants, then bench.py with the CRD-to-first-step phase.
set -o pipefail
O=gpurun_out/r3b1
mkdir -p $O
OUT=r3b1 bash tools/gpu_r3_gemm.sh gemm_base gemm_st gemm_n5 gemm_n5st gemm_base gemm_st gemm_n5 gemm_n5st > /dev/null || exit 1
grep "===\|per step" $O/all.txt
timeout -k 10 600 python bench.py --steps 4 --warmup 2 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -40 $O/bench.log; exit 1; }
grep crd_job $O/bench.log; tail -1 $O/bench.log
