#!/bin/bash
# A/B on one box: activation-gradient GEMMs on transposed weights (KFAMD_DX_T=1) vs plain.
set -o pipefail
mkdir -p gpurun_out/abdxt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k transpose \
  > gpurun_out/abdxt/test.log 2>&1 || { tail -20 gpurun_out/abdxt/test.log; exit 1; }
tail -1 gpurun_out/abdxt/test.log
i=0
for arm in 1 0 1 0; do
  i=$((i+1))
  KFAMD_DX_T=$arm timeout -k 10 300 python bench.py --steps 8 --warmup 3 > gpurun_out/abdxt/b$arm.$i.log 2>&1 || exit 1
  echo "dxt=$arm $(tail -1 gpurun_out/abdxt/b$arm.$i.log | cut -c100-190)"
done
