#!/bin/bash
# A/B on one box: grouped dW launches (KFAMD_GROUP_DW=1) vs separate launches, alternating.
set -o pipefail
mkdir -p gpurun_out/abdw
for arm in 1 0 1 0; do  # (arm switch removed after the A/B; kept for the record)
  KFAMD_GROUP_DW=$arm timeout -k 10 300 python bench.py --steps 8 --warmup 3 > gpurun_out/abdw/b$arm.log 2>&1 || exit 1
  echo "group=$arm $(tail -1 gpurun_out/abdw/b$arm.log | cut -c100-190)"
done
