#!/bin/bash
# A/B the training bench: hipBLASLt heuristics vs the committed TunableOp results file.
set -o pipefail
mkdir -p gpurun_out/tune
F=service_account_auth_improvements_amd/runtime/tuned/tunableop_gfx950.csv
for arm in default tuned default tuned; do
  if [ $arm = tuned ]; then export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$F; \
  else unset PYTORCH_TUNABLEOP_ENABLED PYTORCH_TUNABLEOP_TUNING PYTORCH_TUNABLEOP_FILENAME; fi
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/tune/bench_$arm.log 2>&1 || exit 1
  echo "$arm $(tail -1 gpurun_out/tune/bench_$arm.log | cut -c100-200)"
done
