#!/bin/bash
# After the in-place RCCL parameter all-gather + memory-plan micro-batch: the one-rank RCCL test,
# then the ZeRO-1 fp32 rehearsal at the auto micro-batch (3 at world 1) next to plain mb 3.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2rehearse2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 240 --timeout-method thread > $O/rccl_test.log 2>&1 && \
tail -3 $O/rccl_test.log && \
timeout -k 10 420 python -u bench.py --steps 5 --warmup 2 --force-collectives > $O/zero1_fp32_auto.log 2>&1 && \
grep '^{' $O/zero1_fp32_auto.log && \
timeout -k 10 420 python -u bench.py --steps 5 --warmup 2 --force-collectives --micro-batch 2 > $O/zero1_fp32_mb2.log 2>&1 && \
grep '^{' $O/zero1_fp32_mb2.log
