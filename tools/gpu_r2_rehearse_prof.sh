#!/bin/bash
# rocprofv3 kernel trace of the ZeRO-1 fp32 one-rank rehearsal (mb 2) and of the plain mb-2 step.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r2rehprof
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/z1 -o run -- python3 -u bench.py --steps 3 --warmup 2 --force-collectives --micro-batch 2 > $O/z1.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/plain -o run -- python3 -u bench.py --steps 3 --warmup 2 --micro-batch 2 > $O/plain.log 2>&1 && \
grep '^{' $O/z1.log $O/plain.log | cut -c1-300
