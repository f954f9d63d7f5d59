#!/bin/bash
# A/B: flash-attention backward with dQ on a forked side stream (KFAMD_FA_BWD_FORK=1, default)
# vs serialised dK/dV -> dQ (=0), alternating arms on one box, after the attention numerics tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fork
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "attn or attention or train or step" --timeout 120 --timeout-method thread > gpurun_out/fork/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/fork/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    KFAMD_FA_BWD_FORK=$f timeout -k 10 300 python bench.py --steps 8 --warmup 3 > gpurun_out/fork/b_${f}_${i}.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/fork/b_${f}_${i}.log; exit $rc; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('fork=$f', d['value'], d['ms_per_step'])" gpurun_out/fork/b_${f}_${i}.log
  done
done
