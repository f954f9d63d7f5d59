#!/bin/bash
# In-step A/B of the attention backward arrangement: dQ || dK/dV fork on/off x 64-key / 32-key dK/dV kernel
set -o pipefail
O=gpurun_out/r2bwdab
mkdir -p $O
for rep in 1 2; do
  for cfg in "1 64" "0 64" "1 32" "0 32"; do
    set -- $cfg
    KFAMD_FA_BWD_FORK=$1 KFAMD_FA_DKDV=$2 timeout -k 10 200 python bench.py --steps 6 --warmup 2 > $O/b_$1_$2_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc fork=$1 dkdv=$2"; tail -5 $O/b_$1_$2_$rep.log; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open('$O/b_$1_$2_$rep.log').read().strip().splitlines()[-1]); print('fork=$1 dkdv=$2 rep=$rep', d['value'], d['ms_per_step'])"
  done
done
