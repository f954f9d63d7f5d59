#!/bin/bash
# dK/dV variants (ss-major fragment order, s_setprio), PMC of the pipelined build, 1-GPU bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa2
mkdir -p $O
for b in fa_pipe fa_ssm fa_prio fa_both fa_pipe fa_ssm fa_prio fa_both; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dq \|dkdv\|total\|NUMERICS" $O/fa.txt
bash tools/kbench/pmc.sh $O/pmc fa_pipe 4 8192 32 8 3 0 || { echo "pmc rc=$?"; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
