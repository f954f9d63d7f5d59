#!/bin/bash
# attention backward pre (delta) / post (fp32 -> bf16 dK/dV) kernels: old vs new, then the GPU tier.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_prepost
mkdir -p $O
for b in fa_oldpp fa_newpp fa_oldpp fa_newpp; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|pre \|post \|bwd_total\|NUMERICS" $O/fa.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/bench_tp_shard.py --seq-len 4096 --micro-batch 4 --steps 3 --warmup 1 --tp-comm-chunks 4 --tp-dual-batch 0 > $O/tp.log 2>&1 || { echo "tp rc=$?"; tail -20 $O/tp.log; exit 1; }
grep '^{' $O/tp.log | tail -1 | cut -c1-200
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-260
