#!/bin/bash
# Round 3 closing evidence on the final tree: GPU tier + smoke, attention microbench (B4/B2),
# driver-shaped bench, rocprofv3 step profile, 70B TP=8 shard step, serving decode/prefill.
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3c_final
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for B in 4 2; do
  echo "=== fa B$B S8192" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/fa_pipe $B 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "fa rc=$?"; cat $O/fa.txt; exit 1; }
done
grep "===\|fwd\|dq \|dkdv\|total\|NUMERICS" $O/fa.txt
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-330
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 --crd-jobs 0 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -30 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f 5 > $O/summary.md
cp $f $O/kernel_stats.csv
head -16 $O/summary.md
timeout -k 10 300 python -u tools/bench_tp_shard.py --seq-len 4096 --micro-batch 4 --steps 4 --warmup 2 --tp-comm-chunks 4 --tp-dual-batch 0 > $O/tp.log 2>&1 || { echo "tp rc=$?"; tail -20 $O/tp.log; exit 1; }
grep '^{' $O/tp.log | tail -1
timeout -k 10 400 python -u tools/bench_serve.py --batches 1,8,32,64,128 --steps 32 > $O/serve.log 2>&1 || { echo "serve rc=$?"; tail -20 $O/serve.log; exit 1; }
grep '^{' $O/serve.log | cut -c1-160
