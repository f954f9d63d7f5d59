#!/bin/bash
# Round 3 closing measurements: attention microbench rows at B2/B4 S8192 (HBM-cold inputs), then a
# rocprofv3 kernel-trace + stats of the 1-GPU bench step, summarised per category.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3prof
mkdir -p $O
for B in 2 4; do
  echo "=== fa B$B S8192" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/fa_base $B 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "fa rc=$?"; cat $O/fa.txt; exit 1; }
done
cat $O/fa.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 --crd-jobs 0 > $O/bench.log 2>&1 || { echo "prof rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f 5 > $O/summary.md
cp $f $O/kernel_stats.csv
head -20 $O/summary.md
