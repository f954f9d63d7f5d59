#!/bin/bash
# 1-GPU bench (driver shape) then a rocprofv3 kernel trace of a short bench, summarised per category.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r3c_step}
mkdir -p $O
timeout -k 5 120 tools/kbench/bin/fa_pipe 4 8192 32 8 10 1 > $O/fa.txt 2>&1 || { echo "fa rc=$?"; cat $O/fa.txt; exit 1; }
grep "fwd\|dq \|dkdv\|total\|NUMERICS" $O/fa.txt
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --crd-jobs 0 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 --crd-jobs 0 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -30 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f 5 > $O/summary.md
cp $f $O/kernel_stats.csv
head -24 $O/summary.md
