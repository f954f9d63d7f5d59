#!/bin/bash
# Round 3 re-entry: GPU tier (every GPU test + smoke), attention microbench at B4, then the
# driver-shaped 1-GPU bench (CRD jobs + 20 timed steps).
set -o pipefail
export TMPDIR=/tmp
O=${O_TIER:-gpurun_out/r3c_tier}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 5 120 tools/kbench/bin/fa_pipe 4 8192 32 8 10 1 > $O/fa.txt 2>&1 || { echo "fa rc=$?"; cat $O/fa.txt; exit 1; }
cat $O/fa.txt
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
