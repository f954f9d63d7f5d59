#!/bin/bash
# Round 3: the driver's GPU tier on the current tree -- every GPU test, then smoke().
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3tier
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
