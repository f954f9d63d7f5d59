#!/bin/bash
# Validate a restored tree on one MI355X: gpu tests -> smoke() -> 1-GPU bench.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/validate}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log; exit $rc
