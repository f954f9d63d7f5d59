#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2accum
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_model_gpu.py -k "accumulation" > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; exit $rc
