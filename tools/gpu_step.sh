#!/bin/bash
# Full GPU test suite, then the 1-GPU Llama-3-8B bench (output dir: gpurun_out/$1).
set -o pipefail
D=gpurun_out/${1:-step}
mkdir -p $D
python -c "from service_account_auth_improvements_amd.ops import _build; _build.build()" || exit 1
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $D/pytest.log 2>&1
rc=$?; tail -3 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --steps 10 --warmup 3 > $D/bench.log 2>&1
rc=$?; tail -1 $D/bench.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
