#!/bin/bash
# Round 3: batched-decode GEMM (ops/csrc/bgemm.hip) -- numerics tests, then the microbench vs hipBLASLt.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3bgemm
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_serving_gpu.py -k bgemm > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/bench_bgemm.py > $O/bench.jsonl 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.jsonl
