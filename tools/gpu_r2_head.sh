#!/bin/bash
# Chunked LM head (K5) + bench-shape attention numerics; then bench: head chunk 4096 vs whole
# micro-batch at mb 2, and micro-batch 3 / 4 with the chunked head.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2head
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_model_gpu.py tests/test_attention_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for args in "--head-chunk 4096" "--head-chunk 0" "--micro-batch 3" "--micro-batch 4"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 $args > $O/bench_$tag.log 2>&1
  rc=$?; echo "bench $args rc=$rc"; tail -1 $O/bench_$tag.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
