#!/bin/bash
# fp32 DP reduction: RCCL one-rank test, kernel tests, 2-rank GPU DP tests, and the bench cost
# of fp32 vs bf16 micro-batch accumulation on one GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2fp32
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rccl_gpu.py tests/test_kernels_gpu.py tests/test_custom_ar_gpu.py tests/test_parallel_gpu.py tests/test_serving_tp_gpu.py tests/test_attention_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in fp32 bf16; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --micro-batch 1 --grad-accum 2 --grad-reduce $m > $O/bench_ga2_$m.log 2>&1
  rc=$?; echo "bench $m rc=$rc"; tail -1 $O/bench_ga2_$m.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log; exit $rc
