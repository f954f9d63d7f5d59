#!/bin/bash
# Round 3 decode: single-launch decode attention (ticket merge) -- GPU tests, serve bench, and a
# kernel trace of the B=1 decode step (per-kernel times, gaps).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3dec
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_serving_gpu.py > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_serve.py --batches 1,8,32,64 --steps 32 > $O/serve.log 2>&1 || { echo "serve rc=$?"; tail -30 $O/serve.log; exit 1; }
grep '"decode"' $O/serve.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/bench_serve.py --batches 1 --steps 16 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/trace_gaps.py $f decode_attn_kernel 32 | tee $O/gaps.txt
