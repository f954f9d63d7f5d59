#!/bin/bash
# hipBLASLt solution search (PyTorch TunableOp) on the EXACT GEMM signatures of the mb-4 training
# step (fwd, transposed-weight dX, chunked LM head), recorded by running the step itself; then the
# bench with the results file (tuning off) vs the heuristics, alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_tune
mkdir -p $O
export PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=0 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=15 \
       PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=8 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
       PYTORCH_TUNABLEOP_VERBOSE=1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tuned.csv \
  timeout -k 10 1000 python -u bench.py --steps 1 --warmup 1 --crd-jobs 0 > $O/tune.log 2>&1 || { echo "tune rc=$?"; tail -30 $O/tune.log; exit 1; }
ls $O; F=$(ls $O/tuned*.csv | head -1); wc -l $F
for arm in default tuned default tuned; do
  if [ $arm = tuned ]; then
    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/$F PYTORCH_TUNABLEOP_VERBOSE=0 \
      timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --crd-jobs 0 > $O/bench_$arm.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$arm.log; exit 1; }
  else
    PYTORCH_TUNABLEOP_VERBOSE=0 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --crd-jobs 0 > $O/bench_$arm.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$arm.log; exit 1; }
  fi
  echo "$arm $(tail -1 $O/bench_$arm.log | cut -c100-230)"
done
