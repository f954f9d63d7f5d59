#!/bin/bash
# Default-config candidates at the driver's step counts: micro-batch 4 (chunked head) vs 2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2mb4
mkdir -p $O
for mb in 4 2 4; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --micro-batch $mb > $O/bench_mb${mb}_$RANDOM.log 2>&1
  rc=$?; echo "mb $mb rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for f in $O/*.log; do tail -1 $f | cut -c1-120; tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['micro_batch'], d['ms_per_step'], d['value'], d['peak_mem_gib'], d['peak_reserved_gib'])"; done
