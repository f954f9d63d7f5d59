#!/bin/bash
# gpu tests -> smoke -> bench -> rocprofv3 kernel summary (one call); first failure ends it.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/validate}
bash tools/gpu_validate.sh || exit $?
PROF_OUT=$OUT/prof bash tools/gpu_prof.sh --steps 3 --warmup 2 || exit 1
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 5 > $OUT/prof/summary.md
head -16 $OUT/prof/summary.md
