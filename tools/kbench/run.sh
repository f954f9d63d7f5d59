#!/bin/bash
# Run microbench binaries in order: run.sh OUTDIR bin1 [bin2 ...]; each under its own limit.
set -o pipefail
out=$1; shift
mkdir -p $out
for b in "$@"; do
  name=$(basename ${b%% *})
  echo "=== $b" | tee -a $out/all.log
  timeout -k 5 90 tools/kbench/bin/$b >> $out/all.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc on $b" | tee -a $out/all.log; exit $rc; fi
done
cat $out/all.log
