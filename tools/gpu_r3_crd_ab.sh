#!/bin/bash
# Round 3: CRD-to-first-step A/B of the trainer entry's first-use warm-up thread (KFAMD_WARM=1 vs 0),
# control plane as processes, 5 jobs each, alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3crd
mkdir -p $O
for r in 1 2; do
  for w in 0 1; do
    KFAMD_WARM=$w timeout -k 10 300 python tools/bench_crd_to_step.py --jobs 5 --processes > $O/w${w}_$r.log 2>&1 || { echo "rc=$? w=$w"; tail -20 $O/w${w}_$r.log; exit 1; }
    echo "KFAMD_WARM=$w round $r: $(tail -1 $O/w${w}_$r.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["p50_s"], r["per_job_s"], r["breakdown_p50_s"])')"
  done
done
