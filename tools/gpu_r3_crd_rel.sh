#!/bin/bash
# Round 3: CRD-to-first-step A/B of the between-jobs device-release wait (KFAMD_CRD_RELEASE_WAIT=1 vs 0),
# control plane as processes, 6 jobs each, alternating.  Also records the sysfs VRAM counters seen.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3crdrel
mkdir -p $O
python -c 'from service_account_auth_improvements_amd import crdbench; print("vram_used", crdbench._vram_used())' > $O/sysfs.txt 2>&1
cat $O/sysfs.txt
for r in 1 2; do
  for w in 1 0; do
    KFAMD_CRD_RELEASE_WAIT=$w timeout -k 10 300 python tools/bench_crd_to_step.py --jobs 6 --processes > $O/rel${w}_$r.log 2>&1 || { echo "rc=$? w=$w"; tail -20 $O/rel${w}_$r.log; exit 1; }
    echo "RELEASE_WAIT=$w round $r: $(tail -1 $O/rel${w}_$r.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["p50_s"], r["p90_s"], r["per_job_s"], r.get("device_release_wait_s"))')"
  done
done
