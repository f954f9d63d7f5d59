#!/bin/bash
# Round 3: PMC counters of the decode attention split kernel at B=32, ctx 4096 (what bounds it).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3dpmc
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d $O/p1 -o p1 -- python3 tools/bench_decode_splits.py 32 4096 4096 > $O/p1.log 2>&1 || { echo "p1 rc=$?"; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_MFMA_MOPS_BF16 --output-format csv -d $O/p2 -o p2 -- python3 tools/bench_decode_splits.py 32 4096 4096 > $O/p2.log 2>&1 || { echo "p2 rc=$?"; tail -5 $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d $O/p3 -o p3 -- python3 tools/bench_decode_splits.py 32 4096 4096 > $O/p3.log 2>&1 || { echo "p3 rc=$?"; tail -5 $O/p3.log; exit 1; }
python - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/r3dpmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "decode_split" not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:32s} total {tot[k]:.4g}  per-dispatch {tot[k] / max(1, n[k]):.4g}  (n={n[k]})")
PY
