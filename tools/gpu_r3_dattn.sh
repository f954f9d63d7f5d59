#!/bin/bash
# Round 3: decode attention bandwidth at serving batches and long contexts (VALU split kernel),
# against the HBM stream of the KV bytes it must read.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3dattn
mkdir -p $O
for cfg in "32 4096 4096" "64 4096 4096" "32 8192 8192" "128 2048 2048" "8 16384 16384"; do
  set -- $cfg
  timeout -k 10 120 python -u tools/bench_decode_splits.py $1 $2 $3 >> $O/dattn.jsonl 2>> $O/err.log || { echo "rc=$? $cfg"; tail -5 $O/err.log; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/r3dattn/dattn.jsonl"):
    r = json.loads(l)
    gb = r["B"] * r["ctx"] * 8 * 128 * 2 * 2 / 1e9
    print(json.dumps({**r, "kv_gb": round(gb, 3), "tb_per_s": round(gb / r["us_per_layer"] * 1e3, 2)}))
PY
