#!/bin/bash
# Round 3: one-pass streaming decode attention -- tests, then kernel A/B (KFAMD_DECODE_STREAM=0/1)
# at serving batches / long contexts and the engine at B = 32-128.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3dattn2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_serving_gpu.py -k "decode_attn" > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 0 1 0 1; do
  for cfg in "32 4096 4096" "64 4096 4096" "32 8192 8192" "128 2048 2048" "8 16384 16384" "8 1024 2048" "64 1024 2048"; do
    set -- $cfg
    KFAMD_DECODE_STREAM=$v timeout -k 10 120 python -u tools/bench_decode_splits.py $1 $2 $3 | sed "s/^{/{\"stream\": $v, /" >> $O/dattn.jsonl 2>> $O/err.log || { echo "rc=$? $cfg"; tail -5 $O/err.log; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3dattn2/dattn.jsonl"):
    r = json.loads(l)
    gb = r["B"] * r["ctx"] * 8 * 128 * 2 * 2 / 1e9
    print(r["stream"], r["B"], r["ctx"], r["us_per_layer"], round(gb / r["us_per_layer"] * 1e3, 2), "TB/s")
PY
for v in 0 1; do
  KFAMD_DECODE_STREAM=$v timeout -k 10 300 python -u tools/bench_serve.py --batches 32,64,128 --steps 32 --ctx 2048 --max-len 4096 > $O/serve_$v.log 2>&1 || { echo "serve rc=$?"; tail -20 $O/serve_$v.log; exit 1; }
  echo "stream=$v"; grep '"decode"' $O/serve_$v.log
done
