#!/bin/bash
# Decode GEMMs at batch 32-256: hipBLASLt heuristic vs TunableOp-tuned solutions (writes the tuned file)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2dtune
mkdir -p $O
timeout -k 10 900 python -u tools/tune_decode_gemm.py $O/tunableop_decode_gfx950.csv 32,64,128,256 > $O/tune.log 2>&1
rc=$?; grep -v amdgpu $O/tune.log | tail -25; exit $rc
