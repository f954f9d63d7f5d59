#!/bin/bash
# dK/dV 64-keys-per-wave kernel: microbench A/B + numerics, sanitizer harness, attention GPU tests
set -o pipefail
out=gpurun_out/r2fa64
mkdir -p $out
timeout -k 5 120 tools/kbench/bin/fa64 > $out/fa64_new.txt 2>&1 && cat $out/fa64_new.txt &&
KFAMD_FA_DKDV=32 timeout -k 5 120 tools/kbench/bin/fa64 > $out/fa64_old.txt 2>&1 && cat $out/fa64_old.txt &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_native_sanitize.py -m gpu -s > $out/san.log 2>&1 && tail -5 $out/san.log &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_attention_gpu.py -m gpu > $out/attn.log 2>&1 && tail -5 $out/attn.log
