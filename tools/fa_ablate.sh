#!/bin/bash
set -o pipefail
timeout -k 10 120 python tools/bench_attn.py 8192 2>&1 | grep bwd
KF_FA_DBG=1 timeout -k 10 120 python tools/bench_attn.py 8192 2>&1 | grep bwd
