#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/dbg
timeout -k 10 300 python -u tools/stress_car.py > gpurun_out/dbg/car.log 2>&1; rc=$?
grep -v -E "Gloo|amdgpu|socket.cpp" gpurun_out/dbg/car.log | tail -20; exit $rc
