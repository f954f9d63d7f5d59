#!/bin/bash
# Framework vs eager PyTorch training trajectories from identical weights on the GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2traj
mkdir -p $O
timeout -k 10 300 python -u tools/compare_torch_trajectory.py small 4 1024 12 > $O/small.log 2>&1
rc=$?; tail -13 $O/small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/compare_torch_trajectory.py llama3-8b 2 2048 12 > $O/l8b.log 2>&1
rc=$?; tail -13 $O/l8b.log; exit $rc
