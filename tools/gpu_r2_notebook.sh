#!/bin/bash
# BASELINE configs[1]: Notebook CR -> notebook server on the MI355X (CR-to-ready), in-process
# control plane and apiserver / controller-manager / kubelet as processes over HTTP.
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2nb
mkdir -p $O
timeout -k 10 400 python -u tools/bench_notebook_ready.py --notebooks 5 --gpus 1 > $O/inproc.log 2>&1
rc=$?; tail -1 $O/inproc.log; [ $rc -eq 0 ] || { tail -20 $O/inproc.log; exit $rc; }
timeout -k 10 400 python -u tools/bench_notebook_ready.py --notebooks 5 --gpus 1 --processes > $O/procs.log 2>&1
rc=$?; tail -1 $O/procs.log; head -1 $O/procs.log | cut -c1-900; exit $rc
