"""CRD-to-first-step latency (the second half of BASELINE.json's metric).

Brings up the LocalCluster with an exec kubelet (pods are processes on this node, GPUs
handed out by the amd.com/gpu device plugin as HIP_VISIBLE_DEVICES), then submits N
PyTorchJobs one after another and measures, per job, the wall-clock time from the CR
``create`` call to the first completed optimizer step reported by rank 0 of the job
(the worker's ``first_step`` event).  Breakdown: CR -> pod Running (control plane),
pod -> worker process start (kfamd-launch + Python), process -> init done (torch import,
RCCL init, model allocation + init), init -> first step (first train step incl. kernel
loads / hipBLASLt heuristics).  Prints one JSON line with p50/p90 and the breakdown.

  python tools/bench_crd_to_step.py --jobs 5 --model llama3-8b --gpus 1
  python tools/bench_crd_to_step.py --jobs 3 --model mnist --gpus 0 --nodes 2   # configs[0]
  python tools/bench_crd_to_step.py --processes ...   # apiserver / controller-manager /
      # kubelet(s) as separate processes over HTTP (cluster.ProcessCluster): the job CR, its
      # pods and their status travel through the REST API and watches as on a real cluster
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=5)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--gpus", type=int, default=1, help="GPUs per node (nprocPerNode)")
    ap.add_argument("--nodes", type=int, default=1, help="replicas (Master + Workers)")
    ap.add_argument("--seq-len", type=int, default=8192)
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=300)
    ap.add_argument("--gap", type=float, default=0.0, help="idle seconds between jobs (GPU memory settle)")
    ap.add_argument("--kind", choices=["pytorchjob", "mpijob"], default="pytorchjob",
                    help="mpijob: an upstream-style MPIJob (Launcher mpirun -np G, Worker with G GPUs)")
    ap.add_argument("--processes", action="store_true",
                    help="control plane and node agents as separate processes over HTTP (one kubelet per node)")
    ap.add_argument("--poll", type=float, default=None, help="measuring loop period (s); default 0.05")
    a = ap.parse_args()
    from service_account_auth_improvements_amd.crdbench import measure
    out = measure(jobs=a.jobs, model=a.model, gpus=a.gpus, nodes=a.nodes, seq_len=a.seq_len,
                  micro_batch=a.micro_batch, layers=a.layers, device="cuda" if a.gpus else "cpu", kind=a.kind,
                  processes=a.processes, gap=a.gap, timeout=a.timeout, poll=a.poll, log=lambda s: print(s, flush=True))
    print(json.dumps({"metric": "CRD-to-first-step", "gap_s": a.gap, **out}), flush=True)


if __name__ == "__main__":
    main()
