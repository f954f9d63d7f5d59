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
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mpijob_manifest(name, ns, program, workers, gpus, port):
    from service_account_auth_improvements_amd.controlplane import training
    return training.mpijob_manifest(name, ns, "local", program, workers=workers, gpus_per_worker=gpus,
                                    master_port=port)


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
    a = ap.parse_args()

    from service_account_auth_improvements_amd.cluster import LocalCluster, ProcessCluster
    from service_account_auth_improvements_amd.controlplane import training
    from service_account_auth_improvements_amd.native import build_native
    build_native()
    tmp = tempfile.mkdtemp(prefix="crd2step-")
    events = os.path.join(tmp, "events.jsonl")
    env = {"KFAMD_EVENTS_FILE": events, "OMP_NUM_THREADS": "4"}
    if a.processes:
        cl = ProcessCluster(nodes=a.nodes, gpus_per_node=a.gpus, exec_pods=True, log_dir=tmp, extra_env=env).start()
        client, pod_log = cl.client, cl.pod_log
        client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "bench"}})
    else:
        cl = LocalCluster(n_gpus=a.gpus * a.nodes, exec_pods=True, api_port=None, log_dir=tmp, extra_env=env).start()
        client, pod_log = cl.client, cl.kubelet.pod_log
        cl.server.ensure_namespace("bench")
    dev = "cuda" if a.gpus else "cpu"
    cmd = [sys.executable, "-m", "service_account_auth_improvements_amd", "train", "--model", a.model,
           "--steps", "1", "--device", dev]
    if a.model != "mnist":
        cmd += ["--seq-len", str(a.seq_len), "--micro-batch", str(a.micro_batch)]
    else:
        cmd += ["--micro-batch", "64"]
    if a.layers:
        cmd += ["--layers", str(a.layers)]
    rows = []
    try:
        for j in range(a.jobs):
            if j and a.gap:
                time.sleep(a.gap)
            name = f"job{j}"
            open(events, "w").close()
            if a.kind == "mpijob":
                job = mpijob_manifest(name, "bench", cmd, a.nodes, a.gpus, 29700 + 7 * j)
                rank0_pod = f"{name}-worker-0"
            else:
                job = training.pytorchjob_manifest(name, "bench", "local", cmd, n_nodes=a.nodes,
                                                   gpus_per_node=a.gpus, master_port=29700 + 7 * j)
                if not a.gpus:
                    job["spec"]["nprocPerNode"] = "1"
                rank0_pod = f"{name}-master-0"
            t0 = time.time()
            client.create(job)
            t_running = None
            first = None
            deadline = t0 + a.timeout
            while time.time() < deadline:
                if t_running is None:
                    p = client.get_or_none("v1", "Pod", rank0_pod, "bench")
                    if p and (p.get("status") or {}).get("phase") == "Running":
                        t_running = time.time()
                evs = [json.loads(x) for x in open(events).read().splitlines() if x.strip()]
                fs = [e for e in evs if e["event"] == "first_step" and e.get("rank") == 0]
                if fs:
                    first = fs[0]
                    break
                time.sleep(0.01)
            if first is None:
                log = pod_log("bench", rank0_pod)
                raise SystemExit(f"{name}: no first_step within {a.timeout}s\n{log[-3000:]}")
            r0 = [e for e in evs if e.get("rank") == 0]
            ps = next(e["ts"] for e in r0 if e["event"] == "process_start")
            ini = next(e["ts"] for e in r0 if e["event"] == "init_done")
            imp = next((e["ts"] for e in r0 if e["event"] == "imported"), ps)
            dr = next((e["ts"] for e in r0 if e["event"] == "dist_ready"), imp)
            ie = next(e for e in r0 if e["event"] == "init_done")
            rows.append({"total": first["ts"] - t0, "cr_to_running": (t_running or ps) - t0,
                         "running_to_process": ps - (t_running or ps), "process_to_init": ini - ps,
                         "import": imp - ps, "dist_init": dr - imp, "model_init": ini - dr,
                         "init_to_first_step": first["ts"] - ini,
                         "params_alloc_init": ie.get("params_alloc_init_s", 0.0),
                         "optimizer_state": ie.get("optimizer_state_s", 0.0)})
            print(json.dumps({"job": name, **{k: round(v, 3) for k, v in rows[-1].items()}}), flush=True)
            # wait for the job to finish so the GPUs are free for the next one
            while time.time() < deadline:
                jb = client.get(job["apiVersion"], job["kind"], name, "bench")
                if any(c["type"] in ("Succeeded", "Failed") and c["status"] == "True"
                       for c in (jb.get("status") or {}).get("conditions", [])):
                    break
                time.sleep(0.05)
    finally:
        cl.stop()
    tot = sorted(r["total"] for r in rows)
    out = {"metric": "CRD-to-first-step", "kind": a.kind, "model": a.model, "gpus_per_node": a.gpus,
           "nodes": a.nodes,
           "control_plane": "processes over HTTP" if a.processes else "in-process",
           "gap_s": a.gap,
           "jobs": len(rows), "p50_s": round(statistics.median(tot), 3),
           "p90_s": round(tot[min(len(tot) - 1, int(0.9 * len(tot)))], 3), "min_s": round(tot[0], 3),
           "breakdown_p50_s": {k: round(statistics.median(r[k] for r in rows), 3)
                               for k in ("cr_to_running", "running_to_process", "process_to_init", "import",
                                         "dist_init", "model_init", "params_alloc_init", "optimizer_state",
                                         "init_to_first_step")}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
