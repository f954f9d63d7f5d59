"""BASELINE configs[1]: Notebook CR -> notebook server on one MI355X, CR-to-ready latency.

Setup:
* A local cluster with an exec kubelet and an `amd.com/gpu` device plugin. With `--processes`
  the apiserver, controller-manager and kubelet run as separate processes over HTTP.
* A Profile is created first.
* Each Notebook CR uses the notebook controller's StatefulSet / pod path, with NB_PREFIX and
  port 8888 semantics. Its container runs the notebook server stand-in
  (`runtime/notebook_server.py`: the read-only Jupyter REST subset plus a GPU probe).

Timestamps taken for each Notebook, from the CR create:
* the pod is Running;
* the server answers `{NB_PREFIX}/api/status`;
* `{NB_PREFIX}/api/kfamd/gpu` reports the GPU the pod was given, with one timed bf16 matmul;
* the Notebook's status shows `readyReplicas: 1`.

Notebooks are created one after another. Each is deleted before the next, so the single GPU
is handed over. The tool prints one JSON line per notebook and a p50 summary.

  python tools/bench_notebook_ready.py [--notebooks 5] [--gpus 1] [--processes]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import tempfile
import time
import urllib.request

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NS = "nb-bench"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _get(url: str, timeout: float = 2.0):
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status, json.loads(r.read() or b"null")
    except Exception:
        return None, None


def _wait(pred, timeout: float, period: float = 0.02):
    t = time.time()
    while time.time() - t < timeout:
        v = pred()
        if v:
            return v
        time.sleep(period)
    return None


def notebook(name: str, port: int, gpus: int) -> dict:
    ctr = {"name": name, "image": "kfamd/jupyter-pytorch-rocm:latest",
           "command": [sys.executable, "-m", "service_account_auth_improvements_amd", "nb-server"],
           "env": [{"name": "NB_PORT", "value": str(port)}]}
    if gpus:
        ctr["resources"] = {"limits": {"amd.com/gpu": str(gpus)}}
    return {"apiVersion": "kubeflow.org/v1", "kind": "Notebook", "metadata": {"name": name, "namespace": NS},
            "spec": {"template": {"spec": {"containers": [ctr]}}}}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--notebooks", type=int, default=5)
    ap.add_argument("--gpus", type=int, default=1, help="GPUs on the node and per notebook (0 = CPU only)")
    ap.add_argument("--processes", action="store_true", help="control plane as separate processes over HTTP")
    ap.add_argument("--timeout", type=float, default=120)
    a = ap.parse_args(argv)
    from service_account_auth_improvements_amd.cluster import LocalCluster, ProcessCluster
    tmp = tempfile.mkdtemp(prefix="kfamd-nb-")
    if a.processes:
        cl = ProcessCluster(nodes=1, gpus_per_node=a.gpus, exec_pods=True, log_dir=tmp).start()
    else:
        cl = LocalCluster(n_gpus=a.gpus, exec_pods=True, api_port=None, log_dir=tmp).start()
    c = cl.client
    rows = []
    try:
        c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": NS},
                  "spec": {"owner": {"kind": "User", "name": "bench@example.com"}}})
        assert _wait(lambda: c.get_or_none("v1", "ServiceAccount", "default-editor", NS), 60), "profile not ready"
        for i in range(a.notebooks):
            name, port = f"nb{i}", _free_port()
            base = f"http://127.0.0.1:{port}/notebook/{NS}/{name}"
            t0 = time.time()
            c.create(notebook(name, port, a.gpus))
            pod = _wait(lambda: next((p for p in c.list("v1", "Pod", NS)
                                      if p["metadata"]["name"].startswith(name + "-")
                                      and (p.get("status") or {}).get("phase") == "Running"), None), a.timeout)
            t_pod = time.time()
            assert pod, f"{name}: pod never ran"
            ok = _wait(lambda: _get(base + "/api/status")[0] == 200, a.timeout)
            t_http = time.time()
            assert ok, f"{name}: server never answered"
            code, gpu = _get(base + "/api/kfamd/gpu", timeout=120)
            t_gpu = time.time()
            ready = _wait(lambda: ((c.get("kubeflow.org/v1", "Notebook", name, NS).get("status") or {})
                                   .get("readyReplicas") == 1), a.timeout)
            t_ready = time.time()
            code_k, kernels = _get(base + "/api/kernels")
            env = {e["name"]: e.get("value") for e in pod["spec"]["containers"][0].get("env") or []}
            row = {"notebook": name, "cr_to_pod_running_s": round(t_pod - t0, 3),
                   "cr_to_server_http_s": round(t_http - t0, 3), "cr_to_gpu_probe_s": round(t_gpu - t0, 3),
                   "cr_to_ready_status_s": round(t_ready - t0, 3), "ready": bool(ready),
                   "nb_prefix": env.get("NB_PREFIX"), "kernels_api": code_k == 200 and isinstance(kernels, list),
                   "gpu": gpu}
            print(json.dumps(row), flush=True)
            rows.append(row)
            c.delete("kubeflow.org/v1", "Notebook", name, NS)
            _wait(lambda: not [p for p in c.list("v1", "Pod", NS) if p["metadata"]["name"].startswith(name + "-")],
                  a.timeout)
            _wait(lambda: _get(base + "/api/status", timeout=0.5)[0] is None, 30)   # the server process is gone
    finally:
        cl.stop()
    med = lambda k: round(statistics.median(r[k] for r in rows), 3)  # noqa: E731
    print(json.dumps({"metric": "Notebook CR -> notebook server ready (configs[1])", "notebooks": len(rows),
                      "gpus_per_notebook": a.gpus, "control_plane": "processes" if a.processes else "in-process",
                      "p50_cr_to_pod_running_s": med("cr_to_pod_running_s"),
                      "p50_cr_to_server_http_s": med("cr_to_server_http_s"),
                      "p50_cr_to_gpu_probe_s": med("cr_to_gpu_probe_s"),
                      "p50_cr_to_ready_status_s": med("cr_to_ready_status_s"),
                      "all_ready": all(r["ready"] for r in rows),
                      "device": (rows[0]["gpu"] or {}).get("device") if rows else None}), flush=True)
    return 0 if rows and all(r["ready"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
