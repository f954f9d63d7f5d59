"""configs[1] path on the CPU: the notebook server stand-in (read-only Jupyter REST subset under
NB_PREFIX, no code execution), a Notebook CR driven through controller -> StatefulSet -> exec
kubelet -> a live server, and the kubelet giving a deleted pod's GPUs back."""
import json
import os
import subprocess
import sys
import time
import urllib.error
import urllib.request

import pytest

from service_account_auth_improvements_amd.runtime import notebook_server as nbs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _get(url):
    with urllib.request.urlopen(url, timeout=5) as r:
        return r.status, r.headers.get("Content-Type"), r.read()


def test_server_routes_under_prefix():
    srv = nbs.serve(0, "/notebook/ns/nb", host="127.0.0.1")
    try:
        base = f"http://127.0.0.1:{srv.server_address[1]}/notebook/ns/nb"
        assert json.loads(_get(base + "/api")[2])["version"]
        st = json.loads(_get(base + "/api/status")[2])
        assert {"started", "last_activity", "kernels", "connections"} <= set(st)
        ks = json.loads(_get(base + "/api/kernels")[2])
        assert ks[0]["execution_state"] == "idle" and ks[0]["last_activity"] == st["last_activity"]
        assert _get(base + "/lab")[1].startswith("text/html")
        with pytest.raises(urllib.error.HTTPError) as e:
            _get(f"http://127.0.0.1:{srv.server_address[1]}/other/api/status")     # outside NB_PREFIX
        assert e.value.code == 404
        # read-only: no method but GET
        req = urllib.request.Request(base + "/api/kernels", data=b"{}", method="POST")
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(req, timeout=5)
        assert e.value.code == 501
    finally:
        srv.shutdown()


def test_notebook_cr_to_live_server():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_notebook_ready.py"), "--notebooks", "2",
                        "--gpus", "0"], capture_output=True, text=True, timeout=300, cwd="/tmp",
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    per, summary = rows[:-1], rows[-1]
    assert len(per) == 2 and summary["all_ready"]
    for row in per:
        assert row["nb_prefix"] == f"/notebook/nb-bench/{row['notebook']}" and row["kernels_api"]
        assert row["cr_to_pod_running_s"] <= row["cr_to_server_http_s"] <= row["cr_to_ready_status_s"] + 1e-6


def test_kubelet_returns_gpus_of_deleted_pods():
    from service_account_auth_improvements_amd.cluster import LocalCluster
    cl = LocalCluster(n_gpus=8, api_port=None).start()
    try:
        c = cl.client
        cl.server.ensure_namespace("g")

        def pod(name):
            return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "g"},
                    "spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {"amd.com/gpu": "8"}}}]}}

        def phase(name):
            p = c.get_or_none("v1", "Pod", name, "g")
            return (p or {}).get("status", {}).get("phase")
        c.create(pod("a"))
        assert cl.wait_for(lambda: phase("a") == "Running", 20)
        c.delete("v1", "Pod", "a", "g")
        c.create(pod("b"))                       # needs all 8 GPUs again
        assert cl.wait_for(lambda: phase("b") == "Running", 20), c.get("v1", "Pod", "b", "g").get("status")
    finally:
        cl.stop()
