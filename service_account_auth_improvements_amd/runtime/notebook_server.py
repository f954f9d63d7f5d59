"""Notebook server stand-in for the ROCm notebook image (BASELINE configs[1]).

The real image runs JupyterLab (`images/jupyter-pytorch-rocm`). Jupyter is not installed in
this environment, so this process plays the server's part for the platform. It implements the
read-only subset of the Jupyter REST API that the control plane relies on, under `NB_PREFIX`,
as `jupyter lab --ServerApp.base_url=$NB_PREFIX` would:

* ``GET {NB_PREFIX}/api`` and ``/api/status``: the version and server status (started,
  last_activity, kernels, connections).
* ``GET {NB_PREFIX}/api/kernels``: the kernel list the notebook culler reads
  (controlplane/notebook.py CullingReconciler; reference culling_controller.go). One idle
  kernel carries the server's last activity.
* ``GET {NB_PREFIX}/api/kfamd/gpu``: what a notebook kernel would see of the pod's GPU. It
  reports the device name, total HBM and HIP_VISIBLE_DEVICES, and times one bf16 matmul, so a
  readiness check proves that the pod reaches its MI355X. This path is a kfamd extension.
* ``GET {NB_PREFIX}/`` and ``/lab``: a landing page.

Nothing received over the network is executed. Every route is read-only.

  python -m service_account_auth_improvements_amd nb-server [--port 8888]
  (the port defaults to NB_PORT or 8888; the prefix comes from NB_PREFIX)
"""
from __future__ import annotations

import argparse
import datetime as dt
import json
import os
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

VERSION = "2.14.0-kfamd"


def _now() -> str:
    return dt.datetime.now(dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


class _State:
    def __init__(self):
        self.started = _now()
        self.last_activity = self.started
        self.kernel_id = "00000000-0000-4000-8000-" + f"{os.getpid():012d}"[-12:]
        self.gpu = None
        self.lock = threading.Lock()

    def gpu_info(self) -> dict:
        """Probed once, on first request, so the server starts listening before touching the GPU."""
        with self.lock:
            if self.gpu is None:
                self.gpu = _probe_gpu()
            return self.gpu


def _probe_gpu() -> dict:
    info = {"hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES"), "available": False}
    try:
        import torch
        if not torch.cuda.is_available():
            return info
        dev = torch.device("cuda", 0)
        p = torch.cuda.get_device_properties(dev)
        a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        torch.mm(a, a)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            torch.mm(a, a)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 10 * 1e3
        info.update(available=True, device=p.name, arch=getattr(p, "gcnArchName", ""),
                    total_memory_gib=round(p.total_memory / 2**30, 1),
                    bf16_matmul_4096_ms=round(ms, 3), bf16_matmul_tflops=round(2 * 4096**3 / ms / 1e9, 1),
                    torch=torch.__version__)
    except Exception as e:  # report, do not crash the server
        info["error"] = f"{type(e).__name__}: {e}"
    return info


def make_handler(prefix: str, state: _State):
    prefix = prefix.rstrip("/")

    class H(BaseHTTPRequestHandler):
        def log_message(self, fmt, *args):  # quiet
            pass

        def _send(self, code, body, ctype="application/json"):
            data = body if isinstance(body, bytes) else json.dumps(body).encode()
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def do_GET(self):  # noqa: N802
            path = self.path.split("?", 1)[0]
            if not path.startswith(prefix + "/") and path != prefix:
                return self._send(404, {"message": "not found"})
            sub = path[len(prefix):] or "/"
            if sub in ("/api", "/api/"):
                return self._send(200, {"version": VERSION})
            if sub == "/api/status":
                return self._send(200, {"started": state.started, "last_activity": state.last_activity,
                                        "connections": 0, "kernels": 1})
            if sub == "/api/kernels":
                return self._send(200, [{"id": state.kernel_id, "name": "python3", "last_activity": state.last_activity,
                                         "execution_state": "idle", "connections": 0}])
            if sub == "/api/kfamd/gpu":
                return self._send(200, state.gpu_info())
            if sub in ("/", "/lab", "/lab/", "/tree", "/tree/"):
                html = (f"<!doctype html><title>kfamd notebook</title><h1>{prefix or '/'}</h1>"
                        f"<p>ROCm notebook server stand-in (read-only Jupyter REST subset).</p>").encode()
                return self._send(200, html, "text/html")
            return self._send(404, {"message": "not found"})

    return H


def serve(port: int, prefix: str, host: str = "0.0.0.0") -> ThreadingHTTPServer:
    srv = ThreadingHTTPServer((host, port), make_handler(prefix, _State()))
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kfamd nb-server")
    ap.add_argument("--port", type=int, default=int(os.environ.get("NB_PORT", "8888")))
    ap.add_argument("--host", default="0.0.0.0")
    a = ap.parse_args(argv)
    prefix = os.environ.get("NB_PREFIX", "")
    srv = serve(a.port, prefix, a.host)
    print(json.dumps({"event": "listening", "port": srv.server_address[1], "prefix": prefix}), flush=True)
    threading.Event().wait()
    return 0
