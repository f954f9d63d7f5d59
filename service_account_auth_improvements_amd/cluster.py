"""Single-node local cluster: the whole platform in one process (M3 KinD-harness equivalent).

``LocalCluster`` wires the in-memory API server (+ its Kubernetes REST facade), the node
agent (kubelet with the ``amd.com/gpu`` device plugin that hands pods
``HIP_VISIBLE_DEVICES``), the workload controllers (StatefulSet, Deployment), every platform
controller (Notebook [+culler], Profile, Tensorboard, PVCViewer, PyTorchJob, MPIJob,
InferenceService), the admission webhooks (PodDefault mutator, PVCViewer defaulter /
validator), and optionally the HTTP services: KFAM (:8081), the Jupyter / Volumes /
Tensorboards web apps and the central dashboard.  Manifests (CRDs, kustomize output,
sample CRs) are applied with :meth:`apply`.

CLI::

    python -m service_account_auth_improvements_amd.cluster up [--gpus 8] [--exec-pods]
        [--api-port 8001] [--services] [--apply FILE_OR_DIR ...]

The reference's equivalent is a KinD cluster built by
components/testing/gh-actions/{install_kind.sh, kind-1-25.yaml, install_istio.sh, ...} plus
the per-component kustomize deploys; here the same CRs reconcile against the same object
model without a container runtime -- pods are processes on this node.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading
import time
from typing import Dict, List, Optional

import yaml

from .controlplane import inferenceservice, notebook, poddefault, profile, pvcviewer, tensorboard, training
from .controlplane.apiserver import APIServer, ApiError
from .controlplane.client import InMemoryClient
from .controlplane.httpapi import APIServerHTTP
from .controlplane.kubelet import DeploymentController, Kubelet, StatefulSetController
from .controlplane.runtime import Manager

log = logging.getLogger("cluster")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DEFAULT_LABELS = os.path.join(HERE, "config", "namespace-labels.yaml")


def load_manifests(path: str) -> List[dict]:
    """All YAML documents of a file, or of every *.yaml under a directory (sorted)."""
    files = []
    if os.path.isdir(path):
        for root, _, names in sorted(os.walk(path)):
            files += [os.path.join(root, n) for n in sorted(names)
                      if n.endswith((".yaml", ".yml")) and n != "kustomization.yaml"]
    else:
        files = [path]
    out = []
    for f in files:
        with open(f) as fh:
            out += [d for d in yaml.safe_load_all(fh) if isinstance(d, dict) and d.get("kind")]
    return out


class LocalCluster:
    def __init__(self, n_gpus: int = 8, exec_pods: bool = False, api_port: Optional[int] = 0,
                 workdir: Optional[str] = None, log_dir: Optional[str] = None, extra_env: Optional[dict] = None,
                 services: bool = False, service_ports: Optional[Dict[str, int]] = None,
                 labels_path: str = DEFAULT_LABELS, workers: int = 4, registry=None):
        from prometheus_client import CollectorRegistry
        self.registry = registry or CollectorRegistry()
        self.server = APIServer()
        self.client = InMemoryClient(self.server)
        self.http = APIServerHTTP(self.server, port=api_port) if api_port is not None else None
        for cr in profile.default_cluster_roles():
            self.client.create(cr)
        self.server.ensure_namespace("kubeflow")
        env = {"PYTHONPATH": REPO}
        env.update(extra_env or {})
        self.kubelet = Kubelet(self.client, n_gpus=n_gpus, exec_pods=exec_pods, workdir=workdir or REPO,
                               log_dir=log_dir, extra_env=env)
        self.manager = Manager(self.client, metrics_registry=self.registry)
        c, m = self.client, self.manager
        m.add(StatefulSetController(c)).add(DeploymentController(c)).add(self.kubelet)
        self.notebook_metrics = notebook.setup(m, c, self.registry)
        os.environ.setdefault("TENSORBOARD_IMAGE", "kfamd/tensorboard:latest")
        os.environ.setdefault("ISTIO_GATEWAY", "kubeflow/kubeflow-gateway")
        os.environ.setdefault("ISTIO_HOST", "*")
        self.profiles = profile.ProfileReconciler(c, labels_path=labels_path, ns_wait_s=0.0)
        m.add(self.profiles)
        m.add(tensorboard.TensorboardReconciler(c)).add(pvcviewer.PVCViewerReconciler(c))
        m.add(training.PyTorchJobReconciler(c)).add(training.MPIJobReconciler(c))
        m.add(inferenceservice.InferenceServiceReconciler(c))
        poddefault.register(self.server, c)
        pvcviewer.register(self.server)
        self.workers = workers
        self.services = services
        self.service_ports = dict({"kfam": 8081, "jupyter": 5000, "volumes": 5001, "tensorboards": 5002,
                                   "dashboard": 8082}, **(service_ports or {}))
        self._servers = []

    # ------------------------------------------------------------------ lifecycle
    def start(self):
        if self.http is not None:
            self.http.start()
        self.manager.start(workers=self.workers)
        if self.services:
            self._start_services()
        return self

    def stop(self):
        for s in self._servers:
            s.shutdown()
        self.manager.stop()
        self.kubelet.shutdown()
        if self.http is not None:
            self.http.stop()

    def _serve(self, name, app, port):
        from werkzeug.serving import make_server
        srv = make_server("127.0.0.1", port, app, threaded=True)
        threading.Thread(target=srv.serve_forever, daemon=True, name=f"svc-{name}").start()
        self._servers.append(srv)
        self.service_ports[name] = srv.server_port
        log.info("%s on http://127.0.0.1:%d", name, srv.server_port)

    def _start_services(self):
        from .controlplane.kfam import Kfam
        from .webapps import dashboard, jupyter, tensorboards, volumes
        c = self.client
        kf = Kfam(c, registry=self.registry)
        self._serve("kfam", kf.app(), self.service_ports["kfam"])
        env = {"APP_SECURE_COOKIES": "false"}
        self._serve("jupyter", jupyter.create_app(c, settings_env=env,
                                                  pod_log_reader=lambda ns, pod, ctr: self.kubelet.pod_log(ns, pod)),
                    self.service_ports["jupyter"])
        self._serve("volumes", volumes.create_app(c, settings_env=env), self.service_ports["volumes"])
        self._serve("tensorboards", tensorboards.create_app(c, settings_env=env), self.service_ports["tensorboards"])
        prof = dashboard.ProfilesService(dashboard.http_transport(
            f"http://127.0.0.1:{self.service_ports['kfam']}/kfam"))
        metrics = dashboard.LocalMetricsService(pod_pids=self.kubelet.pod_pids)
        self._serve("dashboard", dashboard.create_app(c, prof, metrics, env={}), self.service_ports["dashboard"])

    # ------------------------------------------------------------------ objects
    def apply(self, docs) -> List[dict]:
        """Create-or-update every document (server-side-apply-like merge of spec/metadata)."""
        if isinstance(docs, str):
            docs = load_manifests(docs)
        out = []
        for d in docs:
            md = d.get("metadata") or {}
            ns = md.get("namespace")
            if ns:
                self.server.ensure_namespace(ns)
            try:
                cur = self.client.get_or_none(d["apiVersion"], d["kind"], md["name"], ns)
            except ApiError:
                cur = None
            if cur is None:
                out.append(self.client.create(d))
            else:
                d = dict(d, metadata=dict(md, resourceVersion=cur["metadata"]["resourceVersion"]))
                out.append(self.client.update(d))
        return out

    def wait_for(self, pred, timeout: float = 60.0, period: float = 0.05):
        deadline = time.time() + timeout
        while time.time() < deadline:
            v = pred()
            if v:
                return v
            time.sleep(period)
        return None


def main(argv=None):
    ap = argparse.ArgumentParser(description="kfamd local single-node cluster")
    sub = ap.add_subparsers(dest="cmd", required=True)
    up = sub.add_parser("up")
    up.add_argument("--gpus", type=int, default=int(os.environ.get("KFAMD_NODE_GPUS", "8")))
    up.add_argument("--exec-pods", action="store_true", help="run pod commands as local processes")
    up.add_argument("--api-port", type=int, default=8001)
    up.add_argument("--services", action="store_true", help="serve KFAM, web apps and dashboard")
    up.add_argument("--apply", nargs="*", default=[])
    up.add_argument("--log-dir", default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    cl = LocalCluster(n_gpus=a.gpus, exec_pods=a.exec_pods, api_port=a.api_port, services=a.services,
                      log_dir=a.log_dir).start()
    for p in a.apply:
        cl.apply(p)
    log.info("cluster up: API %s, services %s", cl.http.url if cl.http else "-",
             cl.service_ports if a.services else "off")
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    cl.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
