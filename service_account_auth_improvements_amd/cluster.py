"""Local clusters (M3 KinD-harness equivalent): the whole platform in one process
(``LocalCluster``, one or several nodes), or as separate OS processes talking HTTP
(``ProcessCluster``: API server, controller manager + scheduler, one kubelet per node).

``LocalCluster`` wires the in-memory API server (+ its Kubernetes REST facade), the node
agent (kubelet with the ``amd.com/gpu`` device plugin that hands pods
``HIP_VISIBLE_DEVICES``), the workload controllers (StatefulSet, Deployment), every platform
controller (Notebook [+culler], Profile, Tensorboard, PVCViewer, PyTorchJob, MPIJob,
InferenceService), the admission webhooks (PodDefault mutator, PVCViewer defaulter /
validator), and optionally the HTTP services: KFAM (:8081), the Jupyter / Volumes /
Tensorboards web apps and the central dashboard.  Manifests (CRDs, kustomize output,
sample CRs) are applied with :meth:`apply`.

CLI::

    python -m service_account_auth_improvements_amd.cluster up [--gpus 8] [--nodes 1] [--exec-pods]
        [--api-port 8001] [--services] [--apply FILE_OR_DIR ...]
    # the same platform split into processes, as on a real cluster:
    python -m service_account_auth_improvements_amd.cluster apiserver --port 8001
    python -m service_account_auth_improvements_amd.cluster controller-manager --api http://127.0.0.1:8001
    python -m service_account_auth_improvements_amd.cluster kubelet --api http://127.0.0.1:8001 \
        --node node-0 --gpus 8 [--gpu-base 0] [--exec-pods] [--log-dir DIR]

In the multi-process form every component reaches the API server only over its REST API
(list-then-watch informers, the ``pods/binding`` subresource, status updates), so the
control-plane latencies measured there (tools/bench_crd_to_step.py --processes) include the
HTTP, watch-propagation and process boundaries a real cluster has.

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
from .controlplane.client import InMemoryClient, RestClient
from .controlplane.httpapi import APIServerHTTP
from .controlplane.kubelet import DeploymentController, Kubelet, StatefulSetController
from .controlplane.runtime import Manager
from .controlplane.scheduler import Scheduler

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


def add_platform_controllers(m: Manager, c, registry, labels_path: str = DEFAULT_LABELS):
    """Every platform controller on manager ``m`` (the controller-manager's set)."""
    nb_metrics = notebook.setup(m, c, registry)
    os.environ.setdefault("TENSORBOARD_IMAGE", "kfamd/tensorboard:latest")
    os.environ.setdefault("ISTIO_GATEWAY", "kubeflow/kubeflow-gateway")
    os.environ.setdefault("ISTIO_HOST", "*")
    profiles = profile.ProfileReconciler(c, labels_path=labels_path, ns_wait_s=0.0)
    m.add(profiles)
    m.add(tensorboard.TensorboardReconciler(c)).add(pvcviewer.PVCViewerReconciler(c))
    m.add(training.PyTorchJobReconciler(c)).add(training.MPIJobReconciler(c))
    m.add(inferenceservice.InferenceServiceReconciler(c))
    return nb_metrics, profiles


def register_admission(server: APIServer):
    """The admission webhooks (PodDefault mutator, PVCViewer defaulter / validator, the
    PyTorchJob / MPIJob validator), called in-process by the API server."""
    poddefault.register(server, InMemoryClient(server))
    pvcviewer.register(server)
    training.register(server)


class LocalCluster:
    def __init__(self, n_gpus: int = 8, exec_pods: bool = False, api_port: Optional[int] = 0,
                 workdir: Optional[str] = None, log_dir: Optional[str] = None, extra_env: Optional[dict] = None,
                 services: bool = False, service_ports: Optional[Dict[str, int]] = None,
                 labels_path: str = DEFAULT_LABELS, workers: int = 4, registry=None, nodes: int = 1):
        from prometheus_client import CollectorRegistry
        self.registry = registry or CollectorRegistry()
        self.server = APIServer()
        self.client = InMemoryClient(self.server)
        self.http = APIServerHTTP(self.server, port=api_port) if api_port is not None else None
        for cr in profile.default_cluster_roles():
            self.client.create(cr)
        self.server.ensure_namespace("kubeflow")
        env = {"PYTHONPATH": REPO}
        if self.http is not None:     # pods that talk to the API server (e.g. the MPIJob launcher)
            env["KUBE_API_URL"] = self.http.url
        env.update(extra_env or {})
        # nodes > 1: n_gpus GPUs per node, distinct device indices, pods placed by the scheduler
        self.kubelets = [Kubelet(self.client, node_name=f"node-{i}", n_gpus=n_gpus, exec_pods=exec_pods,
                                 workdir=workdir or REPO, log_dir=log_dir, extra_env=env,
                                 self_schedule=nodes == 1, gpu_base=i * n_gpus) for i in range(nodes)]
        self.kubelet = self.kubelets[0]
        self.manager = Manager(self.client, metrics_registry=self.registry)
        c, m = self.client, self.manager
        m.add(StatefulSetController(c)).add(DeploymentController(c))
        for k in self.kubelets:
            m.add(k)
        if nodes > 1:
            m.add(Scheduler(c))
        self.notebook_metrics, self.profiles = add_platform_controllers(m, c, self.registry, labels_path)
        register_admission(self.server)
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
        for k in self.kubelets:
            k.shutdown()
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


class ProcessCluster:
    """The platform as separate processes over HTTP: ``apiserver``, ``controller-manager``
    (every platform controller + the scheduler) and one ``kubelet`` per node, each started with
    ``python -m service_account_auth_improvements_amd.cluster <role>``.  ``client`` is a
    RestClient; pod logs land in ``log_dir`` (``<ns>_<pod>.log``)."""

    def __init__(self, nodes: int = 1, gpus_per_node: int = 8, exec_pods: bool = False,
                 log_dir: Optional[str] = None, extra_env: Optional[dict] = None, workdir: Optional[str] = None,
                 api_port: int = 0, workers: int = 4, python: Optional[str] = None):
        import tempfile
        self.nodes, self.gpus, self.exec_pods = nodes, gpus_per_node, exec_pods
        self.log_dir = log_dir or tempfile.mkdtemp(prefix="kfamd-cluster-")
        self.extra_env = dict(extra_env or {})
        self.workdir = workdir or REPO
        self.api_port = api_port
        self.workers = workers
        self.python = python or sys.executable
        self.procs: Dict[str, "subprocess.Popen"] = {}
        self.url = None
        self.client = None

    def _spawn(self, name: str, args: List[str]):
        import subprocess
        env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
        out = open(os.path.join(self.log_dir, f"_{name}.log"), "w")
        self.procs[name] = subprocess.Popen([self.python, "-m", "service_account_auth_improvements_amd.cluster"] + args,
                                            env=env, cwd=REPO, stdout=out, stderr=subprocess.STDOUT,
                                            start_new_session=True)

    def start(self, timeout: float = 120.0):
        ready = os.path.join(self.log_dir, "_apiserver.url")
        self._spawn("apiserver", ["apiserver", "--port", str(self.api_port), "--url-file", ready])
        deadline = time.time() + timeout
        while not (os.path.exists(ready) and open(ready).read().strip()):
            if time.time() > deadline or self.procs["apiserver"].poll() is not None:
                self.stop()
                raise RuntimeError("apiserver did not come up: " + self.component_log("apiserver")[-2000:])
            time.sleep(0.05)
        self.url = open(ready).read().strip()
        self.client = RestClient(self.url)
        self._spawn("controller-manager", ["controller-manager", "--api", self.url, "--workers", str(self.workers)])
        for i in range(self.nodes):
            args = ["kubelet", "--api", self.url, "--node", f"node-{i}", "--gpus", str(self.gpus),
                    "--gpu-base", str(i * self.gpus), "--log-dir", self.log_dir, "--workdir", self.workdir]
            if self.exec_pods:
                args.append("--exec-pods")
            for k, v in dict({"KUBE_API_URL": self.url}, **self.extra_env).items():
                args += ["--env", f"{k}={v}"]
            self._spawn(f"kubelet-{i}", args)
        # ready when every node has registered and the controller manager answers
        while len(self.client.list("v1", "Node")) < self.nodes:
            if time.time() > deadline or any(p.poll() is not None for p in self.procs.values()):
                self.stop()
                raise RuntimeError("nodes did not register: " + " | ".join(
                    self.component_log(n)[-800:] for n in self.procs))
            time.sleep(0.05)
        return self

    def component_log(self, name: str) -> str:
        path = os.path.join(self.log_dir, f"_{name}.log")
        return open(path).read() if os.path.exists(path) else ""

    def pod_log(self, namespace: str, name: str) -> str:
        path = os.path.join(self.log_dir, f"{namespace}_{name}.log")
        return open(path).read() if os.path.exists(path) else ""

    def stop(self):
        for name in reversed(list(self.procs)):
            p = self.procs[name]
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in self.procs.values():
            try:
                p.wait(timeout=20)
            except Exception:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()


def _serve_until_signal(stop_fn):
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    stop_fn()
    return 0


def run_apiserver(port: int, url_file: Optional[str] = None) -> int:
    server = APIServer()
    c = InMemoryClient(server)
    for cr in profile.default_cluster_roles():
        c.create(cr)
    server.ensure_namespace("kubeflow")
    register_admission(server)
    http = APIServerHTTP(server, port=port)
    http.start()
    log.info("apiserver on %s", http.url)
    if url_file:
        tmp = url_file + ".tmp"
        with open(tmp, "w") as f:
            f.write(http.url)
        os.replace(tmp, url_file)
    return _serve_until_signal(http.stop)


def run_controller_manager(api: str, workers: int = 4) -> int:
    from prometheus_client import CollectorRegistry
    c = RestClient(api)
    m = Manager(c, metrics_registry=CollectorRegistry())
    m.add(StatefulSetController(c)).add(DeploymentController(c)).add(Scheduler(c))
    add_platform_controllers(m, c, m.metrics_registry)
    m.start(workers=workers)
    log.info("controller-manager (%d controllers) against %s", len(m.controllers), api)
    return _serve_until_signal(m.stop)


def run_kubelet(api: str, node: str, gpus: int, gpu_base: int, exec_pods: bool, log_dir: Optional[str],
                workdir: Optional[str], env: List[str]) -> int:
    c = RestClient(api)
    extra = {"PYTHONPATH": REPO}
    for kv in env:
        k, _, v = kv.partition("=")
        extra[k] = v
    kub = Kubelet(c, node_name=node, n_gpus=gpus, exec_pods=exec_pods, workdir=workdir or REPO, log_dir=log_dir,
                  extra_env=extra, self_schedule=False, gpu_base=gpu_base)
    m = Manager(c)
    m.add(kub)
    m.start(workers=2)
    log.info("kubelet %s (%d GPUs from index %d) against %s", node, gpus, gpu_base, api)

    def stop():
        m.stop()
        kub.shutdown()
    return _serve_until_signal(stop)


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
    up.add_argument("--nodes", type=int, default=1, help="nodes (each --gpus GPUs); >1 adds the scheduler")
    sa = sub.add_parser("apiserver")
    sa.add_argument("--port", type=int, default=8001)
    sa.add_argument("--url-file", default=None, help="write the serving URL here once up")
    scm = sub.add_parser("controller-manager")
    scm.add_argument("--api", required=True)
    scm.add_argument("--workers", type=int, default=4)
    sk = sub.add_parser("kubelet")
    sk.add_argument("--api", required=True)
    sk.add_argument("--node", default="node-0")
    sk.add_argument("--gpus", type=int, default=int(os.environ.get("KFAMD_NODE_GPUS", "8")))
    sk.add_argument("--gpu-base", type=int, default=0, help="first HIP device index of this node")
    sk.add_argument("--exec-pods", action="store_true")
    sk.add_argument("--log-dir", default=None)
    sk.add_argument("--workdir", default=None)
    sk.add_argument("--env", action="append", default=[], help="K=V added to every pod")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    if a.cmd == "apiserver":
        return run_apiserver(a.port, a.url_file)
    if a.cmd == "controller-manager":
        return run_controller_manager(a.api, a.workers)
    if a.cmd == "kubelet":
        return run_kubelet(a.api, a.node, a.gpus, a.gpu_base, a.exec_pods, a.log_dir, a.workdir, a.env)
    cl = LocalCluster(n_gpus=a.gpus, exec_pods=a.exec_pods, api_port=a.api_port, services=a.services,
                      log_dir=a.log_dir, nodes=a.nodes).start()
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
