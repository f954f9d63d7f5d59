"""Component entrypoints: ``python -m service_account_auth_improvements_amd <component> [flags]``.

These are the processes the manifests' Deployments run (one component per container, as
the reference's Go binaries / Flask apps / Express server).  Each connects to the API
server through :class:`RestClient` (in-cluster service-account config, or ``--kube-api``
/ ``KUBE_API_URL`` for a local cluster's REST facade).

Components (reference flags kept where they exist):

* ``notebook-controller``   --metrics-addr --probe-addr --enable-leader-election
  --leader-election-namespace   (notebook-controller/main.go:52-140)
* ``profile-controller``    --userid-header --userid-prefix --workload-identity
  --namespace-labels-path (+ manager flags)         (profile-controller/main.go:55-110)
* ``kfam``                  --userid-header --userid-prefix --cluster-admin --port
* ``admission-webhook``     --port --tls-cert-file --tls-key-file (admission-webhook/main.go)
* ``tensorboard-controller``, ``pvcviewer-controller`` (--webhook-port),
  ``training-operator`` (PyTorchJob + MPIJob), ``inferenceservice-controller``
* ``jupyter-web-app`` / ``volumes-web-app`` / ``tensorboards-web-app`` --port
* ``centraldashboard``      --port (env: PROFILES_KFAM_SERVICE_HOST/PORT, PROMETHEUS_URL...)
* ``predictor``             the InferenceService model server (serving/server.py)
* ``train``                 the PyTorchJob worker entry (runtime/train_entry.py)
* ``mpi-wait``              the MPIJob launcher for mpirun-style jobs (controlplane/mpi.py)
* ``nb-server``             notebook server stand-in: read-only Jupyter REST subset + GPU probe
  under NB_PREFIX (runtime/notebook_server.py)
* ``cluster``               the single-process local cluster (cluster.py)
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
import threading


def _addr_port(addr: str, default: int) -> int:
    if not addr or addr == "0":
        return 0
    return int(addr.rsplit(":", 1)[-1] or default)


def _client(a):
    from .controlplane.client import RestClient
    url = a.kube_api or os.environ.get("KUBE_API_URL")
    return RestClient(url) if url else RestClient()


def _manager(a, client, le_id):
    from prometheus_client import CollectorRegistry
    from .controlplane.runtime import Manager
    reg = CollectorRegistry()
    m = Manager(client, leader_election=a.enable_leader_election, leader_election_id=le_id,
                leader_election_namespace=a.leader_election_namespace, metrics_registry=reg)
    return m, reg


def _run_manager(m, a):
    port = _addr_port(a.probe_addr, 8081)
    if port:
        m.serve_probes(port=port, host="0.0.0.0")
    m.start(workers=a.workers)
    threading.Event().wait()


def _serve_flask(app, port):
    from werkzeug.serving import make_server
    make_server("0.0.0.0", port, app, threaded=True).serve_forever()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    comp, rest = argv[0], argv[1:]
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    if comp == "predictor":
        from .serving.server import main as m
        return m(rest)
    if comp == "train":
        from .runtime.train_entry import main as m
        return m(rest)
    if comp == "nb-server":
        from .runtime.notebook_server import main as m
        return m(rest)
    if comp == "cluster":
        from .cluster import main as m
        return m(rest)
    if comp == "mpi-wait":
        from .controlplane.mpi import main as m
        return m(rest)

    ap = argparse.ArgumentParser(prog=f"kfamd {comp}")
    ap.add_argument("--kube-api", default=None)
    ap.add_argument("--metrics-addr", default=":8080")
    ap.add_argument("--probe-addr", default=":8081")
    ap.add_argument("--enable-leader-election", action="store_true")
    ap.add_argument("--leader-election-namespace", default="kubeflow")
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--userid-header", default="kubeflow-userid")
    ap.add_argument("--userid-prefix", default="")
    ap.add_argument("--workload-identity", default="")
    ap.add_argument("--namespace-labels-path", default="/etc/profile-controller/namespace-labels.yaml")
    ap.add_argument("--cluster-admin", default="")
    ap.add_argument("--tls-cert-file", default="")
    ap.add_argument("--tls-key-file", default="")
    ap.add_argument("--webhook-port", type=int, default=9443)
    a = ap.parse_args(rest)
    client = _client(a)

    if comp == "notebook-controller":
        from .controlplane import notebook
        m, reg = _manager(a, client, "kubeflow-notebook-controller")
        notebook.setup(m, client, reg)
        return _run_manager(m, a)
    if comp == "profile-controller":
        from .controlplane import profile
        m, reg = _manager(a, client, "kubeflow-profile-controller")
        from .controlplane.cloud_iam import iam_backend
        r = profile.ProfileReconciler(client, user_id_header=a.userid_header, user_id_prefix=a.userid_prefix,
                                      workload_identity=a.workload_identity, labels_path=a.namespace_labels_path,
                                      iam=iam_backend())
        m.add(r)
        r.watch_labels_file(m)
        return _run_manager(m, a)
    if comp == "kfam":
        from .controlplane.kfam import Kfam
        return _serve_flask(Kfam(client, a.userid_header, a.userid_prefix, a.cluster_admin).app(), a.port or 8081)
    if comp == "admission-webhook":
        from .controlplane import poddefault
        tls = poddefault.ReloadingTLS(a.tls_cert_file, a.tls_key_file) if a.tls_cert_file else None
        srv = poddefault.serve_admission({"/apply-poddefault": lambda req: poddefault.mutate_pods(req, client)},
                                         port=a.port or 4443, tls=tls)
        threading.Event().wait()
        return srv
    if comp == "tensorboard-controller":
        from .controlplane.tensorboard import TensorboardReconciler
        m, _ = _manager(a, client, "8fa23c2d.kubeflow.org")
        m.add(TensorboardReconciler(client))
        return _run_manager(m, a)
    if comp == "pvcviewer-controller":
        from .controlplane import poddefault, pvcviewer
        m, _ = _manager(a, client, "57a72bdf.kubeflow.org")
        m.add(pvcviewer.PVCViewerReconciler(client))
        handlers = {p: fn for p, fn in pvcviewer.WEBHOOK_PATHS.items()}
        poddefault.serve_admission(handlers, port=a.webhook_port)
        return _run_manager(m, a)
    if comp == "training-operator":
        from .controlplane import training
        m, _ = _manager(a, client, "training-operator-kfamd")
        m.add(training.PyTorchJobReconciler(client)).add(training.MPIJobReconciler(client))
        return _run_manager(m, a)
    if comp == "inferenceservice-controller":
        from .controlplane.inferenceservice import InferenceServiceReconciler
        m, _ = _manager(a, client, "kserve-controller-kfamd")
        m.add(InferenceServiceReconciler(client))
        return _run_manager(m, a)
    if comp in ("jupyter-web-app", "volumes-web-app", "tensorboards-web-app"):
        from .webapps import crud_backend, jupyter, tensorboards, volumes
        mod = {"jupyter-web-app": jupyter, "volumes-web-app": volumes, "tensorboards-web-app": tensorboards}[comp]
        cfg = crud_backend.get_config(os.environ.get("BACKEND_MODE", "prod"))
        cfg.PREFIX = os.environ.get("APP_PREFIX", "/")
        return _serve_flask(mod.create_app(client, cfg=cfg), a.port or 5000)
    if comp == "centraldashboard":
        from .webapps import dashboard
        host = os.environ.get("PROFILES_KFAM_SERVICE_HOST", "localhost")
        port = os.environ.get("PROFILES_KFAM_SERVICE_PORT", "8081")
        prof = dashboard.ProfilesService(dashboard.http_transport(f"http://{host}:{port}/kfam"))
        metrics = dashboard.metrics_service_for(client)
        return _serve_flask(dashboard.create_app(client, prof, metrics), a.port or 8082)
    print(f"unknown component {comp!r}\n\n{__doc__}", file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
