"""InferenceService controller (``serving.kserve.io/v1beta1``, raw-deployment mode).

North-star component (BASELINE configs[2]: "KServe InferenceService Llama-3-8B bf16 TP=1 on
one MI355X"); the reference only links ``/kserve-endpoints/`` from the dashboard and labels
profile namespaces ``serving.kubeflow.org/inferenceservice=enabled``
(profile-controller/config/base/namespace-labels.yaml), so the API shape follows KServe.

For ``spec.predictor`` it reconciles:

* Deployment ``<name>-predictor`` (labels ``serving.kserve.io/inferenceservice=<name>``,
  ``component=predictor``), replicas ``minReplicas`` (default 1).  ``predictor.model``
  (``modelFormat.name`` in ``kfamd-llama`` / ``huggingface`` / ``pytorch``) becomes the
  container ``kserve-container`` running this repo's predictor
  (``python -m service_account_auth_improvements_amd.serving.server``) on :8080 with the
  model's ``resources`` (``amd.com/gpu``, which the device plugin turns into
  ``HIP_VISIBLE_DEVICES``; more than one GPU runs the predictor tensor-parallel, one process
  per GPU under ``kfamd-launch``, see serving/tp.py); ``storageUri`` ``pvc://<claim>/<path>`` mounts the claim
  read-only at ``/mnt/models`` and passes ``--checkpoint``.  ``predictor.containers``
  (custom predictor) is used verbatim.
* Service ``<name>-predictor`` (80 -> 8080) and, with ``ISTIO_GATEWAY``/``ISTIO_HOST`` set, a
  VirtualService routing ``/kserve-endpoints/<ns>/<name>/``.
* Status: ``url``/``address.url``, ``components.predictor``, conditions
  ``PredictorReady`` / ``IngressReady`` / ``Ready`` from the Deployment's ready replicas, and
  ``modelStatus.states`` (``Pending`` -> ``Loaded``).
"""
from __future__ import annotations

import copy
import os

from . import reconcilehelper
from .apiserver import now_rfc3339, set_controller_reference
from .runtime import Controller, Request, Result, for_kind, owns

ISVC_API = "serving.kserve.io/v1beta1"
ISVC_LABEL = "serving.kserve.io/inferenceservice"
PREDICTOR_MODULE = "service_account_auth_improvements_amd.serving.server"
SUPPORTED_FORMATS = ("kfamd-llama", "huggingface", "pytorch")


def predictor_name(isvc: dict) -> str:
    return f"{isvc['metadata']['name']}-predictor"


def cluster_domain() -> str:
    return os.environ.get("CLUSTER_DOMAIN", "cluster.local")


def predictor_container(isvc: dict) -> tuple:
    """Returns (containers, volumes) for the predictor pod."""
    pred = isvc["spec"].get("predictor") or {}
    if pred.get("containers"):
        return copy.deepcopy(pred["containers"]), copy.deepcopy(pred.get("volumes") or [])
    model = pred.get("model") or {}
    fmt = ((model.get("modelFormat") or {}).get("name") or "kfamd-llama").lower()
    if fmt not in SUPPORTED_FORMATS:
        raise ValueError(f"unsupported modelFormat {fmt!r}; supported: {', '.join(SUPPORTED_FORMATS)}")
    name = isvc["metadata"]["name"]
    args = ["-m", PREDICTOR_MODULE, "--model-name", name, "--port", "8080"]
    volumes, mounts = [], []
    uri = model.get("storageUri") or ""
    if uri.startswith("pvc://"):
        rest = uri[len("pvc://"):]
        claim, _, sub = rest.partition("/")
        volumes.append({"name": "kserve-pvc-source", "persistentVolumeClaim": {"claimName": claim, "readOnly": True}})
        mounts.append({"name": "kserve-pvc-source", "mountPath": "/mnt/pvc", "readOnly": True})
        args += ["--checkpoint", os.path.join("/mnt/pvc", sub) if sub else "/mnt/pvc"]
    args += [str(a) for a in model.get("args") or []]
    command = ["python"]
    resources = model.get("resources") or {}
    gpus = int((resources.get("limits") or {}).get("amd.com/gpu", 0) or 0)
    if gpus > 1:
        # one process per GPU (Megatron TP over the pod's GPUs); rank 0 serves HTTP (serving/tp.py)
        from .training import launcher_path
        command = [launcher_path(), "--nnodes", "1", "--node-rank", "0", "--nproc-per-node", str(gpus),
                   "--master-addr", "127.0.0.1", "--master-port", "29590", "--isolate-devices", "--", "python"]
        args += ["--tp", str(gpus)]
    ctr = {"name": "kserve-container", "image": model.get("image") or os.environ.get(
               "KFAMD_PREDICTOR_IMAGE", "kfamd/predictor-rocm:latest"),
           "command": command, "args": args,
           "env": [{"name": "MODEL_NAME", "value": name}, {"name": "PORT", "value": "8080"}]
           + copy.deepcopy(model.get("env") or []),
           "ports": [{"containerPort": 8080, "name": "http1", "protocol": "TCP"}],
           "readinessProbe": {"httpGet": {"path": f"/v1/models/{name}", "port": 8080}},
           "resources": copy.deepcopy(model.get("resources") or {})}
    if mounts:
        ctr["volumeMounts"] = mounts
    return [ctr], volumes


def generate_deployment(isvc: dict) -> dict:
    m = isvc["metadata"]
    pred = isvc["spec"].get("predictor") or {}
    containers, volumes = predictor_container(isvc)
    labels = {ISVC_LABEL: m["name"], "component": "predictor", "app": predictor_name(isvc)}
    labels.update({k: v for k, v in (m.get("labels") or {}).items()})
    spec = {"containers": containers}
    if volumes:
        spec["volumes"] = volumes
    for k in ("serviceAccountName", "nodeSelector", "tolerations", "affinity"):
        if pred.get(k) is not None:
            spec[k] = copy.deepcopy(pred[k])
    replicas = pred.get("minReplicas")
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": predictor_name(isvc), "namespace": m["namespace"], "labels": dict(labels)},
            "spec": {"replicas": 1 if replicas is None else int(replicas),
                     "selector": {"matchLabels": {"app": predictor_name(isvc)}},
                     "template": {"metadata": {"labels": labels,
                                               "annotations": dict(m.get("annotations") or {})},
                                  "spec": spec}}}


def generate_service(isvc: dict) -> dict:
    m = isvc["metadata"]
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": {"name": predictor_name(isvc), "namespace": m["namespace"],
                         "labels": {ISVC_LABEL: m["name"]}},
            "spec": {"type": "ClusterIP", "selector": {"app": predictor_name(isvc)},
                     "ports": [{"name": "http", "port": 80, "targetPort": 8080, "protocol": "TCP"}]}}


def generate_virtual_service(isvc: dict):
    gw, host = os.environ.get("ISTIO_GATEWAY"), os.environ.get("ISTIO_HOST")
    if not gw or not host:
        return None
    m = isvc["metadata"]
    return {"apiVersion": "networking.istio.io/v1alpha3", "kind": "VirtualService",
            "metadata": {"name": predictor_name(isvc), "namespace": m["namespace"]},
            "spec": {"hosts": [host], "gateways": [gw],
                     "http": [{"match": [{"uri": {"prefix": f"/kserve-endpoints/{m['namespace']}/{m['name']}/"}}],
                               "rewrite": {"uri": "/"},
                               "route": [{"destination": {
                                   "host": f"{predictor_name(isvc)}.{m['namespace']}.svc.{cluster_domain()}",
                                   "port": {"number": 80}}}],
                               "timeout": "600s"}]}}


def _cond(t, ok, reason="", msg=""):
    c = {"type": t, "status": "True" if ok else "False", "lastTransitionTime": now_rfc3339()}
    if not ok:
        c.update(reason=reason, message=msg)
    return c


class InferenceServiceReconciler(Controller):
    name = "inferenceservice-controller"

    def sources(self):
        return [for_kind(ISVC_API, "InferenceService"), owns("apps/v1", "Deployment", "InferenceService")]

    def reconcile(self, req: Request) -> Result:
        c = self.client
        isvc = c.get_or_none(ISVC_API, "InferenceService", req.name, req.namespace)
        if isvc is None or isvc["metadata"].get("deletionTimestamp"):
            return Result()
        try:
            dep = set_controller_reference(isvc, generate_deployment(isvc))
        except ValueError as e:
            return self._set_status(isvc, None, str(e))
        reconcilehelper.deployment(c, dep)
        reconcilehelper.service(c, set_controller_reference(isvc, generate_service(isvc)))
        vs = generate_virtual_service(isvc)
        if vs is not None:
            reconcilehelper.virtual_service(c, set_controller_reference(isvc, vs))
        found = c.get_or_none("apps/v1", "Deployment", predictor_name(isvc), req.namespace)
        return self._set_status(isvc, found, "")

    def _set_status(self, isvc, dep, err) -> Result:
        m = isvc["metadata"]
        ready = dep is not None and int((dep.get("status") or {}).get("readyReplicas") or 0) >= 1
        url = f"http://{predictor_name(isvc)}.{m['namespace']}.svc.{cluster_domain()}"
        old = isvc.get("status") or {}
        old_conds = {x["type"]: x for x in old.get("conditions") or []}

        def keep(cond):   # preserve transition time when the status did not flip
            prev = old_conds.get(cond["type"])
            if prev and prev.get("status") == cond["status"]:
                cond["lastTransitionTime"] = prev.get("lastTransitionTime", cond["lastTransitionTime"])
            return cond

        reason = "InvalidPredictorSpec" if err else "PredictorNotReady"
        msg = err or "predictor deployment has no ready replicas"
        conds = [keep(_cond("IngressReady", not err)), keep(_cond("PredictorReady", ready, reason, msg)),
                 keep(_cond("Ready", ready, reason, msg))]
        st = {"conditions": conds, "url": url, "address": {"url": url + f"/v1/models/{m['name']}:predict"},
              "components": {"predictor": {"url": url}},
              "modelStatus": {"states": {"activeModelState": "Loaded" if ready else "Pending",
                                         "targetModelState": "Loaded"},
                              "transitionStatus": "UpToDate" if ready else ("BlockedByFailedLoad" if err
                                                                            else "InProgress")}}
        if st != old:
            isvc["status"] = st
            self.client.update_status(isvc)
        return Result()
