"""G6 / G6a / G6b: PVCViewer controller + defaulting / validating admission webhooks.

Behavioural reference: components/pvcviewer-controller/controllers/pvcviewer_controller.go:84-445,
api/v1alpha1/pvcviewer_webhook.go:42-199, api/v1alpha1/pvcviewer_types.go:26-105.

A PVCViewer ``{pvc, podSpec, networking{targetPort, basePrefix, rewrite, timeout},
rwoScheduling}`` gets Deployment ``pvcviewer-<name>`` (Recreate), and when networking is
set a Service (80 -> targetPort) and a VirtualService ``<basePrefix>/<ns>/<name>/``.
Status: ``ready``, ``url``, deployment conditions.  With ``rwoScheduling`` the Deployment
is pinned (preferred affinity, set at creation only) to the one node already mounting the
RWO PVC.  The defaulter fills an empty podSpec from ``DEFAULT_POD_SPEC_PATH`` or a
filebrowser container and mounts the PVC as ``viewer-volume``; the validator requires a
PVC name, a podSpec, and that the podSpec mounts the PVC.
"""
from __future__ import annotations

import copy
import os
from typing import Optional

import yaml

from .apiserver import Webhook, create_json_patch, now_rfc3339, set_controller_reference
from .client import Client
from .runtime import Controller, Request, Result, for_kind, owns
from .tensorboard import node_affinity

PV_API = "kubeflow.org/v1alpha1"
RESOURCE_PREFIX = "pvcviewer-"
NAME_LABEL, INSTANCE_LABEL, PART_OF_LABEL, PART_OF_VALUE = (
    "app.kubernetes.io/name", "app.kubernetes.io/instance", "app.kubernetes.io/part-of", "pvc-viewer")
SERVICE_PORT = 80
DEFAULT_ISTIO_GATEWAY = "kubeflow/kubeflow-gateway"
DEFAULT_POD_SPEC_PATH_ENV = "DEFAULT_POD_SPEC_PATH"


# ----------------------------------------------------------------------------- webhooks
def default_viewer(v: dict) -> dict:
    v = copy.deepcopy(v)
    spec = v.setdefault("spec", {})
    if not spec.get("podSpec"):
        pod_spec = {}
        path = os.environ.get(DEFAULT_POD_SPEC_PATH_ENV)
        if path:
            try:
                with open(path) as f:
                    pod_spec = yaml.safe_load(f) or {}
            except OSError:
                return v
        if not pod_spec:
            net = spec.get("networking") or {}
            m = v["metadata"]
            pod_spec = {"containers": [{
                "name": "pvcviewer", "image": "filebrowser/filebrowser:latest",
                "ports": [{"containerPort": 8080, "protocol": "TCP"}],
                "env": [{"name": "FB_ADDRESS", "value": "0.0.0.0"}, {"name": "FB_PORT", "value": "8080"},
                        {"name": "FB_DATABASE", "value": "/tmp/filebrowser.db"}, {"name": "FB_NOAUTH", "value": "true"},
                        {"name": "FB_BASEURL",
                         "value": f"{net.get('basePrefix', '')}/{m.get('namespace')}/{m.get('name')}/"}],
                "workingDir": "/data", "volumeMounts": [{"name": "viewer-volume", "mountPath": "/data"}]}]}
        pod_spec.setdefault("volumes", []).append(
            {"name": "viewer-volume", "persistentVolumeClaim": {"claimName": spec.get("pvc", "")}})
        spec["podSpec"] = pod_spec
    return v


def validate_viewer(v: dict) -> Optional[str]:
    spec = v.get("spec") or {}
    if not spec.get("pvc"):
        return "PVC name must be specified"
    if not spec.get("podSpec"):
        return "PodSpec must be specified"
    for vol in spec["podSpec"].get("volumes") or []:
        if (vol.get("persistentVolumeClaim") or {}).get("claimName") == spec["pvc"]:
            return None
    return f"PVC {spec['pvc']} must be used in the podSpec"


def mutate(request: dict) -> dict:
    obj = request["object"]
    patch = create_json_patch(obj, default_viewer(obj))
    import base64
    import json
    resp = {"uid": request.get("uid"), "allowed": True}
    if patch:
        resp["patchType"] = "JSONPatch"
        resp["patch"] = base64.b64encode(json.dumps(patch).encode()).decode()
    return resp


def validate(request: dict) -> dict:
    if request.get("operation") == "DELETE":
        return {"uid": request.get("uid"), "allowed": True}
    err = validate_viewer(request["object"])
    if err:
        return {"uid": request.get("uid"), "allowed": False,
                "status": {"code": 403, "reason": "Forbidden", "message": err}}
    return {"uid": request.get("uid"), "allowed": True}


def register(server):
    """/mutate-kubeflow-org-v1alpha1-pvcviewer and /validate-kubeflow-org-v1alpha1-pvcviewer."""
    server.add_mutating_webhook(Webhook("mpvcviewer.kb.io", "kubeflow.org", "PVCViewer", ("CREATE", "UPDATE"), mutate))
    server.add_validating_webhook(Webhook("vpvcviewer.kb.io", "kubeflow.org", "PVCViewer", ("CREATE", "UPDATE"),
                                          validate))


WEBHOOK_PATHS = {"/mutate-kubeflow-org-v1alpha1-pvcviewer": mutate,
                 "/validate-kubeflow-org-v1alpha1-pvcviewer": validate}


# ----------------------------------------------------------------------------- controller
class PVCViewerReconciler(Controller):
    name = "pvcviewer-controller"

    def sources(self):
        return [for_kind(PV_API, "PVCViewer"), owns("apps/v1", "Deployment", "PVCViewer"),
                owns("v1", "Service", "PVCViewer"),
                owns("networking.istio.io/v1alpha3", "VirtualService", "PVCViewer")]

    def generate_affinity(self, v: dict) -> Optional[dict]:
        c, ns = self.client, v["metadata"]["namespace"]
        pvc = c.get_or_none("v1", "PersistentVolumeClaim", v["spec"]["pvc"], ns)
        if pvc is None:
            return None
        modes = pvc.get("spec", {}).get("accessModes") or []
        if len(modes) != 1 or modes[0] != "ReadWriteOnce":
            return None
        node = None
        for pod in c.list("v1", "Pod", ns):
            if (pod["metadata"].get("labels") or {}).get(PART_OF_LABEL) == PART_OF_VALUE:
                continue
            for vol in pod.get("spec", {}).get("volumes") or []:
                if (vol.get("persistentVolumeClaim") or {}).get("claimName") == pvc["metadata"]["name"]:
                    nn = pod["spec"].get("nodeName")
                    if node is not None and nn != node:
                        return None   # mounted on several nodes: no preference
                    if not nn:
                        return None
                    node = nn
        return node_affinity(node) if node else None

    def reconcile(self, req: Request) -> Result:
        c = self.client
        v = c.get_or_none(PV_API, "PVCViewer", req.name, req.namespace)
        if v is None:
            return Result()
        if v["metadata"].get("deletionTimestamp"):
            self._status(req)
            return Result()
        labels = {NAME_LABEL: v["metadata"]["name"], INSTANCE_LABEL: RESOURCE_PREFIX + v["metadata"]["name"],
                  PART_OF_LABEL: PART_OF_VALUE}
        name = RESOURCE_PREFIX + v["metadata"]["name"]
        dep = c.get_or_none("apps/v1", "Deployment", name, req.namespace)
        create = dep is None
        if create:
            dep = {"apiVersion": "apps/v1", "kind": "Deployment",
                   "metadata": {"name": name, "namespace": req.namespace, "labels": labels}, "spec": {}}
        affinity = ((dep.get("spec", {}).get("template") or {}).get("spec") or {}).get("affinity")
        if v["spec"].get("rwoScheduling") and create:
            a = self.generate_affinity(v)
            if a:
                affinity = a
        pod_spec = copy.deepcopy(v["spec"].get("podSpec") or {})
        if affinity:
            pod_spec["affinity"] = affinity
        dep["spec"].update({"selector": {"matchLabels": labels},
                            "template": {"metadata": {"labels": labels}, "spec": pod_spec},
                            "strategy": {"type": "Recreate"}})
        dep["spec"].setdefault("replicas", 1)
        set_controller_reference(v, dep)
        c.create(dep) if create else c.update(dep)
        net = v["spec"].get("networking") or {}
        if net:
            svc = c.get_or_none("v1", "Service", name, req.namespace) or \
                {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "namespace": req.namespace,
                                                                      "labels": labels}, "spec": {}}
            svc["spec"].update({"type": "ClusterIP", "selector": labels,
                                "ports": [{"name": "http", "port": SERVICE_PORT, "targetPort": net.get("targetPort")}]})
            set_controller_reference(v, svc)
            c.update(svc) if "uid" in svc["metadata"] else c.create(svc)
            prefix = f"{net.get('basePrefix', '')}/{req.namespace}/{req.name}/"
            vs = c.get_or_none("networking.istio.io/v1alpha3", "VirtualService", name, req.namespace) or \
                {"apiVersion": "networking.istio.io/v1alpha3", "kind": "VirtualService",
                 "metadata": {"name": name, "namespace": req.namespace, "labels": labels}}
            vs["spec"] = {"hosts": ["*"], "gateways": [os.environ.get("ISTIO_GATEWAY") or DEFAULT_ISTIO_GATEWAY],
                          "http": [{"match": [{"uri": {"prefix": prefix}}],
                                    "rewrite": {"uri": net.get("rewrite") or prefix},
                                    "route": [{"destination": {"host": f"{name}.{req.namespace}.svc.cluster.local",
                                                               "port": {"number": SERVICE_PORT}}}],
                                    "timeout": net.get("timeout") or None}]}
            set_controller_reference(v, vs)
            c.update(vs) if "uid" in vs["metadata"] else c.create(vs)
        self._status(req)
        return Result()

    def _status(self, req: Request):
        c = self.client
        v = c.get_or_none(PV_API, "PVCViewer", req.name, req.namespace)
        if v is None:
            return
        st = copy.deepcopy(v.get("status") or {})
        net = v["spec"].get("networking") or {}
        st["url"] = f"{net.get('basePrefix', '')}/{req.namespace}/{req.name}/" if net else None
        dep = c.get_or_none("apps/v1", "Deployment", RESOURCE_PREFIX + req.name, req.namespace)
        if dep is None:
            st["ready"] = False
        else:
            st["ready"] = dep["spec"].get("replicas", 1) == (dep.get("status") or {}).get("readyReplicas", 0)
            dconds = (dep.get("status") or {}).get("conditions") or []
            if dconds:
                cl = st.setdefault("conditions", [])
                if not cl or cl[-1] != dconds[0]:
                    cl.append(copy.deepcopy(dconds[0]))
        if st != (v.get("status") or {}):
            v["status"] = st
            c.update_status(v)
