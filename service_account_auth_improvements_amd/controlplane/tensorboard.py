"""G5: Tensorboard controller (``tensorboard.kubeflow.org/v1alpha1``).

Behavioural reference: components/tensorboard-controller/controllers/tensorboard_controller.go:67-535.

Deployment running ``/usr/local/bin/tensorboard --logdir=<path> --bind_all`` on :6006,
Service 80 -> 6006, VirtualService ``/tensorboard/<ns>/<name>/`` (rewrite ``/``, 300 s
timeout).  Log paths: ``pvc://<pvc>/<subpath>`` mounts read-only at ``/tensorboard_logs/``;
any other non-cloud path mounts PVC ``tb-volume``; ``gs://`` mounts the ``user-gcp-sa``
secret; ``s3://`` and ``/cns/`` are cloud paths.  ``RWO_PVC_SCHEDULING=true`` adds a
preferred node affinity to the node of a running pod that already mounts an RWO PVC.
The kfamd trainer writes TensorBoard event files of its step/loss/tokens-per-second
metrics, so a Tensorboard CR pointed at a job's PVC shows MI355X training curves.
"""
from __future__ import annotations

import copy
import os
from typing import Optional

from . import reconcilehelper
from .apiserver import ApiError, set_controller_reference
from .client import Client
from .runtime import Controller, Request, Result, for_kind, owns

TB_API = "tensorboard.kubeflow.org/v1alpha1"


def is_google_cloud_path(p: str) -> bool:
    return p.startswith("gs://")


def is_cloud_path(p: str) -> bool:
    return is_google_cloud_path(p) or p.startswith("s3://") or p.startswith("/cns/")


def is_pvc_path(p: str) -> bool:
    return p.startswith("pvc://")


def extract_pvc_name(p: str) -> str:
    t = p[len("pvc://"):] if p.startswith("pvc://") else p
    i = t.find("/")
    return t if i == -1 else t[:i]


def extract_pvc_subpath(p: str) -> str:
    t = p[len("pvc://"):] if p.startswith("pvc://") else p
    i = t.find("/")
    if i == -1 or len(t) == i + 1:
        return ""
    return t[i + 1:]


def rwo_pvc_scheduling() -> bool:
    v = os.environ.get("RWO_PVC_SCHEDULING")
    if v is None or v in ("false", "False", "FALSE"):
        return False
    if v in ("true", "True", "TRUE"):
        return True
    raise ValueError("Invalid value for 'RWO_PVC_SCEDULING' env var.")


def pods_using_pvc(client: Client, ns: str, pvc: str):
    """The field index ``spec.volumes.persistentvolumeclaim.claimname`` (main.go:84-105)."""
    out = []
    for p in client.list("v1", "Pod", ns):
        for v in p.get("spec", {}).get("volumes") or []:
            if (v.get("persistentVolumeClaim") or {}).get("claimName") == pvc:
                out.append(p)
                break
    return out


def node_affinity(node: str) -> dict:
    return {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 100, "preference": {"matchExpressions": [
            {"key": "kubernetes.io/hostname", "operator": "In", "values": [node]}]}}]}}


def generate_deployment(tb: dict, client: Client) -> dict:
    m = tb["metadata"]
    logs = tb["spec"]["logspath"]
    mountpath, subpath = logs, ""
    mounts, volumes, affinity = [], [], {}
    image = os.environ.get("TENSORBOARD_IMAGE")
    if image is None:
        raise ValueError("Environment variable TENSORBOARD_IMAGE does not exist")
    if not is_cloud_path(logs):
        if is_pvc_path(logs):
            pvc = extract_pvc_name(logs)
            mountpath, subpath = "/tensorboard_logs/", extract_pvc_subpath(logs)
        else:
            pvc = "tb-volume"
        vm = {"name": "tbpd", "readOnly": True, "mountPath": mountpath}
        if subpath:
            vm["subPath"] = subpath
        mounts.append(vm)
        volumes.append({"name": "tbpd", "persistentVolumeClaim": {"claimName": pvc}})
        if rwo_pvc_scheduling():
            obj = client.get("v1", "PersistentVolumeClaim", pvc, m["namespace"])
            modes = (obj.get("status") or {}).get("accessModes") or []
            if modes and modes[0] == "ReadWriteOnce":
                # the Tensorboard's own pods are excluded: following them would make the
                # affinity (and so the pod template) flip on every pod replacement
                running = [p for p in pods_using_pvc(client, m["namespace"], pvc)
                           if (p.get("status") or {}).get("phase") == "Running"
                           and (p["metadata"].get("labels") or {}).get("app") != m["name"]]
                if running and running[0]["spec"].get("nodeName"):
                    affinity = node_affinity(running[0]["spec"]["nodeName"])
    elif is_google_cloud_path(logs):
        mounts.append({"name": "gcp-creds", "readOnly": True, "mountPath": "/secret/gcp"})
        volumes.append({"name": "gcp-creds", "secret": {"secretName": "user-gcp-sa"}})
    labels = dict(m.get("labels") or {})
    labels["app"] = m["name"]
    ctr = {"name": "tensorboard", "image": image, "imagePullPolicy": "IfNotPresent",
           "command": ["/usr/local/bin/tensorboard"], "workingDir": "/",
           "args": [f"--logdir={mountpath}", "--bind_all"], "ports": [{"containerPort": 6006}]}
    if mounts:
        ctr["volumeMounts"] = mounts
    spec = {"affinity": affinity, "restartPolicy": "Always", "containers": [ctr]}
    if volumes:
        spec["volumes"] = volumes
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": m["name"], "namespace": m["namespace"]},
            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": m["name"]}},
                     "template": {"metadata": {"labels": labels}, "spec": spec}}}


def generate_service(tb: dict) -> dict:
    m = tb["metadata"]
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": m["name"], "namespace": m["namespace"]},
            "spec": {"type": "ClusterIP", "selector": {"app": m["name"]},
                     "ports": [{"name": f"http-{m['name']}", "port": 80, "targetPort": 6006}]}}


def generate_virtual_service(tb: dict) -> dict:
    m = tb["metadata"]
    gw, host = os.environ.get("ISTIO_GATEWAY"), os.environ.get("ISTIO_HOST")
    if gw is None or host is None:
        raise ValueError("Environment variables ISTIO_GATEWAY / ISTIO_HOST must be set")
    return {"apiVersion": "networking.istio.io/v1alpha3", "kind": "VirtualService",
            "metadata": {"name": m["name"], "namespace": m["namespace"]},
            "spec": {"hosts": [host], "gateways": [gw],
                     "http": [{"match": [{"uri": {"prefix": f"/tensorboard/{m['namespace']}/{m['name']}/"}}],
                               "rewrite": {"uri": "/"},
                               "route": [{"destination": {"host": f"{m['name']}.{m['namespace']}.svc.cluster.local",
                                                          "port": {"number": 80}}}],
                               "timeout": "300s"}]}}


def copy_tb_deployment_fields(desired: dict, found: dict) -> bool:
    """Tensorboard's own copier: labels, replicas and affinity only."""
    upd = False
    have = found["metadata"].get("labels") or {}
    want = desired["metadata"].get("labels") or {}
    for k, v in have.items():
        if want.get(k) != v:
            upd = True
    found["metadata"]["labels"] = copy.deepcopy(want)
    if desired["spec"]["replicas"] != found["spec"].get("replicas"):
        found["spec"]["replicas"] = desired["spec"]["replicas"]
        upd = True
    da = desired["spec"]["template"]["spec"].get("affinity")
    if da != found["spec"]["template"]["spec"].get("affinity"):
        upd = True
    found["spec"]["template"]["spec"]["affinity"] = copy.deepcopy(da)
    return upd


class TensorboardReconciler(Controller):
    name = "tensorboard-controller"

    def sources(self):
        return [for_kind(TB_API, "Tensorboard"), owns("apps/v1", "Deployment", "Tensorboard")]

    def reconcile(self, req: Request) -> Result:
        c = self.client
        tb = c.get_or_none(TB_API, "Tensorboard", req.name, req.namespace)
        if tb is None or tb["metadata"].get("deletionTimestamp"):
            return Result()
        dep = set_controller_reference(tb, generate_deployment(tb, c))
        reconcilehelper.reconcile_object(c, dep, copy_tb_deployment_fields)
        reconcilehelper.service(c, set_controller_reference(tb, generate_service(tb)))
        reconcilehelper.virtual_service(c, set_controller_reference(tb, generate_virtual_service(tb)))
        found = c.get_or_none("apps/v1", "Deployment", req.name, req.namespace)
        if found is not None:
            st = copy.deepcopy(tb.get("status") or {})
            conds = (found.get("status") or {}).get("conditions") or []
            if conds:
                cond = {"deploymentState": conds[0]["type"], "lastProbeTime": conds[0].get("lastUpdateTime",
                                                                                          conds[0].get("lastTransitionTime"))}
                cl = st.setdefault("conditions", [])
                if not cl or cl[-1].get("deploymentState") != cond["deploymentState"]:
                    cl.append(cond)
            st["readyReplicas"] = (found.get("status") or {}).get("readyReplicas", 0)
            if st != (tb.get("status") or {}):
                tb["status"] = st
                c.update_status(tb)
        return Result()
