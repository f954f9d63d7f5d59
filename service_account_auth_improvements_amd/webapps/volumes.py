"""P4: Volumes web app (VWA) backend.

Behavioural reference: components/crud-web-apps/volumes/backend/apps/common/{form.py,
status.py, utils.py, viewer.py}, apps/default/routes/{get,post,delete}.py,
manifests/base/viewer-spec.yaml.

* ``GET /api/namespaces/<ns>/pvcs``: capacity (status, else request), modes, class, the
  notebooks mounting it, status (Bound -> ready; else derived from the newest PVC event:
  WaitForFirstConsumer -> unavailable, Provisioning -> waiting, FailedBinding/Warning ->
  warning), and its PVCViewer ``{status, url}``.
* ``POST .../pvcs`` (``{none}`` class -> ``""``, ``{empty}`` -> unset), ``POST .../viewers``
  from the viewer-spec template (``$NAME``/``$NAMESPACE``/``$PVC_NAME``/env substituted).
* ``DELETE .../pvcs/<pvc>``: 409 if any non-viewer pod mounts it; viewer pods' PVCViewers
  are deleted first.  ``DELETE .../viewers/<name>``.
"""
from __future__ import annotations

import copy
import logging
import os
from string import Template

import yaml
from flask import Blueprint, request
from werkzeug import exceptions

from . import crud_backend as cb
from .crud_backend import STATUS_PHASE, api, create_status, success_response

log = logging.getLogger("vwa")
HERE = os.path.dirname(os.path.abspath(__file__))
VIEWER = ("kubeflow.org", "v1alpha1", "pvcviewers")
VIEWER_SPEC_PATHS = ["/etc/config/viewer-spec.yaml", os.path.join(HERE, "config", "viewer-spec.yaml")]
POD_PARENT_VIEWER_LABEL_KEY = "app.kubernetes.io/name"


# ------------------------------------------------------------------ form
def handle_storage_class(vol):
    if "class" not in vol:
        return None
    if vol["class"] == "{none}":
        return ""
    if vol["class"] == "{empty}":
        return None
    return vol["class"]


def pvc_from_dict(body, namespace) -> dict:
    spec = {"accessModes": [body["mode"]], "resources": {"requests": {"storage": body["size"]}}}
    sc = handle_storage_class(body)
    if sc is not None:
        spec["storageClassName"] = sc
    return {"apiVersion": "v1", "kind": "PersistentVolumeClaim",
            "metadata": {"name": body["name"], "namespace": namespace}, "spec": spec}


# ------------------------------------------------------------------ status
def pvc_status(pvc, events=None):
    if pvc["metadata"].get("deletionTimestamp"):
        return create_status(STATUS_PHASE.TERMINATING, "Deleting Volume...")
    if (pvc.get("status") or {}).get("phase") == "Bound":
        return create_status(STATUS_PHASE.READY, "Bound")
    if events is None:
        events = cb.client().list("v1", "Event", pvc["metadata"]["namespace"],
                                  field_selector=cb.events_field_selector("PersistentVolumeClaim",
                                                                          pvc["metadata"]["name"]))
    if not events:
        return create_status(STATUS_PHASE.WAITING, "Provisioning Volume...")
    ev = events[0]
    msg, state, phase = f"Pending: {ev.get('message', '')}", ev.get("reason", ""), STATUS_PHASE.WAITING
    if state == "WaitForFirstConsumer":
        phase = STATUS_PHASE.UNAVAILABLE
        msg = ("Pending: This volume will be bound when its first consumer is created. E.g., when you first "
               "browse its contents, or attach it to a notebook server")
    elif state == "Provisioning":
        phase = STATUS_PHASE.WAITING
    elif state == "FailedBinding" or ev.get("type") == "Warning":
        phase = STATUS_PHASE.WARNING
    elif ev.get("type") == "Normal":
        phase = STATUS_PHASE.READY
    return create_status(phase, msg, state)


def viewer_status(viewer):
    if not viewer:
        return STATUS_PHASE.UNINITIALIZED
    if "deletionTimestamp" in viewer.get("metadata", {}):
        return STATUS_PHASE.TERMINATING
    if (viewer.get("status") or {}).get("ready", False):
        return STATUS_PHASE.READY
    return STATUS_PHASE.WAITING


# ------------------------------------------------------------------ utils
def get_notebook_pvcs(nb):
    vols = nb["spec"]["template"]["spec"].get("volumes") or []
    return [v["persistentVolumeClaim"]["claimName"] for v in vols if v.get("persistentVolumeClaim")]


def get_notebooks_using_pvc(pvc, notebooks):
    return [nb["metadata"]["name"] for nb in notebooks if pvc in get_notebook_pvcs(nb)]


def get_pod_pvcs(pod):
    vols = (pod.get("spec") or {}).get("volumes") or []
    return [v["persistentVolumeClaim"]["claimName"] for v in vols if v.get("persistentVolumeClaim")]


def get_pods_using_pvc(pvc, namespace):
    return [p for p in api.list_pods(namespace) if pvc in get_pod_pvcs(p)]


def parse_pvc(pvc, notebooks, events=None):
    cap = ((pvc.get("status") or {}).get("capacity") or {}).get("storage") or \
        pvc["spec"]["resources"]["requests"]["storage"]
    return {"name": pvc["metadata"]["name"], "namespace": pvc["metadata"]["namespace"],
            "status": pvc_status(pvc, events), "age": pvc["metadata"]["creationTimestamp"], "capacity": cap,
            "modes": pvc["spec"].get("accessModes"), "class": pvc["spec"].get("storageClassName"),
            "notebooks": get_notebooks_using_pvc(pvc["metadata"]["name"], notebooks)}


# ------------------------------------------------------------------ viewer
def _substitute(data, variables):
    if isinstance(data, dict):
        return {k: _substitute(v, variables) for k, v in data.items()}
    if isinstance(data, list):
        return [_substitute(v, variables) for v in data]
    if isinstance(data, str):
        try:
            return Template(data).substitute(**variables)
        except (ValueError, KeyError):
            return data
    return data


def create_viewer_template(name, namespace, env=None):
    path = next((p for p in VIEWER_SPEC_PATHS if os.path.exists(p)), None)
    if path is None:
        raise exceptions.NotFound("viewer-spec.yaml not found")
    with open(path) as f:
        tmpl = yaml.safe_load(f)
    variables = dict(os.environ if env is None else env)
    variables.update(PVC_NAME=name, NAMESPACE=namespace, NAME=name)
    return {"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer",
            "metadata": {"name": name, "namespace": namespace}, "spec": _substitute(copy.deepcopy(tmpl), variables)}


def get_owning_viewer(pod):
    return (pod.get("metadata", {}).get("labels") or {}).get(POD_PARENT_VIEWER_LABEL_KEY)


def is_viewer_pod(pod):
    return get_owning_viewer(pod) is not None


# ------------------------------------------------------------------ routes
bp = Blueprint("vwa_routes", __name__)


@bp.route("/api/namespaces/<namespace>/pvcs")
def get_pvcs(namespace):
    notebooks = api.list_notebooks(namespace)
    content = [parse_pvc(p, notebooks) for p in api.list_pvcs(namespace)]
    viewers = {v["metadata"]["name"]: v for v in api.list_custom_rsrc(*VIEWER, namespace)}
    for pvc in content:
        v = viewers.get(pvc["name"], {})
        pvc["viewer"] = {"status": viewer_status(v), "url": (v.get("status") or {}).get("url")}
    return success_response("pvcs", content)


@bp.route("/api/namespaces/<namespace>/pvcs/<pvc_name>")
def get_pvc(namespace, pvc_name):
    return success_response("pvc", api.get_pvc(pvc_name, namespace))


@bp.route("/api/namespaces/<namespace>/pvcs/<pvc_name>/pods")
def get_pvc_pods(namespace, pvc_name):
    return success_response("pods", get_pods_using_pvc(pvc_name, namespace))


@bp.route("/api/namespaces/<namespace>/pvcs/<pvc_name>/events")
def get_pvc_events(namespace, pvc_name):
    return success_response("events", api.list_pvc_events(namespace, pvc_name))


@bp.route("/api/namespaces/<namespace>/pvcs", methods=["POST"])
@cb.request_is_json_type
@cb.required_body_params("name", "mode", "class", "size", "type")
def post_pvc(namespace):
    api.create_pvc(pvc_from_dict(request.get_json(), namespace), namespace)
    return success_response("message", "PVC created successfully.")


@bp.route("/api/namespaces/<namespace>/viewers", methods=["POST"])
@cb.request_is_json_type
@cb.required_body_params("name")
def post_viewer(namespace):
    api.create_custom_rsrc(*VIEWER, create_viewer_template(request.get_json()["name"], namespace), namespace)
    return success_response("message", "PVCViewer created successfully.")


@bp.route("/api/namespaces/<namespace>/pvcs/<pvc>", methods=["DELETE"])
def delete_pvc(pvc, namespace):
    pods = get_pods_using_pvc(pvc, namespace)
    viewer_pods = [p for p in pods if is_viewer_pod(p)]
    others = [p["metadata"]["name"] for p in pods if not is_viewer_pod(p)]
    if others:
        raise exceptions.Conflict("Cannot delete PVC '%s' because it is being used by pods: %s" % (pvc, others))
    for vp in viewer_pods:
        api.delete_custom_rsrc(*VIEWER, get_owning_viewer(vp), namespace)
    api.delete_pvc(pvc, namespace)
    return success_response("message", "PVC %s successfully deleted." % pvc)


@bp.route("/api/namespaces/<namespace>/viewers/<viewer>", methods=["DELETE"])
def delete_viewer(viewer, namespace):
    api.delete_custom_rsrc(*VIEWER, viewer, namespace)
    return success_response("message", "Viewer %s successfully deleted." % viewer)


def create_app(kube, name="Volumes Web App", cfg=None, settings_env=None):
    cfg = cfg or cb.Config()
    static = os.path.join(HERE, "static", "volumes")
    cfg.STATIC_DIR = static                      # index.html of this app
    app = cb.create_app(name, os.path.join(HERE, "static"), cfg, kube, settings_env=settings_env)
    app.register_blueprint(bp)
    return app
