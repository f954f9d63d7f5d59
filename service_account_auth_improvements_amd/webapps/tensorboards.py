"""P3: Tensorboards web app (TWA) backend.

Behavioural reference: components/crud-web-apps/tensorboards/backend/app/{utils.py,
routes/get.py, routes/post.py, routes/delete.py}.

``GET /api/namespaces/<ns>/tensorboards`` (name, namespace, logspath, age, status ready
iff readyReplicas == 1), ``GET .../pvcs`` (names), ``GET .../poddefaults``,
``POST .../tensorboards`` (``name``, ``logspath``, ``configurations`` -> PodDefault
labels), ``DELETE .../tensorboards/<name>`` (foreground).  A ``pvc://<claim>/<subpath>``
logspath pointed at a training job's output volume shows the kfamd trainer's
loss / tokens-per-second event files.
"""
from __future__ import annotations

import os

from flask import Blueprint, request
from werkzeug import exceptions

from . import crud_backend as cb
from .crud_backend import STATUS_PHASE, api, create_status, success_response

TB = ("tensorboard.kubeflow.org", "v1alpha1", "tensorboards")
HERE = os.path.dirname(os.path.abspath(__file__))


def parse_tensorboard(tb: dict) -> dict:
    if (tb.get("status") or {}).get("readyReplicas", 0) == 1:
        phase, msg = STATUS_PHASE.READY, "The Tensorboard server is ready to connect"
    else:
        phase, msg = STATUS_PHASE.UNAVAILABLE, "The Tensorboard server is currently unavailble"
    return {"name": tb["metadata"]["name"], "namespace": tb["metadata"]["namespace"],
            "logspath": tb["spec"]["logspath"], "age": tb["metadata"]["creationTimestamp"],
            "status": create_status(phase, msg, "")}


def get_tensorboard_configurations(body) -> dict:
    labels = body.get("configurations", None)
    if not isinstance(labels, list):
        raise exceptions.BadRequest("Labels for PodDefaults are not list: %s" % labels)
    return {lab: "true" for lab in labels}


def get_tensorboard_dict(namespace, body) -> dict:
    meta = {"name": body["name"], "namespace": namespace}
    labels = get_tensorboard_configurations(body)
    if labels:
        meta["labels"] = labels
    return {"apiVersion": "tensorboard.kubeflow.org/v1alpha1", "kind": "Tensorboard", "metadata": meta,
            "spec": {"logspath": body["logspath"]}}


bp = Blueprint("twa_routes", __name__)


@bp.route("/api/namespaces/<namespace>/tensorboards")
def get_tensorboards(namespace):
    return success_response("tensorboards", [parse_tensorboard(t) for t in api.list_custom_rsrc(*TB, namespace)])


@bp.route("/api/namespaces/<namespace>/pvcs")
def get_pvcs(namespace):
    return success_response("pvcs", [p["metadata"]["name"] for p in api.list_pvcs(namespace)])


@bp.route("/api/namespaces/<namespace>/poddefaults")
def get_poddefaults(namespace):
    out = []
    for pd in api.list_poddefaults(namespace):
        pd["label"] = list(pd["spec"]["selector"]["matchLabels"].keys())[0]
        pd["desc"] = pd["spec"].get("desc", pd["metadata"]["name"])
        out.append(pd)
    return success_response("poddefaults", out)


@bp.route("/api/namespaces/<namespace>/tensorboards", methods=["POST"])
@cb.request_is_json_type
@cb.required_body_params("name", "logspath")
def post_tensorboard(namespace):
    api.create_custom_rsrc(*TB, get_tensorboard_dict(namespace, request.get_json()), namespace)
    return success_response("message", "Tensorboard created successfully.")


@bp.route("/api/namespaces/<namespace>/tensorboards/<tensorboard>", methods=["DELETE"])
def delete_tensorboard(tensorboard, namespace):
    api.delete_custom_rsrc(*TB, tensorboard, namespace)
    return success_response("message", "Tensorboard deleted successfully.")


def create_app(kube, name="Tensorboards Web App", cfg=None, settings_env=None):
    cfg = cfg or cb.Config()
    static = os.path.join(HERE, "static", "tensorboards")
    cfg.STATIC_DIR = static                      # index.html of this app
    app = cb.create_app(name, os.path.join(HERE, "static"), cfg, kube, settings_env=settings_env)
    app.register_blueprint(bp)
    return app
