"""P2: Jupyter web app (JWA) backend.

Behavioural reference: components/crud-web-apps/jupyter/backend/apps/common/{form.py,
utils.py, status.py, volumes.py, routes/get.py, routes/patch.py, routes/delete.py},
apps/default/routes/post.py, entrypoint.py, apps/common/yaml/spawner_ui_config.yaml.

Routes (same URLs and response fields as the reference, so its Angular frontend works
unchanged): ``GET /api/config``, ``GET /api/gpus``, ``GET /api/namespaces/<ns>/{pvcs,
poddefaults,notebooks}``, ``GET .../notebooks/<name>`` (+ ``processed_status``),
``.../pod``, ``.../pod/<pod>/logs``, ``.../events``, ``POST .../notebooks`` (dry-run the
Notebook and every new PVC first, then create), ``PATCH .../notebooks/<name>``
``{"stopped": bool}`` (the ``kubeflow-resource-stopped`` annotation the notebook
controller scales on), ``DELETE .../notebooks/<name>`` (foreground).

The form's GPU field writes ``limits[vendor] = num``; this deployment's config offers the
``amd.com/gpu`` device-plugin resource (MI355X), which the local kubelet turns into
``HIP_VISIBLE_DEVICES`` for the notebook pod.
"""
from __future__ import annotations

import datetime as dt
import json
import logging
import os
import random
import string
import threading
import time

from flask import Blueprint, request
from werkzeug import exceptions

from . import crud_backend as cb
from .crud_backend import STATUS_PHASE, api, create_status, success_response

log = logging.getLogger("jwa")
HERE = os.path.dirname(os.path.abspath(__file__))
DEV_CONFIG = os.path.join(HERE, "config", "spawner_ui_config.yaml")
CONFIGS = ["/etc/config/spawner_ui_config.yaml", DEV_CONFIG]
SERVER_TYPE_ANNOTATION = "notebooks.kubeflow.org/server-type"
HEADERS_ANNOTATION = "notebooks.kubeflow.org/http-headers-request-set"
URI_REWRITE_ANNOTATION = "notebooks.kubeflow.org/http-rewrite-uri"
LAST_ACTIVITY_ANNOTATION = "notebooks.kubeflow.org/last-activity"
STOP_ANNOTATION = "kubeflow-resource-stopped"
EVENT_TYPE_WARNING = "Warning"
TS_FMT = "%Y-%m-%dT%H:%M:%SZ"

# ------------------------------------------------------------------ config (60 s TTL cache)
_cfg_lock = threading.Lock()
_cfg_cache = {"t": -1e18, "v": None}
CONFIG_TTL_S = 60.0


def load_spawner_ui_config():
    with _cfg_lock:
        if _cfg_cache["v"] is not None and time.monotonic() - _cfg_cache["t"] < CONFIG_TTL_S:
            return _cfg_cache["v"]
        paths = ([os.environ["SPAWNER_UI_CONFIG"]] if os.environ.get("SPAWNER_UI_CONFIG") else []) + CONFIGS
        for p in paths:
            d = cb.load_yaml(p) if os.path.exists(p) else None
            if d is not None:
                log.info("Using config file: %s", p)
                _cfg_cache.update(t=time.monotonic(), v=d["spawnerFormDefaults"])
                return _cfg_cache["v"]
    raise exceptions.NotFound("Couldn't find any config file.")


def clear_config_cache():
    with _cfg_lock:
        _cfg_cache.update(t=-1e18, v=None)


def random_string(size=9, chars=string.ascii_lowercase + string.digits):
    return "".join(random.choice(chars) for _ in range(size))


def notebook_template(name, namespace, service_account, creator) -> dict:
    return {"apiVersion": "kubeflow.org/v1beta1", "kind": "Notebook",
            "metadata": {"name": name, "namespace": namespace, "labels": {"app": name},
                         "annotations": {SERVER_TYPE_ANNOTATION: "", "notebooks.kubeflow.org/creator": creator}},
            "spec": {"template": {"spec": {
                "serviceAccountName": service_account,
                "containers": [{"name": name, "image": "", "volumeMounts": [], "env": [],
                                "resources": {"requests": {"cpu": "0.1", "memory": "0.1Gi"}}}],
                "volumes": [], "tolerations": []}}}}


# ------------------------------------------------------------------ form
def get_form_value(body, defaults, body_field, defaults_field=None, optional=False):
    defaults_field = defaults_field or body_field
    user_value = body.get(body_field, None)
    if defaults_field not in defaults:
        return user_value
    readonly = defaults[defaults_field].get("readOnly", False)
    default_value = defaults[defaults_field]["value"]
    if readonly:
        if body_field in body:
            raise exceptions.BadRequest("'%s' is readonly but a value was provided: %s" % (body_field, user_value))
        return default_value
    if user_value is None:
        if not optional:
            raise exceptions.BadRequest("No value provided for: %s" % body_field)
        return None
    return user_value


def _ctr(nb):
    return nb["spec"]["template"]["spec"]["containers"][0]


def set_notebook_image(nb, body, defaults):
    field = "customImage" if body.get("customImage", False) else "image"
    _ctr(nb)["image"] = get_form_value(body, defaults, field, "image").strip()


def set_notebook_image_pull_policy(nb, body, defaults):
    _ctr(nb)["imagePullPolicy"] = get_form_value(body, defaults, "imagePullPolicy")


def set_server_type(nb, body, defaults):
    server_type = get_form_value(body, defaults, "serverType")
    if server_type not in ("jupyter", "group-one", "group-two"):
        raise exceptions.BadRequest("'%s' is not a valid server type" % server_type)
    name = get_form_value(body, defaults, "name")
    ns = get_form_value(body, defaults, "namespace")
    ann = nb["metadata"]["annotations"]
    ann[SERVER_TYPE_ANNOTATION] = server_type
    if server_type in ("group-one", "group-two"):
        ann[URI_REWRITE_ANNOTATION] = "/"
    if server_type == "group-two":
        ann[HEADERS_ANNOTATION] = '{"X-RStudio-Root-Path":"/notebook/%s/%s/"}' % (ns, name)


def _set_quantity(nb, body, defaults, field, unit):
    ctr = _ctr(nb)
    req = get_form_value(body, defaults, field)
    if req and "nan" in req.lower():
        raise exceptions.BadRequest("Invalid value for %s: %s" % (field, req))
    lim_field = field + "Limit"
    lim = get_form_value(body, defaults, lim_field)
    if lim and "nan" in lim.lower():
        raise exceptions.BadRequest("Invalid value for %s limit: %s" % (field, lim))
    factor = load_spawner_ui_config()[field].get("limitFactor")
    strip = (lambda v: float(v.replace(unit, ""))) if unit else float
    if not lim and factor != "none":
        lim = str(round(strip(req) * float(factor), 1)) + unit
    ctr["resources"]["requests"][field] = req
    if lim is None or lim == "":
        return
    if strip(lim) < strip(req):
        raise exceptions.BadRequest("%s limit must be greater than the request"
                                    % ("CPU" if field == "cpu" else "Memory"))
    ctr["resources"].setdefault("limits", {})[field] = lim


def set_notebook_cpu(nb, body, defaults):
    _set_quantity(nb, body, defaults, "cpu", "")


def set_notebook_memory(nb, body, defaults):
    _set_quantity(nb, body, defaults, "memory", "Gi")


def set_notebook_gpus(nb, body, defaults):
    gpus = get_form_value(body, defaults, "gpus")
    if "num" not in gpus:
        raise exceptions.BadRequest("'gpus' must have a 'num' field")
    if gpus["num"] == "none":
        return
    if "vendor" not in gpus:
        raise exceptions.BadRequest("'gpus' must have a 'vendor' field")
    _ctr(nb)["resources"].setdefault("limits", {})[gpus["vendor"]] = str(gpus["num"])


def set_notebook_tolerations(nb, body, defaults):
    key = get_form_value(body, defaults, "tolerationGroup")
    if key == "none":
        return
    for g in load_spawner_ui_config().get("tolerationGroup", {}).get("options", []):
        if g["groupKey"] == key:
            nb["spec"]["template"]["spec"]["tolerations"].extend(g["tolerations"])
            return
    log.warning("Didn't find any Toleration Group with key '%s' in the config", key)


def set_notebook_affinity(nb, body, defaults):
    key = get_form_value(body, defaults, "affinityConfig")
    if key == "none":
        return
    for a in load_spawner_ui_config().get("affinityConfig", {}).get("options", []):
        if a["configKey"] == key:
            nb["spec"]["template"]["spec"]["affinity"] = a["affinity"]
            return
    log.warning("Didn't find any Affinity Config with key '%s' in the config", key)


def set_notebook_configurations(nb, body, defaults):
    labels = get_form_value(body, defaults, "configurations")
    if not isinstance(labels, list):
        raise exceptions.BadRequest("Labels for PodDefaults are not list: %s" % labels)
    for lab in labels:
        nb["metadata"]["labels"][lab] = "true"


def set_notebook_shm(nb, body, defaults):
    if not get_form_value(body, defaults, "shm"):
        return
    nb["spec"]["template"]["spec"]["volumes"].append({"name": "dshm", "emptyDir": {"medium": "Memory"}})
    _ctr(nb)["volumeMounts"].append({"mountPath": "/dev/shm", "name": "dshm"})


def set_notebook_environment(nb, body, defaults):
    env = get_form_value(body, defaults, "environment")
    env = json.loads(env) if isinstance(env, str) and env else (env or {})
    _ctr(nb)["env"] += [{"name": k, "value": str(v)} for k, v in env.items()]


# ------------------------------------------------------------------ volumes
def check_volume_format(v):
    if "mount" not in v:
        raise exceptions.BadRequest("Volume should have a mount: %s" % v)
    has_ex, has_new = "existingSource" in v, "newPvc" in v
    if not has_ex and not has_new:
        raise exceptions.BadRequest("Volume has neither existingSource nor newPvc: %s" % v)
    if has_ex and has_new:
        raise exceptions.BadRequest("Volume has both existingSource and newPvc: %s" % v)


def get_volume_name(v):
    if "existingSource" not in v:
        raise exceptions.BadRequest("Failed to retrieve a volume name from '%s'" % v)
    src = v["existingSource"]
    if "persistentVolumeClaim" in src:
        if "claimName" not in src["persistentVolumeClaim"]:
            raise exceptions.BadRequest("Failed to retrieve the PVC name from '%s'" % v)
        return src["persistentVolumeClaim"]["claimName"]
    return "existing-source-volume-%s" % random_string(8)


def get_pod_volume(v, pvc):
    check_volume_format(v)
    if pvc is not None:
        n = pvc["metadata"]["name"]
        return {"name": n, "persistentVolumeClaim": {"claimName": n}}
    return dict({"name": get_volume_name(v)}, **v["existingSource"])


def get_container_mount(v, volume_name):
    check_volume_format(v)
    return {"name": volume_name, "mountPath": v["mount"]}


def get_new_pvc(v):
    check_volume_format(v)
    if "newPvc" not in v:
        return None
    pvc = json.loads(json.dumps(v["newPvc"]))
    if not isinstance(pvc.get("metadata"), dict) or not isinstance(pvc.get("spec"), dict):
        raise exceptions.BadRequest("newPvc must have metadata and spec: %s" % v)
    if pvc["metadata"].get("namespace") is not None:
        raise exceptions.BadRequest("PVC should not specify the namespace.")
    return dict(pvc, apiVersion="v1", kind="PersistentVolumeClaim")


def add_notebook_volume(nb, volume):
    nb["spec"]["template"]["spec"].setdefault("volumes", []).append(volume)
    return nb


def add_notebook_container_mount(nb, mount):
    _ctr(nb).setdefault("volumeMounts", []).append(mount)
    return nb


# ------------------------------------------------------------------ status
def _ts(s):
    return dt.datetime.strptime(s, TS_FMT)


def get_empty_status(nb, now=None):
    st = nb.get("status") or {}
    created = _ts(nb["metadata"]["creationTimestamp"])
    now = now or dt.datetime.utcnow().replace(microsecond=0)
    if not st.get("containerState") and not st.get("conditions") and (now - created).total_seconds() <= 10:
        return STATUS_PHASE.WAITING, "Waiting for StatefulSet to create the underlying Pod."
    return None, None


def get_stopped_status(nb):
    ready = (nb.get("status") or {}).get("readyReplicas", 0)
    if STOP_ANNOTATION in (nb["metadata"].get("annotations") or {}):
        if ready == 0:
            return STATUS_PHASE.STOPPED, "No Pods are currently running for this Notebook Server."
        return STATUS_PHASE.WAITING, "Notebook Server is stopping."
    return None, None


def get_deleted_status(nb):
    if "deletionTimestamp" in nb["metadata"]:
        return STATUS_PHASE.TERMINATING, "Deleting this Notebook Server."
    return None, None


def check_ready_nb(nb):
    if (nb.get("status") or {}).get("readyReplicas", 0) == 1:
        return STATUS_PHASE.READY, "Running"
    return None, None


def get_status_from_container_state(nb):
    cs = (nb.get("status") or {}).get("containerState") or {}
    if "waiting" not in cs:
        return None, None
    w = cs["waiting"]
    if w.get("reason") == "PodInitializing":
        return STATUS_PHASE.WAITING, w["reason"]
    return STATUS_PHASE.WARNING, "%s: %s" % (w.get("reason", "Undefined"),
                                              w.get("message", "No available message for container state."))


def get_status_from_conditions(nb):
    for c in (nb.get("status") or {}).get("conditions") or []:
        if "reason" in c:
            return STATUS_PHASE.WARNING, c["reason"] + ": " + c.get("message", "")
    return None, None


def event_timestamp(e):
    t = e["metadata"].get("creationTimestamp") or e.get("lastTimestamp") or "1970-01-01T00:00:00Z"
    return _ts(t)


def get_status_from_events(events):
    for e in sorted(events, key=event_timestamp, reverse=True):
        if e.get("type") == EVENT_TYPE_WARNING:
            return STATUS_PHASE.WARNING, e.get("message", "")
    return None, None


def process_status(nb, events_fn=None, now=None):
    for fn in (lambda n: get_empty_status(n, now), get_stopped_status, get_deleted_status, check_ready_nb,
               get_status_from_container_state, get_status_from_conditions):
        phase, msg = fn(nb)
        if phase is not None:
            return create_status(phase, msg)
    if events_fn is not None:
        created = _ts(nb["metadata"]["creationTimestamp"])
        evs = [e for e in events_fn(nb) if event_timestamp(e) >= created]
        phase, msg = get_status_from_events(evs)
        if phase is not None:
            return create_status(phase, msg)
    return create_status(STATUS_PHASE.WARNING, "Couldn't find any information for the status of this notebook.")


def _api_events(nb):
    return api.list_notebook_events(nb["metadata"]["name"], nb["metadata"]["namespace"])


def process_gpus(container):
    vendors = load_spawner_ui_config().get("gpus", {}).get("value", {}).get("vendors", [])
    names = {v["limitsKey"]: v["uiName"] for v in vendors}
    limits = (container.get("resources") or {}).get("limits") or {}
    count, parts = 0, []
    for key, ui in names.items():
        if key in limits:
            count += int(limits[key])
            parts.append("%s %s" % (limits[key], ui))
    return {"count": count, "message": ", ".join(parts)}


def notebook_dict_from_k8s_obj(nb):
    c = _ctr(nb)
    ann = nb["metadata"].get("annotations") or {}
    return {"name": nb["metadata"]["name"], "namespace": nb["metadata"]["namespace"],
            "serverType": ann.get(SERVER_TYPE_ANNOTATION), "age": nb["metadata"]["creationTimestamp"],
            "last_activity": ann.get(LAST_ACTIVITY_ANNOTATION, ""), "image": c["image"],
            "shortImage": c["image"].split("/")[-1], "cpu": c["resources"]["requests"]["cpu"],
            "gpus": process_gpus(c), "memory": c["resources"]["requests"]["memory"],
            "volumes": [v["name"] for v in c.get("volumeMounts") or []],
            "status": process_status(nb, _api_events), "metadata": nb["metadata"]}


# ------------------------------------------------------------------ routes
bp = Blueprint("jwa_routes", __name__)


@bp.route("/api/config")
def get_config():
    return success_response("config", load_spawner_ui_config())


@bp.route("/api/namespaces/<namespace>/pvcs")
def get_pvcs(namespace):
    return success_response("pvcs", [{"name": p["metadata"]["name"],
                                      "size": p["spec"]["resources"]["requests"]["storage"],
                                      "mode": p["spec"]["accessModes"][0]} for p in api.list_pvcs(namespace)])


@bp.route("/api/namespaces/<namespace>/poddefaults")
def get_poddefaults(namespace):
    out = []
    for pd in api.list_poddefaults(namespace):
        pd["label"] = list(pd["spec"]["selector"]["matchLabels"].keys())[0]
        pd["desc"] = pd["spec"].get("desc", pd["metadata"]["name"])
        out.append(pd)
    return success_response("poddefaults", out)


@bp.route("/api/namespaces/<namespace>/notebooks")
def get_notebooks(namespace):
    return success_response("notebooks", [notebook_dict_from_k8s_obj(nb) for nb in api.list_notebooks(namespace)])


@bp.route("/api/namespaces/<namespace>/notebooks/<name>")
def get_notebook(name, namespace):
    nb = api.get_notebook(name, namespace)
    nb["processed_status"] = process_status(nb, _api_events)
    return success_response("notebook", nb)


@bp.route("/api/namespaces/<namespace>/notebooks/<notebook_name>/pod")
def get_notebook_pod(notebook_name, namespace):
    pods = api.list_pods(namespace, label_selector="notebook-name=" + notebook_name)
    if not pods:
        raise exceptions.NotFound("No pod detected.")
    return success_response("pod", pods[0])


@bp.route("/api/namespaces/<namespace>/notebooks/<notebook_name>/pod/<pod_name>/logs")
def get_pod_logs(namespace, notebook_name, pod_name):
    return success_response("logs", api.get_pod_logs(namespace, pod_name, notebook_name).split("\n"))


@bp.route("/api/namespaces/<namespace>/notebooks/<notebook_name>/events")
def get_notebook_events(notebook_name, namespace):
    return success_response("events", api.list_notebook_events(notebook_name, namespace))


@bp.route("/api/gpus")
def get_gpu_vendors():
    keys = [v.get("limitsKey", "") for v in
            load_spawner_ui_config().get("gpus", {}).get("value", {}).get("vendors", [])]
    installed = set()
    for node in api.list_nodes():
        installed.update(((node.get("status") or {}).get("capacity") or {}).keys())
    return success_response("vendors", sorted(installed.intersection(keys)))


@bp.route("/api/namespaces/<namespace>/notebooks", methods=["POST"])
@cb.request_is_json_type
@cb.required_body_params("name")
def post_notebook(namespace):
    body = request.get_json()
    user = cb.get_username()
    nb = notebook_template(body["name"], namespace, "default-editor",
                           user if user is not None else "anonymous@kubeflow.org")
    defaults = load_spawner_ui_config()
    for setter in (set_notebook_image, set_notebook_image_pull_policy, set_server_type, set_notebook_cpu,
                   set_notebook_memory, set_notebook_gpus, set_notebook_tolerations, set_notebook_affinity,
                   set_notebook_configurations, set_notebook_shm):
        setter(nb, body, defaults)
    if "environment" in body:
        set_notebook_environment(nb, body, defaults)
    vols = list(get_form_value(body, defaults, "datavols", "dataVolumes") or [])
    ws = get_form_value(body, defaults, "workspace", "workspaceVolume", optional=True)
    if ws:
        vols.append(ws)
    # dry-run everything first so a bad PVC does not leave a half-created notebook
    api.create_notebook(nb, namespace, dry_run=True)
    for v in vols:
        pvc = get_new_pvc(v)
        if pvc is not None:
            api.create_pvc(pvc, namespace, dry_run=True)
    for v in vols:
        pvc = get_new_pvc(v)
        if pvc is not None:
            pvc = api.create_pvc(pvc, namespace)
        vol = get_pod_volume(v, pvc)
        add_notebook_volume(nb, vol)
        add_notebook_container_mount(nb, get_container_mount(v, vol["name"]))
    api.create_notebook(nb, namespace)
    return success_response("message", "Notebook created successfully.")


@bp.route("/api/namespaces/<namespace>/notebooks/<notebook>", methods=["PATCH"])
@cb.request_is_json_type
def patch_notebook(namespace, notebook):
    body = request.get_json()
    if body is None:
        raise exceptions.BadRequest("Request doesn't have a body.")
    if "stopped" not in body:
        raise exceptions.BadRequest("Request body must include at least one supported key: ['stopped']")
    if body["stopped"]:
        nb = api.get_notebook(notebook, namespace)
        if STOP_ANNOTATION in (nb["metadata"].get("annotations") or {}):
            raise exceptions.Conflict("Notebook %s/%s is already stopped." % (namespace, notebook))
        ts = dt.datetime.now(dt.timezone.utc).strftime(TS_FMT)
        patch = {"metadata": {"annotations": {STOP_ANNOTATION: ts}}}
    else:
        patch = {"metadata": {"annotations": {STOP_ANNOTATION: None}}}
    api.patch_notebook(notebook, namespace, patch)
    return success_response()


@bp.route("/api/namespaces/<namespace>/notebooks/<notebook>", methods=["DELETE"])
def delete_notebook(notebook, namespace):
    api.delete_notebook(notebook, namespace)
    return success_response("message", "Notebook %s successfully deleted." % notebook)


def create_app(kube, name="Jupyter Web App", cfg=None, settings_env=None, pod_log_reader=None):
    cfg = cfg or cb.Config()
    static = os.path.join(HERE, "static", "jupyter")
    cfg.STATIC_DIR = static                      # index.html of this app
    app = cb.create_app(name, os.path.join(HERE, "static"), cfg, kube, settings_env=settings_env, pod_log_reader=pod_log_reader)
    app.register_blueprint(bp)
    return app
