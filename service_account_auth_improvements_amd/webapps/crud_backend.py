"""P1: the shared CRUD web-app backend library (Flask).

Behavioural reference: components/crud-web-apps/common/backend/kubeflow/kubeflow/crud_backend/
(__init__.py create_app, authn.py, authz.py, csrf.py, settings.py, config.py, errors/handlers.py,
probes.py, serving.py, decorators.py, status.py, helpers.py, api/*.py, routes/get.py).

Differences by design: the Kubernetes client is this repo's :class:`Client` (in-memory API
server or :class:`RestClient`) carried on the Flask app, objects are plain dicts, and the
settings are read when the app is created (not at import), so several apps with different
settings can live in one process.  The behaviour the frontends depend on is kept:

* authn: user = ``USERID_HEADER`` (default ``kubeflow-userid``) minus ``USERID_PREFIX``
  (default ``:``); every route needs a user unless decorated ``no_authentication``;
  ``APP_DISABLE_AUTH=true`` or dev mode skips authn and authz.
* authz: a SubjectAccessReview per API call (``ensure_authorized``), 403 with the
  reference's message text on denial.
* csrf: double-submit cookie ``XSRF-TOKEN`` / header ``X-XSRF-TOKEN`` for unsafe methods;
  the cookie is refreshed every time ``index.html`` is served (``CSRF_SAMESITE``,
  ``APP_SECURE_COOKIES``).
* errors: every failure is ``{"success": false, "log": msg, "status": code, "user": u}``;
  success is ``{"status": 200, "success": true, "user": u, <field>: data}``.
* probes ``/healthz/liveness`` ``/healthz/readiness``; SPA serving with ``<base href=PREFIX>``.
"""
from __future__ import annotations

import datetime as dt
import enum
import functools
import logging
import os
import re
import secrets
from typing import Optional

import yaml
from flask import Blueprint, Flask, Response, current_app, jsonify, request
from werkzeug import exceptions

from ..controlplane.apiserver import ApiError
from ..controlplane.client import Client

log = logging.getLogger("crud_backend")
LOG_FORMAT = "%(asctime)s | %(name)s | %(levelname)s | %(message)s"

CSRF_COOKIE = "XSRF-TOKEN"
CSRF_HEADER = "X-" + CSRF_COOKIE
SAMESITE_VALUES = ["Strict", "Lax", "None"]
NO_CACHE = "no-cache, no-store, must-revalidate, max-age=0"


# ------------------------------------------------------------------ settings / config
class Settings:
    def __init__(self, env=None):
        env = os.environ if env is None else env
        self.SECURE_COOKIES = env.get("APP_SECURE_COOKIES", "true").lower() == "true"
        self.DISABLE_AUTH = env.get("APP_DISABLE_AUTH", "false").lower() == "true"
        self.USER_HEADER = env.get("USERID_HEADER", "kubeflow-userid")
        self.USER_PREFIX = env.get("USERID_PREFIX", ":")
        self.CSRF_SAMESITE = env.get("CSRF_SAMESITE", "Strict")


class BackendMode(enum.Enum):
    DEVELOPMENT = "dev"
    DEVELOPMENT_FULL = "development"
    PRODUCTION = "prod"
    PRODUCTION_FULL = "production"


class Config:
    ENV = "generic"
    DEBUG = False
    STATIC_DIR = "./static/"
    LOG_LEVEL = logging.INFO
    PREFIX = "/"

    def __init__(self):
        if os.environ.get("LOG_LEVEL_DEBUG", "false") == "true":
            self.LOG_LEVEL = logging.DEBUG


class DevConfig(Config):
    ENV = BackendMode.DEVELOPMENT_FULL.value
    DEBUG = True
    LOG_LEVEL = logging.DEBUG


class ProdConfig(Config):
    ENV = BackendMode.PRODUCTION_FULL.value


def get_config(mode: str) -> Config:
    classes = {BackendMode.DEVELOPMENT.value: DevConfig, BackendMode.DEVELOPMENT_FULL.value: DevConfig,
               BackendMode.PRODUCTION.value: ProdConfig, BackendMode.PRODUCTION_FULL.value: ProdConfig}
    if mode not in classes:
        raise RuntimeError("Backend mode '%s' is not implemented. Choose one of %s" % (mode, list(classes)))
    return classes[mode]()


def dev_mode_enabled() -> bool:
    return current_app.config.get("ENV") in (BackendMode.DEVELOPMENT.value, BackendMode.DEVELOPMENT_FULL.value)


def settings() -> Settings:
    return current_app.extensions["kfamd_settings"]


def client() -> Client:
    return current_app.extensions["kfamd_client"]


# ------------------------------------------------------------------ authn
authn_bp = Blueprint("authn", __name__)


def get_username() -> Optional[str]:
    s = settings()
    if s.USER_HEADER not in request.headers:
        return None
    return request.headers[s.USER_HEADER].replace(s.USER_PREFIX, "")


def no_authentication(func):
    func.no_authentication = True
    return func


@authn_bp.before_app_request
def check_authentication():
    if dev_mode_enabled() or settings().DISABLE_AUTH:
        return
    if request.endpoint and getattr(current_app.view_functions.get(request.endpoint), "no_authentication", False):
        return
    if get_username() is None:
        raise exceptions.Unauthorized("No user detected.")


# ------------------------------------------------------------------ authz
def is_authorized(user, verb, group, version, resource, namespace=None, subresource=None) -> bool:
    if dev_mode_enabled() or settings().DISABLE_AUTH:
        return True
    if user is None:
        raise exceptions.Unauthorized(description="No user credentials were found!")
    ra = {"group": group, "namespace": namespace, "verb": verb, "resource": resource, "version": version,
          "subresource": subresource}
    sar = client().create_subject_access_review({"user": user, "resourceAttributes": ra})
    st = sar.get("status")
    if st is None:
        log.error("SubjectAccessReview doesn't have status.")
        return False
    return bool(st.get("allowed"))


def generate_unauthorized_message(user, verb, group, version, resource, subresource=None, namespace=None):
    msg = "User '%s' is not authorized to %s" % (user, verb)
    msg += " %s/%s" % (version, resource) if group == "" else " %s/%s/%s" % (group, version, resource)
    if subresource is not None:
        msg += "/%s" % subresource
    if namespace is not None:
        msg += " in namespace '%s'" % namespace
    return msg


def ensure_authorized(verb, group, version, resource, namespace=None, subresource=None):
    user = get_username()
    if not is_authorized(user, verb, group, version, resource, namespace=namespace, subresource=subresource):
        raise exceptions.Forbidden(description=generate_unauthorized_message(
            user, verb, group, version, resource, subresource=subresource, namespace=namespace))


def needs_authorization(verb, group, version, resource, namespace=None, subresource=None):
    def wrapper(func):
        @functools.wraps(func)
        def runner(*a, **kw):
            ensure_authorized(verb, group, version, resource, namespace=namespace, subresource=subresource)
            return func(*a, **kw)
        return runner
    return wrapper


# ------------------------------------------------------------------ csrf
csrf_bp = Blueprint("csrf", __name__)


def set_cookie(resp: Response):
    s = settings()
    samesite = s.CSRF_SAMESITE if s.CSRF_SAMESITE in SAMESITE_VALUES else "Strict"
    resp.set_cookie(key=CSRF_COOKIE, value=secrets.token_urlsafe(32), samesite=samesite, httponly=False,
                    secure=s.SECURE_COOKIES, path=current_app.config["PREFIX"])
    resp.headers["Cache-Control"] = NO_CACHE


@csrf_bp.before_app_request
def check_endpoint():
    if request.method in ("GET", "HEAD", "OPTIONS", "TRACE"):
        return
    if CSRF_COOKIE not in request.cookies:
        raise exceptions.Forbidden("Could not find CSRF cookie %s in the request." % CSRF_COOKIE)
    if CSRF_HEADER not in request.headers:
        raise exceptions.Forbidden("Could not detect CSRF protection header %s." % CSRF_HEADER)
    if request.headers[CSRF_HEADER] != request.cookies[CSRF_COOKIE]:
        raise exceptions.Forbidden("CSRF check failed. Token in cookie %s doesn't match token in header %s."
                                   % (CSRF_COOKIE, CSRF_HEADER))


# ------------------------------------------------------------------ responses / errors
def success_response(data_field=None, data=None):
    resp = {"status": 200, "success": True, "user": get_username()}
    if data_field is None and data is None:
        return jsonify(resp)
    resp[data_field] = data
    return jsonify(resp)


def failed_response(msg, error_code):
    return {"success": False, "log": msg, "status": error_code, "user": get_username()}, error_code


def events_field_selector(kind, name):
    return "involvedObject.kind=%s,involvedObject.name=%s" % (kind, name)


errors_bp = Blueprint("errors", __name__)


@errors_bp.app_errorhandler(ApiError)
def api_exception_handler(e: ApiError):
    log.error("An error occured talking to k8s while working on %s: %s", request.url, e)
    msg = "The requested resource could not be found in the API Server" if e.code == 404 else (e.message or str(e))
    return failed_response(msg, e.code)


@errors_bp.app_errorhandler(exceptions.HTTPException)
def handle_http_errors(e):
    return failed_response(e.description, e.code)


@errors_bp.app_errorhandler(Exception)
def catch_all(e):
    log.exception(e)
    return failed_response("An error occured in the backend.", 500)


# ------------------------------------------------------------------ decorators / status
def request_is_json_type(func):
    @functools.wraps(func)
    def wrapper(*a, **kw):
        if request.content_type != "application/json":
            raise exceptions.BadRequest("Request is not in JSON format.")
        return func(*a, **kw)
    return wrapper


def required_body_params(*params):
    def wrapper(func):
        @functools.wraps(func)
        def runner(*a, **kw):
            body = request.get_json()
            for p in params:
                if p not in body:
                    raise exceptions.BadRequest("Parameter '%s' is missing from the request's body." % p)
            return func(*a, **kw)
        return runner
    return wrapper


class STATUS_PHASE:
    READY = "ready"
    WAITING = "waiting"
    WARNING = "warning"
    ERROR = "error"
    UNINITIALIZED = "uninitialized"
    UNAVAILABLE = "unavailable"
    TERMINATING = "terminating"
    STOPPED = "stopped"


def create_status(phase="", message="", state="", key=None):
    return {"phase": phase, "message": message, "state": state}


# ------------------------------------------------------------------ helpers
def load_yaml(path):
    try:
        with open(path) as f:
            text = f.read()
    except IOError:
        log.error("Error opening: %s", path)
        return None
    try:
        c = yaml.safe_load(text)
        return {} if c is None else c
    except yaml.YAMLError:
        return None


def load_param_yaml(path, **kwargs):
    try:
        with open(path) as f:
            text = f.read().format(**kwargs)
    except IOError:
        log.error("Error opening: %s", path)
        return None
    try:
        c = yaml.safe_load(text)
        return {} if c is None else c
    except yaml.YAMLError:
        return None


def get_uptime(then, now: Optional[dt.datetime] = None) -> str:
    if isinstance(then, str):
        then = dt.datetime.strptime(then, "%Y-%m-%dT%H:%M:%SZ")
    diff = (now or dt.datetime.now()) - then.replace(tzinfo=None)
    days, hours, mins = diff.days, int(diff.seconds / 3600), int((diff.seconds % 3600) / 60)
    if days > 0:
        age = "1 day" if days == 1 else f"{days} days"
    elif hours > 0:
        age = "1 hour" if hours == 1 else f"{hours} hours"
    else:
        if mins == 0:
            return "just now"
        age = "1 min" if mins == 1 else f"{mins} mins"
    return age + " ago"


def get_prefixed_index_html() -> str:
    prefix = os.path.join("/", current_app.config["PREFIX"], "")
    with open(os.path.join(current_app.config["STATIC_DIR"], "index.html")) as f:
        return re.sub(r"\<base href=\".*\".*\>", '<base href="%s">' % prefix, f.read())


# ------------------------------------------------------------------ Kubernetes API helpers
class api:
    """The reference's ``crud_backend.api`` module: every call is SAR-checked first."""

    # notebooks (kubeflow.org/v1beta1)
    @staticmethod
    def get_notebook(name, ns):
        ensure_authorized("get", "kubeflow.org", "v1beta1", "notebooks", ns)
        return client().get("kubeflow.org/v1beta1", "Notebook", name, ns)

    @staticmethod
    def create_notebook(nb, ns, dry_run=False):
        ensure_authorized("create", "kubeflow.org", "v1beta1", "notebooks", ns)
        nb = dict(nb, apiVersion=nb.get("apiVersion", "kubeflow.org/v1beta1"), kind="Notebook")
        nb.setdefault("metadata", {})["namespace"] = ns
        return client().create(nb, dry_run=dry_run)

    @staticmethod
    def list_notebooks(ns):
        ensure_authorized("list", "kubeflow.org", "v1beta1", "notebooks", ns)
        return client().list("kubeflow.org/v1beta1", "Notebook", ns)

    @staticmethod
    def delete_notebook(name, ns):
        ensure_authorized("delete", "kubeflow.org", "v1beta1", "notebooks", ns)
        return client().delete("kubeflow.org/v1beta1", "Notebook", name, ns, propagation="Foreground")

    @staticmethod
    def patch_notebook(name, ns, body):
        ensure_authorized("patch", "kubeflow.org", "v1beta1", "notebooks", ns)
        return client().patch("kubeflow.org/v1beta1", "Notebook", name, ns, body)

    @staticmethod
    def list_notebook_events(name, ns):
        return api.list_events(ns, events_field_selector("Notebook", name))

    # core
    @staticmethod
    def list_events(ns, field_selector):
        ensure_authorized("list", "", "v1", "events", ns)
        return client().list("v1", "Event", ns, field_selector=field_selector)

    @staticmethod
    def create_pvc(pvc, ns, dry_run=False):
        ensure_authorized("create", "", "v1", "persistentvolumeclaims", ns)
        pvc = dict(pvc, apiVersion="v1", kind="PersistentVolumeClaim")
        pvc.setdefault("metadata", {})["namespace"] = ns
        return client().create(pvc, dry_run=dry_run)

    @staticmethod
    def delete_pvc(name, ns):
        ensure_authorized("delete", "", "v1", "persistentvolumeclaims", ns)
        return client().delete("v1", "PersistentVolumeClaim", name, ns)

    @staticmethod
    def list_pvcs(ns):
        ensure_authorized("list", "", "v1", "persistentvolumeclaims", ns)
        return client().list("v1", "PersistentVolumeClaim", ns)

    @staticmethod
    def get_pvc(name, ns):
        ensure_authorized("get", "", "v1", "persistentvolumeclaims", ns)
        return client().get("v1", "PersistentVolumeClaim", name, ns)

    @staticmethod
    def patch_pvc(name, ns, body, auth=True):
        if auth:
            ensure_authorized("patch", "", "v1", "persistentvolumeclaims", ns)
        return client().patch("v1", "PersistentVolumeClaim", name, ns, body)

    @staticmethod
    def list_pvc_events(ns, name):
        return api.list_events(ns, events_field_selector("PersistentVolumeClaim", name))

    @staticmethod
    def list_pods(ns, auth=True, label_selector=None):
        if auth:
            ensure_authorized("list", "", "v1", "pods", ns)
        return client().list("v1", "Pod", ns, label_selector=label_selector)

    @staticmethod
    def get_pod_logs(ns, pod, container, auth=True):
        if auth:
            ensure_authorized("get", "", "v1", "pods", ns, "log")
        reader = current_app.extensions.get("kfamd_pod_logs")
        if reader is None:
            raise exceptions.NotImplemented("pod log reader not configured")
        return reader(ns, pod, container)

    @staticmethod
    def get_secret(ns, name, auth=True):
        if auth:
            ensure_authorized("get", "", "v1", "secrets", ns)
        return client().get("v1", "Secret", name, ns)

    @staticmethod
    def create_secret(ns, secret, auth=True):
        if auth:
            ensure_authorized("create", "", "v1", "secrets", ns)
        secret = dict(secret, apiVersion="v1", kind="Secret")
        secret.setdefault("metadata", {})["namespace"] = ns
        return client().create(secret)

    @staticmethod
    def list_namespaces():
        ensure_authorized("list", "core", "v1", "namespaces")
        return client().list("v1", "Namespace")

    @staticmethod
    def list_nodes():
        return client().list("v1", "Node")

    @staticmethod
    def list_storageclasses():
        return client().list("storage.k8s.io/v1", "StorageClass")

    @staticmethod
    def list_poddefaults(ns):
        ensure_authorized("list", "kubeflow.org", "v1alpha1", "poddefaults", ns)
        return client().list("kubeflow.org/v1alpha1", "PodDefault", ns)

    # generic custom resources (group, version, plural)
    @staticmethod
    def create_custom_rsrc(group, version, plural, data, ns):
        ensure_authorized("create", group, version, plural, ns)
        av, kind = client_kind(group, version, plural)
        data = dict(data, apiVersion=av, kind=kind)
        data.setdefault("metadata", {})["namespace"] = ns
        return client().create(data)

    @staticmethod
    def delete_custom_rsrc(group, version, plural, name, ns, policy="Foreground"):
        ensure_authorized("delete", group, version, plural, ns)
        av, kind = client_kind(group, version, plural)
        return client().delete(av, kind, name, ns, propagation=policy)

    @staticmethod
    def list_custom_rsrc(group, version, plural, ns):
        ensure_authorized("list", group, version, plural, ns)
        av, kind = client_kind(group, version, plural)
        return client().list(av, kind, ns)

    @staticmethod
    def get_custom_rsrc(group, version, plural, ns, name):
        ensure_authorized("get", group, version, plural, ns)
        av, kind = client_kind(group, version, plural)
        return client().get(av, kind, name, ns)


def client_kind(group, version, plural):
    """(group, version, plural) -> (apiVersion, Kind) through the API server's type table."""
    from ..controlplane.apiserver import BUILTIN_TYPES
    for t in BUILTIN_TYPES:
        if t.group == group and t.plural == plural:
            return (f"{group}/{version}" if group else version), t.kind
    raise exceptions.NotFound(f"unknown resource {group}/{version}/{plural}")


# ------------------------------------------------------------------ probes / serving / base routes
probes_bp = Blueprint("probes", __name__)


@probes_bp.route("/healthz/liveness")
@no_authentication
def liveness():
    return jsonify("alive"), 200


@probes_bp.route("/healthz/readiness")
@no_authentication
def readiness():
    return jsonify("ready"), 200


serving_bp = Blueprint("serving", __name__)


@serving_bp.route("/index.html")
@serving_bp.route("/")
@serving_bp.route("/<path:path>")
def serve_index(path="/"):
    resp = Response(get_prefixed_index_html(), mimetype="text/html", headers={"Cache-Control": NO_CACHE})
    set_cookie(resp)
    return resp


base_bp = Blueprint("base_routes", __name__)


@base_bp.route("/info")
def get_info():
    return success_response("info", {})


@base_bp.route("/api/namespaces")
def get_namespaces():
    return success_response("namespaces", [n["metadata"]["name"] for n in api.list_namespaces()])


@base_bp.route("/api/storageclasses")
def get_storageclasses():
    return success_response("storageClasses", [s["metadata"]["name"] for s in api.list_storageclasses()])


@base_bp.route("/api/storageclasses/default")
def get_default_storageclass():
    for sc in api.list_storageclasses():
        ann = sc["metadata"].get("annotations") or {}
        for key in ("storageclass.kubernetes.io/is-default-class", "storageclass.beta.kubernetes.io/is-default-class"):
            if ann.get(key, "false") == "true":
                return success_response("defaultStorageClass", sc["metadata"]["name"])
    return success_response("defaultStorageClass", "")


def create_app(name: str, static_folder: str, config: Config, kube: Client, settings_env=None,
               pod_log_reader=None) -> Flask:
    """Reference ``crud_backend.create_app``: authn, errors, csrf, probes, serving, base routes.

    The SPA catch-all ``/<path:path>`` never shadows ``/api/...``: werkzeug ranks rules
    without converters first."""
    logging.basicConfig(format=LOG_FORMAT, level=config.LOG_LEVEL)
    app = Flask(name, static_folder=static_folder)
    app.config.from_object(config)
    app.config["ENV"] = config.ENV
    app.config["STATIC_DIR"] = getattr(config, "STATIC_DIR", static_folder)
    app.extensions["kfamd_client"] = kube
    app.extensions["kfamd_settings"] = Settings(settings_env)
    if pod_log_reader is not None:
        app.extensions["kfamd_pod_logs"] = pod_log_reader
    for bp in (authn_bp, errors_bp, csrf_bp, probes_bp, serving_bp, base_bp):
        app.register_blueprint(bp)
    return app
