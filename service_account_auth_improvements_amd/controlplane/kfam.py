"""G3 / G3a: KFAM -- the access-management REST service (:8081).

Behavioural reference: components/access-management/kfam/routers.go:32-106,
api_default.go:36-310, bindings.go:38-238, profiles.go:24-95, monitoring.go, logger.go,
api/swagger.yaml:17-160.

Routes: ``GET /kfam/``, ``POST|GET|DELETE /kfam/v1/bindings``, ``POST /kfam/v1/profiles``,
``DELETE /kfam/v1/profiles/<profile>``, ``GET /kfam/v1/role/clusteradmin?user=``,
``GET /metrics``.  A binding = a RoleBinding + an Istio AuthorizationPolicy, both named
``<kind>-<user>-<rolekind>-<role>`` (non-alphanumerics -> ``-``, lower-cased), annotated
``user`` / ``role``; role names map kubeflow-{admin,edit,view} <-> {admin,edit,view}.
Mutations require the caller (user-id header minus prefix) to own the profile or be the
cluster admin (403; a forbidden profile delete answers 401, as the reference does).
Bindings are listed from a RoleBinding cache refreshed at most every ``resync_s``
(the informer with 60 min resync) and invalidated on writes.
"""
from __future__ import annotations

import json
import logging
import re
import threading
import time
import urllib.parse
from typing import Dict, List, Optional

from .apiserver import ApiError
from .client import Client
from .monitoring import SEVERITY_MAJOR, RequestMetrics
from .runtime import get_env_default

log = logging.getLogger("kfam")
USER, ROLE = "user", "role"
ROLE_MAP = {"kubeflow-admin": "admin", "kubeflow-edit": "edit", "kubeflow-view": "view",
            "admin": "kubeflow-admin", "edit": "kubeflow-edit", "view": "kubeflow-view"}
PROFILE_API = "kubeflow.org/v1beta1"


def binding_name(b: dict) -> str:
    reg = re.compile(r"[^a-zA-Z0-9]+")
    raw = "-".join([b["user"]["kind"], urllib.parse.quote_plus(reg.sub("-", b["user"]["name"])),
                    b["roleRef"]["kind"], b["roleRef"]["name"]]).lower()
    return reg.sub("-", raw)


def binding_authorization_policy(b: dict, header: str, prefix: str) -> dict:
    igw = get_env_default("ISTIO_INGRESS_GATEWAY_PRINCIPAL",
                          "cluster.local/ns/istio-system/sa/istio-ingressgateway-service-account")
    kfp = get_env_default("KFP_UI_PRINCIPAL", "cluster.local/ns/kubeflow/sa/ml-pipeline-ui")
    return {"rules": [{"when": [{"key": f"request.headers[{header}]", "values": [prefix + b["user"]["name"]]}],
                       "from": [{"source": {"principals": [igw, kfp]}}]}]}


class BindingClient:
    def __init__(self, client: Client, resync_s: float = 3600.0):
        self.c = client
        self.resync_s = resync_s
        self._cache: Dict[str, List[dict]] = {}
        self._stamp: Dict[str, float] = {}
        self._lock = threading.Lock()

    def _rolebindings(self, ns: str) -> List[dict]:
        with self._lock:
            if ns not in self._cache or time.time() - self._stamp.get(ns, 0) > self.resync_s:
                self._cache[ns] = self.c.list("rbac.authorization.k8s.io/v1", "RoleBinding", ns)
                self._stamp[ns] = time.time()
            return self._cache[ns]

    def _invalidate(self, ns: str):
        with self._lock:
            self._cache.pop(ns, None)

    def create(self, b: dict, header: str, prefix: str):
        name = binding_name(b)
        ns = b["referredNamespace"]
        rr = b["roleRef"]
        self.c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                       "metadata": {"name": name, "namespace": ns,
                                    "annotations": {USER: b["user"]["name"], ROLE: rr["name"]}},
                       "roleRef": {"apiGroup": rr.get("apiGroup", "rbac.authorization.k8s.io"),
                                   "kind": rr["kind"], "name": ROLE_MAP.get(rr["name"], rr["name"])},
                       "subjects": [b["user"]]})
        self._invalidate(ns)
        self.c.create({"apiVersion": "security.istio.io/v1beta1", "kind": "AuthorizationPolicy",
                       "metadata": {"name": name, "namespace": ns,
                                    "annotations": {USER: b["user"]["name"], ROLE: rr["name"]}},
                       "spec": binding_authorization_policy(b, header, prefix)})

    def delete(self, b: dict):
        name = binding_name(b)
        ns = b["referredNamespace"]
        self.c.get("rbac.authorization.k8s.io/v1", "RoleBinding", name, ns)
        self.c.get("security.istio.io/v1beta1", "AuthorizationPolicy", name, ns)
        self.c.delete("rbac.authorization.k8s.io/v1", "RoleBinding", name, ns)
        self._invalidate(ns)
        self.c.delete("security.istio.io/v1beta1", "AuthorizationPolicy", name, ns)

    def list(self, user: str, namespaces: List[str], role: str) -> dict:
        out = []
        for ns in namespaces:
            for rb in self._rolebindings(ns):
                ann = rb["metadata"].get("annotations") or {}
                if USER not in ann or (user and user != ann[USER]):
                    continue
                if ROLE not in ann or (role and role != ann[ROLE]):
                    continue
                subs = rb.get("subjects") or []
                if len(subs) != 1:
                    raise ValueError(f"binding subject length not equal to 1, actual length: {len(subs)}")
                out.append({"user": {"kind": subs[0]["kind"], "name": subs[0]["name"]}, "referredNamespace": ns,
                            "roleRef": {"kind": rb["roleRef"]["kind"],
                                        "name": ROLE_MAP.get(rb["roleRef"]["name"], rb["roleRef"]["name"])}})
        return {"bindings": out}


class Kfam:
    def __init__(self, client: Client, user_id_header: str = "x-goog-authenticated-user-email",
                 user_id_prefix: str = "accounts.google.com:", cluster_admin: str = "", registry=None):
        self.c = client
        self.header, self.prefix = user_id_header, user_id_prefix
        self.cluster_admin = [cluster_admin] if cluster_admin else []
        self.bindings = BindingClient(client)
        self.metrics = RequestMetrics("kfam", registry, extra_labels=("user", "action", "path"))

    def user_email(self, headers) -> str:
        v = headers.get(self.header) or ""
        return v[len(self.prefix):]

    def is_cluster_admin(self, user: str) -> bool:
        return user in self.cluster_admin

    def is_owner_or_admin(self, user: str, profile: str) -> bool:
        try:
            prof = self.c.get(PROFILE_API, "Profile", profile)
        except ApiError:
            return False
        return self.is_cluster_admin(user) or prof["spec"]["owner"]["name"] == user

    # --------------------------------------------------------------- WSGI app
    def app(self):
        from flask import Flask, Response, request
        app = Flask("kfam")
        m = self.metrics

        def resp(code, body=b""):
            return Response(body, status=code, content_type="application/json; charset=UTF-8")

        @app.before_request
        def _t0():
            request._kfam_t0 = time.time()

        @app.after_request
        def _log(r):
            log.info("%s %s %s", request.method, request.full_path, time.time() - getattr(request, "_kfam_t0", time.time()))
            return r

        @app.get("/kfam/")
        def index():
            return resp(200, b"Hello World!")

        @app.post("/kfam/v1/bindings")
        def create_binding():
            try:
                b = json.loads(request.data)
            except ValueError as e:
                m.inc_error("decode request error", SEVERITY_MAJOR, "", "create", request.path)
                return resp(403, str(e).encode())
            user = self.user_email(request.headers)
            if not self.is_owner_or_admin(user, b.get("referredNamespace", "")):
                m.inc_request("forbidden", user, "create", request.path)
                return resp(403)
            try:
                self.bindings.create(b, self.header, self.prefix)
            except (ApiError, KeyError) as e:
                m.inc_error(str(e), SEVERITY_MAJOR, user, "create", request.path)
                return resp(403, str(e).encode())
            m.inc_request("", user, "create", request.path)
            return resp(200)

        @app.delete("/kfam/v1/bindings")
        def delete_binding():
            try:
                b = json.loads(request.data)
            except ValueError as e:
                return resp(403, str(e).encode())
            user = self.user_email(request.headers)
            if not self.is_owner_or_admin(user, b.get("referredNamespace", "")):
                m.inc_request("forbidden", user, "delete", request.path)
                return resp(403)
            try:
                self.bindings.delete(b)
            except (ApiError, KeyError) as e:
                m.inc_error(str(e), SEVERITY_MAJOR, user, "delete", request.path)
                return resp(403, str(e).encode())
            m.inc_request("", user, "delete", request.path)
            return resp(200)

        @app.get("/kfam/v1/bindings")
        def read_binding():
            q = request.args
            if q.get("namespace"):
                namespaces = [q["namespace"]]
            else:
                namespaces = [p["metadata"]["name"] for p in self.c.list(PROFILE_API, "Profile")]
            try:
                out = self.bindings.list(q.get("user", ""), namespaces, q.get("role", ""))
            except (ApiError, ValueError) as e:
                m.inc_error(str(e), SEVERITY_MAJOR, "", "read", request.path)
                return resp(401, str(e).encode())
            m.inc_request("", "", "read", request.path)
            return resp(200, json.dumps(out).encode())

        @app.post("/kfam/v1/profiles")
        def create_profile():
            try:
                prof = json.loads(request.data)
                prof.setdefault("apiVersion", PROFILE_API)
                prof.setdefault("kind", "Profile")
                self.c.create(prof)
            except (ValueError, ApiError) as e:
                m.inc_error(str(e), SEVERITY_MAJOR, "", "create", request.path)
                return resp(403, str(e).encode())
            m.inc_request("", "", "create", request.path)
            return resp(200)

        @app.delete("/kfam/v1/profiles/<profile>")
        def delete_profile(profile):
            user = self.user_email(request.headers)
            if not self.is_owner_or_admin(user, profile):
                m.inc_request("forbidden", user, "delete", request.path)
                return resp(401)
            try:
                self.c.delete(PROFILE_API, "Profile", profile)
            except ApiError as e:
                m.inc_error(str(e), SEVERITY_MAJOR, user, "delete", request.path)
                return resp(401, str(e).encode())
            m.inc_request("", user, "delete", request.path)
            return resp(200)

        @app.get("/kfam/v1/role/clusteradmin")
        def cluster_admin():
            m.inc_request("", "", "read", request.path)
            return resp(200, ("true" if self.is_cluster_admin(request.args.get("user", "")) else "false").encode())

        @app.get("/metrics")
        def metrics():
            from prometheus_client import CONTENT_TYPE_LATEST, generate_latest
            return Response(generate_latest(self.metrics.registry), content_type=CONTENT_TYPE_LATEST)

        return app
