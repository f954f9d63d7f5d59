"""Kubernetes clients used by every controller, webhook and web backend.

Two interchangeable implementations of one small interface (the subset of
controller-runtime's ``client.Client`` + watches the reference uses):

* :class:`InMemoryClient` -- direct calls into :class:`.apiserver.APIServer` (tests, the
  single-process "local cluster", the fake kubelet);
* :class:`RestClient` -- the Kubernetes REST protocol over HTTP(S) (in-cluster
  service-account token + CA, or an explicit server URL).  The reference's Python
  backends use the ``kubernetes`` package, which is not installed here, so this client
  speaks the wire protocol itself; it is exercised in tests against the REST facade of
  the in-memory server (:mod:`.httpapi`).
"""
from __future__ import annotations

import json
import os
import ssl
import threading
import urllib.error
import urllib.parse
import urllib.request
from typing import Callable, List, Optional

from .apiserver import APIServer, ApiError, split_api_version


class Client:
    def get(self, api_version, kind, name, namespace=None) -> dict: ...
    def list(self, api_version, kind, namespace=None, label_selector=None, field_selector=None) -> List[dict]: ...
    def create(self, obj, dry_run=False) -> dict: ...
    def update(self, obj, dry_run=False) -> dict: ...
    def update_status(self, obj) -> dict: ...
    def patch(self, api_version, kind, name, namespace, patch, patch_type="merge", subresource=None) -> dict: ...
    def delete(self, api_version, kind, name, namespace=None, propagation="Background") -> dict: ...
    def watch(self, fn, api_version=None, kind=None, resource_version=None) -> Callable[[], None]: ...

    # helpers shared by all implementations
    def get_or_none(self, api_version, kind, name, namespace=None):
        try:
            return self.get(api_version, kind, name, namespace)
        except ApiError as e:
            if e.code == 404:
                return None
            raise

    def create_subject_access_review(self, spec: dict) -> dict:
        return self.create({"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
                            "spec": spec})

    def record_event(self, involved, etype, reason, message, source="controller"):
        m = involved["metadata"]
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"generateName": f'{m["name"]}.', "namespace": m.get("namespace") or "default"},
              "involvedObject": {"kind": involved.get("kind"), "name": m["name"],
                                 "namespace": m.get("namespace"), "uid": m.get("uid"),
                                 "apiVersion": involved.get("apiVersion")},
              "type": etype, "reason": reason, "message": message, "source": {"component": source}}
        try:
            return self.create(ev)
        except ApiError:
            return ev


class InMemoryClient(Client):
    def __init__(self, server: APIServer, user: str = "system:admin"):
        self.server, self.user = server, user

    def get(self, api_version, kind, name, namespace=None):
        return self.server.get(api_version, kind, name, namespace)

    def list(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        return self.server.list(api_version, kind, namespace, label_selector, field_selector)

    def create(self, obj, dry_run=False):
        return self.server.create(obj, dry_run=dry_run, user=self.user)

    def update(self, obj, dry_run=False):
        return self.server.update(obj, dry_run=dry_run, user=self.user)

    def update_status(self, obj):
        return self.server.update_status(obj)

    def patch(self, api_version, kind, name, namespace, patch, patch_type="merge", subresource=None):
        return self.server.patch(api_version, kind, name, namespace, patch, patch_type, subresource,
                                 user=self.user)

    def delete(self, api_version, kind, name, namespace=None, propagation="Background"):
        return self.server.delete(api_version, kind, name, namespace, propagation)

    def bind(self, namespace, name, node):
        return self.server.bind_pod(namespace, name, node)

    def list_with_rv(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        return self.server.list_with_rv(api_version, kind, namespace, label_selector, field_selector)

    def watch(self, fn, api_version=None, kind=None, resource_version=None):
        return self.server.watch(fn, api_version, kind, resource_version=resource_version)


class RestClient(Client):
    """Kubernetes REST client (JSON).  ``server`` like https://10.0.0.1:443."""

    SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

    def __init__(self, server: Optional[str] = None, token: Optional[str] = None,
                 ca_file: Optional[str] = None, insecure: bool = False, plural_map: Optional[dict] = None):
        if server is None:
            host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
            if not host:
                raise RuntimeError("no API server: pass server= or run in-cluster")
            server = f"https://{host}:{port or 443}"
            tok = os.path.join(self.SA_DIR, "token")
            if token is None and os.path.exists(tok):
                token = open(tok).read().strip()
            ca = os.path.join(self.SA_DIR, "ca.crt")
            if ca_file is None and os.path.exists(ca):
                ca_file = ca
        self.server = server.rstrip("/")
        self.token = token
        self.ctx = None
        if self.server.startswith("https"):
            self.ctx = ssl.create_default_context(cafile=ca_file)
            if insecure:
                self.ctx.check_hostname = False
                self.ctx.verify_mode = ssl.CERT_NONE
        # kind -> (plural, namespaced); discovered lazily from the server's type registry
        from .apiserver import BUILTIN_TYPES
        self.plurals = {(t.group, t.kind): (t.plural, t.namespaced) for t in BUILTIN_TYPES}
        if plural_map:
            self.plurals.update(plural_map)

    # --- URL building
    def _path(self, api_version, kind, namespace=None, name=None, subresource=None):
        g, v = split_api_version(api_version)
        plural, namespaced = self.plurals[(g, kind)]
        base = f"/api/{v}" if not g else f"/apis/{g}/{v}"
        if namespaced and namespace:
            base += f"/namespaces/{namespace}"
        base += f"/{plural}"
        if name:
            base += f"/{name}"
        if subresource:
            base += f"/{subresource}"
        return base

    def _req(self, method, path, body=None, params=None, content_type="application/json", stream=False):
        url = self.server + path
        if params:
            url += "?" + urllib.parse.urlencode({k: v for k, v in params.items() if v is not None})
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(url, data=data, method=method)
        req.add_header("Accept", "application/json")
        if data is not None:
            req.add_header("Content-Type", content_type)
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        try:
            resp = urllib.request.urlopen(req, context=self.ctx, timeout=None if stream else 30)
        except urllib.error.HTTPError as e:
            try:
                st = json.loads(e.read().decode())
            except Exception:
                st = {"reason": e.reason, "message": str(e)}
            raise ApiError(e.code, st.get("reason", ""), st.get("message", ""))
        if stream:
            return resp
        return json.loads(resp.read().decode() or "{}")

    def get(self, api_version, kind, name, namespace=None):
        return self._req("GET", self._path(api_version, kind, namespace, name))

    def list_with_rv(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        """Items plus the list's ``metadata.resourceVersion`` (the point to watch from)."""
        if isinstance(label_selector, dict):
            parts = [f"{k}={v}" for k, v in (label_selector.get("matchLabels") or {}).items()]
            label_selector = ",".join(parts)
        out = self._req("GET", self._path(api_version, kind, namespace),
                        params={"labelSelector": label_selector or None, "fieldSelector": field_selector})
        items = out.get("items", [])
        for it in items:
            it.setdefault("apiVersion", api_version)
            it.setdefault("kind", kind)
        return items, (out.get("metadata") or {}).get("resourceVersion")

    def list(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        return self.list_with_rv(api_version, kind, namespace, label_selector, field_selector)[0]

    def create(self, obj, dry_run=False):
        ns = obj.get("metadata", {}).get("namespace")
        return self._req("POST", self._path(obj["apiVersion"], obj["kind"], ns), obj,
                         params={"dryRun": "All" if dry_run else None})

    def update(self, obj, dry_run=False):
        m = obj["metadata"]
        return self._req("PUT", self._path(obj["apiVersion"], obj["kind"], m.get("namespace"), m["name"]), obj,
                         params={"dryRun": "All" if dry_run else None})

    def update_status(self, obj):
        m = obj["metadata"]
        return self._req("PUT", self._path(obj["apiVersion"], obj["kind"], m.get("namespace"), m["name"], "status"),
                         obj)

    def patch(self, api_version, kind, name, namespace, patch, patch_type="merge", subresource=None):
        ct = {"merge": "application/merge-patch+json", "json": "application/json-patch+json",
              "strategic": "application/strategic-merge-patch+json"}[patch_type]
        return self._req("PATCH", self._path(api_version, kind, namespace, name, subresource), patch,
                         content_type=ct)

    def delete(self, api_version, kind, name, namespace=None, propagation="Background"):
        return self._req("DELETE", self._path(api_version, kind, namespace, name),
                         {"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": propagation})

    def bind(self, namespace, name, node):
        """POST pods/{name}/binding (a Binding to node ``node``)."""
        body = {"apiVersion": "v1", "kind": "Binding", "metadata": {"name": name, "namespace": namespace},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        return self._req("POST", self._path("v1", "Pod", namespace, name, "binding"), body)

    WATCH_TIMEOUT = 300        # seconds per watch request before it is re-opened from the last RV

    def watch(self, fn, api_version=None, kind=None, resource_version=None):
        """List-then-watch with kube-apiserver resourceVersion semantics (client-go reflector):

        * before returning, the current state is LISTed (unless ``resource_version`` is given)
          and the stream is opened from that list's RV, so every change made after
          ``watch()`` returns is delivered -- also one that happens before the streaming
          connection is up (the server replays its event history from that RV);
        * a dropped connection or a ``timeoutSeconds`` end re-opens the watch from the last
          RV seen (events or BOOKMARKs);
        * a 410 Expired (the RV fell out of the server's history) triggers a RE-LIST, diffed
          against the objects this watch knows about, so the handler gets the ADDED /
          MODIFIED / DELETED events it missed instead of silently losing them.

        Runs in a daemon thread; returns a cancel callable."""
        stop = threading.Event()
        known: dict = {}          # (namespace, name) -> last object seen
        state = {"rv": resource_version}

        def key(o):
            m = o.get("metadata", {})
            return (m.get("namespace"), m.get("name"))

        def relist(deliver: bool):
            items, rv = self.list_with_rv(api_version, kind)
            seen = set()
            for o in items:
                k = key(o)
                seen.add(k)
                old = known.get(k)
                known[k] = o
                if deliver and (old is None or old["metadata"].get("resourceVersion") !=
                                o["metadata"].get("resourceVersion")):
                    fn("ADDED" if old is None else "MODIFIED", o)
            for k in [k for k in known if k not in seen]:
                o = known.pop(k)
                if deliver:
                    fn("DELETED", o)
            state["rv"] = rv

        if state["rv"] is None:
            relist(deliver=False)

        def run():
            while not stop.is_set():
                try:
                    resp = self._req("GET", self._path(api_version, kind),
                                     params={"watch": "true", "resourceVersion": state["rv"],
                                             "allowWatchBookmarks": "true",
                                             "timeoutSeconds": str(self.WATCH_TIMEOUT)}, stream=True)
                    expired = False
                    for line in resp:
                        if stop.is_set():
                            break
                        line = line.strip()
                        if not line:
                            continue
                        ev = json.loads(line)
                        et, obj = ev["type"], ev["object"]
                        if et == "ERROR":
                            expired = obj.get("code") == 410
                            break
                        rv = (obj.get("metadata") or {}).get("resourceVersion")
                        if rv:
                            state["rv"] = rv
                        if et == "BOOKMARK":
                            continue
                        if et == "DELETED":
                            known.pop(key(obj), None)
                        else:
                            known[key(obj)] = obj
                        fn(et, obj)
                    if expired and not stop.is_set():
                        relist(deliver=True)
                except Exception:
                    if stop.wait(1.0):
                        break
        th = threading.Thread(target=run, daemon=True)
        th.start()
        return stop.set
