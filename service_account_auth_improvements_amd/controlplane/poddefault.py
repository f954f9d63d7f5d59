"""G4 / G4a: PodDefault mutating admission webhook (``kubeflow.org/v1alpha1`` PodDefault).

Behavioural reference: components/admission-webhook/main.go:72-773 and
pkg/apis/settings/v1alpha1/poddefault_types.go:27-125.

On pod CREATE in a profile namespace: list the namespace's PodDefaults, keep those whose
``spec.selector`` matches the pod labels, refuse (deny with a conflict message) if any
field would be merged with a *different* value under the same key, otherwise merge
volumes, tolerations, imagePullSecrets, annotations, labels, env, envFrom, volumeMounts
(by name AND by mount path), initContainers, sidecars, serviceAccountName,
automountServiceAccountToken and command/args (only when unset; never on istio-proxy),
stamp ``poddefault.admission.kubeflow.org/poddefault-<name>: <resourceVersion>`` and answer
with an RFC 6902 JSONPatch.  Pods annotated ``.../exclude: "true"`` and mirror pods are
skipped.  On MI355X clusters a PodDefault is the natural way to inject e.g. shared RCCL /
HSA environment or a dataset PVC into every notebook of a team.

Served in-process (APIServer admission chain) or over HTTPS on :4443 at
``/apply-poddefault`` with certificates re-read when they change on disk (cert-manager
rotation, the certwatcher equivalent).
"""
from __future__ import annotations

import base64
import copy
import json
import os
import ssl
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import List, Optional, Tuple

from .apiserver import Webhook, create_json_patch, labels_match
from .client import Client

ANNOTATION_PREFIX = "poddefault.admission.kubeflow.org"
ISTIO_PROXY = "istio-proxy"
MIRROR_POD_ANNOTATION = "kubernetes.io/config.mirror"
PD_API = "kubeflow.org/v1alpha1"


class MergeConflict(Exception):
    pass


def filter_pod_defaults(pds: List[dict], pod: dict) -> List[dict]:
    out = []
    for pd in pds:
        if pd["metadata"].get("namespace") != pod["metadata"].get("namespace"):
            continue
        sel = pd.get("spec", {}).get("selector") or {}
        if labels_match(pod["metadata"].get("labels"), sel):
            out.append(pd)
    return out


def _merge_keyed(orig: List[dict], pds: List[dict], field: str, key: str, what: str, errs: list) -> List[dict]:
    seen = {x.get(key): x for x in orig or []}
    merged = list(copy.deepcopy(orig or []))
    for pd in pds:
        for v in pd.get("spec", {}).get(field) or []:
            found = seen.get(v.get(key))
            if found is None:
                seen[v.get(key)] = v
                merged.append(copy.deepcopy(v))
            elif found != v:
                errs.append(f"merging {what} for {pd['metadata']['name']} has a conflict on {v.get(key)}")
    return merged


def merge_volume_mounts(mounts: List[dict], pds: List[dict], errs: list) -> List[dict]:
    by_name = {m["name"]: m for m in mounts or []}
    by_path = {m.get("mountPath"): m for m in mounts or []}
    merged = list(copy.deepcopy(mounts or []))
    for pd in pds:
        for v in pd.get("spec", {}).get("volumeMounts") or []:
            f = by_name.get(v["name"])
            if f is None:
                by_name[v["name"]] = v
                merged.append(copy.deepcopy(v))
            elif f != v:
                errs.append(f"merging volume mounts for {pd['metadata']['name']} has a conflict on {v['name']}")
            f = by_path.get(v.get("mountPath"))
            if f is None:
                by_path[v.get("mountPath")] = v
            elif f != v:
                errs.append(f"merging volume mounts for {pd['metadata']['name']} has a conflict on mount path "
                            f"{v.get('mountPath')}")
    return merged


def merge_map(existing: Optional[dict], defaults: List[Optional[dict]], errs: list) -> dict:
    out = dict(existing or {})
    for d in defaults:
        for k, v in (d or {}).items():
            if k not in out:
                out[k] = v
            elif out[k] != v:
                errs.append(f"merging has conflict on {k}: {v!r} does not match {out[k]!r} in pod")
    return out


def safe_to_apply(pod: dict, pds: List[dict]) -> List[str]:
    errs: List[str] = []
    spec = pod.get("spec", {})
    _merge_keyed(spec.get("volumes"), pds, "volumes", "name", "volumes", errs)
    _merge_keyed(spec.get("tolerations"), pds, "tolerations", "key", "tolerations", errs)
    _merge_keyed(spec.get("imagePullSecrets"), pds, "imagePullSecrets", "name", "imagePullSecret", errs)
    for ctr in spec.get("containers") or []:
        _merge_keyed(ctr.get("env"), pds, "env", "name", "env", errs)
        merge_volume_mounts(ctr.get("volumeMounts"), pds, errs)
    merge_map(pod["metadata"].get("annotations"), [pd.get("spec", {}).get("annotations") for pd in pds], errs)
    merge_map(pod["metadata"].get("labels"), [pd.get("spec", {}).get("labels") for pd in pds], errs)
    _merge_keyed(spec.get("initContainers"), pds, "initContainers", "name", "containers", errs)
    _merge_keyed(spec.get("containers"), pds, "sidecars", "name", "containers", errs)
    return errs


def set_command_and_args(ctr: dict, pds: List[dict]):
    if ctr.get("name") == ISTIO_PROXY:
        return
    for pd in pds:
        s = pd.get("spec", {})
        if ctr.get("command") is None and s.get("command") is not None:
            ctr["command"] = copy.deepcopy(s["command"])
        if ctr.get("args") is None and s.get("args") is not None:
            ctr["args"] = copy.deepcopy(s["args"])


def apply_pod_defaults_on_pod(pod: dict, pds: List[dict]) -> dict:
    if not pds:
        return pod
    errs: List[str] = []
    spec = pod.setdefault("spec", {})
    meta = pod.setdefault("metadata", {})

    def set_or_drop(key, val):
        if val:
            spec[key] = val
        else:
            spec.pop(key, None)

    set_or_drop("volumes", _merge_keyed(spec.get("volumes"), pds, "volumes", "name", "volumes", errs))
    set_or_drop("tolerations", _merge_keyed(spec.get("tolerations"), pds, "tolerations", "key", "tolerations", errs))
    ips = _merge_keyed(spec.get("imagePullSecrets"), pds, "imagePullSecrets", "name", "imagePullSecret", errs)
    set_or_drop("imagePullSecrets", ips)
    for pd in pds:
        s = pd.get("spec", {})
        if s.get("automountServiceAccountToken") is not None:
            spec["automountServiceAccountToken"] = s["automountServiceAccountToken"]
        if s.get("serviceAccountName"):
            spec["serviceAccountName"] = s["serviceAccountName"]
    meta["annotations"] = merge_map(meta.get("annotations"), [pd.get("spec", {}).get("annotations") for pd in pds], errs)
    meta["labels"] = merge_map(meta.get("labels"), [pd.get("spec", {}).get("labels") for pd in pds], errs)
    for ctr in spec.get("containers") or []:
        env = _merge_keyed(ctr.get("env"), pds, "env", "name", "env", errs)
        if env:
            ctr["env"] = env
        vm = merge_volume_mounts(ctr.get("volumeMounts"), pds, errs)
        if vm:
            ctr["volumeMounts"] = vm
        ef = list(ctr.get("envFrom") or [])
        for pd in pds:
            ef.extend(copy.deepcopy(pd.get("spec", {}).get("envFrom") or []))
        if ef:
            ctr["envFrom"] = ef
        set_command_and_args(ctr, pds)
    set_or_drop("initContainers", _merge_keyed(spec.get("initContainers"), pds, "initContainers", "name",
                                               "containers", errs))
    spec["containers"] = _merge_keyed(spec.get("containers"), pds, "sidecars", "name", "containers", errs)
    for pd in pds:
        meta["annotations"][f"{ANNOTATION_PREFIX}/poddefault-{pd['metadata']['name']}"] = \
            pd["metadata"].get("resourceVersion", "")
    return pod


def mutate_pods(request: dict, client: Client) -> dict:
    """AdmissionReview.request -> AdmissionReview.response."""
    res = request.get("resource") or {}
    if (res.get("group"), res.get("version"), res.get("resource")) != ("", "v1", "pods"):
        return {"uid": request.get("uid"), "allowed": True}
    pod = copy.deepcopy(request["object"])
    if not pod.get("metadata", {}).get("namespace"):
        pod.setdefault("metadata", {})["namespace"] = request.get("namespace")
    resp = {"uid": request.get("uid"), "allowed": True}
    ann = pod["metadata"].get("annotations") or {}
    if ann.get(f"{ANNOTATION_PREFIX}/exclude") == "true" or MIRROR_POD_ANNOTATION in ann:
        return resp
    try:
        pds = client.list(PD_API, "PodDefault", pod["metadata"]["namespace"])
    except Exception as e:
        return {"uid": request.get("uid"), "allowed": False, "status": {"message": str(e)}}
    matching = filter_pod_defaults(pds, pod)
    if not matching:
        return resp
    errs = safe_to_apply(pod, matching)
    if errs:
        names = ",".join(pd["metadata"]["name"] for pd in matching)
        return {"uid": request.get("uid"), "allowed": False,
                "status": {"code": 403, "reason": "Forbidden",
                           "message": f"conflict occurred while applying poddefaults: {names} on pod: "
                                      f"{pod['metadata'].get('name', '')} err: {'; '.join(errs)}"}}
    orig = copy.deepcopy(pod)
    mutated = apply_pod_defaults_on_pod(pod, matching)
    patch = create_json_patch(orig, mutated)
    resp["patchType"] = "JSONPatch"
    resp["patch"] = base64.b64encode(json.dumps(patch).encode()).decode()
    return resp


def register(server, client: Client):
    """Install as a MutatingWebhook on pod CREATE in profile namespaces, failurePolicy Fail
    (admission-webhook/manifests/base/mutating-webhook-configuration.yaml)."""
    server.add_mutating_webhook(Webhook(
        name="admission-webhook-deployment.kubeflow.org", group="", kind="Pod", operations=("CREATE",),
        fn=lambda req: mutate_pods(req, client),
        namespace_selector={"matchLabels": {"app.kubernetes.io/part-of": "kubeflow-profile"}},
        failure_policy="Fail"))


class ReloadingTLS:
    """TLS context whose cert/key are re-read whenever the files change (certwatcher)."""

    def __init__(self, cert_file: str, key_file: str):
        self.cert, self.key = cert_file, key_file
        self._mt = None
        self._ctx = None
        self._lock = threading.Lock()

    def context(self) -> ssl.SSLContext:
        mt = (os.stat(self.cert).st_mtime, os.stat(self.key).st_mtime)
        with self._lock:
            if mt != self._mt:
                ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
                ctx.load_cert_chain(self.cert, self.key)
                self._ctx, self._mt = ctx, mt
            return self._ctx


def serve_admission(handlers: dict, port: int = 4443, host: str = "0.0.0.0", tls: Optional[ReloadingTLS] = None):
    """HTTP(S) AdmissionReview server. handlers: path -> fn(request) -> response."""
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_POST(self):
            fn = handlers.get(self.path.split("?")[0])
            if fn is None:
                self.send_response(404)
                self.end_headers()
                return
            if self.headers.get("Content-Type") != "application/json":
                self.send_response(415)
                self.end_headers()
                return
            n = int(self.headers.get("Content-Length") or 0)
            try:
                ar = json.loads(self.rfile.read(n).decode())
                resp = fn(ar["request"])
            except Exception as e:
                ar, resp = {"request": {}}, {"allowed": False, "status": {"message": str(e)}}
            resp["uid"] = ar.get("request", {}).get("uid")
            body = json.dumps({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                               "response": resp}).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

    httpd = ThreadingHTTPServer((host, port), H)
    if tls is not None:
        orig = httpd.get_request

        def get_request():
            sock, addr = orig()
            return tls.context().wrap_socket(sock, server_side=True), addr
        httpd.get_request = get_request
    threading.Thread(target=httpd.serve_forever, daemon=True).start()
    return httpd
