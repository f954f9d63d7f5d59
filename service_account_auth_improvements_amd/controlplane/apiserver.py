"""In-memory Kubernetes-compatible API server (the envtest / KinD replacement).

SURVEY.md §7.3 step 1: the reference tests its controllers against envtest (a real
kube-apiserver + etcd without kubelet) and KinD clusters; neither exists here, so the
control plane of this repo is built and tested against this server.  It implements the
API semantics the controllers, webhooks and web apps depend on:

* typed registry of group/version/kind/plural/scope (core, apps, rbac, coordination,
  authorization, Istio, kubeflow.org CRDs incl. the new PyTorchJob/MPIJob, KServe);
  objects are plain JSON dicts (like ``unstructured.Unstructured``); CRD versions are
  converted trivially (conversion strategy ``None``, as the reference's Notebook CRD);
* create / get / list (label + field selectors) / update (optimistic concurrency on
  ``metadata.resourceVersion``) / merge- and JSON-patch / delete, ``dryRun``,
  ``generateName``, ``generation`` bumps on spec changes;
* ``status`` subresource semantics (main-resource updates ignore status, status updates
  ignore everything else);
* finalizers + ``deletionTimestamp``; ownerReference garbage collection with
  Background / Foreground / Orphan propagation (the JWA deletes notebooks in foreground);
  namespace deletion cascades;
* watches (ADDED / MODIFIED / DELETED) delivered synchronously to subscribers, with
  kube-apiserver resourceVersion semantics: every event carries a cluster-wide increasing
  RV (a deletion gets an RV of its own), lists report the RV they were taken at, a watch
  started from an RV first replays the retained event history after it (a bounded ring,
  like the watch cache) and is refused with 410 Gone/Expired when that history no longer
  reaches back far enough -- the client then re-lists;
* admission chain: mutating then validating webhooks (in-process callables receiving
  an AdmissionReview-shaped request), e.g. the PodDefault mutator and the PVCViewer
  defaulter/validator;
* SubjectAccessReview evaluated against Roles/ClusterRoles/(Cluster)RoleBindings.
"""
from __future__ import annotations

import copy
import datetime as _dt
import fnmatch
import json
import threading
import uuid
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple


# ----------------------------------------------------------------------------- errors
class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str = ""):
        super().__init__(f"{code} {reason}: {message}")
        self.code, self.reason, self.message = code, reason, message

    def status(self) -> dict:
        return {"kind": "Status", "apiVersion": "v1", "status": "Failure", "code": self.code,
                "reason": self.reason, "message": self.message}


def NotFound(msg=""):
    return ApiError(404, "NotFound", msg)


def AlreadyExists(msg=""):
    return ApiError(409, "AlreadyExists", msg)


def Conflict(msg=""):
    return ApiError(409, "Conflict", msg)


def Invalid(msg=""):
    return ApiError(422, "Invalid", msg)


def Gone(msg=""):
    """410: the requested resourceVersion is older than the retained watch history."""
    return ApiError(410, "Expired", msg)


def Forbidden(msg=""):
    return ApiError(403, "Forbidden", msg)


def is_not_found(e) -> bool:
    return isinstance(e, ApiError) and e.code == 404


# ----------------------------------------------------------------------------- types
@dataclass(frozen=True)
class ResourceType:
    group: str
    kind: str
    plural: str
    namespaced: bool
    versions: Tuple[str, ...]
    status_subresource: bool = True

    @property
    def storage_version(self):
        return self.versions[-1]

    def api_version(self, version: Optional[str] = None) -> str:
        v = version or self.storage_version
        return f"{self.group}/{v}" if self.group else v


BUILTIN_TYPES = [
    ResourceType("", "Namespace", "namespaces", False, ("v1",)),
    ResourceType("", "Pod", "pods", True, ("v1",)),
    ResourceType("", "Service", "services", True, ("v1",)),
    ResourceType("", "Event", "events", True, ("v1",), False),
    ResourceType("", "PersistentVolumeClaim", "persistentvolumeclaims", True, ("v1",)),
    ResourceType("", "ConfigMap", "configmaps", True, ("v1",), False),
    ResourceType("", "Secret", "secrets", True, ("v1",), False),
    ResourceType("", "ServiceAccount", "serviceaccounts", True, ("v1",), False),
    ResourceType("", "Node", "nodes", False, ("v1",)),
    ResourceType("", "ResourceQuota", "resourcequotas", True, ("v1",)),
    ResourceType("storage.k8s.io", "StorageClass", "storageclasses", False, ("v1",), False),
    ResourceType("apps", "StatefulSet", "statefulsets", True, ("v1",)),
    ResourceType("apps", "Deployment", "deployments", True, ("v1",)),
    ResourceType("rbac.authorization.k8s.io", "Role", "roles", True, ("v1",), False),
    ResourceType("rbac.authorization.k8s.io", "ClusterRole", "clusterroles", False, ("v1",), False),
    ResourceType("rbac.authorization.k8s.io", "RoleBinding", "rolebindings", True, ("v1",), False),
    ResourceType("rbac.authorization.k8s.io", "ClusterRoleBinding", "clusterrolebindings", False,
                 ("v1",), False),
    ResourceType("coordination.k8s.io", "Lease", "leases", True, ("v1",), False),
    ResourceType("authorization.k8s.io", "SubjectAccessReview", "subjectaccessreviews", False, ("v1",)),
    ResourceType("networking.istio.io", "VirtualService", "virtualservices", True, ("v1alpha3", "v1beta1")),
    ResourceType("security.istio.io", "AuthorizationPolicy", "authorizationpolicies", True, ("v1beta1",)),
    ResourceType("app.k8s.io", "Application", "applications", True, ("v1beta1",)),
    ResourceType("apiextensions.k8s.io", "CustomResourceDefinition", "customresourcedefinitions", False, ("v1",)),
    ResourceType("admissionregistration.k8s.io", "MutatingWebhookConfiguration",
                 "mutatingwebhookconfigurations", False, ("v1",), False),
    ResourceType("admissionregistration.k8s.io", "ValidatingWebhookConfiguration",
                 "validatingwebhookconfigurations", False, ("v1",), False),
    # kubeflow CRDs (reference)
    ResourceType("kubeflow.org", "Notebook", "notebooks", True, ("v1alpha1", "v1beta1", "v1")),
    ResourceType("kubeflow.org", "Profile", "profiles", False, ("v1beta1", "v1")),
    ResourceType("kubeflow.org", "PodDefault", "poddefaults", True, ("v1alpha1",), False),
    ResourceType("kubeflow.org", "PVCViewer", "pvcviewers", True, ("v1alpha1",)),
    ResourceType("tensorboard.kubeflow.org", "Tensorboard", "tensorboards", True, ("v1alpha1",)),
    # north-star data-plane CRDs
    ResourceType("kubeflow.org", "PyTorchJob", "pytorchjobs", True, ("v1",)),
    ResourceType("kubeflow.org", "MPIJob", "mpijobs", True, ("v2beta1",)),
    ResourceType("serving.kserve.io", "InferenceService", "inferenceservices", True, ("v1beta1",)),
]


def _check_schema(v, sch: dict, path: str, errs: List[str]):
    """Structural openAPI subset used by CRD validation: type, required, properties,
    additionalProperties (maps), items, enum, minimum, minLength, minItems, maxItems, pattern,
    x-kubernetes-int-or-string and x-kubernetes-preserve-unknown-fields (an object that declares
    properties AND preserves unknown fields validates the declared ones and keeps the rest)."""
    if not sch or sch.get("x-kubernetes-preserve-unknown-fields") and "properties" not in sch:
        return
    if sch.get("x-kubernetes-int-or-string"):
        if not isinstance(v, (int, str)) or isinstance(v, bool):
            errs.append(f"{path or '.'}: must be an integer or a string")
        return
    typ = sch.get("type")
    ok = {"object": lambda x: isinstance(x, dict), "array": lambda x: isinstance(x, list),
          "string": lambda x: isinstance(x, str), "boolean": lambda x: isinstance(x, bool),
          "integer": lambda x: isinstance(x, int) and not isinstance(x, bool),
          "number": lambda x: isinstance(x, (int, float)) and not isinstance(x, bool)}.get(typ)
    if ok is not None and not ok(v):
        errs.append(f"{path or '.'}: must be of type {typ}")
        return
    if "enum" in sch and v not in sch["enum"]:
        errs.append(f"{path}: unsupported value {v!r}, supported: {sch['enum']}")
    if "minimum" in sch and isinstance(v, (int, float)) and v < sch["minimum"]:
        errs.append(f"{path}: must be >= {sch['minimum']}")
    if "minLength" in sch and isinstance(v, str) and len(v) < sch["minLength"]:
        errs.append(f"{path}: must be at least {sch['minLength']} characters")
    if "minItems" in sch and isinstance(v, list) and len(v) < sch["minItems"]:
        errs.append(f"{path}: must have at least {sch['minItems']} items")
    if "maxItems" in sch and isinstance(v, list) and len(v) > sch["maxItems"]:
        errs.append(f"{path}: must have at most {sch['maxItems']} items")
    if "pattern" in sch and isinstance(v, str):
        import re
        if not re.search(sch["pattern"], v):
            errs.append(f"{path}: must match {sch['pattern']!r}")
    if typ == "object" and isinstance(v, dict):
        for r in sch.get("required") or []:
            if r not in v:
                errs.append(f"{path}.{r}: Required value")
        props = sch.get("properties") or {}
        for k, sub in props.items():
            if k in v and v[k] is not None:
                _check_schema(v[k], sub, f"{path}.{k}", errs)
        extra = sch.get("additionalProperties")
        if isinstance(extra, dict):        # map types (resources.limits, nodeSelector, ...)
            for k, x in v.items():
                if k not in props:
                    _check_schema(x, extra, f"{path}.{k}", errs)
    if typ == "array" and isinstance(v, list) and sch.get("items"):
        for i, x in enumerate(v):
            _check_schema(x, sch["items"], f"{path}[{i}]", errs)


def _prune_unknown(v, sch: dict, path: str, found: List[str]):
    """Structural-schema pruning (apiextensions.k8s.io/v1): drop, in place, every object field
    the schema does not declare, and record its path.  Objects that preserve unknown fields,
    maps (``additionalProperties``) and schema-less objects (``type: object`` alone) keep
    everything."""
    if not isinstance(sch, dict) or sch.get("x-kubernetes-preserve-unknown-fields"):
        return
    if isinstance(v, dict):
        props = sch.get("properties")
        extra = sch.get("additionalProperties")
        if props is None and not isinstance(extra, dict):
            return
        for k in list(v):
            if props is not None and k in props:
                _prune_unknown(v[k], props[k], f"{path}.{k}", found)
            elif isinstance(extra, dict):
                _prune_unknown(v[k], extra, f"{path}.{k}", found)
            else:
                found.append(f"{path}.{k}")
                del v[k]
    elif isinstance(v, list) and isinstance(sch.get("items"), dict):
        for i, x in enumerate(v):
            _prune_unknown(x, sch["items"], f"{path}[{i}]", found)


def split_api_version(api_version: str) -> Tuple[str, str]:
    if "/" in api_version:
        g, v = api_version.split("/", 1)
        return g, v
    return "", api_version


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


# ----------------------------------------------------------------------------- selectors
def parse_label_selector(sel) -> List[Tuple[str, str, List[str]]]:
    """Parse "a=b,c!=d,e in (x,y),!f,g" or a LabelSelector dict into requirements."""
    reqs = []
    if sel is None or sel == "":
        return reqs
    if isinstance(sel, dict):
        for k, v in (sel.get("matchLabels") or {}).items():
            reqs.append((k, "=", [v]))
        for e in sel.get("matchExpressions") or []:
            op = {"In": "in", "NotIn": "notin", "Exists": "exists", "DoesNotExist": "!"}[e["operator"]]
            reqs.append((e["key"], op, list(e.get("values") or [])))
        return reqs
    parts, depth, cur = [], 0, ""
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        parts.append(cur)
    for p in parts:
        p = p.strip()
        if " notin " in p:
            k, v = p.split(" notin ", 1)
            reqs.append((k.strip(), "notin", [x.strip() for x in v.strip()[1:-1].split(",")]))
        elif " in " in p:
            k, v = p.split(" in ", 1)
            reqs.append((k.strip(), "in", [x.strip() for x in v.strip()[1:-1].split(",")]))
        elif "!=" in p:
            k, v = p.split("!=", 1)
            reqs.append((k.strip(), "!=", [v.strip()]))
        elif "==" in p:
            k, v = p.split("==", 1)
            reqs.append((k.strip(), "=", [v.strip()]))
        elif "=" in p:
            k, v = p.split("=", 1)
            reqs.append((k.strip(), "=", [v.strip()]))
        elif p.startswith("!"):
            reqs.append((p[1:].strip(), "!", []))
        else:
            reqs.append((p, "exists", []))
    return reqs


def labels_match(labels: Optional[dict], sel) -> bool:
    labels = labels or {}
    for k, op, vals in parse_label_selector(sel):
        if op == "=" and labels.get(k) != vals[0]:
            return False
        if op == "!=" and labels.get(k) == vals[0]:
            return False
        if op == "in" and labels.get(k) not in vals:
            return False
        if op == "notin" and labels.get(k) in vals:
            return False
        if op == "exists" and k not in labels:
            return False
        if op == "!" and k in labels:
            return False
    return True


def _get_path(obj, path: str):
    cur = obj
    for p in path.split("."):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(p)
    return cur


def fields_match(obj: dict, sel: Optional[str]) -> bool:
    if not sel:
        return True
    for part in sel.split(","):
        neg = "!=" in part
        k, v = part.split("!=" if neg else "=", 1)
        k = k.strip().lstrip("=")
        v = v.strip().lstrip("=")
        got = _get_path(obj, k)
        got = "" if got is None else str(got)
        if (got == v) == neg:
            return False
    return True


# ----------------------------------------------------------------------------- patches
def merge_patch(target, patch):
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def _ptr(path: str) -> List[str]:
    if path == "":
        return []
    return [p.replace("~1", "/").replace("~0", "~") for p in path.lstrip("/").split("/")]


def json_patch(doc, ops: List[dict]):
    """RFC 6902 JSON patch (add/remove/replace/move/copy/test)."""
    doc = copy.deepcopy(doc)

    def parent(d, parts):
        cur = d
        for p in parts[:-1]:
            cur = cur[int(p)] if isinstance(cur, list) else cur[p]
        return cur, parts[-1]

    for op in ops:
        o = op["op"]
        parts = _ptr(op["path"])
        if o == "test":
            cur = doc
            for p in parts:
                cur = cur[int(p)] if isinstance(cur, list) else cur[p]
            if cur != op["value"]:
                raise Invalid(f"test failed at {op['path']}")
            continue
        if o in ("move", "copy"):
            src = _ptr(op["from"])
            sp, sk = parent(doc, src)
            val = sp[int(sk)] if isinstance(sp, list) else sp[sk]
            if o == "move":
                if isinstance(sp, list):
                    sp.pop(int(sk))
                else:
                    del sp[sk]
            ops_val = copy.deepcopy(val)
            o, op = "add", {"op": "add", "path": op["path"], "value": ops_val}
            parts = _ptr(op["path"])
        if not parts:
            doc = copy.deepcopy(op["value"]) if o != "remove" else None
            continue
        par, key = parent(doc, parts)
        if isinstance(par, list):
            if o == "add":
                idx = len(par) if key == "-" else int(key)
                par.insert(idx, copy.deepcopy(op["value"]))
            elif o == "remove":
                par.pop(int(key))
            elif o == "replace":
                par[int(key)] = copy.deepcopy(op["value"])
        else:
            if o in ("add", "replace"):
                if o == "replace" and key not in par:
                    raise Invalid(f"replace of missing path {op['path']}")
                par[key] = copy.deepcopy(op["value"])
            elif o == "remove":
                if key not in par:
                    raise Invalid(f"remove of missing path {op['path']}")
                del par[key]
    return doc


def create_json_patch(src, dst, path: str = "") -> List[dict]:
    """Minimal RFC 6902 diff (used by admission webhooks to answer with a JSONPatch)."""
    ops = []
    esc = lambda k: str(k).replace("~", "~0").replace("/", "~1")  # noqa: E731
    if isinstance(src, dict) and isinstance(dst, dict):
        for k in src:
            if k not in dst:
                ops.append({"op": "remove", "path": f"{path}/{esc(k)}"})
        for k, v in dst.items():
            if k not in src:
                ops.append({"op": "add", "path": f"{path}/{esc(k)}", "value": copy.deepcopy(v)})
            else:
                ops.extend(create_json_patch(src[k], v, f"{path}/{esc(k)}"))
        return ops
    if isinstance(src, list) and isinstance(dst, list) and len(src) == len(dst):
        for i, (a, b) in enumerate(zip(src, dst)):
            ops.extend(create_json_patch(a, b, f"{path}/{i}"))
        return ops
    if src != dst:
        ops.append({"op": "replace", "path": path or "", "value": copy.deepcopy(dst)})
    return ops


# ----------------------------------------------------------------------------- server
WatchFn = Callable[[str, dict], None]


@dataclass
class Webhook:
    name: str
    group: str
    kind: str
    operations: Tuple[str, ...]
    fn: Callable[[dict], dict]      # AdmissionReview.request -> AdmissionReview.response
    namespace_selector: Optional[dict] = None
    object_selector: Optional[dict] = None
    failure_policy: str = "Fail"


class _RVCounter:
    """Cluster-wide resourceVersion sequence (``next()`` issues, ``value`` = last issued)."""

    def __init__(self):
        self.value = 0

    def __iter__(self):
        return self

    def __next__(self) -> int:
        self.value += 1
        return self.value


class APIServer:
    """Thread-safe in-memory API server. All returned objects are deep copies."""

    HISTORY = 4096        # retained watch events (kube-apiserver's watch cache window)

    def __init__(self, types: Optional[List[ResourceType]] = None, history: Optional[int] = None):
        self._lock = threading.RLock()
        # unknown CRD fields when a request does not say (kube-apiserver's default): pruned
        # ("Warn"/"Ignore"); "Strict" rejects them
        self.field_validation = "Warn"
        self._types: Dict[Tuple[str, str], ResourceType] = {}
        self._by_plural: Dict[Tuple[str, str], ResourceType] = {}
        for t in (types or BUILTIN_TYPES):
            self.register_type(t)
        self._store: Dict[Tuple[str, str], Dict[Tuple[str, str], dict]] = {}
        self._rv = _RVCounter()
        self._watchers: List[Tuple[Optional[str], Optional[str], WatchFn]] = []
        # event history for resourceVersion-based watches: (rv, type, group, kind, obj)
        self._history_max = history or self.HISTORY
        self._history: List[Tuple[int, str, str, str, dict]] = []
        self._history_head = 0          # index of the oldest retained event
        self._history_floor = 0         # rv of the newest DROPPED event
        self._schemas: Dict[Tuple[str, str], Dict[str, Optional[dict]]] = {}
        self.mutating: List[Webhook] = []
        self.validating: List[Webhook] = []
        self.clock = lambda: now_rfc3339()

    # --- registry
    def register_type(self, t: ResourceType):
        self._types[(t.group, t.kind)] = t
        self._by_plural[(t.group, t.plural)] = t

    def _register_crd(self, crd: dict):
        """A CustomResourceDefinition makes its kind servable and its per-version
        openAPIV3Schema enforced on create/update (structural subset: type, required,
        properties, items, enum, minimum, minLength, preserve-unknown-fields)."""
        sp = crd.get("spec") or {}
        names = sp.get("names") or {}
        vers = [v for v in sp.get("versions") or [] if v.get("served", True)]
        if not (sp.get("group") and names.get("kind") and names.get("plural") and vers):
            raise Invalid("CustomResourceDefinition needs spec.group, spec.names.{kind,plural}, spec.versions")
        storage = [v["name"] for v in vers if v.get("storage")]
        order = [v["name"] for v in vers if v["name"] not in storage] + storage   # storage version last
        self.register_type(ResourceType(sp["group"], names["kind"], names["plural"],
                                        sp.get("scope", "Namespaced") == "Namespaced", tuple(order),
                                        "status" in ((vers[0].get("subresources") or {}))))
        self._schemas[(sp["group"], names["kind"])] = {
            v["name"]: (v.get("schema") or {}).get("openAPIV3Schema") for v in vers}

    def _validate_schema(self, t: ResourceType, obj: dict, field_validation: Optional[str] = None):
        """CRD schema validation.  Fields the structural schema does not declare are pruned
        (as kube-apiserver does); with ``fieldValidation=Strict`` (kubectl's default) they are an
        error instead, so a misspelt field is reported rather than dropped."""
        schemas = self._schemas.get((t.group, t.kind))
        if not schemas:
            return
        _, ver = split_api_version(obj.get("apiVersion", ""))
        sch = schemas.get(ver) or schemas.get(t.storage_version)
        if not sch:
            return
        errs: List[str] = []
        unknown: List[str] = []
        for k in list(obj):
            if k in ("metadata", "apiVersion", "kind"):
                continue
            if k not in (sch.get("properties") or {}):
                if not sch.get("x-kubernetes-preserve-unknown-fields"):
                    unknown.append(f".{k}")
                    del obj[k]
                continue
            _prune_unknown(obj[k], sch["properties"][k], f".{k}", unknown)
        if unknown and (field_validation or self.field_validation) == "Strict":
            raise Invalid(f'{t.kind}.{t.group} "{obj.get("metadata", {}).get("name")}" is invalid: strict decoding '
                          "error: " + ", ".join(f'unknown field "{u[1:]}"' for u in unknown))
        body = {k: v for k, v in obj.items() if k not in ("metadata", "apiVersion", "kind")}
        _check_schema(body, {k: v for k, v in sch.items() if k != "properties"} | {
            "type": "object", "properties": {k: v for k, v in (sch.get("properties") or {}).items()
                                             if k not in ("metadata", "apiVersion", "kind")}}, "", errs)
        if errs:
            raise Invalid(f'{t.kind}.{t.group} "{obj.get("metadata", {}).get("name")}" is invalid: ' + "; ".join(errs))

    def type_for(self, api_version: str, kind: str) -> ResourceType:
        g, _ = split_api_version(api_version)
        t = self._types.get((g, kind))
        if t is None:
            raise NotFound(f"no kind {kind} in {api_version}")
        return t

    def type_for_plural(self, group: str, plural: str) -> ResourceType:
        t = self._by_plural.get((group, plural))
        if t is None:
            raise NotFound(f"the server could not find the requested resource {group}/{plural}")
        return t

    def types(self) -> List[ResourceType]:
        return list(self._types.values())

    # --- helpers
    def _bucket(self, t: ResourceType):
        return self._store.setdefault((t.group, t.kind), {})

    @staticmethod
    def _key(t: ResourceType, ns: Optional[str], name: str):
        return (ns if t.namespaced else "", name)

    @property
    def resource_version(self) -> str:
        """The latest issued resourceVersion (what a list taken now reports)."""
        return str(self._rv.value)

    def _record(self, etype: str, t: ResourceType, obj: dict):
        h = self._history
        h.append((int(obj["metadata"]["resourceVersion"]), etype, t.group, t.kind, obj))
        if len(h) - self._history_head > self._history_max:
            self._history_floor = h[self._history_head][0]
            self._history_head += 1
            if self._history_head > self._history_max:      # compact the ring occasionally
                del h[:self._history_head]
                self._history_head = 0

    def _emit(self, etype: str, t: ResourceType, obj: dict):
        if etype == "DELETED":      # a deletion is a write of its own: fresh resourceVersion
            obj = copy.deepcopy(obj)
            obj["metadata"]["resourceVersion"] = str(next(self._rv))
        obj = copy.deepcopy(obj)
        obj["apiVersion"] = t.api_version()
        self._record(etype, t, obj)
        for g, k, fn in list(self._watchers):
            if (g is None or g == t.group) and (k is None or k == t.kind):
                try:
                    fn(etype, copy.deepcopy(obj))
                except Exception:  # a broken watcher must not break the write path
                    import logging
                    logging.getLogger("apiserver").exception("watch handler failed")

    def watch(self, fn: WatchFn, api_version: Optional[str] = None, kind: Optional[str] = None,
              resource_version: Optional[str] = None):
        """Subscribe to events; returns an unsubscribe callable.

        ``resource_version`` (an RV from a list or an earlier event): the retained events
        newer than it are delivered first, then live events -- atomically, so none is
        missed or repeated.  Raises 410 Gone when events after it were already dropped.
        None / "" / "0" start from now."""
        g = split_api_version(api_version)[0] if api_version else None
        entry = (g, kind, fn)
        with self._lock:
            if resource_version not in (None, "", "0"):
                rv = int(resource_version)
                if rv < self._history_floor:
                    raise Gone(f"too old resource version: {rv} ({self._history_floor})")
                for erv, et, eg, ek, o in self._history[self._history_head:]:
                    if erv > rv and (g is None or g == eg) and (kind is None or kind == ek):
                        fn(et, copy.deepcopy(o))
            self._watchers.append(entry)

        def cancel():
            with self._lock:
                if entry in self._watchers:
                    self._watchers.remove(entry)
        return cancel

    # --- admission
    def add_mutating_webhook(self, wh: Webhook):
        self.mutating.append(wh)

    def add_validating_webhook(self, wh: Webhook):
        self.validating.append(wh)

    def _admit(self, op: str, t: ResourceType, obj: dict, old: Optional[dict], dry_run: bool,
               user: str = "system:admin") -> dict:
        ns = obj.get("metadata", {}).get("namespace")
        for chain, mutating in ((self.mutating, True), (self.validating, False)):
            for wh in chain:
                if wh.group != t.group or wh.kind != t.kind or op not in wh.operations:
                    continue
                if wh.namespace_selector and t.namespaced:
                    nsobj = self._bucket(self._types[("", "Namespace")]).get(("", ns))
                    labels = (nsobj or {}).get("metadata", {}).get("labels", {})
                    if not labels_match(labels, wh.namespace_selector):
                        continue
                if wh.object_selector and not labels_match(obj.get("metadata", {}).get("labels"),
                                                           wh.object_selector):
                    continue
                req = {"uid": str(uuid.uuid4()), "kind": {"group": t.group, "version": t.storage_version,
                                                          "kind": t.kind},
                       "resource": {"group": t.group, "version": t.storage_version, "resource": t.plural},
                       "namespace": ns, "name": obj.get("metadata", {}).get("name"), "operation": op,
                       "userInfo": {"username": user}, "object": copy.deepcopy(obj),
                       "oldObject": copy.deepcopy(old), "dryRun": dry_run}
                try:
                    resp = wh.fn(req)
                except Exception as e:  # webhook unreachable / crashed
                    if wh.failure_policy == "Fail":
                        raise ApiError(500, "InternalError",
                                       f'failed calling webhook "{wh.name}": {e}')
                    continue
                if not resp.get("allowed", False):
                    st = resp.get("status") or {}
                    raise ApiError(int(st.get("code", 403)), st.get("reason", "Forbidden"),
                                   f'admission webhook "{wh.name}" denied the request: '
                                   f'{st.get("message", "")}')
                if mutating and resp.get("patch"):
                    patch = resp["patch"]
                    if isinstance(patch, (bytes, str)):
                        import base64
                        try:
                            patch = json.loads(base64.b64decode(patch))
                        except Exception:
                            patch = json.loads(patch)
                    obj = json_patch(obj, patch)
        return obj

    # --- CRUD
    def create(self, obj: dict, dry_run: bool = False, user: str = "system:admin",
               field_validation: Optional[str] = None) -> dict:
        obj = copy.deepcopy(obj)
        t = self.type_for(obj.get("apiVersion", ""), obj.get("kind", ""))
        meta = obj.setdefault("metadata", {})
        if t.kind == "SubjectAccessReview":   # virtual: evaluated, never stored
            obj["status"] = self.evaluate_sar(obj.get("spec", {}))
            return obj
        with self._lock:
            if not meta.get("name"):
                gen = meta.get("generateName")
                if not gen:
                    raise Invalid("metadata.name or generateName required")
                meta["name"] = gen + uuid.uuid4().hex[:5]
            ns = meta.get("namespace") if t.namespaced else None
            if t.namespaced:
                if not ns:
                    raise Invalid(f"{t.kind} requires a namespace")
                nsobj = self._bucket(self._types[("", "Namespace")]).get(("", ns))
                if nsobj is None:
                    raise NotFound(f'namespaces "{ns}" not found')
                if nsobj["metadata"].get("deletionTimestamp"):
                    raise Forbidden(f"namespace {ns} is being terminated")
            else:
                meta.pop("namespace", None)
            bucket = self._bucket(t)
            key = self._key(t, ns, meta["name"])
            if key in bucket:
                raise AlreadyExists(f'{t.plural} "{meta["name"]}" already exists')
            obj = self._admit("CREATE", t, obj, None, dry_run, user)
            self._validate_schema(t, obj, field_validation)
            if t.kind == "CustomResourceDefinition" and not dry_run:
                self._register_crd(obj)
            meta = obj["metadata"]
            meta["uid"] = str(uuid.uuid4())
            meta["creationTimestamp"] = self.clock()
            meta["generation"] = 1
            meta["resourceVersion"] = str(next(self._rv))
            obj["apiVersion"] = t.api_version()
            if dry_run:
                return copy.deepcopy(obj)
            bucket[key] = obj
            self._emit("ADDED", t, obj)
            return copy.deepcopy(obj)

    def get(self, api_version: str, kind: str, name: str, namespace: Optional[str] = None) -> dict:
        t = self.type_for(api_version, kind)
        with self._lock:
            o = self._bucket(t).get(self._key(t, namespace, name))
            if o is None:
                raise NotFound(f'{t.plural}.{t.group or "core"} "{name}" not found')
            out = copy.deepcopy(o)
        out["apiVersion"] = api_version if "/" in api_version or not t.group else t.api_version()
        return out

    def list_with_rv(self, api_version: str, kind: str, namespace: Optional[str] = None,
                     label_selector=None, field_selector: Optional[str] = None) -> Tuple[List[dict], str]:
        """A list and the resourceVersion it is consistent with (watch from it to follow)."""
        with self._lock:
            return self.list(api_version, kind, namespace, label_selector, field_selector), self.resource_version

    def list(self, api_version: str, kind: str, namespace: Optional[str] = None,
             label_selector=None, field_selector: Optional[str] = None) -> List[dict]:
        t = self.type_for(api_version, kind)
        with self._lock:
            items = [copy.deepcopy(o) for (ns, _), o in sorted(self._bucket(t).items())
                     if (namespace is None or not t.namespaced or ns == namespace)
                     and labels_match(o.get("metadata", {}).get("labels"), label_selector)
                     and fields_match(o, field_selector)]
        for o in items:
            o["apiVersion"] = api_version if "/" in api_version or not t.group else t.api_version()
        return items

    def _write(self, t, cur, new, status_only: bool, dry_run: bool, user: str,
               field_validation: Optional[str] = None):
        meta, cmeta = new.setdefault("metadata", {}), cur["metadata"]
        rv = meta.get("resourceVersion")
        if rv and rv != cmeta["resourceVersion"]:
            raise Conflict(f'Operation cannot be fulfilled on {t.plural} "{cmeta["name"]}": the object '
                           "has been modified; please apply your changes to the latest version and try again")
        if status_only:
            out = copy.deepcopy(cur)
            out["status"] = copy.deepcopy(new.get("status"))
        else:
            out = copy.deepcopy(new)
            for k in ("uid", "creationTimestamp", "namespace", "name", "generation"):
                if k in cmeta:
                    out["metadata"][k] = cmeta[k]
                else:
                    out["metadata"].pop(k, None)
            if cmeta.get("deletionTimestamp"):
                out["metadata"]["deletionTimestamp"] = cmeta["deletionTimestamp"]
            if t.status_subresource:
                if "status" in cur:
                    out["status"] = copy.deepcopy(cur["status"])
                else:
                    out.pop("status", None)
            out = self._admit("UPDATE", t, out, cur, dry_run, user)
            self._validate_schema(t, out, field_validation)
            if t.kind == "CustomResourceDefinition" and not dry_run:
                self._register_crd(out)
            strip = lambda o: {k: v for k, v in o.items() if k not in ("metadata", "status", "apiVersion")}  # noqa
            if strip(out) != strip(cur):
                out["metadata"]["generation"] = cmeta.get("generation", 1) + 1
        out["apiVersion"] = t.api_version()
        if out == cur or (strip_rv(out) == strip_rv(cur)):
            return copy.deepcopy(cur)
        out["metadata"]["resourceVersion"] = str(next(self._rv))
        if dry_run:
            return copy.deepcopy(out)
        key = self._key(t, cmeta.get("namespace"), cmeta["name"])
        bucket = self._bucket(t)
        if out["metadata"].get("deletionTimestamp") and not out["metadata"].get("finalizers"):
            del bucket[key]
            self._emit("DELETED", t, out)
            self._gc_dependents(out, "Background")
            return copy.deepcopy(out)
        bucket[key] = out
        self._emit("MODIFIED", t, out)
        return copy.deepcopy(out)

    def update(self, obj: dict, dry_run: bool = False, user: str = "system:admin",
               field_validation: Optional[str] = None) -> dict:
        t = self.type_for(obj.get("apiVersion", ""), obj.get("kind", ""))
        meta = obj.get("metadata", {})
        with self._lock:
            cur = self._bucket(t).get(self._key(t, meta.get("namespace"), meta.get("name")))
            if cur is None:
                raise NotFound(f'{t.plural} "{meta.get("name")}" not found')
            return self._write(t, cur, copy.deepcopy(obj), False, dry_run, user, field_validation)

    def update_status(self, obj: dict) -> dict:
        t = self.type_for(obj.get("apiVersion", ""), obj.get("kind", ""))
        meta = obj.get("metadata", {})
        with self._lock:
            cur = self._bucket(t).get(self._key(t, meta.get("namespace"), meta.get("name")))
            if cur is None:
                raise NotFound(f'{t.plural} "{meta.get("name")}" not found')
            return self._write(t, cur, copy.deepcopy(obj), t.status_subresource, False, "system:admin")

    def bind_pod(self, namespace: str, name: str, node: str, user: str = "system:kube-scheduler") -> dict:
        """The ``pods/binding`` subresource (what kube-scheduler POSTs): sets ``spec.nodeName``
        of an unbound pod; binding a pod that is already bound (to any node) is a 409."""
        t = self.type_for("v1", "Pod")
        with self._lock:
            cur = self._bucket(t).get(self._key(t, namespace, name))
            if cur is None:
                raise NotFound(f'pods "{name}" not found')
            if cur["metadata"].get("deletionTimestamp"):
                raise Conflict(f'pod {name} is being deleted, cannot be assigned to a host')
            bound = (cur.get("spec") or {}).get("nodeName")
            if bound:
                raise Conflict(f'Operation cannot be fulfilled on pods/binding "{name}": pod {name} is already '
                               f'assigned to node "{bound}"')
            new = copy.deepcopy(cur)
            new["spec"]["nodeName"] = node
            self._write(t, cur, new, False, False, user)
        return {"kind": "Status", "apiVersion": "v1", "status": "Success", "code": 201}

    def patch(self, api_version: str, kind: str, name: str, namespace: Optional[str], patch,
              patch_type: str = "merge", subresource: Optional[str] = None, dry_run: bool = False,
              field_validation: Optional[str] = None,
              user: str = "system:admin") -> dict:
        t = self.type_for(api_version, kind)
        with self._lock:
            cur = self._bucket(t).get(self._key(t, namespace, name))
            if cur is None:
                raise NotFound(f'{t.plural} "{name}" not found')
            if patch_type == "json":
                new = json_patch(cur, patch)
            else:  # merge / strategic-merge treated as JSON merge patch
                new = merge_patch(cur, patch)
            new["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            return self._write(t, cur, new, subresource == "status" and t.status_subresource, dry_run, user,
                               field_validation)

    def delete(self, api_version: str, kind: str, name: str, namespace: Optional[str] = None,
               propagation: str = "Background", dry_run: bool = False) -> dict:
        t = self.type_for(api_version, kind)
        with self._lock:
            bucket = self._bucket(t)
            key = self._key(t, namespace, name)
            cur = bucket.get(key)
            if cur is None:
                raise NotFound(f'{t.plural} "{name}" not found')
            if dry_run:
                return copy.deepcopy(cur)
            meta = cur["metadata"]
            fins = list(meta.get("finalizers") or [])
            if propagation == "Foreground" and self._dependents(cur):
                if "foregroundDeletion" not in fins:
                    fins.append("foregroundDeletion")
            if fins:
                if not meta.get("deletionTimestamp"):
                    new = copy.deepcopy(cur)
                    new["metadata"]["deletionTimestamp"] = self.clock()
                    new["metadata"]["finalizers"] = fins
                    new["metadata"]["resourceVersion"] = str(next(self._rv))
                    bucket[key] = new
                    self._emit("MODIFIED", t, new)
                    if "foregroundDeletion" in fins:
                        self._gc_dependents(new, "Foreground")
                        self._maybe_finish_foreground(new)
                return copy.deepcopy(bucket.get(key, cur))
            del bucket[key]
            self._emit("DELETED", t, cur)
            if t.kind == "Namespace":
                self._delete_namespace_contents(meta["name"])
            self._gc_dependents(cur, propagation)
            return copy.deepcopy(cur)

    # --- garbage collection
    def _dependents(self, owner: dict) -> List[Tuple[ResourceType, dict]]:
        uid = owner["metadata"].get("uid")
        out = []
        for (g, k), bucket in self._store.items():
            t = self._types[(g, k)]
            for o in bucket.values():
                for ref in o.get("metadata", {}).get("ownerReferences") or []:
                    if ref.get("uid") == uid:
                        out.append((t, o))
        return out

    def _gc_dependents(self, owner: dict, propagation: str):
        for t, dep in self._dependents(owner):
            m = dep["metadata"]
            if propagation == "Orphan":
                new = copy.deepcopy(dep)
                new["metadata"]["ownerReferences"] = [r for r in m.get("ownerReferences", [])
                                                      if r.get("uid") != owner["metadata"]["uid"]]
                self._bucket(t)[self._key(t, m.get("namespace"), m["name"])] = new
                continue
            try:
                self.delete(t.api_version(), t.kind, m["name"], m.get("namespace"),
                            propagation="Foreground" if propagation == "Foreground" else "Background")
            except ApiError:
                pass

    def _maybe_finish_foreground(self, owner: dict):
        t = self.type_for(owner["apiVersion"], owner["kind"])
        m = owner["metadata"]
        cur = self._bucket(t).get(self._key(t, m.get("namespace"), m["name"]))
        if cur is None or "foregroundDeletion" not in (cur["metadata"].get("finalizers") or []):
            return
        if not self._dependents(cur):
            new = copy.deepcopy(cur)
            new["metadata"]["finalizers"] = [f for f in new["metadata"]["finalizers"] if f != "foregroundDeletion"]
            self._write(t, cur, new, False, False, "system:gc")

    def reconcile_foreground(self):
        """Finish foreground deletions whose dependents are gone (the GC controller loop)."""
        with self._lock:
            for (g, k), bucket in list(self._store.items()):
                for o in list(bucket.values()):
                    if "foregroundDeletion" in (o["metadata"].get("finalizers") or []):
                        self._maybe_finish_foreground(o)

    def _delete_namespace_contents(self, ns: str):
        for (g, k), bucket in list(self._store.items()):
            t = self._types[(g, k)]
            if not t.namespaced:
                continue
            for (ons, name), o in list(bucket.items()):
                if ons == ns:
                    o = copy.deepcopy(o)
                    o["metadata"]["finalizers"] = []
                    bucket.pop((ons, name), None)
                    self._emit("DELETED", t, o)

    # --- events
    def record_event(self, involved: dict, etype: str, reason: str, message: str,
                     source: str = "controller") -> dict:
        m = involved["metadata"]
        ns = m.get("namespace") or "default"
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"generateName": f'{m["name"]}.', "namespace": ns},
              "involvedObject": {"kind": involved.get("kind"), "name": m["name"], "namespace": m.get("namespace"),
                                 "uid": m.get("uid"), "apiVersion": involved.get("apiVersion")},
              "type": etype, "reason": reason, "message": message, "source": {"component": source},
              "firstTimestamp": self.clock(), "lastTimestamp": self.clock(), "count": 1}
        try:
            return self.create(ev)
        except ApiError:
            return ev

    # --- RBAC / SubjectAccessReview
    def evaluate_sar(self, spec: dict) -> dict:
        user = spec.get("user", "")
        groups = set(spec.get("groups") or [])
        ra = spec.get("resourceAttributes") or {}
        ns = ra.get("namespace")
        if user in ("system:admin",) or "system:masters" in groups:
            return {"allowed": True}

        def subj_match(s):
            k = s.get("kind")
            if k == "User":
                return s.get("name") == user
            if k == "Group":
                return s.get("name") in groups
            if k == "ServiceAccount":
                return user == f'system:serviceaccount:{s.get("namespace")}:{s.get("name")}'
            return False

        def rules_allow(rules):
            for r in rules or []:
                if not any(g in ("*", ra.get("group", "")) for g in r.get("apiGroups", [])):
                    continue
                res = ra.get("resource", "")
                if ra.get("subresource"):
                    res = f'{res}/{ra["subresource"]}'
                if not any(x == "*" or x == res for x in r.get("resources", [])):
                    continue
                if not any(v in ("*", ra.get("verb")) for v in r.get("verbs", [])):
                    continue
                names = r.get("resourceNames")
                if names and ra.get("name") not in names:
                    continue
                return True
            return False

        def role_rules(ref, bns):
            kind = ref.get("kind")
            try:
                if kind == "ClusterRole":
                    role = self.get("rbac.authorization.k8s.io/v1", "ClusterRole", ref["name"])
                    rules = list(role.get("rules") or [])
                    agg = role.get("aggregationRule")
                    if agg:
                        for sel in agg.get("clusterRoleSelectors", []):
                            for cr in self.list("rbac.authorization.k8s.io/v1", "ClusterRole", label_selector=sel):
                                rules.extend(cr.get("rules") or [])
                    return rules
                return self.get("rbac.authorization.k8s.io/v1", "Role", ref["name"], bns).get("rules")
            except ApiError:
                return []

        with self._lock:
            for crb in self.list("rbac.authorization.k8s.io/v1", "ClusterRoleBinding"):
                if any(subj_match(s) for s in crb.get("subjects") or []) and \
                        rules_allow(role_rules(crb["roleRef"], None)):
                    return {"allowed": True}
            if ns:
                for rb in self.list("rbac.authorization.k8s.io/v1", "RoleBinding", namespace=ns):
                    if any(subj_match(s) for s in rb.get("subjects") or []) and \
                            rules_allow(role_rules(rb["roleRef"], ns)):
                        return {"allowed": True}
        return {"allowed": False, "reason": "no RBAC rule allows this request"}

    # --- convenience
    def ensure_namespace(self, name: str, labels: Optional[dict] = None) -> dict:
        try:
            return self.get("v1", "Namespace", name)
        except ApiError:
            return self.create({"apiVersion": "v1", "kind": "Namespace",
                                "metadata": {"name": name, "labels": labels or {}}})


def strip_rv(o: dict) -> dict:
    o = copy.deepcopy(o)
    o.get("metadata", {}).pop("resourceVersion", None)
    return o


def owner_reference(owner: dict, controller: bool = True) -> dict:
    return {"apiVersion": owner["apiVersion"], "kind": owner["kind"], "name": owner["metadata"]["name"],
            "uid": owner["metadata"]["uid"], "controller": controller, "blockOwnerDeletion": True}


def set_controller_reference(owner: dict, obj: dict) -> dict:
    refs = [r for r in obj.setdefault("metadata", {}).get("ownerReferences", []) if not r.get("controller")]
    refs.append(owner_reference(owner))
    obj["metadata"]["ownerReferences"] = refs
    return obj


def glob_match(pattern: str, s: str) -> bool:
    return fnmatch.fnmatchcase(s, pattern)
