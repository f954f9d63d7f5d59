"""G1/G1a/G1b: Notebook controller, idle-notebook culler and notebook metrics.

Behavioural reference (read, not translated):
  components/notebook-controller/controllers/notebook_controller.go:89-739
  components/notebook-controller/controllers/culling_controller.go:25-420
  components/notebook-controller/pkg/metrics/metrics.go:13-99
  components/notebook-controller/main.go:57-147

A Notebook CR gets a StatefulSet (replicas 1, or 0 while ``kubeflow-resource-stopped``
is set), a ClusterIP Service (80 -> container 8888), and with ``USE_ISTIO=true`` an Istio
VirtualService at ``/notebook/<ns>/<name>/``; Pod/StatefulSet Events are re-emitted on the
Notebook and pod conditions / container state are mirrored into ``.status``.
For MI355X notebooks the pod simply requests ``amd.com/gpu`` (set by the JWA form) --
the device plugin and ``HIP_VISIBLE_DEVICES`` are the kubelet's business.
"""
from __future__ import annotations

import copy
import datetime as dt
import json
import logging
import os
import urllib.request
from typing import Callable, List, Optional

from . import reconcilehelper
from .apiserver import ApiError, now_rfc3339, set_controller_reference
from .client import Client
from .runtime import Controller, Request, Result, for_kind, get_env_default, owns, watches

log = logging.getLogger("notebook-controller")

NB_API = "kubeflow.org/v1beta1"
DEFAULT_CONTAINER_PORT = 8888
DEFAULT_SERVING_PORT = 80
ANNOTATION_REWRITE_URI = "notebooks.kubeflow.org/http-rewrite-uri"
ANNOTATION_HEADERS_REQUEST_SET = "notebooks.kubeflow.org/http-headers-request-set"
PREFIX_ENV_VAR = "NB_PREFIX"
DEFAULT_FS_GROUP = 100
STOP_ANNOTATION = "kubeflow-resource-stopped"
LAST_ACTIVITY_ANNOTATION = "notebooks.kubeflow.org/last-activity"
LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION = "notebooks.kubeflow.org/last_activity_check_timestamp"


# ----------------------------------------------------------------------------- metrics (G1b)
class NotebookMetrics:
    """notebook_running (scraped from StatefulSets on collect), notebook_create_total,
    notebook_create_failed_total, notebook_culling_total, last_notebook_culling_timestamp_seconds."""

    def __init__(self, client: Client, registry=None):
        from prometheus_client import CollectorRegistry, Counter, Gauge
        from prometheus_client.core import GaugeMetricFamily
        self.client = client
        self.registry = registry or CollectorRegistry()
        self.create = Counter("notebook_create", "Total times of creating notebooks", ["namespace"],
                              registry=self.registry)
        self.create_failed = Counter("notebook_create_failed", "Total failure times of creating notebooks",
                                     ["namespace"], registry=self.registry)
        self.culling = Counter("notebook_culling", "Total times of culling notebooks", ["namespace", "name"],
                               registry=self.registry)
        self.culling_ts = Gauge("last_notebook_culling_timestamp_seconds",
                                "Timestamp of the last notebook culling in seconds", ["namespace", "name"],
                                registry=self.registry)
        outer = self

        class Running:
            def collect(self):
                g = GaugeMetricFamily("notebook_running", "Current running notebooks in the cluster",
                                      labels=["namespace"])
                for ns, n in sorted(outer.running().items()):
                    g.add_metric([ns], n)
                yield g

        self.registry.register(Running())

    def running(self) -> dict:
        out = {}
        try:
            for sts in self.client.list("apps/v1", "StatefulSet"):
                tl = sts.get("spec", {}).get("template", {}).get("metadata", {}).get("labels", {}) or {}
                if tl.get("notebook-name") == sts["metadata"]["name"]:
                    ns = sts["metadata"]["namespace"]
                    out[ns] = out.get(ns, 0) + 1
        except ApiError:
            pass
        return out


# ----------------------------------------------------------------------------- generators
def _container(nb: dict) -> dict:
    return nb["spec"]["template"]["spec"]["containers"][0]


def set_prefix_env_var(nb: dict, container: dict):
    prefix = f'/notebook/{nb["metadata"]["namespace"]}/{nb["metadata"]["name"]}'
    env = container.setdefault("env", [])
    for e in env:
        if e.get("name") == PREFIX_ENV_VAR:
            return  # an explicit NB_PREFIX is kept (reference semantics)
    env.append({"name": PREFIX_ENV_VAR, "value": prefix})


def generate_statefulset(nb: dict) -> dict:
    m = nb["metadata"]
    name, ns = m["name"], m["namespace"]
    annotations = m.get("annotations") or {}
    replicas = 0 if STOP_ANNOTATION in annotations else 1
    pod_spec = copy.deepcopy(nb["spec"]["template"]["spec"])
    labels = {"statefulset": name, "notebook-name": name}
    labels.update(m.get("labels") or {})
    pod_ann = {k: v for k, v in annotations.items() if "kubectl" not in k and "notebook" not in k}
    c = pod_spec["containers"][0]
    if not c.get("workingDir"):
        c["workingDir"] = "/home/jovyan"
    if c.get("ports") is None:
        c["ports"] = [{"containerPort": DEFAULT_CONTAINER_PORT, "name": "notebook-port", "protocol": "TCP"}]
    set_prefix_env_var(nb, c)
    if os.environ.get("ADD_FSGROUP", "true") == "true" and pod_spec.get("securityContext") is None:
        pod_spec["securityContext"] = {"fsGroup": DEFAULT_FS_GROUP}
    return {"apiVersion": "apps/v1", "kind": "StatefulSet",
            "metadata": {"name": name, "namespace": ns},
            "spec": {"replicas": replicas, "selector": {"matchLabels": {"statefulset": name}},
                     "serviceName": "",
                     "template": {"metadata": {"labels": labels, "annotations": pod_ann},
                                  "spec": pod_spec}}}


def generate_service(nb: dict) -> dict:
    m = nb["metadata"]
    port = DEFAULT_CONTAINER_PORT
    ports = _container(nb).get("ports")
    if ports:
        port = int(ports[0]["containerPort"])
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": {"name": m["name"], "namespace": m["namespace"]},
            "spec": {"type": "ClusterIP", "selector": {"statefulset": m["name"]},
                     "ports": [{"name": f'http-{m["name"]}', "port": DEFAULT_SERVING_PORT,
                                "targetPort": port, "protocol": "TCP"}]}}


def virtual_service_name(name: str, namespace: str) -> str:
    return f"notebook-{namespace}-{name}"


def generate_virtual_service(nb: dict) -> dict:
    m = nb["metadata"]
    name, ns = m["name"], m["namespace"]
    ann = m.get("annotations") or {}
    prefix = f"/notebook/{ns}/{name}/"
    rewrite = ann.get(ANNOTATION_REWRITE_URI) or prefix
    domain = os.environ.get("CLUSTER_DOMAIN", "cluster.local")
    headers = {}
    if ann.get(ANNOTATION_HEADERS_REQUEST_SET):
        try:
            headers = json.loads(ann[ANNOTATION_HEADERS_REQUEST_SET])
            if not isinstance(headers, dict):
                headers = {}
        except ValueError:
            headers = {}
    return {"apiVersion": "networking.istio.io/v1alpha3", "kind": "VirtualService",
            "metadata": {"name": virtual_service_name(name, ns), "namespace": ns},
            "spec": {"hosts": [os.environ.get("ISTIO_HOST") or "*"],
                     "gateways": [os.environ.get("ISTIO_GATEWAY") or "kubeflow/kubeflow-gateway"],
                     "http": [{"headers": {"request": {"set": headers}},
                               "match": [{"uri": {"prefix": prefix}}],
                               "rewrite": {"uri": rewrite},
                               "route": [{"destination": {"host": f"{name}.{ns}.svc.{domain}",
                                                          "port": {"number": DEFAULT_SERVING_PORT}}}]}]}}


def pod_cond_to_notebook_cond(pc: dict) -> dict:
    c = {}
    for k in ("type", "status", "message", "reason"):
        if pc.get(k):
            c[k] = pc[k]
    c["lastProbeTime"] = pc.get("lastProbeTime") or now_rfc3339()
    c["lastTransitionTime"] = pc.get("lastTransitionTime") or now_rfc3339()
    return c


def create_notebook_status(nb: dict, sts: dict, pod: Optional[dict]) -> dict:
    status = {"conditions": [], "readyReplicas": (sts.get("status") or {}).get("readyReplicas", 0),
              "containerState": {}}
    if not pod or not pod.get("status"):
        return status
    old_state = (nb.get("status") or {}).get("containerState") or {}
    for cs in pod["status"].get("containerStatuses") or []:
        if cs.get("name") != nb["metadata"]["name"]:
            continue
        if cs.get("state") == old_state:
            continue
        status["containerState"] = cs.get("state") or {}
        break
    status["conditions"] = [pod_cond_to_notebook_cond(c) for c in pod["status"].get("conditions") or []]
    return status


# ----------------------------------------------------------------------------- controller (G1)
class NotebookReconciler(Controller):
    name = "notebook-controller"

    def __init__(self, client: Client, metrics: Optional[NotebookMetrics] = None):
        super().__init__(client)
        self.metrics = metrics

    def _nb_name_from_involved(self, io: dict) -> Optional[str]:
        if io.get("kind") == "StatefulSet":
            return io.get("name")
        if io.get("kind") == "Pod":
            pod = self.client.get_or_none("v1", "Pod", io.get("name"), io.get("namespace"))
            if pod:
                return (pod["metadata"].get("labels") or {}).get("notebook-name")
        return None

    def sources(self):
        def pod_labeled(et, o):
            return "notebook-name" in (o["metadata"].get("labels") or {})

        def pod_map(et, o):
            return [Request(o["metadata"]["namespace"], o["metadata"]["labels"]["notebook-name"])]

        def event_pred(et, o):
            if et == "DELETED":
                return False
            io = o.get("involvedObject") or {}
            if io.get("kind") not in ("Pod", "StatefulSet"):
                return False
            nb = self._nb_name_from_involved(io)
            if nb is None:
                return False
            try:
                self.client.get(NB_API, "Notebook", nb, o["metadata"]["namespace"])
                return True
            except ApiError as e:
                return e.code != 404

        srcs = [for_kind(NB_API, "Notebook"), owns("apps/v1", "StatefulSet", "Notebook"),
                owns("v1", "Service", "Notebook"),
                watches("v1", "Pod", pod_map, pod_labeled),
                watches("v1", "Event",
                        lambda et, o: [Request(o["metadata"]["namespace"], o["metadata"]["name"])], event_pred)]
        if os.environ.get("USE_ISTIO") == "true":
            srcs.append(owns("networking.istio.io/v1alpha3", "VirtualService", "Notebook"))
        return srcs

    def reconcile(self, req: Request) -> Result:
        c = self.client
        ev = c.get_or_none("v1", "Event", req.name, req.namespace)
        if ev is not None:
            nb_name = self._nb_name_from_involved(ev.get("involvedObject") or {})
            if nb_name is None:
                raise ApiError(400, "BadRequest", "object isn't related to a Notebook")
            nb = c.get_or_none(NB_API, "Notebook", nb_name, req.namespace)
            if nb is None:
                return Result()
            io = ev["involvedObject"]
            c.record_event(nb, ev.get("type", "Normal"), ev.get("reason", ""),
                           f'Reissued from {io["kind"].lower()}/{io["name"]}: {ev.get("message", "")}',
                           source="notebook-controller")
            return Result()
        nb = c.get_or_none(NB_API, "Notebook", req.name, req.namespace)
        if nb is None:
            return Result()
        if nb["metadata"].get("deletionTimestamp"):
            return Result()   # foreground deletion in progress: do not recreate children
        # StatefulSet
        ss = set_controller_reference(nb, generate_statefulset(nb))
        found = c.get_or_none("apps/v1", "StatefulSet", ss["metadata"]["name"], req.namespace)
        if found is None:
            if self.metrics:
                self.metrics.create.labels(req.namespace).inc()
            try:
                found = c.create(ss)
            except ApiError:
                if self.metrics:
                    self.metrics.create_failed.labels(req.namespace).inc()
                raise
        elif reconcilehelper.copy_statefulset_fields(ss, found):
            found = c.update(found)
        # Service
        reconcilehelper.service(c, set_controller_reference(nb, generate_service(nb)))
        if os.environ.get("USE_ISTIO") == "true":
            reconcilehelper.virtual_service(c, set_controller_reference(nb, generate_virtual_service(nb)))
        pod = c.get_or_none("v1", "Pod", f'{ss["metadata"]["name"]}-0', req.namespace)
        new = create_notebook_status(nb, found, pod)
        old = nb.get("status") or {}
        # keep condition timestamps of unchanged conditions: a status write that only
        # moves timestamps would re-trigger this reconcile forever
        old_conds = {(x.get("type"), x.get("status"), x.get("reason"), x.get("message")): x
                     for x in old.get("conditions") or []}
        for cd in new["conditions"]:
            prev = old_conds.get((cd.get("type"), cd.get("status"), cd.get("reason"), cd.get("message")))
            if prev:
                cd["lastProbeTime"] = prev.get("lastProbeTime", cd["lastProbeTime"])
                cd["lastTransitionTime"] = prev.get("lastTransitionTime", cd["lastTransitionTime"])
        if not new["containerState"] and old.get("containerState"):
            new["containerState"] = old["containerState"] if pod else {}
        if new != old:
            nb["status"] = new
            c.update_status(nb)
        return Result()


# ----------------------------------------------------------------------------- culler (G1a)
def _parse_ts(s: str) -> Optional[dt.datetime]:
    try:
        return dt.datetime.strptime(s, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=dt.timezone.utc)
    except (TypeError, ValueError):
        try:
            return dt.datetime.fromisoformat(s.replace("Z", "+00:00"))
        except (TypeError, ValueError, AttributeError):
            return None


def _fmt(t: dt.datetime) -> str:
    return t.astimezone(dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


class CullingReconciler(Controller):
    """Stops notebooks whose Jupyter kernels have been idle for CULL_IDLE_TIME minutes,
    checking every IDLENESS_CHECK_PERIOD minutes via GET <svc>/notebook/<ns>/<nb>/api/kernels."""
    name = "culling-controller"

    def __init__(self, client: Client, metrics: Optional[NotebookMetrics] = None,
                 now: Callable[[], dt.datetime] = lambda: dt.datetime.now(dt.timezone.utc),
                 kernels_fetcher: Optional[Callable[[str, str], Optional[list]]] = None):
        super().__init__(client)
        self.metrics = metrics
        self.now = now
        self.fetch = kernels_fetcher or self.get_notebook_api_kernels
        self.cull_idle_minutes = self._int_env("CULL_IDLE_TIME", "1440")
        self.check_period_minutes = self._int_env("IDLENESS_CHECK_PERIOD", "1")
        self.dev = get_env_default("DEV", "false") != "false"

    @staticmethod
    def _int_env(name, default):
        try:
            return int(get_env_default(name, default))
        except ValueError:
            return int(default)

    def sources(self):
        return [for_kind(NB_API, "Notebook")]

    def requeue(self) -> Result:
        return Result(requeue_after=self.check_period_minutes * 60.0)

    def get_notebook_api_kernels(self, name: str, ns: str) -> Optional[list]:
        domain = get_env_default("CLUSTER_DOMAIN", "cluster.local")
        url = f"http://{name}.{ns}.svc.{domain}/notebook/{ns}/{name}/api/kernels"
        if self.dev:
            url = (f"http://localhost:8001/api/v1/namespaces/{ns}/services/{name}:http-{name}/proxy/"
                   f"notebook/{ns}/{name}/api/kernels")
        try:
            with urllib.request.urlopen(url, timeout=10) as r:
                if r.status != 200:
                    return None
                return json.loads(r.read().decode())
        except Exception as e:
            log.info("Error talking to %s: %s", url, e)
            return None

    def update_timestamp_from_kernels(self, ann: dict, kernels: list):
        if any(k.get("execution_state") != "idle" for k in kernels):
            ann[LAST_ACTIVITY_ANNOTATION] = _fmt(self.now())
            return
        times = [_parse_ts(k.get("last_activity", "")) for k in kernels]
        if any(t is None for t in times):
            return
        ann[LAST_ACTIVITY_ANNOTATION] = _fmt(max(times))

    def notebook_is_idle(self, ann: dict) -> bool:
        if STOP_ANNOTATION in ann:
            return False
        last = _parse_ts(ann.get(LAST_ACTIVITY_ANNOTATION, ""))
        if last is None:
            return False
        return self.now() > last + dt.timedelta(minutes=self.cull_idle_minutes)

    def check_period_passed(self, ann: dict) -> bool:
        ts = _parse_ts(ann.get(LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION, ""))
        if ts is None:
            return False
        return ts + dt.timedelta(minutes=self.check_period_minutes) < self.now()

    def reconcile(self, req: Request) -> Result:
        c = self.client
        nb = c.get_or_none(NB_API, "Notebook", req.name, req.namespace)
        if nb is None:
            return Result()
        ann = nb["metadata"].setdefault("annotations", {})
        if STOP_ANNOTATION in ann:
            ann.pop(LAST_ACTIVITY_ANNOTATION, None)
            ann.pop(LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION, None)
            c.update(nb)
            return Result()
        pod = c.get_or_none("v1", "Pod", f"{req.name}-0", req.namespace)
        if pod is None:
            ann.pop(LAST_ACTIVITY_ANNOTATION, None)
            ann.pop(LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION, None)
            c.update(nb)
            return Result()
        if LAST_ACTIVITY_ANNOTATION not in ann or LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION not in ann:
            t = _fmt(self.now())
            ann[LAST_ACTIVITY_ANNOTATION] = t
            ann[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION] = t
            nb = c.update(nb)
            ann = nb["metadata"]["annotations"]
        if not self.check_period_passed(ann):
            return self.requeue()
        kernels = self.fetch(req.name, req.namespace)
        if kernels:
            self.update_timestamp_from_kernels(ann, kernels)
        ann[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION] = _fmt(self.now())
        nb = c.update(nb)
        ann = nb["metadata"]["annotations"]
        if self.notebook_is_idle(ann):
            t = self.now()
            ann[STOP_ANNOTATION] = _fmt(t)
            if self.metrics:
                self.metrics.culling.labels(req.namespace, req.name).inc()
                self.metrics.culling_ts.labels(req.namespace, req.name).set(t.timestamp())
            c.update(nb)
        return self.requeue()


def setup(manager, client: Client, registry=None):
    """main.go equivalent: register the notebook controller (+ culler when ENABLE_CULLING)."""
    metrics = NotebookMetrics(client, registry)
    manager.add(NotebookReconciler(client, metrics))
    if os.environ.get("ENABLE_CULLING", "false") == "true":
        manager.add(CullingReconciler(client, metrics))
    return metrics
