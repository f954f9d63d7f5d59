"""T1: Central dashboard server (the Express app on :8082) -- Python/Flask.

Behavioural reference: components/centraldashboard/app/{server.ts, api.ts,
api_workgroup.ts, k8s_service.ts, attach_user_middleware.ts, metrics_service.ts,
prometheus_metrics_service.ts, metrics_service_factory.ts}.

* user: ``USERID_HEADER`` (default ``X-Goog-Authenticated-User-Email``) minus
  ``USERID_PREFIX`` (``accounts.google.com:``); no header -> ``anonymous@kubeflow.org``,
  ``hasAuth = false``.
* ``/api``: ``metrics`` (charts link), ``metrics/{node,podcpu,podmem}?interval=Last15m``,
  ``namespaces``, ``activities/<ns>`` (events), ``dashboard-links`` /
  ``dashboard-settings`` (JSON in the ``centraldashboard-config`` ConfigMap).
* ``/api/workgroup``: ``exists``, ``create``, ``env-info``, then (authenticated only)
  ``nuke-self``, ``get-all-namespaces``, ``get-contributors/<ns>``,
  ``add-contributor/<ns>``, ``remove-contributor/<ns>`` -- all through KFAM, forwarding
  only the identity headers.  Roles map admin<->owner, edit<->contributor, view<->viewer.
* Metrics (``metrics_service_for``, the provider factory): Stackdriver / Cloud Monitoring
  on GCE/GKE nodes, Prometheus range queries when ``PROMETHEUS_URL`` is set, otherwise a
  local sampler (host CPU via psutil, kubelet pod CPU/RSS, and MI355X busy % / VRAM from
  ``rocm-smi`` when present) so a single-node install still has charts.
"""
from __future__ import annotations

import json
import logging
import os
import re
import subprocess
import threading
import time
import urllib.parse
import urllib.request
from typing import Callable, Dict, List, Optional, Tuple

from flask import Flask, Response, jsonify, request, send_from_directory

from ..controlplane.apiserver import ApiError
from ..controlplane.client import Client

log = logging.getLogger("centraldashboard")
HERE = os.path.dirname(os.path.abspath(__file__))
EMAIL_RGX = re.compile(r"^[a-zA-Z0-9.!#$%&'*+/=?^_`{|}~-]+@[a-zA-Z0-9](?:[a-zA-Z0-9-]{0,61}[a-zA-Z0-9])?"
                       r"(?:\.[a-zA-Z0-9](?:[a-zA-Z0-9-]{0,61}[a-zA-Z0-9])?)*$")
ROLE_MAP = {"admin": "owner", "owner": "admin", "edit": "contributor", "contributor": "edit",
            "view": "viewer", "viewer": "view"}
INTERVALS = {"Last5m": 5, "Last15m": 15, "Last30m": 30, "Last60m": 60, "Last180m": 180}
ERRORS = {"no_metrics_service_configured": "No metrics service configured",
          "operation_not_supported": "Operation not supported",
          "invalid_links_config": "Cannot load dashboard menu link",
          "invalid_settings": "Cannot load dashboard settings"}


class KfamError(Exception):
    def __init__(self, status: int, body: str):
        super().__init__(f"HTTP {status}: {body}")
        self.status, self.body = status, body


# ------------------------------------------------------------------ KFAM client
Transport = Callable[[str, str, Optional[bytes], Dict[str, str]], Tuple[int, bytes]]


def http_transport(base_url: str) -> Transport:
    def do(method, path, body, headers):
        req = urllib.request.Request(base_url + path, data=body, method=method,
                                     headers=dict(headers, **{"Content-Type": "application/json"}))
        try:
            with urllib.request.urlopen(req, timeout=30) as r:
                return r.status, r.read()
        except urllib.error.HTTPError as e:
            return e.code, e.read()
    return do


class ProfilesService:
    """The generated ``DefaultApi`` KFAM client (clients/profile_controller)."""

    def __init__(self, transport: Transport):
        self.t = transport

    def _call(self, method, path, body=None, headers=None):
        data = json.dumps(body).encode() if body is not None else None
        code, out = self.t(method, path, data, headers or {})
        if code >= 300:
            raise KfamError(code, out.decode(errors="replace"))
        return out

    def read_bindings(self, user=None, namespace=None, role=None) -> List[dict]:
        q = {k: v for k, v in (("user", user), ("namespace", namespace), ("role", role)) if v}
        out = self._call("GET", "/v1/bindings" + ("?" + urllib.parse.urlencode(q) if q else ""))
        return (json.loads(out) or {}).get("bindings") or []

    def is_cluster_admin(self, user) -> bool:
        return self._call("GET", "/v1/role/clusteradmin?" + urllib.parse.urlencode({"user": user})).strip() == b"true"

    def create_binding(self, b, headers):
        self._call("POST", "/v1/bindings", b, headers)

    def delete_binding(self, b, headers):
        self._call("DELETE", "/v1/bindings", b, headers)

    def create_profile(self, p):
        self._call("POST", "/v1/profiles", p)

    def delete_profile(self, name, headers):
        return self._call("DELETE", f"/v1/profiles/{name}", None, headers).decode()


def to_simple(bindings: List[dict]) -> List[dict]:
    return [{"user": b["user"]["name"], "namespace": b["referredNamespace"],
             "role": ROLE_MAP.get(b["roleRef"]["name"])} for b in bindings]


def to_workgroup_binding(user, namespace, role) -> dict:
    return {"user": {"kind": "User", "name": user}, "referredNamespace": namespace,
            "roleRef": {"kind": "ClusterRole", "name": ROLE_MAP[role]}}


# ------------------------------------------------------------------ metrics services
class MetricsService:
    def node_cpu(self, minutes: int) -> List[dict]:
        raise NotImplementedError

    def pod_cpu(self, minutes: int) -> List[dict]:
        raise NotImplementedError

    def pod_mem(self, minutes: int) -> List[dict]:
        raise NotImplementedError

    def charts_link(self) -> dict:
        raise NotImplementedError


class PrometheusMetricsService(MetricsService):
    def __init__(self, url: str, dashboard_url: Optional[str], fetch=None):
        self.url, self.dashboard_url = url.rstrip("/"), dashboard_url
        self.fetch = fetch or (lambda u: urllib.request.urlopen(u, timeout=30).read())

    def _range(self, query, minutes):
        end = time.time()
        q = urllib.parse.urlencode({"query": query, "start": end - minutes * 60, "end": end, "step": 10})
        body = json.loads(self.fetch(f"{self.url}/api/v1/query_range?{q}"))
        data = body.get("data") or {}
        if data.get("resultType") != "matrix":
            log.warning("The prometheus server returned invalid result type: %s", data.get("resultType"))
            return []
        out = []
        for serie in data.get("result") or []:
            label = ",".join(f"{k}={v}" for k, v in (serie.get("metric") or {}).items())
            for ts, v in serie.get("values") or []:
                out.append({"timestamp": float(ts), "label": label, "value": float(v) / 100})
        return out

    def node_cpu(self, minutes):
        return self._range("sum(rate(node_cpu_seconds_total[5m])) by (instance)", minutes)

    def pod_cpu(self, minutes):
        return self._range("sum(rate(container_cpu_usage_seconds_total[5m]))", minutes)

    def pod_mem(self, minutes):
        return self._range("sum(container_memory_usage_bytes)", minutes)

    def charts_link(self):
        return {"resourceChartsLink": self.dashboard_url, "resourceChartsLinkText": "View in dashboard"}


class StackdriverMetricsService(MetricsService):
    """Cloud Monitoring (Stackdriver) time series for GKE clusters
    (reference: centraldashboard/app/stackdriver_metrics_service.ts:15-204).

    ``projects.timeSeries.list`` over the Monitoring REST API v3, aligned to 1-minute means
    (ALIGN_MEAN, REDUCE_NONE) over the requested interval, with the reference's filters:
    node CPU = ``kubernetes.io/node/cpu/allocatable_utilization`` of this cluster's nodes,
    pod CPU = ``kubernetes.io/container/cpu/limit_utilization`` and pod memory =
    ``kubernetes.io/container/memory/used_bytes`` (non-evictable) of this cluster (its name
    from the GCE metadata server).  Points come back chronologically sorted; a failed query
    yields no points (logged), as in the reference.  The access token comes from the same
    ADC code the Profile controller uses (controlplane/cloud_iam.GcpToken)."""

    BASE = "kubernetes.io"
    NODE_CPU = f"{BASE}/node/cpu/allocatable_utilization"
    CONTAINER_CPU = f"{BASE}/container/cpu/limit_utilization"
    CONTAINER_MEM = f"{BASE}/container/memory/used_bytes"
    CLUSTER_NAME_URL = "http://metadata.google.internal/computeMetadata/v1/instance/attributes/cluster-name"
    API = "https://monitoring.googleapis.com/v3"

    def __init__(self, project_id: str, node_names: List[str], transport=None, token=None,
                 clock: Callable[[], float] = time.time):
        from ..controlplane.cloud_iam import GcpToken
        from ..utils import iap
        self.project_id, self.node_names = project_id, list(node_names)
        self.t = transport or iap.urllib_transport
        self.token = token or GcpToken(self.t, scope="https://www.googleapis.com/auth/monitoring.read")
        self.clock = clock
        self._cluster: Optional[str] = None

    def cluster_name(self) -> str:
        if self._cluster is None:
            try:
                code, text = self.t("GET", self.CLUSTER_NAME_URL, {"Metadata-Flavor": "Google"}, None)
                self._cluster = text.strip() if code == 200 else ""
            except ConnectionError:
                log.warning("Unable to obtain cluster name from Metadata server")
                self._cluster = ""
        return self._cluster

    def _fetch(self, flt: str, minutes: int) -> List[dict]:
        now = int(self.clock())
        fmt = lambda t: time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))   # noqa: E731
        params = {"filter": flt, "interval.startTime": fmt(now - 60 * minutes), "interval.endTime": fmt(now),
                  "aggregation.alignmentPeriod": "60s", "aggregation.perSeriesAligner": "ALIGN_MEAN",
                  "aggregation.crossSeriesReducer": "REDUCE_NONE"}
        series, page = [], None
        while True:
            q = dict(params, **({"pageToken": page} if page else {}))
            url = f"{self.API}/projects/{self.project_id}/timeSeries?" + urllib.parse.urlencode(q)
            code, text = self.t("GET", url, {"Authorization": f"Bearer {self.token.token()}"}, None)
            if code != 200:
                raise RuntimeError(f"timeSeries.list HTTP {code}: {text[:200]}")
            body = json.loads(text or "{}")
            series.extend(body.get("timeSeries") or [])
            page = body.get("nextPageToken")
            if not page:
                return series

    @staticmethod
    def _ts(point) -> float:
        end = (point.get("interval") or {}).get("endTime", "")
        try:
            import datetime as _dt
            return _dt.datetime.strptime(end[:19], "%Y-%m-%dT%H:%M:%S").replace(tzinfo=_dt.timezone.utc).timestamp()
        except ValueError:
            return 0.0

    def _points(self, flt, minutes, label_fn, what) -> List[dict]:
        out = []
        try:
            for ts in self._fetch(flt, minutes):
                labels = (ts.get("resource") or {}).get("labels") or {}
                for p in ts.get("points") or []:
                    v = (p.get("value") or {})
                    val = v.get("doubleValue", v.get("int64Value", 0))
                    out.append({"timestamp": self._ts(p), "label": label_fn(labels), "value": float(val)})
        except Exception as e:        # the reference logs and returns what it has
            log.error("Unable to fetch %s metrics: %s", what, e)
        out.sort(key=lambda x: x["timestamp"])
        return out

    def node_cpu(self, minutes):
        names = self.node_names
        flt = f'metric.type="{self.NODE_CPU}" AND resource.label.node_name='
        flt += ('one_of("' + '", "'.join(names) + '")') if len(names) > 1 else f'"{names[0] if names else ""}"'
        return self._points(flt, minutes, lambda lab: lab.get("node_name"), "Node CPU Utilization")

    def _cluster_filter(self, flt):
        c = self.cluster_name()
        return flt + (f' AND resource.label.cluster_name="{c}"' if c else "")

    def pod_cpu(self, minutes):
        return self._points(self._cluster_filter(f'metric.type="{self.CONTAINER_CPU}"'), minutes,
                            lambda lab: lab.get("container_name") or lab.get("pod_name"), "Pod CPU Utilization")

    def pod_mem(self, minutes):
        flt = self._cluster_filter(f'metric.type="{self.CONTAINER_MEM}" AND metric.label.memory_type = "non-evictable"')
        return self._points(flt, minutes, lambda lab: lab.get("container_name") or lab.get("pod_name"),
                            "Pod Memory Utilization")

    def charts_link(self):
        return {"resourceChartsLink": f"https://app.google.stackdriver.com/kubernetes?project={self.project_id}",
                "resourceChartsLinkText": "View in Stackdriver"}


def metrics_service_for(kube: Client, env: Optional[dict] = None, transport=None) -> Optional[MetricsService]:
    """Provider factory (reference: centraldashboard/app/metrics_service_factory.ts:13-35): on GCE/GKE
    (node ``providerID`` ``gce://<project>/<zone>/<instance>``) the Stackdriver service over this
    cluster's nodes; else Prometheus when ``PROMETHEUS_URL`` is set; else the local sampler
    (single-node installs: host CPU, pod CPU/RSS, MI355X busy %).  ``KFAMD_METRICS=none``
    disables metrics (the reference's unsupported-platform ``null``)."""
    env = dict(os.environ if env is None else env)
    if env.get("KFAMD_METRICS") == "none":
        return None
    try:
        nodes = kube.list("v1", "Node")
    except ApiError:
        nodes = []
    provider = next(((n.get("spec") or {}).get("providerID") for n in nodes
                     if (n.get("spec") or {}).get("providerID")), "other://")
    if provider.split(":")[0] == "gce":
        project = provider.split("/")[2]
        return StackdriverMetricsService(project, [n["metadata"]["name"] for n in nodes], transport=transport)
    if env.get("PROMETHEUS_URL"):
        return PrometheusMetricsService(env["PROMETHEUS_URL"], env.get("METRICS_DASHBOARD"))
    log.warning('"%s" is not a supported platform for cloud metrics; using the local sampler',
                provider.split(":")[0])
    return LocalMetricsService()


def read_gpu_stats() -> List[dict]:
    """MI355X busy % and VRAM used per GPU from ``rocm-smi --json`` (absent -> [])."""
    for cmd in (["rocm-smi", "--showuse", "--showmemuse", "--json"],):
        try:
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=10).stdout
            d = json.loads(out)
        except Exception:
            continue
        res = []
        for card, v in sorted(d.items()):
            if not card.startswith("card"):
                continue
            busy = next((float(x) for k, x in v.items() if "GPU use" in k), 0.0)
            mem = next((float(x) for k, x in v.items() if "Memory Allocated" in k or "VRAM%" in k), 0.0)
            res.append({"gpu": card, "busy": busy, "vram": mem})
        return res
    return []


class LocalMetricsService(MetricsService):
    """Samples every ``period`` seconds into a ring buffer (3 h)."""

    def __init__(self, pod_pids: Callable[[], Dict[str, int]] = lambda: {}, period: float = 10.0,
                 start: bool = True):
        self.pod_pids, self.period = pod_pids, period
        self.samples: List[Tuple[float, str, str, float]] = []   # (ts, series, label, value)
        self._lock = threading.Lock()
        self._stop = threading.Event()
        if start:
            threading.Thread(target=self._loop, daemon=True).start()

    def sample(self, now=None):
        import psutil
        now = now or time.time()
        rows = [(now, "node", "instance=localhost", psutil.cpu_percent(interval=None) / 100)]
        for pod, pid in self.pod_pids().items():
            try:
                p = psutil.Process(pid)
                rows.append((now, "podcpu", f"pod={pod}", p.cpu_percent(interval=None) / 100))
                rows.append((now, "podmem", f"pod={pod}", float(p.memory_info().rss)))
            except Exception:
                pass
        for g in read_gpu_stats():
            rows.append((now, "gpu", f"gpu={g['gpu']}", g["busy"] / 100))
        with self._lock:
            self.samples.extend(rows)
            cut = now - 180 * 60
            self.samples = [s for s in self.samples if s[0] >= cut]

    def _loop(self):
        while not self._stop.wait(self.period):
            try:
                self.sample()
            except Exception:
                log.exception("metrics sample failed")

    def _series(self, name, minutes):
        cut = time.time() - minutes * 60
        with self._lock:
            return [{"timestamp": t, "label": lab, "value": v} for t, s, lab, v in self.samples
                    if s == name and t >= cut]

    def node_cpu(self, minutes):
        return self._series("node", minutes)

    def pod_cpu(self, minutes):
        return self._series("podcpu", minutes)

    def pod_mem(self, minutes):
        return self._series("podmem", minutes)

    def gpu_busy(self, minutes):
        return self._series("gpu", minutes)

    def charts_link(self):
        return {"resourceChartsLink": None, "resourceChartsLinkText": "View in dashboard"}

    def stop(self):
        self._stop.set()


# ------------------------------------------------------------------ app
def api_error(error: str, code: int = 400):
    return jsonify({"error": error}), code


def create_app(kube: Client, profiles: ProfilesService, metrics: Optional[MetricsService] = None,
               env: Optional[dict] = None, static_dir: Optional[str] = None) -> Flask:
    env = dict(os.environ if env is None else env)
    production = env.get("NODE_ENV") == "production"
    code_env = "production" if production else "development"
    user_header = env.get("USERID_HEADER", "X-Goog-Authenticated-User-Email")
    user_prefix = env.get("USERID_PREFIX", "accounts.google.com:")
    registration = env.get("REGISTRATION_FLOW", "true").lower() == "true"
    cm_name = env.get("DASHBOARD_CONFIGMAP", "centraldashboard-config")
    logout_url = env.get("LOGOUT_URL", "/logout")
    pod_ns = env.get("POD_NAMESPACE", "kubeflow")
    # two frontends on the same API (the reference ships centraldashboard and
    # centraldashboard-angular): DASHBOARD_FRONTEND=angular serves the second one at "/"; it is
    # always reachable under /ng/ as well (static/dashboard-ng.js)
    ng_dir = os.path.join(HERE, "static", "dashboard-ng")
    if static_dir is None and env.get("DASHBOARD_FRONTEND", "").lower() in ("angular", "ng"):
        static_dir = ng_dir
    static_dir = static_dir or os.path.join(HERE, "static", "dashboard")
    app = Flask("centraldashboard", static_folder=None)
    platform_cache = {}

    def user():
        v = request.headers.get(user_header)
        email, auth = "anonymous@kubeflow.org", None
        if v:
            email, auth = v[len(user_prefix):], {user_header: v}
        return {"email": email, "username": email.split("@")[0],
                "domain": email.split("@")[1] if "@" in email else None, "hasAuth": auth is not None, "auth": auth}

    def platform_info():
        if not platform_cache:
            provider = "other://"
            try:
                for n in kube.list("v1", "Node"):
                    pid = (n.get("spec") or {}).get("providerID")
                    if pid:
                        provider = pid
                        break
            except ApiError:
                pass
            version = "unknown"
            try:
                for a in kube.list("app.k8s.io/v1beta1", "Application", pod_ns):
                    d = ((a.get("spec") or {}).get("descriptor") or {})
                    if re.fullmatch(r"kubeflow", d.get("type", ""), re.I):
                        version = d.get("version", version)
                        break
            except (ApiError, KeyError):
                pass
            platform_cache.update(kubeflowVersion=version, provider=provider, providerName=provider.split(":")[0],
                                  logoutUrl=logout_url)
        return dict(platform_cache)

    def config_map():
        try:
            return kube.get("v1", "ConfigMap", cm_name, pod_ns)
        except ApiError:
            return None

    def surface(msg, err):
        if isinstance(err, KfamError):
            return api_error(err.body or msg, err.status)
        log.exception(msg)
        return api_error(msg, 400)

    def workgroup_info(u):
        return {"isClusterAdmin": profiles.is_cluster_admin(u["email"]),
                "namespaces": to_simple(profiles.read_bindings(user=u["email"]))}

    def all_workgroups(fake_user):
        names = sorted({b["namespace"] for b in to_simple(profiles.read_bindings())})
        return [{"namespace": n, "role": "contributor", "user": fake_user} for n in names]

    def contributors(ns):
        return [b["user"] for b in to_simple(profiles.read_bindings(namespace=ns)) if b["role"] == "contributor"]

    # --- top level
    @app.get("/debug")
    def debug():
        u = user()
        return jsonify({"user": u, "profilesServiceUrl": env.get("PROFILES_SERVICE_URL", ""),
                        "codeEnvironment": code_env, "registrationFlowAllowed": registration,
                        "headersForIdentity": {"USERID_HEADER": user_header, "USERID_PREFIX": user_prefix}})

    @app.get("/healthz")
    def healthz():
        return jsonify({"codeEnvironment": code_env, "message": "I tick, therfore I am!"})

    # --- /api
    @app.get("/api/metrics")
    def metrics_link():
        if metrics is None:
            return api_error(ERRORS["operation_not_supported"], 405)
        return jsonify(metrics.charts_link())

    @app.get("/api/metrics/<mtype>")
    def metrics_series(mtype):
        if mtype not in ("node", "podcpu", "podmem", "gpu"):
            return api_error("Could not find the route you're looking for", 404)
        if metrics is None:
            return api_error(ERRORS["operation_not_supported"], 405)
        minutes = INTERVALS.get(request.args.get("interval", ""), 15)
        if mtype == "gpu":
            fn = getattr(metrics, "gpu_busy", None)
            return jsonify(fn(minutes) if fn else [])
        return jsonify({"node": metrics.node_cpu, "podcpu": metrics.pod_cpu, "podmem": metrics.pod_mem}[mtype](minutes))

    @app.get("/api/namespaces")
    def namespaces():
        try:
            return jsonify(kube.list("v1", "Namespace"))
        except ApiError:
            return jsonify([])

    @app.get("/api/activities/<ns>")
    def activities(ns):
        try:
            return jsonify(kube.list("v1", "Event", ns))
        except ApiError:
            return jsonify([])

    @app.get("/api/dashboard-links")
    def dashboard_links():
        cm = config_map()
        try:
            return jsonify(json.loads(cm["data"]["links"]))
        except (TypeError, KeyError, ValueError):
            return api_error(ERRORS["invalid_links_config"], 500)

    @app.get("/api/dashboard-settings")
    def dashboard_settings():
        cm = config_map()
        try:
            return jsonify(json.loads(cm["data"]["settings"]))
        except (TypeError, KeyError, ValueError):
            return api_error(ERRORS["invalid_settings"], 500)

    # --- /api/workgroup
    @app.get("/api/workgroup/exists")
    def wg_exists():
        u = user()
        try:
            resp = {"hasAuth": u["hasAuth"], "user": u["username"], "hasWorkgroup": False,
                    "registrationFlowAllowed": registration}
            if u["hasAuth"]:
                resp["hasWorkgroup"] = any(b["role"] == "owner" for b in workgroup_info(u)["namespaces"])
            else:
                resp["hasWorkgroup"] = bool(all_workgroups(u["username"]))
            return jsonify(resp)
        except Exception as e:
            return surface("Unable to contact Profile Controller", e)

    @app.post("/api/workgroup/create")
    def wg_create():
        u = user()
        body = request.get_json(silent=True) or {}
        ns = body.get("namespace") or u["username"]
        try:
            profiles.create_profile({"metadata": {"name": ns},
                                     "spec": {"owner": {"kind": "User", "name": body.get("user") or u["email"]}}})
            return jsonify({"message": f"Created namespace {ns}"})
        except Exception as e:
            return surface("Unexpected error creating profile", e)

    @app.get("/api/workgroup/env-info")
    def wg_env_info():
        u = user()
        try:
            if u["hasAuth"]:
                info = workgroup_info(u)
                return jsonify({"user": u["email"], "platform": platform_info(), "namespaces": info["namespaces"],
                                "isClusterAdmin": info["isClusterAdmin"]})
            return jsonify({"user": u["email"], "platform": platform_info(),
                            "namespaces": all_workgroups(u["email"]), "isClusterAdmin": True})
        except KfamError as e:
            return api_error(e.body or "Unexpected error getting environment info", e.status)

    def require_auth():
        if not user()["hasAuth"]:
            return api_error("Unable to ascertain user identity from request, cannot access route.", 405)
        return None

    @app.delete("/api/workgroup/nuke-self")
    def wg_nuke_self():
        err = require_auth()
        if err:
            return err
        u = user()
        try:
            body = profiles.delete_profile(u["username"], u["auth"])
            return jsonify({"message": f"Removed namespace/profile {u['username']}", "serverBody": body})
        except Exception as e:
            return surface("Unexpected error deleting profile", e)

    @app.get("/api/workgroup/get-all-namespaces")
    def wg_all_namespaces():
        err = require_auth()
        if err:
            return err
        try:
            nss: Dict[str, dict] = {}
            for b in to_simple(profiles.read_bindings()):
                ent = nss.setdefault(b["namespace"], {"contributors": []})
                if b["role"] == "owner":
                    ent["owner"] = b["user"]
                else:
                    ent["contributors"].append(b["user"])
            return jsonify([[n, v.get("owner"), ", ".join(v["contributors"])] for n, v in nss.items()])
        except Exception as e:
            return surface("Unable to fetch all workgroup data", e)

    @app.get("/api/workgroup/get-contributors/<ns>")
    def wg_get_contributors(ns):
        err = require_auth()
        if err:
            return err
        try:
            return jsonify(contributors(ns))
        except Exception as e:
            return surface(f"Unable to fetch contributors for {ns}", e)

    def handle_contributor(action, ns):
        err = require_auth()
        if err:
            return err
        body = request.get_json(silent=True) or {}
        contributor = body.get("contributor")
        if not contributor or not ns:
            missing = [f for f, v in (("contributor", contributor), ("namespace", ns)) if not v]
            return api_error(f"Missing {' and '.join(missing)} field{'s' if len(missing) > 1 else ''}.")
        if not EMAIL_RGX.match(contributor):
            return api_error("Contributor doesn't look like a valid email address")
        keep = {"authorization", "cookie", user_header.lower()}
        headers = {k: v for k, v in request.headers.items() if k.lower() in keep}
        b = to_workgroup_binding(contributor, ns, "contributor")
        stage = 0
        try:
            (profiles.create_binding if action == "create" else profiles.delete_binding)(b, headers)
            stage = 1
            return jsonify(contributors(ns))
        except KfamError as e:
            msg = [f"Unable to add new contributor for {ns}. HTTP {e.status}",
                   f"Unable to fetch contributors for {ns}. HTTP {e.status}"][stage]
            return api_error(e.body or msg, e.status)

    @app.post("/api/workgroup/add-contributor/<ns>")
    def wg_add(ns):
        return handle_contributor("create", ns)

    @app.delete("/api/workgroup/remove-contributor/<ns>")
    def wg_remove(ns):
        return handle_contributor("remove", ns)

    @app.route("/api/<path:rest>", methods=["GET", "POST", "DELETE", "PUT", "PATCH"])
    def api_404(rest):
        return api_error("Could not find the route you're looking for", 404)

    # --- SPA
    @app.get("/")
    @app.get("/<path:path>")
    def spa(path="index.html"):
        if path.startswith("static/"):         # the shared UI bundle (webapps/static/kfamd-ui.js)
            return send_from_directory(os.path.join(HERE, "static"), path[len("static/"):])
        if path == "ng" or path.startswith("ng/"):
            return send_from_directory(ng_dir, "index.html")
        full = os.path.join(static_dir, path)
        if path != "index.html" and os.path.isfile(full):
            return send_from_directory(static_dir, path)
        idx = os.path.join(static_dir, "index.html")
        if not os.path.exists(idx):
            return Response("central dashboard", mimetype="text/html")
        return send_from_directory(static_dir, "index.html")

    return app
