"""Controller runtime ("reconcile kit"): the controller-runtime equivalent used by every
controller in this repo.

* ``Controller``: a ``reconcile(Request) -> Result`` function plus watch sources.  A watch
  maps an API event to requests: ``for_kind`` (the object itself), ``owns`` (the
  controller owner of the object), or an arbitrary map function, each with an optional
  predicate -- the shapes used by the reference controllers (e.g. the Notebook
  controller watches Pods labelled ``notebook-name`` and re-emits Pod/STS Events).
* ``Informer``: one shared list+watch per watched kind (LIST, then a watch from the list's
  resourceVersion, so no event between them is lost), keeping a local object store.
  Controllers added to a caching Manager read through :class:`CachedClient`: ``get`` /
  ``list`` of watched kinds are served from the informer stores (controller-runtime's
  cache-backed client), writes and other kinds go to the API server.
* ``Manager``: de-duplicating work queue with client-go semantics in O(1) (FIFO deque +
  dirty set + processing set: a key is never reconciled by two workers at once, and a key
  re-added while in flight runs again once after it finishes), per-item exponential
  back-off on error
  (5 ms doubling to 1000 s, controller-runtime's default rate limiter),
  ``RequeueAfter`` timers, worker threads, optional leader election through a
  ``coordination.k8s.io/v1`` Lease, ``/healthz`` ``/readyz`` ``/metrics`` endpoints
  (prometheus_client).  ``run_until_idle()`` drains the queue synchronously for tests.
"""
from __future__ import annotations

import copy
import heapq
import logging
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, Tuple

from .apiserver import ApiError, NotFound, fields_match, labels_match, now_rfc3339, split_api_version
from .client import Client

log = logging.getLogger("controlplane.runtime")


@dataclass(frozen=True)
class Request:
    namespace: Optional[str]
    name: str


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float = 0.0   # seconds


MapFn = Callable[[str, dict], List[Request]]
Predicate = Callable[[str, dict], bool]


@dataclass
class WatchSource:
    api_version: str
    kind: str
    mapper: MapFn
    predicate: Optional[Predicate] = None


def for_kind(api_version: str, kind: str, predicate: Optional[Predicate] = None) -> WatchSource:
    return WatchSource(api_version, kind,
                       lambda et, o: [Request(o["metadata"].get("namespace"), o["metadata"]["name"])],
                       predicate)


def owns(api_version: str, kind: str, owner_kind: str, predicate: Optional[Predicate] = None) -> WatchSource:
    def m(et, o):
        out = []
        for ref in o.get("metadata", {}).get("ownerReferences") or []:
            if ref.get("controller") and ref.get("kind") == owner_kind:
                out.append(Request(o["metadata"].get("namespace"), ref["name"]))
        return out
    return WatchSource(api_version, kind, m, predicate)


def watches(api_version: str, kind: str, mapper: MapFn, predicate: Optional[Predicate] = None) -> WatchSource:
    return WatchSource(api_version, kind, mapper, predicate)


class Controller:
    name: str = "controller"

    def __init__(self, client: Client):
        self.client = client

    def sources(self) -> List[WatchSource]:
        return []

    def reconcile(self, req: Request) -> Result:
        raise NotImplementedError


class RateLimiter:
    """Per-item exponential failure back-off (controller-runtime default: 5 ms * 2^n, cap 1000 s)."""

    def __init__(self, base: float = 0.005, cap: float = 1000.0):
        self.base, self.cap = base, cap
        self.failures: Dict[Tuple[str, Request], int] = {}

    def when(self, key) -> float:
        n = self.failures.get(key, 0)
        self.failures[key] = n + 1
        return min(self.cap, self.base * (2 ** n))

    def forget(self, key):
        self.failures.pop(key, None)


class WorkQueue:
    """client-go ``workqueue`` semantics, every operation O(1): ``add`` de-duplicates (a key
    waiting in the queue is not queued twice); a key added while a worker processes it is
    marked dirty and re-queued by ``done``, so it is never processed concurrently and never
    lost."""

    def __init__(self):
        self._q: deque = deque()
        self._dirty: set = set()
        self._processing: set = set()

    def add(self, item):
        if item in self._dirty:
            return
        self._dirty.add(item)
        if item not in self._processing:
            self._q.append(item)

    def get(self):
        """Next item to process (marked in flight) or None."""
        if not self._q:
            return None
        item = self._q.popleft()
        self._processing.add(item)
        self._dirty.discard(item)
        return item

    def done(self, item):
        self._processing.discard(item)
        if item in self._dirty:
            self._q.append(item)

    def __len__(self):
        return len(self._q)

    def __contains__(self, item):
        return item in self._dirty


class Informer:
    """Shared list+watch of one kind with a local store (client-go SharedIndexInformer)."""

    def __init__(self, client: Client, api_version: str, kind: str):
        self.client, self.api_version, self.kind = client, api_version, kind
        self.group = split_api_version(api_version)[0]
        self.store: Dict[Tuple[Optional[str], str], dict] = {}
        self.handlers: List[Callable[[str, dict], None]] = []
        self.synced = False
        self._lock = threading.RLock()
        self._cancel: Optional[Callable] = None

    @staticmethod
    def _key(o: dict):
        m = o.get("metadata", {})
        return (m.get("namespace"), m["name"])

    def _on_event(self, et: str, obj: dict):
        with self._lock:
            if et == "DELETED":
                self.store.pop(self._key(obj), None)
            else:
                self.store[self._key(obj)] = obj
        for h in list(self.handlers):
            h(et, obj)

    def start(self):
        lister = getattr(self.client, "list_with_rv", None)
        if lister is not None:
            items, rv = lister(self.api_version, self.kind)
        else:
            items, rv = self.client.list(self.api_version, self.kind), None
        with self._lock:
            for o in items:
                self.store[self._key(o)] = o
            self.synced = True
        try:
            self._cancel = self.client.watch(self._on_event, self.api_version, self.kind, resource_version=rv)
        except TypeError:       # a client without resourceVersion support
            self._cancel = self.client.watch(self._on_event, self.api_version, self.kind)
        return self

    def stop(self):
        if self._cancel:
            self._cancel()

    def get(self, name: str, namespace: Optional[str]) -> Optional[dict]:
        with self._lock:
            o = self.store.get((namespace, name))
            if o is None and namespace is not None:       # cluster-scoped kind asked with a namespace
                o = self.store.get((None, name))
            return copy.deepcopy(o) if o is not None else None

    def list(self, namespace=None, label_selector=None, field_selector=None) -> List[dict]:
        with self._lock:
            items = [o for (ns, _), o in sorted(self.store.items(), key=lambda kv: (kv[0][0] or "", kv[0][1]))
                     if (namespace is None or ns == namespace or ns is None)]
            return [copy.deepcopy(o) for o in items
                    if labels_match(o.get("metadata", {}).get("labels"), label_selector)
                    and fields_match(o, field_selector)]


class CachedClient(Client):
    """Cache-backed reads for the kinds the manager watches; everything else is delegated."""

    def __init__(self, live: Client, informers: Dict[Tuple[str, str], Informer]):
        self.live = live
        self.informers = informers

    def _inf(self, api_version, kind) -> Optional[Informer]:
        inf = self.informers.get((split_api_version(api_version)[0], kind))
        return inf if inf is not None and inf.synced else None

    def get(self, api_version, kind, name, namespace=None):
        inf = self._inf(api_version, kind)
        if inf is None:
            return self.live.get(api_version, kind, name, namespace)
        o = inf.get(name, namespace)
        if o is None:
            raise NotFound(f'{kind} "{name}" not found')
        return o

    def list(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        inf = self._inf(api_version, kind)
        if inf is None:
            return self.live.list(api_version, kind, namespace, label_selector, field_selector)
        return inf.list(namespace, label_selector, field_selector)

    def create(self, obj, dry_run=False):
        return self.live.create(obj, dry_run)

    def update(self, obj, dry_run=False):
        return self.live.update(obj, dry_run)

    def update_status(self, obj):
        return self.live.update_status(obj)

    def patch(self, api_version, kind, name, namespace, patch, patch_type="merge", subresource=None):
        return self.live.patch(api_version, kind, name, namespace, patch, patch_type, subresource)

    def delete(self, api_version, kind, name, namespace=None, propagation="Background"):
        return self.live.delete(api_version, kind, name, namespace, propagation)

    def watch(self, fn, api_version=None, kind=None, resource_version=None):
        return self.live.watch(fn, api_version, kind, resource_version=resource_version)

    def __getattr__(self, name):          # server-specific extras of the live client
        return getattr(self.live, name)


class Manager:
    def __init__(self, client: Client, leader_election: bool = False, leader_election_id: str = "",
                 leader_election_namespace: str = "kubeflow", identity: Optional[str] = None,
                 metrics_registry=None, clock: Callable[[], float] = time.time, cache: bool = True):
        self.client = client
        self.controllers: Dict[str, Controller] = {}
        self.wq = WorkQueue()
        self.informers: Dict[Tuple[str, str], Informer] = {}
        self.cache = cache
        self._timers: List[Tuple[float, int, str, Request]] = []
        self._seq = 0
        self._cv = threading.Condition()
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._cancels: List[Callable] = []
        self.rate = RateLimiter()
        self.clock = clock
        self.leader_election = leader_election
        self.le_id = leader_election_id
        self.le_ns = leader_election_namespace
        self.identity = identity or f"mgr-{id(self):x}"
        self.is_leader = not leader_election
        self.metrics_registry = metrics_registry
        self.reconcile_errors = 0
        self.reconciles = 0
        self._http = None

    # --- wiring
    def informer(self, api_version: str, kind: str) -> Informer:
        """The shared informer of a kind (started on first use)."""
        key = (split_api_version(api_version)[0], kind)
        inf = self.informers.get(key)
        if inf is None:
            inf = Informer(self.client, api_version, kind)
            self.informers[key] = inf
            try:
                inf.start()
            except ApiError:
                inf.synced = False
            self._cancels.append(inf.stop)
        return inf

    def add(self, ctrl: Controller):
        self.controllers[ctrl.name] = ctrl
        for src in ctrl.sources():
            def handler(et, obj, src=src, cname=ctrl.name):
                if src.predicate is not None and not src.predicate(et, obj):
                    return
                for req in src.mapper(et, obj):
                    self.enqueue(cname, req)
            inf = self.informer(src.api_version, src.kind)
            inf.handlers.append(handler)
            # objects that existed before this controller joined the informer
            for obj in inf.list():
                handler("ADDED", obj)
        if self.cache and not isinstance(ctrl.client, CachedClient):
            ctrl.client = CachedClient(ctrl.client, self.informers)
        return self

    def enqueue(self, cname: str, req: Request, after: float = 0.0):
        with self._cv:
            if after > 0:
                self._seq += 1
                heapq.heappush(self._timers, (self.clock() + after, self._seq, cname, req))
            else:
                self.wq.add((cname, req))
            self._cv.notify()

    def _pop_due(self):
        now = self.clock()
        while self._timers and self._timers[0][0] <= now:
            _, _, c, r = heapq.heappop(self._timers)
            self.wq.add((c, r))

    def _process_one(self) -> bool:
        with self._cv:
            self._pop_due()
            item = self.wq.get()
            if item is None:
                return False
        cname, req = item
        try:
            return self._reconcile_one(cname, req)
        finally:
            with self._cv:
                self.wq.done(item)
                self._cv.notify()

    def _reconcile_one(self, cname, req) -> bool:
        ctrl = self.controllers[cname]
        self.reconciles += 1
        try:
            res = ctrl.reconcile(req) or Result()
            self.rate.forget((cname, req))
            if res.requeue_after > 0:
                self.enqueue(cname, req, res.requeue_after)
            elif res.requeue:
                self.enqueue(cname, req, self.rate.when((cname, req)))
        except Exception as e:  # error -> exponential back-off requeue
            self.reconcile_errors += 1
            level = logging.DEBUG if isinstance(e, ApiError) and e.code == 409 else logging.WARNING
            log.log(level, "reconcile %s %s failed: %s", cname, req, e)
            self.enqueue(cname, req, self.rate.when((cname, req)))
        return True

    def run_until_idle(self, max_iters: int = 10000, include_timers_within: float = 0.0) -> int:
        """Synchronously drain the queue (and timers due within the window). Tests only."""
        n = 0
        while n < max_iters:
            if self._process_one():
                n += 1
                continue
            with self._cv:
                due = [t for t in self._timers if t[0] <= self.clock() + include_timers_within]
                if not due:
                    break
                # pull the earliest due timer forward
                t = heapq.heappop(self._timers)
                self.wq.add((t[2], t[3]))
        return n

    def enqueue_all(self, cname: str, api_version: str, kind: str):
        for o in self.client.list(api_version, kind):
            self.enqueue(cname, Request(o["metadata"].get("namespace"), o["metadata"]["name"]))

    # --- leader election (Lease)
    def try_acquire_lease(self, lease_duration: float = 15.0) -> bool:
        if not self.leader_election:
            return True
        av, kind = "coordination.k8s.io/v1", "Lease"
        try:
            self.client.get("v1", "Namespace", self.le_ns)
        except ApiError:
            try:
                self.client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": self.le_ns}})
            except ApiError:
                pass
        now = self.clock()
        lease = self.client.get_or_none(av, kind, self.le_id, self.le_ns)
        spec = {"holderIdentity": self.identity, "leaseDurationSeconds": int(lease_duration),
                "renewTime": now_rfc3339(), "renewEpoch": now}
        try:
            if lease is None:
                self.client.create({"apiVersion": av, "kind": kind,
                                    "metadata": {"name": self.le_id, "namespace": self.le_ns}, "spec": spec})
                self.is_leader = True
            else:
                s = lease.get("spec", {})
                expired = now - float(s.get("renewEpoch", 0)) > float(s.get("leaseDurationSeconds", 15))
                if s.get("holderIdentity") in (self.identity, None, "") or expired:
                    lease["spec"] = spec
                    self.client.update(lease)
                    self.is_leader = True
                else:
                    self.is_leader = False
        except ApiError:
            self.is_leader = False
        return self.is_leader

    # --- threaded run
    def start(self, workers: int = 2, lease_renew: float = 5.0):
        def loop():
            while not self._stop.is_set():
                if not self.is_leader:
                    self._stop.wait(0.5)
                    continue
                if not self._process_one():
                    with self._cv:
                        wait = 0.5
                        if self._timers:
                            wait = max(0.0, min(wait, self._timers[0][0] - self.clock()))
                        self._cv.wait(wait)

        def lease_loop():
            while not self._stop.is_set():
                self.try_acquire_lease()
                self._stop.wait(lease_renew)

        if self.leader_election:
            t = threading.Thread(target=lease_loop, daemon=True)
            t.start()
            self._threads.append(t)
        for _ in range(workers):
            t = threading.Thread(target=loop, daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self):
        self._stop.set()
        with self._cv:
            self._cv.notify_all()
        for c in self._cancels:
            c()
        if self._http:
            self._http.shutdown()

    # --- probes + metrics endpoint
    def serve_probes(self, port: int = 0, host: str = "127.0.0.1"):
        mgr = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                if self.path in ("/healthz", "/readyz"):
                    body, ct = b"ok", "text/plain"
                elif self.path == "/metrics" and mgr.metrics_registry is not None:
                    from prometheus_client import CONTENT_TYPE_LATEST, generate_latest
                    body, ct = generate_latest(mgr.metrics_registry), CONTENT_TYPE_LATEST
                else:
                    self.send_response(404)
                    self.end_headers()
                    return
                self.send_response(200)
                self.send_header("Content-Type", ct)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self._http = ThreadingHTTPServer((host, port), H)
        threading.Thread(target=self._http.serve_forever, daemon=True).start()
        return self._http.server_address[1]


def get_env_default(name: str, default: str) -> str:
    import os
    v = os.environ.get(name, "")
    return v if v else default
