"""Watch / informer semantics of the control plane (kube-apiserver resourceVersion contract):
event history replay from an RV, 410 Gone on an expired RV, list RVs, the REST client's
list-then-watch (no event lost between watch() returning and the stream attaching), its re-list
on 410 with synthetic DELETED events, bookmarks, the O(1) client-go work queue and the Manager's
cache-backed reads."""
import json
import threading
import time
import urllib.request

import pytest

from service_account_auth_improvements_amd.controlplane.apiserver import APIServer, ApiError
from service_account_auth_improvements_amd.controlplane.client import InMemoryClient, RestClient
from service_account_auth_improvements_amd.controlplane.httpapi import APIServerHTTP
from service_account_auth_improvements_amd.controlplane.runtime import (CachedClient, Controller, Manager,
                                                                        Request, Result, WorkQueue, for_kind)


def _cm(name, ns="default", data=None):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": ns},
            "data": data or {"k": name}}


def _wait(fn, timeout=10.0):
    end = time.time() + timeout
    while time.time() < end:
        if fn():
            return True
        time.sleep(0.01)
    return False


def test_watch_from_resource_version_replays_history():
    s = APIServer()
    s.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "default"}})
    s.create(_cm("a"))
    _, rv = s.list_with_rv("v1", "ConfigMap")
    s.create(_cm("b"))
    s.delete("v1", "ConfigMap", "a", "default")
    got = []
    cancel = s.watch(lambda et, o: got.append((et, o["metadata"]["name"], int(o["metadata"]["resourceVersion"]))),
                     "v1", "ConfigMap", resource_version=rv)
    s.create(_cm("c"))
    cancel()
    assert [(et, n) for et, n, _ in got] == [("ADDED", "b"), ("DELETED", "a"), ("ADDED", "c")]
    rvs = [r for _, _, r in got]
    assert rvs == sorted(rvs) and len(set(rvs)) == 3 and rvs[0] > int(rv)   # the deletion has an RV of its own


def test_expired_resource_version_is_gone():
    s = APIServer(history=8)
    s.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "default"}})
    _, rv = s.list_with_rv("v1", "ConfigMap")
    for i in range(20):
        s.create(_cm(f"x{i}"))
    with pytest.raises(ApiError) as ei:
        s.watch(lambda *a: None, "v1", "ConfigMap", resource_version=rv)
    assert ei.value.code == 410
    # a recent RV is still served
    _, rv2 = s.list_with_rv("v1", "ConfigMap")
    s.watch(lambda *a: None, "v1", "ConfigMap", resource_version=rv2)()


@pytest.fixture
def rest():
    s = APIServer(history=16)
    s.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "default"}})
    h = APIServerHTTP(s).start()
    yield s, RestClient(h.url)
    h.stop()


def test_rest_list_reports_resource_version(rest):
    s, c = rest
    items, rv = c.list_with_rv("v1", "ConfigMap")
    assert items == [] and rv == s.resource_version


def test_delete_right_after_watch_returns_is_never_missed(rest):
    s, c = rest
    for i in range(25):
        c.create(_cm(f"o{i}"))
        seen = []
        stop = c.watch(lambda et, o, seen=seen: seen.append((et, o["metadata"]["name"])), "v1", "ConfigMap")
        c.delete("v1", "ConfigMap", f"o{i}", "default")       # before the stream is attached, often
        assert _wait(lambda: ("DELETED", f"o{i}") in seen), (i, seen)
        stop()


def test_rest_watch_relists_on_410_and_synthesises_deletes(rest, monkeypatch):
    """A watcher cut off long enough for its RV to expire re-lists on the 410 and reports what it
    missed: the objects created meanwhile (ADDED) and the one deleted meanwhile (DELETED)."""
    s, c = rest
    monkeypatch.setattr(RestClient, "WATCH_TIMEOUT", 0.2)     # short streams: reconnects happen often
    for n in ("a", "b"):
        c.create(_cm(n))
    seen = []
    down = {"v": False}
    orig = c._req

    def flaky(method, path, body=None, params=None, **kw):
        if params and params.get("watch") and down["v"]:
            raise ConnectionError("partition")
        return orig(method, path, body, params, **kw)
    c._req = flaky
    stop = c.watch(lambda et, o: seen.append((et, o["metadata"]["name"])), "v1", "ConfigMap")
    c.create(_cm("c"))
    assert _wait(lambda: ("ADDED", "c") in seen)
    down["v"] = True
    time.sleep(0.6)                          # the live stream has ended; reconnects fail
    s.delete("v1", "ConfigMap", "b", "default")
    for i in range(30):                      # roll the 16-event history past the client's RV
        s.create(_cm(f"m{i}"))
    down["v"] = False
    assert _wait(lambda: ("DELETED", "b") in seen), seen
    assert _wait(lambda: sum(1 for et, n in seen if et == "ADDED" and n.startswith("m")) == 30), seen
    stop()


def test_watch_bookmarks_and_timeout(rest, monkeypatch):
    from service_account_auth_improvements_amd.controlplane import httpapi
    monkeypatch.setattr(httpapi, "BOOKMARK_PERIOD", 0.05)
    s, c = rest
    url = c.server + "/api/v1/configmaps?watch=true&allowWatchBookmarks=true&timeoutSeconds=0.3&resourceVersion=" + \
        s.resource_version
    with urllib.request.urlopen(url, timeout=5) as r:
        lines = [json.loads(l) for l in r.read().decode().splitlines() if l.strip()]
    assert lines and all(e["type"] == "BOOKMARK" for e in lines)
    assert lines[-1]["object"]["metadata"]["resourceVersion"] == s.resource_version


def test_bookmark_never_covers_an_unsent_event(monkeypatch):
    """Writers race short watch streams that bookmark constantly and end at timeoutSeconds: the
    client resumes from its last BOOKMARK / event RV each time, so a bookmark whose RV covers an
    event not yet written to the stream would lose that event for good.  The history
    is large enough that no resume hits 410 (whose re-list would mask a loss)."""
    from service_account_auth_improvements_amd.controlplane import httpapi
    monkeypatch.setattr(httpapi, "BOOKMARK_PERIOD", 0.002)
    monkeypatch.setattr(RestClient, "WATCH_TIMEOUT", 0.05)
    s = APIServer(history=100000)
    s.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "default"}})
    emit = s._emit

    def slow_emit(*a, **kw):        # widen the window between RV assignment and the event
        time.sleep(0.01)
        return emit(*a, **kw)
    s._emit = slow_emit
    h = APIServerHTTP(s).start()
    try:
        c = RestClient(h.url)
        seen, lk = set(), threading.Lock()

        def on(et, o):
            if et == "ADDED":
                with lk:
                    seen.add(o["metadata"]["name"])
        stop = c.watch(on, "v1", "ConfigMap")

        def writer(k):
            for i in range(40):
                s.create(_cm(f"w{k}-{i}"))
        ws = [threading.Thread(target=writer, args=(k,)) for k in range(3)]
        for w in ws:
            w.start()
        for w in ws:
            w.join()
        ok = _wait(lambda: len(seen) == 120, timeout=20)
        stop()
        assert ok, sorted({f"w{k}-{i}" for k in range(3) for i in range(40)} - seen)[:10]
    finally:
        h.stop()


def test_workqueue_is_fifo_dedup_and_never_concurrent():
    q = WorkQueue()
    for k in ("a", "b", "a", "c"):
        q.add(k)
    assert len(q) == 3
    a = q.get()
    assert a == "a"
    q.add("a")                 # re-added while in flight: dirty, not queued
    assert q.get() == "b" and q.get() == "c" and q.get() is None
    q.done("a")                # finished: runs once more
    assert q.get() == "a" and q.get() is None


def test_workqueue_is_constant_time():
    q = WorkQueue()
    t0 = time.perf_counter()
    for i in range(200000):
        q.add(i)
    while (it := q.get()) is not None:
        q.done(it)
    assert time.perf_counter() - t0 < 5.0


class _Counter(Controller):
    name = "counter"

    def __init__(self, client):
        super().__init__(client)
        self.seen = []

    def sources(self):
        return [for_kind("v1", "ConfigMap")]

    def reconcile(self, req: Request) -> Result:
        cm = self.client.get("v1", "ConfigMap", req.name, req.namespace)
        self.seen.append(cm["data"]["k"])
        return Result()


def test_manager_reads_from_informer_cache():
    s = APIServer()
    s.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "default"}})
    s.create(_cm("pre"))
    live = InMemoryClient(s)
    calls = {"get": 0}
    orig = live.get

    def counting_get(*a, **k):
        calls["get"] += 1
        return orig(*a, **k)
    live.get = counting_get
    mgr = Manager(live)
    ctrl = _Counter(live)
    mgr.add(ctrl)
    assert isinstance(ctrl.client, CachedClient)
    live.create(_cm("post"))
    mgr.run_until_idle()
    assert sorted(ctrl.seen) == ["post", "pre"]
    assert calls["get"] == 0, "ConfigMap reads must come from the informer store"
    # the store follows updates and deletes
    live.update({**live.get("v1", "ConfigMap", "post", "default"), "data": {"k": "post2"}})
    mgr.run_until_idle()
    assert ctrl.seen[-1] == "post2"
    live.delete("v1", "ConfigMap", "pre", "default")
    assert ctrl.client.get_or_none("v1", "ConfigMap", "pre", "default") is None
    mgr.stop()
