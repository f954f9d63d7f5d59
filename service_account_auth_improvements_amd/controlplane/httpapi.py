"""Kubernetes REST facade over the in-memory :class:`.apiserver.APIServer`.

Serves the standard paths (``/api/v1/...``, ``/apis/<group>/<version>/...``, namespaced
and cluster scoped, ``/status`` subresource, ``?watch=true`` chunked JSON event stream,
``labelSelector`` / ``fieldSelector`` / ``dryRun``) so that out-of-process components
(the C++ launcher, web apps run as separate processes, :class:`.client.RestClient`)
can talk to the local cluster exactly as they would to a real kube-apiserver.
"""
from __future__ import annotations

import json
import queue
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

from .apiserver import APIServer, ApiError


def _parse(path: str):
    """-> (group, version, namespace, plural, name, subresource)"""
    parts = [p for p in path.split("/") if p]
    if parts[:1] == ["api"]:
        g, v, rest = "", parts[1], parts[2:]
    elif parts[:1] == ["apis"]:
        g, v, rest = parts[1], parts[2], parts[3:]
    else:
        raise ApiError(404, "NotFound", path)
    ns = None
    if len(rest) >= 3 and rest[0] == "namespaces" and rest[2] not in ("status", "finalize"):
        ns, rest = rest[1], rest[2:]
    plural = rest[0] if rest else None
    name = rest[1] if len(rest) > 1 else None
    sub = rest[2] if len(rest) > 2 else None
    return g, v, ns, plural, name, sub


BOOKMARK_PERIOD = 5.0     # seconds between BOOKMARK events on an idle watch that asked for them


def make_handler(server: APIServer):
    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def _send(self, code, body):
            data = json.dumps(body).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def _body(self):
            n = int(self.headers.get("Content-Length") or 0)
            return json.loads(self.rfile.read(n).decode()) if n else None

        def _handle(self, method):
            u = urlparse(self.path)
            q = {k: v[0] for k, v in parse_qs(u.query).items()}
            try:
                if u.path in ("/healthz", "/readyz", "/livez"):
                    data = b"ok"
                    self.send_response(200)
                    self.send_header("Content-Length", "2")
                    self.end_headers()
                    self.wfile.write(data)
                    return
                g, v, ns, plural, name, sub = _parse(u.path)
                t = server.type_for_plural(g, plural)
                av = f"{g}/{v}" if g else v
                dry = q.get("dryRun") == "All"
                fv = q.get("fieldValidation")       # Strict | Warn | Ignore (unknown CRD fields)
                if method == "GET" and q.get("watch") in ("true", "1"):
                    return self._watch(av, t.kind, ns, q.get("resourceVersion"),
                                       q.get("allowWatchBookmarks") in ("true", "1"),
                                       float(q["timeoutSeconds"]) if q.get("timeoutSeconds") else None)
                if method == "GET" and name:
                    return self._send(200, server.get(av, t.kind, name, ns))
                if method == "GET":
                    items, rv = server.list_with_rv(av, t.kind, ns, q.get("labelSelector"), q.get("fieldSelector"))
                    return self._send(200, {"apiVersion": av, "kind": f"{t.kind}List", "items": items,
                                            "metadata": {"resourceVersion": rv}})
                if method == "POST" and sub == "binding" and t.kind == "Pod":
                    body = self._body() or {}
                    return self._send(201, server.bind_pod(ns, name, (body.get("target") or {}).get("name", "")))
                if method == "POST":
                    body = self._body()
                    body.setdefault("apiVersion", av)
                    body.setdefault("kind", t.kind)
                    if ns:
                        body.setdefault("metadata", {}).setdefault("namespace", ns)
                    return self._send(201, server.create(body, dry_run=dry, field_validation=fv))
                if method == "PUT":
                    body = self._body()
                    if sub == "status":
                        return self._send(200, server.update_status(body))
                    return self._send(200, server.update(body, dry_run=dry, field_validation=fv))
                if method == "PATCH":
                    ct = self.headers.get("Content-Type", "")
                    pt = "json" if "json-patch" in ct else "merge"
                    return self._send(200, server.patch(av, t.kind, name, ns, self._body(), pt, sub, dry,
                                                        field_validation=fv))
                if method == "DELETE":
                    body = self._body() or {}
                    return self._send(200, server.delete(av, t.kind, name, ns,
                                                         body.get("propagationPolicy", "Background")))
                raise ApiError(405, "MethodNotAllowed", method)
            except ApiError as e:
                self._send(e.code, e.status())
            except Exception as e:  # malformed request
                self._send(400, {"kind": "Status", "status": "Failure", "code": 400,
                                 "reason": "BadRequest", "message": str(e)})

        def _chunk(self, ev):
            data = (json.dumps(ev) + "\n").encode()
            self.wfile.write(f"{len(data):x}\r\n".encode() + data + b"\r\n")
            self.wfile.flush()

        def _watch(self, av, kind, ns, rv, bookmarks, timeout):
            qq: "queue.Queue" = queue.Queue()

            def fn(etype, obj):
                if ns is None or obj.get("metadata", {}).get("namespace") == ns:
                    qq.put({"type": etype, "object": obj})
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Transfer-Encoding", "chunked")
            self.end_headers()
            try:
                cancel = server.watch(fn, av, kind, resource_version=rv)
            except ApiError as e:       # 410 Expired: one ERROR event, then the stream ends
                try:
                    self._chunk({"type": "ERROR", "object": e.status()})
                    self.wfile.write(b"0\r\n\r\n")
                except (BrokenPipeError, ConnectionResetError):
                    pass
                return
            deadline = time.time() + timeout if timeout else None
            try:
                while deadline is None or time.time() < deadline:
                    wait = BOOKMARK_PERIOD if deadline is None else max(0.01, min(BOOKMARK_PERIOD, deadline - time.time()))
                    try:
                        ev = qq.get(timeout=wait)
                    except queue.Empty:
                        if bookmarks:
                            # The server assigns an RV and emits its event under its lock, so an
                            # RV read under that lock with this stream's queue empty is covered:
                            # every event up to it has been written to the client already.  A
                            # bookmark read outside the lock could claim an event not yet queued,
                            # and a client resuming from it would never see that event.
                            with server._lock:
                                brv = server.resource_version if qq.empty() else None
                            if brv is not None:
                                self._chunk({"type": "BOOKMARK", "object": {
                                    "apiVersion": av, "kind": kind,
                                    "metadata": {"resourceVersion": brv}}})
                        continue
                    self._chunk(ev)
                # timeoutSeconds reached: flush what is queued, then end cleanly (anything
                # emitted after this is replayed when the client resumes from its last RV)
                cancel()
                while True:
                    try:
                        self._chunk(qq.get_nowait())
                    except queue.Empty:
                        break
                self.wfile.write(b"0\r\n\r\n")
            except (BrokenPipeError, ConnectionResetError):
                pass
            finally:
                cancel()

        def do_GET(self):
            self._handle("GET")

        def do_POST(self):
            self._handle("POST")

        def do_PUT(self):
            self._handle("PUT")

        def do_PATCH(self):
            self._handle("PATCH")

        def do_DELETE(self):
            self._handle("DELETE")

    return H


class APIServerHTTP:
    """Run the REST facade on 127.0.0.1:<port> in a daemon thread."""

    def __init__(self, server: APIServer, host: str = "127.0.0.1", port: int = 0):
        self.httpd = ThreadingHTTPServer((host, port), make_handler(server))
        self.httpd.daemon_threads = True
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    @property
    def url(self):
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self):
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()
