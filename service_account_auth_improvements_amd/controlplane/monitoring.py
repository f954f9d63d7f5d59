"""G2c / G3a: request counters and heartbeat shared by the profile controller and KFAM
(reference: profile-controller/controllers/monitoring.go:25-77, access-management/kfam/
monitoring.go:24-77).  Metric names and label keys are kept byte-compatible:
``request_kf{component,kind}``, ``request_kf_failure{component,kind,severity}``,
``service_heartbeat{component,severity}`` (incremented every 10 s)."""
from __future__ import annotations

import logging
import threading
import time

SEVERITY_MINOR, SEVERITY_MAJOR, SEVERITY_CRITICAL = "minor", "major", "critical"
MAX_TAG_LEN = 30
log = logging.getLogger("monitoring")


class RequestMetrics:
    def __init__(self, component: str, registry=None, extra_labels=(), heartbeat_period: float = 10.0,
                 start_heartbeat: bool = False):
        from prometheus_client import CollectorRegistry, Counter
        self.component = component
        self.registry = registry or CollectorRegistry()
        self.extra = tuple(extra_labels)
        self.requests = Counter("request_kf", "Number of request_counter", ["component", "kind", *self.extra],
                                registry=self.registry)
        self.failures = Counter("request_kf_failure", "Number of request_failure_counter",
                                ["component", "kind", *self.extra, "severity"], registry=self.registry)
        self.heartbeat = Counter("service_heartbeat", "Heartbeat signal every 10 seconds indicating pods are alive.",
                                 ["component", "severity"], registry=self.registry)
        self._stop = threading.Event()
        self.period = heartbeat_period
        if start_heartbeat:
            threading.Thread(target=self._beat, daemon=True).start()

    def _beat(self):
        while not self._stop.wait(self.period):
            self.heartbeat.labels(self.component, SEVERITY_CRITICAL).inc()

    def stop(self):
        self._stop.set()

    def inc_request(self, kind: str, *extra):
        self.requests.labels(self.component, kind[:MAX_TAG_LEN], *extra).inc()

    def inc_error(self, kind: str, severity: str, *extra):
        log.error("Failed request with kind: %s", kind)
        self.failures.labels(self.component, kind[:MAX_TAG_LEN], *extra, severity).inc()
