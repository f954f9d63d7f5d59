"""Prometheus ``/metrics`` for the training worker (SURVEY.md §5 "Metrics / logging /
observability": tokens/s, step time, HBM use, collective bandwidth).

The reference serves Prometheus metrics from every binary it ships -- the notebook controller's
``notebook_running`` / ``notebook_create_total`` family
(/root/reference/components/notebook-controller/pkg/metrics/metrics.go:13-99, served from
main.go:64).  The PyTorchJob worker is this framework's data-plane binary and gets the same
treatment: rank 0 (every rank with ``KFAMD_METRICS_ALL_RANKS=1``, on ``port + LOCAL_RANK``)
serves

  train_steps_total / train_tokens_total                        counters
  train_step_seconds / train_tokens_per_second / train_loss      gauges (last step)
  hip_memory_allocated_bytes / hip_memory_reserved_bytes /
  hip_memory_peak_allocated_bytes                                gauges (the HIP caching allocator)
  train_collective_{calls,bytes,seconds}_total{op}               counters (parallel/ddp.CollectiveStats)
  train_collective_bus_bandwidth_bytes_per_second{op}           gauge: cumulative bytes x bus factor / seconds
  train_checkpoint_last_step / train_checkpoint_save_seconds    gauges (runtime/checkpoint.PeriodicCheckpointer)

Every value is fed by the worker loop ONE STEP LATE from data that is already on the host
(the previous step's end event, its pinned loss copy): nothing here synchronises the device.
The port comes from ``KFAMD_METRICS_PORT``; the PyTorchJob operator sets it from the job's
``kfamd.io/metrics-port`` annotation and adds the ``prometheus.io/*`` scrape annotations to the
pods (controlplane/training.py).
"""
from __future__ import annotations

import os
from typing import Optional


class TrainMetrics:
    def __init__(self, port: int, addr: str = "0.0.0.0", rank: int = 0, registry=None):
        from prometheus_client import CollectorRegistry, Counter, Gauge
        self.registry = registry or CollectorRegistry()
        r = self.registry
        lab = ["rank"]
        self.rank = str(rank)
        self.steps = Counter("train_steps", "Optimizer steps completed", lab, registry=r)
        self.tokens = Counter("train_tokens", "Tokens trained on by this rank's replica", lab, registry=r)
        self.step_s = Gauge("train_step_seconds", "Device time of the last step (end event to end event)", lab,
                            registry=r)
        self.tps = Gauge("train_tokens_per_second", "Tokens per second of the last step (this rank's replica)",
                         lab, registry=r)
        self.loss = Gauge("train_loss", "Loss of the last step", lab, registry=r)
        self.mem_alloc = Gauge("hip_memory_allocated_bytes", "HBM held by live tensors", lab, registry=r)
        self.mem_res = Gauge("hip_memory_reserved_bytes", "HBM reserved by the caching allocator", lab, registry=r)
        self.mem_peak = Gauge("hip_memory_peak_allocated_bytes", "Peak HBM held by live tensors", lab, registry=r)
        cl = ["rank", "op"]
        self.c_calls = Counter("train_collective_calls", "DP collectives completed", cl, registry=r)
        self.c_bytes = Counter("train_collective_bytes", "Bytes handed to DP collectives", cl, registry=r)
        self.c_secs = Counter("train_collective_seconds", "Time inside timed DP collectives", cl, registry=r)
        self.c_bus = Gauge("train_collective_bus_bandwidth_bytes_per_second",
                           "Bus bandwidth of the DP collectives (cumulative; nccl-tests bus factor)", cl, registry=r)
        self.ck_step = Gauge("train_checkpoint_last_step", "Step of the last published checkpoint", lab, registry=r)
        self.ck_secs = Gauge("train_checkpoint_save_seconds", "Wall time of the last checkpoint write", lab,
                             registry=r)
        self._seen = {}              # op -> [calls, bytes, seconds, timed bytes] already exported
        self._server = None
        self.port = None
        if port is not None and port >= 0:
            from prometheus_client import start_http_server
            res = start_http_server(port, addr=addr, registry=r)
            self._server = res[0] if isinstance(res, tuple) else None
            self.port = self._server.server_port if self._server is not None else port

    def observe_step(self, seconds: Optional[float], tokens: int, loss: Optional[float]):
        self.steps.labels(self.rank).inc()
        self.tokens.labels(self.rank).inc(tokens)
        if seconds is not None and seconds > 0:
            self.step_s.labels(self.rank).set(seconds)
            self.tps.labels(self.rank).set(tokens / seconds)
        if loss is not None:
            self.loss.labels(self.rank).set(loss)

    def observe_memory(self, device):
        import torch
        if getattr(device, "type", "cpu") != "cuda":
            return
        self.mem_alloc.labels(self.rank).set(torch.cuda.memory_allocated(device))
        self.mem_res.labels(self.rank).set(torch.cuda.memory_reserved(device))
        self.mem_peak.labels(self.rank).set(torch.cuda.max_memory_allocated(device))

    def observe_collectives(self, stats):
        if stats is None:
            return
        stats.harvest()
        for op, (calls, nbytes, secs, timed_bytes) in stats.totals.items():
            seen = self._seen.setdefault(op, [0, 0, 0.0, 0])
            self.c_calls.labels(self.rank, op).inc(calls - seen[0])
            self.c_bytes.labels(self.rank, op).inc(nbytes - seen[1])
            self.c_secs.labels(self.rank, op).inc(max(0.0, secs - seen[2]))
            self._seen[op] = [calls, nbytes, secs, timed_bytes]
            if secs > 0:
                self.c_bus.labels(self.rank, op).set(timed_bytes * stats.bus_factor(op) / secs)

    def observe_checkpoint(self, step: int, seconds: float):
        self.ck_step.labels(self.rank).set(step)
        self.ck_secs.labels(self.rank).set(seconds)

    def close(self):
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None


def from_env(rank: int, local_rank: int) -> Optional[TrainMetrics]:
    """The worker's metrics endpoint, or None: ``KFAMD_METRICS_PORT`` unset/empty means off; port
    0 picks a free port (tests); rank 0 serves unless ``KFAMD_METRICS_ALL_RANKS=1``."""
    port = os.environ.get("KFAMD_METRICS_PORT", "")
    if port == "":
        return None
    all_ranks = os.environ.get("KFAMD_METRICS_ALL_RANKS", "0") == "1"
    if rank != 0 and not all_ranks:
        return None
    p = int(port)
    if p > 0 and all_ranks:
        p += local_rank
    return TrainMetrics(p, addr=os.environ.get("KFAMD_METRICS_ADDR", "0.0.0.0"), rank=rank)
