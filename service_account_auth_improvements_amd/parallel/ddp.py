"""Data-parallel gradient reduction over RCCL (C1 in SURVEY.md §2.8).

Buckets are fixed-size slices of the flat bf16 gradient buffer (runtime/flat.py).  The
model registers its parameters in reverse execution order, so as backward proceeds the
finished gradients form a growing prefix of the buffer; every time the prefix crosses a
bucket boundary the bucket's collective is launched immediately (async, on the process
group's own stream, ordered after the producing GEMMs by the PG's stream wait) and it
overlaps the rest of the backward pass.

Two modes:
  * ``allreduce`` (classic DDP): every rank ends with the full summed gradient and runs
    the full optimizer.
  * ``reduce_scatter`` (ZeRO-1): every rank receives the summed gradient of its own 1/dp
    shard of each bucket, updates only that shard's fp32 master/moments, and the updated
    bf16 parameters are all-gathered bucket by bucket.  Same bytes on the wire as an
    all-reduce (RS + AG = AR) but 1/dp of the optimizer traffic and state per GPU.

Sizing for xGMI: a ring collective is bound by one ~153 GB/s link per hop, so per-call
latency matters little at these sizes and large buckets (default 256 MB) minimise launch
count; the whole 8B gradient is 16 GB -> ~64 buckets.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..runtime.flat import FlatGroup


class Bucket:
    __slots__ = ("group", "lo", "hi", "work", "launched", "staged")

    def __init__(self, group: FlatGroup, lo: int, hi: int):
        self.group, self.lo, self.hi = group, lo, hi
        self.work = None
        self.launched = False
        self.staged = None      # (shard view, separate output) when the backend must not alias


class GradReducer:
    def __init__(self, groups: List[FlatGroup], dp_group=None, dp_size: int = 1,
                 bucket_bytes: int = 256 << 20, mode: str = "allreduce"):
        assert mode in ("allreduce", "reduce_scatter")
        self.dp_group, self.dp = dp_group, dp_size
        self.mode = mode
        self.groups = groups
        self.buckets: dict = {}
        for g in groups:
            elems = max(bucket_bytes // g.grads.element_size(), 1)
            if mode == "reduce_scatter":
                # bucket length must split evenly over dp ranks (g.numel is padded to dp*ALIGN)
                quant = dp_size * 64
                elems = max(quant, elems // quant * quant)
            bl, lo = [], 0
            while lo < g.numel:
                hi = min(g.numel, lo + elems)
                bl.append(Bucket(g, lo, hi))
                lo = hi
            self.buckets[g.name] = bl
        self.enabled = dp_size > 1
        self._pending: List[Bucket] = []
        self._gathers: dict = {}          # (group name, bucket index) -> async all-gather work

    # -- shard geometry (reduce_scatter mode): rank r owns [lo + r*n/dp, lo + (r+1)*n/dp) of each bucket
    def shard_ranges(self, group: FlatGroup, rank: int) -> List[Tuple[int, int]]:
        out = []
        for b in self.buckets[group.name]:
            n = (b.hi - b.lo) // self.dp
            out.append((b.lo + rank * n, b.lo + (rank + 1) * n))
        return out

    def start_step(self):
        for bl in self.buckets.values():
            for b in bl:
                b.work, b.launched = None, False
        self._pending = []

    def _launch(self, b: Bucket):
        if b.launched:
            return
        b.launched = True
        if not self.enabled:
            return
        x = b.group.grads[b.lo:b.hi]
        if self.mode == "allreduce":
            b.work = dist.all_reduce(x, group=self.dp_group, async_op=True)
        else:
            n = (b.hi - b.lo) // self.dp
            r = dist.get_rank(self.dp_group) if self.dp_group is not None else dist.get_rank()
            out = x[r * n:(r + 1) * n]
            if x.is_cuda and dist.get_backend(self.dp_group) == "gloo":
                # in-place reduce-scatter (output = input + rank * n) is an RCCL/NCCL contract;
                # the gloo rehearsal backend gets a separate output, copied back in finish()
                b.staged = (out, torch.empty_like(out))
                out = b.staged[1]
            b.work = dist.reduce_scatter_tensor(out, x, group=self.dp_group, async_op=True)
        self._pending.append(b)

    def grad_ready(self, group: FlatGroup, end_offset: int):
        """Model callback: every gradient of ``group`` below ``end_offset`` is final."""
        for b in self.buckets[group.name]:
            if b.launched:
                continue
            if b.hi <= end_offset:
                self._launch(b)
            else:
                break

    def finish(self):
        """Launch whatever is left and wait for every collective (stream-ordered wait)."""
        for bl in self.buckets.values():
            for b in bl:
                self._launch(b)
        for b in self._pending:
            if b.work is not None:
                b.work.wait()
            if b.staged is not None:
                b.staged[0].copy_(b.staged[1])
                b.staged = None
        self._pending = []

    def all_gather_params(self, overlap: bool = False):
        """ZeRO-1: after the sharded update, gather every bucket's bf16 params.

        ``overlap=True`` only LAUNCHES the gathers -- in forward order (the end of each flat
        buffer holds the first layers, see runtime/flat.py) -- and returns; the model's
        ``param_wait`` hook makes the compute stream wait on a bucket just before the next
        forward first reads it (:meth:`wait_params`), so the gather hides behind the
        previous layers' compute instead of sitting between optimizer and forward."""
        if not self.enabled or self.mode != "reduce_scatter":
            return
        r = dist.get_rank(self.dp_group) if self.dp_group is not None else dist.get_rank()
        # small groups (norm weights) first: every layer reads one of them, and the gathers
        # complete in launch order on the communicator's stream
        for name, bl in sorted(self.buckets.items(), key=lambda kv: kv[1][-1].hi if kv[1] else 0):
            for idx in reversed(range(len(bl))):
                b = bl[idx]
                x = b.group.params[b.lo:b.hi]
                n = (b.hi - b.lo) // self.dp
                self._gathers[(name, idx)] = dist.all_gather_into_tensor(
                    x, x[r * n:(r + 1) * n].clone(), group=self.dp_group, async_op=True)
        if not overlap:
            self.wait_all_params()

    def wait_params(self, group: FlatGroup, lo: int, hi: int):
        """Stream-wait for the pending gathers of every bucket overlapping [lo, hi)."""
        if not self._gathers:
            return
        for idx, b in enumerate(self.buckets[group.name]):
            if b.hi > lo and b.lo < hi:
                w = self._gathers.pop((group.name, idx), None)
                if w is not None:
                    w.wait()

    def wait_all_params(self):
        for w in self._gathers.values():
            w.wait()
        self._gathers = {}

    def broadcast_params(self, src_global_rank: int = 0):
        """C2: make every DP replica start from identical weights."""
        if not self.enabled:
            return
        for g in self.groups:
            dist.broadcast(g.params, src=src_global_rank, group=self.dp_group)
