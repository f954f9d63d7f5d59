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

Reduction precision (``reduce_dtype``):
  * ``bf16``: the bucket is reduced in bf16 by RCCL (a ring rounds every partial sum:
    N-1 bf16 roundings per element at N ranks).
  * ``fp32`` (default for N > 1): no partial sum is ever rounded.
      - ZeRO-1: each bucket moves as an ALL-TO-ALL of its bf16 shards (same bytes per GPU
        as a bf16 reduce-scatter; on the fully connected xGMI mesh each shard rides its own
        point-to-point link) and the N received shards are summed in fp32 by a HIP kernel
        (ops/csrc/grad_reduce.hip) into an fp32 gradient shard that AdamW reads directly.
      - all-reduce DDP: the bucket is staged into an fp32 buffer and all-reduced in fp32
        (2x the wire bytes; the ZeRO-1 path is the default for N > 1).
      - grad_accum > 1: micro-batches accumulate in an fp32 main-gradient buffer instead of
        bf16 beta=1 GEMM accumulation; the last micro-batch is folded in (one rounding)
        right before its bucket is sent.

Sizing for xGMI: a ring collective is bound by one ~153 GB/s link per hop, so per-call
latency matters little at these sizes and large buckets (default 256 MB) minimise launch
count; the whole 8B gradient is 16 GB -> ~64 buckets.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops
from ..runtime import progress
from ..runtime.flat import FlatGroup


class CollectiveStats:
    """Counts, bytes and seconds of the DP collectives, per op (``all_to_all``, ``all_reduce``,
    ``reduce_scatter``, ``all_gather``) -- the training worker's ``/metrics`` series
    (runtime/metrics.py).  Bytes are counted at launch on the host.  Seconds come from the
    communicator's own start/end events (``Work._get_duration``; RCCL records them when
    ``TORCH_NCCL_ENABLE_TIMING=1``, which the worker sets when metrics are on), or -- for a
    backend whose ``wait()`` blocks the host (gloo) -- from launch to the return of ``wait()``.
    Nothing here blocks: :meth:`harvest` folds in only collectives that already finished, so the
    worker calls it once per step and reads the totals one step late."""

    # bus-bandwidth factor per op at n ranks (the nccl-tests convention: bytes each link carries)
    _BUS = {"all_reduce": lambda n: 2.0 * (n - 1) / n}

    def __init__(self, world: int, host_timed: bool):
        self.world = max(1, world)
        self.host_timed = host_timed
        self.totals: Dict[str, List[float]] = {}     # op -> [count, bytes, timed seconds, timed bytes]
        self._open: Dict[int, list] = {}             # id(work) -> [op, bytes, work, t_launch, t_waited]

    def launched(self, op: str, nbytes: int, work):
        if work is not None:
            self._open[id(work)] = [op, int(nbytes), work, time.perf_counter(), None]

    def waited(self, work):
        rec = self._open.get(id(work))
        if rec is not None and rec[4] is None:
            rec[4] = time.perf_counter()

    def bus_factor(self, op: str) -> float:
        n = self.world
        return self._BUS.get(op, lambda n: (n - 1) / n)(n)

    def harvest(self):
        for key in list(self._open):
            op, nb, w, t0, t1 = self._open[key]
            try:
                if not w.is_completed():
                    continue
            except RuntimeError:
                continue
            secs = None
            try:
                ms = w._get_duration()          # the communicator's own event pair
                if ms is not None and ms >= 0:
                    secs = ms / 1e3
            except Exception:                   # noqa: BLE001 -- timing off / not supported
                pass
            if secs is None and self.host_timed and t1 is not None:
                secs = t1 - t0
            tot = self.totals.setdefault(op, [0, 0, 0.0, 0])
            tot[0] += 1
            tot[1] += nb
            if secs is not None:
                tot[2] += secs
                tot[3] += nb
            del self._open[key]


class Bucket:
    __slots__ = ("group", "lo", "hi", "idx", "work", "launched", "staged", "recv")

    def __init__(self, group: FlatGroup, lo: int, hi: int, idx: int):
        self.group, self.lo, self.hi, self.idx = group, lo, hi, idx
        self.work = None
        self.launched = False
        self.staged = None      # (shard view, separate output) when the backend must not alias
        self.recv = None        # fp32 ZeRO-1: the bucket's received bf16 shards [dp * n]


class GradReducer:
    def __init__(self, groups: List[FlatGroup], dp_group=None, dp_size: int = 1,
                 bucket_bytes: int = 256 << 20, mode: str = "allreduce",
                 reduce_dtype: str = "bf16", grad_accum: int = 1, force_collectives: bool = False):
        """``force_collectives`` runs the DP collectives even at dp_size 1 (a one-rank RCCL
        group exercises the exact call sequence on a one-GPU box)."""
        assert mode in ("allreduce", "reduce_scatter")
        assert reduce_dtype in ("bf16", "fp32"), reduce_dtype
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
                bl.append(Bucket(g, lo, hi, len(bl)))
                lo = hi
            self.buckets[g.name] = bl
        self.enabled = dp_size > 1 or force_collectives
        self.fp32 = reduce_dtype == "fp32"
        self.reduce_dtype = reduce_dtype
        self.grad_accum = grad_accum
        self._pending: List[Bucket] = []
        self._gathers: dict = {}          # (group name, bucket index) -> async all-gather work
        # fp32 buffers: main[g] = full fp32 gradient (micro-batch accumulator and/or the
        # all-reduce staging buffer); out32[g] = this rank's reduced fp32 shards (ZeRO-1),
        # bucket i's shard at out32[g][off32[g][i] : + n_i]
        self.main: dict = {}
        self.out32: dict = {}
        self.off32: dict = {}
        self.a2a = self.fp32 and self.enabled and mode == "reduce_scatter"
        self._accumulated = False     # accumulate_micro ran in this step
        self.stats: Optional[CollectiveStats] = None   # set by the worker when /metrics is on
        # one-GPU stand-in for the N > 1 collectives' CU / HBM footprint (tools/dp8_overlap_proxy.py):
        # called at every bucket launch, at finish() and at the parameter gather
        self.traffic_proxy = None
        if self.fp32:
            for g in groups:
                dev = g.grads.device
                if grad_accum > 1 or (self.enabled and mode == "allreduce"):
                    self.main[g.name] = torch.zeros(g.numel, device=dev, dtype=torch.float32)
                if self.a2a:
                    offs, tot = [], 0
                    for b in self.buckets[g.name]:
                        offs.append(tot)
                        tot += (b.hi - b.lo) // self.dp
                    self.off32[g.name] = offs
                    self.out32[g.name] = torch.zeros(tot, device=dev, dtype=torch.float32)

    @property
    def fp32_accumulation(self) -> bool:
        """True when micro-batch gradients accumulate in the fp32 main buffer (the model
        then writes each micro-batch's gradients fresh, ``accumulate=False``)."""
        return self.fp32 and self.grad_accum > 1

    def accumulate_micro(self, first: bool, groups: Optional[List[FlatGroup]] = None):
        """After a NON-final micro-batch's backward: main (=|+=) grads, in fp32 (``groups``:
        only those, e.g. the one pipeline chunk whose backward just ran)."""
        if not self.fp32_accumulation:
            return
        self._accumulated = True
        for g in (self.groups if groups is None else groups):
            ops.grad_accum_(self.main[g.name], g.grads, ops.GRAD_SET if first else ops.GRAD_ADD)

    def grad_view(self, group: FlatGroup, lo: int, hi: int) -> torch.Tensor:
        """The optimizer's gradient operand for flat range [lo, hi) of ``group``: the reduced
        fp32 shard (fp32 ZeRO-1), the fp32 main buffer (fp32 all-reduce / accumulation), or
        the bf16 flat gradients."""
        if self.a2a:
            for b in self.buckets[group.name]:
                n = (b.hi - b.lo) // self.dp
                r0 = b.lo + self._rank() * n
                if r0 <= lo and hi <= r0 + n:
                    off = self.off32[group.name][b.idx] + (lo - r0)
                    return self.out32[group.name][off:off + (hi - lo)]
            raise ValueError(f"[{lo}, {hi}) is not inside one of this rank's shards")
        if group.name in self.main:
            return self.main[group.name][lo:hi]
        return group.grads[lo:hi]

    def _rank(self) -> int:
        if not dist.is_initialized():
            return 0
        return dist.get_rank(self.dp_group) if self.dp_group is not None else dist.get_rank()

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
        self._accumulated = False

    def _launch(self, b: Bucket):
        if b.launched:
            return
        b.launched = True
        x = b.group.grads[b.lo:b.hi]
        main = self.main.get(b.group.name)
        if main is not None:
            m = main[b.lo:b.hi]
            if self._accumulated:
                # earlier micro-batches sit in main: fold the last one in -- one rounding
                # before an all-to-all send, none when the fp32 buffer itself is reduced /
                # read by the optimizer
                ops.grad_accum_(m, x, ops.GRAD_FOLD if self.a2a else ops.GRAD_ADD)
            elif not self.a2a:
                ops.grad_accum_(m, x, ops.GRAD_SET)       # fp32 all-reduce / optimizer operand
        if self.traffic_proxy is not None:
            self.traffic_proxy.on_bucket(x.numel() * x.element_size())
        if not self.enabled:
            return
        self._drain_completed()
        progress.mark("dp collective", f"{'all_to_all' if self.a2a else self.mode} {b.group.name}[{b.idx}]")
        if self.a2a:
            b.recv = torch.empty_like(x)
            b.work = dist.all_to_all_single(b.recv, x, group=self.dp_group, async_op=True)
            self._note("all_to_all", x, b.work)
        elif self.mode == "allreduce":
            t = main[b.lo:b.hi] if self.fp32 else x
            b.work = dist.all_reduce(t, group=self.dp_group, async_op=True)
            self._note("all_reduce", t, b.work)
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
            self._note("reduce_scatter", x, b.work)
        self._pending.append(b)

    def _note(self, op: str, t: torch.Tensor, work):
        if self.stats is not None:
            self.stats.launched(op, t.numel() * t.element_size(), work)

    def _waited(self, work):
        if self.stats is not None:
            self.stats.waited(work)

    def grad_ready(self, group: FlatGroup, end_offset: int):
        """Model callback: every gradient of ``group`` below ``end_offset`` is final."""
        for b in self.buckets[group.name]:
            if b.launched:
                continue
            if b.hi <= end_offset:
                self._launch(b)
            else:
                break

    def _complete(self, b: Bucket):
        if b.work is not None:
            b.work.wait()
            self._waited(b.work)
            b.work = None
        if b.staged is not None:
            b.staged[0].copy_(b.staged[1])
            b.staged = None
        if b.recv is not None:      # fp32 sum of the dp received shards -> this rank's fp32 shard
            n = (b.hi - b.lo) // self.dp
            off = self.off32[b.group.name][b.idx]
            ops.shard_sum_(b.recv, self.dp, self.out32[b.group.name][off:off + n])
            b.recv = None

    def _drain_completed(self):
        """Reduce (and release the receive buffers of) buckets whose all-to-all already
        finished, oldest first -- a non-blocking poll, so backward never waits here."""
        while self._pending and self._pending[0].recv is not None and self._pending[0].work.is_completed():
            self._complete(self._pending.pop(0))

    def finish(self):
        """Launch whatever is left and wait for every collective (stream-ordered wait)."""
        for bl in self.buckets.values():
            for b in bl:
                self._launch(b)
        if self.traffic_proxy is not None:
            self.traffic_proxy.on_finish()
        progress.mark("dp collective wait", f"{len(self._pending)} buckets")
        for b in self._pending:
            self._complete(b)
        self._pending = []

    def all_gather_params(self, overlap: bool = False):
        """ZeRO-1: after the sharded update, gather every bucket's bf16 params.

        ``overlap=True`` only LAUNCHES the gathers -- in forward order (the end of each flat
        buffer holds the first layers, see runtime/flat.py) -- and returns; the model's
        ``param_wait`` hook makes the compute stream wait on a bucket just before the next
        forward first reads it (:meth:`wait_params`), so the gather hides behind the
        previous layers' compute instead of sitting between optimizer and forward."""
        if self.traffic_proxy is not None:
            for bl in self.buckets.values():
                for b in bl:
                    self.traffic_proxy.on_gather((b.hi - b.lo) * b.group.params.element_size())
        if not self.enabled or self.mode != "reduce_scatter":
            return
        r = dist.get_rank(self.dp_group) if self.dp_group is not None else dist.get_rank()
        progress.mark("zero1 param all_gather")
        # RCCL gathers in place (input = output + rank * n, the NCCL in-place contract): no
        # staging copy of the shard and no transient 1/dp-of-the-model buffer; gloo needs one
        in_place = dist.get_backend(self.dp_group) == "nccl"
        # small groups (norm weights) first: every layer reads one of them, and the gathers
        # complete in launch order on the communicator's stream
        for name, bl in sorted(self.buckets.items(), key=lambda kv: kv[1][-1].hi if kv[1] else 0):
            for idx in reversed(range(len(bl))):
                b = bl[idx]
                x = b.group.params[b.lo:b.hi]
                n = (b.hi - b.lo) // self.dp
                mine = x[r * n:(r + 1) * n]
                w = dist.all_gather_into_tensor(x, mine if in_place else mine.clone(), group=self.dp_group,
                                                async_op=True)
                self._gathers[(name, idx)] = w
                self._note("all_gather", x, w)
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
                    self._waited(w)

    def wait_all_params(self):
        for w in self._gathers.values():
            w.wait()
            self._waited(w)
        self._gathers = {}

    def broadcast_params(self, src_global_rank: int = 0):
        """C2: make every DP replica start from identical weights."""
        if not self.enabled:
            return
        for g in self.groups:
            dist.broadcast(g.params, src=src_global_rank, group=self.dp_group)
