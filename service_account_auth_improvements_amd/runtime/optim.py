"""AdamW over flat parameter groups (K6), optionally ZeRO-1 sharded across DP ranks.

State per group: fp32 master weights, fp32 exp_avg, fp32 exp_avg_sq -- either for the
whole flat buffer or only for this rank's shard ranges (one range per DP bucket).  The
global gradient norm for clipping is reduced on device (sum of squares per group/shard,
then an all-reduce of a single float when sharded) and consumed by the kernel directly,
so a step never synchronises with the host.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops
from .flat import FlatGroup


@dataclass
class AdamWConfig:
    lr: float = 3e-4
    betas: Tuple[float, float] = (0.9, 0.95)
    eps: float = 1e-8
    weight_decay: float = 0.1
    max_grad_norm: float = 1.0


class _Shard:
    __slots__ = ("group", "lo", "hi", "master", "m", "v", "decay")

    def __init__(self, group: FlatGroup, lo: int, hi: int, decay: bool):
        self.group, self.lo, self.hi, self.decay = group, lo, hi, decay
        p = group.params[lo:hi]
        self.master = p.float().clone()
        self.m = torch.zeros_like(self.master)
        self.v = torch.zeros_like(self.master)


class FlatAdamW:
    def __init__(self, groups: List[FlatGroup], cfg: AdamWConfig = AdamWConfig(),
                 shard_ranges: Optional[dict] = None, dp_group=None, norm_groups=None,
                 tp_sharded: Optional[dict] = None, grad_view=None):
        """``shard_ranges[group.name] = [(lo, hi), ...]`` restricts state to this rank's
        ZeRO-1 shard; None keeps full state.  ``tp_sharded[group.name] = process group``
        marks flat groups whose parameters are split over that (tensor-parallel) group: their
        squared gradient norm is summed over it, while replicated groups (norm weights) are
        counted once -- so every TP rank clips with the same global norm."""
        self.cfg = cfg
        self.groups = groups
        self.grad_view = grad_view or (lambda g, lo, hi: g.grads[lo:hi])
        self.step_count = 0
        self.dp_group = dp_group
        # extra groups whose members hold DISJOINT parameters (pipeline stages): the
        # squared gradient norm is summed over them too
        self.norm_groups = [g for g in (norm_groups or []) if g is not None]
        self.sharded = shard_ranges is not None
        self.shards: List[_Shard] = []
        for g in groups:
            decay = any(s.decay for s in g.specs)
            assert all(s.decay == decay for s in g.specs), "mixed decay inside one flat group"
            ranges = shard_ranges[g.name] if shard_ranges else [(0, g.numel)]
            for lo, hi in ranges:
                if hi > lo:
                    self.shards.append(_Shard(g, lo, hi, decay))
        dev = groups[0].params.device
        self._sumsq = torch.zeros(1, device=dev, dtype=torch.float32)
        self.tp_sharded = dict(tp_sharded or {})
        self._pending: list = []   # (group name, lo, hi, event) of in-flight async update segments
        self._sumsq_tp = torch.zeros(1, device=dev, dtype=torch.float32)

    def grad_norm_sq(self) -> torch.Tensor:
        """Global sum of squared (summed-over-DP) gradients, on device."""
        first, first_tp = True, True
        for sh in self.shards:
            if sh.group.name in self.tp_sharded:
                ops.sumsq_(self.grad_view(sh.group, sh.lo, sh.hi), self._sumsq_tp, accumulate=not first_tp)
                first_tp = False
            else:
                ops.sumsq_(self.grad_view(sh.group, sh.lo, sh.hi), self._sumsq, accumulate=not first)
                first = False
        if first:
            self._sumsq.zero_()
        if not first_tp:
            tpg = next(iter(self.tp_sharded.values()))
            if tpg is not None:
                dist.all_reduce(self._sumsq_tp, group=tpg)
            self._sumsq.add_(self._sumsq_tp)
        if self.sharded and self.dp_group is not None:
            dist.all_reduce(self._sumsq, group=self.dp_group)
        elif self.sharded and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(self._sumsq)
        for g in self.norm_groups:
            dist.all_reduce(self._sumsq, group=g)
        return self._sumsq

    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None, segments=None, stream=None):
        """grad_scale multiplies raw gradients (e.g. 1/dp for SUM-reduced grads).

        ``stream`` + ``segments`` (a forward-ordered list of ``(group, lo, hi)`` parameter
        ranges): after the gradient norm is known, the update runs segment by segment on
        ``stream`` and each segment records an event; :meth:`wait_params` makes the compute
        stream wait for exactly the segment the next forward is about to read, so the
        HBM-bound AdamW overlaps the next step's MFMA-bound forward instead of serialising
        with it."""
        c = self.cfg
        self.step_count += 1
        lr = c.lr if lr is None else lr
        sumsq = self.grad_norm_sq() if c.max_grad_norm > 0 else None

        def upd(sh, a, b):
            ops.adamw_(sh.group.params[a:b], sh.master[a - sh.lo:b - sh.lo], sh.m[a - sh.lo:b - sh.lo],
                       sh.v[a - sh.lo:b - sh.lo], self.grad_view(sh.group, a, b), (b - a) if sh.decay else 0,
                       lr, c.betas[0], c.betas[1], c.eps, c.weight_decay, self.step_count,
                       grad_scale, sumsq, c.max_grad_norm)

        if stream is None or segments is None:
            for sh in self.shards:
                upd(sh, sh.lo, sh.hi)
            return
        self.wait_all()
        ready = torch.cuda.Event()
        ready.record()
        stream.wait_event(ready)
        with torch.cuda.stream(stream):
            for g, lo, hi in segments:
                for sh in self.shards:
                    if sh.group is g and sh.hi > lo and sh.lo < hi:
                        upd(sh, max(lo, sh.lo), min(hi, sh.hi))
                ev = torch.cuda.Event()
                ev.record(stream)
                self._pending.append((g.name, lo, hi, ev))

    def wait_params(self, group: FlatGroup, lo: int, hi: int):
        """Compute stream waits for the pending update segments overlapping [lo, hi)."""
        if not self._pending:
            return
        keep = []
        for name, a, b, ev in self._pending:
            if name == group.name and a < hi and b > lo:
                torch.cuda.current_stream().wait_event(ev)
            else:
                keep.append((name, a, b, ev))
        self._pending = keep

    def wait_all(self):
        for _, _, _, ev in self._pending:
            torch.cuda.current_stream().wait_event(ev)
        self._pending = []

    def state_dict(self):
        return {"step": self.step_count,
                "shards": [(sh.group.name, sh.lo, sh.hi, sh.master, sh.m, sh.v) for sh in self.shards]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        by_key = {(n, lo, hi): (w, m, v) for n, lo, hi, w, m, v in sd["shards"]}
        for sh in self.shards:
            w, m, v = by_key[(sh.group.name, sh.lo, sh.hi)]
            sh.master.copy_(w)
            sh.m.copy_(m)
            sh.v.copy_(v)
            sh.group.params[sh.lo:sh.hi].copy_(sh.master)
