"""One-shot all-reduce over peer-mapped HIP IPC buffers for latency-bound TP collectives.

SURVEY.md §2.8 C7 / §5 "distributed communication backend": the decode step of an
InferenceService with TP > 1 all-reduces a [B, hidden] bf16 activation twice per layer.
Those messages are a few KB to a few MB, so a ring all-reduce (RCCL) is bound by its
2(N-1) per-hop latencies, not by bandwidth.  Inside one MI355X node every GPU pair has a
direct xGMI link, so each rank publishes its input in an uncached IPC buffer and reads every
peer's copy in ONE hop (ops/csrc/custom_ar.hip).  The kernel needs no host-side epoch, so it
is captured inside the decode HIP graph like any other kernel.

Messages larger than ``max_bytes`` (prefill, training) go to ``torch.distributed`` (RCCL).

    car = OneShotAllReduce(group)          # collective: every rank of ``group`` calls it
    car(x)                                 # == dist.all_reduce(x) (in place) for small bf16 x
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _ext


class OneShotAllReduce:
    """Collective constructor over ``group`` (all ranks on GPUs of this node)."""

    def __init__(self, group=None, max_bytes: int = 4 << 20, blocks: int = 32):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert self.world in (1, 2, 4, 8), "one-shot all-reduce supports 1, 2, 4 or 8 ranks"
        self.max_bytes = int(max_bytes)
        self.blocks = int(blocks)
        k = _ext.ops()
        self._own, handle = k.car_alloc(self.max_bytes)
        handles: List[Optional[torch.Tensor]] = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        self.ptrs = []
        self._opened = []
        for r, h in enumerate(handles):
            if r == self.rank:
                self.ptrs.append(self._own)
            else:
                p = k.car_open(h)
                self._opened.append(p)
                self.ptrs.append(p)
        dist.barrier(group=group)
        self.failed = False

    def supports(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0
                and 2 * x.numel() <= self.max_bytes)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """Sum ``x`` over the group IN PLACE (as ``dist.all_reduce``); returns ``x``."""
        if not self.supports(x):
            dist.all_reduce(x, group=self.group)
            return x
        _ext.ops().car_allreduce_(self.ptrs, self.rank, x, self.max_bytes, self.blocks)
        return x

    def error(self) -> int:
        """1 when a peer failed to arrive within the kernel's spin budget since the last check."""
        return int(_ext.ops().car_error(self._own))

    def check(self):
        """Raise if any all-reduce since the last check timed out waiting for a peer.

        A timed-out kernel summed whatever sat in the peer slots, so the step's outputs are
        garbage, and the ranks' device epochs are out of step from then on: the communicator
        is poisoned for good (``failed``) and every later check raises too -- the serving
        process must be restarted (the predictor's readiness probe reports it)."""
        if self.failed or self.error():
            self.failed = True
            raise RuntimeError("one-shot all-reduce: a tensor-parallel peer did not arrive within the "
                               "spin budget; this step's results are invalid and the communicator is "
                               "out of step (restart the predictor)")

    def close(self):
        k = _ext.ops()
        for p in self._opened:
            k.car_close(p)
        self._opened = []
        if self._own:
            torch.cuda.synchronize()
            k.car_free(self._own)
            self._own = 0
