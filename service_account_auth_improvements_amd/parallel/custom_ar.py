"""Peer-mapped HIP IPC collectives for tensor parallelism inside one MI355X node.

``OneShotAllReduce``: latency-bound decode messages (below).  ``TwoShot``: bandwidth-bound
training messages (reduce-scatter / all-gather / all-reduce of 16-268 MB activations).

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

    def __init__(self, group=None, max_bytes: int = 4 << 20, blocks: int = 32, timeout_s: float = 10.0):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert self.world in (1, 2, 4, 8), "one-shot all-reduce supports 1, 2, 4 or 8 ranks"
        self.max_bytes = int(max_bytes)
        self.blocks = int(blocks)
        # wall-clock budget a kernel block waits for a peer before it sets the error word
        self.timeout_s = float(timeout_s)
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
        _ext.ops().car_allreduce_(self.ptrs, self.rank, x, self.max_bytes, self.blocks, self.timeout_s)
        return x

    def error(self) -> int:
        """1 when a peer failed to arrive within ``timeout_s`` since the last check."""
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


class _Done:
    """Work handle of a two-shot collective: ``wait()`` orders the CURRENT stream after it
    (the ``torch.distributed`` async-work contract the model code uses)."""

    def __init__(self, event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)
        return True


def two_shot_blocks(requested: Optional[int], sharing: int, cus: int) -> int:
    """Workgroups per two-shot call: ``requested`` as given (capped to TwoShot.MAX_BLOCKS), else
    the measured default, capped when ``sharing`` ranks drive the same GPU so that their spinning
    calls leave half of its ``cus`` compute units to the peers' other kernels."""
    if requested is None:
        requested = TwoShot.DEFAULT_BLOCKS
        if sharing > 1:
            requested = min(requested, max(1, cus // (2 * sharing)))
    return max(1, min(int(requested), TwoShot.MAX_BLOCKS))


def uniform_two_shot_blocks(requested: Optional[int], dev_keys: List[tuple], cus: List[int]) -> int:
    """The ONE block count every rank of a communicator uses.  The kernel splits each chunk by
    ``gridDim.x`` and pairs its peer flags by ``blockIdx``, so ranks that disagree read peer
    ranges no peer block wrote (wrong sums) and leave blocks spinning until the wait budget
    runs out.  Derived only from values every rank gathered -- the most ranks that share any one
    GPU and the fewest CUs of any rank's GPU -- so an uneven spread (8 ranks on 3 GPUs: 3/3/2)
    still yields one value."""
    counts: dict = {}
    for k in dev_keys:
        counts[k] = counts.get(k, 0) + 1
    return two_shot_blocks(requested, max(counts.values()), min(cus))


class TwoShot:
    """Two-shot reduce-scatter / all-gather / all-reduce over xGMI (ops/csrc/custom_ar.hip, ts).

    RCCL runs a TP=8 reduction as a ring: 2(N-1) steps, each over ONE xGMI link at a time, so
    a 128 MB all-reduce moves 2*(7/8)*128 MB through a single ~50 GB/s link direction per GPU.
    On the full-mesh xGMI of an MI355X node every GPU has a direct link to every peer, so here
    rank r pulls chunk r of every peer's input over all N-1 links AT ONCE, sums it in fp32 in
    rank order, and (all-gather half) every rank pulls every peer's reduced chunk: each link
    carries 2 S / N bytes per direction and the N-1 links work concurrently (per-link bytes
    for the 70B TP=8 shard: profiles/llama3_70b_tp8_shard.md).  Results are bit-identical on
    every rank (the chunk owner sums once) and, for N = 2, bit-identical to RCCL (one bf16
    rounding of the exact fp32 sum).  For N > 2 RCCL's ring order differs: within rounding.

    Layouts match ``dist.reduce_scatter_tensor`` / ``dist.all_gather_into_tensor`` (rank r's
    block is the r-th contiguous 1/N of the full tensor), so :mod:`parallel.state` swaps it in
    for those calls.  Every call runs on the communicator's own stream (the kernel's slot
    protocol needs ONE stream and ONE grid size per communicator) ordered after the caller's
    stream; ``async_op=True`` returns a handle whose ``wait()`` orders the caller's stream after
    it, else the caller's stream is ordered immediately.  CPU tensors, other dtypes and sizes
    outside the buffer fall back to ``torch.distributed`` (gloo / RCCL).

        st.tp_comm = TwoShot(st.tp_group)      # collective over the TP group
        tp_reduce_scatter_rows(x, st)          # now runs the two-shot kernel
    """

    MAX_BLOCKS = 128

    # workgroups per call (blocks=None): measured on one MI355X at 16/64/268 MB for 32/64/128
    # blocks (tools/bench_two_shot.py, profiles/two_shot_blocks_r5.md): 128 is fastest at every
    # size and mode (RS 268 MB: 0.44 ms vs 0.70 at 64 and 1.21 at 32) -- each block keeps only a
    # few uncached loads in flight, so the kernel needs the blocks to reach bandwidth
    DEFAULT_BLOCKS = 128

    def __init__(self, group=None, max_bytes: int = 288 << 20, blocks: Optional[int] = None,
                 timeout_s: float = 300.0):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert self.world in (1, 2, 4, 8), "two-shot collectives support 1, 2, 4 or 8 ranks"
        self.max_bytes = int(max_bytes) // (16 * self.world) * (16 * self.world)
        # wall-clock budget (s_memrealtime) a kernel block waits for a peer: a late peer -- one
        # rank's first-step GEMM heuristics, a checkpoint write -- is waited for; only one that
        # stays away this long sets the error word.  The trainer passes its process-group
        # timeout, so the kernel gives up no sooner than RCCL would.
        self.timeout_s = float(timeout_s)
        k = _ext.ops()
        self._own, handle = k.ts_alloc(self.max_bytes, self.world)
        props = torch.cuda.get_device_properties(torch.cuda.current_device())
        dev_key = (str(props.uuid), props.pci_domain_id, props.pci_bus_id, props.pci_device_id)
        gathered: List[Optional[tuple]] = [None] * self.world
        dist.all_gather_object(gathered, (handle, dev_key, props.multi_processor_count), group=group)
        handles = [g[0] for g in gathered]
        # Ranks that share one GPU (the one-GPU multi-process tests and rehearsals): a call's
        # blocks spin on the card until every peer's call arrives, so with W ranks x 128 blocks
        # they can fill every CU and starve a peer's preceding kernels (its attention needs a
        # whole CU's LDS) until the wait budget runs out.  The automatic count is then capped
        # to leave half the CUs free; one rank per GPU (production) keeps the measured 128.
        # Every rank must launch the same count: computed from the gathered values only.
        self.blocks = uniform_two_shot_blocks(blocks, [g[1] for g in gathered], [g[2] for g in gathered])
        self.ptrs, self._opened = [], []
        for r, h in enumerate(handles):
            if r == self.rank:
                self.ptrs.append(self._own)
            else:
                p = k.car_open(h)
                self._opened.append(p)
                self.ptrs.append(p)
        self.stream = torch.cuda.Stream()
        # asynchronous error-word reads: copied into pinned memory on the comm stream, looked
        # at once the copy's event has completed (no host synchronisation per step)
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_event = None
        dist.barrier(group=group)
        self.failed = False
        self.calls = 0

    def supports(self, full_numel: int, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and full_numel % (8 * self.world) == 0
                and 2 * full_numel <= self.max_bytes)

    def _run(self, mode: int, x: torch.Tensor, out: torch.Tensor, async_op: bool):
        cur = torch.cuda.current_stream()
        x = x.contiguous()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            _ext.ops().ts_run(mode, self.ptrs, self.rank, x, out, self.max_bytes, self.blocks, self.timeout_s)
        # both stay allocated until the comm stream has used them
        x.record_stream(self.stream)
        out.record_stream(self.stream)
        self.calls += 1
        ev = torch.cuda.Event()
        ev.record(self.stream)
        done = _Done(ev)
        if not async_op:
            done.wait()
        return done

    def all_reduce(self, x: torch.Tensor, async_op: bool = False):
        """In place, as ``dist.all_reduce``; returns a work handle (``async_op``) or None."""
        if not (x.is_contiguous() and self.supports(x.numel(), x)):
            return dist.all_reduce(x, group=self.group, async_op=async_op)
        w = self._run(0, x, x, async_op)
        return w if async_op else None

    def reduce_scatter(self, out: torch.Tensor, x: torch.Tensor, async_op: bool = False):
        """``dist.reduce_scatter_tensor(out, x)``: out = rank r's 1/N block of the sum."""
        if not (out.is_contiguous() and self.supports(x.numel(), x)):
            return dist.reduce_scatter_tensor(out, x, group=self.group, async_op=async_op)
        if out.numel() * self.world != x.numel() or out.dtype != x.dtype or out.device != x.device:
            raise ValueError(f"reduce_scatter: out {tuple(out.shape)} is not 1/{self.world} of x {tuple(x.shape)}")
        w = self._run(1, x, out, async_op)
        return w if async_op else None

    def all_gather(self, out: torch.Tensor, x: torch.Tensor, async_op: bool = False):
        """``dist.all_gather_into_tensor(out, x)``: out = every rank's x in rank order."""
        if not (out.is_contiguous() and self.supports(out.numel(), x)):
            return dist.all_gather_into_tensor(out, x, group=self.group, async_op=async_op)
        if x.numel() * self.world != out.numel() or out.dtype != x.dtype or out.device != x.device:
            raise ValueError(f"all_gather: out {tuple(out.shape)} is not {self.world} x {tuple(x.shape)}")
        w = self._run(2, x, out, async_op)
        return w if async_op else None

    def _raise(self):
        self.failed = True
        raise RuntimeError(f"two-shot TP collective: a peer did not arrive within {self.timeout_s:.0f} s; "
                           "results since the error are invalid and the communicator is out of step "
                           "(restart the job)")

    def check(self, sync: bool = False):
        """Raise if a call timed out waiting for a peer (the communicator is then out of step
        for good, as the one-shot one).

        Default (every training step): no host synchronisation.  The error word of the calls
        issued so far is copied on the communicator's stream into pinned memory; the check
        reads the PREVIOUS copy once its event has completed and queues the next one, so an
        error surfaces a step or two late (the step that produced it already counted as
        garbage either way).  ``sync=True`` (checkpoint, end of run) waits for every call
        issued so far and reads the word now."""
        if self.failed:
            self._raise()
        k = _ext.ops()
        if sync:
            self.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                k.ts_error_async(self._own, self._err_host)
            self.stream.synchronize()
            self._err_event = None
            if int(self._err_host[0]):
                self._raise()
            return
        if self._err_event is not None:
            if not self._err_event.query():
                return                      # the previous read is still in flight: look next time
            self._err_event = None
            if int(self._err_host[0]):
                self._raise()
        with torch.cuda.stream(self.stream):
            k.ts_error_async(self._own, self._err_host)
            self._err_event = torch.cuda.Event()
            self._err_event.record(self.stream)

    def close(self):
        k = _ext.ops()
        torch.cuda.synchronize()
        for p in self._opened:
            k.car_close(p)
        self._opened = []
        if self._own:
            k.car_free(self._own)
            self._own = 0


def make_tp_comm(kind: str, st):
    """The TP communicator a trainer installs as ``st.tp_comm``: ``"twoshot"`` -> :class:`TwoShot`
    over ``st.tp_group`` when the ranks drive GPUs (fails loudly if the HIP extension is missing);
    ``"rccl"``, tp == 1 or a CPU (gloo) job -> None, i.e. plain ``torch.distributed``."""
    if kind not in ("rccl", "twoshot"):
        raise ValueError(f"tp_comm must be 'rccl' or 'twoshot', not {kind!r}")
    if kind == "rccl" or st.tp == 1 or st.device.type != "cuda":
        return None
    return TwoShot(st.tp_group, timeout_s=float(getattr(st, "timeout_s", 300.0)))
