"""Process-group state for one-process-per-GPU training over RCCL (xGMI).

Rank layout inside one node (8 x MI355X) is [pp][dp][tp] with TP innermost, so a TP
group is the set of GPUs with the most point-to-point traffic per layer; on an 8-GPU
xGMI mesh every pair of GPUs has its own link, so any contiguous block works and TP=8
spans the whole node.

``torch.distributed``'s ``nccl`` backend IS RCCL on ROCm.  CPU runs (tests) use gloo.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    tp: int = 1
    pp: int = 1
    dp: int = 1
    tp_rank: int = 0
    pp_rank: int = 0
    dp_rank: int = 0
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    pp_group: Optional[object] = None
    pp_prev: Optional[int] = None   # global rank of previous stage
    pp_next: Optional[int] = None
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    # TP collective backend: None = torch.distributed (RCCL / gloo); a parallel.custom_ar.TwoShot
    # takes the TP reduce-scatter / all-gather / all-reduce it supports (runtime.trainer tp_comm)
    tp_comm: Optional[object] = None
    # the process-group timeout: the budget the two-shot TP kernels wait for a late peer
    timeout_s: float = 1800.0

    @property
    def is_first_stage(self):
        return self.pp_rank == 0

    @property
    def is_last_stage(self):
        return self.pp_rank == self.pp - 1


_STATE: Optional[ParallelState] = None


def visible_gpu_count() -> int:
    """GPUs this process may use, counted WITHOUT initialising the HIP runtime, so a launcher
    can call it before it starts its ranks.  ``KFAMD_VISIBLE_GPUS`` (set by a launcher that
    already knows, or a test) wins; otherwise torch's amdsmi-based count (no HIP call) and, if
    amdsmi cannot answer, the KFD topology in sysfs restricted by the ``*_VISIBLE_DEVICES``
    lists.  Never ``hipGetDeviceCount`` (that creates the HIP runtime in the caller)."""
    forced = os.environ.get("KFAMD_VISIBLE_GPUS")
    if forced is not None:
        return int(forced)
    if not torch.version.hip:
        return 0
    try:
        n = torch.cuda._device_count_amdsmi()
    except Exception:       # noqa: BLE001 -- any amdsmi failure falls through to sysfs
        n = -1
    if n >= 0:
        return n
    root = os.environ.get("KFAMD_KFD_TOPOLOGY", "/sys/class/kfd/kfd/topology/nodes")
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        return 0
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def local_device_index(local_rank: Optional[int] = None) -> int:
    """The GPU index a rank with ``LOCAL_RANK`` uses (one rank per GPU; the gloo several-ranks-
    per-GPU rehearsal wraps around) -- shared by :func:`init_distributed` and the trainer's
    device warm-up thread, so both touch the same device."""
    local = int(os.environ.get("LOCAL_RANK", "0")) if local_rank is None else local_rank
    return local % max(1, torch.cuda.device_count())


def init_distributed(tp: int = 1, pp: int = 1, backend: Optional[str] = None,
                     device: Optional[str] = None, timeout_s: int = 1800) -> ParallelState:
    """Initialise the default process group from torchrun env vars (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT) and build TP/DP/PP groups.  Works with world_size 1
    without any env."""
    global _STATE
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() if device is None else device.startswith("cuda")
    if backend is None:
        # KFAMD_DIST_BACKEND=gloo: rehearse multi-rank code paths with several ranks on ONE
        # GPU (RCCL refuses duplicate devices); never for performance numbers
        backend = os.environ.get("KFAMD_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        ndev = torch.cuda.device_count()
        if local >= ndev and backend != "gloo":
            # one rank per GPU: a rank without a GPU of its own must not silently share one
            # (KFAMD_DIST_BACKEND=gloo is the explicit several-ranks-per-GPU rehearsal)
            raise RuntimeError(f"LOCAL_RANK {local} but only {ndev} visible GPU(s): one rank per GPU "
                               f"needs {local + 1}")
        idx = local_device_index(local)
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
    else:
        dev = torch.device("cpu")
    assert world % (tp * pp) == 0, f"world {world} not divisible by tp*pp={tp * pp}"
    dp = world // (tp * pp)
    st = ParallelState(world_size=world, rank=rank, local_rank=local, tp=tp, pp=pp, dp=dp,
                       device=dev, backend=backend, timeout_s=float(timeout_s))
    if world > 1:
        if not dist.is_initialized():
            kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = dev
                # at least 32 RCCL channels: the one-GPU DP8 proxy (profiles/dp8_overlap_proxy.md)
                # moves the step's ~28 GB at the modelled 7-link xGMI rate only from 32 channel
                # workgroups up (8 / 16 fall short and the all-to-all is exposed, +4 %); 32 and 64 cost
                # the step 0.7 / 1.1 %, inside the run spread, so no upper cap is set
                os.environ.setdefault("NCCL_MIN_NCHANNELS", "32")
            dist.init_process_group(**kw)
        # rank = ((pp_rank * dp) + dp_rank) * tp + tp_rank
        st.tp_rank = rank % tp
        st.dp_rank = (rank // tp) % dp
        st.pp_rank = rank // (tp * dp)
        for p in range(pp):
            for d in range(dp):
                ranks = [(p * dp + d) * tp + t for t in range(tp)]
                g = dist.new_group(ranks) if tp > 1 else None
                if rank in ranks:
                    st.tp_group = g
        for p in range(pp):
            for t in range(tp):
                ranks = [(p * dp + d) * tp + t for d in range(dp)]
                g = dist.new_group(ranks) if dp > 1 else None
                if rank in ranks:
                    st.dp_group = g
        for d in range(dp):
            for t in range(tp):
                ranks = [(p * dp + d) * tp + t for p in range(pp)]
                g = dist.new_group(ranks) if pp > 1 else None
                if rank in ranks:
                    st.pp_group = g
                    i = ranks.index(rank)
                    st.pp_prev = ranks[i - 1] if i > 0 else None
                    st.pp_next = ranks[i + 1] if i < pp - 1 else None
    _STATE = st
    return st


def get_state() -> ParallelState:
    global _STATE
    if _STATE is None:
        _STATE = ParallelState()
    return _STATE


def set_state(st: ParallelState):
    global _STATE
    _STATE = st


def tp_all_reduce(x: torch.Tensor, st: Optional[ParallelState] = None) -> torch.Tensor:
    st = st or get_state()
    if st.tp > 1:
        tp_all_reduce_work(x, st, async_op=False)
    return x


def tp_all_reduce_work(x: torch.Tensor, st: ParallelState, async_op: bool = True):
    """In-place TP all-reduce on ``st.tp_comm`` (two-shot) or ``torch.distributed``."""
    if st.tp_comm is not None:
        return st.tp_comm.all_reduce(x, async_op=async_op)
    return dist.all_reduce(x, group=st.tp_group, async_op=async_op)


def tp_reduce_scatter_into(out: torch.Tensor, x: torch.Tensor, st: ParallelState, async_op: bool = True):
    """``dist.reduce_scatter_tensor`` over the TP group, on ``st.tp_comm`` when it is set."""
    if st.tp_comm is not None:
        return st.tp_comm.reduce_scatter(out, x, async_op=async_op)
    return dist.reduce_scatter_tensor(out, x, group=st.tp_group, async_op=async_op)


def tp_all_gather_into(out: torch.Tensor, x: torch.Tensor, st: ParallelState, async_op: bool = True):
    """``dist.all_gather_into_tensor`` over the TP group, on ``st.tp_comm`` when it is set."""
    if st.tp_comm is not None:
        return st.tp_comm.all_gather(out, x, async_op=async_op)
    return dist.all_gather_into_tensor(out, x, group=st.tp_group, async_op=async_op)


def _chunk_rows(n: int, chunks: int, tp: int) -> int:
    """The chunk count actually used for ``n`` rows: ``chunks`` when every chunk splits evenly
    over the TP ranks, else 1 (so one model always uses one layout for a given token count)."""
    return chunks if chunks > 1 and n % (chunks * tp) == 0 else 1


def tp_all_gather_rows(x: torch.Tensor, st: Optional[ParallelState] = None, chunks: int = 1,
                       async_op: bool = False):
    """Sequence parallelism: this rank's token rows -> all rows.

    Row layout with ``chunks`` = c: the global rows are c consecutive chunks and each rank holds
    the r-th 1/tp block of every chunk (c = 1: one contiguous block per rank, rank order).  The
    matching :func:`tp_reduce_scatter_rows` produces exactly this layout, so a model that uses
    one c for both everywhere (its residual stream, norms, pipeline hand-offs) is consistent,
    and the chunked form lets a GEMM consume chunk k while chunk k+1 is still on the wire.
    ``async_op``: returns (out, [work per chunk]) -- ``work[k].wait()`` before reading chunk k."""
    st = st or get_state()
    if st.tp == 1:
        return (x, []) if async_op else x
    c = _chunk_rows(x.shape[0] * st.tp, chunks, st.tp)
    out = torch.empty((x.shape[0] * st.tp,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    x = x.contiguous()
    n = x.shape[0] // c
    works = [tp_all_gather_into(out[k * n * st.tp:(k + 1) * n * st.tp], x[k * n:(k + 1) * n], st, async_op)
             for k in range(c)]
    return (out, works) if async_op else out


def tp_reduce_scatter_rows(x: torch.Tensor, st: Optional[ParallelState] = None, chunks: int = 1,
                           async_op: bool = False):
    """Sequence parallelism: partial sums over all token rows -> this rank's summed rows in the
    layout of :func:`tp_all_gather_rows` (replaces the all-reduce after a row-parallel GEMM:
    same result rows, half the bytes).  ``async_op``: returns (out, [work per chunk])."""
    st = st or get_state()
    if st.tp == 1:
        return (x, []) if async_op else x
    assert x.shape[0] % st.tp == 0, (x.shape, st.tp)
    c = _chunk_rows(x.shape[0], chunks, st.tp)
    out = torch.empty((x.shape[0] // st.tp,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    x = x.contiguous()
    n = x.shape[0] // c
    works = [tp_reduce_scatter_into(out[k * n // st.tp:(k + 1) * n // st.tp], x[k * n:(k + 1) * n], st, async_op)
             for k in range(c)]
    return (out, works) if async_op else out


def barrier():
    if dist.is_initialized():
        dist.barrier()


def destroy():
    global _STATE
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE = None
