"""Training step driver for the Llama worker runtime.

One process per GPU.  A step = micro-batches of explicit forward+backward (no autograd),
weight gradients written into flat buffers, DP gradient buckets reduced over RCCL while
backward is still running, then one fused AdamW kernel per flat group.  Pipeline
parallel training uses :mod:`..parallel.pipeline` on top of the same pieces.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..models.llama import Llama, LlamaConfig
from ..parallel.custom_ar import make_tp_comm
from ..parallel.ddp import GradReducer
from ..parallel.state import ParallelState, get_state
from .optim import AdamWConfig, FlatAdamW


@dataclass
class TrainConfig:
    model: str = "llama3-8b"
    seq_len: int = 8192
    micro_batch: int = 1
    grad_accum: int = 1
    zero1: bool = False
    overlap_allgather: bool = True   # ZeRO-1: hide the param all-gather behind the next forward
    # AdamW on a side stream overlapped with the next forward (GPU, no ZeRO).  Measured on MI355X:
    # 64% of AdamW time overlaps, but both sides slow down (HBM/CU contention) -- no net gain
    # at 8B (profiles/async_optimizer_overlap.txt), so it is off by default.
    async_optimizer: bool = False
    bucket_mb: int = 256
    # DP gradient reduction precision (parallel/ddp.py): "fp32" sums every rank's bf16
    # gradient in fp32 (all-to-all + HIP fp32 shard sum under ZeRO-1) and accumulates
    # micro-batches in fp32; "bf16" reduces in bf16 with RCCL and accumulates in bf16
    grad_reduce: str = "fp32"
    force_collectives: bool = False  # run the DP collectives at dp=1 (one-GPU RCCL test)
    lr: float = 3e-4
    weight_decay: float = 0.1
    max_grad_norm: float = 1.0
    seed: int = 1234
    n_layers: Optional[int] = None   # override (tests only; benches must use the full model)
    recompute: bool = False          # per-layer activation recomputation (memory for compute)
    head_chunk: int = 4096           # K5: LM head + CE row chunk (tokens); 0 = whole micro-batch
    sequence_parallel: bool = False  # Megatron SP on top of TP (token-row-sharded norms / residual)
    # context parallelism (parallel/context.py): the DP group becomes ONE context-parallel group --
    # its ranks share the same sequences, each holding 1/dp of every sequence's tokens
    context_parallel: bool = False
    # TP forward communication overlap: token chunks per row-/column-parallel projection
    # (models/llama.py _row_parallel / _col_parallel); 1 = one GEMM + one blocking collective
    tp_comm_chunks: int = 4
    # TP collective backend: "rccl" (torch.distributed) or "twoshot" (parallel/custom_ar.py TwoShot:
    # peer-mapped reduce-scatter / all-gather over all xGMI links at once; GPU jobs only, a CPU
    # job keeps torch.distributed)
    tp_comm: str = "rccl"
    # TP forward: split each micro-batch into two half-batches whose layers are interleaved at
    # every TP collective, then one full-batch backward (models/llama.py stage_forward_dual);
    # needs an even micro-batch, one pipeline stage, no recomputation and no SP.
    tp_dual_batch: bool = False
    # pipeline: model chunks (virtual stages) per rank; > 1 selects the interleaved 1F1B schedule
    # (parallel/pipeline.py interleaved_1f1b; micro-batches per step a multiple of pp)
    pp_virtual: int = 1


class Trainer:
    def __init__(self, tcfg: TrainConfig, st: Optional[ParallelState] = None,
                 mcfg: Optional[LlamaConfig] = None, full_init: bool = False):
        self.tcfg = tcfg
        self.st = st or get_state()
        mcfg = mcfg or LlamaConfig.preset(tcfg.model)
        if tcfg.n_layers is not None:
            mcfg = mcfg.with_(n_layers=tcfg.n_layers)
        if tcfg.seq_len > mcfg.max_seq:
            mcfg = mcfg.with_(max_seq=tcfg.seq_len)
        self.mcfg = mcfg
        assert self.st.pp == 1, "use parallel.pipeline.PipelineTrainer for pp > 1"
        t0 = time.time()
        self.model = Llama(mcfg, self.st, seed=tcfg.seed, full_init=full_init)
        self.model.recompute = tcfg.recompute
        self.model.head_chunk = tcfg.head_chunk
        self.model.sequence_parallel = tcfg.sequence_parallel
        if self.st.tp > 1:
            self.model.tp_comm_chunks = getattr(tcfg, "tp_comm_chunks", self.model.tp_comm_chunks)
            self.st.tp_comm = make_tp_comm(getattr(tcfg, "tp_comm", "rccl"), self.st)
        self.cp = self.st.dp if tcfg.context_parallel else 1
        if self.cp > 1:
            self.model.set_context_parallel(self.st.dp_group, self.st.dp, self.st.dp_rank)
        self.model.allocate(pad_to=self.st.dp * 64 if tcfg.zero1 else 1)
        self._sync()
        self.init_times = {"params_alloc_init_s": time.time() - t0}
        t0 = time.time()
        mode = "reduce_scatter" if (tcfg.zero1 and (self.st.dp > 1 or tcfg.force_collectives)) else "allreduce"
        # dual half-batch TP forward (tp_dual_batch, models/llama.py stage_forward_dual)
        self.dual = (self.st.tp > 1 and getattr(tcfg, "tp_dual_batch", False) and tcfg.micro_batch % 2 == 0
                     and not tcfg.recompute and self.cp == 1 and not tcfg.sequence_parallel)
        self.reducer = GradReducer(self.model.groups, self.st.dp_group, self.st.dp,
                                   bucket_bytes=tcfg.bucket_mb << 20, mode=mode,
                                   reduce_dtype=tcfg.grad_reduce, grad_accum=tcfg.grad_accum,
                                   force_collectives=tcfg.force_collectives)
        # identical replicas: broadcast from the first rank of this DP group (C2)
        if self.st.dp > 1:
            src = self.st.rank - self.st.dp_rank * self.st.tp
            self.reducer.broadcast_params(src)
        shard = None
        if mode == "reduce_scatter":
            shard = {g.name: self.reducer.shard_ranges(g, self.st.dp_rank) for g in self.model.groups}
        self.opt = FlatAdamW(self.model.groups,
                             AdamWConfig(lr=tcfg.lr, weight_decay=tcfg.weight_decay,
                                         max_grad_norm=tcfg.max_grad_norm),
                             shard_ranges=shard, dp_group=self.st.dp_group,
                             tp_sharded={"matrices": self.st.tp_group} if self.st.tp > 1 else None,
                             grad_view=self.reducer.grad_view)
        self._sync()
        self.init_times["optimizer_state_s"] = time.time() - t0
        self.step_idx = 0
        # events the next optimizer update must stream-wait for: an asynchronous checkpoint's
        # device-to-host snapshot of the state that update rewrites (runtime/checkpoint.py)
        self.pre_opt_waits: list = []
        self._opt_stream = None
        self._segments = None
        if mode == "reduce_scatter" and tcfg.overlap_allgather:
            self.model.param_wait = self.reducer.wait_params
        elif mode == "allreduce" and tcfg.async_optimizer and self.st.device.type == "cuda":
            self._opt_stream = torch.cuda.Stream(device=self.st.device)
            self._segments = self.model.param_segments()
            self.model.param_wait = self.opt.wait_params

    def _sync(self):
        if self.st.device.type == "cuda":
            torch.cuda.synchronize()

    def release(self):
        """Drop every device buffer (params, grads, optimizer state) -- end of job."""
        self.sync_params()
        for g in self.model.groups:
            g.params = g.grads = None
        self.opt.shards = []

    def sync_params(self):
        """Complete in-flight ZeRO-1 parameter gathers / async optimizer segments (before
        checkpoint, eval or host reads of the parameters)."""
        self.reducer.wait_all_params()
        self.opt.wait_all()

    def reduced_grads(self, group) -> torch.Tensor:
        """fp32 copy of the DP-summed gradient of a flat group as the optimizer saw it in the
        last step.  Under ZeRO-1 only this rank's shards are reduced: other elements are NaN."""
        r = self.reducer
        if r.mode == "reduce_scatter" and r.enabled:
            out = torch.full((group.numel,), float("nan"), device=group.grads.device)
            for lo, hi in r.shard_ranges(group, self.st.dp_rank):
                out[lo:hi] = r.grad_view(group, lo, hi).float()
            return out
        return r.grad_view(group, 0, group.numel).float().clone()

    @property
    def tokens_per_step(self) -> int:
        """Tokens processed by THIS rank per step."""
        return self.tcfg.micro_batch * self.tcfg.seq_len * self.tcfg.grad_accum // self.cp

    def train_step(self, micro_batches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """``micro_batches``: [B, S] token / label pairs.  Under context parallelism every rank of
        the group passes the SAME full sequences and trains on its own token block of them; the
        returned loss is then the mean over this rank's tokens."""
        if self.cp > 1:
            from ..parallel.context import shard_tokens
            micro_batches = [(shard_tokens(t, self.cp, self.st.dp_rank), shard_tokens(l, self.cp, self.st.dp_rank))
                             for t, l in micro_batches]
        n = len(micro_batches)
        ntok = sum(t.numel() for t, _ in micro_batches)
        scale = 1.0 / ntok
        self.reducer.start_step()
        f32acc = self.reducer.fp32_accumulation
        total = None
        dual = self.dual and all(t.shape[0] % 2 == 0 for t, _ in micro_batches)
        for j, (tok, lab) in enumerate(micro_batches):
            self.model.on_grad_ready = self.reducer.grad_ready if j == n - 1 else None
            if dual:      # two interleaved half-batches forward, one full-batch backward
                B, S = tok.shape
                loss, ctx = self.model.stage_forward_dual(tok.reshape(-1), lab.reshape(-1), B, S, scale)
                self.model.stage_backward(ctx, None, B, S, accumulate=j > 0 and not f32acc)
                del ctx
            else:
                loss = self.model.forward_backward(tok, lab, accumulate=j > 0 and not f32acc, scale=scale)
            if j < n - 1:
                self.reducer.accumulate_micro(first=j == 0)
            total = loss if total is None else total + loss
        self.model.on_grad_ready = None
        self.reducer.wait_all_params()     # a bucket the forward never read (padding) must land too
        self.reducer.finish()
        wait_pre_opt(self, self._opt_stream)
        self.opt.step(grad_scale=1.0 / self.st.dp, segments=self._segments, stream=self._opt_stream)
        self.reducer.all_gather_params(overlap=self.tcfg.overlap_allgather)
        self.step_idx += 1
        if self.st.tp_comm is not None:
            # a two-shot collective whose peer never arrived produced garbage: fail the step
            # (and the job) instead of training on it
            self.st.tp_comm.check()
        return total


def wait_pre_opt(trainer, extra_stream=None):
    """Stream-wait (never a host wait) for the events queued in ``trainer.pre_opt_waits``."""
    if not trainer.pre_opt_waits:
        return
    cur = torch.cuda.current_stream()
    for ev in trainer.pre_opt_waits:
        cur.wait_event(ev)
        if extra_stream is not None:
            extra_stream.wait_event(ev)
    trainer.pre_opt_waits = []


class SyntheticData:
    """Deterministic synthetic token batches (random ids, labels = next token)."""

    def __init__(self, vocab: int, micro_batch: int, seq_len: int, device, seed: int = 0,
                 rank: int = 0):
        self.vocab, self.mb, self.S = vocab, micro_batch, seq_len
        self.device = device
        self.g = torch.Generator(device="cpu").manual_seed(seed * 7919 + rank)

    def next(self):
        """The next micro-batch; the stream position lives in the generator state, which
        checkpoints save and resume restores (runtime/checkpoint.py)."""
        x = torch.randint(0, self.vocab, (self.mb, self.S + 1), generator=self.g)
        x = x.to(self.device, non_blocking=True)
        return x[:, :-1].contiguous(), x[:, 1:].contiguous()
