"""Llama-3 decoder (8B / 70B shapes) with an explicit, autograd-free training step.

Design (MI355X-first):

* Activations are 2-D ``[T, hidden]`` bf16 (T = micro_batch * seq).  Per layer there are
  exactly four GEMMs (hipBLASLt): fused QKV, O, fused gate/up, down -- and the rest is
  hand-written gfx950 kernels: fused residual-add+RMSNorm (K1), in-place RoPE on the fused
  QKV buffer (K2), flash attention reading q/k/v straight out of that buffer (K3), SwiGLU
  (K4), fused CE with in-place gradient (K5); AdamW (K6) runs over the flat buffers.
* The residual add is deferred into the next RMSNorm: a layer maps (r, d) -> (h2, d_mlp)
  with h1 = r + d computed inside the norm kernel, so no stand-alone add kernel exists.
* Forward and backward are explicit (no autograd graph): ``layer_fwd`` returns a context
  of saved tensors, ``layer_bwd`` consumes it.  Weight gradients are written by the
  backward GEMMs straight into their slice of the flat gradient buffer (``out=`` for the
  first micro-batch, ``addmm_`` with beta=1 afterwards) and the DP engine is told the
  moment each layer's slice is final, so its bucket all-reduce overlaps the remaining
  backward.
* Tensor parallelism (Megatron column/row split, vocab-parallel embedding / LM head / CE)
  is built in: local head counts and FFN width are the global ones divided by ``tp``; the
  two per-layer reductions go through RCCL over xGMI.
* 288 GB of HBM per GPU means no activation recomputation is needed for 8B at 8k tokens
  per micro-batch (~1.1 GB of saved activations per layer): everything is kept resident.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, replace
from typing import Callable, List, Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .. import ops
from ..ops.attention import attention_bwd, attention_fwd
from ..parallel import context as cpx
from ..parallel.state import (ParallelState, _chunk_rows, get_state, tp_all_gather_rows, tp_all_reduce,
                              tp_all_reduce_work, tp_reduce_scatter_into, tp_reduce_scatter_rows)

# KFAMD_DX_T=0 runs the activation-gradient GEMMs on the untransposed weights (A/B switch)
_DX_T = os.environ.get("KFAMD_DX_T", "1") != "0"
from ..runtime.flat import FlatGroup


@dataclass
class LlamaConfig:
    name: str = "llama3-8b"
    vocab_size: int = 128256
    hidden: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    head_dim: int = 128
    ffn: int = 14336
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq: int = 8192
    init_std: float = 0.02

    @staticmethod
    def preset(name: str) -> "LlamaConfig":
        name = name.lower()
        if name in ("llama3-8b", "llama-3-8b", "8b"):
            return LlamaConfig()
        if name in ("llama3-70b", "llama-3-70b", "70b"):
            return LlamaConfig(name="llama3-70b", hidden=8192, n_layers=80, n_heads=64,
                               n_kv_heads=8, ffn=28672)
        if name in ("tiny", "llama3-tiny"):
            return LlamaConfig(name="llama3-tiny", vocab_size=512, hidden=256, n_layers=2,
                               n_heads=4, n_kv_heads=2, head_dim=128, ffn=512, max_seq=256)
        if name in ("small", "llama3-small"):
            return LlamaConfig(name="llama3-small", vocab_size=32000, hidden=1024, n_layers=4,
                               n_heads=8, n_kv_heads=2, head_dim=128, ffn=3584, max_seq=2048)
        raise ValueError(f"unknown preset {name}")

    def with_(self, **kw) -> "LlamaConfig":
        return replace(self, **kw)

    def num_params(self) -> int:
        H, F_, V, L = self.hidden, self.ffn, self.vocab_size, self.n_layers
        qkv = H * (self.n_heads + 2 * self.n_kv_heads) * self.head_dim
        o = self.n_heads * self.head_dim * H
        per_layer = qkv + o + 3 * H * F_ + 2 * H
        return L * per_layer + 2 * V * H + H

    def flops_per_token(self, seq: int) -> float:
        """Training FLOPs/token: 6*N_matmul + causal attention (fwd+bwd = 3x fwd)."""
        H, L = self.hidden, self.n_layers
        n_mm = self.num_params() - self.vocab_size * H - (2 * L + 1) * H  # no embed gather, no norms
        attn = 3 * 2 * 2 * self.n_heads * self.head_dim * seq / 2 * L   # causal: half of S^2
        return 6 * n_mm + attn


def _run(gen):
    """Drive a generator to completion and return its value."""
    while True:
        try:
            next(gen)
        except StopIteration as e:
            return e.value


def _interleave(gens):
    """Alternate independent generators (one step each in turn) until all have returned; the
    values come back in order.  A step ends where a generator yielded after launching an
    asynchronous collective, so each one's communication overlaps the others' compute."""
    out, live = [None] * len(gens), list(range(len(gens)))
    while live:
        for k in list(live):
            try:
                next(gens[k])
            except StopIteration as e:
                out[k] = e.value
                live.remove(k)
    return out


class _LayerCtx:
    __slots__ = ("h1", "rstd1", "a", "qkv", "o", "o_tok", "lse", "h2", "rstd2", "m", "gu", "s")


class Llama:
    """One pipeline stage (all layers when pp == 1) of a Llama-3 model shard."""

    def __init__(self, cfg: LlamaConfig, st: Optional[ParallelState] = None, device=None,
                 layer_range: Optional[range] = None, seed: int = 1234, full_init: bool = False):
        self.cfg = cfg
        self.st = st or get_state()
        tp = self.st.tp
        assert cfg.n_heads % tp == 0 and cfg.n_kv_heads % tp == 0 and cfg.ffn % tp == 0
        assert cfg.vocab_size % tp == 0
        self.tp = tp
        self.hq = cfg.n_heads // tp
        self.hkv = cfg.n_kv_heads // tp
        self.ff = cfg.ffn // tp
        self.vl = cfg.vocab_size // tp
        self.vstart = self.st.tp_rank * self.vl
        self.device = torch.device(device) if device is not None else self.st.device
        self.layers = list(layer_range if layer_range is not None else range(cfg.n_layers))
        self.first = self.layers[0] == 0 if self.layers else self.st.is_first_stage
        self.last = (self.layers[-1] == cfg.n_layers - 1) if self.layers else self.st.is_last_stage
        H, D = cfg.hidden, cfg.head_dim
        self.qkv_w = (self.hq + 2 * self.hkv) * D
        # ---- parameter registration in reverse execution order (see runtime/flat.py)
        mats, norms = FlatGroup("matrices"), FlatGroup("norms")
        if self.last:
            mats.add("lm_head", (self.vl, H), std=cfg.init_std)
            norms.add("final_norm", (H,), init="ones", decay=False)
        out_std = cfg.init_std / math.sqrt(2 * cfg.n_layers)
        for i in reversed(self.layers):
            mats.add(f"l{i}.wd", (H, self.ff), std=out_std)
            mats.add(f"l{i}.wgu", (2 * self.ff, H), std=cfg.init_std)
            mats.add(f"l{i}.wo", (H, self.hq * D), std=out_std)
            mats.add(f"l{i}.wqkv", (self.qkv_w, H), std=cfg.init_std)
            norms.add(f"l{i}.norm2", (H,), init="ones", decay=False)
            norms.add(f"l{i}.norm1", (H,), init="ones", decay=False)
        if self.first:
            mats.add("embed", (self.vl, H), std=cfg.init_std)
        self.mats, self.norms = mats, norms
        self.groups = [mats, norms]
        self._full_init = full_init
        self._seed = seed
        self.on_grad_ready: Optional[Callable[[FlatGroup, int], None]] = None
        # ZeRO-1 overlap: called with (group, lo, hi) before a parameter range is first
        # read in forward, so the async all-gather of that range can be waited on lazily
        self.param_wait: Optional[Callable[[FlatGroup, int, int], None]] = None
        # activation recomputation: keep only each layer's input (r, d) from the forward and
        # re-run the layer's forward right before its backward (memory plans where the saved
        # activations do not fit: 70B at long sequence / larger micro-batch)
        self.recompute = False
        # K5: LM head + cross-entropy in row chunks of this many tokens (0 = one chunk): the
        # [T, vocab] logits are never materialised -- only one [chunk, vocab] slab at a time
        self.head_chunk = 4096
        # Megatron sequence parallelism (tp > 1): the residual stream, the RMSNorms and their
        # saved activations hold only this rank's 1/tp block of token rows; an all-gather feeds
        # each column-parallel GEMM and a reduce-scatter (instead of the all-reduce) ends each
        # row-parallel one -- the same bytes per layer, 1/tp of the norm/residual activations
        self.sequence_parallel = False
        self._sp_norm_parts: list = []
        # TP communication chunks: each row-parallel GEMM (wo, wd) runs in this many token
        # chunks, chunk k's all-reduce / SP reduce-scatter on the wire while chunk k+1
        # multiplies, and under SP each column-parallel GEMM (wqkv, wgu) multiplies chunk k
        # while the all-gather of chunk k+1 is in flight (parallel/state.py row layout)
        self.tp_comm_chunks = 4 if tp > 1 else 1
        # context parallelism (parallel/context.py): this rank holds 1/cp of every sequence's
        # tokens; attention runs on all tokens for 1/cp of the heads between two all-to-alls
        self.cp, self.cp_rank, self.cp_group = 1, 0, None
        cos, sin = ops.rope_tables(cfg.max_seq, D, cfg.rope_theta)
        self.cos = cos.to(self.device)
        self.sin = sin.to(self.device)

    # ------------------------------------------------------------------ storage
    def allocate(self, pad_to: int = 1, grads: bool = True):
        for g in self.groups:
            g.allocate(self.device, pad_to=pad_to, grads=grads)
        self._init()
        return self

    def _tp_slicers(self):
        """Map each TP-sharded tensor to (full_shape, slicer) so every TP degree draws the
        same full matrix (exact TP==1 equivalence in tests)."""
        cfg, r, tp = self.cfg, self.st.tp_rank, self.tp
        H, D, F_, V = cfg.hidden, cfg.head_dim, cfg.ffn, cfg.vocab_size
        Hq, Hkv = cfg.n_heads, cfg.n_kv_heads
        out = {}

        def rows(lo, hi):
            return lambda t: t[lo:hi]

        for i in self.layers:
            def qkv_slice(t, r=r):
                q = t[:Hq * D].view(Hq, D, H)[r * self.hq:(r + 1) * self.hq].reshape(-1, H)
                k = t[Hq * D:(Hq + Hkv) * D].view(Hkv, D, H)[r * self.hkv:(r + 1) * self.hkv].reshape(-1, H)
                v = t[(Hq + Hkv) * D:].view(Hkv, D, H)[r * self.hkv:(r + 1) * self.hkv].reshape(-1, H)
                return torch.cat([q, k, v], 0)

            def gu_slice(t, r=r):
                return torch.cat([t[r * self.ff:(r + 1) * self.ff], t[F_ + r * self.ff:F_ + (r + 1) * self.ff]], 0)

            out[f"l{i}.wqkv"] = ((( Hq + 2 * Hkv) * D, H), qkv_slice)
            out[f"l{i}.wo"] = ((H, Hq * D), lambda t, r=r: t[:, r * self.hq * D:(r + 1) * self.hq * D])
            out[f"l{i}.wgu"] = ((2 * F_, H), gu_slice)
            out[f"l{i}.wd"] = ((H, F_), lambda t, r=r: t[:, r * self.ff:(r + 1) * self.ff])
        if self.first:
            out["embed"] = ((V, H), rows(r * self.vl, (r + 1) * self.vl))
        if self.last:
            out["lm_head"] = ((V, H), rows(r * self.vl, (r + 1) * self.vl))
        return out

    def _init(self):
        full = self._tp_slicers() if self._full_init else None
        for g in self.groups:
            g.init_(self._seed, full)

    def P(self, name):
        g = self.mats if name in self.mats._index else self.norms
        return g.param(name)

    def G(self, name):
        g = self.mats if name in self.mats._index else self.norms
        return g.grad(name)

    def _ready(self, group: FlatGroup, name: str):
        if self.on_grad_ready is not None:
            self.on_grad_ready(group, group.end_offset(name))

    @staticmethod
    def _mm_into(out, a, b, accumulate):
        """out (+)= a . b.  Weight gradients (a = dY^T, a transposed view of [T, N]) go to the
        hand-written gfx950 dW kernel (ops/csrc/gemm.hip, faster than hipBLASLt's TN
        solutions at every Llama shape) when its tiling constraints hold."""
        if a.is_cuda and a.stride(0) == 1 and ops.gemm_tn_ok(a.t(), b, out):
            ops.gemm_tn_(a.t(), b, out, accumulate)
            return
        if accumulate:
            out.addmm_(a, b)
        else:
            torch.mm(a, b, out=out)

    @staticmethod
    def _mm_dx(dy, w):
        """Activation gradient dy . w for w [N, K] row-major.  On the GPU w is first
        transposed into scratch (ops/csrc/transpose.hip) so hipBLASLt sees the forward's
        operand layout (dy . (w^T)^T), whose solutions run 10-30 % faster at the Llama shapes
        than the plain "dy . w" ones; the copy costs one streaming pass over w."""
        if _DX_T and dy.is_cuda and ops.transpose_ok(w):
            return torch.mm(dy, ops.transpose(w).t())
        return torch.mm(dy, w)

    def _mm_into2(self, p0, p1, accumulate):
        """Two dW products ``(out, a, b)`` of one layer half: one grouped launch of the dW
        kernel when both fit it (fills each other's partial last wave), else two calls."""
        (o0, a0, b0), (o1, a1, b1) = p0, p1
        if (a0.is_cuda and a0.stride(0) == 1 and a1.stride(0) == 1 and a0.shape[1] == a1.shape[1]
                and ops.gemm_tn_ok(a0.t(), b0, o0) and ops.gemm_tn_ok(a1.t(), b1, o1)):
            ops.gemm_tn2_(a0.t(), b0, o0, a1.t(), b1, o1, accumulate)
            return
        self._mm_into(o0, a0, b0, accumulate)
        self._mm_into(o1, a1, b1, accumulate)

    def set_context_parallel(self, group, size: int, rank: int):
        assert self.hq % size == 0 and self.hkv % size == 0, \
            f"context parallelism needs the (per-TP-rank) heads {self.hq}/{self.hkv} divisible by cp={size}"
        self.cp, self.cp_rank, self.cp_group = size, rank, group

    # ------------------------------------------------------------------ TP / SP collectives
    @property
    def _sp(self) -> bool:
        return self.sequence_parallel and self.tp > 1

    def _gather(self, x):
        """SP: this rank's token rows -> all rows (identity without SP)."""
        return tp_all_gather_rows(x, self.st, self.tp_comm_chunks) if self._sp else x

    def _reduce_out(self, x):
        """Partial sums of a row-parallel product: SP -> this rank's rows (reduce-scatter),
        else all rows (all-reduce; a no-op at tp 1)."""
        return tp_reduce_scatter_rows(x, self.st, self.tp_comm_chunks) if self._sp else tp_all_reduce(x, self.st)

    def _reduce_out_async(self, x):
        """:meth:`_reduce_out` launched asynchronously on the TP communicator's stream; returns
        (result, handles) -- :meth:`_finish` makes the compute stream wait for them.  The
        backward overlaps its input-gradient reductions with the weight-gradient GEMMs that do
        not need them (at TP=8 over xGMI each all-reduce costs several times its producing GEMM)."""
        if self.tp == 1:
            return x, []
        if self._sp:
            return tp_reduce_scatter_rows(x, self.st, self.tp_comm_chunks, async_op=True)
        return x, [tp_all_reduce_work(x, self.st)]

    @staticmethod
    def _finish(pending):
        y, works = pending
        for w in works:
            w.wait()
        return y

    def _row_parallel(self, x, W):
        """Forward of a row-parallel projection: (x W^T) reduced over the TP group, in
        ``tp_comm_chunks`` token chunks so the reduction of chunk k overlaps the GEMM of chunk
        k+1 (each chunk's rows are complete products: the same values as one big GEMM)."""
        T = x.shape[0]
        c = _chunk_rows(T, self.tp_comm_chunks, self.tp)
        if self.tp == 1 or c == 1:
            return self._reduce_out(torch.mm(x, W.t()))
        n, tp = T // c, self.tp
        works, keep = [], []
        if self._sp:
            out = torch.empty((T // tp, W.shape[0]), dtype=x.dtype, device=x.device)
            for k in range(c):
                yk = torch.mm(x[k * n:(k + 1) * n], W.t())
                keep.append(yk)               # alive until its reduce-scatter has run
                works.append(tp_reduce_scatter_into(out[k * n // tp:(k + 1) * n // tp], yk, self.st))
        else:
            out = torch.empty((T, W.shape[0]), dtype=x.dtype, device=x.device)
            for k in range(c):
                torch.mm(x[k * n:(k + 1) * n], W.t(), out=out[k * n:(k + 1) * n])
                works.append(tp_all_reduce_work(out[k * n:(k + 1) * n], self.st))
        for w in works:
            w.wait()
        return out

    def _col_parallel(self, a, W):
        """Forward of a column-parallel projection on the SP-gathered input: chunk k's GEMM
        starts as soon as chunk k's all-gather has landed, while the later chunks are still on
        the wire.  Without SP the input is already complete: one GEMM."""
        if not self._sp:
            return torch.mm(a, W.t())
        full, works = tp_all_gather_rows(a, self.st, self.tp_comm_chunks, async_op=True)
        c = len(works)
        if c == 1:
            works[0].wait()
            return torch.mm(full, W.t())
        n = full.shape[0] // c
        out = torch.empty((full.shape[0], W.shape[0]), dtype=a.dtype, device=a.device)
        for k in range(c):
            works[k].wait()
            torch.mm(full[k * n:(k + 1) * n], W.t(), out=out[k * n:(k + 1) * n])
        return out

    def _norm_bwd(self, dy, h, rstd, name: str, accumulate: bool, dres=None):
        """K1 backward.  Under SP each rank sees 1/tp of the rows, so the norm weight gradient
        is a partial sum: it goes to a scratch row and is all-reduced (fp32) over the TP group
        at the end of the stage's backward (:meth:`_sp_finish_norms`)."""
        if not self._sp:
            return ops.rmsnorm_bwd(dy, h, rstd, self.P(name), self.G(name), accumulate, dres=dres)
        part = torch.empty_like(self.G(name))
        dh = ops.rmsnorm_bwd(dy, h, rstd, self.P(name), part, False, dres=dres)
        self._sp_norm_parts.append((name, part, accumulate))
        return dh

    def _sp_finish_norms(self):
        if not self._sp_norm_parts:
            return
        parts, self._sp_norm_parts = self._sp_norm_parts, []
        tot = torch.stack([p.float() for _, p, _ in parts])
        dist.all_reduce(tot, group=self.st.tp_group)
        for k, (name, _, acc) in enumerate(parts):
            G = self.G(name)
            G.copy_(tot[k] + G.float() if acc else tot[k])

    # ------------------------------------------------------------------ embedding
    def embed_fwd(self, tokens: torch.Tensor) -> torch.Tensor:
        """K7 gather (vocab-parallel: rows outside this rank's shard are zero, then summed)."""
        x = ops.embed_fwd(tokens, self.P("embed"), self.vstart if self.tp > 1 else 0)
        return self._reduce_out(x) if self.tp > 1 else x

    def embed_bwd(self, tokens: torch.Tensor, g: torch.Tensor, accumulate: bool):
        """K7 scatter-add straight into the flat gradient buffer's embedding slice."""
        g = self._gather(g)
        ops.embed_bwd_(tokens, g, self.G("embed"), self.vstart if self.tp > 1 else 0, accumulate)
        self._ready(self.mats, "embed")

    # ------------------------------------------------------------------ decoder layer
    def layer_fwd(self, i: int, r: torch.Tensor, d: Optional[torch.Tensor], B: int, S: int):
        return _run(self._layer_fwd_steps(i, r, d, B, S, interleave=False))

    def _layer_fwd_steps(self, i: int, r: torch.Tensor, d: Optional[torch.Tensor], B: int, S: int,
                         interleave: bool):
        """One decoder layer's forward as a generator.  ``interleave=False``: never yields (the
        TP collectives overlap their own GEMM chunks, :meth:`_row_parallel`).  ``interleave=True``:
        each TP collective is launched asynchronously and the generator yields right after, so a
        caller alternating two independent half-batches (:meth:`stage_forward_dual`) runs one
        half's GEMMs / attention while the other half's reduction is on the wire."""
        cfg = self.cfg
        c = _LayerCtx()
        a, h1, rstd1 = ops.rmsnorm_fwd(r, self.P(f"l{i}.norm1"), cfg.norm_eps, residual=d)
        if interleave and self._sp:
            pend = tp_all_gather_rows(a, self.st, self.tp_comm_chunks, async_op=True)
            yield
            qkv = torch.mm(self._finish(pend), self.P(f"l{i}.wqkv").t())
        else:
            qkv = self._col_parallel(a, self.P(f"l{i}.wqkv"))
        D, cp = cfg.head_dim, self.cp
        hq, hkv, Sa = self.hq // cp, self.hkv // cp, S * cp
        if cp > 1:   # own tokens x all heads -> all tokens x own head group
            qkv = cpx.to_heads(qkv, B, S, [self.hq * D, self.hkv * D, self.hkv * D], cp, self.cp_group)
        ops.rope_(qkv, hq + hkv, D, self.cos, self.sin, seq_len=Sa)
        o, lse = attention_fwd(qkv, B, Sa, hq, hkv, D)
        o_tok = cpx.to_tokens(o, B, S, [hq * D], cp, self.cp_group) if cp > 1 else o
        if interleave:
            pend = self._reduce_out_async(torch.mm(o_tok, self.P(f"l{i}.wo").t()))
            yield
            da = self._finish(pend)
        else:
            da = self._row_parallel(o_tok, self.P(f"l{i}.wo"))
        m, h2, rstd2 = ops.rmsnorm_fwd(h1, self.P(f"l{i}.norm2"), cfg.norm_eps, residual=da)
        del da
        if interleave and self._sp:
            pend = tp_all_gather_rows(m, self.st, self.tp_comm_chunks, async_op=True)
            yield
            gu = torch.mm(self._finish(pend), self.P(f"l{i}.wgu").t())
        else:
            gu = self._col_parallel(m, self.P(f"l{i}.wgu"))
        s = ops.swiglu_fwd(gu)
        if interleave:
            pend = self._reduce_out_async(torch.mm(s, self.P(f"l{i}.wd").t()))
            yield
            dm = self._finish(pend)
        else:
            dm = self._row_parallel(s, self.P(f"l{i}.wd"))
        c.h1, c.rstd1, c.a, c.qkv, c.o, c.o_tok, c.lse = h1, rstd1, a, qkv, o, o_tok, lse
        c.h2, c.rstd2, c.m, c.gu, c.s = h2, rstd2, m, gu, s
        return h2, dm, c

    def layer_bwd(self, i: int, c: _LayerCtx, g: torch.Tensor, B: int, S: int, accumulate: bool):
        cfg = self.cfg
        Wd, Wgu, Wo, Wqkv = (self.P(f"l{i}.{n}") for n in ("wd", "wgu", "wo", "wqkv"))
        # The four weight gradients run as two grouped dW launches whose tile counts fill whole
        # waves of the 256 CUs: {wgu, wo} (7 + 1 waves at Llama-3-8B) as soon as dh2 exists,
        # {wd, wqkv} (3.5 + 1.5) at the end -- separately, wd and wqkv each end on a half wave.
        # Under SP, g / dh2 / the saved norm outputs a, m are this rank's token rows: the GEMMs
        # read their all-gathered forms (the backward of a reduce-scatter is an all-gather) and
        # the input gradients of the column-parallel GEMMs are reduce-scattered.
        # MLP
        gf = self._gather(g)
        gs = self._mm_dx(gf, Wd)
        dgu = ops.swiglu_bwd(c.gu, gs)
        del gs
        c.gu = None
        if self.tp == 1:
            dmm = self._mm_dx(dgu, Wgu)
            dh2 = self._norm_bwd(dmm, c.h2, c.rstd2, f"l{i}.norm2", accumulate, dres=g)
            del dmm
            dh2f = dh2
            self._mm_into2((self.G(f"l{i}.wgu"), dgu.t(), c.m), (self.G(f"l{i}.wo"), dh2f.t(), c.o_tok), accumulate)
        else:
            # TP: the dmm reduction runs while the wgu weight gradient (which does not need it)
            # is computed; SP gathers m before the reduce-scatter goes out on the communicator
            mf = self._gather(c.m)
            pend = self._reduce_out_async(self._mm_dx(dgu, Wgu))
            self._mm_into(self.G(f"l{i}.wgu"), dgu.t(), mf, accumulate)
            del mf
            dmm = self._finish(pend)
            dh2 = self._norm_bwd(dmm, c.h2, c.rstd2, f"l{i}.norm2", accumulate, dres=g)
            del dmm, pend
            dh2f = self._gather(dh2)
            self._mm_into(self.G(f"l{i}.wo"), dh2f.t(), c.o_tok, accumulate)
        del dgu
        # attention (context parallel: the same all-to-alls as forward, in reverse roles)
        D, cp = cfg.head_dim, self.cp
        hq, hkv, Sa = self.hq // cp, self.hkv // cp, S * cp
        do = self._mm_dx(dh2f, Wo)
        del dh2f
        if cp > 1:
            do = cpx.to_heads(do, B, S, [self.hq * D], cp, self.cp_group)
        dqkv = attention_bwd(c.qkv, c.o, c.lse, do, B, Sa, hq, hkv, D)
        del do
        ops.rope_(dqkv, hq + hkv, D, self.cos, self.sin, seq_len=Sa, inverse=True)
        if cp > 1:
            dqkv = cpx.to_tokens(dqkv, B, S, [hq * D, hkv * D, hkv * D], cp, self.cp_group)
        af = self._gather(c.a)
        pend = self._reduce_out_async(self._mm_dx(dqkv, Wqkv))     # overlaps the two dW GEMMs below
        self._mm_into2((self.G(f"l{i}.wd"), gf.t(), c.s), (self.G(f"l{i}.wqkv"), dqkv.t(), af), accumulate)
        da = self._finish(pend)
        c.s = None
        del dqkv, gf, af, pend
        dh1 = self._norm_bwd(da, c.h1, c.rstd1, f"l{i}.norm1", accumulate, dres=dh2)
        self._ready(self.mats, f"l{i}.wqkv")
        return dh1

    # ------------------------------------------------------------------ LM head + CE
    def head_fwd(self, r, d, labels: torch.Tensor, scale: float):
        """Final RMSNorm only.  Returns (loss, ctx): ``loss`` is a 0-d fp32 device tensor that
        :meth:`head_bwd` fills in (already multiplied by ``scale``) -- the logits are produced,
        consumed and discarded chunk by chunk there (K5), never as one [T, vocab] buffer.
        Until then it holds NaN, so a caller that reads it without running the backward gets an
        unmistakable value, never a plausible 0; forward-only callers use :meth:`head_loss`."""
        cfg = self.cfg
        y, h, rstd = ops.rmsnorm_fwd(r, self.P("final_norm"), cfg.norm_eps, residual=d)
        loss = torch.full((), float("nan"), device=y.device, dtype=torch.float32)
        return loss, (h, rstd, y, labels, scale, loss)

    @torch.no_grad()
    def head_loss(self, ctx) -> torch.Tensor:
        """Forward-only K5: the chunked LM head + CE loss (times ``scale``) without gradients --
        evaluation and any caller that wants the loss without a backward pass."""
        h, rstd, y, labels, scale, _ = ctx
        y = self._gather(y)
        W = self.P("lm_head")
        T = y.shape[0]
        tc = self.head_chunk if self.head_chunk and self.head_chunk < T else T
        tot = None
        for c0 in range(0, T, tc):
            c1 = min(T, c0 + tc)
            rows = self._ce_chunk(torch.mm(y[c0:c1], W.t()), labels[c0:c1], scale)
            tot = rows.sum() if tot is None else tot + rows.sum()
        return (tot * scale).float()

    def _ce_chunk(self, logits, labels, scale):
        """Cross-entropy of one row chunk: loss rows (fp32); ``logits`` now hold dlogits."""
        if self.tp == 1:
            loss_rows, _ = ops.cross_entropy_fused_(logits, labels, scale)
            return loss_rows
        m, s, xy = ops.cross_entropy_stats(logits, labels, self.vstart)
        M = m.clone()
        dist.all_reduce(M, op=dist.ReduceOp.MAX, group=self.st.tp_group)
        s = s * torch.exp(m - M)
        sx = torch.stack([s, xy])
        dist.all_reduce(sx, group=self.st.tp_group)
        lse = M + torch.log(sx[0])
        ops.cross_entropy_grad_(logits, labels, lse, scale, self.vstart)
        return torch.where(labels != -100, lse - sx[1], torch.zeros_like(lse))

    def head_bwd(self, ctx, accumulate: bool):
        """Row-chunked LM head + CE (K5): per chunk of ``head_chunk`` tokens, logits = y W^T
        (one [chunk, vocab] slab), the fused CE kernel turns them into dlogits in place and
        writes the loss rows, dy = dlogits W and dW_head (+)= dlogits^T y; the slab is then
        reused by the next chunk.  At Llama-3-8B, micro-batch 2 x 8192 that replaces a 4.2 GB
        [16384, 128256] buffer by a 1.05 GB one.  The weight is transposed once per step for
        the dy products (forward operand layout, see _mm_dx).  dW_head is accumulated across
        chunks by the dW kernel (bf16 output, fp32 inside each chunk)."""
        h, rstd, y, labels, scale, loss = ctx
        y = self._gather(y)
        W = self.P("lm_head")
        T = y.shape[0]
        tc = self.head_chunk if self.head_chunk and self.head_chunk < T else T
        Wt = ops.transpose(W) if (_DX_T and y.is_cuda and ops.transpose_ok(W)) else None
        dy = torch.empty_like(y)
        tot = None
        for c0 in range(0, T, tc):
            c1 = min(T, c0 + tc)
            yc = y[c0:c1]
            logits = torch.mm(yc, W.t())
            rows = self._ce_chunk(logits, labels[c0:c1], scale)
            tot = rows.sum() if tot is None else tot + rows.sum()
            if Wt is not None:
                torch.mm(logits, Wt.t(), out=dy[c0:c1])
            else:
                torch.mm(logits, W, out=dy[c0:c1])
            self._mm_into(self.G("lm_head"), logits.t(), yc, accumulate or c0 > 0)
            del logits, rows
        loss.copy_(tot * scale)
        del Wt
        dy = self._reduce_out(dy)
        self._ready(self.mats, "lm_head")
        dh = self._norm_bwd(dy, h, rstd, "final_norm", accumulate)
        return dh

    # ------------------------------------------------------------------ stage-level API
    def _wait(self, first: str, last: str, group: Optional[FlatGroup] = None):
        """Tell the ZeRO-1 engine that params ``first``..``last`` (one contiguous range of
        one flat group, reverse-registration order) are about to be read."""
        if self.param_wait is None:
            return
        g = group or self.mats
        lo = g.spec(first).offset
        self.param_wait(g, lo, g.end_offset(last))

    def param_segments(self):
        """Forward-ordered parameter ranges ``(group, lo, hi)``: exactly the ranges the
        forward's ``param_wait`` hook asks for (embedding, per-layer matrices / norms, head)."""
        segs = []
        rng = lambda g, a, b: (g, g.spec(a).offset, g.end_offset(b))  # noqa: E731
        if self.first:
            segs.append(rng(self.mats, "embed", "embed"))
        for i in self.layers:
            segs.append(rng(self.mats, f"l{i}.wd", f"l{i}.wqkv"))
            segs.append(rng(self.norms, f"l{i}.norm2", f"l{i}.norm1"))
        if self.last:
            segs.append(rng(self.mats, "lm_head", "lm_head"))
            segs.append(rng(self.norms, "final_norm", "final_norm"))
        return segs

    def _wait_layer(self, i: int):
        if self.param_wait is not None:
            self._wait(f"l{i}.wd", f"l{i}.wqkv")
            self._wait(f"l{i}.norm2", f"l{i}.norm1", self.norms)

    def stage_forward(self, inp, B: int, S: int, labels=None, scale: float = 1.0):
        """inp: tokens [B*S] (first stage) or activation [B*S, H].  Returns (out, ctx) where
        out is the loss (last stage) or the activation handed to the next stage.  The last
        stage's loss is computed by :meth:`stage_backward` (K5 fuses it with the head's
        gradient) and is NaN until then; :meth:`forward_loss` is the forward-only form."""
        ctx = {"layers": []}
        if self._sp:
            assert (B * S) % self.tp == 0, f"sequence parallelism needs B*S divisible by tp ({B}x{S}, tp {self.tp})"
        if self.first:
            ctx["tokens"] = inp
            self._wait("embed", "embed")
            r, d = self.embed_fwd(inp), None
        else:
            r, d = inp, None
        for i in self.layers:
            self._wait_layer(i)
            if self.recompute:
                inp = (r, d)
                r, d, _ = self.layer_fwd(i, r, d, B, S)
                ctx["layers"].append(inp)
            else:
                r, d, c = self.layer_fwd(i, r, d, B, S)
                ctx["layers"].append(c)
        if self.last:
            self._wait("lm_head", "lm_head")
            self._wait("final_norm", "final_norm", self.norms)
            loss, hctx = self.head_fwd(r, d, labels, scale)
            ctx["head"] = hctx
            return loss, ctx
        out = r + d if d is not None else r
        return out, ctx

    def stage_forward_dual(self, tokens, labels, B: int, S: int, scale: float):
        """Forward of one micro-batch ``tokens``/``labels`` [B*S] (single-stage model, TP > 1,
        no SP, B even) as two half-batches whose layers are interleaved at every TP collective:
        half A's all-reduce is on the wire while half B's GEMMs and attention run, and the other
        way round -- at TP=8 over xGMI each forward reduction costs several times its producing
        GEMM, so this hides what the chunked form cannot.  The halves' saved activations are then
        concatenated into ONE full-batch context (rows in batch order) and the head runs once, so
        the caller does one :meth:`stage_backward` as for the plain forward: no second backward,
        no extra gradient accumulation.  Returns (loss placeholder, ctx)."""
        assert self.first and self.last and not self._sp and B % 2 == 0
        Bh, T = B // 2, B * S
        half = T // 2
        self._wait("embed", "embed")
        state = [(self.embed_fwd(tokens[:half]), None), (self.embed_fwd(tokens[half:]), None)]
        ctx = {"layers": [], "tokens": tokens}
        for i in self.layers:
            self._wait_layer(i)
            res = _interleave([self._layer_fwd_steps(i, r, d, Bh, S, interleave=True) for r, d in state])
            (r0, d0, c0), (r1, d1, c1) = res
            c = _LayerCtx()
            for f in _LayerCtx.__slots__:
                x0, x1 = getattr(c0, f), getattr(c1, f)
                if f == "o_tok" and x0 is c0.o:
                    setattr(c, f, None)           # aliases o (set below)
                else:
                    setattr(c, f, torch.cat([x0, x1], 0))
            if c.o_tok is None:
                c.o_tok = c.o
            del c0, c1, res
            ctx["layers"].append(c)
            state = [(r0, d0), (r1, d1)]
        (r0, d0), (r1, d1) = state
        r = torch.cat([r0, r1], 0)
        d = torch.cat([d0, d1], 0) if d0 is not None else None
        del state, r0, r1, d0, d1
        self._wait("lm_head", "lm_head")
        self._wait("final_norm", "final_norm", self.norms)
        loss, ctx["head"] = self.head_fwd(r, d, labels, scale)
        return loss, ctx

    def stage_backward(self, ctx, grad_out: Optional[torch.Tensor], B: int, S: int,
                       accumulate: bool):
        """grad_out: None on the last stage (loss), else d(out).  Returns d(inp) or None."""
        if self.last:
            g = self.head_bwd(ctx.pop("head"), accumulate)
        else:
            g = grad_out
        layers = ctx["layers"]
        for i in reversed(self.layers):
            c = layers.pop()
            if self.recompute:
                r, d = c
                _, _, c = self.layer_fwd(i, r, d, B, S)   # same kernels, same inputs: same values
                del r, d
            g = self.layer_bwd(i, c, g, B, S, accumulate)
            del c
        if self.first:
            self.embed_bwd(ctx["tokens"], g, accumulate)
            g = None
        self._sp_finish_norms()
        return g

    def forward_backward(self, tokens: torch.Tensor, labels: torch.Tensor, accumulate: bool = False,
                         scale: Optional[float] = None):
        """Single-stage fused step: tokens/labels [B, S] -> loss (device scalar); grads
        written into the flat gradient buffers."""
        B, S = tokens.shape
        scale = scale if scale is not None else 1.0 / (B * S)
        loss, ctx = self.stage_forward(tokens.reshape(-1), B, S, labels.reshape(-1), scale)
        self.stage_backward(ctx, None, B, S, accumulate)
        return loss

    @torch.no_grad()
    def forward_loss(self, tokens: torch.Tensor, labels: torch.Tensor, scale: Optional[float] = None):
        """Mean next-token loss of tokens/labels [B, S] with no backward pass (evaluation)."""
        B, S = tokens.shape
        scale = scale if scale is not None else 1.0 / (B * S)
        _, ctx = self.stage_forward(tokens.reshape(-1), B, S, labels.reshape(-1), scale)
        return self.head_loss(ctx["head"])

    @torch.no_grad()
    def forward_logits(self, tokens: torch.Tensor) -> torch.Tensor:
        """Plain forward to logits [B, S, V_local] (evaluation / tests)."""
        B, S = tokens.shape
        r, d = self.embed_fwd(tokens.reshape(-1)), None
        for i in self.layers:
            r, d, _ = self.layer_fwd(i, r, d, B, S)
        y, _, _ = ops.rmsnorm_fwd(r, self.P("final_norm"), self.cfg.norm_eps, residual=d)
        return torch.mm(self._gather(y), self.P("lm_head").t()).view(B, S, -1)
