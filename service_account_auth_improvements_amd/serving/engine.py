"""Llama-3 inference engine for the InferenceService predictor (BASELINE configs[2]).

MI355X-first design:

* Weights live in the same flat bf16 buffer the trainer uses (``Llama.allocate(grads=False)``)
  so a training checkpoint loads with zero re-layout.
* KV cache: one slot-major tensor per layer, ``[n_slots, Hkv, max_len, 128]`` bf16.  Slots
  are preallocated at full context length -- 288 GB of HBM holds ~2M tokens of Llama-3-8B
  KV (128 KB/token) -- so there is no paging indirection on the memory-bound decode path.
* Prefill runs the training forward kernels (fused residual+RMSNorm, fused QKV GEMM, in-place
  RoPE, MFMA flash attention, SwiGLU) and streams K/V into the slot with ``kv_fill_``.
* Decode appends K/V (``kv_append_``) and runs the split-K GQA decode kernel (K8); for
  batches <= 16 the projections use the weight-streaming skinny GEMM (ops/csrc/skinny_gemm.hip,
  gate/up GEMM fused with SwiGLU), larger batches hipBLASLt.  For batches <= 8 the two
  residual-add + RMSNorms of a layer are the QKV and gate/up GEMMs' prologues (no norm
  launches on the decode path).  Every
  decode step for a batch-size bucket is captured once in a HIP graph (static input
  buffers, padded rows point at a scratch slot), so a token costs one graph launch instead
  of ~350 kernel launches.
* Continuous batching: ``Scheduler`` admits requests into free slots between decode steps
  (prefill one sequence at a time), retires finished sequences immediately.
* TP > 1 (one process per GPU): Megatron split; prefill all-reduces over RCCL, the decode
  step's [B, hidden] all-reduces one-shot over peer-mapped IPC buffers (xGMI, one hop,
  graph-capturable: parallel/custom_ar.py); vocab-parallel logits are all-gathered for
  sampling.
"""
from __future__ import annotations

import math
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from .. import ops
from ..models.llama import Llama, LlamaConfig
from ..ops.attention import attention_fwd, decode_attention, kv_fill_, rope_append_, rope_append_parts
from ..parallel.state import ParallelState, tp_all_reduce

BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128, 256)
# decode batches up to this use the weight-streaming skinny GEMM (KFAMD_SKINNY_MAX_ROWS: A/B, <= 64)
SKINNY_MAX_ROWS = min(64, int(os.environ.get("KFAMD_SKINNY_MAX_ROWS", "16")))
SKINNY_MAX_N = 32768          # beyond this (LM head) hipBLASLt streams faster than the MFMA skinny kernel
GEMV_MAX_ROWS = 4             # ... but not than the VALU GEMV (ops/csrc/gemv.hip) the 1-4 row case takes
# above SKINNY_MAX_ROWS the narrow projections (N <= 4096: wo, wd) go to the batched-decode GEMM
# (ops/csrc/bgemm.hip: W streamed into registers, K split over the CUs) up to BGEMM_MAX_ROWS;
# hipBLASLt's tiles leave most CUs idle there.  The wide ones (wqkv ties, gate/up and the LM
# head lose) stay on hipBLASLt (profiles/serve_bgemm.md).  KFAMD_BGEMM=0: off.
BGEMM = os.environ.get("KFAMD_BGEMM", "1") != "0"
BGEMM_MAX_N = 4096
BGEMM_MIN_ROWS, BGEMM_MAX_ROWS = 33, 128   # at 32 rows its reduce launch costs more than it saves
# the K-split partials of the wo / wd batched-decode GEMMs go straight into the RMSNorm that
# consumes the residual branch (ops.rmsnorm_fwd_parts), without the separate reduce launch;
# KFAMD_DECODE_FUSE_SPLITS=0: reduce launch + plain RMSNorm (A/Bs)
FUSE_SPLITS = os.environ.get("KFAMD_DECODE_FUSE_SPLITS", "1") != "0"
# ... and the qkv projection on the batched-decode GEMM with its partials summed inside the RoPE /
# KV-append launch (KFAMD_DECODE_FUSE_QKV=0: hipBLASLt + rope_append_)
FUSE_QKV = os.environ.get("KFAMD_DECODE_FUSE_QKV", "1") != "0"
QKV_PARTS_MIN_ROWS = 65       # at 64 rows hipBLASLt's qkv GEMM is faster than this pair (+1 %, s18)
# prompts admitted in one scheduler iteration are prefilled together up to this many tokens
PREFILL_MAX_TOKENS = int(os.environ.get("KFAMD_PREFILL_MAX_TOKENS", "16384"))
PREFILL_PAD_RATIO = 1.25      # ... in length groups padded to at most 1.25x
# batches 1-4 run the same kernel-per-op graph as larger batches.  A whole-step persistent kernel
# (one launch per token, grid barriers between the layer phases) measured 3.54-3.65 ms/token at
# batch 1 against 3.15 for this graph and was moved out of the production library into
# tools/kbench/decode_step_lab.hip (profiles/decode_step_ablation_r4p.txt, docs/ROUND6.md).
# hipBLASLt/rocBLAS solutions for the decode GEMM shapes above SKINNY_MAX_ROWS where the library
# heuristic picks a poor kernel (tools/tune_decode_gemm.py; only the shapes that measured >= 5 %
# faster HBM-cold are kept, profiles/serve_large_batch.md).  Loaded into PyTorch TunableOp with
# tuning off; KFAMD_DECODE_TUNED=0 disables it, =<file> uses another results file.
TUNED_DECODE_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "decode_gemm_gfx950.csv")


def _load_tuned_decode_gemms(dev, cfg, tp: int) -> bool:
    path = os.environ.get("KFAMD_DECODE_TUNED", TUNED_DECODE_FILE)
    if dev.type != "cuda" or path == "0" or not os.path.exists(path):
        return False
    if path == TUNED_DECODE_FILE and (cfg.hidden, cfg.ffn, cfg.vocab_size, tp) != (4096, 14336, 128256, 1):
        return False                  # the shipped file holds Llama-3-8B TP=1 shapes only
    if torch.cuda.get_device_properties(dev).gcnArchName.split(":")[0] != "gfx950":
        return False
    import torch.cuda.tunable as tn
    tn.enable(True)
    tn.tuning_enable(False)           # never tune inside a serving process
    tn.read_file(path)
    return True


class _SplitSum:
    """A decode projection's output left as the batched-decode GEMM's fp32 K-split partials
    [S, M, N]; the RMSNorm that adds it to the residual stream sums them (:meth:`Engine._norm`)."""
    __slots__ = ("part",)

    def __init__(self, part):
        self.part = part

    def dense(self):
        d = self.part[0].clone()
        for t in range(1, self.part.shape[0]):
            d += self.part[t]
        return d.to(torch.bfloat16)


def _dense(d):
    return d.dense() if isinstance(d, _SplitSum) else d


class Engine:
    def __init__(self, model: Llama, n_slots: int = 64, max_len: int = 4096, use_graphs: Optional[bool] = None):
        self.m = model
        cfg = model.cfg
        self.cfg = cfg
        self.dev = model.device
        self.n_slots = n_slots + 1            # last slot = scratch for padded graph rows
        self.scratch = n_slots
        self.max_len = max_len
        assert max_len <= cfg.max_seq, "max_len exceeds the RoPE table"
        L = len(model.layers)
        shape = (L, self.n_slots, model.hkv, max_len, cfg.head_dim)
        self.kc = torch.zeros(shape, dtype=torch.bfloat16, device=self.dev)
        self.vc = torch.zeros(shape, dtype=torch.bfloat16, device=self.dev)
        self.use_graphs = (self.dev.type == "cuda") if use_graphs is None else use_graphs
        self.tuned_gemms = _load_tuned_decode_gemms(self.dev, cfg, model.tp)
        # TP > 1 on GPUs: the decode step's small all-reduces go one-shot over peer-mapped
        # IPC buffers (parallel/custom_ar.py, C7) instead of an RCCL ring
        self.car = None
        if model.tp > 1 and self.dev.type == "cuda":
            from ..parallel.custom_ar import OneShotAllReduce
            self.car = OneShotAllReduce(model.st.tp_group)
        self._graphs: Dict[int, tuple] = {}
        self._staging: Dict[int, tuple] = {}   # bucket -> (pinned host [3, Bb], device [3, Bb], copy-done event)

    # ------------------------------------------------------------------ helpers
    def _logits_full(self, y):
        m = self.m
        w = m.P("lm_head")
        if y.is_cuda and y.shape[0] <= GEMV_MAX_ROWS:
            logits = ops.skinny_gemm(y, w)      # VALU GEMV: streams the LM head faster than hipBLASLt
        else:
            logits = torch.mm(y, w.t())
        if m.tp > 1:
            parts = [torch.empty_like(logits) for _ in range(m.tp)]
            dist.all_gather(parts, logits, group=m.st.tp_group)
            logits = torch.cat(parts, -1)
        return logits

    def _embed(self, tokens):
        return self.m.embed_fwd(tokens)

    def _mlp(self, i, h1, da):
        m, cfg = self.m, self.cfg
        mm, h2, _ = ops.rmsnorm_fwd(h1, m.P(f"l{i}.norm2"), cfg.norm_eps, residual=da)
        s = ops.swiglu_fwd(torch.mm(mm, m.P(f"l{i}.wgu").t()))
        return h2, tp_all_reduce(torch.mm(s, m.P(f"l{i}.wd").t()), m.st)

    # ------------------------------------------------------------------ prefill
    @torch.no_grad()
    def prefill(self, slot: int, tokens: List[int]) -> torch.Tensor:
        """Run the prompt through the model, fill the slot's KV; returns last-position logits."""
        m, cfg = self.m, self.cfg
        S = len(tokens)
        assert 0 < S <= self.max_len
        Sp = S if self.dev.type != "cuda" else ((S + 127) // 128) * 128   # flash kernel tiles of 128
        tok = torch.zeros(Sp, dtype=torch.long, device=self.dev)
        tok[:S] = torch.tensor(tokens, dtype=torch.long, device=self.dev)
        r = self._embed(tok)
        d = None
        for li, i in enumerate(m.layers):
            a, h1, _ = ops.rmsnorm_fwd(r, m.P(f"l{i}.norm1"), cfg.norm_eps, residual=d)
            qkv = torch.mm(a, m.P(f"l{i}.wqkv").t())
            ops.rope_(qkv, m.hq + m.hkv, cfg.head_dim, m.cos, m.sin, seq_len=Sp)
            o, _ = attention_fwd(qkv, 1, Sp, m.hq, m.hkv, cfg.head_dim)
            kv_fill_(qkv, S, m.hq, slot, self.kc[li], self.vc[li])
            da = tp_all_reduce(torch.mm(o, m.P(f"l{i}.wo").t()), m.st)
            r, d = self._mlp(i, h1, da)
        y, _, _ = ops.rmsnorm_fwd(r[S - 1:S].contiguous(), m.P("final_norm"), cfg.norm_eps,
                                  residual=d[S - 1:S].contiguous())
        return self._logits_full(y)[0]

    @torch.no_grad()
    def prefill_batch(self, slots: List[int], prompts: List[List[int]]) -> torch.Tensor:
        """Several prompts in ONE pass: each is padded to the longest (rounded to the flash
        kernel's 128-row tiles) and the batch runs as B sequences of that length, so every
        projection is one GEMM over all B * Sp rows instead of B GEMMs over Sp rows (causal
        attention: the pad rows after a prompt never reach its real rows).  Fills every slot's
        KV; returns the last-position logits [B, V].  == ``prefill`` per prompt up to the
        GEMMs' row-count-dependent rounding."""
        m, cfg = self.m, self.cfg
        n = len(prompts)
        assert n == len(slots) and n > 0
        lens = [len(t) for t in prompts]
        assert 0 < min(lens) and max(lens) <= self.max_len
        Sp = max(lens) if self.dev.type != "cuda" else ((max(lens) + 127) // 128) * 128
        tok = torch.zeros(n, Sp, dtype=torch.long)
        for b, t in enumerate(prompts):
            tok[b, :len(t)] = torch.tensor(t, dtype=torch.long)
        r = self._embed(tok.reshape(-1).to(self.dev))
        d = None
        for li, i in enumerate(m.layers):
            a, h1, _ = ops.rmsnorm_fwd(r, m.P(f"l{i}.norm1"), cfg.norm_eps, residual=d)
            qkv = torch.mm(a, m.P(f"l{i}.wqkv").t())
            ops.rope_(qkv, m.hq + m.hkv, cfg.head_dim, m.cos, m.sin, seq_len=Sp)   # position = row % Sp
            o, _ = attention_fwd(qkv, n, Sp, m.hq, m.hkv, cfg.head_dim)
            for b in range(n):
                kv_fill_(qkv[b * Sp:(b + 1) * Sp], lens[b], m.hq, slots[b], self.kc[li], self.vc[li])
            da = tp_all_reduce(torch.mm(o, m.P(f"l{i}.wo").t()), m.st)
            r, d = self._mlp(i, h1, da)
        last = torch.tensor([b * Sp + lens[b] - 1 for b in range(n)], device=self.dev)
        y, _, _ = ops.rmsnorm_fwd(r.index_select(0, last), m.P("final_norm"), cfg.norm_eps,
                                  residual=d.index_select(0, last))
        return self._logits_full(y)

    # ------------------------------------------------------------------ decode
    def _tp_ar(self, x):
        if self.car is not None and self.car.supports(x):
            return self.car(x)
        return tp_all_reduce(x, self.m.st)

    def _use_bgemm(self, x, w) -> bool:
        # measured at TP=1 (a TP shard's K of 512-1792 leaves too few K stages to split); above
        # BGEMM_MAX_ROWS only the deep narrow projection (wd, K = 14336) gains, with two W tiles
        # per wave: 53 vs 62 us at 256 rows (wo loses: 28 vs 24; profiles/serve_bgemm_wt_r5.md)
        rows = x.shape[0]
        in_range = (max(SKINNY_MAX_ROWS + 1, BGEMM_MIN_ROWS) <= rows <= BGEMM_MAX_ROWS
                    or (BGEMM_MAX_ROWS < rows <= 256 and w.shape[1] >= 8192))
        return BGEMM and self.m.tp == 1 and in_range and w.shape[0] <= BGEMM_MAX_N and ops.bgemm_ok(x, w)

    def _mm(self, x, w):
        """Decode GEMM: the skinny weight-streaming kernels for small batches on the GPU, the
        batched-decode GEMM up to 256 rows, hipBLASLt beyond."""
        # 9-16 rows, deep narrow weights (wd: K = 14336, N = 4096): the skinny kernel's 256
        # workgroups walk K in 7 serial rounds; the batched-decode GEMM splits K over the CUs
        # (batch 16: 5.43 -> 5.30 ms per step; batch 8 and the K = 4096 projections: no gain or
        # worse, profiles/serve_gemv_upfront_loads_r4.txt)
        if (x.is_cuda and 8 < x.shape[0] <= SKINNY_MAX_ROWS and w.shape[1] >= 8192 and BGEMM and self.m.tp == 1
                and w.shape[0] <= BGEMM_MAX_N and ops.bgemm_ok(x, w)):
            return ops.bgemm(x, w)
        if x.is_cuda and (x.shape[0] <= GEMV_MAX_ROWS or (
                x.shape[0] <= SKINNY_MAX_ROWS and w.shape[0] <= SKINNY_MAX_N and w.shape[1] % 256 == 0)):
            return ops.skinny_gemm(x, w)
        if self._use_bgemm(x, w):
            return ops.bgemm(x, w)
        return torch.mm(x, w.t())

    def _mm_res(self, x, w):
        """A projection whose output only feeds the next residual add + RMSNorm: with the
        batched-decode GEMM at a K split, its fp32 partials (:class:`_SplitSum`), no reduce launch."""
        if FUSE_SPLITS and x.is_cuda and self._use_bgemm(x, w):
            y = ops.bgemm_parts(x, w)
            return _SplitSum(y) if y.dim() == 3 else y
        return self._tp_ar(self._mm(x, w))

    def _qkv_parts(self, a, w):
        """The qkv projection at 65-128 rows: the batched-decode GEMM's fp32 partials for
        rope_append_parts (its K split's reduce folded into that launch), else the bf16 product.
        Unfused, hipBLASLt ties the batched-decode GEMM here (profiles/serve_bgemm.md)."""
        rows = a.shape[0]
        if (FUSE_SPLITS and FUSE_QKV and a.is_cuda and BGEMM and self.m.tp == 1
                and QKV_PARTS_MIN_ROWS <= rows <= BGEMM_MAX_ROWS and ops.bgemm_ok(a, w)):
            return ops.bgemm_parts(a, w)
        return self._mm(a, w)

    def _norm(self, x, w, d):
        """Residual add + RMSNorm; ``d`` may be a projection's unreduced partials."""
        if isinstance(d, _SplitSum):
            return ops.rmsnorm_fwd_parts(x, d.part, w, self.cfg.norm_eps)
        return ops.rmsnorm_fwd(x, w, self.cfg.norm_eps, residual=d)

    def _decode_mlp(self, i, h1, da):
        m, cfg = self.m, self.cfg
        wgu = m.P(f"l{i}.wgu")
        if ops.skinny_gemm_norm_ok(h1, wgu.shape[1]):
            # residual add + RMSNorm + gate/up GEMM + SwiGLU: one kernel
            s, h2 = ops.skinny_gemm_norm(h1, _dense(da), m.P(f"l{i}.norm2"), cfg.norm_eps, wgu, swiglu=True)
            return h2, self._mm_res(s, m.P(f"l{i}.wd"))
        mm, h2, _ = self._norm(h1, m.P(f"l{i}.norm2"), da)
        if mm.is_cuda and (mm.shape[0] <= GEMV_MAX_ROWS or (mm.shape[0] <= SKINNY_MAX_ROWS and wgu.shape[1] % 256 == 0)):
            s = ops.skinny_gemm(mm, wgu, swiglu=True)          # gate/up GEMM + SwiGLU in one kernel
        elif mm.is_cuda and self._use_bgemm(mm, wgu):
            s = ops.bgemm(mm, wgu, swiglu=True)
        else:
            s = ops.swiglu_fwd(torch.mm(mm, wgu.t()))
        return h2, self._mm_res(s, m.P(f"l{i}.wd"))

    def _decode_body(self, tokens, slots, pos, lengths):
        m, cfg = self.m, self.cfg
        r = self._embed(tokens)
        d = None
        for li, i in enumerate(m.layers):
            wqkv = m.P(f"l{i}.wqkv")
            if ops.gemv_norm_rope_ok(r, wqkv.shape[1], cfg.head_dim):
                # residual add + RMSNorm + qkv GEMV + RoPE + KV-cache append: one kernel
                qkv, h1 = ops.gemv_norm_rope(r, _dense(d), m.P(f"l{i}.norm1"), cfg.norm_eps, wqkv, m.hq, m.cos,
                                             m.sin, slots, pos, self.kc[li], self.vc[li])
            else:
                if ops.skinny_gemm_norm_ok(r, wqkv.shape[1]):
                    qkv, h1 = ops.skinny_gemm_norm(r, _dense(d), m.P(f"l{i}.norm1"), cfg.norm_eps, wqkv)
                else:
                    a, h1, _ = self._norm(r, m.P(f"l{i}.norm1"), d)
                    qkv = self._qkv_parts(a, wqkv)
                if qkv.dim() == 3:      # K-split partials: summed inside the RoPE / append launch
                    qkv = rope_append_parts(qkv, m.hq, m.cos, m.sin, slots, pos, self.kc[li], self.vc[li])
                else:
                    rope_append_(qkv, m.hq, m.cos, m.sin, slots, pos, self.kc[li], self.vc[li])
            o = decode_attention(qkv, self.kc[li], self.vc[li], slots, lengths, m.hq)
            da = self._mm_res(o, m.P(f"l{i}.wo"))
            r, d = self._decode_mlp(i, h1, da)
        y, _, _ = self._norm(r, m.P("final_norm"), d)
        return self._logits_full(y)

    def _graph_for(self, Bb: int):
        g = self._graphs.get(Bb)
        if g is not None:
            return g
        dev = self.dev
        tokens = torch.zeros(Bb, dtype=torch.long, device=dev)
        slots = torch.full((Bb,), self.scratch, dtype=torch.int32, device=dev)
        pos = torch.zeros(Bb, dtype=torch.int32, device=dev)
        lengths = torch.ones(Bb, dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):          # warm-up (allocator, hipBLASLt heuristics)
            for _ in range(2):
                self._decode_body(tokens, slots, pos, lengths)
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = self._decode_body(tokens, slots, pos, lengths)
        g = (graph, tokens, slots, pos, lengths, out)
        self._graphs[Bb] = g
        return g

    @torch.no_grad()
    def decode(self, tokens: List[int], slots: List[int], pos: List[int]) -> torch.Tensor:
        """One decode step: token t_b at position pos_b of slot s_b.  Returns logits [B, V]."""
        B = len(tokens)
        if not self.use_graphs:
            dev = self.dev
            t = torch.tensor(tokens, dtype=torch.long, device=dev)
            sl = torch.tensor(slots, dtype=torch.int32, device=dev)
            p = torch.tensor(pos, dtype=torch.int32, device=dev)
            out = self._decode_body(t, sl, p, p + 1)
            self._check_comm()
            return out
        Bb = next((b for b in BUCKETS if b >= B), None)
        if Bb is None:
            raise ValueError(f"decode batch {B} exceeds the largest graph bucket {BUCKETS[-1]}")
        graph, gt, gs, gp, gl, out = self._graph_for(Bb)
        pad = Bb - B
        # one pinned staging buffer per bucket, reused every step (allocating and pinning a
        # fresh host tensor per token costs more than the copy); the event keeps the next step
        # from overwriting it while the previous step's async copy may still read it
        st = self._staging.get(Bb)
        if st is None:
            st = self._staging[Bb] = (torch.empty((3, Bb), dtype=torch.int64).pin_memory(),
                                      torch.empty((3, Bb), dtype=torch.int64, device=self.dev),
                                      torch.cuda.Event())
        host, dev_rows, done = st
        done.synchronize()
        h = host.numpy()
        h[0, :B], h[1, :B], h[2, :B] = tokens, slots, pos
        if pad:
            h[0, B:], h[1, B:], h[2, B:] = 0, self.scratch, 0
        dev_rows.copy_(host, non_blocking=True)
        done.record()
        gt.copy_(dev_rows[0])
        gs.copy_(dev_rows[1])
        gp.copy_(dev_rows[2])
        gl.copy_(dev_rows[2] + 1)
        graph.replay()
        self._check_comm()
        return out[:B]

    def _check_comm(self):
        """TP decode: fail the step (and the engine) when a one-shot all-reduce timed out on a
        peer, instead of returning logits summed from stale peer slots.  The check waits for
        the step (the scheduler reads the logits on the host right after anyway)."""
        if self.car is not None:
            self.car.check()

    @property
    def healthy(self) -> bool:
        return self.car is None or not self.car.failed

    def release(self, slot: int):
        pass   # slots are overwritten in place; nothing to free


def sample(logits: torch.Tensor, temperature: float = 0.0, top_p: float = 1.0,
           generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Greedy (temperature 0) or nucleus sampling over fp32 logits [B, V] -> [B]."""
    if temperature <= 0:
        return logits.argmax(-1)
    probs = torch.softmax(logits.float() / temperature, -1)
    if top_p < 1.0:
        sp, idx = probs.sort(-1, descending=True)
        keep = sp.cumsum(-1) - sp < top_p
        sp = sp * keep
        choice = torch.multinomial(sp / sp.sum(-1, keepdim=True), 1, generator=generator)
        return idx.gather(-1, choice).squeeze(-1)
    return torch.multinomial(probs, 1, generator=generator).squeeze(-1)


# ------------------------------------------------------------------ continuous batching
@dataclass
class Request:
    prompt: List[int]
    max_new_tokens: int = 64
    temperature: float = 0.0
    top_p: float = 1.0
    stop: Optional[List[int]] = None
    output: List[int] = field(default_factory=list)
    done: threading.Event = field(default_factory=threading.Event)
    t_submit: float = field(default_factory=time.time)
    t_first: float = 0.0
    t_done: float = 0.0
    error: Optional[str] = None


class Scheduler:
    """Admit -> prefill -> joint decode steps; one engine loop thread."""

    def __init__(self, engine: Engine, max_batch: int = 64):
        self.e = engine
        self.max_batch = min(max_batch, engine.scratch)
        self.q: "queue.Queue[Request]" = queue.Queue()
        self.active: Dict[int, Request] = {}           # slot -> request
        self.free = list(range(engine.scratch))
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.tokens_generated = 0
        self.steps = 0

    def submit(self, req: Request) -> Request:
        if len(req.prompt) + req.max_new_tokens > self.e.max_len:
            req.error = f"prompt + max_new_tokens exceeds max_len {self.e.max_len}"
            req.done.set()
            return req
        self.q.put(req)
        return req

    def _finish(self, slot, req):
        req.t_done = time.time()
        req.done.set()
        del self.active[slot]
        self.free.append(slot)

    def _admit(self, batch: List[tuple]):
        """Prefill newly admitted (slot, request) pairs (Engine.prefill_batch) and sample their
        first tokens.  Prompts are length-sorted and grouped so that no group pads a prompt
        to more than PREFILL_PAD_RATIO x its rows (every row of a group is computed; on the GPU
        a prompt's rows are already rounded up to the flash kernel's 128-row tiles)."""
        tile = 128 if self.e.dev.type == "cuda" else 1
        rows = lambda sr: -(-len(sr[1].prompt) // tile) * tile      # noqa: E731
        batch = sorted(batch, key=rows)
        g0 = 0
        for j in range(1, len(batch) + 1):
            if j == len(batch) or rows(batch[j]) > PREFILL_PAD_RATIO * rows(batch[g0]):
                self._admit_group(batch[g0:j])
                g0 = j

    def _admit_group(self, batch: List[tuple]):
        logits = self.e.prefill_batch([s for s, _ in batch], [r.prompt for _, r in batch])
        for j, (slot, req) in enumerate(batch):
            tok = int(sample(logits[j:j + 1], req.temperature, req.top_p)[0])
            req.output.append(tok)
            req.t_first = time.time()
            self.active[slot] = req
            if len(req.output) >= req.max_new_tokens or (req.stop and tok in req.stop):
                self._finish(slot, req)

    def step(self) -> bool:
        """One scheduling iteration; returns False when idle."""
        admitted = False
        batch: List[tuple] = []
        ntok = 0
        while self.free and len(self.active) + len(batch) < self.max_batch:
            try:
                req = self.q.get_nowait()
            except queue.Empty:
                break
            if batch and ntok + len(req.prompt) > PREFILL_MAX_TOKENS:
                self._admit(batch)
                batch, ntok = [], 0
            batch.append((self.free.pop(), req))
            ntok += len(req.prompt)
            admitted = True
        if batch:
            self._admit(batch)
        if not self.active:
            return admitted
        slots = sorted(self.active)
        reqs = [self.active[s] for s in slots]
        toks = [r.output[-1] for r in reqs]
        pos = [len(r.prompt) + len(r.output) - 1 for r in reqs]
        logits = self.e.decode(toks, slots, pos)
        temps = {r.temperature for r in reqs}
        if temps == {0.0}:
            nxt = logits.argmax(-1).tolist()
        else:
            nxt = [int(sample(logits[j:j + 1], r.temperature, r.top_p)[0]) for j, r in enumerate(reqs)]
        self.steps += 1
        for s, r, t in zip(slots, reqs, nxt):
            r.output.append(t)
            self.tokens_generated += 1
            if len(r.output) >= r.max_new_tokens or (r.stop and t in r.stop):
                self._finish(s, r)
        return True

    def run_until_idle(self):
        while self.step() or not self.q.empty():
            pass

    def start(self):
        def loop():
            while not self._stop.is_set():
                try:
                    busy = self.step()
                except Exception as ex:     # fail the in-flight requests, keep serving
                    for s, r in list(self.active.items()):
                        r.error = str(ex)
                        self._finish(s, r)
                    busy = False
                if not busy:
                    time.sleep(0.001)
        self._thread = threading.Thread(target=loop, daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)


def build_engine(model_name: str = "llama3-8b", device=None, n_slots: int = 64, max_len: int = 4096,
                 checkpoint: Optional[str] = None, n_layers: Optional[int] = None, seed: int = 1234,
                 st: Optional[ParallelState] = None, use_graphs: Optional[bool] = None,
                 full_init: bool = False) -> Engine:
    cfg = LlamaConfig.preset(model_name)
    if n_layers:
        cfg = cfg.with_(n_layers=n_layers)
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    st = st or ParallelState(device=torch.device(device))
    model = Llama(cfg, st=st, device=device, seed=seed, full_init=full_init).allocate(grads=False)
    if checkpoint:
        from ..runtime.checkpoint import load_params
        load_params(model, checkpoint)
    return Engine(model, n_slots=n_slots, max_len=max_len, use_graphs=use_graphs)
