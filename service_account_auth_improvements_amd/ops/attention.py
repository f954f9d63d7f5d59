"""K3/K8: causal GQA attention on the fused QKV activation.

The Llama block keeps q, k and v inside one [T, (Hq + 2*Hkv) * D] bf16 buffer (one QKV
GEMM, RoPE in place).  The gfx950 flash kernels read q/k/v straight out of that buffer
with its row stride, so no transpose/copy to [B, H, S, D] is ever made, and write the
output as [T, Hq*D] -- exactly the operand the O-projection GEMM wants.

GPU tensors always run the hand-written MFMA flash attention (ops/csrc/flash_attn.hip);
there is no second GPU backend in the dispatch (the torch-SDPA comparison lives in
``tools/bench_attn.py``).  CPU tensors use the fp32 reference.
"""
from __future__ import annotations

import math
import os

import torch

from . import _ext, reference


def _split(qkv, B, S, Hq, Hkv, D):
    q = qkv[:, : Hq * D].reshape(B, S, Hq, D).transpose(1, 2)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].reshape(B, S, Hkv, D).transpose(1, 2)
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(B, S, Hkv, D).transpose(1, 2)
    return q, k, v


def attention_fwd(qkv, B, S, Hq, Hkv, D, causal=True):
    """Returns (o [T, Hq*D] bf16, lse [B, Hq, S] fp32)."""
    scale = 1.0 / math.sqrt(D)
    if qkv.is_cuda:
        return _ext.ops().flash_fwd(qkv, B, S, Hq, Hkv, D, scale, causal)
    q, k, v = _split(qkv, B, S, Hq, Hkv, D)
    o, lse = reference.attention(q, k, v, causal, scale)
    o = o.to(qkv.dtype)
    return o.transpose(1, 2).reshape(B * S, Hq * D), lse


def deterministic_default() -> bool:
    """The attention backward is bitwise run-to-run reproducible by default: each dK/dV work item
    stores its partial sums in its own slot and the post pass adds a key block's slots in a fixed
    order, instead of fp32 atomics whose order varies once a key block has several query chunks
    (S > 1536).  Same box, B4 S8192: backward 7.130 vs 7.065-7.098 ms, ~1-2 ms per training step
    (profiles/restart_gpu_r6.md); it is what makes a restarted GPU job's losses equal an
    uninterrupted run's bit for bit.  ``KFAMD_DETERMINISTIC=0`` selects the atomic form."""
    return os.environ.get("KFAMD_DETERMINISTIC", "1") != "0"


def attention_bwd(qkv, o, lse, do, B, S, Hq, Hkv, D, causal=True, deterministic=None):
    """Returns dqkv [T, (Hq + 2*Hkv)*D] in the fused layout."""
    scale = 1.0 / math.sqrt(D)
    if qkv.is_cuda:
        det = deterministic_default() if deterministic is None else bool(deterministic)
        return _ext.ops().flash_bwd(qkv, o, lse, do.contiguous(), B, S, Hq, Hkv, D, scale, causal, det)
    # CPU: recompute the fp32 reference through autograd
    with torch.enable_grad():
        x = qkv.detach().requires_grad_(True)
        q, k, v = _split(x, B, S, Hq, Hkv, D)
        oo = reference.attention(q, k, v, causal, scale)[0].to(qkv.dtype)
        oo = oo.transpose(1, 2).reshape(B * S, Hq * D)
        (dqkv,) = torch.autograd.grad(oo, x, do)
    return dqkv


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, S, Hq, Hkv, D, causal):
        qkv = qkv.contiguous()
        o, lse = attention_fwd(qkv, B, S, Hq, Hkv, D, causal)
        ctx.save_for_backward(qkv, o, lse)
        ctx.cfg = (B, S, Hq, Hkv, D, causal)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        return (attention_bwd(qkv, o, lse, do, *ctx.cfg),) + (None,) * 6


def attention(qkv, B, S, Hq, Hkv, D, causal=True):
    """Autograd-aware attention over a fused [B*S, (Hq+2Hkv)*D] qkv tensor."""
    return _AttnFn.apply(qkv, B, S, Hq, Hkv, D, causal)


def decode_attention(q2d, k_cache, v_cache, slots, lengths, Hq, scale=None):
    """Single-query GQA attention over a slot-major KV cache (K8, InferenceService decode).

    q2d [B, >=Hq*D] rows (the q columns of fused qkv rows are used in place);
    k_cache/v_cache [n_slots, Hkv, Lmax, D]; slots/lengths int32 [B] (cache slot of each
    row and its number of valid keys, including the current token). Returns [B, Hq*D]."""
    D = k_cache.shape[3]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if q2d.is_cuda:
        return _ext.ops().decode_attn(q2d, k_cache, v_cache, slots, lengths, Hq, scale)
    B, Hkv = q2d.shape[0], k_cache.shape[1]
    rep = Hq // Hkv
    out = torch.empty(B, Hq * D, dtype=q2d.dtype)
    for b in range(B):
        L, sl = int(lengths[b]), int(slots[b])
        q = q2d[b, : Hq * D].float().view(Hq, D)
        k = k_cache[sl, :, :L].float().repeat_interleave(rep, 0)   # [Hq, L, D]
        v = v_cache[sl, :, :L].float().repeat_interleave(rep, 0)
        p = torch.softmax(torch.einsum("hd,hld->hl", q, k) * scale, -1)
        out[b] = torch.einsum("hl,hld->hd", p, v).reshape(-1).to(q2d.dtype)
    return out


def kv_append_(qkv, Hq, slots, pos, k_cache, v_cache):
    """Write each row's (post-RoPE) K/V into position pos[b] of slot slots[b]."""
    if qkv.is_cuda:
        return _ext.ops().kv_append_(qkv, Hq, slots, pos, k_cache, v_cache)
    Hkv, D = k_cache.shape[1], k_cache.shape[3]
    for b in range(qkv.shape[0]):
        sl, p = int(slots[b]), int(pos[b])
        k_cache[sl, :, p] = qkv[b, Hq * D:(Hq + Hkv) * D].view(Hkv, D)
        v_cache[sl, :, p] = qkv[b, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].view(Hkv, D)


def rope_append_(qkv, Hq, cos_t, sin_t, slots, pos, k_cache, v_cache):
    """Decode prologue in one launch: RoPE on the q/k heads of each fused qkv row at pos[b],
    then the rotated k and v appended at pos[b] of slot slots[b]."""
    if qkv.is_cuda:
        return _ext.ops().rope_append_(qkv, Hq, cos_t, sin_t, slots, pos, k_cache, v_cache)
    Hkv, D = k_cache.shape[1], k_cache.shape[3]
    reference.rope_(qkv, Hq + Hkv, D, cos_t, sin_t, pos=pos)
    kv_append_(qkv, Hq, slots, pos, k_cache, v_cache)


def rope_append_parts(part, Hq, cos_t, sin_t, slots, pos, k_cache, v_cache):
    """:func:`rope_append_` on the qkv projection's fp32 K-split partials [S, B, N]
    (``ops.bgemm_parts``): the partials are summed and rounded to bf16 in the same launch.
    Returns the rotated qkv rows [B, N]."""
    if part.is_cuda:
        return _ext.ops().rope_append_parts(part, Hq, cos_t, sin_t, slots, pos, k_cache, v_cache)
    d = part[0].clone()
    for t in range(1, part.shape[0]):
        d += part[t]
    qkv = d.to(k_cache.dtype)
    rope_append_(qkv, Hq, cos_t, sin_t, slots, pos, k_cache, v_cache)
    return qkv


def kv_fill_(qkv, S, Hq, slot, k_cache, v_cache):
    """Prefill: rows [0, S) of one sequence's fused qkv -> positions [0, S) of `slot`."""
    if qkv.is_cuda:
        return _ext.ops().kv_fill_(qkv, S, Hq, slot, k_cache, v_cache)
    Hkv, D = k_cache.shape[1], k_cache.shape[3]
    k_cache[slot, :, :S] = qkv[:S, Hq * D:(Hq + Hkv) * D].reshape(S, Hkv, D).transpose(0, 1)
    v_cache[slot, :, :S] = qkv[:S, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(S, Hkv, D).transpose(0, 1)
