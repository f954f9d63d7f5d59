"""Plain-PyTorch autograd Llama-3 (fp32 math) used ONLY as a numerics oracle.

It reads the weights of a TP=1 :class:`..llama.Llama` shard and computes the same loss
with textbook ops (HF-style rotate_half RoPE, GQA via repeat_interleave, softmax
attention, SwiGLU, RMSNorm).  Tests compare the explicit forward/backward engine (HIP
kernels on GPU, references on CPU) against ``torch.autograd`` on this module.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def _rope(x, cos, sin):
    # x [B, S, H, D]; cos/sin [S, D/2]
    D = x.shape[-1]
    a, b = x[..., : D // 2], x[..., D // 2:]
    c = cos[None, :, None, :]
    s = sin[None, :, None, :]
    return torch.cat([a * c - b * s, b * c + a * s], -1)


def _weights(model, dtype):
    assert model.tp == 1
    names = [s.name for g in model.groups for s in g.specs]
    return {n: model.P(n).detach().to(dtype).clone().requires_grad_(True) for n in names}


def reference_loss(model, tokens, labels, dtype=torch.float32):
    """Returns (mean loss, {name: fp32 leaf weight}) -- call .backward() for grads."""
    W = _weights(model, dtype)
    logits = _logits(model, tokens, W, dtype)
    loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1))
    return loss, W


@torch.no_grad()
def reference_last_logits(model, tokens, dtype=torch.float32):
    """fp32 logits of the LAST position of each row of ``tokens`` [B, S] (decode oracle)."""
    W = _weights(model, dtype)
    return _logits(model, tokens, W, dtype, last_only=True)


def _logits(model, tokens, W, dtype, last_only=False):
    cfg = model.cfg
    B, S = tokens.shape
    H, D, Hq, Hkv = cfg.hidden, cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
    cos, sin = model.cos[:S].to(dtype), model.sin[:S].to(dtype)
    x = F.embedding(tokens, W["embed"])
    for i in model.layers:
        a = _rms(x, W[f"l{i}.norm1"], cfg.norm_eps)
        qkv = a @ W[f"l{i}.wqkv"].t()
        q = qkv[..., : Hq * D].view(B, S, Hq, D)
        k = qkv[..., Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D)
        v = qkv[..., (Hq + Hkv) * D:].view(B, S, Hkv, D)
        q, k = _rope(q, cos, sin), _rope(k, cos, sin)
        q, k, v = (t.transpose(1, 2) for t in (q, k, v))
        rep = Hq // Hkv
        k = k.repeat_interleave(rep, 1)
        v = v.repeat_interleave(rep, 1)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(D)
        mask = torch.ones(S, S, dtype=torch.bool, device=s.device).tril()
        s = s.masked_fill(~mask, float("-inf"))
        o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, S, Hq * D)
        x = x + o @ W[f"l{i}.wo"].t()
        m = _rms(x, W[f"l{i}.norm2"], cfg.norm_eps)
        gu = m @ W[f"l{i}.wgu"].t()
        g, u = gu[..., : cfg.ffn], gu[..., cfg.ffn:]
        x = x + (F.silu(g) * u) @ W[f"l{i}.wd"].t()
    if last_only:
        x = x[:, -1]
    y = _rms(x, W["final_norm"], cfg.norm_eps)
    return y @ W["lm_head"].t()
