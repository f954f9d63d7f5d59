"""Plain-PyTorch fp32 reference implementations of every kernel in ``ops/csrc``.

They define the semantics the HIP kernels are tested against (numerics tests compare the
gfx950 kernel to these on the same inputs) and they serve CPU tensors in CPU-only tests
(the gloo multi-process tests of the parallel engines run the model through them).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rmsnorm_fwd(a, b, w, eps):
    """Returns (y, h, rstd) with h = a + b (rounded to a's dtype) or h = a."""
    h = a if b is None else (a.float() + b.float()).to(a.dtype)
    hf = h.float()
    rstd = torch.rsqrt(hf.pow(2).mean(-1) + eps)
    y = (hf * rstd.unsqueeze(-1) * w.float()).to(a.dtype)
    return y, (h if b is not None else h.new_empty(0)), rstd.reshape(-1)


def rmsnorm_bwd(dy, h, rstd, w, dres=None):
    """Returns (dh, dw) in fp32 math, dh cast to h.dtype, dw fp32."""
    H = h.shape[-1]
    hf = h.float().reshape(-1, H)
    dyf = dy.float().reshape(-1, H)
    r = rstd.reshape(-1, 1).float()
    g = dyf * w.float()
    dot = (g * hf).sum(-1, keepdim=True)
    dh = r * g - hf * (r ** 3) * dot / H
    if dres is not None:
        dh = dh + dres.float().reshape(-1, H)
    dw = (dyf * hf * r).sum(0)
    return dh.to(h.dtype).reshape(h.shape), dw


def rope_tables(max_pos: int, head_dim: int, theta: float = 500000.0, device=None):
    """fp32 cos/sin tables [max_pos, head_dim/2] computed in fp64 (Llama-3 RoPE)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def rope_(x, nheads, head_dim, cos_t, sin_t, pos=None, seq_len=None, inverse=False):
    """In-place half-split rotary on the first nheads*head_dim columns of x [T, C]."""
    T = x.shape[0]
    p = pos.long() if pos is not None else torch.arange(T, device=x.device) % seq_len
    c = cos_t[p].unsqueeze(1)  # [T,1,D/2]
    s = sin_t[p].unsqueeze(1)
    if inverse:
        s = -s
    v = x[:, : nheads * head_dim].float().reshape(T, nheads, head_dim)
    a, b = v[..., : head_dim // 2], v[..., head_dim // 2:]
    out = torch.cat([a * c - b * s, b * c + a * s], dim=-1)
    x[:, : nheads * head_dim] = out.reshape(T, nheads * head_dim).to(x.dtype)
    return x


def swiglu_fwd(gu):
    F_ = gu.shape[-1] // 2
    g, u = gu[..., :F_].float(), gu[..., F_:].float()
    return (F.silu(g) * u).to(gu.dtype)


def swiglu_bwd(gu, dout):
    F_ = gu.shape[-1] // 2
    g, u = gu[..., :F_].float(), gu[..., F_:].float()
    d = dout.float()
    s = torch.sigmoid(g)
    du = d * g * s
    dg = d * u * s * (1 + g * (1 - s))
    return torch.cat([dg, du], dim=-1).to(gu.dtype)


def cross_entropy(logits, labels, ignore_index=-100, scale=None):
    """Returns (loss_rows fp32, lse fp32, dlogits fp32) for mean-style scaling `scale`."""
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = labels != ignore_index
    safe = labels.clamp(min=0)
    xy = lf.gather(1, safe.unsqueeze(1)).squeeze(1)
    loss = torch.where(valid, lse - xy, torch.zeros_like(lse))
    if scale is None:
        scale = 1.0 / max(int(valid.sum()), 1)
    p = torch.softmax(lf, dim=-1)
    p[torch.arange(p.shape[0], device=p.device)[valid], safe[valid]] -= 1.0
    p = p * scale
    p[~valid] = 0
    return loss, lse, p


def adamw_(p, w, m, v, g, n_decay, lr, b1, b2, eps, wd, step, gscale=1.0, sumsq=None,
           max_norm=0.0):
    gf = g.float() * gscale
    if sumsq is not None and max_norm > 0:
        nrm = math.sqrt(float(sumsq)) * gscale
        gf = gf * min(1.0, max_norm / (nrm + 1e-6))
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    decay = torch.ones_like(w)
    decay[:n_decay] = 1 - lr * wd
    m.mul_(b1).add_(gf, alpha=1 - b1)
    v.mul_(b2).addcmul_(gf, gf, value=1 - b2)
    denom = v.sqrt() / math.sqrt(bc2) + eps
    w.mul_(decay).sub_(lr * (m / bc1) / denom)
    p.copy_(w.to(p.dtype))


def attention(q, k, v, causal=True, scale=None):
    """q [B,Hq,S,D], k/v [B,Hkv,S,D] -> (o [B,Hq,S,D], lse [B,Hq,S]) in fp32 math (GQA)."""
    B, Hq, S, D = q.shape
    Hkv = k.shape[1]
    rep = Hq // Hkv
    kf = k.float().repeat_interleave(rep, dim=1)
    vf = v.float().repeat_interleave(rep, dim=1)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = torch.matmul(q.float(), kf.transpose(-1, -2)) * scale
    if causal:
        Sk = k.shape[2]
        mask = torch.ones(S, Sk, dtype=torch.bool, device=q.device).tril(Sk - S)
        s = s.masked_fill(~mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf)
    return o, lse
