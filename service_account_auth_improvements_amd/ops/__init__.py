"""Hot-path kernels of the worker runtime.

Raw (non-autograd) entry points take and return plain tensors; GPU tensors run the
hand-written gfx950 HIP kernels (``torch.ops.kfamd``), CPU tensors run the fp32
references in :mod:`.reference`.  There is no GPU-side fallback: if the HIP library
cannot be loaded on a GPU box these functions raise.

Autograd wrappers (``rmsnorm``, ``swiglu``, ``attention``, ...) are provided for users
composing their own models; the Llama runtime uses the raw entry points inside its
fused per-layer autograd functions.
"""
from __future__ import annotations

import torch

from . import _ext, reference
from .attention import attention, attention_bwd, attention_fwd, decode_attention  # noqa: F401


def _k():
    return _ext.ops()


# ---------------------------------------------------------------- RMSNorm (K1)
def rmsnorm_fwd(a, w, eps, residual=None):
    """y = rmsnorm(a [+ residual]) * w. Returns (y, h, rstd); h is the summed residual
    stream (== a when residual is None)."""
    if a.is_cuda:
        y, h, rstd = _k().rmsnorm_fwd(a, residual, w, eps)
    else:
        y, h, rstd = reference.rmsnorm_fwd(a, residual, w, eps)
    if residual is None:
        h = a
    return y, h, rstd


def rmsnorm_fwd_parts(a, part, w, eps):
    """rmsnorm_fwd(a, residual=bf16(part.sum(0))) for ``part`` the fp32 K-split partials
    [S, rows, H] of :func:`bgemm_parts`: the batched-decode GEMM's reduce launch folded into the
    norm (ops/csrc/rmsnorm.hip).  Returns (y, h, rstd); h is bitwise the unfused path's."""
    if a.is_cuda:
        return _k().rmsnorm_fwd_parts(a, part, w, eps)
    d = part[0].clone()
    for t in range(1, part.shape[0]):
        d += part[t]
    return reference.rmsnorm_fwd(a, d.to(a.dtype), w, eps)


def rmsnorm_bwd(dy, h, rstd, w, dw_out, accumulate=False, dres=None):
    """Returns dh (+ dres); writes (or accumulates) dw into ``dw_out``."""
    if dy.is_cuda:
        return _k().rmsnorm_bwd(dy.contiguous(), h, rstd, w, dres, dw_out, accumulate)
    dh, dw = reference.rmsnorm_bwd(dy, h, rstd, w, dres)
    if accumulate:
        dw_out.add_(dw.to(dw_out.dtype))
    else:
        dw_out.copy_(dw)
    return dh


# ---------------------------------------------------------------- RoPE (K2)
def rope_(x, nheads, head_dim, cos_t, sin_t, seq_len=None, pos=None, inverse=False):
    if x.is_cuda:
        _k().rope_(x, nheads, head_dim, cos_t, sin_t, pos, int(seq_len or 0), inverse)
        return x
    return reference.rope_(x, nheads, head_dim, cos_t, sin_t, pos, seq_len, inverse)


rope_tables = reference.rope_tables


# ---------------------------------------------------------------- embedding (K7)
def embed_fwd(tokens, E, vstart: int = 0):
    """Rows E[tok - vstart] for tokens inside this rank's vocab shard, zero elsewhere."""
    if E.is_cuda:
        return _k().embed_fwd(tokens.reshape(-1).contiguous(), E, vstart)
    loc = tokens.reshape(-1) - vstart
    mask = (loc >= 0) & (loc < E.shape[0])
    return torch.nn.functional.embedding(loc.clamp(0, E.shape[0] - 1), E) * mask.unsqueeze(-1).to(E.dtype)


def embed_bwd_(tokens, g, dE, vstart: int = 0, accumulate: bool = False):
    """dE[tok - vstart] += g rows (deterministic sorted-run reduction on the GPU)."""
    if g.is_cuda:
        return _k().embed_bwd_(tokens.reshape(-1).contiguous(), g.contiguous(), dE, vstart, accumulate)
    loc = tokens.reshape(-1) - vstart
    mask = (loc >= 0) & (loc < dE.shape[0])
    gE = torch.zeros(dE.shape, dtype=torch.float32)
    gE.index_add_(0, loc[mask], g[mask].float())
    if accumulate:
        gE += dE.float()          # fp32 sum, one rounding -- as the GPU kernel
    dE.copy_(gE)


# ---------------------------------------------------------------- decode GEMM
def skinny_gemm(x, w, swiglu: bool = False):
    """Decode-shaped GEMM x[M<=64, K] . w[N, K]^T (weight-streaming HIP kernel on the GPU).
    ``swiglu``: w = [gate; up] -> silu(x.gate^T) * (x.up^T)."""
    if x.is_cuda:
        return _k().skinny_gemm(x, w, swiglu)
    y = torch.mm(x.float(), w.float().t())
    if swiglu:
        F_ = y.shape[1] // 2
        y = torch.nn.functional.silu(y[:, :F_]) * y[:, F_:]
    return y.to(x.dtype)


def bgemm_ok(x, w, swiglu: bool = False) -> bool:
    """True when the batched-decode GEMM (ops/csrc/bgemm.hip) takes x [M, K] . w^T."""
    return (x.is_cuda and 1 <= x.shape[0] <= 256 and x.shape[1] % 256 == 0 and w.shape[0] % 64 == 0
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous())


def bgemm(x, w, swiglu: bool = False, splits: int = 0):
    """Batched-decode GEMM x[M<=256, K] . w[N, K]^T: the HIP weight-streaming MFMA kernel on
    the GPU (K split ``splits`` ways, 0 = automatic).  ``swiglu``: w = [gate; up] ->
    silu(x.gate^T) * (x.up^T)."""
    if x.is_cuda:
        return _k().bgemm(x, w, bool(swiglu), int(splits))
    y = torch.mm(x.float(), w.float().t())
    if swiglu:
        F_ = y.shape[1] // 2
        y = torch.nn.functional.silu(y[:, :F_]) * y[:, F_:]
    return y.to(x.dtype)


def bgemm_parts(x, w):
    """:func:`bgemm` with the K-split reduce left to the consumer: the fp32 partials [S, M, N]
    when the automatic split is S > 1 (sum them with :func:`rmsnorm_fwd_parts`), else the bf16
    [M, N] product."""
    if x.is_cuda:
        return _k().bgemm_parts(x, w)
    return bgemm(x, w)


def skinny_gemm_norm_ok(x, K: int) -> bool:
    """True when the fused residual+RMSNorm decode GEMM handles these rows."""
    # up to 4 rows: at 5-8 the MFMA kernel with the prologue holds 131-163 VGPRs (one workgroup per
    # CU) and the unfused RMSNorm + skinny GEMM pair is faster: batch 8 4.77 vs 5.27 ms per step
    # (profiles/serve_gemv_upfront_loads_r4.txt)
    return x.is_cuda and 1 <= x.shape[0] <= 4 and 4 * K <= 32768 and K % 256 == 0


def skinny_gemm_norm(x, residual, norm_w, eps, w, swiglu: bool = False):
    """h = x (+ residual); y = (rmsnorm(h) * norm_w) . w^T (SwiGLU epilogue when ``swiglu``).
    One kernel on the GPU: the norm is the decode GEMM's prologue.  Returns (y, h)."""
    if x.is_cuda:
        return _k().skinny_gemm_norm(x.contiguous(), None if residual is None else residual.contiguous(),
                                     norm_w, float(eps), w, swiglu)
    a, h, _ = rmsnorm_fwd(x, norm_w, eps, residual=residual)
    return skinny_gemm(a, w, swiglu), h


def gemv_norm_rope_ok(x, K: int, head_dim: int) -> bool:
    """True when the fully fused decode qkv projection (norm + GEMV + RoPE + KV append) applies."""
    return x.is_cuda and 1 <= x.shape[0] <= 4 and x.shape[0] * K * 2 <= 65536 and K % 8 == 0 and head_dim == 128


def gemv_norm_rope(x, residual, norm_w, eps, w, Hq, cos_t, sin_t, slots, pos, k_cache, v_cache):
    """Decode qkv projection with its neighbours fused (one GPU kernel): h = x (+ residual);
    qkv = (rmsnorm(h) * norm_w) . w^T; RoPE at pos on the q/k heads; the rotated k and v
    appended to the KV cache at (slots, pos).  Returns (qkv, h); equals skinny_gemm_norm +
    attention.rope_append_ bit for bit."""
    if x.is_cuda:
        return _k().gemv_norm_rope(x.contiguous(), None if residual is None else residual.contiguous(), norm_w,
                                   float(eps), w, int(Hq), cos_t, sin_t, slots, pos, k_cache, v_cache)
    from .attention import rope_append_
    qkv, h = skinny_gemm_norm(x, residual, norm_w, eps, w)
    rope_append_(qkv, Hq, cos_t, sin_t, slots, pos, k_cache, v_cache)
    return qkv, h


def transpose_ok(w) -> bool:
    return (w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.stride(1) == 1
            and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0 and w.stride(0) % 8 == 0
            and w.data_ptr() % 16 == 0)


def transpose(w):
    """Row-major copy of w^T (LDS-tiled HIP kernel on the GPU)."""
    if w.is_cuda:
        return _k().transpose_bf16(w)
    return w.t().contiguous()


# ---------------------------------------------------------------- weight-gradient GEMM
def gemm_tn_ok(a, b, c) -> bool:
    """True when the HIP weight-gradient GEMM handles c = a^T b for these operands."""
    return a.is_cuda and _k().gemm_tn_ok(a, b, c)


def gemm_tn_(a, b, c, accumulate: bool = False):
    """c[M, N] (+)= a^T . b, a = [K, M], b = [K, N] (K = tokens): the dW = dY^T X product,
    hand-written MFMA kernel (ops/csrc/gemm.hip) on the GPU."""
    if a.is_cuda:
        return _k().gemm_tn_(a, b, c, accumulate)
    r = torch.mm(a.float().t(), b.float())
    if accumulate:
        r += c.float()
    c.copy_(r)


def gemm_tn2_(a0, b0, c0, a1, b1, c1, accumulate: bool = False):
    """Two weight-gradient products c_i (+)= a_i^T b_i over the same K in ONE launch (the
    tiles of both share the grid, so one product's partial last wave is filled by the
    other's tiles).  GPU only; both pairs must satisfy :func:`gemm_tn_ok`."""
    _k().gemm_tn2_(a0, b0, c0, a1, b1, c1, accumulate)


# ---------------------------------------------------------------- SwiGLU (K4)
def swiglu_fwd(gu):
    return _k().swiglu_fwd(gu) if gu.is_cuda else reference.swiglu_fwd(gu)


def swiglu_bwd(gu, dout):
    return _k().swiglu_bwd(gu, dout.contiguous()) if gu.is_cuda else reference.swiglu_bwd(gu, dout)


# ---------------------------------------------------------------- Cross entropy (K5)
CE_FUSED, CE_STATS, CE_GRAD = 0, 1, 2


def cross_entropy_fused_(logits, labels, scale, ignore_index=-100, vocab_start=0):
    """Loss rows + in-place gradient. ``scale`` may be a float or a 1-element fp32 device
    tensor (e.g. 1/num_valid computed on device, avoiding a host sync).
    Returns (loss_rows fp32 [T], lse fp32 [T]); logits now hold dlogits."""
    T = logits.shape[0]
    if logits.is_cuda:
        loss = torch.empty(T, device=logits.device, dtype=torch.float32)
        lse = torch.empty_like(loss)
        st = scale if torch.is_tensor(scale) else None
        sh = 0.0 if torch.is_tensor(scale) else float(scale)
        _k().cross_entropy_(logits, labels, vocab_start, ignore_index, st, sh, CE_FUSED, loss, lse,
                            None, None, None)
        return loss, lse
    sc = float(scale) if not torch.is_tensor(scale) else float(scale.reshape(-1)[0])
    loss, lse, g = reference.cross_entropy(logits, labels - vocab_start if vocab_start else labels,
                                           ignore_index, sc)
    logits.copy_(g.to(logits.dtype))
    return loss, lse


def cross_entropy_stats(logits, labels, vocab_start, ignore_index=-100):
    """Per-row (max, sumexp, target-logit-or-0) of one vocab shard (TP)."""
    T, V = logits.shape
    if logits.is_cuda:
        f = dict(device=logits.device, dtype=torch.float32)
        m, s, xy = torch.empty(T, **f), torch.empty(T, **f), torch.empty(T, **f)
        dummy = torch.empty(T, **f)
        _k().cross_entropy_(logits, labels, vocab_start, ignore_index, None, 0.0, CE_STATS, dummy,
                            dummy, m, s, xy)
        return m, s, xy
    lf = logits.float()
    m = lf.max(-1).values
    s = (lf - m.unsqueeze(1)).exp().sum(-1)
    loc = labels - vocab_start
    inr = (loc >= 0) & (loc < V)
    xy = torch.where(inr, lf.gather(1, loc.clamp(0, V - 1).unsqueeze(1)).squeeze(1),
                     torch.zeros_like(m))
    return m, s, xy


def cross_entropy_grad_(logits, labels, lse, scale, vocab_start, ignore_index=-100):
    """Write the shard's dlogits in place given the GLOBAL log-sum-exp."""
    T, V = logits.shape
    if logits.is_cuda:
        st = scale if torch.is_tensor(scale) else None
        sh = 0.0 if torch.is_tensor(scale) else float(scale)
        dummy = torch.empty(T, device=logits.device, dtype=torch.float32)
        _k().cross_entropy_(logits, labels, vocab_start, ignore_index, st, sh, CE_GRAD, dummy,
                            lse.contiguous(), None, None, None)
        return logits
    sc = float(scale) if not torch.is_tensor(scale) else float(scale.reshape(-1)[0])
    p = (logits.float() - lse.unsqueeze(1)).exp()
    loc = labels - vocab_start
    inr = (loc >= 0) & (loc < V) & (labels != ignore_index)
    rows = torch.arange(T, device=logits.device)[inr]
    p[rows, loc[inr]] -= 1.0
    p = p * sc
    p[labels == ignore_index] = 0
    logits.copy_(p.to(logits.dtype))
    return logits


# ---------------------------------------------------------------- AdamW (K6)
def adamw_(p, w, m, v, g, n_decay, lr, b1, b2, eps, wd, step, gscale=1.0, sumsq=None,
           max_norm=0.0):
    if p.is_cuda:
        _k().adamw_(p, w, m, v, g, int(n_decay), lr, b1, b2, eps, wd, int(step), gscale, sumsq,
                    max_norm)
    else:
        reference.adamw_(p, w, m, v, g, n_decay, lr, b1, b2, eps, wd, step, gscale,
                         None if sumsq is None else float(sumsq.reshape(-1)[0]), max_norm)


def shard_sum_(recv, nranks: int, out, accumulate: bool = False):
    """out (+)= sum over r of recv[r*n:(r+1)*n] (bf16 shards summed in fp32, rank order):
    the local half of the fp32 all-to-all gradient reduction (ops/csrc/grad_reduce.hip)."""
    if recv.is_cuda:
        _k().shard_sum_(recv, int(nranks), out, accumulate)
        return out
    s = recv.view(int(nranks), -1).float()
    acc = out.clone() if accumulate else torch.zeros_like(out)
    for r in range(int(nranks)):
        acc += s[r]
    out.copy_(acc)
    return out


GRAD_SET, GRAD_ADD, GRAD_FOLD = 0, 1, 2


def grad_accum_(main, g, mode: int):
    """fp32 micro-batch gradient accumulation: GRAD_SET main = g; GRAD_ADD main += g;
    GRAD_FOLD g = bf16(main + g) (one rounding, right before the bucket is sent)."""
    if g.is_cuda:
        _k().grad_accum_(main, g, int(mode))
    elif mode == GRAD_SET:
        main.copy_(g)
    elif mode == GRAD_ADD:
        main.add_(g.float())
    else:
        g.copy_(main + g.float())


def sumsq_(g, out, accumulate=False):
    """out[0] (+)= sum(g^2) (fp32, deterministic); g is bf16 or fp32."""
    if g.is_cuda:
        _k().sumsq(g, out, accumulate)
    else:
        s = g.float().pow(2).sum()
        out.copy_(out + s if accumulate else s.reshape(out.shape))
    return out


# ---------------------------------------------------------------- autograd wrappers
class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        y, h, rstd = rmsnorm_fwd(x.contiguous(), w, eps)
        ctx.save_for_backward(h, rstd, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        h, rstd, w = ctx.saved_tensors
        dw = torch.empty_like(w)
        dh = rmsnorm_bwd(dy.contiguous(), h, rstd, w, dw)
        return dh, dw, None


def rmsnorm(x, w, eps=1e-5):
    return _RMSNormFn.apply(x, w, eps)


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, d):
        (gu,) = ctx.saved_tensors
        return swiglu_bwd(gu, d)


def swiglu(gu):
    return _SwiGLUFn.apply(gu)
