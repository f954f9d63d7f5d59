"""Flash attention (K3) numerics vs an fp32 PyTorch reference (full tensors)."""
import math

import pytest
import torch

from service_account_auth_improvements_amd.ops import _ext, reference
from service_account_auth_improvements_amd.ops.attention import _split

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _qkv(B, S, Hq, Hkv, D=128, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B * S, (Hq + 2 * Hkv) * D, generator=g) * scale
    return x.to(DEV, torch.bfloat16)


@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 128, 2, 1, True), (2, 256, 8, 2, True), (1, 1024, 32, 8, True),
    (1, 384, 4, 4, False), (2, 512, 8, 1, True)])
def test_flash_fwd(B, S, Hq, Hkv, causal):
    assert _ext.load()
    qkv = _qkv(B, S, Hq, Hkv, seed=S + Hq)
    o, lse = torch.ops.kfamd.flash_fwd(qkv, B, S, Hq, Hkv, 128, 1 / math.sqrt(128), causal)
    q, k, v = _split(qkv, B, S, Hq, Hkv, 128)
    o_ref, lse_ref = reference.attention(q, k, v, causal)
    o_ref = o_ref.transpose(1, 2).reshape(B * S, Hq * 128)
    err = (o.float() - o_ref).abs().max().item()
    assert err < 2e-2, err
    assert torch.allclose(lse, lse_ref, atol=2e-3, rtol=1e-4), (lse - lse_ref).abs().max().item()


def test_flash_fwd_spiky_scores():
    """Large-magnitude inputs force big running-max jumps inside the online softmax."""
    B, S, Hq, Hkv = 1, 512, 4, 2
    qkv = _qkv(B, S, Hq, Hkv, seed=7, scale=4.0)
    o, lse = torch.ops.kfamd.flash_fwd(qkv, B, S, Hq, Hkv, 128, 1 / math.sqrt(128), True)
    q, k, v = _split(qkv, B, S, Hq, Hkv, 128)
    o_ref, lse_ref = reference.attention(q, k, v, True)
    o_ref = o_ref.transpose(1, 2).reshape(B * S, Hq * 128)
    assert (o.float() - o_ref).abs().max().item() < 8e-2
    assert torch.allclose(lse, lse_ref, atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 256, 2, 1, True), (2, 512, 8, 2, True), (1, 1024, 32, 8, True),
    (1, 512, 4, 4, False), (1, 768, 8, 1, True)])
def test_flash_bwd(B, S, Hq, Hkv, causal):
    """dQ and dK/dV kernels against fp32 autograd."""
    qkv = _qkv(B, S, Hq, Hkv, seed=S + 3 * Hq)
    sc = 1 / math.sqrt(128)
    o, lse = torch.ops.kfamd.flash_fwd(qkv, B, S, Hq, Hkv, 128, sc, causal)
    g = torch.Generator(device="cpu").manual_seed(11)
    do = torch.randn(o.shape, generator=g).to(DEV, torch.bfloat16)
    dqkv = torch.ops.kfamd.flash_bwd(qkv, o, lse, do, B, S, Hq, Hkv, 128, sc, causal, False)
    x = qkv.float().detach().requires_grad_(True)
    q, k, v = _split(x, B, S, Hq, Hkv, 128)
    o_ref, _ = reference.attention(q, k, v, causal)
    o_ref = o_ref.transpose(1, 2).reshape(B * S, Hq * 128)
    (ref,) = torch.autograd.grad(o_ref, x, do.float())
    for name, lo, hi in (("dq", 0, Hq * 128), ("dk", Hq * 128, (Hq + Hkv) * 128),
                         ("dv", (Hq + Hkv) * 128, (Hq + 2 * Hkv) * 128)):
        a, r = dqkv[:, lo:hi].float(), ref[:, lo:hi]
        rel = ((a - r).abs().max() / r.abs().max()).item()
        assert rel < 3e-2, (name, rel)


@pytest.mark.parametrize("causal", [True, False])
def test_flash_bwd_deterministic_mode_is_bitwise_and_matches_the_atomic_mode(causal):
    """KFAMD_DETERMINISTIC / flash_bwd(..., deterministic=True): at S = 4096 every key block's
    dK/dV gets 2-3 query chunks (QCH 1536), whose fp32 atomic sums vary in their last bits run to
    run.  The deterministic mode stores each chunk's partial in its own slot and the post pass sums
    them in item order: repeated calls are bitwise equal, and equal to the atomic mode within fp32
    rounding (bf16 output)."""
    B, S, Hq, Hkv = 1, 4096, 8, 2
    sc = 1 / math.sqrt(128)
    qkv = _qkv(B, S, Hq, Hkv, seed=33)
    o, lse = torch.ops.kfamd.flash_fwd(qkv, B, S, Hq, Hkv, 128, sc, causal)
    do = torch.randn(o.shape, generator=torch.Generator(device="cpu").manual_seed(9)).to(DEV, torch.bfloat16)
    det = [torch.ops.kfamd.flash_bwd(qkv, o, lse, do, B, S, Hq, Hkv, 128, sc, causal, True) for _ in range(4)]
    for x in det[1:]:
        assert torch.equal(x, det[0])
    ato = torch.ops.kfamd.flash_bwd(qkv, o, lse, do, B, S, Hq, Hkv, 128, sc, causal, False)
    assert torch.equal(det[0][:, :Hq * 128], ato[:, :Hq * 128])             # dQ: the same kernel
    err = ((det[0].float() - ato.float()).abs().max() / ato.float().abs().max()).item()
    assert err < 1e-2, err


def test_flash_bwd_stream_fork_ordering():
    """The backward forks its dK/dV chain (accumulator memset -> dK/dV) onto a side stream and
    joins before the fp32->bf16 post-pass.  Back-to-back calls on a NON-default stream, with the
    caching allocator recycling the accumulator between them, must agree with a call after a
    full device sync: a missing fork/join edge shows up as stale or unzeroed dK/dV."""
    B, S, Hq, Hkv = 2, 1024, 8, 2
    sc = 1 / math.sqrt(128)
    qkv = _qkv(B, S, Hq, Hkv, seed=21)
    o, lse = torch.ops.kfamd.flash_fwd(qkv, B, S, Hq, Hkv, 128, sc, True)
    do = torch.randn(o.shape, generator=torch.Generator(device="cpu").manual_seed(5)).to(DEV, torch.bfloat16)
    base = torch.ops.kfamd.flash_bwd(qkv, o, lse, do, B, S, Hq, Hkv, 128, sc, True, False)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=DEV)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        outs = [torch.ops.kfamd.flash_bwd(qkv, o, lse, do, B, S, Hq, Hkv, 128, sc, True, False) for _ in range(4)]
        outs = [x.float().clone() for x in outs]
    torch.cuda.synchronize()
    ref = base.float()
    for x in outs:
        # dQ is written once (bitwise); dK/dV are fp32 atomic sums (order-dependent last bits)
        assert torch.equal(x[:, :Hq * 128], ref[:, :Hq * 128])
        err = ((x - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-2, err


@pytest.mark.parametrize("B,b,g", [(2, 0, 0), (2, 1, 5), (4, 3, 7), (4, 1, 2)])
def test_flash_fwd_bwd_at_bench_shape(B, b, g):
    """The bench's exact launch: micro-batch B = 4 (bench.py's default on a 288 GB MI355X; B = 2
    too), S=8192, Hq=32, Hkv=8, causal -- the grid size, the XCD remap and the dK/dV work-item
    split all change with B -- checked on one (batch, kv-head) GQA group: its 4 query heads'
    O / lse / dQ and the group's dK / dV against an fp32 autograd reference of that slice."""
    S, Hq, Hkv, D = 8192, 32, 8, 128
    G = Hq // Hkv
    sc = 1 / math.sqrt(D)
    qkv = _qkv(B, S, Hq, Hkv, seed=99)
    o, lse = torch.ops.kfamd.flash_fwd(qkv, B, S, Hq, Hkv, D, sc, True)
    do = torch.randn(o.shape, generator=torch.Generator(device="cpu").manual_seed(13)).to(DEV, torch.bfloat16)
    dqkv = torch.ops.kfamd.flash_bwd(qkv, o, lse, do, B, S, Hq, Hkv, D, sc, True, False)
    torch.cuda.synchronize()
    rows = slice(b * S, (b + 1) * S)
    heads = range(g * G, (g + 1) * G)
    q = torch.stack([qkv[rows, h * D:(h + 1) * D] for h in heads]).float().requires_grad_(True)   # [G, S, D]
    k = qkv[rows, (Hq + g) * D:(Hq + g + 1) * D].float().requires_grad_(True)
    v = qkv[rows, (Hq + Hkv + g) * D:(Hq + Hkv + g + 1) * D].float().requires_grad_(True)
    s = (q @ k.t()) * sc
    mask = torch.ones(S, S, dtype=torch.bool, device=DEV).triu(1)
    s = s.masked_fill(mask, float("-inf"))
    lse_ref = torch.logsumexp(s, -1)
    o_ref = torch.softmax(s, -1) @ v
    do_s = torch.stack([do[rows, h * D:(h + 1) * D] for h in heads]).float()
    dq_r, dk_r, dv_r = torch.autograd.grad(o_ref, (q, k, v), do_s)
    o_s = torch.stack([o[rows, h * D:(h + 1) * D] for h in heads]).float()
    assert (o_s - o_ref).abs().max().item() < 2e-2
    lse_s = torch.stack([lse[b, h] for h in heads])
    assert torch.allclose(lse_s, lse_ref, atol=2e-3, rtol=1e-4)

    def rel(a, r):
        return ((a - r).abs().max() / r.abs().max()).item()
    dq_s = torch.stack([dqkv[rows, h * D:(h + 1) * D] for h in heads]).float()
    assert rel(dq_s, dq_r) < 3e-2
    assert rel(dqkv[rows, (Hq + g) * D:(Hq + g + 1) * D].float(), dk_r) < 3e-2
    assert rel(dqkv[rows, (Hq + Hkv + g) * D:(Hq + Hkv + g + 1) * D].float(), dv_r) < 3e-2


def test_flash_long_context_32k():
    """Long context: S = 32768, causal GQA 8/2, B = 1.  The forward's O / lse and
    the backward's dQ are checked on the LAST 256 query rows of one head (they attend to every
    key), dK / dV on the first 256 keys of one kv-head (every query attends to them), against
    fp32 references over the full key / query range of that slice."""
    assert _ext.load()
    B, S, Hq, Hkv, D = 1, 32768, 8, 2, 128
    G = Hq // Hkv
    sc = 1 / math.sqrt(D)
    qkv = _qkv(B, S, Hq, Hkv, seed=5)
    o, lse = torch.ops.kfamd.flash_fwd(qkv, B, S, Hq, Hkv, D, sc, True)
    do = torch.randn(o.shape, generator=torch.Generator(device="cpu").manual_seed(21)).to(DEV, torch.bfloat16)
    dqkv = torch.ops.kfamd.flash_bwd(qkv, o, lse, do, B, S, Hq, Hkv, D, sc, True, False)
    torch.cuda.synchronize()
    h, g = 5, 5 // G
    k = qkv[:, (Hq + g) * D:(Hq + g + 1) * D].float()
    v = qkv[:, (Hq + Hkv + g) * D:(Hq + Hkv + g + 1) * D].float()

    def rel(a, r):
        return ((a - r).abs().max() / r.abs().max()).item()
    # last 256 query rows of head h: O, lse, dQ
    rows = slice(S - 256, S)
    q = qkv[rows, h * D:(h + 1) * D].float().requires_grad_(True)
    s = (q @ k.t()) * sc
    qi = torch.arange(S - 256, S, device=DEV)[:, None]
    s = s.masked_fill(torch.arange(S, device=DEV)[None, :] > qi, float("-inf"))
    o_ref = torch.softmax(s, -1) @ v
    assert (o[rows, h * D:(h + 1) * D].float() - o_ref).abs().max().item() < 2e-2
    assert torch.allclose(lse[0, h, rows], torch.logsumexp(s, -1), atol=2e-3, rtol=1e-4)
    (dq_r,) = torch.autograd.grad(o_ref, q, do[rows, h * D:(h + 1) * D].float())
    assert rel(dqkv[rows, h * D:(h + 1) * D].float(), dq_r) < 3e-2
    # first 256 keys of kv-head g: dK / dV summed over the group's query heads and all queries
    dk_r = torch.zeros(256, D, device=DEV)
    dv_r = torch.zeros(256, D, device=DEV)
    for hq in range(g * G, (g + 1) * G):
        for c0 in range(0, S, 4096):            # query chunks bound the fp32 score memory
            qc = qkv[c0:c0 + 4096, hq * D:(hq + 1) * D].float()
            # probabilities need the full causal row: keys 0 .. c0 + 4095
            kf = k[:c0 + 4096]
            sf = (qc @ kf.t()) * sc
            sf = sf.masked_fill(torch.arange(c0 + 4096, device=DEV)[None, :] >
                                torch.arange(c0, c0 + 4096, device=DEV)[:, None], float("-inf"))
            lse_c = torch.logsumexp(sf, -1, keepdim=True)
            p = torch.exp(sf[:, :256] - lse_c)                 # probabilities on the 256 keys
            dO = do[c0:c0 + 4096, hq * D:(hq + 1) * D].float()
            dP = dO @ v[:c0 + 4096].t()
            delta = (dO * (torch.exp(sf - lse_c) @ v[:c0 + 4096])).sum(-1, keepdim=True)
            ds = p * (dP[:, :256] - delta)
            dv_r += p.t() @ dO
            dk_r += (ds.t() @ qc) * sc
    assert rel(dqkv[:256, (Hq + g) * D:(Hq + g + 1) * D].float(), dk_r) < 3e-2
    assert rel(dqkv[:256, (Hq + Hkv + g) * D:(Hq + Hkv + g + 1) * D].float(), dv_r) < 3e-2
