"""K8 decode attention + KV-cache kernels vs fp32 references, and the predictor engine on
the GPU (HIP graphs) vs its own eager path."""
import math

import pytest
import torch

from service_account_auth_improvements_amd.ops import _ext
from service_account_auth_improvements_amd.ops.attention import decode_attention, kv_append_, kv_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref_decode(q2d, kc, vc, slots, lengths, Hq):
    B, Hkv, D = q2d.shape[0], kc.shape[1], kc.shape[3]
    rep = Hq // Hkv
    out = torch.empty(B, Hq * D)
    for b in range(B):
        L, s = int(lengths[b]), int(slots[b])
        q = q2d[b, :Hq * D].float().cpu().view(Hq, D)
        k = kc[s, :, :L].float().cpu().repeat_interleave(rep, 0)
        v = vc[s, :, :L].float().cpu().repeat_interleave(rep, 0)
        p = torch.softmax(torch.einsum("hd,hld->hl", q, k) / math.sqrt(D), -1)
        out[b] = torch.einsum("hl,hld->hd", p, v).reshape(-1)
    return out


@pytest.mark.parametrize("B,Hq,Hkv,Lmax,lens", [
    (1, 32, 8, 256, [1]), (3, 32, 8, 1024, [1000, 17, 512]), (8, 8, 8, 4096, [4096, 1, 100, 2049, 3000, 64, 65, 7]),
    (2, 16, 2, 8192, [8192, 5000]), (4, 4, 4, 128, [128, 3, 64, 100]),
    # one-pass streaming kernel (chunks >= 256 keys): ragged lengths, tails, an empty split
    (32, 32, 8, 4096, [4096, 1, 17, 255, 256, 257, 1000, 3071] * 4),
    (8, 64, 8, 16384, [16384, 9000, 1, 300, 5000, 16383, 2048, 7]), (16, 16, 2, 2048, [2048, 1500] * 8),
    # large batch: 2 splits (B * Hkv = 512) and 1 split (1024, normalised in the split kernel, no
    # combine); chunks longer than one 1024-key sub-chunk are merged online inside the workgroup
    (64, 32, 8, 4096, [4096, 1, 2048, 2049, 3071, 1025, 17, 4000] * 8),
    (128, 32, 8, 3000, [3000, 1, 1024, 1025, 2049, 64, 2999, 700] * 16),
    # the direct (one-split) path at the other GQA widths: G = 8 and G = 1, with sub-chunks
    (128, 64, 8, 1500, [1500, 1030, 1, 999] * 32), (64, 8, 8, 2100, [2100, 2, 1024, 1025] * 16)])
def test_decode_attn(B, Hq, Hkv, Lmax, lens):
    assert _ext.load()
    g = torch.Generator(device="cpu").manual_seed(B * 7 + Lmax)
    n_slots = B + 2
    kc = torch.randn(n_slots, Hkv, Lmax, 128, generator=g).to(DEV, torch.bfloat16)
    vc = torch.randn(n_slots, Hkv, Lmax, 128, generator=g).to(DEV, torch.bfloat16)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * 128, generator=g).to(DEV, torch.bfloat16)
    slots = torch.randperm(n_slots, generator=g)[:B].to(torch.int32).to(DEV)
    lengths = torch.tensor(lens, dtype=torch.int32, device=DEV)
    o = decode_attention(qkv, kc, vc, slots, lengths, Hq)
    ref = _ref_decode(qkv, kc, vc, slots, lengths, Hq)
    err = (o.float().cpu() - ref).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("B,Lmax,lens", [(1, 1024, [1024]), (1, 8192, [8192]), (1, 8192, [1]),
                                        (4, 1024, [1024, 1, 517, 33]), (4, 8192, [8192, 4096, 100, 7777]),
                                        (2, 4096, [16, 17])])
def test_decode_attn_fused_matches_two_kernel_and_fp32(B, Lmax, lens, monkeypatch):
    """The small-batch single-launch kernel (split-K + last-arriver merge) against the
    two-kernel form and the fp32 reference at B = 1 / 4, contexts up to 8k (Llama-3-8B heads)."""
    assert _ext.load()
    Hq, Hkv = 32, 8
    g = torch.Generator(device="cpu").manual_seed(B * 131 + Lmax)
    kc = torch.randn(B + 1, Hkv, Lmax, 128, generator=g).to(DEV, torch.bfloat16)
    vc = torch.randn(B + 1, Hkv, Lmax, 128, generator=g).to(DEV, torch.bfloat16)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * 128, generator=g).to(DEV, torch.bfloat16)
    slots = torch.arange(1, B + 1, dtype=torch.int32, device=DEV)
    lengths = torch.tensor(lens, dtype=torch.int32, device=DEV)
    monkeypatch.setenv("KFAMD_DECODE_FUSED", "1")
    fused = decode_attention(qkv, kc, vc, slots, lengths, Hq)
    monkeypatch.setenv("KFAMD_DECODE_FUSED", "0")
    two = decode_attention(qkv, kc, vc, slots, lengths, Hq)
    ref = _ref_decode(qkv, kc, vc, slots, lengths, Hq)
    assert (fused.float().cpu() - ref).abs().max().item() < 2e-2
    assert (fused.float() - two.float()).abs().max().item() < 2e-2


def test_decode_attn_fused_in_a_graph_rearms_its_tickets(monkeypatch):
    """Captured once, replayed many times with changing lengths: each replay's last-arriving
    block re-arms the tickets, so every replay matches an eager call."""
    monkeypatch.setenv("KFAMD_DECODE_FUSED", "1")                # opt-in form
    Hq, Hkv, Lmax = 32, 8, 2048
    g = torch.Generator(device="cpu").manual_seed(9)
    kc = torch.randn(2, Hkv, Lmax, 128, generator=g).to(DEV, torch.bfloat16)
    vc = torch.randn(2, Hkv, Lmax, 128, generator=g).to(DEV, torch.bfloat16)
    qkv = torch.randn(1, (Hq + 2 * Hkv) * 128, generator=g).to(DEV, torch.bfloat16)
    slots = torch.tensor([1], dtype=torch.int32, device=DEV)
    lengths = torch.tensor([5], dtype=torch.int32, device=DEV)
    decode_attention(qkv, kc, vc, slots, lengths, Hq)            # allocates the tickets (outside capture)
    s = torch.cuda.Stream(device=DEV)
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        decode_attention(qkv, kc, vc, slots, lengths, Hq)
        with torch.cuda.graph(graph):
            out = decode_attention(qkv, kc, vc, slots, lengths, Hq)
    torch.cuda.synchronize()
    for L in (1, 33, 1024, 2048, 700, 1):
        lengths.fill_(L)
        graph.replay()
        torch.cuda.synchronize()
        eager = decode_attention(qkv, kc, vc, slots, lengths, Hq)
        assert torch.equal(out, eager), L
        ref = _ref_decode(qkv, kc, vc, slots, lengths, Hq)
        assert (out.float().cpu() - ref).abs().max().item() < 2e-2, L


def test_kv_append_and_fill():
    Hq, Hkv, Lmax = 8, 2, 64
    kc = torch.zeros(4, Hkv, Lmax, 128, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    qkv = torch.randn(3, (Hq + 2 * Hkv) * 128, device=DEV).to(torch.bfloat16)
    slots = torch.tensor([2, 0, 3], dtype=torch.int32, device=DEV)
    pos = torch.tensor([5, 0, 63], dtype=torch.int32, device=DEV)
    kv_append_(qkv, Hq, slots, pos, kc, vc)
    kc_r, vc_r = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    kv_append_(qkv.cpu(), Hq, slots.cpu(), pos.cpu(), kc_r, vc_r)
    assert torch.equal(kc.cpu(), kc_r) and torch.equal(vc.cpu(), vc_r)
    S = 40
    pre = torch.randn(S, (Hq + 2 * Hkv) * 128, device=DEV).to(torch.bfloat16)
    kv_fill_(pre, S, Hq, 1, kc, vc)
    kv_fill_(pre.cpu(), S, Hq, 1, kc_r, vc_r)
    assert torch.equal(kc.cpu(), kc_r) and torch.equal(vc.cpu(), vc_r)


def test_engine_gpu_graphs_match_eager_and_full_forward():
    from service_account_auth_improvements_amd.serving.engine import Request, Scheduler, build_engine
    e = build_engine("small", device=DEV, n_slots=8, max_len=512, n_layers=2)
    prompt = list(range(3, 3 + 200))
    cont = [7, 8, 9]
    full = e.m.forward_logits(torch.tensor([prompt + cont + [0] * (256 - len(prompt) - 3)], device=DEV))[0].float()
    lg = e.prefill(0, prompt).float()
    assert (lg - full[len(prompt) - 1]).abs().max().item() < 0.1
    for j, t in enumerate(cont):
        g = e.decode([t], [0], [len(prompt) + j])[0].float()
        assert (g - full[len(prompt) + j]).abs().max().item() < 0.1, j
    # graphs vs eager on a batch
    e.prefill(1, prompt[:50])
    e.prefill(2, prompt[:120])
    rows = ([11, 12, 13], [0, 1, 2], [len(prompt) + 3, 50, 120])
    kc0, vc0 = e.kc.clone(), e.vc.clone()
    a = e.decode(*rows).float()
    e.kc.copy_(kc0)
    e.vc.copy_(vc0)
    e.use_graphs = False
    b = e.decode(*rows).float()
    assert (a - b).abs().max().item() < 1e-2
    e.use_graphs = True
    s = Scheduler(e, max_batch=4)
    r = [s.submit(Request(prompt=prompt[:k], max_new_tokens=8)) for k in (10, 33, 10)]
    s.run_until_idle()
    assert r[0].output == r[2].output and all(len(x.output) == 8 for x in r)


@pytest.mark.parametrize("M,N,K,swiglu", [(1, 6144, 4096, False), (7, 4096, 4096, False), (16, 4096, 14336, False),
                                          (33, 1024, 4096, False), (64, 512, 2048, False),
                                          (1, 14336, 4096, True), (20, 2048, 4096, True)])
def test_skinny_gemm(M, N, K, swiglu):
    from service_account_auth_improvements_amd import ops
    g = torch.Generator(device="cpu").manual_seed(M * 31 + N)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn((2 * N if swiglu else N), K, generator=g) * 0.02).to(DEV, torch.bfloat16)
    y = ops.skinny_gemm(x, w, swiglu)
    ref = ops.skinny_gemm(x.cpu(), w.cpu(), swiglu).float()   # fp32 reference path
    err = ((y.float().cpu() - ref).abs().max() / ref.abs().max()).item()
    assert y.shape == (M, N) and err < 1e-2, err
    # strided X rows (the q / activation columns of a wider buffer)
    xs = torch.randn(M, K + 256, generator=g).to(DEV, torch.bfloat16)[:, :K]
    assert torch.allclose(ops.skinny_gemm(xs, w, swiglu).float(), ops.skinny_gemm(xs.contiguous(), w, swiglu).float())


def test_engine_prefill_batch_matches_per_prompt():
    """Batched prefill on the GPU (flash attention over B padded sequences, GEMMs over all rows)
    == per-prompt prefill: last-position logits and the KV rows below each prompt's length."""
    from service_account_auth_improvements_amd.serving.engine import build_engine
    e = build_engine("small", device=DEV, n_slots=6, max_len=512, n_layers=2)
    prompts = [list(range(3, 3 + 200)), list(range(7, 7 + 33)), list(range(1, 1 + 130))]
    slots = [4, 0, 2]
    one = [e.prefill(s, p).float() for s, p in zip(slots, prompts)]
    kc1, vc1 = e.kc.clone(), e.vc.clone()
    e.kc.zero_()
    e.vc.zero_()
    lg = e.prefill_batch(slots, prompts).float()
    for j, (s, p) in enumerate(zip(slots, prompts)):
        assert (lg[j] - one[j]).abs().max().item() < 5e-2, j
        n = len(p)
        assert (e.kc[:, s, :, :n].float() - kc1[:, s, :, :n].float()).abs().max().item() < 5e-2
        assert (e.vc[:, s, :, :n].float() - vc1[:, s, :, :n].float()).abs().max().item() < 5e-2


@pytest.mark.parametrize("M,N,K,swiglu", [(1, 1000, 1792, False), (2, 4104, 520, True), (3, 16032, 4096, False),
                                         (4, 4096, 14336, False), (1, 4096, 14336, False), (2, 1000, 9000, False),
                                         (1, 2052, 8192, True), (1, 128256, 4096, False)])
def test_gemv_odd_shapes(M, N, K, swiglu):
    """The VALU decode GEMV (M <= 4): TP-shard widths (K = 1792), ragged N, LM-head size; the
    in-workgroup K split (K >= 8192 on narrow N: wd, ragged K quarters, SwiGLU rows)."""
    from service_account_auth_improvements_amd import ops
    g = torch.Generator(device="cpu").manual_seed(M * 13 + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn((2 * N if swiglu else N), K, generator=g) * 0.02).to(DEV, torch.bfloat16)
    y = ops.skinny_gemm(x, w, swiglu)
    ref = torch.mm(x.double(), w.double().t())
    if swiglu:
        ref = torch.nn.functional.silu(ref[:, :N]) * ref[:, N:]
    err = ((y.double() - ref).abs().max() / ref.abs().max()).item()
    assert y.shape == (M, N) and err < 1e-2, err


@pytest.mark.parametrize("M,N,K,swiglu,res", [(1, 6144, 4096, False, True), (1, 14336, 4096, True, True),
                                              (4, 6144, 4096, False, False), (8, 2048, 4096, True, True),
                                              # MFMA kernel, 4 row slots (TP-shard sizes, K up to 8192)
                                              (3, 768, 4096, False, True), (4, 1024, 8192, True, False),
                                              # 8 row slots: the batch 5-8 decode projections
                                              (6, 6144, 4096, False, True), (5, 14336, 4096, True, False)])
def test_skinny_gemm_norm_matches_unfused(M, N, K, swiglu, res):
    """Residual-add + RMSNorm prologue fused into the decode GEMM == rmsnorm_fwd + skinny_gemm."""
    from service_account_auth_improvements_amd import ops
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    r = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16) if res else None
    nw = (1 + 0.1 * torch.randn(K, generator=g)).to(DEV, torch.bfloat16)
    w = (torch.randn((2 * N if swiglu else N), K, generator=g) * 0.02).to(DEV, torch.bfloat16)
    y, h = ops.skinny_gemm_norm(x, r, nw, 1e-5, w, swiglu)
    a, h_ref, _ = ops.rmsnorm_fwd(x, nw, 1e-5, residual=r)
    y_ref = ops.skinny_gemm(a, w, swiglu)
    assert torch.equal(h, h_ref)                       # the residual stream is bit-identical
    err = ((y.float() - y_ref.float()).abs().max() / y_ref.float().abs().max()).item()
    assert y.shape == (M, N) and err < 1e-2, err


@pytest.mark.parametrize("B,res", [(1, True), (2, False), (4, True)])
def test_gemv_norm_rope_matches_unfused(B, res):
    """Fused decode qkv projection (norm + GEMV + RoPE + KV append) == skinny_gemm_norm +
    rope_append_, bit for bit (qkv rows, residual stream and both caches)."""
    from service_account_auth_improvements_amd import ops
    from service_account_auth_improvements_amd.ops import reference
    from service_account_auth_improvements_amd.ops.attention import rope_append_
    Hq, Hkv, K, Lmax = 32, 8, 4096, 256
    g = torch.Generator(device="cpu").manual_seed(B * 5 + res)
    x = torch.randn(B, K, generator=g).to(DEV, torch.bfloat16)
    r = torch.randn(B, K, generator=g).to(DEV, torch.bfloat16) if res else None
    nw = (1 + 0.1 * torch.randn(K, generator=g)).to(DEV, torch.bfloat16)
    w = (torch.randn((Hq + 2 * Hkv) * 128, K, generator=g) * 0.02).to(DEV, torch.bfloat16)
    cos, sin = (t.to(DEV) for t in reference.rope_tables(Lmax, 128))
    slots = torch.tensor([3, 0, 5, 1][:B], dtype=torch.int32, device=DEV)
    pos = torch.tensor([17, 255, 0, 100][:B], dtype=torch.int32, device=DEV)
    kc = torch.zeros(6, Hkv, Lmax, 128, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    kc2, vc2 = kc.clone(), vc.clone()
    qkv, h = ops.gemv_norm_rope(x, r, nw, 1e-5, w, Hq, cos, sin, slots, pos, kc, vc)
    q_ref, h_ref = ops.skinny_gemm_norm(x, r, nw, 1e-5, w)
    rope_append_(q_ref, Hq, cos, sin, slots, pos, kc2, vc2)
    assert torch.equal(h, h_ref)
    assert torch.equal(qkv, q_ref)
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)
    assert kc.abs().sum() > 0 and vc.abs().sum() > 0


def test_rope_append_matches_reference():
    from service_account_auth_improvements_amd.ops import reference
    from service_account_auth_improvements_amd.ops.attention import rope_append_
    Hq, Hkv, Lmax = 32, 8, 256
    cos, sin = reference.rope_tables(Lmax, 128)
    qkv = torch.randn(5, (Hq + 2 * Hkv) * 128).to(torch.bfloat16)
    slots = torch.tensor([0, 3, 1, 2, 4], dtype=torch.int32)
    pos = torch.tensor([0, 17, 255, 3, 100], dtype=torch.int32)
    kc = torch.zeros(6, Hkv, Lmax, 128, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    q_ref, kc_ref, vc_ref = qkv.clone(), kc.clone(), vc.clone()
    rope_append_(q_ref, Hq, cos, sin, slots, pos, kc_ref, vc_ref)
    qd, kcd, vcd = qkv.to(DEV), kc.to(DEV), vc.to(DEV)
    rope_append_(qd, Hq, cos.to(DEV), sin.to(DEV), slots.to(DEV), pos.to(DEV), kcd, vcd)
    assert (qd.float().cpu() - q_ref.float()).abs().max().item() < 2e-2
    assert (kcd.float().cpu() - kc_ref.float()).abs().max().item() < 2e-2
    assert torch.equal(vcd.cpu(), vc_ref)


def test_decode_attn_repeated_calls_stable():
    """Repeated calls (and graph replays in the engine tests) produce bit-identical results."""
    g = torch.Generator(device="cpu").manual_seed(5)
    kc = torch.randn(4, 8, 2048, 128, generator=g).to(DEV, torch.bfloat16)
    vc = torch.randn(4, 8, 2048, 128, generator=g).to(DEV, torch.bfloat16)
    qkv = torch.randn(3, 48 * 128, generator=g).to(DEV, torch.bfloat16)
    slots = torch.tensor([2, 0, 3], dtype=torch.int32, device=DEV)
    lens = torch.tensor([2048, 700, 33], dtype=torch.int32, device=DEV)
    first = decode_attention(qkv, kc, vc, slots, lens, 32)
    for _ in range(200):
        o = decode_attention(qkv, kc, vc, slots, lens, 32)
    torch.cuda.synchronize()
    assert torch.equal(o, first)
    ref = _ref_decode(qkv, kc, vc, slots, lens, 32)
    assert (first.float().cpu() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("M", [17, 32, 64, 65, 128, 129, 200, 256])
@pytest.mark.parametrize("swiglu", [False, True], ids=["plain", "swiglu"])
def test_bgemm_matches_fp32(M, swiglu):
    """Batched-decode GEMM (ops/csrc/bgemm.hip) vs an fp32 reference, every MT bucket and its
    M padding, each K split (the fp32 partials + reduce launch included)."""
    from service_account_auth_improvements_amd import ops
    g = torch.Generator(device="cpu").manual_seed(M + 1000 * swiglu)
    K, Nw = 2048, 512
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(Nw, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    ref = torch.mm(x.float(), w.float().t())
    if swiglu:
        ref = torch.nn.functional.silu(ref[:, :Nw // 2]) * ref[:, Nw // 2:]
    for S in (0, 1, 2, 4, 8):
        y = ops.bgemm(x, w, swiglu=swiglu, splits=S)
        torch.cuda.synchronize()
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-2, (S, err)


def test_bgemm_decode_shapes_and_strided_rows():
    """The Llama-3-8B decode projections at batch 128, and X rows with a stride (a view)."""
    from service_account_auth_improvements_amd import ops
    g = torch.Generator(device="cpu").manual_seed(7)
    for N, K in ((6144, 4096), (4096, 4096), (4096, 14336)):
        xb = torch.randn(128, K + 64, generator=g).to(DEV, torch.bfloat16)
        x = xb[:, :K]                                   # row stride K + 64
        w = (torch.randn(N, K, generator=g) * 0.02).to(DEV, torch.bfloat16)
        y = ops.bgemm(x, w)
        ref = torch.mm(x.float(), w.float().t())
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-2, (N, K, err)


def test_bgemm_split_launches_are_bitwise_stable_and_replay_in_graphs():
    """Split-K batched-decode GEMMs (fp32 partials + the reduce launch): interleaved launches of
    different shapes and splits give bitwise the first result of each, and a captured graph
    replays it."""
    from service_account_auth_improvements_amd import ops
    g = torch.Generator(device="cpu").manual_seed(11)
    cases = [(128, 4096, 4096, False), (64, 2048, 8192, False), (128, 1024, 2048, True), (200, 4096, 14336, False)]
    data = []
    for M, N, K, sw in cases:
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.02).to(DEV, torch.bfloat16)
        ref = torch.mm(x.float(), w.float().t())
        if sw:
            ref = torch.nn.functional.silu(ref[:, :N // 2]) * ref[:, N // 2:]
        data.append((x, w, sw, ref))
    first = {}
    for rnd in range(6):
        for ci, (x, w, sw, ref) in enumerate(data):
            for S in (0, 2, 4):
                y = ops.bgemm(x, w, swiglu=sw, splits=S)
                if rnd == 0:
                    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                    assert err < 1e-2, (ci, S, err)
                    first[ci, S] = y
                else:
                    assert torch.equal(y, first[ci, S]), (rnd, ci, S)
    x, w, sw, _ = data[0]
    s = torch.cuda.Stream(device=DEV)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.bgemm(x, w, splits=4)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = ops.bgemm(x, w, splits=4)
    for _ in range(5):
        out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, first[0, 4])


def _llama8b_engine(n_layers, use_graphs, max_len=4096):
    from service_account_auth_improvements_amd.serving.engine import build_engine
    return build_engine("llama3-8b", device=DEV, n_slots=4, max_len=max_len, n_layers=n_layers, use_graphs=use_graphs)


@pytest.mark.parametrize("ctxs", [[1024], [8000], [7000, 100, 4000, 1]], ids=["b1-1k", "b1-8k", "b4-to-7k"])
def test_small_batch_decode_matches_fp32(ctxs):
    """The batch 1-4 decode step (kernel-per-op: fused norm/GEMV/RoPE, split-K decode attention)
    against the fp32 autograd-free oracle (models/llama_ref.py) on the full prompt + new token,
    Llama-3-8B shapes (2 layers), contexts 1k / 8k at batch 1 and mixed lengths up to 7k at batch 4."""
    from service_account_auth_improvements_amd.models.llama_ref import reference_last_logits
    B = len(ctxs)
    e = _llama8b_engine(2, use_graphs=False, max_len=8192)
    g = torch.Generator().manual_seed(sum(ctxs) + 1)
    prompts = [torch.randint(0, e.cfg.vocab_size, (c,), generator=g).tolist() for c in ctxs]
    for b, p in enumerate(prompts):
        e.prefill(b, p)
    toks = [int(x) for x in torch.randint(0, e.cfg.vocab_size, (B,), generator=g)]
    slots, pos = list(range(B)), list(ctxs)
    got = e.decode(toks, slots, pos).float()
    for b in range(B):
        ref = reference_last_logits(e.m, torch.tensor([prompts[b] + [toks[b]]], device=DEV))[0].float()
        cos = torch.nn.functional.cosine_similarity(got[b], ref, dim=0)
        assert cos > 0.995, (b, float(cos))
        assert (got[b] - ref).abs().max() <= 0.08 * ref.abs().max(), b


def test_small_batch_decode_graph_replays_the_eager_step():
    """Captured in the bucket-1/2/4 HIP graphs, replays give the eager step's logits, step after step."""
    eg = _llama8b_engine(2, use_graphs=True, max_len=1024)
    ee = _llama8b_engine(2, use_graphs=False, max_len=1024)
    prompt = list(range(10, 74))
    tg = int(eg.prefill(0, prompt).float().argmax())
    te = int(ee.prefill(0, prompt).float().argmax())
    assert tg == te
    for step in range(6):
        pos = len(prompt) + step
        lg = eg.decode([tg], [0], [pos]).clone()
        le = ee.decode([te], [0], [pos]).clone()
        assert torch.equal(lg, le), step
        tg = te = int(le.float().argmax())
    for B in (2, 3):
        slots = list(range(B))
        toks = [tg] * B
        for step in range(3):
            pos = [len(prompt) + 6 + step] * B
            lg = eg.decode(toks, slots, pos).clone()
            le = ee.decode(toks, slots, pos).clone()
            assert torch.nn.functional.cosine_similarity(lg.float().flatten(), le.float().flatten(), dim=0) > 0.999
            toks = le.float().argmax(-1).tolist()


@pytest.mark.parametrize("M,K", [(64, 4096), (128, 4096), (128, 14336)])
def test_rmsnorm_fwd_parts_matches_the_reduce_and_norm(M, K):
    """The decode projection's K-split partials summed inside the next RMSNorm
    (ops.rmsnorm_fwd_parts) against the bgemm reduce launch + plain RMSNorm: h bitwise, y and
    rstd to the last rounding, and y against an fp32 reference of the whole op."""
    from service_account_auth_improvements_amd import ops
    g = torch.Generator(device="cpu").manual_seed(M + K)
    N = 4096
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.02).to(DEV, torch.bfloat16)
    h1 = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(N, generator=g)).to(DEV, torch.bfloat16)
    part = ops.bgemm_parts(x, w)
    assert part.dim() == 3 and part.shape[1:] == (M, N) and part.shape[0] > 1
    y0, h0, r0 = ops.rmsnorm_fwd(h1, nw, 1e-5, residual=ops.bgemm(x, w))
    y1, h1f, r1 = ops.rmsnorm_fwd_parts(h1, part, nw, 1e-5)
    torch.cuda.synchronize()
    assert torch.equal(h1f, h0)
    assert torch.allclose(r1, r0, rtol=1e-6, atol=0)
    assert (y1.float() - y0.float()).abs().max().item() <= 0.02 * y0.float().abs().max().item()
    hf = h1.float() + torch.mm(x.float(), w.float().t())
    ref = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float()
    assert ((y1.float() - ref).abs().max() / ref.abs().max()).item() < 2e-2


def test_large_batch_decode_with_fused_splits_matches_the_reduce_launches(monkeypatch):
    """Batch 80 decode (Llama-3-8B shapes, 2 layers): with the wo / wd partials summed in the
    following RMSNorms and the qkv partials inside the RoPE / KV-append launch, the logits equal
    the reduce-launch step's to rounding, and the fused path is the one that ran."""
    from service_account_auth_improvements_amd import ops
    from service_account_auth_improvements_amd.serving import engine as eng
    e = eng.build_engine("llama3-8b", device=DEV, n_slots=80, max_len=256, n_layers=2, use_graphs=False)
    g = torch.Generator().manual_seed(5)
    B = 80
    for b in range(B):
        e.prefill(b, torch.randint(0, e.cfg.vocab_size, (16 + b,), generator=g).tolist())
    toks = [int(t) for t in torch.randint(0, e.cfg.vocab_size, (B,), generator=g)]
    slots, pos = list(range(B)), [16 + b for b in range(B)]
    kc0, vc0 = e.kc.clone(), e.vc.clone()
    calls = []
    real = ops.bgemm_parts
    monkeypatch.setattr(ops, "bgemm_parts", lambda x, w: calls.append(x.shape[0]) or real(x, w))
    monkeypatch.setattr(eng, "FUSE_SPLITS", True)
    fused = e.decode(toks, slots, pos).float()
    assert len(calls) == 3 * 2 and all(m == B for m in calls), calls     # qkv, wo, wd per layer
    e.kc.copy_(kc0)
    e.vc.copy_(vc0)
    monkeypatch.setattr(eng, "FUSE_SPLITS", False)
    plain = e.decode(toks, slots, pos).float()
    cos = torch.nn.functional.cosine_similarity(fused.flatten(), plain.flatten(), dim=0)
    assert cos > 0.9999, float(cos)
    assert (fused - plain).abs().max().item() <= 0.02 * plain.abs().max().item()


@pytest.mark.parametrize("M", [64, 128])
def test_rope_append_parts_matches_reduce_then_rope_append(M):
    """The qkv projection's K-split partials summed inside the RoPE / KV-append launch: qkv rows
    and both caches bitwise equal to bgemm's reduce launch followed by rope_append_."""
    from service_account_auth_improvements_amd import ops
    from service_account_auth_improvements_amd.ops.attention import rope_append_, rope_append_parts
    from service_account_auth_improvements_amd.ops import reference
    g = torch.Generator(device="cpu").manual_seed(M)
    Hq, Hkv, D, K, L = 32, 8, 128, 4096, 64
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn((Hq + 2 * Hkv) * D, K, generator=g) * 0.02).to(DEV, torch.bfloat16)
    cos, sin = (t.to(DEV) for t in reference.rope_tables(L, D))
    slots = torch.randperm(M, generator=g).to(DEV, torch.int32)
    pos = torch.randint(0, L, (M,), generator=g).to(DEV, torch.int32)
    kc = torch.zeros(M, Hkv, L, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    kc2, vc2 = kc.clone(), vc.clone()
    part = ops.bgemm_parts(x, w)
    assert part.dim() == 3
    got = rope_append_parts(part, Hq, cos, sin, slots, pos, kc, vc)
    ref = ops.bgemm(x, w)
    rope_append_(ref, Hq, cos, sin, slots, pos, kc2, vc2)
    torch.cuda.synchronize()
    assert torch.equal(got, ref) and torch.equal(kc, kc2) and torch.equal(vc, vc2)
