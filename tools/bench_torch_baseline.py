"""Library baseline for the headline metric: the same Llama-3-8B training step written the
standard PyTorch-ROCm way -- nn.Module, autograd, bf16 autocast over fp32 parameters,
fused SDPA attention (the vendor flash path), torch RMSNorm, full-logit cross-entropy,
gradient clipping and fused torch AdamW.  No kfamd code runs.  The comparison point for
bench.py, which runs the same architecture, sequence length, optimizer and clipping on the
framework's own kernels and runtime.

  python tools/bench_torch_baseline.py [--micro-batch N] [--steps K] [--warmup W] [--layers L]

Prints one JSON line (tokens/s, ms/step, peak memory).  --layers is a debug override.
"""
from __future__ import annotations

import argparse
import json
import math
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

V, H, L, HQ, HKV, D, FF, THETA, EPS = 128256, 4096, 32, 32, 8, 128, 14336, 500000.0, 1e-5


def rope_tables(S, device):
    inv = 1.0 / THETA ** (torch.arange(0, D, 2, device=device, dtype=torch.float32) / D)
    f = torch.outer(torch.arange(S, device=device, dtype=torch.float32), inv)
    return f.cos(), f.sin()                                # [S, D/2]


def rope(x, cos, sin):                                     # x [B, H, S, D], rotate-half pairing
    x1, x2 = x[..., : D // 2], x[..., D // 2:]
    c, s = cos.to(x.dtype), sin.to(x.dtype)
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)


class Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.n1, self.n2 = nn.RMSNorm(H, eps=EPS), nn.RMSNorm(H, eps=EPS)
        self.wqkv = nn.Linear(H, (HQ + 2 * HKV) * D, bias=False)
        self.wo = nn.Linear(HQ * D, H, bias=False)
        self.wgu = nn.Linear(H, 2 * FF, bias=False)
        self.wd = nn.Linear(FF, H, bias=False)

    def forward(self, x, cos, sin):
        B, S, _ = x.shape
        q, k, v = self.wqkv(self.n1(x)).split([HQ * D, HKV * D, HKV * D], -1)
        q = rope(q.view(B, S, HQ, D).transpose(1, 2), cos, sin)
        k = rope(k.view(B, S, HKV, D).transpose(1, 2), cos, sin)
        v = v.view(B, S, HKV, D).transpose(1, 2)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
        h = x + self.wo(o.transpose(1, 2).reshape(B, S, HQ * D))
        g, u = self.wgu(self.n2(h)).chunk(2, -1)
        return h + self.wd(F.silu(g) * u)


class Llama(nn.Module):
    def __init__(self, n_layers):
        super().__init__()
        self.embed = nn.Embedding(V, H)
        self.blocks = nn.ModuleList(Block() for _ in range(n_layers))
        self.norm = nn.RMSNorm(H, eps=EPS)
        self.head = nn.Linear(H, V, bias=False)
        for p in self.parameters():
            if p.dim() == 2:
                nn.init.normal_(p, std=0.02)

    def forward(self, tok, lab, cos, sin):
        x = self.embed(tok)
        for b in self.blocks:
            x = b(x, cos, sin)
        logits = self.head(self.norm(x))
        return F.cross_entropy(logits.float().view(-1, V), lab.view(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--seq-len", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--layers", type=int, default=L)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = Llama(a.layers).to(dev)
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4, weight_decay=0.1, fused=True)
    cos, sin = rope_tables(a.seq_len, dev)
    g = torch.Generator().manual_seed(1)
    batches = []
    for _ in range(2):
        x = torch.randint(0, V, (a.micro_batch, a.seq_len + 1), generator=g).to(dev)
        batches.append((x[:, :-1].contiguous(), x[:, 1:].contiguous()))

    def step(i):
        tok, lab = batches[i % 2]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = model(tok, lab, cos, sin)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / a.steps
    tok = a.micro_batch * a.seq_len
    print(json.dumps({"what": "PyTorch-ROCm eager baseline (autocast bf16, SDPA, fused AdamW)",
                      "model": "Llama-3-8B" if a.layers == L else f"Llama-3-8B ({a.layers} layers: INVALID)",
                      "micro_batch": a.micro_batch, "seq_len": a.seq_len, "steps": a.steps,
                      "tokens_per_s": round(tok / el, 1), "ms_per_step": round(el * 1e3, 2),
                      "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1),
                      "loss_last": round(float(loss), 4), "torch": torch.__version__}), flush=True)


if __name__ == "__main__":
    main()
