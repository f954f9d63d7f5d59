"""InferenceService predictor benchmark (BASELINE configs[2]: Llama-3-8B bf16 TP=1, 1 MI355X).

Random-init Llama-3-8B weights, synthetic prompts.  Reports prefill tokens/s, per-step decode
latency and decode tokens/s at several batch sizes (HIP-graph decode), and the split-K
decode-attention kernel's effective HBM bandwidth.  One JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from service_account_auth_improvements_amd.serving.engine import build_engine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--ctx", type=int, default=1024, help="prompt length")
    ap.add_argument("--batches", nargs="+", default=["1,8,32,64"],
                    help="batch sizes: comma-separated and/or space-separated")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--max-len", type=int, default=2048)
    ap.add_argument("--prefill-batch", type=int, default=16, help="prompts per batched prefill pass")
    a = ap.parse_args()
    batches = [int(x) for b in a.batches for x in b.split(",") if x]
    nb = max(batches)
    t0 = time.time()
    e = build_engine(a.model, device="cuda", n_slots=nb, max_len=a.max_len, n_layers=a.layers)
    torch.cuda.synchronize()
    init_s = time.time() - t0
    prompt = [(i * 7919) % 1000 + 1 for i in range(a.ctx)]
    # prefill all slots (also the prefill throughput number)
    e.prefill(0, prompt)
    torch.cuda.synchronize()
    t0 = time.time()
    for s in range(nb):
        e.prefill(s, prompt)
    torch.cuda.synchronize()
    pf = time.time() - t0
    print(json.dumps({"bench": "prefill", "model": a.model, "prompt_len": a.ctx, "sequences": nb,
                      "tokens_per_s": round(nb * a.ctx / pf, 1), "ms_per_seq": round(1e3 * pf / nb, 2),
                      "init_s": round(init_s, 1)}), flush=True)
    # the scheduler's path: prompts admitted together are prefilled in one pass
    pb = max(1, min(nb, a.prefill_batch))
    e.prefill_batch(list(range(pb)), [prompt] * pb)
    torch.cuda.synchronize()
    t0 = time.time()
    for s0 in range(0, nb - pb + 1, pb):
        e.prefill_batch(list(range(s0, s0 + pb)), [prompt] * pb)
    torch.cuda.synchronize()
    pf = time.time() - t0
    done = (nb // pb) * pb
    print(json.dumps({"bench": "prefill_batch", "model": a.model, "prompt_len": a.ctx, "sequences": done,
                      "batch": pb, "tokens_per_s": round(done * a.ctx / pf, 1),
                      "ms_per_seq": round(1e3 * pf / done, 2)}), flush=True)
    for B in batches:
        toks, slots = [1] * B, list(range(B))
        pos = [a.ctx] * B
        for _ in range(3):                     # capture + warm
            e.decode(toks, slots, pos)
        torch.cuda.synchronize()
        t0 = time.time()
        for k in range(a.steps):
            e.decode(toks, slots, [a.ctx + k] * B)
        torch.cuda.synchronize()
        dt = (time.time() - t0) / a.steps
        print(json.dumps({"bench": "decode", "model": a.model, "batch": B, "context": a.ctx,
                          "ms_per_step": round(1e3 * dt, 3), "tokens_per_s": round(B / dt, 1),
                          "decode_path": "kernel-per-op graph"}),
              flush=True)
    # decode-attention kernel alone: HBM bytes of K+V read per call
    from service_account_auth_improvements_amd.ops.attention import decode_attention
    m = e.m
    kc, vc = e.kc[0], e.vc[0]
    for B in batches:
        q = torch.randn(B, (m.hq + 2 * m.hkv) * 128, device="cuda", dtype=torch.bfloat16)
        slots = torch.arange(B, dtype=torch.int32, device="cuda")
        lens = torch.full((B,), a.ctx, dtype=torch.int32, device="cuda")
        for _ in range(5):
            decode_attention(q, kc, vc, slots, lens, m.hq)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(50):
            decode_attention(q, kc, vc, slots, lens, m.hq)
        ev1.record()
        torch.cuda.synchronize()
        us = ev0.elapsed_time(ev1) / 50 * 1e3
        gbs = B * m.hkv * a.ctx * 128 * 2 * 2 / (us * 1e-6) / 1e9
        print(json.dumps({"bench": "decode_attn_kernel", "batch": B, "context": a.ctx, "us": round(us, 1),
                          "kv_GBps": round(gbs, 1)}), flush=True)


if __name__ == "__main__":
    main()
