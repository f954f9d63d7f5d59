"""Decode-attention split count sweep inside a HIP graph (as the decode step runs it):
32 layers' worth of split + combine launches, Llama-3-8B heads, B rows, context C.
Run once per KFAMD_DECODE_SPLITS value (the override is read once per process)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from service_account_auth_improvements_amd.ops.attention import decode_attention

B, C, Lmax, Hq, Hkv = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), 32, 8
kc = torch.randn(max(B, 1), Hkv, Lmax, 128, device="cuda", dtype=torch.bfloat16)
vc = torch.randn_like(kc)
q = torch.randn(B, (Hq + 2 * Hkv) * 128, device="cuda", dtype=torch.bfloat16)
slots = torch.arange(B, dtype=torch.int32, device="cuda")
lens = torch.full((B,), C, dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        decode_attention(q, kc, vc, slots, lens, Hq)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    outs = [decode_attention(q, kc, vc, slots, lens, Hq) for _ in range(32)]
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    g.replay()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"splits": os.environ.get("KFAMD_DECODE_SPLITS", "auto"), "B": B, "ctx": C,
                  "us_per_layer": round(e0.elapsed_time(e1) / 20 / 32 * 1e3, 2)}), flush=True)
