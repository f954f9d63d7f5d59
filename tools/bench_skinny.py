"""Decode GEMM microbench: skinny HIP kernel vs torch.mm (hipBLASLt) at Llama-3-8B shapes."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from service_account_auth_improvements_amd import ops

def t(fn, it=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3

for name, (N, K) in {"wqkv": (6144, 4096), "wo": (4096, 4096), "wgu": (28672, 4096), "wd": (4096, 14336),
                     "lm_head": (128256, 4096)}.items():
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    for M in (1, 8, 32, 64):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        us_mm = t(lambda: torch.mm(x, w.t()))
        us_sk = t(lambda: ops.skinny_gemm(x, w))
        r = {"gemm": name, "M": M, "hipblaslt_us": round(us_mm, 1), "skinny_us": round(us_sk, 1),
             "skinny_TBps": round(N * K * 2 / us_sk / 1e6, 2)}
        if name == "wgu":
            r["skinny_swiglu_us"] = round(t(lambda: ops.skinny_gemm(x, w, True)), 1)
        print(json.dumps(r), flush=True)
