"""Microbench: RMSNorm fwd/bwd, SwiGLU fwd/bwd at Llama-3-8B training shapes (T=16384);
reports achieved HBM GB/s."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from service_account_auth_improvements_amd import ops

def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3

T, H, F = 16384, 4096, 14336
x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
d = torch.randn_like(x)
w = torch.ones(H, device="cuda", dtype=torch.bfloat16)
y, hh, rstd = ops.rmsnorm_fwd(x, w, 1e-5, residual=d)
us = t(lambda: ops.rmsnorm_fwd(x, w, 1e-5, residual=d))
print(json.dumps({"op": "rmsnorm_fwd+res", "us": round(us, 1), "GBps": round(4 * T * H * 2 / us / 1e3, 0)}))
dw = torch.zeros(H, device="cuda", dtype=torch.bfloat16)
us = t(lambda: ops.rmsnorm_bwd(d, hh, rstd, w, dw, False, dres=x))
print(json.dumps({"op": "rmsnorm_bwd+dres", "us": round(us, 1), "GBps": round(4 * T * H * 2 / us / 1e3, 0)}))
gu = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)
us = t(lambda: ops.swiglu_fwd(gu))
print(json.dumps({"op": "swiglu_fwd", "us": round(us, 1), "GBps": round(3 * T * F * 2 / us / 1e3, 0)}))
do = torch.randn(T, F, device="cuda", dtype=torch.bfloat16)
us = t(lambda: ops.swiglu_bwd(gu, do))
print(json.dumps({"op": "swiglu_bwd", "us": round(us, 1), "GBps": round(5 * T * F * 2 / us / 1e3, 0)}))
