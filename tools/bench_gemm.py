"""Time every Llama-3-8B training GEMM (T=16384 tokens/step) as the engine issues them:
fwd y = x @ W^T, dX = dY @ W, dW = dY^T @ x; report TFLOP/s.  Run with and without
PYTORCH_TUNABLEOP_ENABLED=1 to compare hipBLASLt heuristics vs tuned solutions."""
import json
import os
import sys

import torch

T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
H, F, V, Q = 4096, 14336, 128256, 6144
SHAPES = {"wqkv": (Q, H), "wo": (H, H), "wgu": (2 * F, H), "wd": (H, F), "lm_head": (V, H)}
if os.environ.get("GEMM_SKIP"):
    for k in os.environ["GEMM_SKIP"].split(","):
        SHAPES.pop(k, None)


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = "cuda"
    torch.manual_seed(0)
    res = {}
    tot_ms = 0.0
    for name, (N, K) in SHAPES.items():
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        g = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * N * K
        r = {}
        r["fwd"] = timeit(lambda: torch.mm(x, W.t()))
        r["dx"] = timeit(lambda: torch.mm(g, W))
        r["dw"] = timeit(lambda: torch.mm(g.t(), x, out=dW))
        r["dw_acc"] = timeit(lambda: dW.addmm_(g.t(), x))
        mult = 1 if name == "lm_head" else 32
        tot_ms += mult * (r["fwd"] + r["dx"] + r["dw"])
        res[name] = {k: {"ms": round(v, 3), "tflops": round(fl / v / 1e9, 1)} for k, v in r.items()}
        print(name, json.dumps(res[name]), flush=True)
        del W, x, g, dW
        torch.cuda.empty_cache()
    print(json.dumps({"gemm_ms_per_step_est": round(tot_ms, 1)}))


if __name__ == "__main__":
    main()
