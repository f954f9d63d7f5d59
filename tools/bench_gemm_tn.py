"""Weight-gradient GEMM dW = dY^T X at the Llama-3-8B training shapes (T tokens): the
hand-written gfx950 kernel (ops.gemm_tn_) vs hipBLASLt (torch.mm(dY.t(), X)); TFLOP/s."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from service_account_auth_improvements_amd import ops  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
SHAPES = {"wqkv": (6144, 4096), "wo": (4096, 4096), "wgu": (28672, 4096), "wd": (4096, 14336),
          "lm_head": (128256, 4096)}


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
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        g = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        d1 = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        d2 = torch.empty_like(d1)
        fl = 2.0 * T * N * K
        blas = timeit(lambda: torch.mm(g.t(), x, out=d1))
        hip = timeit(lambda: ops.gemm_tn_(g, x, d2))
        hip_acc = timeit(lambda: ops.gemm_tn_(g, x, d2, True))
        ops.gemm_tn_(g, x, d2)
        err = ((d1.float() - d2.float()).abs().max() / d1.float().abs().max()).item()
        print(json.dumps({"shape": name, "M": N, "N": K, "K": T,
                          "hipblaslt_ms": round(blas, 3), "hipblaslt_tflops": round(fl / blas / 1e9, 1),
                          "hip_ms": round(hip, 3), "hip_tflops": round(fl / hip / 1e9, 1),
                          "hip_acc_tflops": round(fl / hip_acc / 1e9, 1), "rel_err": err}), flush=True)
        del g, x, d1, d2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
