"""Batched-decode GEMMs (17..256 rows, Llama-3-8B projections): hipBLASLt (torch.mm, plus the
separate SwiGLU for gate/up) vs ops.bgemm at each K split; weights rotated over >= 1 GB so
every call streams them from HBM.

    python tools/bench_bgemm.py [M,M,...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from service_account_auth_improvements_amd import ops  # noqa: E402

MS = [int(m) for a in (sys.argv[1:] or ["32,64,128,256"]) for m in a.split(",")]
SHAPES = {"wqkv": (6144, 4096, False), "wo": (4096, 4096, False), "wd": (4096, 14336, False),
          "wgu": (28672, 4096, True), "lm_head": (128256, 4096, False)}


def _time(fn, ws, x, reps=40):
    for w in ws[:2]:
        fn(x, w)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(x, ws[i % len(ws)])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    for name, (N, K, sw) in SHAPES.items():
        copies = max(2, -(-(1 << 30) // (N * K * 2)))
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        gb = N * K * 2 / 1e9
        for M in MS:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            if sw:
                lib = lambda a, b: ops.swiglu_fwd(torch.mm(a, b.t()))      # noqa: E731
            else:
                lib = lambda a, b: torch.mm(a, b.t())                      # noqa: E731
            rec = {"gemm": name, "M": M, "hipblaslt_us": round(_time(lib, ws, x), 1)}
            ref = lib(x, ws[0]).float()
            for S in (0, 1, 2, 4, 8):
                if (K // 256) % max(S, 1):
                    continue
                f = lambda a, b, S=S: ops.bgemm(a, b, swiglu=sw, splits=S)   # noqa: E731
                us = _time(f, ws, x)
                err = ((f(x, ws[0]).float() - ref).abs().max() / ref.abs().max()).item()
                rec[f"bgemm_S{S or 'auto'}_us"] = round(us, 1)
                rec[f"bgemm_S{S or 'auto'}_err"] = float(f"{err:.1e}")
            best = min(v for k, v in rec.items() if k.startswith("bgemm") and k.endswith("_us"))
            rec["best_tbps"] = round(gb / best * 1e3, 2)
            rec["speedup_auto"] = round(rec["hipblaslt_us"] / rec["bgemm_Sauto_us"], 2)
            print(json.dumps(rec), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
