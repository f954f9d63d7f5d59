"""Decode GEMM orientation probe: y = x . w^T (hipBLASLt sees M = batch rows, N = weight rows)
against y^T = w . x^T (M = weight rows, N = batch rows: other tile shapes), HBM-cold (weights
rotated over >= 1 GB), Llama-3-8B projections at 32-256 rows.  One JSON line per (shape, M).

    python tools/bench_decode_gemm_orient.py [M,M,...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

MS = [int(m) for a in (sys.argv[1:] or ["64,128"]) for m in a.split(",")]
SHAPES = {"wqkv": (6144, 4096), "wo": (4096, 4096), "wd": (4096, 14336), "wgu": (28672, 4096),
          "lm_head": (128256, 4096)}


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
    for name, (N, K) in SHAPES.items():
        copies = max(2, -(-(1 << 30) // (N * K * 2)))
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in MS:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            a = _time(lambda x, w: torch.mm(x, w.t()), ws, x)
            b = _time(lambda x, w: torch.mm(w, x.t()), ws, x)
            ref = torch.mm(x, ws[0].t())
            err = (torch.mm(ws[0], x.t()).t().float() - ref.float()).abs().max().item()
            print(json.dumps({"gemm": name, "M": M, "xwT_us": round(a, 1), "wxT_us": round(b, 1),
                              "tbps_best": round(N * K * 2 / min(a, b) / 1e6, 2), "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
