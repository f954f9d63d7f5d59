"""Decode GEMMs at 32-256 rows: torch.mm (hipBLASLt heuristic) vs a K-split batched GEMM
(torch.bmm over S K-slices with fp32 output, then a sum over S), weights rotated over >= 1 GB.

    python tools/bench_decode_splitbmm.py [M,M,...]
"""
import sys
import time

import torch

MS = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "32,64,128,256").split(",")]
SHAPES = {"wqkv": (6144, 4096), "wo": (4096, 4096), "wd": (4096, 14336), "wgu": (28672, 4096)}


def split_mm(x, w, S):
    M, K = x.shape
    N = w.shape[0]
    xs = x.view(M, S, K // S).transpose(0, 1)               # [S, M, K/S]
    wt = w.view(N, S, K // S).transpose(0, 1).transpose(1, 2)  # [S, K/S, N]
    return torch.bmm(xs, wt, out_dtype=torch.float32).sum(0).to(x.dtype)


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
    mm = lambda x, w: torch.mm(x, w.t())      # noqa: E731
    for name, (N, K) in SHAPES.items():
        copies = max(2, -(-(1 << 30) // (N * K * 2)))
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in MS:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            gb = N * K * 2 / 1e9
            tb = _time(mm, ws, x)
            line = f"{name:5s} M={M:4d} mm {tb:7.1f} us ({gb / tb * 1e3:5.2f} TB/s)"
            ref = torch.mm(x.double(), ws[0].double().t())
            for S in (2, 4, 8):
                ts = _time(lambda a, b: split_mm(a, b, S), ws, x)
                err = ((split_mm(x, ws[0], S).double() - ref).abs().max() / ref.abs().max()).item()
                line += f" | S={S} {ts:7.1f} us {tb / ts:4.2f}x err {err:.1e}"
            print(line, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
