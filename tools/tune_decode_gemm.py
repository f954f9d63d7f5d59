"""Decode GEMMs at batch 32-256 (Y[M, N] = X[M, K] . W[N, K]^T, the serving engine's
hipBLASLt path above SKINNY_MAX_ROWS): time hipBLASLt's heuristic choice, tune the same
shapes with PyTorch TunableOp, time the tuned choice, and write the results file that
serving/engine.py loads (tuning off) when KFAMD_DECODE_TUNED=<file> is set.

Weights rotate over enough copies (>= 1 GB) that every call streams from HBM, as in decode.

    python tools/tune_decode_gemm.py OUT.csv [M,M,...]
"""
import sys
import time

import torch

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tunableop_decode_gfx950.csv"
MS = [int(m) for m in (sys.argv[2] if len(sys.argv) > 2 else "32,64,128,256").split(",")]
H, F, V, Q = 4096, 14336, 128256, 6144
SHAPES = {"wqkv": (Q, H), "wo": (H, H), "wgu": (2 * F, H), "wd": (H, F), "lm_head": (V, H)}


def _time(fn, ws, x, reps=30):
    for w in ws[:2]:
        fn(x, w)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(x, ws[i % len(ws)])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    import torch.cuda.tunable as tn
    mm = lambda x, w: torch.mm(x, w.t())      # noqa: E731
    weights = {}
    for name, (N, K) in SHAPES.items():
        copies = max(2, -(-(1 << 30) // (N * K * 2)))
        weights[name] = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
    base = {}
    for M in MS:
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            base[(M, name)] = _time(mm, weights[name], x)
    tn.enable(True)
    tn.tuning_enable(True)
    tn.set_max_tuning_duration(60)
    tn.set_max_tuning_iterations(30)
    tn.set_filename(OUT, insert_device_ordinal=False)
    for M in MS:
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            mm(x, weights[name][0])                 # tunes this shape
            torch.cuda.synchronize()
    # the results file is written by TunableOp itself (at exit and as shapes are tuned)
    tn.tuning_enable(False)
    for M in MS:
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            t = _time(mm, weights[name], x)
            b = base[(M, name)]
            gb = N * K * 2 / 1e9
            print(f"M={M:4d} {name:8s} heuristic {b:8.1f} us ({gb / b * 1e3:5.2f} TB/s)  tuned {t:8.1f} us "
                  f"({gb / t * 1e3:5.2f} TB/s)  {b / t:5.2f}x", flush=True)
    print("wrote", OUT, flush=True)


if __name__ == "__main__":
    main()
