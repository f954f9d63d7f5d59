"""Tune hipBLASLt solutions (PyTorch TunableOp) for the training step's forward and dX GEMMs
(the dW products run the hand-written kernel) and write the results file that
runtime/trainer.py loads with tuning disabled.  Prints one line per shape as it goes.

    python tools/tune_gemm.py [out.csv]
"""
import os
import sys
import time

import torch

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tunableop_gfx950.csv"
T = 16384
H, F, V, Q = 4096, 14336, 128256, 6144
SHAPES = {"wqkv": (Q, H), "wo": (H, H), "wgu": (2 * F, H), "wd": (H, F), "lm_head": (V, H)}


def main():
    import torch.cuda.tunable as tn
    tn.enable(True)
    tn.tuning_enable(True)
    tn.set_max_tuning_duration(40)
    tn.set_max_tuning_iterations(20)
    tn.set_filename(OUT, insert_device_ordinal=False)
    for name, (N, K) in SHAPES.items():
        W = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        g = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        for op, fn in (("fwd", lambda: torch.mm(x, W.t())), ("dx", lambda: torch.mm(g, W))):
            t0 = time.time()
            fn()
            torch.cuda.synchronize()
            print(f"tuned {name} {op} in {time.time() - t0:.1f}s", flush=True)
        del W, x, g
        torch.cuda.empty_cache()
    tn.write_file(OUT)
    print("wrote", OUT, flush=True)


if __name__ == "__main__":
    main()
