"""Weight-gradient GEMM layouts at the 1-GPU bench shapes (Llama-3-8B, micro-batch 4 x 8192 tokens).

dW[N, K] = dY^T X with dY [T, N], X [T, K] (T = tokens, the contraction).  Times, per shape and for
the step's per-layer mix (32 x {wqkv, wo, wgu, wd} + lm_head):
  hip_tn     the hand-written TN kernel on the row-major operands (ops/csrc/gemm.hip, shipped)
  blas_tn    torch.mm(dY.t(), X): hipBLASLt on the same operands
  blas_nn    dY transposed once by the LDS-tiled kernel, then torch.mm(dYt, X) (NN); the
             transpose is included
  blas_nn_pre / blas_nt_pre  the library CEILING (transpose cost excluded): dYt [N, T] laid out
             beforehand, then torch.mm(dYt, X) (NN), and dYt with Xt [K, T] both contraction-
             contiguous, torch.mm(dYt, Xt.t()) -- the layout hipBLASLt is fastest in
  --tunable  the same rows again with PyTorch TunableOp tuning every shape (all hipBLASLt /
             rocBLAS solutions timed, the fastest kept): "tuned_*" keys
One JSON line per shape and one for the step mix.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from service_account_auth_improvements_amd import ops

T = 32768
SHAPES = {"wqkv": (6144, 4096), "wo": (4096, 4096), "wgu": (28672, 4096), "wd": (4096, 14336)}
TUNABLE = "--tunable" in sys.argv
ONLY = next((a.split("=", 1)[1].split(",") for a in sys.argv if a.startswith("--shapes=")), None)
HEAD = ("lm_head", (128256, 4096), 4096)          # chunked head: 4096 tokens per product, 8 chunks


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def run(name, N, K, tokens):
    g = torch.Generator(device="cuda").manual_seed(1)
    dy = (torch.randn(tokens, N, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    x = (torch.randn(tokens, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    c = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    out = {"shape": name, "N": N, "K": K, "tokens": tokens}
    flops = 2.0 * N * K * tokens
    if ops.gemm_tn_ok(dy, x, c):
        out["hip_tn_ms"] = round(timed(lambda: ops.gemm_tn_(dy, x, c)), 3)
    out["blas_tn_ms"] = round(timed(lambda: torch.mm(dy.t(), x, out=c)), 3)
    if ops.transpose_ok(dy):
        out["blas_nn_ms"] = round(timed(lambda: torch.mm(ops.transpose(dy), x, out=c)), 3)
        out["transpose_ms"] = round(timed(lambda: ops.transpose(dy)), 3)
    dyt = dy.t().contiguous()
    xt = x.t().contiguous()
    out["blas_nn_pre_ms"] = round(timed(lambda: torch.mm(dyt, x, out=c)), 3)
    out["blas_nt_pre_ms"] = round(timed(lambda: torch.mm(dyt, xt.t(), out=c)), 3)
    if TUNABLE:
        import torch.cuda.tunable as tn
        tn.enable(True)
        tn.tuning_enable(True)
        tn.set_max_tuning_iterations(10)
        tn.set_filename("gpurun_out/tunableop_dw.csv", insert_device_ordinal=False)
        for key, fn in (("tuned_tn_ms", lambda: torch.mm(dy.t(), x, out=c)),
                        ("tuned_nn_pre_ms", lambda: torch.mm(dyt, x, out=c)),
                        ("tuned_nt_pre_ms", lambda: torch.mm(dyt, xt.t(), out=c))):
            fn()                       # the tuning pass for this shape / layout
            torch.cuda.synchronize()
            out[key] = round(timed(fn), 3)
        tn.tuning_enable(False)
        tn.enable(False)
    del dyt, xt
    for k in ("hip_tn_ms", "blas_tn_ms", "blas_nn_ms", "blas_nn_pre_ms", "blas_nt_pre_ms",
              "tuned_tn_ms", "tuned_nn_pre_ms", "tuned_nt_pre_ms"):
        if k in out:
            out[k.replace("_ms", "_tflops")] = round(flops / (out[k] * 1e-3) / 1e12, 1)
    print(json.dumps(out), flush=True)
    return out


def main():
    res = {n: run(n, N, K, T) for n, (N, K) in SHAPES.items() if ONLY is None or n in ONLY}
    if ONLY is not None and HEAD[0] not in ONLY:
        return
    head = run(HEAD[0], *HEAD[1], HEAD[2])
    if ONLY is not None:
        return                      # a partial run: the step mix needs every shape
    mix = {}
    for k in ("hip_tn_ms", "blas_tn_ms", "blas_nn_ms", "blas_nn_pre_ms", "blas_nt_pre_ms",
              "tuned_tn_ms", "tuned_nn_pre_ms", "tuned_nt_pre_ms"):
        if all(k in r for r in res.values()) and k in head:
            mix[k] = round(32 * sum(r[k] for r in res.values()) + 8 * head[k], 1)
    print(json.dumps({"step_mix_ms": mix, "note": "32 layers x 4 products + 8 lm_head chunks"}), flush=True)


if __name__ == "__main__":
    main()
