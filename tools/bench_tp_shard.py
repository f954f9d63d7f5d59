"""One TP rank's share of a tensor-parallel training step, timed on one GPU (BASELINE configs[4]:
Llama-3-70B TP=8).

The model is built exactly as rank 0 of a TP=`--tp` group builds it:
* 1/tp of the heads, of the FFN and of the vocabulary;
* all 80 layers;
* full fp32 master weights and AdamW state for the shard.

One training step is then timed. The TP collectives go to a ONE-rank RCCL group, so each
all-reduce is a local copy. The time measured is therefore the per-GPU compute of the TP step,
a lower bound for the 8-GPU step. The missing part is the wire time of the all-reduces: four
per layer, each [tokens, hidden] bf16. The tool prints that estimate from an assumed xGMI
all-reduce bus bandwidth (`--busbw-gbs`).

Losses are not meaningful: with one rank the vocab-parallel cross-entropy sees 1/tp of the
vocabulary. This is a timing tool, not a training run.

  python tools/bench_tp_shard.py [--model llama3-70b] [--tp 8] [--seq-len 4096] [--micro-batch 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--recompute", action="store_true")
    ap.add_argument("--tp-comm-chunks", type=int, default=4,
                    help="token chunks per TP projection (forward comm/compute overlap; 1 = off)")
    ap.add_argument("--tp-dual-batch", type=int, default=0,
                    help="1: split an even micro-batch into two halves interleaved at every TP collective")
    ap.add_argument("--busbw-gbs", type=float, default=300.0,
                    help="assumed RCCL all-reduce bus bandwidth over xGMI for the wire-time estimate")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29641")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from service_account_auth_improvements_amd.parallel.state import ParallelState, set_state
    from service_account_auth_improvements_amd.runtime.trainer import SyntheticData, TrainConfig, Trainer
    st = ParallelState(world_size=1, rank=0, tp=a.tp, tp_rank=0, device=dev, backend="nccl")
    set_state(st)
    t0 = time.time()
    tr = Trainer(TrainConfig(model=a.model, seq_len=a.seq_len, micro_batch=a.micro_batch, recompute=a.recompute,
                                 tp_comm_chunks=a.tp_comm_chunks, tp_dual_batch=bool(a.tp_dual_batch)), st)
    torch.cuda.synchronize()
    init_s = time.time() - t0
    data = SyntheticData(tr.mcfg.vocab_size, a.micro_batch, a.seq_len, dev, seed=1)
    batches = [[data.next()] for _ in range(2)]
    for i in range(a.warmup):
        tr.train_step(batches[i % 2])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(a.steps):
        tr.train_step(batches[i % 2])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / a.steps * 1e3
    c = tr.mcfg
    T = a.micro_batch * a.seq_len
    # wire time of the TP all-reduces the 8-GPU step adds: 2 per layer forward + 2 backward,
    # [T, hidden] bf16 each (the embedding / LM-head reductions are small next to them)
    msg = T * c.hidden * 2
    n_ar = 4 * c.n_layers
    wire_ms = n_ar * msg * 2 * (a.tp - 1) / a.tp / (a.busbw_gbs * 1e9) * 1e3
    tok_s = T / (ms / 1e3)
    flops = c.flops_per_token(a.seq_len) * T / a.tp
    print(json.dumps({"what": f"one TP={a.tp} rank's share of a {a.model} step (collectives are one-rank copies)",
                      "seq_len": a.seq_len, "micro_batch": a.micro_batch, "n_layers": c.n_layers,
                      "recompute": a.recompute, "tp_comm_chunks": a.tp_comm_chunks,
                      "ms_per_step_compute": round(ms, 1),
                      "model_tflops_per_gpu": round(flops / (ms / 1e3) / 1e12, 1),
                      "tokens_per_s_per_tp_group_compute_bound": round(tok_s, 1),
                      "tp_allreduce_wire_ms_est": round(wire_ms, 1), "assumed_busbw_GBps": a.busbw_gbs,
                      "tokens_per_s_per_tp_group_est_no_overlap": round(T / ((ms + wire_ms) / 1e3), 1),
                      "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1),
                      "init_s": round(init_s, 1)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
