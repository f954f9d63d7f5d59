"""Two-shot TP collective (ops/csrc/custom_ar.hip ts, parallel/custom_ar.py TwoShot): kernel time
per call and per MB by workgroup count, on the box's one GPU.

  python tools/bench_two_shot.py [--world 1|2] [--sizes-mb 16,64,268] [--blocks 32,64,128]

world 1: one rank; the kernel still stages its input through the uncached IPC buffer, reduces
and (AR) gathers, so this is the kernel's own per-byte cost with no peer.  world 2: two ranks
share the GPU (peer reads are local HBM reads instead of xGMI) -- the protocol's cost with a
real second participant.  Times are device time between events on the communicator's stream,
median of --iters calls after 2 warm-up calls.  One JSON line per (mode, size, blocks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(rank, world, port, a, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist

    from service_account_auth_improvements_amd.parallel.custom_ar import TwoShot
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    sizes = [int(float(s) * (1 << 20)) for s in a.sizes_mb.split(",")]
    recs = []
    for blocks in [int(b) for b in a.blocks.split(",")]:
        comm = TwoShot(max_bytes=max(sizes) + (1 << 20), blocks=blocks, timeout_s=60.0)
        for nbytes in sizes:
            n = nbytes // 2 // (8 * world) * (8 * world)
            x = torch.randn(n, device="cuda:0").to(torch.bfloat16)
            rs_out = torch.empty(n // world, dtype=torch.bfloat16, device="cuda:0")
            ag_out = torch.empty(n, dtype=torch.bfloat16, device="cuda:0")
            ag_in = x[: n // world].contiguous()
            for mode, fn in (("ar", lambda: comm.all_reduce(x)),
                             ("rs", lambda: comm.reduce_scatter(rs_out, x)),
                             ("ag", lambda: comm.all_gather(ag_out, ag_in))):
                ts = []
                for i in range(2 + a.iters):
                    dist.barrier()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(comm.stream)
                    fn()
                    e1.record(comm.stream)
                    torch.cuda.synchronize()
                    if i >= 2:
                        ts.append(e0.elapsed_time(e1))
                ts.sort()
                ms = ts[len(ts) // 2]
                recs.append({"world": world, "rank": rank, "mode": mode, "mb": round(nbytes / 2**20, 1),
                             "blocks": blocks, "ms": round(ms, 4), "ms_per_mb": round(ms / (nbytes / 2**20), 5),
                             "gb_s": round(nbytes / ms / 1e6, 1)})
        comm.check(sync=True)
        comm.close()
    q.put(recs)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--sizes-mb", default="16,64,268")
    ap.add_argument("--blocks", default="32,64,128")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, a.world, port, a, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    recs = []
    for _ in range(a.world):
        recs += q.get(timeout=900)
    for p in ps:
        p.join(timeout=60)
    for r in sorted(recs, key=lambda r: (r["mode"], r["mb"], r["blocks"], r["rank"])):
        if r["rank"] == 0:
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
