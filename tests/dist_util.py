"""Run a test body in N CPU processes with the gloo backend (127.0.0.1 rendezvous)."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _detach(x):
    """Tensors -> numpy copies (queue transfer by value; the child may exit first)."""
    import torch
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy().copy()
    if isinstance(x, (list, tuple)):
        return type(x)(_detach(v) for v in x)
    if isinstance(x, dict):
        return {k: _detach(v) for k, v in x.items()}
    return x


def _attach(x):
    import numpy as np
    import torch
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_attach(v) for v in x)
    if isinstance(x, dict):
        return {k: _attach(v) for k, v in x.items()}
    return x


def _entry(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        import torch
        torch.set_num_threads(1)
        res = fn(rank, world, *args)
        q.put((rank, "ok", _detach(res)))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def run_ranks(fn, world=2, args=(), timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{res}")
            out[rank] = _attach(res)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [out[r] for r in range(world)]
