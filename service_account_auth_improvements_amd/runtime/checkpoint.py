"""Sharded safetensors checkpoints for the flat-buffer trainer (SURVEY.md §5 "Checkpoint /
resume": bf16 params + fp32 master + AdamW moments; resume restores the step, every rank's
CPU/GPU RNG state and its data-stream position, so a resumed job continues exactly where an
uninterrupted one would be -- tests/test_checkpoint_resume.py checks bit-identity).

Layout of a checkpoint directory::

    meta.json                      step, model config, parallel layout, per-file index
    tp{t}-pp{p}-dp{d}.safetensors  one file per (tp, pp, dp) shard that owns unique state
    rank{r}.state.safetensors      every rank: CPU / GPU RNG state, data generator state
    module.safetensors             plain nn.Module jobs (MNIST): weights + optimizer buffers

Each file holds the flat bf16 parameter buffers of its stage/TP shard (``param/<group>``)
and its optimizer shard(s) (``opt/<group>/<lo>-<hi>/{master,m,v}``).  Without ZeRO only
dp rank 0 writes (replicas are identical); with ZeRO-1 every dp rank writes its slices.
Tensors are written straight from device memory via safetensors (no pickling), and are
loaded with the safe loader only.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch


def _fname(st) -> str:
    return f"tp{st.tp_rank}-pp{st.pp_rank}-dp{st.dp_rank}.safetensors"


def _rank_state(data) -> dict:
    t = {"rng/cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        t["rng/cuda"] = torch.cuda.get_rng_state()
    if data is not None and hasattr(data, "g"):
        t["data/gen"] = data.g.get_state()
    return t


def _restore_rank_state(path: str, rank: int, data) -> bool:
    from safetensors.torch import load_file
    f = os.path.join(path, f"rank{rank}.state.safetensors")
    if not os.path.exists(f):
        return False
    t = load_file(f, device="cpu")
    torch.set_rng_state(t["rng/cpu"])
    if "rng/cuda" in t and torch.cuda.is_available():
        torch.cuda.set_rng_state(t["rng/cuda"])
    if data is not None and "data/gen" in t:
        data.g.set_state(t["data/gen"])
    return True


def _rank() -> int:
    import torch.distributed as dist
    return dist.get_rank() if dist.is_initialized() else 0


def save_module_checkpoint(path: str, trainer, step: int, data=None, extra: Optional[dict] = None):
    """Checkpoint for plain nn.Module jobs (the MNIST plumbing job): module weights and the
    optimizer's per-parameter buffers, written by rank 0 (DDP replicas are identical)."""
    from safetensors.torch import save_file
    import torch.distributed as dist
    os.makedirs(path, exist_ok=True)
    rank = _rank()
    save_file({k: v.contiguous().cpu() for k, v in _rank_state(data).items()},
              os.path.join(path, f"rank{rank}.state.safetensors"))
    if rank == 0:
        save_file({k: v.contiguous().cpu() for k, v in trainer.state_tensors().items()},
                  os.path.join(path, "module.safetensors"))
        meta = {"step": int(step), "format": "kfamd-module-v1"}
        meta.update(extra or {})
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(meta, f)
    if dist.is_initialized():
        dist.barrier()


def load_module_checkpoint(path: str, trainer, data=None) -> dict:
    from safetensors.torch import load_file
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    trainer.load_state_tensors(load_file(os.path.join(path, "module.safetensors"), device="cpu"))
    _restore_rank_state(path, _rank(), data)
    return meta


def save_checkpoint(path: str, trainer, extra: Optional[dict] = None, data=None):
    """Every rank calls this.  ``data`` (the rank's batch stream) has its generator state saved
    so resume continues the stream instead of replaying it."""
    from safetensors.torch import save_file
    import torch.distributed as dist
    if not hasattr(trainer, "model") or not hasattr(trainer.model, "groups"):
        return save_module_checkpoint(path, trainer, getattr(trainer, "step_idx", 0), data, extra)
    st = trainer.st
    if hasattr(trainer, "sync_params"):
        trainer.sync_params()        # land in-flight ZeRO-1 parameter gathers first
    if getattr(st, "tp_comm", None) is not None:
        st.tp_comm.check(sync=True)  # never persist state a timed-out TP collective produced
    os.makedirs(path, exist_ok=True)
    opt = trainer.opt
    writes_params = st.dp_rank == 0
    writes_opt = opt.sharded or st.dp_rank == 0
    tensors = {}
    if writes_params:
        for g in trainer.model.groups:
            tensors[f"param/{g.name}"] = g.params.detach().contiguous()
    if writes_opt:
        for sh in opt.shards:
            k = f"opt/{sh.group.name}/{sh.lo}-{sh.hi}"
            tensors[k + "/master"] = sh.master
            tensors[k + "/m"] = sh.m
            tensors[k + "/v"] = sh.v
    if tensors:
        save_file({k: v.cpu() for k, v in tensors.items()}, os.path.join(path, _fname(st)))
    save_file({k: v.contiguous().cpu() for k, v in _rank_state(data).items()},
              os.path.join(path, f"rank{st.rank}.state.safetensors"))
    if dist.is_initialized():
        dist.barrier()
    if st.rank == 0:
        meta = {"step": opt.step_count, "model": trainer.mcfg.__dict__,
                "parallel": {"tp": st.tp, "pp": st.pp, "dp": st.dp, "zero1": opt.sharded},
                "format": "kfamd-flat-v2"}
        meta.update(extra or {})
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(meta, f)
    if dist.is_initialized():
        dist.barrier()


def load_checkpoint(path: str, trainer, data=None) -> dict:
    from safetensors.torch import load_file
    if not hasattr(trainer, "model") or not hasattr(trainer.model, "groups"):
        return load_module_checkpoint(path, trainer, data)
    st = trainer.st
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    p = meta["parallel"]
    if (p["tp"], p["pp"]) != (st.tp, st.pp):
        raise ValueError(f"checkpoint layout tp{p['tp']}/pp{p['pp']} != current tp{st.tp}/pp{st.pp}")
    dev = trainer.model.groups[0].params.device
    pfile = os.path.join(path, f"tp{st.tp_rank}-pp{st.pp_rank}-dp0.safetensors")
    ptens = load_file(pfile, device="cpu")
    for g in trainer.model.groups:
        g.params.copy_(ptens[f"param/{g.name}"].to(dev))
    opt = trainer.opt
    ofile = os.path.join(path, _fname(st) if p.get("zero1") else os.path.basename(pfile))
    otens = ptens if ofile == pfile else load_file(ofile, device="cpu")
    for sh in opt.shards:
        k = f"opt/{sh.group.name}/{sh.lo}-{sh.hi}"
        if k + "/master" not in otens:
            raise KeyError(f"optimizer shard {k} not in {ofile}")
        sh.master.copy_(otens[k + "/master"].to(dev))
        sh.m.copy_(otens[k + "/m"].to(dev))
        sh.v.copy_(otens[k + "/v"].to(dev))
    opt.step_count = int(meta["step"])
    if hasattr(trainer, "step_idx"):
        trainer.step_idx = int(meta["step"])
    _restore_rank_state(path, st.rank, data)
    return meta


def load_params(model, path: str) -> dict:
    """Inference load: the flat bf16 parameter buffers of this (tp, pp) shard only (the
    optimizer state in the file is never read)."""
    from safetensors import safe_open
    st = model.st
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    p = meta["parallel"]
    if (p["tp"], p["pp"]) != (st.tp, st.pp):
        raise ValueError(f"checkpoint layout tp{p['tp']}/pp{p['pp']} != current tp{st.tp}/pp{st.pp}")
    pfile = os.path.join(path, f"tp{st.tp_rank}-pp{st.pp_rank}-dp0.safetensors")
    with safe_open(pfile, framework="pt", device="cpu") as f:
        for g in model.groups:
            t = f.get_tensor(f"param/{g.name}")
            if t.numel() != g.params.numel():
                raise ValueError(f"param/{g.name}: {t.numel()} elements, model expects {g.params.numel()}")
            g.params.copy_(t.to(g.params.device))
    return meta
