"""Sharded safetensors checkpoints for the flat-buffer trainer (SURVEY.md §5 "Checkpoint /
resume": bf16 params + fp32 master + AdamW moments; resume restores the step, every rank's
CPU/GPU RNG state and its data-stream position, so a resumed job continues exactly where an
uninterrupted one would be -- tests/test_checkpoint_resume.py checks bit-identity).

Layout of a checkpoint directory::

    meta.json                      step, model config, parallel layout, save token
    tp{t}-pp{p}-dp{d}.safetensors  the main file of each (tp, pp, dp) shard that owns unique state
    tp{t}-pp{p}-dp{d}.part{j}.safetensors   the rest of that shard's optimizer state
    rank{r}.state.safetensors      every rank: CPU / GPU RNG state, data generator state
    rank{r}.done                   periodic saves: the save token and the files rank r wrote
    module.safetensors             plain nn.Module jobs (MNIST): weights + optimizer buffers

The main file holds the flat bf16 parameter buffers of its stage/TP shard (``param/<group>``);
the optimizer shard(s) (``opt/<group>/<lo>-<hi>/{master,m,v}``) are cut into runs of flat
ranges spread over up to 8 files so that they are written concurrently (:func:`_flat_state`).
Without ZeRO only dp rank 0 writes (replicas are identical); with ZeRO-1 every dp rank writes
its slices.
Files are written by a streaming writer (the safetensors format: an 8-byte header length, a
JSON header, the raw tensor bytes -- straight from host memory, no serialisation copy, then
fsync) and loaded with the safe loader only.

Periodic checkpoint-restart (:class:`PeriodicCheckpointer`, worker flags ``--ckpt-dir`` /
``--save-every``) -- the data-plane counterpart of the reference's level-triggered recovery,
where controller state lives in the API object and survives restarts
(/root/reference/components/notebook-controller/controllers/culling_controller.go:50-52):

    <ckpt-dir>/step-00000040/...   one checkpoint directory per save (the layout above)
    <ckpt-dir>/latest              name of the newest COMPLETE one, replaced atomically

* the step's state is snapshotted into pinned host buffers on a side stream (the next step's
  forward/backward runs meanwhile; only its optimizer update waits for the copy to finish),
  and a writer thread streams the files out and fsyncs them;
* every rank then drops a ``rank{r}.done`` marker carrying this world's save token; rank 0
  publishes ``latest`` (tmp file, fsync, ``os.replace``) only once EVERY rank's marker is
  there, so a world killed mid-save leaves the previous ``latest`` in place;
* on (re)start every rank resumes from ``latest`` (an elastic restart or an OnFailure pod
  restart loses at most ``--save-every`` steps), and a changed data-parallel world re-shards
  the ZeRO-1 optimizer state by flat-range overlap (:func:`load_checkpoint`); a changed TP/PP
  layout is refused with a clear error.
"""
from __future__ import annotations

import json
import os
import re
import struct
import threading
import time
import uuid
from typing import Dict, List, Optional, Tuple

import torch

LATEST = "latest"
_STEP_DIR = re.compile(r"^step-(\d+)$")
_OPT_KEY = re.compile(r"^opt/(.+)/(\d+)-(\d+)/(master|m|v)$")
_ST_DTYPE = {torch.bfloat16: "BF16", torch.float32: "F32", torch.float16: "F16", torch.float64: "F64",
             torch.int64: "I64", torch.int32: "I32", torch.int16: "I16", torch.int8: "I8",
             torch.uint8: "U8", torch.bool: "BOOL"}


def _fname(st, part: int = 0) -> str:
    base = f"tp{st.tp_rank}-pp{st.pp_rank}-dp{st.dp_rank}"
    return f"{base}.safetensors" if part == 0 else f"{base}.part{part}.safetensors"


def _writers() -> int:
    """Files one rank's shard is spread over, written concurrently (KFAMD_CKPT_WRITERS, 8):
    writes into ONE file serialise on its inode lock (tmpfs, ext4 and xfs buffered writes alike),
    separate files do not -- 4 GB into /dev/shm: 2.1 GB/s one file, 14.2 GB/s over 8 files."""
    return max(1, int(os.environ.get("KFAMD_CKPT_WRITERS", "8")))


def _part_min() -> int:
    """Smallest optimizer part worth its own file (KFAMD_CKPT_PART_MIN bytes, 256 MB)."""
    return max(1, int(os.environ.get("KFAMD_CKPT_PART_MIN", str(256 << 20))))


def _opt_parts(shards, nparts: int, first: int):
    """Cut the optimizer shards' flat ranges into ``nparts`` runs of (nearly) equal element count:
    [(shard, lo, hi, file part)].  A range that is cut is stored as two keys; the loader fills
    by flat-range overlap, so it reads any cut."""
    total = sum(sh.hi - sh.lo for sh in shards)
    target = max(1, -(-total // nparts))
    out, pos = [], 0
    for sh in shards:
        if sh.hi == sh.lo:
            out.append((sh, sh.lo, sh.hi, first + min(pos // target, nparts - 1)))
            continue
        a = sh.lo
        while a < sh.hi:
            j = min(pos // target, nparts - 1)
            b = sh.hi if j == nparts - 1 else min(sh.hi, a + (j + 1) * target - pos)
            out.append((sh, a, b, first + j))
            pos += b - a
            a = b
    return out


def _fsync_dir(path: str):
    try:
        fd = os.open(path, os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


class HostPieces:
    """A tensor's host copy as consecutive byte pieces (page-locked snapshot buffers): its shape
    and dtype, and the uint8 CPU tensors holding its bytes in order."""
    __slots__ = ("shape", "dtype", "pieces")

    def __init__(self, shape, dtype, pieces):
        self.shape, self.dtype, self.pieces = tuple(shape), dtype, pieces

    @property
    def nbytes(self) -> int:
        return sum(p.numel() for p in self.pieces)


def write_safetensors(path: str, tensors: Dict[str, torch.Tensor], metadata: Optional[dict] = None):
    """Stream CPU tensors (or :class:`HostPieces`) into a safetensors file: header, then each
    tensor's bytes written straight from its memory (no bytes copy of a 30 GB master shard),
    fsync, atomic rename."""
    header, off, order = {}, 0, []
    for k in sorted(tensors):
        t = tensors[k]
        if isinstance(t, HostPieces):
            n = t.nbytes
            header[k] = {"dtype": _ST_DTYPE[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + n]}
            order.append(k)
            off += n
            continue
        if t.device.type != "cpu":
            raise ValueError(f"{k}: write_safetensors takes host tensors")
        n = t.numel() * t.element_size()
        header[k] = {"dtype": _ST_DTYPE[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + n]}
        order.append(k)
        off += n
    if metadata:
        header["__metadata__"] = {str(a): str(b) for a, b in metadata.items()}
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * (-len(hb) % 8)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        for k in order:
            t = tensors[k]
            if isinstance(t, HostPieces):
                for piece in t.pieces:
                    f.write(memoryview(piece.numpy()))
                continue
            t = t.contiguous()
            if t.numel():
                f.write(memoryview(t.reshape(-1).view(torch.uint8).numpy()))
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


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


def _world() -> int:
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_initialized() else 1


def tp_check_all(st):
    """Read the two-shot TP communicator's error word (a host sync) and fail EVERY rank of the
    TP group together when any one of them timed out (a timed-out block sets only its
    own rank's word, so without the MAX the healthy ranks would walk into the checkpoint's
    collectives and hang until the process-group timeout)."""
    comm = getattr(st, "tp_comm", None)
    if comm is None:
        return
    import torch.distributed as dist
    err = 0
    try:
        comm.check(sync=True)
    except RuntimeError:
        err = 1
    if st.tp > 1 and dist.is_initialized():
        t = torch.tensor([err], dtype=torch.int32, device=st.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=st.tp_group)
        err = int(t.item())
    if err:
        comm._raise()


def save_module_checkpoint(path: str, trainer, step: int, data=None, extra: Optional[dict] = None):
    """Checkpoint for plain nn.Module jobs (the MNIST plumbing job): module weights and the
    optimizer's per-parameter buffers, written by rank 0 (DDP replicas are identical)."""
    import torch.distributed as dist
    os.makedirs(path, exist_ok=True)
    rank = _rank()
    write_safetensors(os.path.join(path, f"rank{rank}.state.safetensors"),
                      {k: v.contiguous().cpu() for k, v in _rank_state(data).items()})
    if rank == 0:
        write_safetensors(os.path.join(path, "module.safetensors"),
                          {k: v.contiguous().cpu() for k, v in trainer.state_tensors().items()})
        meta = {"step": int(step), "format": "kfamd-module-v1"}
        meta.update(extra or {})
        _write_json(os.path.join(path, "meta.json"), meta)
    if dist.is_initialized():
        dist.barrier()


def load_module_checkpoint(path: str, trainer, data=None) -> dict:
    from safetensors.torch import load_file
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    trainer.load_state_tensors(load_file(os.path.join(path, "module.safetensors"), device="cpu"))
    _restore_rank_state(path, _rank(), data)
    return meta


def _write_json(path: str, obj):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def _flat_state(trainer) -> Tuple[Dict[str, torch.Tensor], dict, Dict[str, List[str]]]:
    """This rank's unique device state, the meta record, and the file plan (file name -> keys).

    The parameters stay whole in the rank's main file (``load_params`` reads them from there);
    the optimizer state (6x their bytes) is cut into up to :func:`_writers` runs of at least
    :func:`_part_min` bytes, one file each, so the writer streams them out in parallel."""
    st, opt = trainer.st, trainer.opt
    tensors: Dict[str, torch.Tensor] = {}
    plan: Dict[str, List[str]] = {}

    def put(part, k, v):
        tensors[k] = v
        plan.setdefault(_fname(st, part), []).append(k)
    pbytes = 0
    if st.dp_rank == 0:
        for g in trainer.model.groups:
            put(0, f"param/{g.name}", g.params.detach())
            pbytes += g.params.numel() * g.params.element_size()
    if opt.sharded or st.dp_rank == 0:
        shards = list(opt.shards)
        obytes = sum(sh.master.numel() * sh.master.element_size() * 3 for sh in shards)
        nopt = max(1, min(_writers() - (1 if pbytes else 0), obytes // _part_min()))
        first = 1 if pbytes and nopt > 1 else 0
        for sh, a, b, part in _opt_parts(shards, nopt, first):
            k = f"opt/{sh.group.name}/{a}-{b}"
            put(part, k + "/master", sh.master[a - sh.lo:b - sh.lo])
            put(part, k + "/m", sh.m[a - sh.lo:b - sh.lo])
            put(part, k + "/v", sh.v[a - sh.lo:b - sh.lo])
    meta = {"step": opt.step_count, "model": trainer.mcfg.__dict__,
            "parallel": {"tp": st.tp, "pp": st.pp, "dp": st.dp, "zero1": opt.sharded},
            "format": "kfamd-flat-v2"}
    return tensors, meta, plan


def _write_plan(path: str, plan: Dict[str, List[str]], host: Dict[str, object]):
    """Write the plan's files concurrently, one thread per file (the writes release the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    items = [(fn, {k: host[k] for k in keys}) for fn, keys in plan.items()]
    if len(items) <= 1:
        for fn, t in items:
            write_safetensors(os.path.join(path, fn), t)
        return
    with ThreadPoolExecutor(len(items), thread_name_prefix="kfamd-ckpt-write") as ex:
        for f in [ex.submit(write_safetensors, os.path.join(path, fn), t) for fn, t in items]:
            f.result()


def save_checkpoint(path: str, trainer, extra: Optional[dict] = None, data=None):
    """Every rank calls this (synchronous; the periodic path is :class:`PeriodicCheckpointer`).
    ``data`` (the rank's batch stream) has its generator state saved so resume continues the
    stream instead of replaying it."""
    import torch.distributed as dist
    if not hasattr(trainer, "model") or not hasattr(trainer.model, "groups"):
        return save_module_checkpoint(path, trainer, getattr(trainer, "step_idx", 0), data, extra)
    st = trainer.st
    if hasattr(trainer, "sync_params"):
        trainer.sync_params()        # land in-flight ZeRO-1 parameter gathers first
    tp_check_all(st)                 # never persist state a timed-out TP collective produced
    os.makedirs(path, exist_ok=True)
    tensors, meta, plan = _flat_state(trainer)
    _write_plan(path, plan, {k: v.contiguous().cpu() for k, v in tensors.items()})
    write_safetensors(os.path.join(path, f"rank{st.rank}.state.safetensors"),
                      {k: v.contiguous().cpu() for k, v in _rank_state(data).items()})
    if dist.is_initialized():
        dist.barrier()
    if st.rank == 0:
        meta.update(extra or {})
        _write_json(os.path.join(path, "meta.json"), meta)
    if dist.is_initialized():
        dist.barrier()


def _saved_files(path: str) -> Optional[set]:
    """The shard files the PUBLISHING world wrote: the union of the file lists in the done
    markers that carry meta.json's save token.  A world killed mid-save can leave files of its
    own in a step directory that a later world (another data-parallel size, another part count)
    saves again; those are not in the list.  None (read every file) for checkpoints without
    markers (the synchronous ``save_checkpoint``)."""
    try:
        with open(os.path.join(path, "meta.json")) as f:
            tok = json.load(f).get("token")
    except (OSError, ValueError):
        return None
    if not tok:
        return None
    files = set()
    for fn in os.listdir(path):
        if re.match(r"^rank\d+\.done$", fn):
            try:
                with open(os.path.join(path, fn)) as f:
                    d = json.load(f)
            except (OSError, ValueError):
                continue
            if d.get("token") == tok:
                if "files" not in d:
                    return None
                files.update(d["files"])
    return files


def _opt_sources(path: str, st) -> List[Tuple[str, str, int, int, str]]:
    """Every optimizer range stored for this (tp, pp) shard by ANY dp rank of the saving world:
    (file, group, lo, hi, key prefix)."""
    out = []
    pre = f"tp{st.tp_rank}-pp{st.pp_rank}-dp"
    listed = _saved_files(path)
    for fn in sorted(os.listdir(path)):
        if not (fn.startswith(pre) and fn.endswith(".safetensors")):
            continue
        if listed is not None and fn not in listed:
            continue                 # left in the directory by an earlier, killed world
        f = os.path.join(path, fn)
        fi = _FileIndex(f)
        try:
            for k in fi.keys():
                m = _OPT_KEY.match(k)
                if m and m.group(4) == "master":
                    out.append((f, m.group(1), int(m.group(2)), int(m.group(3)), k[:-len("/master")]))
        finally:
            fi.close()
    return out


class _FileIndex:
    """Byte spans of the tensors in a safetensors file (its JSON header, parsed directly) and a
    read-only descriptor for positional reads.  Nothing in the file is executed or unpickled."""

    def __init__(self, path: str):
        with open(path, "rb") as f:
            (n,) = struct.unpack("<Q", f.read(8))
            hdr = json.loads(f.read(n))
        self.path, self.base = path, 8 + n
        self.meta = {k: v for k, v in hdr.items() if k != "__metadata__"}
        self.fd = os.open(path, os.O_RDONLY)

    def keys(self):
        return self.meta.keys()

    def span(self, key: str):
        m = self.meta[key]
        a, b = m["data_offsets"]
        return m["dtype"], tuple(m["shape"]), self.base + a, b - a

    def close(self):
        os.close(self.fd)


class _Loader:
    """Checkpoint reader for resume: byte ranges of the files are read with positional reads on
    8 threads (the syscalls release the GIL) into two page-locked 128 MB staging buffers, each
    copied to the GPU on a side stream while the next one is read, so disk/page-cache reads and
    host-to-device copies overlap.  CPU destinations are read into directly."""

    CHUNK = 128 << 20

    def __init__(self, device):
        from concurrent.futures import ThreadPoolExecutor
        self.cuda = device.type == "cuda"
        self.pool = ThreadPoolExecutor(8, thread_name_prefix="kfamd-ckpt-read")
        self.k = 0
        if self.cuda:
            self.pin = PinnedPieces()
            self.bufs = [self.pin.alloc(self.CHUNK) for _ in range(2)]
            self.events = [None, None]
            self.stream = torch.cuda.Stream(device=device)
            self.stream.wait_stream(torch.cuda.current_stream(device))   # e.g. zero-fills queued before

    @staticmethod
    def _pread_part(fd: int, off: int, mv):
        got = 0
        while got < len(mv):
            r = os.preadv(fd, [mv[got:]], off + got)
            if r <= 0:
                raise IOError(f"short read at byte {off + got}")
            got += r

    def _pread(self, fd: int, off: int, mv):
        n = len(mv)
        step = max(4 << 20, -(-n // 8))
        for fut in [self.pool.submit(self._pread_part, fd, off + a, mv[a:a + step]) for a in range(0, n, step)]:
            fut.result()

    def load(self, fi: _FileIndex, key: str, elem_lo: int, dst: torch.Tensor):
        """Fill contiguous ``dst`` with elements [elem_lo, elem_lo + dst.numel()) of ``key``."""
        dtype, _, start, nbytes = fi.span(key)
        if _ST_DTYPE[dst.dtype] != dtype:
            raise TypeError(f"{fi.path}:{key} is {dtype}, the destination {dst.dtype}")
        bdst = dst.reshape(-1).view(torch.uint8)
        off = start + elem_lo * dst.element_size()
        if off + bdst.numel() > start + nbytes:
            raise ValueError(f"{fi.path}:{key}: range past the tensor")
        if not self.cuda:
            self._pread(fi.fd, off, memoryview(bdst.numpy()))
            return
        for a in range(0, bdst.numel(), self.CHUNK):
            i = self.k % 2
            self.k += 1
            if self.events[i] is not None:
                self.events[i].synchronize()          # the copy out of this buffer has finished
            m = min(self.CHUNK, bdst.numel() - a)
            buf = self.bufs[i][:m]
            self._pread(fi.fd, off + a, memoryview(buf.numpy()))
            with torch.cuda.stream(self.stream):
                bdst[a:a + m].copy_(buf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
            self.events[i] = ev

    def close(self):
        if self.cuda:
            self.stream.synchronize()
            self.bufs = []
            self.pin.free()
        self.pool.shutdown()


def load_checkpoint(path: str, trainer, data=None) -> dict:
    """Restore params, optimizer state, step, RNG and data position.  The optimizer shards of
    this rank are filled by flat-range overlap with whatever ranges the saving world stored, so
    a checkpoint written at one data-parallel size (or with / without ZeRO-1) resumes at another:
    ZeRO-1 state is re-sharded, elements past the saved (padded) length are zero.  A different
    TP or PP layout cannot be re-sharded this way and is refused.  Reads go through
    :class:`_Loader` (parallel positional reads overlapped with host-to-device copies)."""
    if not hasattr(trainer, "model") or not hasattr(trainer.model, "groups"):
        return load_module_checkpoint(path, trainer, data)
    st = trainer.st
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    p = meta["parallel"]
    if (p["tp"], p["pp"]) != (st.tp, st.pp):
        raise ValueError(f"checkpoint {path}: layout tp{p['tp']}/pp{p['pp']} != current tp{st.tp}/pp{st.pp}; "
                         "TP/PP re-sharding is not supported -- resume with the saving layout")
    dev = trainer.model.groups[0].params.device
    pfile = os.path.join(path, f"tp{st.tp_rank}-pp{st.pp_rank}-dp0.safetensors")
    sources = _opt_sources(path, st)
    # zero what the checkpoint does not cover (padding past the saved length) before the loader's
    # stream starts writing the rest
    pidx = _FileIndex(pfile)
    plen = {}
    for g in trainer.model.groups:
        n = min(pidx.span(f"param/{g.name}")[1][0], g.numel)
        plen[g.name] = n
        if n < g.numel:
            g.params[n:].zero_()
    for sh in trainer.opt.shards:
        for buf in (sh.master, sh.m, sh.v):
            buf.zero_()
    files = {pfile: pidx}
    ld = _Loader(dev)
    try:
        for g in trainer.model.groups:
            ld.load(pidx, f"param/{g.name}", 0, g.params[:plen[g.name]])
        for sh in trainer.opt.shards:
            filled = 0
            for f, gname, lo, hi, pre in sources:
                if gname != sh.group.name or hi <= sh.lo or lo >= sh.hi:
                    continue
                a, b = max(lo, sh.lo), min(hi, sh.hi)
                fi = files.get(f) or files.setdefault(f, _FileIndex(f))
                for suf, buf in (("master", sh.master), ("m", sh.m), ("v", sh.v)):
                    ld.load(fi, f"{pre}/{suf}", a - lo, buf[a - sh.lo:b - sh.lo])
                filled += b - a
            saved_len = max((hi for _, gname, _, hi, _ in sources if gname == sh.group.name), default=0)
            need = min(sh.hi, saved_len) - min(sh.lo, saved_len)
            if filled < need:
                raise KeyError(f"optimizer range {sh.group.name}[{sh.lo}, {sh.hi}) is not covered by {path}")
    finally:
        ld.close()
        for fi in files.values():
            fi.close()
    trainer.opt.step_count = int(meta["step"])
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


# ---------------------------------------------------------------- periodic checkpoint-restart

def latest_checkpoint(root: str) -> Optional[str]:
    """The newest COMPLETE checkpoint under ``root`` (the one ``latest`` names), or None."""
    try:
        with open(os.path.join(root, LATEST)) as f:
            name = f.read().strip()
    except OSError:
        return None
    path = os.path.join(root, name)
    return path if name and os.path.exists(os.path.join(path, "meta.json")) else None


def step_dir(root: str, step: int) -> str:
    return os.path.join(root, f"step-{step:08d}")


PIN_PIECE = 256 << 20          # bytes per page-locked snapshot piece


class PinnedPieces:
    """Page-locked host memory for checkpoint snapshots, from the HIP runtime torch itself loaded,
    called through ctypes (which releases the GIL for the whole call) in pieces of at most
    ``PIN_PIECE`` bytes (which keeps the runtime's own locks short).  ``torch.empty(...,
    pin_memory=True)`` of whole multi-GB tensors on a side thread held both for seconds: the
    training loop's first step waited 4.2 s behind it (profiles/ckpt_cost_r6.md).  Freed by
    :meth:`free` (the checkpointer's ``close``)."""

    def __init__(self):
        import ctypes
        self._ct = ctypes
        lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        self._hip = ctypes.CDLL(lib) if os.path.exists(lib) else ctypes.CDLL("libamdhip64.so")
        self._ptrs: List[int] = []

    def alloc(self, nbytes: int) -> torch.Tensor:
        ct = self._ct
        p = ct.c_void_p()
        rc = self._hip.hipHostMalloc(ct.byref(p), ct.c_size_t(nbytes), ct.c_uint(0))
        if rc != 0 or not p.value:
            raise MemoryError(f"hipHostMalloc({nbytes}) failed: {rc}")
        self._ptrs.append(p.value)
        return torch.frombuffer((ct.c_ubyte * nbytes).from_address(p.value), dtype=torch.uint8)

    def pieces(self, nbytes: int) -> List[torch.Tensor]:
        return [self.alloc(min(PIN_PIECE, nbytes - a)) for a in range(0, nbytes, PIN_PIECE)]

    def free(self):
        for p in self._ptrs:
            self._hip.hipHostFree(self._ct.c_void_p(p))
        self._ptrs = []


class PeriodicCheckpointer:
    """Asynchronous periodic checkpoints with an atomically published ``latest`` (module doc).

    ``save(step)`` returns once the snapshot is queued: on a GPU the device-to-host copies run
    on a side stream into pinned buffers that are allocated once and reused, and the trainer's
    NEXT optimizer update stream-waits for them (``trainer.pre_opt_waits``) -- the only point
    where the step can be slowed.  A writer thread streams the files out; rank 0 publishes."""

    def __init__(self, root: str, trainer, data=None, keep: int = 2, publish_timeout: float = 1800.0,
                 on_published=None):
        import torch.distributed as dist
        self.root, self.trainer, self.data = root, trainer, data
        self.keep = max(1, int(keep))
        self.publish_timeout = publish_timeout
        self.on_published = on_published
        self.rank, self.world = _rank(), _world()
        self.flat = hasattr(trainer, "model") and hasattr(trainer.model, "groups")
        st = getattr(trainer, "st", None)
        self.device = getattr(st, "device", torch.device("cpu")) if st is not None else torch.device("cpu")
        # one token per world: a rank's done marker left by a killed earlier world for the same
        # step number is never mistaken for this world's
        tok = [uuid.uuid4().hex if self.rank == 0 else None]
        if dist.is_initialized() and self.world > 1:
            dist.broadcast_object_list(tok, src=0)
        self.token = tok[0]
        os.makedirs(root, exist_ok=True)
        self._pinned: Dict[str, HostPieces] = {}
        self._stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        self._pin = PinnedPieces() if self._stream is not None else None
        # page-locking the host snapshot (112 GB at 8B on one rank) takes seconds: done once, on a
        # side thread (GIL-free, in pieces: PinnedPieces), so the first save() finds the buffers
        # ready instead of stalling.  The thread starts at start_prep(), which the worker calls
        # once its first step has completed (KFAMD_CKPT_PREPIN=init: at construction; =0: never,
        # the first save allocates)
        self._prep = None
        self._prep_shapes = None
        mode = os.environ.get("KFAMD_CKPT_PREPIN", "1")
        if self._stream is not None and self.flat and mode != "0":
            self._prep_shapes = {k: (tuple(v.shape), v.dtype) for k, v in _flat_state(trainer)[0].items()}
            if mode == "init":
                self.start_prep()
        # device staging: when the card has room for a second copy of the state beside the step's
        # peak, the snapshot is a device-to-device copy (~3 TB/s) that the next optimizer update
        # waits for, and the device-to-host copy (~56 GB/s) runs from that copy while the
        # following steps proceed.  Decided at the first save (the peak is known by then);
        # KFAMD_CKPT_DEVICE_STAGE=0 turns it off.
        self._stage: Optional[Dict[str, torch.Tensor]] = None
        self._stage_decided = self._stream is None or os.environ.get("KFAMD_CKPT_DEVICE_STAGE", "1") == "0"
        self.staged = False
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        self.last_published: Optional[int] = None
        self.last_seconds: Optional[float] = None
        self.snapshot_seconds: Optional[float] = None

    def start_prep(self):
        """Start page-locking the snapshot buffers on a side thread (once).  Pinning tens of GB
        while the first step was being launched delayed that step by ~1 s (profiles/
        restart_gpu_r6.md), so the worker starts it after its first step."""
        if self._prep is None and self._prep_shapes is not None:
            shapes, self._prep_shapes = self._prep_shapes, None
            self._prep = threading.Thread(target=self._allocate_pinned, args=(shapes,), name="kfamd-ckpt-pin",
                                          daemon=True)
            self._prep.start()

    def _host_buffer(self, shape, dtype) -> HostPieces:
        n = 1
        for d in shape:
            n *= int(d)
        return HostPieces(shape, dtype, self._pin.pieces(n * torch.empty((), dtype=dtype).element_size()))

    def _allocate_pinned(self, shapes):
        for k, (shape, dtype) in shapes.items():
            self._pinned[k] = self._host_buffer(shape, dtype)

    # -- snapshot (caller's thread)
    STAGE_MARGIN = 8 << 30          # HBM left free beside the step's peak and the staging copy

    def _decide_stage(self, tensors: Dict[str, torch.Tensor]):
        self._stage_decided = True
        need = sum(t.numel() * t.element_size() for t in tensors.values())
        total = torch.cuda.get_device_properties(self.device).total_memory
        peak = torch.cuda.max_memory_allocated(self.device)
        if peak + need + self.STAGE_MARGIN <= total:
            self._stage = {k: torch.empty_like(v) for k, v in tensors.items()}
            self.staged = True

    def _host_copy(self, key: str, t: torch.Tensor):
        if self._stream is None:
            return t.detach().contiguous().clone()
        buf = self._pinned.get(key)
        if buf is None or buf.shape != tuple(t.shape) or buf.dtype != t.dtype:
            buf = self._pinned[key] = self._host_buffer(tuple(t.shape), t.dtype)
        src = t.detach().reshape(-1).view(torch.uint8)
        a = 0
        for piece in buf.pieces:
            piece.copy_(src[a:a + piece.numel()], non_blocking=True)
            a += piece.numel()
        return buf

    def save(self, step: int):
        """Snapshot the state after optimizer step ``step`` and write it in the background."""
        self.wait()                       # the previous write owns the pinned buffers
        if self._prep is not None:
            self._prep.join()
            self._prep = None
        tr = self.trainer
        t0 = time.perf_counter()
        path = step_dir(self.root, step)
        if not self.flat:                 # plain nn.Module jobs (MNIST): small, synchronous
            save_module_checkpoint(path, tr, step, self.data)
            self._done_marker(path)
            if self.rank == 0:
                self._publish(path, step, t0)
            return
        if hasattr(tr, "sync_params"):
            tr.sync_params()              # in-flight ZeRO-1 parameter gathers land first
        tp_check_all(tr.st)
        tensors, meta, plan = _flat_state(tr)
        meta["token"] = self.token
        rank_state = {k: v.contiguous().clone() for k, v in _rank_state(self.data).items()}
        host = {}
        ev = None
        if self._stream is not None:
            if not self._stage_decided:
                self._decide_stage(tensors)
            self._stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._stream):
                src = tensors
                if self._stage is not None:
                    for k, v in tensors.items():
                        self._stage[k].copy_(v, non_blocking=True)
                    src = self._stage
                ev_state = torch.cuda.Event()
                ev_state.record(self._stream)      # the state has been read (into the staging copy)
                for k, v in src.items():
                    host[k] = self._host_copy(k, v)
            ev = torch.cuda.Event()
            ev.record(self._stream)                # ... and is on the host
            # the next optimizer update rewrites master / m / v / params: it waits for the state
            # to have been read -- the device copy when staged, else the host copy
            gate = ev_state if self._stage is not None else ev
            waits = getattr(tr, "pre_opt_waits", None)
            if waits is not None:
                waits.append(gate)
            else:
                gate.synchronize()
        else:
            host = {k: self._host_copy(k, v) for k, v in tensors.items()}
        self.snapshot_seconds = time.perf_counter() - t0
        self._thread = threading.Thread(target=self._write, name="kfamd-ckpt-writer", daemon=True,
                                        args=(path, step, plan, host, rank_state, meta, ev, t0))
        self._thread.start()

    # -- writer thread
    def _write(self, path, step, plan, host, rank_state, meta, ev, t0):
        try:
            if ev is not None:
                ev.synchronize()
            os.makedirs(path, exist_ok=True)
            _write_plan(path, plan, host)
            write_safetensors(os.path.join(path, f"rank{self.rank}.state.safetensors"), rank_state)
            if self.rank == 0:
                _write_json(os.path.join(path, "meta.json"), meta)
            self._done_marker(path, sorted(plan))
            if self.rank == 0:
                self._publish(path, step, t0)
        except BaseException as e:        # noqa: BLE001 -- surfaced by wait() on the main thread
            self._error = e

    def _done_marker(self, path: str, files=None):
        _fsync_dir(path)
        rec = {"token": self.token}
        if files is not None:
            rec["files"] = list(files)
        _write_json(os.path.join(path, f"rank{self.rank}.done"), rec)

    def _all_done(self, path: str) -> bool:
        for r in range(self.world):
            try:
                with open(os.path.join(path, f"rank{r}.done")) as f:
                    if json.load(f).get("token") != self.token:
                        return False
            except (OSError, ValueError):
                return False
        return True

    def _publish(self, path: str, step: int, t0: float):
        deadline = time.time() + self.publish_timeout
        while not self._all_done(path):
            if time.time() > deadline:
                raise TimeoutError(f"checkpoint {path}: not every rank finished within {self.publish_timeout:.0f} s")
            time.sleep(0.05)
        _fsync_dir(path)
        tmp = os.path.join(self.root, LATEST + ".tmp")
        with open(tmp, "w") as f:
            f.write(os.path.basename(path) + "\n")
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, os.path.join(self.root, LATEST))
        _fsync_dir(self.root)
        self.last_published = step
        self.last_seconds = time.perf_counter() - t0
        self._prune(os.path.basename(path))
        if self.on_published is not None:
            self.on_published(step, self.last_seconds)

    def _prune(self, newest: str):
        import shutil
        dirs = sorted(d for d in os.listdir(self.root) if _STEP_DIR.match(d))
        done = [d for d in dirs if d <= newest]
        for d in done[:-self.keep]:
            shutil.rmtree(os.path.join(self.root, d), ignore_errors=True)

    def wait(self):
        """Block until the in-flight write (if any) has finished; re-raise its error."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError(f"checkpoint write failed: {e}") from e

    def close(self):
        self.wait()
        if self._prep is not None:
            self._prep.join()
            self._prep = None
        if self._pin is not None:
            if self._stream is not None:
                self._stream.synchronize()
            self._pinned = {}
            self._stage = None
            self._pin.free()
