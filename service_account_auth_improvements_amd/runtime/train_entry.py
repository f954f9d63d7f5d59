"""Worker entry point run inside PyTorchJob / MPIJob pods (one process per GPU, started by
kfamd-launch).  Emits JSON event lines (``first_step`` carries the wall-clock timestamp
used for the CRD-to-first-step metric), touches the launcher heartbeat file every step,
serves Prometheus ``/metrics`` when ``KFAMD_METRICS_PORT`` is set (runtime/metrics.py),
writes periodic asynchronous checkpoints and resumes from the newest one on (re)start
(``--ckpt-dir`` / ``--save-every``, runtime/checkpoint.py), and saves a sharded checkpoint
at the end when asked (``--save``).

The step loop is the benched loop (bench.py): it never synchronises the device per step.
After the first step (one synchronisation, for the ``first_step`` event) each step's loss is
copied to pinned memory on the compute stream and its end event recorded; the host reads
step N-1's loss and device time while step N is already queued, so the GPU always has the
next step to run (tests/test_worker_loop.py).

  python -m service_account_auth_improvements_amd.runtime.train_entry \
      --model llama3-8b --seq-len 8192 --micro-batch 2 --steps 100 \
      --ckpt-dir /mnt/ckpt --save-every 50
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def _device_sync():
    import torch
    torch.cuda.synchronize()


def _end_event():
    """The step's end marker on the compute stream (its timing gives the device step time)."""
    import torch
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    return ev


def _host_scalar(loss):
    """A pinned host copy of the loss, queued on the compute stream (read once the end event
    has completed)."""
    import torch
    h = torch.empty((), dtype=loss.dtype, pin_memory=True)
    h.copy_(loss.detach(), non_blocking=True)
    return h


class _StepRecord:
    __slots__ = ("step", "loss", "event", "t_host")

    def __init__(self, step, loss, cuda: bool):
        self.step = step
        self.t_host = time.perf_counter()
        if cuda:
            self.loss = _host_scalar(loss) if loss is not None else None
            self.event = _end_event()
        else:
            self.loss = loss.detach() if loss is not None else None
            self.event = None

    def finish(self):
        """Wait for this step's end (the NEXT step is already queued) and read its loss."""
        if self.event is not None:
            self.event.synchronize()
        return float(self.loss) if self.loss is not None else None

    def seconds_since(self, prev: "_StepRecord"):
        if prev is None:
            return None
        if self.event is not None:
            return prev.event.elapsed_time(self.event) / 1e3
        return self.t_host - prev.t_host


def _event(kind: str, **kw):
    rec = {"event": kind, "ts": time.time(), "rank": int(os.environ.get("RANK", "0")), "pid": os.getpid(), **kw}
    line = json.dumps(rec)
    print(line, flush=True)
    path = os.environ.get("KFAMD_EVENTS_FILE")
    if path:
        with open(path, "a") as f:
            f.write(line + "\n")


def _heartbeat():
    hb = os.environ.get("KFAMD_HEARTBEAT_FILE")
    if hb:
        with open(hb, "a"):
            os.utime(hb, None)


def _hip_preinit(device_arg: str):
    """Start HIP runtime + device initialisation on a side thread BEFORE ``import torch``, so the
    ~0.2 s of runtime / device / context set-up runs under the ~1.4 s import instead of after it
    (CRD-to-first-step; profiles/crd_to_first_step_r6.md).  It loads the very HIP runtime torch
    will use (torch/lib/libamdhip64.so, found without importing torch: one runtime per process),
    counts devices, selects this rank's (LOCAL_RANK modulo the count, as
    parallel/state.local_device_index) and creates its context with ``hipFree(NULL)``.
    ``KFAMD_HIP_PREINIT=0`` or ``--device cpu`` turns it off; any failure leaves the work to
    torch's own lazy init.  ``KFAMD_HIP_PREINIT=after-c`` starts the device work only once the
    import has loaded ``torch._C`` (its native libraries, the HIP runtime among them), so the
    runtime init overlaps the Python part of the import but not its dynamic loading."""
    mode = os.environ.get("KFAMD_HIP_PREINIT", "1")
    if device_arg == "cpu" or mode == "0":
        return None
    import ctypes
    import importlib.util
    import threading
    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        return None
    lib = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if not os.path.exists(lib) or not os.path.exists("/dev/kfd"):
        return None

    def run():
        try:
            if mode == "after-c":
                import sys
                import time as _t
                deadline = _t.monotonic() + 30.0
                while "torch._C" not in sys.modules and _t.monotonic() < deadline:
                    _t.sleep(0.005)
            h = ctypes.CDLL(lib, mode=ctypes.RTLD_GLOBAL)
            n = ctypes.c_int(0)
            if h.hipGetDeviceCount(ctypes.byref(n)) != 0 or n.value < 1:
                return
            if h.hipSetDevice(int(os.environ.get("LOCAL_RANK", "0")) % n.value) == 0:
                h.hipFree(ctypes.c_void_p(0))
        except Exception:   # noqa: BLE001 -- torch's lazy init does the same work later
            pass
    t = threading.Thread(target=run, name="kfamd-hip-preinit", daemon=True)
    t.start()
    return t


def _warm_blas(index: int):
    """A fresh GPU process pays ~0.6 s of first-use costs before its first step can run: HIP
    runtime / device init (~0.2 s), hipBLASLt's first GEMM (library and kernel catalog, ~0.17 s),
    the HIP extension's code objects on its first launch (~0.19 s) -- tools/probe_first_use.py.
    Paid on two side threads (this one: hipBLASLt; `_warm_ext`: the extension), concurrently
    with each other and with the main thread's rendezvous and trainer construction (everything
    they share is lock-protected: torch's lazy CUDA init, ops/_ext.load).  Errors are left for
    the main thread to hit and report."""
    try:
        import torch
        torch.cuda.set_device(index)
        a = torch.zeros(128, 128, device=f"cuda:{index}", dtype=torch.bfloat16)
        torch.mm(a, a)
        torch.cuda.synchronize(index)
    except Exception:       # noqa: BLE001 -- the main thread reports real failures
        pass


def _warm_ext(index: int):
    """The in-tree HIP extension: load the library and launch one kernel (see _warm_blas)."""
    try:
        import torch
        torch.cuda.set_device(index)
        from ..ops import _ext
        if _ext.load():
            from .. import ops
            a = torch.zeros(128, 128, device=f"cuda:{index}", dtype=torch.bfloat16)
            ops.rmsnorm_fwd(a, torch.ones(128, device=a.device, dtype=a.dtype), 1e-5)
            torch.cuda.synchronize(index)
    except Exception:       # noqa: BLE001
        pass


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=8192)
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10,
                    help="steps to run; with --ckpt-dir the job's TOTAL step count (a restarted world runs "
                         "only what is left after the checkpoint it resumed from)")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--pp", type=int, default=1)
    ap.add_argument("--pp-virtual", type=int, default=1,
                    help="model chunks per pipeline rank (> 1: interleaved 1F1B; --grad-accum a multiple of --pp)")
    ap.add_argument("--zero1", action="store_true")
    ap.add_argument("--sp", action="store_true", help="sequence parallelism on top of --tp (Megatron SP)")
    ap.add_argument("--cp", action="store_true",
                    help="context parallelism: the data-parallel ranks share each sequence (long context)")
    ap.add_argument("--recompute", action="store_true", help="per-layer activation recomputation")
    ap.add_argument("--grad-reduce", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--head-chunk", type=int, default=4096)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    ap.add_argument("--save", default=None, help="checkpoint directory written at the end")
    ap.add_argument("--resume", default=None, help="checkpoint directory to resume from")
    ap.add_argument("--ckpt-dir", default=os.environ.get("KFAMD_CKPT_DIR") or None,
                    help="periodic checkpoints (a PVC path shared by the job's pods): step-N/ directories and "
                         "an atomically published 'latest'; every (re)start resumes from 'latest'")
    ap.add_argument("--save-every", type=int, default=int(os.environ.get("KFAMD_SAVE_EVERY", "0") or 0),
                    help="steps between periodic checkpoints (0 = none)")
    ap.add_argument("--keep-checkpoints", type=int, default=2)
    a = ap.parse_args(argv)

    t_start = time.time()
    _event("process_start")
    pre = _hip_preinit(a.device)
    if os.environ.get("KFAMD_METRICS_PORT", "") != "":
        # the communicator records start/end events per collective: the /metrics bus bandwidth
        os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")
    import torch
    from ..parallel.state import init_distributed, local_device_index
    from .trainer import SyntheticData, TrainConfig, Trainer
    _event("imported", seconds=time.time() - t_start, hip_preinit=pre is not None)

    dev = None if a.device == "auto" else a.device
    if dev == "cuda" or (dev is None and torch.cuda.is_available()):
        dev = "cuda"
    else:
        dev = "cpu"
    warm = []
    if dev == "cuda" and os.environ.get("KFAMD_WARM", "1") != "0":
        import threading
        # the device init_distributed will select (not the raw LOCAL_RANK, which differs in the
        # several-ranks-per-GPU gloo rehearsal)
        idx = local_device_index()
        warm = [threading.Thread(target=f, args=(idx,), name=f"kfamd-{f.__name__[1:]}", daemon=True)
                for f in (_warm_blas, _warm_ext)]
        for t in warm:
            t.start()
    st = init_distributed(tp=a.tp, pp=a.pp, device=dev)
    _event("dist_ready", seconds=time.time() - t_start)
    if a.model == "mnist":     # BASELINE configs[0]: operator/launcher plumbing job
        from ..models.mnist import MnistTrainer, SyntheticMnist
        tr = MnistTrainer(st.device)
        data = SyntheticMnist(a.micro_batch, st.device, seed=17, rank=st.dp_rank)
        tokens = a.micro_batch * a.grad_accum
    else:
        tcfg = TrainConfig(model=a.model, seq_len=a.seq_len, micro_batch=a.micro_batch, grad_accum=a.grad_accum,
                           zero1=a.zero1, n_layers=a.layers, sequence_parallel=a.sp, context_parallel=a.cp,
                           recompute=a.recompute,
                           grad_reduce=a.grad_reduce, head_chunk=a.head_chunk, pp_virtual=a.pp_virtual)
        if a.pp > 1:
            from ..parallel.pipeline import PipelineTrainer
            tr = PipelineTrainer(tcfg, st)
        else:
            tr = Trainer(tcfg, st)
        data = SyntheticData(tr.mcfg.vocab_size, a.micro_batch, a.seq_len, st.device, seed=17,
                             rank=0 if a.cp else st.dp_rank)     # --cp: the group shares its sequences
        tokens = a.micro_batch * a.seq_len * a.grad_accum
    resume = a.resume
    if resume is None and a.ckpt_dir:
        from .checkpoint import latest_checkpoint
        resume = latest_checkpoint(a.ckpt_dir)
    if resume:
        # weights, optimizer state, step, RNG and the data stream position: the resumed job
        # continues exactly where it stopped instead of replaying batches it already saw
        from .checkpoint import load_checkpoint
        meta = load_checkpoint(resume, tr, data=data)
        tr.step_idx = int(meta["step"])
        _event("resumed", path=resume, step=int(meta["step"]), auto=a.resume is None)
    for t in warm:
        t.join()
    return _loop(a, tr, data, st, t_start, tokens)


def _loop(a, tr, data, st, t_start, tokens_per_step):
    import torch
    from . import metrics as metrics_mod
    _event("init_done", seconds=time.time() - t_start, **getattr(tr, "init_times", {}))
    start = int(getattr(tr, "step_idx", 0))
    end = max(start, a.steps) if a.ckpt_dir else start + a.steps
    cuda = st.device.type == "cuda"
    mx = metrics_mod.from_env(st.rank, int(os.environ.get("LOCAL_RANK", "0")))
    reducer = getattr(tr, "reducer", None)
    if mx is not None:
        _event("metrics_serving", port=mx.port)
        if reducer is not None and reducer.enabled:
            import torch.distributed as dist
            from ..parallel.ddp import CollectiveStats
            reducer.stats = CollectiveStats(st.dp, host_timed=dist.get_backend(reducer.dp_group) != "nccl")
    ckpt = None
    if a.ckpt_dir and a.save_every > 0:
        from .checkpoint import PeriodicCheckpointer

        def published(step, secs):
            _event("checkpoint_published", step=step, seconds=round(secs, 3))
            if mx is not None:
                mx.observe_checkpoint(step, secs)
        ckpt = PeriodicCheckpointer(a.ckpt_dir, tr, data=data, keep=a.keep_checkpoints, on_published=published)
    prev = pending = None

    def emit(rec):
        lv = rec.finish()
        secs = rec.seconds_since(prev)
        _event("step", step=rec.step, loss=lv, **({"step_s": round(secs, 6)} if secs is not None else {}))
        if mx is not None:
            mx.observe_step(secs, tokens_per_step, lv)
            mx.observe_memory(st.device)
            mx.observe_collectives(getattr(reducer, "stats", None))

    for step in range(start, end):
        batch = [data.next() for _ in range(a.grad_accum)]
        loss = tr.train_step(batch)
        rec = _StepRecord(step, loss, cuda)
        if step == start:
            if cuda:
                _device_sync()           # once: the first_step timestamp is a completed step
            _event("first_step", loss=float(rec.loss) if rec.loss is not None else None)
            if ckpt is not None:
                ckpt.start_prep()        # page-lock the snapshot buffers now, off the first step
        if pending is not None:
            emit(pending)                # step N-1, while step N runs on the device
            prev = pending
        pending = rec
        _heartbeat()
        if ckpt is not None and (step + 1) % a.save_every == 0 and step + 1 < end:
            ckpt.save(step + 1)
            _event("checkpoint_queued", step=step + 1, device_staged=ckpt.staged)
    if pending is not None:
        emit(pending)
    if ckpt is not None:
        ckpt.close()
    if getattr(st, "tp_comm", None) is not None:
        # the per-step check reads the error word one step late -- read the last
        # steps' word now, before reporting success
        from .checkpoint import tp_check_all
        tp_check_all(st)
    if a.save:
        from .checkpoint import save_checkpoint
        save_checkpoint(a.save, tr, data=data)
        _event("checkpoint_saved", path=a.save)
    _event("done")
    if mx is not None:
        mx.close()
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    # hand the ~200 GB of HBM back before the process exits, so the driver's reclaim runs
    # while this pod is still terminating instead of stalling the next pod's first allocation
    if hasattr(tr, "release"):
        tr.release()
    if torch.cuda.is_available() and st.device.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
