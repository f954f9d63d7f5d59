"""Pipeline parallelism: 1F1B schedule over point-to-point RCCL send/recv (C5).

Each pipeline stage is a :class:`..models.llama.Llama` shard holding a contiguous layer
range (stage 0 also the embedding, the last stage the final norm + LM head + CE).  The
boundary activation is one [micro_batch * seq, hidden] bf16 tensor; on an xGMI mesh every
stage pair has a direct link, so a stage hop is a single point-to-point transfer.

Schedule (non-interleaved 1F1B): stage r runs ``pp - r - 1`` warm-up forwards, then
alternates one forward / one backward, then drains the remaining backwards.  Send and
receive of opposite directions are posted together through ``batch_isend_irecv`` so no
ordering of blocking calls can deadlock; send-only groups are left in flight behind the next
micro-batch's compute (:class:`P2P`).  Only ``pp - r`` micro-batches of activations are ever
alive on stage r.  With ``zero1`` every stage's DP group shards its optimizer state (ZeRO-1).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..models.llama import Llama, LlamaConfig
from .ddp import GradReducer
from .state import ParallelState


def stage_layers(n_layers: int, pp: int, rank: int) -> range:
    """Even split of layers; the remainder goes to the middle stages (the first stage
    also owns the embedding, the last the 128k-vocab LM head)."""
    base, rem = divmod(n_layers, pp)
    sizes = [base] * pp
    order = list(range(1, pp - 1)) + [0, pp - 1] if pp > 2 else list(range(pp))
    for i in range(rem):
        sizes[order[i % len(order)]] += 1
    start = sum(sizes[:rank])
    return range(start, start + sizes[rank])


class P2P:
    """Stage-boundary point-to-point transfers.  A group that only SENDS is not waited for: the
    compute stream goes on with the next micro-batch while the activation (or its gradient)
    is on the wire -- at micro-batch 4 x 8k tokens a boundary tensor is 268 MB, several ms on
    one xGMI link.  Its tensor is kept alive until :meth:`flush` (end of the step).  Receives
    are waited for (a stream dependency under RCCL) before their data is used.  Every group
    pairs with one posted by the peer in the same order, and a receive is never posted ahead
    of a send the peer needs first: RCCL runs P2P groups in order on one stream.

    Live boundary tensors stay bounded by ``max_inflight`` (= max(2, pp), the 1F1B bound), not by
    the step's micro-batch x chunk count: after every post, records of groups that have completed
    are dropped (a completed group needs no wait), and the oldest still-running send-carrying
    groups beyond the cap are waited for.  A group record keeps only its SEND tensors alive; its
    receive buffers belong to whoever :meth:`take` s them."""

    def __init__(self, st: ParallelState, shape, dtype, device):
        self.st, self.shape, self.dtype, self.device = st, shape, dtype, device
        # gloo (the one-GPU rehearsal backend) moves send/recv payloads without ordering them
        # against the HIP stream, so GPU tensors are staged through host memory there; RCCL
        # orders its own stream against the compute stream.
        self._host = torch.device(device).type == "cuda" and dist.get_backend() == "gloo"
        self._inflight: list = []       # (works, tensors) of send-only groups not yet waited for
        self._groups: list = []         # interleaved schedule: (group record, send tensors)
        self.sends_deferred = 0         # send-only groups left in flight (tests)
        self.max_inflight = max(2, st.pp)
        self.peak_live = 0              # most un-retired send-carrying groups held at once (tests)
        self._seq = 0

    def _buf(self):
        return torch.empty(self.shape, dtype=self.dtype, device=self.device)

    # -- interleaved schedule: ring neighbours and tick exchanges (see interleaved_1f1b)
    @property
    def ring_next(self) -> int:
        st = self.st
        return ((((st.pp_rank + 1) % st.pp) * st.dp + st.dp_rank) * st.tp + st.tp_rank)

    @property
    def ring_prev(self) -> int:
        st = self.st
        return ((((st.pp_rank - 1) % st.pp) * st.dp + st.dp_rank) * st.tp + st.tp_rank)

    def exchange(self, sends, recvs):
        """Post one group: ``sends`` = [(tensor, peer)], ``recvs`` = [(kind, key, peer)].
        Returns [(kind, key, peer, handle)]; :meth:`take` waits for a handle and returns its
        tensor.  Send-only groups are deferred like the 1F1B path's."""
        ops_ = [dist.P2POp(dist.isend, t.contiguous(), peer) for t, peer in sends]
        bufs = [(kind, key, peer, self._buf()) for kind, key, peer in recvs]
        ops_ += [dist.P2POp(dist.irecv, b, peer) for _, _, peer, b in bufs]
        if not ops_:
            return []
        if not bufs or self._host:
            self._run(ops_)              # gloo + GPU tensors: staged and waited here
            return [(kind, key, peer, (None, b)) for kind, key, peer, b in bufs]
        # one record per group, waited at most once (a second wait() on a completed gloo receive
        # waits for ANOTHER message): by the first take() of one of its tensors, else by flush()
        grp = {"works": dist.batch_isend_irecv(ops_), "done": False}
        if sends:
            self._seq += 1
            self._groups.append((grp, [op.tensor for op in ops_[:len(sends)]], self._seq))
            self._retire()
        return [(kind, key, peer, (grp, b)) for kind, key, peer, b in bufs]

    @staticmethod
    def _completed(works) -> bool:
        return all(w.is_completed() for w in works)

    def _retire(self):
        """Drop finished group records; wait for the oldest running ones beyond the cap."""
        keep = []
        for rec in self._groups:
            grp = rec[0]
            if not grp["done"] and self._completed(grp["works"]):
                grp["done"] = True           # its receives are complete: take() returns at once
            if not grp["done"]:
                keep.append(rec)
        self._groups = keep
        self._inflight = [x for x in self._inflight if not self._completed(x[0])]
        # the cap covers both kinds of record together, oldest post first
        while len(self._groups) + len(self._inflight) > self.max_inflight:
            if self._inflight and (not self._groups or self._inflight[0][2] < self._groups[0][2]):
                for w in self._inflight.pop(0)[0]:
                    w.wait()
            else:
                grp = self._groups.pop(0)[0]
                for w in grp["works"]:
                    w.wait()
                grp["done"] = True
        self.peak_live = max(self.peak_live, len(self._groups) + len(self._inflight))

    @staticmethod
    def take(handle):
        grp, t = handle
        if grp is not None and not grp["done"]:
            for w in grp["works"]:
                w.wait()
            grp["done"] = True
        return t

    def flush(self):
        """Wait for every deferred send (before the optimizer step reuses any buffer)."""
        for works, _, _ in self._inflight:
            for w in works:
                w.wait()
        self._inflight.clear()
        for grp, _, _ in self._groups:
            if not grp["done"]:
                for w in grp["works"]:
                    w.wait()
                grp["done"] = True
        self._groups.clear()

    def _run(self, ops):
        if not ops:
            return
        if all(op.op is dist.isend for op in ops):
            if self._host:
                ops = [dist.P2POp(dist.isend, op.tensor.cpu(), op.peer) for op in ops]
            self._seq += 1
            self._inflight.append((dist.batch_isend_irecv(ops), [op.tensor for op in ops], self._seq))
            self.sends_deferred += 1
            self._retire()
            return
        copies = []
        if self._host:
            staged = []
            for op in ops:
                if op.op is dist.isend:
                    staged.append(dist.P2POp(dist.isend, op.tensor.cpu(), op.peer))
                else:
                    h = torch.empty(op.tensor.shape, dtype=op.tensor.dtype)
                    copies.append((op.tensor, h))
                    staged.append(dist.P2POp(dist.irecv, h, op.peer))
            ops = staged
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        for dev_t, h in copies:
            dev_t.copy_(h)

    def recv_forward(self):
        if self.st.pp_prev is None:
            return None
        x = self._buf()
        self._run([dist.P2POp(dist.irecv, x, self.st.pp_prev)])
        return x

    def send_forward(self, y):
        if self.st.pp_next is not None:
            self._run([dist.P2POp(dist.isend, y.contiguous(), self.st.pp_next)])

    def recv_backward(self):
        if self.st.pp_next is None:
            return None
        g = self._buf()
        self._run([dist.P2POp(dist.irecv, g, self.st.pp_next)])
        return g

    def send_backward(self, g):
        if self.st.pp_prev is not None and g is not None:
            self._run([dist.P2POp(dist.isend, g.contiguous(), self.st.pp_prev)])

    def send_forward_recv_backward(self, y):
        if self.st.pp_next is None:
            return None
        g = self._buf()
        self._run([dist.P2POp(dist.isend, y.contiguous(), self.st.pp_next),
                   dist.P2POp(dist.irecv, g, self.st.pp_next)])
        return g

    def send_backward_recv_forward(self, g):
        if self.st.pp_prev is None:
            return None
        x = self._buf()
        ops = [dist.P2POp(dist.irecv, x, self.st.pp_prev)]
        if g is not None:
            ops.insert(0, dist.P2POp(dist.isend, g.contiguous(), self.st.pp_prev))
        self._run(ops)
        return x


def one_f_one_b(model: Llama, p2p: P2P, micro_batches: List[Tuple[torch.Tensor, torch.Tensor]],
                scale: float, on_last_backward=None, reducer=None) -> Optional[torch.Tensor]:
    """Run one optimizer step's worth of micro-batches through this stage.
    Returns the summed (scaled) loss on the last stage, None elsewhere.  With a ``reducer``
    doing fp32 micro-batch accumulation every backward writes fresh gradients and the
    non-final ones are added into its fp32 buffer."""
    st = p2p.st
    M = len(micro_batches)
    B, S = micro_batches[0][0].shape
    warm = min(st.pp - st.pp_rank - 1, M)
    steady = M - warm
    ctxs, total, losses = [], None, []
    n_bwd = 0

    def fwd(i, x):
        tok, lab = micro_batches[i]
        inp = tok.reshape(-1) if model.first else x
        out, ctx = model.stage_forward(inp, B, S, lab.reshape(-1), scale)
        ctxs.append(ctx)
        if model.last:
            losses.append(out)     # filled in by this micro-batch's head backward (K5)
            return None
        return out

    def bwd(g):
        nonlocal n_bwd
        ctx = ctxs.pop(0)
        if n_bwd == M - 1 and on_last_backward is not None:
            on_last_backward(True)
        f32acc = reducer is not None and reducer.fp32_accumulation
        gin = model.stage_backward(ctx, g, B, S, accumulate=n_bwd > 0 and not f32acc)
        if reducer is not None and n_bwd < M - 1:
            reducer.accumulate_micro(first=n_bwd == 0)
        n_bwd += 1
        return gin

    for i in range(warm):
        x = p2p.recv_forward()
        p2p.send_forward(fwd(i, x))
    x = p2p.recv_forward() if steady > 0 else None
    for j in range(steady):
        y = fwd(warm + j, x)
        g = p2p.send_forward_recv_backward(y) if not model.last else None
        gin = bwd(g)
        if j == steady - 1:
            p2p.send_backward(gin)
        else:
            x = p2p.send_backward_recv_forward(gin)
    for _ in range(warm):
        g = p2p.recv_backward()
        p2p.send_backward(bwd(g))
    if on_last_backward is not None:
        on_last_backward(False)
    p2p.flush()
    for lv in losses:
        total = lv if total is None else total + lv
    return total


# ---------------------------------------------------------------------------------------------
# Interleaved 1F1B (virtual pipeline stages)
# ---------------------------------------------------------------------------------------------
# Each rank holds v layer chunks; chunk c of rank r is virtual stage c*pp + r, so a micro-batch
# passes every rank v times and the fill/drain bubble shrinks by v.  The per-rank op order is
# the usual interleaved one (micro-batches in groups of pp, chunk-major inside a group; warm-up
# 2(pp - r - 1) + (v - 1) pp forwards, then one forward / one backward, then the drain).
#
# Transfers: every rank simulates the SAME global timeline -- in each tick a rank runs its next
# op if that op's inputs were produced in an earlier tick -- and in tick t posts one P2P group:
# the output it produced in tick t (to the ring neighbour that consumes it) plus receives for
# what its two neighbours produced in tick t for it.  Both ends of every transfer derive it from
# the same simulation, so the groups match pairwise and nothing can deadlock.  A received tensor
# is waited for only when the op that consumes it runs (a stream dependency under RCCL), and
# send-only groups stay in flight until the end of the step.


def interleaved_order(pp: int, v: int, M: int, rank: int) -> List[Tuple[str, int, int]]:
    """Op list ("F" | "B", micro-batch, chunk) of pipeline rank ``rank``."""
    assert M % pp == 0, f"interleaved schedule: micro-batches ({M}) must be a multiple of pp ({pp})"
    N = M * v

    def mb(k):
        return (k // (pp * v)) * pp + k % pp

    def fchunk(k):
        return (k // pp) % v

    def bchunk(k):
        return v - 1 - (k // pp) % v

    warm = N if M == pp else min(N, 2 * (pp - rank - 1) + (v - 1) * pp)
    ops_: List[Tuple[str, int, int]] = [("F", mb(k), fchunk(k)) for k in range(warm)]
    for i in range(N - warm):
        ops_.append(("F", mb(warm + i), fchunk(warm + i)))
        ops_.append(("B", mb(i), bchunk(i)))
    ops_ += [("B", mb(k), bchunk(k)) for k in range(N - warm, N)]
    return ops_


def simulate_interleaved(pp: int, v: int, M: int):
    """Global lockstep timeline: ``ticks[t][r]`` = the op rank r runs in tick t (or None).
    An op runs once its remote input was produced in an EARLIER tick (a backward also needs
    its own forward, which always precedes it in the rank's list)."""
    orders = [interleaved_order(pp, v, M, r) for r in range(pp)]
    last_vs = pp * v - 1
    done = {}                     # (kind, m, vs) -> tick
    pos = [0] * pp
    ticks = []
    while any(pos[r] < len(orders[r]) for r in range(pp)):
        t = len(ticks)
        row = [None] * pp
        for r in range(pp):
            if pos[r] >= len(orders[r]):
                continue
            kind, m, c = orders[r][pos[r]]
            vs = c * pp + r
            if kind == "F":
                ok = vs == 0 or done.get(("F", m, vs - 1), t) < t
            else:
                ok = done.get(("F", m, vs), t) < t and (vs == last_vs or done.get(("B", m, vs + 1), t) < t)
            if ok:
                row[r] = (kind, m, c)
        if not any(row):
            raise RuntimeError("interleaved schedule simulation stalled")
        for r, op in enumerate(row):
            if op is not None:
                done[(op[0], op[1], op[2] * pp + r)] = t
                pos[r] += 1
        ticks.append(row)
    return ticks


def interleaved_1f1b(chunks: List[Llama], st: ParallelState, p2p: "P2P", micro_batches,
                     scale: float, on_last_backward=None, reducer=None) -> Optional[torch.Tensor]:
    """One optimizer step of micro-batches through this rank's ``chunks`` (virtual stages
    c*pp + pp_rank).  Returns the summed loss on the rank holding the last virtual stage."""
    pp, v, r = st.pp, len(chunks), st.pp_rank
    M = len(micro_batches)
    B, S = micro_batches[0][0].shape
    last_vs = pp * v - 1
    ticks = simulate_interleaved(pp, v, M)
    nxt, prv = p2p.ring_next, p2p.ring_prev
    acts, grads, ctxs, losses = {}, {}, {}, []
    n_bwd = [0] * v
    f32acc = reducer is not None and reducer.fp32_accumulation

    for row in ticks:
        op = row[r]
        out = None
        if op is not None:
            kind, m, c = op
            vs = c * pp + r
            model = chunks[c]
            if kind == "F":
                tok, lab = micro_batches[m]
                inp = tok.reshape(-1) if vs == 0 else p2p.take(acts.pop((m, c)))
                y, ctx = model.stage_forward(inp, B, S, lab.reshape(-1), scale)
                ctxs[(m, c)] = ctx
                if vs == last_vs:
                    losses.append(y)          # filled in by this micro-batch's head backward
                else:
                    out = y
            else:
                g = None if vs == last_vs else p2p.take(grads.pop((m, c)))
                last_of_chunk = n_bwd[c] == M - 1
                if on_last_backward is not None:
                    on_last_backward(last_of_chunk, model)
                gin = model.stage_backward(ctxs.pop((m, c)), g, B, S,
                                           accumulate=n_bwd[c] > 0 and not f32acc)
                if reducer is not None and not last_of_chunk:
                    reducer.accumulate_micro(first=n_bwd[c] == 0, groups=model.groups)
                if on_last_backward is not None and last_of_chunk:
                    on_last_backward(False, model)
                n_bwd[c] += 1
                out = gin if vs > 0 else None
        # this tick's transfers (identical derivation on both ends)
        sends, recvs = [], []
        if out is not None:
            kind = op[0]
            sends.append((out, nxt if kind == "F" else prv))
        pr, nr = (r - 1) % pp, (r + 1) % pp
        po, no = row[pr], row[nr]
        if po is not None and po[0] == "F" and po[2] * pp + pr != last_vs:
            c_me = po[2] + 1 if r == 0 else po[2]        # rank pp-1 feeds chunk c+1 of rank 0
            recvs.append(("act", (po[1], c_me), prv))
        if no is not None and no[0] == "B" and no[2] * pp + nr != 0:
            c_me = no[2] - 1 if r == pp - 1 else no[2]   # rank 0 feeds chunk c-1 of rank pp-1
            recvs.append(("grad", (no[1], c_me), nxt))
        for kind, key, peer, handle in p2p.exchange(sends, [(k, key, peer) for k, key, peer in recvs]):
            (acts if kind == "act" else grads)[key] = handle
    p2p.flush()
    total = None
    for lv in losses:
        total = lv if total is None else total + lv
    return total


class _Chunks:
    """This rank's v virtual-stage models seen as one model: the optimizer and the DP reducer
    work on all their flat groups (renamed per chunk), P / G look a parameter up by name."""

    def __init__(self, chunks: List[Llama]):
        self.chunks = chunks
        self.groups = [g for c in chunks for g in c.groups]
        self.first = chunks[0].first
        self.last = chunks[-1].last

    def _owner(self, name):
        for c in self.chunks:
            if name in c.mats._index or name in c.norms._index:
                return c
        raise KeyError(name)

    def P(self, name):
        return self._owner(name).P(name)

    def G(self, name):
        return self._owner(name).G(name)

    def __setattr__(self, key, value):
        # per-model hooks (param_wait, on_grad_ready, recompute, ...) go to every chunk
        if key in ("chunks", "groups", "first", "last"):
            object.__setattr__(self, key, value)
        else:
            for c in self.chunks:
                setattr(c, key, value)

    # settings every chunk shares; anything per chunk (mats, norms, layers, ...) must be reached
    # through ``chunks`` -- no silent fallback to chunk 0
    _SHARED = frozenset({"cfg", "st", "tp", "hq", "hkv", "ff", "vl", "device", "head_chunk", "recompute",
                         "sequence_parallel", "tp_comm_chunks", "cp", "param_wait", "on_grad_ready"})

    def __getattr__(self, key):
        if key in _Chunks._SHARED:
            return getattr(self.chunks[0], key)
        raise AttributeError(f"{key!r} is per pipeline chunk: use .chunks[c].{key}")


class PipelineTrainer:
    """DP x PP (x TP) training with 1F1B; same optimizer / reducer as the DP trainer."""

    def __init__(self, tcfg, st: ParallelState, mcfg: Optional[LlamaConfig] = None,
                 full_init: bool = False):
        from ..runtime.optim import AdamWConfig, FlatAdamW
        self.tcfg, self.st = tcfg, st
        mcfg = mcfg or LlamaConfig.preset(tcfg.model)
        if tcfg.n_layers is not None:
            mcfg = mcfg.with_(n_layers=tcfg.n_layers)
        if tcfg.seq_len > mcfg.max_seq:
            mcfg = mcfg.with_(max_seq=tcfg.seq_len)
        self.mcfg = mcfg
        self.v = v = max(1, int(getattr(tcfg, "pp_virtual", 1)))
        if v == 1:
            lr = stage_layers(mcfg.n_layers, st.pp, st.pp_rank)
            self.model = Llama(mcfg, st, layer_range=lr, seed=tcfg.seed, full_init=full_init)
        else:
            # interleaved schedule: chunk c holds virtual stage c*pp + pp_rank; its flat groups are
            # renamed per chunk (the reducer and the optimizer key their state by group name)
            assert st.pp > 1 and mcfg.n_layers >= st.pp * v, "pp_virtual needs pp > 1 and >= pp*v layers"
            chunks = []
            for c in range(v):
                lr = stage_layers(mcfg.n_layers, st.pp * v, c * st.pp + st.pp_rank)
                m = Llama(mcfg, st, layer_range=lr, seed=tcfg.seed, full_init=full_init)
                for g in m.groups:
                    g.name = f"{g.name}.v{c}"
                chunks.append(m)
            self.model = _Chunks(chunks)
        self.model.recompute = tcfg.recompute
        self.model.head_chunk = getattr(tcfg, "head_chunk", self.model.head_chunk)
        self.model.sequence_parallel = getattr(tcfg, "sequence_parallel", False)
        if self.st.tp > 1:
            self.model.tp_comm_chunks = getattr(tcfg, "tp_comm_chunks", self.model.tp_comm_chunks)
            from .custom_ar import make_tp_comm
            self.st.tp_comm = make_tp_comm(getattr(tcfg, "tp_comm", "rccl"), self.st)
        assert not getattr(tcfg, "context_parallel", False), "context parallelism is not combined with PP"
        zero1 = getattr(tcfg, "zero1", False)
        force = getattr(tcfg, "force_collectives", False)
        for m in (self.model.chunks if v > 1 else [self.model]):
            m.allocate(pad_to=st.dp * 64 if zero1 else 1)
        # ZeRO-1 per stage: each DP replica group of a stage reduce-scatters its gradients, owns
        # 1/dp of the stage's AdamW state and all-gathers the updated parameters, which the next
        # step's forward waits for bucket by bucket (as the flat DP trainer does)
        mode = "reduce_scatter" if zero1 and (st.dp > 1 or force) else "allreduce"
        self.reducer = GradReducer(self.model.groups, st.dp_group, st.dp,
                                   bucket_bytes=tcfg.bucket_mb << 20, mode=mode,
                                   reduce_dtype=getattr(tcfg, "grad_reduce", "bf16"),
                                   grad_accum=tcfg.grad_accum, force_collectives=force)
        if st.dp > 1:       # identical replicas of this stage: broadcast from its first DP rank (C2)
            self.reducer.broadcast_params(st.rank - st.dp_rank * st.tp)
        shard = None
        if mode == "reduce_scatter":
            shard = {g.name: self.reducer.shard_ranges(g, st.dp_rank) for g in self.model.groups}
        self.opt = FlatAdamW(self.model.groups,
                             AdamWConfig(lr=tcfg.lr, weight_decay=tcfg.weight_decay,
                                         max_grad_norm=tcfg.max_grad_norm),
                             shard_ranges=shard, dp_group=st.dp_group,
                             norm_groups=[st.pp_group] if st.pp > 1 else None,
                             tp_sharded={g.name: st.tp_group for g in self.model.groups
                                         if g.name.split(".")[0] == "matrices"} if st.tp > 1 else None,
                             grad_view=self.reducer.grad_view)
        self.overlap_allgather = mode == "reduce_scatter" and getattr(tcfg, "overlap_allgather", True)
        if self.overlap_allgather:
            self.model.param_wait = self.reducer.wait_params
        T = tcfg.micro_batch * tcfg.seq_len
        if self.model.sequence_parallel and st.tp > 1:
            T //= st.tp                     # stages exchange this rank's block of token rows
        self.p2p = P2P(st, (T, mcfg.hidden), torch.bfloat16, st.device)
        self.step_idx = 0          # optimizer steps taken (restored by load_checkpoint)
        self.pre_opt_waits: list = []   # asynchronous checkpoint snapshots (runtime/checkpoint.py)

    def _hook(self, on: bool, model=None):
        (model if model is not None else self.model).on_grad_ready = self.reducer.grad_ready if on else None

    def train_step(self, micro_batches):
        ntok = sum(t.numel() for t, _ in micro_batches)
        self.reducer.start_step()
        if self.v > 1:
            loss = interleaved_1f1b(self.model.chunks, self.st, self.p2p, micro_batches, 1.0 / ntok, self._hook,
                                    reducer=self.reducer)
        else:
            loss = one_f_one_b(self.model, self.p2p, micro_batches, 1.0 / ntok, self._hook, reducer=self.reducer)
        self.reducer.wait_all_params()     # a bucket the forward never read (padding) must land too
        self.reducer.finish()
        from ..runtime.trainer import wait_pre_opt
        wait_pre_opt(self)
        self.opt.step(grad_scale=1.0 / self.st.dp)
        self.reducer.all_gather_params(overlap=self.overlap_allgather)
        self.step_idx += 1
        if self.st.tp_comm is not None:
            self.st.tp_comm.check()          # two-shot TP collectives: fail loudly on a lost peer
        return loss

    def sync_params(self):
        """Complete in-flight ZeRO-1 parameter gathers (before checkpoint, eval or host reads)."""
        self.reducer.wait_all_params()

    def reduced_grads(self, group) -> torch.Tensor:
        """fp32 copy of the DP-summed gradient of a flat group as the optimizer saw it (ZeRO-1:
        this rank's shards only, NaN elsewhere)."""
        r = self.reducer
        if r.mode == "reduce_scatter" and r.enabled:
            out = torch.full((group.numel,), float("nan"), device=group.grads.device)
            for lo, hi in r.shard_ranges(group, self.st.dp_rank):
                out[lo:hi] = r.grad_view(group, lo, hi).float()
            return out
        return r.grad_view(group, 0, group.numel).float().clone()
