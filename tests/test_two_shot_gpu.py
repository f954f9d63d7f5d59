"""Two-shot reduce-scatter / all-gather / all-reduce (ops/csrc/custom_ar.hip namespace ts,
parallel/custom_ar.py TwoShot) with two ranks sharing the test box's one GPU (gloo carries only
the IPC-handle exchange; the data moves through the peer-mapped uncached buffers, as over xGMI
on an 8-GPU node).

Two ranks: RCCL's sum of two bf16 tensors is one bf16 rounding of their exact fp32 sum, so the
expected results below are exactly RCCL's (RCCL itself refuses two ranks on one GPU, so it
cannot be run side by side here)."""
import os

import pytest
import torch

from dist_util import run_ranks

pytestmark = pytest.mark.gpu


def _x(n, rank, it):
    g = torch.Generator(device="cpu").manual_seed(7919 * n + 31 * it + rank)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def _body(rank, world, sizes):
    import torch.distributed as dist

    from service_account_auth_improvements_amd.parallel.custom_ar import TwoShot

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    comm = TwoShot(max_bytes=64 << 20, blocks=64)
    bad = []
    for n in sizes:
        for it in range(2):
            xs = [_x(n, r, it) for r in range(world)]
            ref = (xs[0].float() + xs[1].float()).to(torch.bfloat16)
            x = xs[rank].to("cuda:0")
            # all-reduce, in place (blocking)
            y = x.clone()
            comm.all_reduce(y)
            if not torch.equal(y.cpu(), ref):
                bad.append(("ar", n, it))
            # reduce-scatter, async handle
            out = torch.empty(n // world, dtype=torch.bfloat16, device="cuda:0")
            w = comm.reduce_scatter(out, x, async_op=True)
            w.wait()
            if not torch.equal(out.cpu(), ref[rank * n // world:(rank + 1) * n // world]):
                bad.append(("rs", n, it))
            # all-gather of every rank's full x
            full = torch.empty(n * world, dtype=torch.bfloat16, device="cuda:0")
            comm.all_gather(full, x)
            if not torch.equal(full.cpu(), torch.cat(xs)):
                bad.append(("ag", n, it))
    torch.cuda.synchronize()
    calls = comm.calls
    comm.check()
    # outside the buffer / not bf16 -> torch.distributed (gloo here)
    big = torch.ones(8, dtype=torch.float32)
    comm.all_reduce(big)
    dist.barrier()
    comm.close()
    return bad, calls, float(big[0])


def test_two_shot_rs_ag_ar_bit_identical_two_ranks_one_gpu():
    sizes = [16, 4096 * 8, 1 << 20, 16 << 20]      # up to 32 MB in, 64 MB gathered
    res = run_ranks(_body, world=2, args=(sizes,), timeout=300)
    for bad, calls, fallback in res:
        assert bad == [], bad
        assert calls == 3 * 2 * len(sizes)
        assert fallback == 2.0


def _train_body(rank, world, kind, sp):
    os.environ["KFAMD_DIST_BACKEND"] = "gloo"
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=world, pp=1, device="cuda")
    tr = Trainer(TrainConfig(model="tiny", seq_len=128, micro_batch=2, n_layers=2, lr=1e-3, sequence_parallel=sp,
                             tp_comm_chunks=2, tp_comm=kind), st, full_init=True)
    assert type(st.tp_comm).__name__ == "TwoShot"
    g = torch.Generator().manual_seed(11)
    v = tr.mcfg.vocab_size
    losses = []
    for _ in range(2):
        b = [(torch.randint(0, v, (2, 128), generator=g).cuda(), torch.randint(0, v, (2, 128), generator=g).cuda())]
        losses.append(float(tr.train_step(b)))
    torch.cuda.synchronize()
    st.tp_comm.check()
    return losses, st.tp_comm.calls


@pytest.mark.parametrize("sp", [False, True], ids=["tp2", "tp2+sp"])
def test_two_shot_tp2_training_matches_one_rank(sp):
    """A TP=2 training step whose every activation collective (row-parallel reduce-scatter /
    all-reduce, SP all-gather, backward input-gradient reductions) runs on the two-shot kernel
    follows the single-rank step's losses."""
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    res = run_ranks(_train_body, world=2, args=("twoshot", sp), timeout=300)
    tr = Trainer(TrainConfig(model="tiny", seq_len=128, micro_batch=2, n_layers=2, lr=1e-3),
                 ParallelState(device=torch.device("cuda", 0)), full_init=True)
    g = torch.Generator().manual_seed(11)
    v = tr.mcfg.vocab_size
    ref = []
    for _ in range(2):
        b = [(torch.randint(0, v, (2, 128), generator=g).cuda(), torch.randint(0, v, (2, 128), generator=g).cuda())]
        ref.append(float(tr.train_step(b)))
    (l0, c0), (l1, c1) = res
    assert l0 == l1                       # both ranks computed the same bits
    assert c0 == c1 and c0 > 0
    for a, b in zip(l0, ref):
        assert abs(a - b) <= 2e-2 * abs(b), (l0, ref)
