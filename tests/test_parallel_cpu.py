"""Multi-process (gloo, world 2) correctness of DP (all-reduce and ZeRO-1) and TP."""
import pytest
import torch

from dist_util import run_ranks


def _tiny_batches(vocab, n, B=2, S=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randint(0, vocab, (B, S), generator=g), torch.randint(0, vocab, (B, S), generator=g))
            for _ in range(n)]


def _dp_body(rank, world, zero1, overlap=True):
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=1, pp=1, device="cpu")
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, zero1=zero1, bucket_mb=1, lr=1e-3,
                             overlap_allgather=overlap), st)
    batches = _tiny_batches(tr.mcfg.vocab_size, world)
    mine = [batches[rank]]
    # one step with the optimizer disabled (lr 0) exposes the reduced gradients
    lr = tr.opt.cfg.lr
    tr.opt.cfg.lr = 0.0
    tr.train_step(mine)
    grads = tr.reduced_grads(tr.model.mats) / world
    tr.opt.cfg.lr = lr
    losses = [float(tr.train_step(mine)) for _ in range(3)]
    tr.sync_params()
    return losses, tr.model.mats.params.float().clone(), tr.model.norms.params.float().clone(), grads


def _single_body(world):
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, bucket_mb=1, lr=1e-3), ParallelState())
    batches = _tiny_batches(tr.mcfg.vocab_size, world)
    # one big step = mean over both ranks' batches == accumulate 2 micro-batches
    tr.opt.cfg.lr = 0.0
    tr.train_step(batches)
    return tr.reduced_grads(tr.model.mats)


def _close(a, b, tol):
    return ((a - b).abs().max() / b.abs().max()).item() < tol


def test_ddp_allreduce_matches_single_process():
    res = run_ranks(_dp_body, world=2, args=(False,))
    p0, p1 = res[0][1], res[1][1]
    assert torch.equal(p0, p1), "replicas diverged"
    ref = _single_body(2)
    assert _close(res[0][3], ref, 2e-2)


def test_zero1_matches_allreduce():
    a = run_ranks(_dp_body, world=2, args=(False,))
    z = run_ranks(_dp_body, world=2, args=(True,))
    assert torch.equal(z[0][1], z[1][1]), "ZeRO-1 replicas diverged after all-gather"
    # reduce-scatter and all-reduce may sum in different orders: AdamW's sign-like first
    # steps can flip near-zero elements by <= 2*lr per step; everything else must agree
    diff = (z[0][1] - a[0][1]).abs()
    assert diff.max().item() <= 2 * 1e-3 * 3 + 1e-2
    assert (diff < 1e-3).float().mean().item() > 0.99
    assert _close(z[0][2], a[0][2], 2e-2)
    # the forward-overlapped parameter all-gather is bit-identical to the blocking one
    zb = run_ranks(_dp_body, world=2, args=(True, False))
    assert torch.equal(zb[0][1], z[0][1]) and zb[0][0] == z[0][0]


def _tp_body(rank, world, sp=False):
    from service_account_auth_improvements_amd.models.llama import Llama, LlamaConfig
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    st = init_distributed(tp=world, pp=1, device="cpu")
    cfg = LlamaConfig.preset("tiny")
    m = Llama(cfg, st, device="cpu", seed=9, full_init=True).allocate()
    m.sequence_parallel = sp
    assert m._sp == sp
    tok, lab = _tiny_batches(cfg.vocab_size, 1, seed=3)[0]
    loss = m.forward_backward(tok, lab)
    return float(loss), {s.name: m.G(s.name).float().clone() for g in m.groups for s in g.specs}


@pytest.mark.parametrize("sp", [False, True], ids=["tp", "tp+sp"])
def test_tensor_parallel_matches_tp1(sp):
    """TP=2 (and TP=2 with Megatron sequence parallelism: row-sharded norms / residual, all-gather
    before and reduce-scatter after the TP GEMMs, TP-summed norm gradients) == TP=1 gradients."""
    from service_account_auth_improvements_amd.models.llama import Llama, LlamaConfig
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    cfg = LlamaConfig.preset("tiny")
    ref = Llama(cfg, ParallelState(), device="cpu", seed=9, full_init=True).allocate()
    tok, lab = _tiny_batches(cfg.vocab_size, 1, seed=3)[0]
    ref_loss = float(ref.forward_backward(tok, lab))
    res = run_ranks(_tp_body, world=2, args=(sp,))
    for rank, (loss, grads) in enumerate(res):
        assert abs(loss - ref_loss) < 1e-2 * ref_loss, (loss, ref_loss)
        # shard the reference grads exactly like the TP model shards its weights
        shard = Llama(cfg, ParallelState(tp=2, tp_rank=rank), device="cpu", seed=9, full_init=True)
        sl = shard._tp_slicers()
        for name, g in grads.items():
            r = ref.G(name).float()
            if name in sl:
                r = sl[name][1](r)
            assert _close(g, r, 3e-2), (rank, name)


def _pp_body(rank, world, n_micro):
    from service_account_auth_improvements_amd.parallel.pipeline import PipelineTrainer
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig
    st = init_distributed(tp=1, pp=world, device="cpu")
    tr = PipelineTrainer(TrainConfig(model="tiny", seq_len=32, lr=0.0, micro_batch=2, n_layers=4), st)
    mbs = _tiny_batches(tr.mcfg.vocab_size, n_micro, seed=5)
    loss = tr.train_step(mbs)
    grads = {s.name: tr.model.G(s.name).float().clone() for g in tr.model.groups for s in g.specs}
    return (float(loss) if loss is not None else None), grads


def test_pipeline_1f1b_matches_single_stage():
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    n_micro = 3
    ref = Trainer(TrainConfig(model="tiny", seq_len=32, lr=0.0, micro_batch=2, n_layers=4), ParallelState())
    mbs = _tiny_batches(ref.mcfg.vocab_size, n_micro, seed=5)
    ref_loss = float(ref.train_step(mbs))
    res = run_ranks(_pp_body, world=2, args=(n_micro,))
    assert res[0][0] is None and abs(res[1][0] - ref_loss) < 5e-3 * ref_loss
    seen = set()
    for _, grads in res:
        for name, g in grads.items():
            assert _close(g, ref.model.G(name).float(), 2e-2), name
            seen.add(name)
    assert seen == {s.name for g in ref.model.groups for s in g.specs}


def _tp_train_body(rank, world, clip):
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=world, pp=1, device="cpu")
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, lr=1e-3, max_grad_norm=clip), st, full_init=True)
    batches = _tiny_batches(tr.mcfg.vocab_size, 2, seed=11)
    losses = [float(tr.train_step([b])) for b in batches]
    return losses, tr.model.norms.params.float().clone()


def test_tensor_parallel_training_with_clipping_matches_tp1():
    """TP=2 full steps (AdamW + global-norm clipping across TP shards) == TP=1."""
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    clip = 0.05            # small: clipping is active, so a wrong (per-rank) norm would diverge
    res = run_ranks(_tp_train_body, world=2, args=(clip,))
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, lr=1e-3, max_grad_norm=clip), ParallelState(), full_init=True)
    batches = _tiny_batches(tr.mcfg.vocab_size, 2, seed=11)
    ref = [float(tr.train_step([b])) for b in batches]
    for r in res:
        assert abs(r[0][1] - ref[1]) < 2e-2 * abs(ref[1]), (r[0], ref)
    # replicated norm weights: identical across TP ranks and close to TP=1
    assert torch.equal(res[0][1], res[1][1])
    assert _close(res[0][1], tr.model.norms.params.float(), 1e-2)


def test_traffic_proxy_sees_every_bucket_the_finish_and_the_gather():
    """GradReducer.traffic_proxy (tools/dp8_overlap_proxy.py): one step hands it every gradient
    bucket's bytes as the bucket is launched, one finish() before the optimizer, and every
    parameter bucket's bytes at the gather -- also at dp 1, where no collective runs."""
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import SyntheticData, TrainConfig, Trainer
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, zero1=True, bucket_mb=1),
                 ParallelState(device=torch.device("cpu")))
    seen = {"bucket": [], "finish": 0, "gather": []}

    class Rec:
        def on_bucket(self, n):
            seen["bucket"].append(n)

        def on_finish(self):
            seen["finish"] += 1

        def on_gather(self, n):
            seen["gather"].append(n)

    tr.reducer.traffic_proxy = Rec()
    data = SyntheticData(tr.mcfg.vocab_size, 2, 32, "cpu", seed=0)
    tr.train_step([data.next()])
    total = sum(g.numel * g.grads.element_size() for g in tr.model.groups)
    nb = sum(len(bl) for bl in tr.reducer.buckets.values())
    assert len(seen["bucket"]) == nb > 1 and sum(seen["bucket"]) == total
    assert seen["finish"] == 1
    assert sum(seen["gather"]) == total
