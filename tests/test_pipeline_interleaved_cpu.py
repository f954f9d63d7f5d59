"""Interleaved 1F1B (virtual pipeline stages, parallel/pipeline.py ``interleaved_1f1b``) on gloo:
the simulated tick timeline, then pp2 x v2, pp4 x v2, dp2 x pp2 x v2 (ZeRO-1, fp32 micro-batch
accumulation) and tp2 x pp2 x v2 training against one process running the same global batch."""
import pytest
import torch

from dist_util import run_ranks

LR = 1e-3
STEPS = 2


def _batches(vocab, n, B=2, S=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randint(0, vocab, (B, S), generator=g), torch.randint(0, vocab, (B, S), generator=g))
            for _ in range(n)]


@pytest.mark.parametrize("pp,v,M", [(2, 2, 2), (2, 2, 4), (2, 3, 6), (4, 2, 4), (4, 2, 8), (8, 2, 8), (4, 4, 12)])
def test_interleaved_timeline_is_complete_and_causal(pp, v, M):
    from service_account_auth_improvements_amd.parallel.pipeline import interleaved_order, simulate_interleaved
    ticks = simulate_interleaved(pp, v, M)
    last = pp * v - 1
    when = {}
    for t, row in enumerate(ticks):
        for r, op in enumerate(row):
            if op is not None:
                when[(op[0], op[1], op[2] * pp + r)] = t
    # every rank runs each (micro-batch, chunk) forward and backward exactly once, in its list order
    for r in range(pp):
        order = interleaved_order(pp, v, M, r)
        assert sorted(order) == sorted([(k, m, c) for k in "FB" for m in range(M) for c in range(v)])
        ran = [op for row in ticks for op in [row[r]] if op is not None]
        assert ran == order
    # data dependencies: strictly earlier ticks
    for m in range(M):
        for vs in range(pp * v):
            if vs > 0:
                assert when[("F", m, vs - 1)] < when[("F", m, vs)]
            assert when[("F", m, vs)] < when[("B", m, vs)]
            if vs < last:
                assert when[("B", m, vs + 1)] < when[("B", m, vs)]
    # fewer chunk-op ticks than the non-interleaved schedule would take at the same pp and M
    assert len(ticks) < v * (2 * M + 2 * (pp - 1))


def test_interleaved_order_rejects_partial_groups():
    from service_account_auth_improvements_amd.parallel.pipeline import interleaved_order
    with pytest.raises(AssertionError):
        interleaved_order(4, 2, 6, 0)


def _body(rank, world, pp, v, n_micro, dp_steps, tp=1):
    from service_account_auth_improvements_amd.parallel.pipeline import PipelineTrainer
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig
    st = init_distributed(tp=tp, pp=pp, device="cpu")
    tcfg = TrainConfig(model="tiny", seq_len=32, micro_batch=2, grad_accum=n_micro, n_layers=pp * v, lr=LR,
                       zero1=st.dp > 1, bucket_mb=1, grad_reduce="fp32", pp_virtual=v)
    tr = PipelineTrainer(tcfg, st, full_init=True)
    losses = []
    for step in range(dp_steps):
        allb = _batches(tr.mcfg.vocab_size, st.dp * n_micro, seed=100 + step)
        mine = allb[st.dp_rank * n_micro:(st.dp_rank + 1) * n_micro]
        loss = tr.train_step(mine)
        losses.append(None if loss is None else float(loss))
    tr.sync_params()
    params = {s.name: tr.model.P(s.name).float().clone() for g in tr.model.groups for s in g.specs}
    names = sorted(g.name for g in tr.model.groups)
    return dict(losses=losses, params=params, coords=(st.dp_rank, st.pp_rank), dp=st.dp, groups=names,
                deferred=tr.p2p.sends_deferred, tp_rank=st.tp_rank, peak_live=tr.p2p.peak_live,
                max_inflight=tr.p2p.max_inflight, left=len(tr.p2p._groups) + len(tr.p2p._inflight))


def _reference(n_layers, n_batches_per_step):
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, grad_accum=n_batches_per_step,
                             n_layers=n_layers, lr=LR), ParallelState(), full_init=True)
    losses = [float(tr.train_step(_batches(tr.mcfg.vocab_size, n_batches_per_step, seed=100 + s)))
              for s in range(STEPS)]
    return tr, losses


@pytest.mark.parametrize("world,pp,v,n_micro,tp", [(2, 2, 2, 2, 1), (2, 2, 2, 4, 1), (4, 4, 2, 4, 1), (4, 2, 2, 2, 1),
                                                   (4, 2, 2, 2, 2), (2, 2, 2, 8, 1)],
                         ids=["pp2v2m2", "pp2v2m4", "pp4v2m4", "dp2xpp2v2-zero1", "tp2xpp2v2", "pp2v2m8"])
def test_interleaved_training_matches_single_process(world, pp, v, n_micro, tp):
    from service_account_auth_improvements_amd.models.llama import Llama
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    res = run_ranks(_body, world=world, args=(pp, v, n_micro, STEPS, tp), timeout=600)
    dp = world // (pp * tp)
    ref, ref_losses = _reference(pp * v, dp * n_micro)
    # each rank holds v chunks (groups renamed per chunk) and left send-only groups in flight
    for r in res:
        assert r["groups"] == sorted(f"{n}.v{c}" for n in ("matrices", "norms") for c in range(v))
        assert r["deferred"] > 0
        # boundary tensors kept alive by posted sends stay at the 1F1B bound (max(2, pp)) mid-step,
        # not 2 * M * v, and nothing is left over after the step's flush
        assert r["peak_live"] <= r["max_inflight"] == max(2, pp), (r["peak_live"], r["max_inflight"])
        assert r["left"] == 0
    for step in range(STEPS):
        per_replica = {r["coords"][0]: r["losses"][step] for r in res if r["coords"][1] == pp - 1}
        assert len(per_replica) == dp and all(x is not None for x in per_replica.values())
        got = sum(per_replica.values()) / dp
        assert abs(got - ref_losses[step]) < 1e-2 * ref_losses[step], (step, got, ref_losses[step])
    seen = set()
    for r in res:
        sl = Llama(ref.mcfg, ParallelState(tp=tp, tp_rank=r["tp_rank"]), device="cpu", seed=1234,
                   full_init=True)._tp_slicers() if tp > 1 else {}
        for name, got in r["params"].items():
            want = ref.model.P(name).float()
            if name in sl:
                want = sl[name][1](want)
            diff = (got - want).abs()
            assert diff.max().item() <= 2 * LR * STEPS + 1e-3, (r["coords"], name, diff.max().item())
            assert (diff <= 2e-4 + 1e-2 * want.abs()).float().mean().item() > 0.98, (r["coords"], name)
            seen.add(name)
    assert seen == {s.name for g in ref.model.groups for s in g.specs}
    by = {}
    for r in res:
        by.setdefault((r["coords"][1], r["tp_rank"]), []).append(r["params"])
    for reps in by.values():
        for other in reps[1:]:
            for name in reps[0]:
                assert torch.equal(reps[0][name], other[name]), name
