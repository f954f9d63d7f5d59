"""Context parallelism (parallel/context.py) over gloo: the head/token all-to-alls are exact
inverses, and cp=2 / cp=4 training (the DP group as one context-parallel group: same sequences,
1/cp of the tokens per rank, attention on all tokens for 1/cp of the heads) matches one process
training the whole sequences."""
import pytest
import torch

from dist_util import run_ranks

LR = 1e-3
STEPS = 2


def _batches(vocab, n, B=2, S=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randint(0, vocab, (B, S), generator=g), torch.randint(0, vocab, (B, S), generator=g))
            for _ in range(n)]


def _a2a_body(rank, world):
    import torch.distributed as dist

    from service_account_auth_improvements_amd.parallel import context as cpx
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    init_distributed(device="cpu")
    B, S, widths = 2, 8 * world, [4 * world, 2 * world, 2 * world]
    g = torch.Generator().manual_seed(0)
    full = torch.randn(B, S, sum(widths), generator=g)            # every rank builds the same tensor
    mine = cpx.shard_tokens(full, world, rank).reshape(B * S // world, -1)
    h = cpx.to_heads(mine, B, S // world, widths, world, None)
    # expected: all tokens, this rank's slice of every block
    cols, off = [], 0
    for w in widths:
        cols.append(full[..., off + rank * w // world:off + (rank + 1) * w // world])
        off += w
    want = torch.cat(cols, -1).reshape(B * S, -1)
    back = cpx.to_tokens(h, B, S // world, [w // world for w in widths], world, None)
    dist.barrier()
    return bool(torch.equal(h, want)), bool(torch.equal(back, mine))


@pytest.mark.parametrize("world", [2, 4])
def test_all_to_all_layouts(world):
    for heads_ok, back_ok in run_ranks(_a2a_body, world=world):
        assert heads_ok and back_ok


def _mcfg(kv):
    from service_account_auth_improvements_amd.models.llama import LlamaConfig
    return LlamaConfig.preset("tiny").with_(n_heads=2 * kv, n_kv_heads=kv)


def _cp_body(rank, world, zero1, n_layers, kv, tp=1):
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=tp, device="cpu")
    tr = Trainer(TrainConfig(model="tiny", seq_len=64, micro_batch=2, n_layers=n_layers, lr=LR, max_grad_norm=0.05,
                             zero1=zero1, bucket_mb=1, context_parallel=True), st, mcfg=_mcfg(kv), full_init=True)
    assert tr.cp == world // tp and tr.model.cp == world // tp
    losses = []
    for step in range(STEPS):
        losses.append(float(tr.train_step(_batches(tr.mcfg.vocab_size, 1, seed=50 + step))))
    tr.sync_params()
    return losses, {s.name: tr.model.P(s.name).float().clone() for g in tr.model.groups for s in g.specs}, st.tp_rank


@pytest.mark.parametrize("world,zero1,kv,tp", [(2, False, 2, 1), (2, True, 2, 1), (4, True, 4, 1), (4, True, 4, 2)],
                         ids=["cp2", "cp2-zero1", "cp4-zero1", "cp2xtp2-zero1"])
def test_context_parallel_training_matches_single_process(world, zero1, kv, tp):
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    n_layers = 2
    from service_account_auth_improvements_amd.models.llama import Llama
    res = run_ranks(_cp_body, world=world, args=(zero1, n_layers, kv, tp), timeout=600)
    ref = Trainer(TrainConfig(model="tiny", seq_len=64, micro_batch=2, n_layers=n_layers, lr=LR, max_grad_norm=0.05),
                  ParallelState(), mcfg=_mcfg(kv), full_init=True)
    ref_losses = [float(ref.train_step(_batches(ref.mcfg.vocab_size, 1, seed=50 + step))) for step in range(STEPS)]
    cp = world // tp
    for step in range(STEPS):
        got = sum(r[0][step] for r in res) / world        # equal token blocks: mean of means (TP ranks agree)
        assert abs(got - ref_losses[step]) < 1e-2 * ref_losses[step], (step, got, ref_losses[step])
    slicers = {}
    for t in range(tp):
        slicers[t] = Llama(ref.mcfg, ParallelState(tp=tp, tp_rank=t), device="cpu", seed=1234,
                           full_init=True)._tp_slicers() if tp > 1 else {}
    for name, full in ((s.name, ref.model.P(s.name).float()) for g in ref.model.groups for s in g.specs):
        for losses, params, t in res:
            want = slicers[t][name][1](full) if name in slicers[t] else full
            diff = (params[name] - want).abs()
            assert diff.max().item() <= 2 * LR * STEPS + 1e-3, (name, diff.max().item())
            assert (diff <= 2e-4 + 1e-2 * want.abs()).float().mean().item() > 0.98, name
    # replicas of the weights stay identical across the context-parallel group
    for name in res[0][1]:
        for other in res[1:]:
            if other[2] == res[0][2]:
                assert torch.equal(res[0][1][name], other[1][name]), name
    assert cp * tp == world
