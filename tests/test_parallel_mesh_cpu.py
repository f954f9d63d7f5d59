"""4-rank (gloo) training on 2-D process meshes -- dp2 x tp2, dp2 x pp2 (ZeRO-1 per stage), tp2 x pp2 -- against one
process running the same global batch, plus the fp32 DP gradient reduction and fp32 micro-batch
accumulation against exact (float64) sums.

Covers the rank -> (pp, dp, tp) mapping of ``parallel/state.py:init_distributed`` with two
dimensions > 1 at once, ZeRO-1 under TP, and DP x PP gradient reduction."""
import pytest
import torch

from dist_util import run_ranks

LR = 1e-3
STEPS = 2


def _batches(vocab, n, B=2, S=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randint(0, vocab, (B, S), generator=g), torch.randint(0, vocab, (B, S), generator=g))
            for _ in range(n)]


def _mesh_body(rank, world, tp, pp, n_micro, grad_reduce, sp=False):
    from service_account_auth_improvements_amd.parallel.pipeline import PipelineTrainer
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=tp, pp=pp, device="cpu")
    tcfg = TrainConfig(model="tiny", seq_len=32, micro_batch=2, grad_accum=n_micro, n_layers=4, lr=LR,
                       zero1=st.dp > 1, bucket_mb=1, grad_reduce=grad_reduce, sequence_parallel=sp)
    tr = PipelineTrainer(tcfg, st, full_init=True) if pp > 1 else Trainer(tcfg, st, full_init=True)
    losses = []
    for step in range(STEPS):
        allb = _batches(tr.mcfg.vocab_size, st.dp * n_micro, seed=100 + step)
        mine = allb[st.dp_rank * n_micro:(st.dp_rank + 1) * n_micro]
        loss = tr.train_step(mine)
        losses.append(None if loss is None else float(loss))
    if hasattr(tr, "sync_params"):
        tr.sync_params()
    params = {s.name: tr.model.P(s.name).float().clone() for g in tr.model.groups for s in g.specs}
    deferred = tr.p2p.sends_deferred if pp > 1 else 0
    zero1 = tr.reducer.mode == "reduce_scatter"
    return dict(losses=losses, params=params, coords=(st.dp_rank, st.tp_rank, st.pp_rank), dp=st.dp,
                deferred=deferred, zero1=zero1)


def _reference(n_batches_per_step, n_layers=4):
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, grad_accum=n_batches_per_step,
                             n_layers=n_layers, lr=LR), ParallelState(), full_init=True)
    losses = []
    for step in range(STEPS):
        losses.append(float(tr.train_step(_batches(tr.mcfg.vocab_size, n_batches_per_step, seed=100 + step))))
    return tr, losses


@pytest.mark.parametrize("tp,pp,sp", [(2, 1, False), (1, 2, False), (2, 2, False), (2, 1, True), (2, 2, True)],
                         ids=["dp2xtp2", "dp2xpp2", "tp2xpp2", "dp2xtp2+sp", "tp2xpp2+sp"])
def test_2d_mesh_training_matches_single_process(tp, pp, sp):
    from service_account_auth_improvements_amd.models.llama import Llama
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    world = 4
    dp = world // (tp * pp)
    n_micro = 2
    res = run_ranks(_mesh_body, world=world, args=(tp, pp, n_micro, "fp32", sp), timeout=600)
    ref, ref_losses = _reference(dp * n_micro)
    # PP: send-only P2P groups are left in flight behind compute; dp > 1: ZeRO-1 on every stage
    if pp > 1:
        assert all(r["deferred"] > 0 for r in res), [r["deferred"] for r in res]
    assert all(r["zero1"] == (dp > 1) for r in res)
    # every (dp, tp, pp) coordinate appears exactly once
    assert sorted(r["coords"] for r in res) == sorted((d, t, p) for d in range(dp) for t in range(tp)
                                                     for p in range(pp))
    # loss: the last stage's local mean, averaged over DP replicas == the global-batch loss
    for step in range(STEPS):
        last = [r["losses"][step] for r in res if r["coords"][2] == pp - 1]
        per_replica = {}
        for r in res:
            if r["coords"][2] == pp - 1:
                per_replica[r["coords"][0]] = r["losses"][step]
        got = sum(per_replica.values()) / dp
        assert all(v is not None for v in last)
        assert abs(got - ref_losses[step]) < 1e-2 * ref_losses[step], (step, got, ref_losses[step])
    # parameters after STEPS AdamW steps: shard the reference like each rank's model
    cfg = ref.mcfg
    seen = set()
    for r in res:
        d, t, p = r["coords"]
        sl = Llama(cfg.with_(n_layers=4), ParallelState(tp=tp, tp_rank=t), device="cpu", seed=1234,
                   full_init=True)._tp_slicers() if tp > 1 else {}
        for name, got in r["params"].items():
            want = ref.model.P(name).float()
            if name in sl:
                want = sl[name][1](want)
            diff = (got - want).abs()
            # AdamW's first steps are sign-like: an element whose gradient is ~0 may move by
            # up to lr per step either way under a different summation order
            assert diff.max().item() <= 2 * LR * STEPS + 1e-3, (r["coords"], name, diff.max().item())
            assert (diff <= 2e-4 + 1e-2 * want.abs()).float().mean().item() > 0.98, (r["coords"], name)
            seen.add(name)
    assert seen == {s.name for g in ref.model.groups for s in g.specs}
    # DP replicas of the same (tp, pp) coordinate hold identical parameters
    by = {}
    for r in res:
        by.setdefault(r["coords"][1:], []).append(r["params"])
    for reps in by.values():
        for other in reps[1:]:
            for name in reps[0]:
                assert torch.equal(reps[0][name], other[name]), name


# ------------------------------------------------------------------ fp32 gradient reduction
def _dp_grad_body(rank, world, grad_reduce, zero1):
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=1, pp=1, device="cpu")
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, lr=0.0, zero1=zero1, bucket_mb=1,
                             grad_reduce=grad_reduce), st, full_init=True)
    b = _batches(tr.mcfg.vocab_size, world, seed=7)[rank]
    tr.train_step([b])
    return tr.reduced_grads(tr.model.mats)


def _per_batch_grads(n, seed=7):
    """Each batch's own bf16 gradient (one process, grad_accum 1), as float64."""
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, lr=0.0), ParallelState(), full_init=True)
    out = []
    for b in _batches(tr.mcfg.vocab_size, n, seed=seed):
        tr.train_step([b])
        out.append(tr.model.mats.grads.double().clone())
    return out


def _rel(a, b):
    own = ~torch.isnan(a)
    return ((a[own].double() - b[own]).abs().max() / b.abs().max()).item()


@pytest.mark.parametrize("zero1", [True, False], ids=["zero1", "allreduce"])
def test_fp32_dp_reduction_is_exact_sum_of_rank_gradients(zero1):
    """4 ranks: the fp32 reduction equals the float64 sum of the ranks' bf16 gradients to fp32
    rounding; the bf16 RCCL-style reduction is measurably worse.  Both are within 1e-2 of the
    single-process full-batch gradient."""
    world = 4
    exact = sum(_per_batch_grads(world))
    f32 = run_ranks(_dp_grad_body, world=world, args=("fp32", zero1))
    b16 = run_ranks(_dp_grad_body, world=world, args=("bf16", zero1))
    err32 = max(_rel(g, exact) for g in f32)
    err16 = max(_rel(g, exact) for g in b16)
    if zero1:   # fp32 ZeRO-1 shards feed AdamW unrounded
        assert err32 < 1e-6, err32
    else:       # fp32 all-reduce of the fp32-staged buckets
        assert err32 < 1e-6, err32
    assert err32 < err16, (err32, err16)
    assert err16 < 1e-2
    if zero1:   # the four shards tile the buffer
        assert bool(torch.stack([~torch.isnan(g) for g in f32]).any(0).all())


def test_fp32_microbatch_accumulation():
    """grad_accum=4 in one process: fp32 main-gradient accumulation == float64 sum of the four
    micro-batch gradients; bf16 beta=1 accumulation rounds three times."""
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    n = 4
    exact = sum(_per_batch_grads(n)) / n
    errs = {}
    for mode in ("fp32", "bf16"):
        tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, grad_accum=n, lr=0.0, grad_reduce=mode),
                     ParallelState(), full_init=True)
        tr.train_step(_batches(tr.mcfg.vocab_size, n, seed=7))
        g = tr.reduced_grads(tr.model.mats)
        errs[mode] = _rel(g, exact)
        # a second step must not inherit the first step's accumulator
        tr.train_step(_batches(tr.mcfg.vocab_size, n, seed=7))
        assert _rel(tr.reduced_grads(tr.model.mats), exact) <= errs[mode] * 1.0001 + 1e-12
    assert errs["fp32"] < 1e-6, errs
    assert errs["fp32"] < errs["bf16"], errs


# ------------------------------------------------------------------ TP forward overlap
def _chunk_body(rank, world, chunks, sp):
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=world, pp=1, device="cpu")
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, n_layers=2, lr=LR, sequence_parallel=sp,
                             tp_comm_chunks=chunks, tp_dual_batch=False), st, full_init=True)
    assert tr.model.tp_comm_chunks == chunks
    losses = [float(tr.train_step(_batches(tr.mcfg.vocab_size, 1, seed=500 + s))) for s in range(STEPS)]
    return dict(losses=losses, params={s.name: tr.model.P(s.name).float() for g in tr.model.groups
                                       for s in g.specs})


@pytest.mark.parametrize("sp", [False, True], ids=["tp2", "tp2+sp"])
def test_tp_chunked_forward_overlap_is_bit_identical(sp):
    """Row-parallel GEMMs in 4 token chunks with each chunk's all-reduce / reduce-scatter in
    flight behind the next chunk's GEMM (and, under SP, chunked all-gathers feeding the
    column-parallel GEMMs) give bit-identical losses and parameters to one GEMM + one blocking
    collective (two ranks: the reduction order of a sum of two is fixed)."""
    one = run_ranks(_chunk_body, world=2, args=(1, sp))
    four = run_ranks(_chunk_body, world=2, args=(4, sp))
    for a, b in zip(one, four):
        assert a["losses"] == b["losses"]
        for name in a["params"]:
            assert torch.equal(a["params"][name], b["params"][name]), name


def _dual_body(rank, world, dual):
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=world, pp=1, device="cpu")
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=4, n_layers=2, lr=LR, tp_dual_batch=dual), st,
                 full_init=True)
    assert tr.dual == dual
    losses = [float(tr.train_step(_batches(tr.mcfg.vocab_size, 1, B=4, seed=700 + s))) for s in range(STEPS)]
    return dict(losses=losses, params={s.name: tr.model.P(s.name).float() for g in tr.model.groups
                                       for s in g.specs})


def test_tp_dual_batch_forward_matches_plain_forward():
    """The dual half-batch forward (two halves' layers interleaved at every TP collective, their
    saved activations concatenated for ONE full-batch backward) computes the same step as the
    plain forward: same losses, parameters equal to fp32 GEMM-blocking noise."""
    dual = run_ranks(_dual_body, world=2, args=(True,))
    plain = run_ranks(_dual_body, world=2, args=(False,))
    for a, b in zip(dual, plain):
        for x, y in zip(a["losses"], b["losses"]):
            assert abs(x - y) <= 1e-5 * abs(y), (a["losses"], b["losses"])
        for name in a["params"]:
            assert torch.allclose(a["params"][name], b["params"][name], rtol=0, atol=1e-6), name


class _RecordingComm:
    """Stands in for parallel.custom_ar.TwoShot on CPU: counts what the model routes to it and
    delegates to torch.distributed (gloo)."""

    def __init__(self, group):
        self.group, self.calls = group, {"ar": 0, "rs": 0, "ag": 0}

    def all_reduce(self, x, async_op=False):
        import torch.distributed as dist
        self.calls["ar"] += 1
        return dist.all_reduce(x, group=self.group, async_op=async_op)

    def reduce_scatter(self, out, x, async_op=False):
        import torch.distributed as dist
        self.calls["rs"] += 1
        return dist.reduce_scatter_tensor(out, x, group=self.group, async_op=async_op)

    def all_gather(self, out, x, async_op=False):
        import torch.distributed as dist
        self.calls["ag"] += 1
        return dist.all_gather_into_tensor(out, x, group=self.group, async_op=async_op)

    def check(self):
        self.calls["check"] = self.calls.get("check", 0) + 1


def _comm_body(rank, world, sp, install):
    from service_account_auth_improvements_amd.parallel.custom_ar import make_tp_comm
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    st = init_distributed(tp=world, pp=1, device="cpu")
    # a CPU (gloo) job asking for the two-shot communicator keeps torch.distributed
    tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, n_layers=2, lr=LR, sequence_parallel=sp,
                             tp_comm_chunks=4, tp_comm="twoshot"), st, full_init=True)
    assert st.tp_comm is None and make_tp_comm("rccl", st) is None
    rec = _RecordingComm(st.tp_group) if install else None
    st.tp_comm = rec
    losses = [float(tr.train_step(_batches(tr.mcfg.vocab_size, 1, seed=900 + s))) for s in range(STEPS)]
    return dict(losses=losses, calls=rec.calls if rec else None,
                params={s.name: tr.model.P(s.name).float() for g in tr.model.groups for s in g.specs})


@pytest.mark.parametrize("sp", [False, True], ids=["tp2", "tp2+sp"])
def test_tp_collectives_route_through_the_tp_communicator(sp):
    """Every activation collective of the TP forward and backward (chunked row-parallel
    reductions, SP all-gathers, async input-gradient reductions) goes to ``st.tp_comm`` when one
    is installed (the two-shot kernel on GPU), with results identical to plain torch.distributed."""
    plain = run_ranks(_comm_body, world=2, args=(sp, False))
    routed = run_ranks(_comm_body, world=2, args=(sp, True))
    for a, b in zip(plain, routed):
        assert a["losses"] == b["losses"]
        for name in a["params"]:
            assert torch.equal(a["params"][name], b["params"][name]), name
        c = b["calls"]
        assert c["check"] == STEPS          # the trainer checks the communicator after every step
        if sp:
            assert c["rs"] > 0 and c["ag"] > 0
        else:
            assert c["ar"] > 0 and c["rs"] == 0 and c["ag"] == 0


def test_make_tp_comm_rejects_unknown_backends():
    from service_account_auth_improvements_amd.parallel.custom_ar import make_tp_comm
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    with pytest.raises(ValueError):
        make_tp_comm("nvls", ParallelState(tp=2))
    assert make_tp_comm("twoshot", ParallelState(tp=1)) is None


def test_two_shot_block_count():
    """TwoShot's workgroup count: the measured 128 for one rank per GPU, an explicit request
    as given (capped to MAX_BLOCKS), and for ranks sharing one GPU half the CUs split among them
    (profiles/two_shot_blocks_r5.md; the shared-GPU TP tests rely on it)."""
    from service_account_auth_improvements_amd.parallel.custom_ar import TwoShot, two_shot_blocks
    assert two_shot_blocks(None, 1, 256) == TwoShot.DEFAULT_BLOCKS == 128
    assert two_shot_blocks(None, 4, 256) == 32 and two_shot_blocks(None, 8, 256) == 16
    assert two_shot_blocks(None, 2, 256) == 64
    assert two_shot_blocks(64, 4, 256) == 64 and two_shot_blocks(1000, 1, 256) == TwoShot.MAX_BLOCKS
    assert two_shot_blocks(None, 1024, 256) == 1


def test_two_shot_block_count_is_uniform_over_uneven_gpu_sharing():
    """every rank must launch the same block count.  8 ranks on 3 GPUs (3/3/2) and
    mixed CU counts give ONE value on every rank, from the gathered keys only."""
    from service_account_auth_improvements_amd.parallel.custom_ar import uniform_two_shot_blocks
    keys = ["g0", "g0", "g0", "g1", "g1", "g1", "g2", "g2"]
    cus = [256] * 8
    per_rank = {uniform_two_shot_blocks(None, keys, cus) for _ in range(8)}
    assert per_rank == {256 // (2 * 3)}
    assert uniform_two_shot_blocks(None, ["a", "b"], [256, 240]) == 128      # one rank per GPU
    assert uniform_two_shot_blocks(None, ["a", "a", "b", "b"], [256, 256, 240, 240]) == 240 // 4
    assert uniform_two_shot_blocks(32, keys, cus) == 32
