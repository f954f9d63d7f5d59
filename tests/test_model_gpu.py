"""End-to-end numerics of the HIP training path on cuda:0 vs torch.autograd fp32 reference."""
import pytest
import torch

from service_account_auth_improvements_amd.models.llama import Llama, LlamaConfig
from service_account_auth_improvements_amd.models.llama_ref import reference_loss
from service_account_auth_improvements_amd.ops import _ext
from service_account_auth_improvements_amd.parallel.state import ParallelState
from service_account_auth_improvements_amd.runtime.trainer import SyntheticData, TrainConfig, Trainer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset,B,S", [("tiny", 2, 128), ("small", 1, 512)])
def test_engine_gpu_matches_reference(preset, B, S):
    assert _ext.load()
    cfg = LlamaConfig.preset(preset)
    m = Llama(cfg, ParallelState(device=torch.device("cuda:0")), device="cuda:0", seed=3).allocate()
    torch.manual_seed(0)
    tok = torch.randint(0, cfg.vocab_size, (B, S), device="cuda:0")
    lab = torch.randint(0, cfg.vocab_size, (B, S), device="cuda:0")
    loss = m.forward_backward(tok, lab)
    ref, W = reference_loss(m, tok, lab)
    ref.backward()
    ref_v = float(ref.detach())
    assert abs(float(loss) - ref_v) < 1e-2 * ref_v
    for n, w in W.items():
        g, r = m.G(n).float(), w.grad
        rel = ((g - r).abs().max() / r.abs().max().clamp_min(1e-8)).item()
        assert rel < 5e-2, (n, rel)


def test_trainer_loss_decreases_gpu():
    st = ParallelState(device=torch.device("cuda:0"))
    tr = Trainer(TrainConfig(model="small", seq_len=256, lr=1e-3), st)
    data = SyntheticData(tr.mcfg.vocab_size, 2, 256, "cuda:0", seed=0)
    batch = [data.next()]
    losses = [float(tr.train_step(batch)) for _ in range(8)]
    assert losses[-1] < losses[0] - 0.5, losses


def test_async_optimizer_is_bit_identical():
    """AdamW on the side stream (segment events waited by the next forward) == in-order AdamW."""
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import SyntheticData, TrainConfig, Trainer
    st = ParallelState(device=torch.device("cuda", 0))
    out = []
    for asyn in (True, False):
        tr = Trainer(TrainConfig(model="small", seq_len=256, micro_batch=2, n_layers=2, async_optimizer=asyn), st)
        assert (tr._opt_stream is not None) == asyn, "async_optimizer flag not honoured"
        data = SyntheticData(tr.mcfg.vocab_size, 2, 256, st.device, seed=3)
        losses = [float(tr.train_step([data.next()])) for _ in range(4)]
        tr.sync_params()
        out.append((losses, tr.model.mats.params.clone(), tr.model.norms.params.clone()))
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][2], out[1][2])


def test_training_is_bitwise_reproducible_run_to_run_at_long_sequence():
    """Two runs of the same training job (Llama-3-8B widths, 2 layers, S 4096: several query
    chunks per dK/dV key block) produce bit-identical losses and parameters -- what bitwise
    checkpoint-restart rests on (the attention backward's deterministic slots are the default;
    profiles/restart_gpu_r6.md)."""
    out = []
    for _ in range(2):
        st = ParallelState(device=torch.device("cuda", 0))
        tr = Trainer(TrainConfig(model="llama3-8b", seq_len=4096, micro_batch=1, n_layers=2, lr=1e-4), st)
        data = SyntheticData(tr.mcfg.vocab_size, 1, 4096, "cuda:0", seed=9)
        losses = [float(tr.train_step([data.next()])) for _ in range(3)]
        tr.sync_params()
        out.append((losses, tr.model.mats.params.clone(), tr.model.norms.params.clone()))
        del tr
        torch.cuda.empty_cache()
    assert out[0][0] == out[1][0], (out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][2], out[1][2])


def test_activation_recompute_bit_identical_gpu():
    """Per-layer recomputation on the GPU kernels: same loss, gradients and parameters."""
    out = []
    for rc in (False, True):
        st = ParallelState(device=torch.device("cuda", 0))
        tr = Trainer(TrainConfig(model="small", seq_len=256, micro_batch=2, n_layers=2, recompute=rc), st)
        data = SyntheticData(tr.mcfg.vocab_size, 2, 256, "cuda:0", seed=4)
        losses = [float(tr.train_step([data.next()])) for _ in range(2)]
        out.append((losses, tr.model.mats.params.clone(), tr.model.mats.grads.clone()))
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][2], out[1][2])


def test_grad_accumulation_at_llama3_8b_widths():
    """Micro-batch accumulation on the bench's kernels (Llama-3-8B widths, vocab 128256, 2 layers):
    both the fp32 main-gradient path and the bf16 beta=1 path must equal the float64 sum of the
    per-micro-batch gradients, parameter by parameter; fp32 to fp32 rounding."""
    S = 2048
    st = ParallelState(device=torch.device("cuda:0"))
    g = torch.Generator().manual_seed(21)
    mbs = [(torch.randint(0, 128256, (1, S), generator=g).cuda(), torch.randint(0, 128256, (1, S), generator=g).cuda())
           for _ in range(2)]
    tr = Trainer(TrainConfig(model="llama3-8b", seq_len=S, micro_batch=1, grad_accum=1, n_layers=2, lr=0.0), st)
    exact = {}
    for mb in mbs:
        tr.train_step([mb])
        for grp in tr.model.groups:
            gr = grp.grads.double() / 2
            exact[grp.name] = gr if grp.name not in exact else exact[grp.name] + gr
    specs = [(grp.name, s) for grp in tr.model.groups for s in grp.specs]
    del tr
    torch.cuda.empty_cache()
    worst = {}
    for mode in ("fp32", "bf16"):
        tr = Trainer(TrainConfig(model="llama3-8b", seq_len=S, micro_batch=1, grad_accum=2, n_layers=2, lr=0.0,
                                 grad_reduce=mode), st)
        tr.train_step(mbs)
        got = {grp.name: tr.reduced_grads(grp).double() for grp in tr.model.groups}
        errs = {}
        for gname, s in specs:
            a = got[gname][s.offset:s.offset + s.numel]
            b = exact[gname][s.offset:s.offset + s.numel]
            errs[s.name] = ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
        worst[mode] = max(errs.items(), key=lambda kv: kv[1])
        assert worst[mode][1] < (1e-5 if mode == "fp32" else 1.6e-2), (mode, sorted(errs.items(), key=lambda kv: -kv[1])[:5])
        del tr
        torch.cuda.empty_cache()
    print("worst per-parameter relative error:", worst)


def test_fp32_and_bf16_accumulation_train_alike_at_llama3_8b_widths():
    """Same data, AdamW + clipping, 6 steps: the two accumulation precisions track each other."""
    S = 2048
    st = ParallelState(device=torch.device("cuda:0"))
    curves = {}
    for mode in ("fp32", "bf16"):
        tr = Trainer(TrainConfig(model="llama3-8b", seq_len=S, micro_batch=1, grad_accum=2, n_layers=2,
                                 grad_reduce=mode), st)
        data = SyntheticData(tr.mcfg.vocab_size, 1, S, "cuda:0", seed=1)
        batches = [[data.next() for _ in range(2)] for _ in range(2)]
        curves[mode] = [float(tr.train_step(batches[i % 2])) for i in range(6)]
        del tr
        torch.cuda.empty_cache()
    print("loss curves:", curves)
    for a, b in zip(curves["fp32"], curves["bf16"]):
        assert abs(a - b) < 0.05 * a, curves


def test_chunked_lm_head_at_llama3_8b_vocab_matches_fp32_reference():
    """K5 at the bench's head shape (hidden 4096, vocab 128256): the row-chunked LM head + fused
    CE (4 chunks here) against an fp32 autograd reference of the same 1-layer model."""
    cfg = LlamaConfig.preset("llama3-8b").with_(n_layers=1, max_seq=4096)
    m = Llama(cfg, ParallelState(device=torch.device("cuda:0")), device="cuda:0", seed=7).allocate()
    m.head_chunk = 1024
    torch.manual_seed(0)
    tok = torch.randint(0, cfg.vocab_size, (1, 4096), device="cuda:0")
    lab = torch.randint(0, cfg.vocab_size, (1, 4096), device="cuda:0")
    lab[0, 100:110] = -100
    loss = m.forward_backward(tok, lab, scale=1.0 / 4086)
    ref, W = reference_loss(m, tok, lab)
    ref.backward()
    ref_v = float(ref.detach())
    assert abs(float(loss) - ref_v) < 2e-3 * ref_v, (float(loss), ref_v)
    for n in ("lm_head", "final_norm", "l0.wd", "l0.wqkv", "embed"):
        g, r = m.G(n).float(), W[n].grad
        rel = ((g - r).abs().max() / r.abs().max().clamp_min(1e-8)).item()
        assert rel < 5e-2, (n, rel)
