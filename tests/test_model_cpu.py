"""The explicit forward/backward engine vs torch.autograd on a plain reference Llama (CPU)."""
import pytest
import torch

from service_account_auth_improvements_amd.models.llama import Llama, LlamaConfig
from service_account_auth_improvements_amd.models.llama_ref import reference_loss
from service_account_auth_improvements_amd.parallel.state import ParallelState


def _grads_match(m, W, tol=2.5e-2):
    for n, w in W.items():
        g, r = m.G(n).float(), w.grad
        rel = ((g - r).abs().max() / r.abs().max().clamp_min(1e-8)).item()
        assert rel < tol, (n, rel)


def test_engine_matches_autograd_reference():
    cfg = LlamaConfig.preset("tiny")
    m = Llama(cfg, ParallelState(), device="cpu", seed=3).allocate()
    B, S = 2, 32
    torch.manual_seed(0)
    tok = torch.randint(0, cfg.vocab_size, (B, S))
    lab = torch.randint(0, cfg.vocab_size, (B, S))
    loss = m.forward_backward(tok, lab)
    ref, W = reference_loss(m, tok, lab)
    ref.backward()
    ref_v = float(ref.detach())
    assert abs(float(loss) - ref_v) < 1e-2 * ref_v
    _grads_match(m, W)


def test_grad_accumulation_equals_big_batch():
    cfg = LlamaConfig.preset("tiny")
    m = Llama(cfg, ParallelState(), device="cpu", seed=5).allocate()
    torch.manual_seed(1)
    tok = torch.randint(0, cfg.vocab_size, (4, 16))
    lab = torch.randint(0, cfg.vocab_size, (4, 16))
    m.forward_backward(tok, lab, scale=1.0 / tok.numel())
    big = m.mats.grads.float().clone()
    m.forward_backward(tok[:2], lab[:2], accumulate=False, scale=1.0 / tok.numel())
    m.forward_backward(tok[2:], lab[2:], accumulate=True, scale=1.0 / tok.numel())
    acc = m.mats.grads.float()
    rel = ((acc - big).abs().max() / big.abs().max()).item()
    assert rel < 2e-2, rel


def test_param_count_llama3_8b():
    cfg = LlamaConfig.preset("llama3-8b")
    assert abs(cfg.num_params() - 8.03e9) / 8.03e9 < 0.01
    cfg70 = LlamaConfig.preset("llama3-70b")
    assert abs(cfg70.num_params() - 70.6e9) / 70.6e9 < 0.01


def test_activation_recompute_matches_saved_activations():
    """recompute=True (only layer inputs kept, layer forward re-run before its backward)
    gives bit-identical losses, gradients and updated parameters."""
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.runtime.trainer import TrainConfig, Trainer
    out = []
    for rc in (False, True):
        tr = Trainer(TrainConfig(model="tiny", seq_len=32, micro_batch=2, lr=1e-3, recompute=rc), ParallelState())
        assert tr.model.recompute == rc
        g = torch.Generator().manual_seed(3)
        mbs = [(torch.randint(0, tr.mcfg.vocab_size, (2, 32), generator=g),
                torch.randint(0, tr.mcfg.vocab_size, (2, 32), generator=g)) for _ in range(2)]
        losses = [float(tr.train_step(mbs)) for _ in range(2)]
        out.append((losses, tr.model.mats.params.clone(), tr.model.mats.grads.clone()))
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][2], out[1][2])


@pytest.mark.parametrize("tp_vocab", [False])
def test_chunked_lm_head_matches_unchunked(tp_vocab):
    """K5: the row-chunked LM head + CE (logits never materialised whole) gives the same loss
    and gradients as one chunk, including ignored labels inside a chunk."""
    cfg = LlamaConfig.preset("tiny")
    torch.manual_seed(2)
    tok = torch.randint(0, cfg.vocab_size, (2, 32))
    lab = torch.randint(0, cfg.vocab_size, (2, 32))
    lab[0, 5] = -100
    res = {}
    for chunk in (0, 16, 24):
        m = Llama(cfg, ParallelState(), device="cpu", seed=5).allocate()
        m.head_chunk = chunk
        loss = m.forward_backward(tok, lab)
        res[chunk] = (float(loss), m.mats.grads.float().clone(), m.norms.grads.float().clone())
    for chunk in (16, 24):
        assert abs(res[chunk][0] - res[0][0]) < 1e-5 * res[0][0]
        for a, b in zip(res[chunk][1:], res[0][1:]):
            assert ((a - b).abs().max() / b.abs().max()).item() < 1e-2


def test_loss_before_backward_is_not_a_silent_zero_and_forward_loss_matches():
    """K5 fuses the loss with the head's backward: the stage's loss tensor is NaN until
    stage_backward fills it, and forward_loss gives the same value with no backward."""
    import math
    from service_account_auth_improvements_amd.models.llama import Llama, LlamaConfig
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    cfg = LlamaConfig.preset("tiny")
    m = Llama(cfg, ParallelState(), device="cpu").allocate()
    m.head_chunk = 16                       # several chunks
    g = torch.Generator().manual_seed(3)
    tok = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
    lab = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
    loss, ctx = m.stage_forward(tok.reshape(-1), 2, 32, lab.reshape(-1), 1.0 / 64)
    assert math.isnan(float(loss))
    m.stage_backward(ctx, None, 2, 32, accumulate=False)
    trained = float(loss)
    assert math.isfinite(trained) and trained > 0
    assert abs(float(m.forward_loss(tok, lab)) - trained) < 1e-5 * trained
