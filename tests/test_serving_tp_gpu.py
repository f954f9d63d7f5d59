"""TP=2 InferenceService decode with both ranks sharing the test GPU (KFAMD_DIST_BACKEND=gloo
carries the prefill / embedding / logit collectives; the decode step's all-reduces run one-shot
over the peer-mapped IPC buffers of parallel/custom_ar.py): the logits match a TP=1 engine
built from the same full-size initialisation."""
import os

import pytest
import torch

from dist_util import run_ranks

pytestmark = pytest.mark.gpu
PROMPT = list(range(5, 45))
CONT = [7, 8, 9]


def _run(e):
    out = [e.prefill(0, PROMPT).float().cpu()]
    for j, t in enumerate(CONT):
        out.append(e.decode([t], [0], [len(PROMPT) + j])[0].float().cpu())
    return torch.stack(out)


def _cfg():
    from service_account_auth_improvements_amd.models.llama import LlamaConfig
    return LlamaConfig.preset("small").with_(n_layers=2)


def _tp_body(rank, world):
    os.environ["KFAMD_DIST_BACKEND"] = "gloo"
    from service_account_auth_improvements_amd.models.llama import Llama
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.serving.engine import Engine

    st = init_distributed(tp=world, pp=1, device="cuda")
    m = Llama(_cfg(), st, device="cuda:0", seed=3, full_init=True).allocate(grads=False)
    e = Engine(m, n_slots=2, max_len=256, use_graphs=False)
    assert e.car is not None
    out = _run(e)
    err = e.car.error()
    e.car.close()
    return out, err


def test_tp2_decode_one_shot_allreduce_matches_tp1():
    from service_account_auth_improvements_amd.models.llama import Llama
    from service_account_auth_improvements_amd.parallel.state import ParallelState
    from service_account_auth_improvements_amd.serving.engine import Engine

    dev = torch.device("cuda:0")
    ref_m = Llama(_cfg(), ParallelState(device=dev), device=dev, seed=3, full_init=True).allocate(grads=False)
    ref = _run(Engine(ref_m, n_slots=2, max_len=256, use_graphs=False))
    for out, err in run_ranks(_tp_body, world=2, timeout=240):
        assert err == 0
        assert (out - ref).abs().max().item() < 0.15
