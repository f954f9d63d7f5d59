"""Checkpoint save -> resume is faithful (runtime/checkpoint.py, runtime/train_entry.py): k steps,
save, resume in a fresh trainer, k more steps == 2k uninterrupted steps, bit for bit (weights,
fp32 master, AdamW moments, losses), because the step, the RNG state and the data-stream
position are restored.  Covers the flat-buffer Llama trainer (single process and 2-rank ZeRO-1
over gloo) and the MNIST plumbing job."""
import json
import os

import pytest
import torch

from dist_util import run_ranks


def _run(tmp, tag, argv, env_extra=None):
    from service_account_auth_improvements_amd.runtime import train_entry
    ev = os.path.join(tmp, f"{tag}.events")
    os.environ["KFAMD_EVENTS_FILE"] = ev
    try:
        assert train_entry.main(argv) == 0
    finally:
        os.environ.pop("KFAMD_EVENTS_FILE", None)
    with open(ev) as f:
        recs = [json.loads(l) for l in f]
    return [(r["step"], r["loss"]) for r in recs if r["event"] == "step"]


def _tensors(path):
    from safetensors.torch import load_file
    out = {}
    for fn in sorted(os.listdir(path)):
        if fn.endswith(".safetensors") and not fn.endswith(".state.safetensors"):
            for k, v in load_file(os.path.join(path, fn)).items():
                out[f"{fn}:{k}"] = v
    return out


@pytest.mark.parametrize("model,extra", [("tiny", ["--seq-len", "32", "--micro-batch", "2", "--grad-accum", "2"]),
                                         ("mnist", ["--micro-batch", "8"])])
def test_resume_is_bit_identical_to_uninterrupted(tmp_path, model, extra):
    base = ["--model", model, "--device", "cpu", *extra]
    full = _run(tmp_path, "full", base + ["--steps", "4", "--save", str(tmp_path / "A")])
    first = _run(tmp_path, "p1", base + ["--steps", "2", "--save", str(tmp_path / "B1")])
    second = _run(tmp_path, "p2", base + ["--steps", "2", "--resume", str(tmp_path / "B1"),
                                          "--save", str(tmp_path / "B2")])
    assert [s for s, _ in second] == [2, 3]
    assert first + second == full
    a, b = _tensors(tmp_path / "A"), _tensors(tmp_path / "B2")
    assert a.keys() == b.keys() and a
    for k in a:
        assert torch.equal(a[k], b[k]), k
    with open(tmp_path / "B2" / "meta.json") as f:
        assert json.load(f)["step"] == 4


def _zero1_body(rank, world, tmp, phase):
    from service_account_auth_improvements_amd.runtime import train_entry
    argv = ["--model", "tiny", "--device", "cpu", "--seq-len", "32", "--micro-batch", "2", "--zero1"]
    if phase == "full":
        argv += ["--steps", "4", "--save", os.path.join(tmp, "A")]
    elif phase == "p1":
        argv += ["--steps", "2", "--save", os.path.join(tmp, "B1")]
    else:
        argv += ["--steps", "2", "--resume", os.path.join(tmp, "B1"), "--save", os.path.join(tmp, "B2")]
    return train_entry.main(argv)


def test_zero1_two_ranks_resume_is_bit_identical(tmp_path):
    for phase in ("full", "p1", "p2"):
        assert run_ranks(_zero1_body, world=2, args=(str(tmp_path), phase)) == [0, 0]
    a, b = _tensors(tmp_path / "A"), _tensors(tmp_path / "B2")
    assert any("dp1" in k for k in a), "ZeRO-1: every dp rank writes its optimizer shard"
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k


def _pp_body(rank, world, tmp, phase, v=1):
    from service_account_auth_improvements_amd.runtime import train_entry
    ev = os.path.join(tmp, f"{phase}.r{rank}.events")
    os.environ["KFAMD_EVENTS_FILE"] = ev
    argv = ["--model", "tiny", "--device", "cpu", "--seq-len", "32", "--micro-batch", "2", "--grad-accum", "2",
            "--pp", "2"] + (["--pp-virtual", str(v), "--layers", str(2 * v)] if v > 1 else [])
    if phase == "full":
        argv += ["--steps", "4", "--save", os.path.join(tmp, "A")]
    elif phase == "p1":
        argv += ["--steps", "2", "--save", os.path.join(tmp, "B1")]
    else:
        argv += ["--steps", "2", "--resume", os.path.join(tmp, "B1"), "--save", os.path.join(tmp, "B2")]
    assert train_entry.main(argv) == 0
    with open(ev) as f:
        return [(r["step"], r["loss"]) for r in map(json.loads, f) if r["event"] == "step"]


@pytest.mark.parametrize("v", [1, 2], ids=["1f1b", "interleaved-v2"])
def test_pipeline_two_stages_resume_is_bit_identical(tmp_path, v):
    """pp=2 (1F1B, and interleaved with 2 chunks per rank; gloo): the resumed run numbers its
    steps after the checkpoint and ends bit-identical to the uninterrupted one; the
    last stage's losses continue exactly."""
    full = run_ranks(_pp_body, world=2, args=(str(tmp_path), "full", v))
    p1 = run_ranks(_pp_body, world=2, args=(str(tmp_path), "p1", v))
    p2 = run_ranks(_pp_body, world=2, args=(str(tmp_path), "p2", v))
    for r in range(2):
        assert [s for s, _ in p2[r]] == [2, 3]
        assert p1[r] + p2[r] == full[r]
    assert all(l is not None for _, l in full[1])          # rank 1 is the last stage
    a, b = _tensors(tmp_path / "A"), _tensors(tmp_path / "B2")
    assert a.keys() == b.keys() and a
    for k in a:
        assert torch.equal(a[k], b[k]), k
