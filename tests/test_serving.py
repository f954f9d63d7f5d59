"""InferenceService: engine (prefill/decode vs full forward), continuous batching,
predictor HTTP API, and the InferenceService controller (object level + CPU end to end)."""
import json
import os
import socket
import sys
import time
import urllib.request

import pytest
import torch

from service_account_auth_improvements_amd.controlplane import inferenceservice as isvcmod
from service_account_auth_improvements_amd.controlplane.apiserver import APIServer
from service_account_auth_improvements_amd.controlplane.client import InMemoryClient
from service_account_auth_improvements_amd.controlplane.kubelet import DeploymentController, Kubelet
from service_account_auth_improvements_amd.controlplane.runtime import Manager
from service_account_auth_improvements_amd.serving.engine import Request, Scheduler, build_engine
from service_account_auth_improvements_amd.serving.server import create_app

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def eng():
    return build_engine("tiny", device="cpu", n_slots=4, max_len=64)


def test_prefill_decode_match_full_forward(eng):
    prompt = [5, 17, 99, 3, 42, 7]
    cont = [11, 12, 13]
    full = eng.m.forward_logits(torch.tensor([prompt + cont]))[0].float()
    lg = eng.prefill(2, prompt).float()
    assert torch.allclose(lg, full[len(prompt) - 1], atol=1e-2)
    for j, t in enumerate(cont):
        out = eng.decode([t], [2], [len(prompt) + j])[0].float()
        assert torch.allclose(out, full[len(prompt) + j], atol=1e-2)


def test_prefill_batch_matches_per_prompt_prefill(eng):
    """Batched prefill of prompts of different lengths == one prefill per prompt: logits and
    every slot's KV cache (positions below each prompt's length)."""
    prompts = [[5, 17, 99, 3, 42, 7], [9, 8], [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]]
    slots = [0, 3, 1]
    one = [eng.prefill(s, p).float() for s, p in zip(slots, prompts)]
    kc1, vc1 = eng.kc.clone(), eng.vc.clone()
    eng.kc.zero_()
    eng.vc.zero_()
    lg = eng.prefill_batch(slots, prompts).float()
    assert lg.shape == (3, eng.cfg.vocab_size)
    for j, (s, p) in enumerate(zip(slots, prompts)):
        assert torch.allclose(lg[j], one[j], atol=1e-4), j
        n = len(p)
        assert torch.allclose(eng.kc[:, s, :, :n].float(), kc1[:, s, :, :n].float(), atol=1e-3)
        assert torch.allclose(eng.vc[:, s, :, :n].float(), vc1[:, s, :, :n].float(), atol=1e-3)


def test_scheduler_groups_prompts_by_length(eng, monkeypatch):
    """Admitted prompts are prefilled in length groups (padding <= 1.25x of a prompt's rows);
    the outputs equal one request at a time."""
    calls = []
    orig = eng.prefill_batch

    def spy(slots, prompts):
        calls.append(sorted(len(p) for p in prompts))
        return orig(slots, prompts)

    monkeypatch.setattr(eng, "prefill_batch", spy)
    monkeypatch.setattr("service_account_auth_improvements_amd.serving.engine.PREFILL_PAD_RATIO", 1.25)
    s = Scheduler(eng, max_batch=4)
    prompts = [[3] * 4, [5] * 40, [7] * 5, [9] * 38]
    reqs = [s.submit(Request(prompt=p, max_new_tokens=3)) for p in prompts]
    monkeypatch.setattr("service_account_auth_improvements_amd.serving.engine.PREFILL_MAX_TOKENS", 1 << 20)
    s.step()
    assert calls == [[4, 5], [38, 40]]
    s.run_until_idle()
    solo = []
    for p in prompts:
        one = Scheduler(eng, max_batch=1)
        r = one.submit(Request(prompt=p, max_new_tokens=3))
        one.run_until_idle()
        solo.append(r.output)
    assert [r.output for r in reqs] == solo


def test_continuous_batching_is_order_independent(eng):
    s = Scheduler(eng, max_batch=3)
    a = s.submit(Request(prompt=[1, 2, 3, 4], max_new_tokens=6))
    b = s.submit(Request(prompt=[9, 8], max_new_tokens=3))
    c = s.submit(Request(prompt=[1, 2, 3, 4], max_new_tokens=6))
    d = s.submit(Request(prompt=[7] * 10, max_new_tokens=4))    # waits for a free slot
    s.run_until_idle()
    assert a.output == c.output and len(a.output) == 6 and len(b.output) == 3 and len(d.output) == 4
    solo = Scheduler(eng, max_batch=1)
    e = solo.submit(Request(prompt=[1, 2, 3, 4], max_new_tokens=6))
    solo.run_until_idle()
    assert e.output == a.output
    bad = s.submit(Request(prompt=[1] * 60, max_new_tokens=10))
    assert bad.error and bad.done.is_set()


def test_predictor_http_api(eng):
    s = Scheduler(eng, max_batch=4).start()
    try:
        app = create_app(s, "llama").test_client()
        assert app.get("/v1/models/llama").json == {"name": "llama", "ready": True}
        assert app.get("/v1/models/other").status_code == 404
        r = app.post("/v1/models/llama:predict", json={"instances": [{"token_ids": [1, 2, 3], "max_new_tokens": 4},
                                                                     {"prompt": "hi", "max_new_tokens": 2}]})
        preds = r.json["predictions"]
        assert len(preds[0]["token_ids"]) == 4 and len(preds[1]["token_ids"]) == 2
        r = app.post("/v2/models/llama/infer", json={"inputs": [{"name": "input_ids", "datatype": "INT64",
                                                                  "shape": [3], "data": [1, 2, 3]}],
                                                      "parameters": {"max_new_tokens": 4}})
        assert r.json["outputs"][0]["data"] == preds[0]["token_ids"]
        r = app.post("/v1/completions", json={"prompt": "hello", "max_tokens": 3})
        assert r.json["usage"] == {"prompt_tokens": 5, "completion_tokens": 3}
        assert b"predictor_generated_tokens_total" in app.get("/metrics").data
    finally:
        s.stop()


def _isvc(name="llama", **model):
    m = {"modelFormat": {"name": "kfamd-llama"}, "resources": {"limits": {"amd.com/gpu": "1"}}}
    m.update(model)
    return {"apiVersion": "serving.kserve.io/v1beta1", "kind": "InferenceService",
            "metadata": {"name": name, "namespace": "team"}, "spec": {"predictor": {"model": m}}}


def test_isvc_controller_objects_and_status():
    srv = APIServer()
    c = InMemoryClient(srv)
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
    mgr = Manager(c).add(isvcmod.InferenceServiceReconciler(c))
    c.create(_isvc(storageUri="pvc://models/llama3-8b"))
    mgr.run_until_idle()
    dep = c.get("apps/v1", "Deployment", "llama-predictor", "team")
    ctr = dep["spec"]["template"]["spec"]["containers"][0]
    assert ctr["resources"]["limits"]["amd.com/gpu"] == "1"
    assert "--checkpoint" in ctr["args"] and "/mnt/pvc/llama3-8b" in ctr["args"]
    assert dep["spec"]["template"]["spec"]["volumes"][0]["persistentVolumeClaim"]["claimName"] == "models"
    assert c.get("v1", "Service", "llama-predictor", "team")["spec"]["ports"][0]["targetPort"] == 8080
    st = c.get("serving.kserve.io/v1beta1", "InferenceService", "llama", "team")["status"]
    assert {x["type"]: x["status"] for x in st["conditions"]}["Ready"] == "False"
    assert st["url"] == "http://llama-predictor.team.svc.cluster.local"
    dep["status"] = {"readyReplicas": 1}
    c.update_status(dep)
    mgr.run_until_idle()
    st = c.get("serving.kserve.io/v1beta1", "InferenceService", "llama", "team")["status"]
    assert {x["type"]: x["status"] for x in st["conditions"]}["Ready"] == "True"
    assert st["modelStatus"]["states"]["activeModelState"] == "Loaded"
    c.create(_isvc("bad", modelFormat={"name": "tensorflow"}))
    mgr.run_until_idle()
    st = c.get("serving.kserve.io/v1beta1", "InferenceService", "bad", "team")["status"]
    assert st["conditions"][1]["reason"] == "InvalidPredictorSpec"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_isvc_end_to_end_cpu(tmp_path):
    """InferenceService CR -> Deployment -> Pod -> predictor process -> HTTP predict."""
    srv = APIServer()
    c = InMemoryClient(srv)
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
    kub = Kubelet(c, n_gpus=0, exec_pods=True, workdir=ROOT, log_dir=str(tmp_path),
                  extra_env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1"})
    mgr = Manager(c).add(isvcmod.InferenceServiceReconciler(c)).add(DeploymentController(c)).add(kub)
    port = _free_port()
    isvc = _isvc(args=["--model", "tiny", "--slots", "2", "--max-len", "64", "--port", str(port),
                       "--host", "127.0.0.1"], resources={})
    c.create(isvc)
    mgr.start(workers=2)
    try:
        deadline = time.time() + 120
        out = None
        while time.time() < deadline:
            try:
                req = urllib.request.Request(f"http://127.0.0.1:{port}/v1/models/llama:predict",
                                             data=json.dumps({"instances": [{"token_ids": [1, 2, 3],
                                                                             "max_new_tokens": 3}]}).encode(),
                                             headers={"Content-Type": "application/json"})
                out = json.loads(urllib.request.urlopen(req, timeout=10).read())
                break
            except OSError:
                time.sleep(0.5)
        assert out is not None, kub.pod_log("team", c.list("v1", "Pod", "team")[0]["metadata"]["name"])
        assert len(out["predictions"][0]["token_ids"]) == 3
        deadline = time.time() + 20
        while time.time() < deadline:
            st = c.get("serving.kserve.io/v1beta1", "InferenceService", "llama", "team").get("status") or {}
            if {x["type"]: x["status"] for x in st.get("conditions", [])}.get("Ready") == "True":
                break
            time.sleep(0.2)
        assert {x["type"]: x["status"] for x in st["conditions"]}["Ready"] == "True"
    finally:
        mgr.stop()
        kub.shutdown()


def test_isvc_multi_gpu_predictor_runs_tensor_parallel():
    srv = APIServer()
    c = InMemoryClient(srv)
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
    mgr = Manager(c).add(isvcmod.InferenceServiceReconciler(c))
    c.create(_isvc(resources={"limits": {"amd.com/gpu": "4"}}))
    mgr.run_until_idle()
    ctr = c.get("apps/v1", "Deployment", "llama-predictor", "team")["spec"]["template"]["spec"]["containers"][0]
    cmd = ctr["command"]
    assert cmd[0].endswith("kfamd_launch") and cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert "--isolate-devices" in cmd and cmd[-2:] == ["--", "python"]
    assert ctr["args"][ctr["args"].index("--tp") + 1] == "4"


def _tp_predictor_body(rank, world):
    import torch.distributed as dist

    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.serving.engine import Request, Scheduler, build_engine
    from service_account_auth_improvements_amd.serving.tp import TPLeaderEngine, follower_loop

    st = init_distributed(tp=world, pp=1, device="cpu")
    ctrl = dist.new_group(backend="gloo")
    e = build_engine("tiny", device="cpu", n_slots=4, max_len=128, st=st, full_init=True)
    if rank != 0:
        return follower_loop(e, ctrl)
    lead = TPLeaderEngine(e, ctrl)
    logits = [lead.prefill(0, list(range(3, 40)))]
    for j, t in enumerate((5, 6)):
        logits.append(lead.decode([t], [0], [37 + j])[0])
    s = Scheduler(lead, max_batch=2)
    reqs = [s.submit(Request(prompt=list(range(k, k + 9)), max_new_tokens=4)) for k in (1, 20)]
    s.run_until_idle()
    lead.stop()
    return torch.stack([x.float() for x in logits]), [r.output for r in reqs]


def test_tp_predictor_leader_drives_followers():
    """Rank 0 (HTTP + scheduler) broadcasts every engine call; rank 1 replays it: the TP=2
    logits match a TP=1 engine and the scheduler completes requests through the leader."""
    from dist_util import run_ranks
    from service_account_auth_improvements_amd.serving.engine import build_engine

    res = run_ranks(_tp_predictor_body, world=2, timeout=300)
    logits, outs = res[0]
    # follower replayed: 1 prefill + 2 decodes, then the scheduler's ONE batched prefill of
    # both admitted prompts (first tokens) and 3 joint decode steps (tokens 2..4 of both)
    assert res[1] == 3 + 1 + 3
    ref = build_engine("tiny", device="cpu", n_slots=4, max_len=128, full_init=True)
    exp = [ref.prefill(0, list(range(3, 40)))]
    for j, t in enumerate((5, 6)):
        exp.append(ref.decode([t], [0], [37 + j])[0])
    assert (logits - torch.stack([x.float() for x in exp])).abs().max().item() < 5e-2
    assert all(len(o) == 4 for o in outs)


def test_split_partials_norm_reference_equals_reduce_then_norm():
    """CPU reference of ops.rmsnorm_fwd_parts (the decode engine's reduce-in-norm path): the
    partials summed in slice order and rounded to bf16, then the plain residual RMSNorm."""
    from service_account_auth_improvements_amd import ops
    from service_account_auth_improvements_amd.serving.engine import _SplitSum, _dense
    g = torch.Generator().manual_seed(3)
    a = torch.randn(5, 64, generator=g).bfloat16()
    part = torch.randn(4, 5, 64, generator=g)
    w = (1 + 0.1 * torch.randn(64, generator=g)).bfloat16()
    y, h, r = ops.rmsnorm_fwd_parts(a, part, w, 1e-5)
    d = _dense(_SplitSum(part))
    y2, h2, r2 = ops.rmsnorm_fwd(a, w, 1e-5, residual=d)
    assert torch.equal(h, h2) and torch.equal(y, y2) and torch.equal(r, r2)
    assert _dense(None) is None and _dense(d) is d


def test_rope_append_parts_reference_equals_reduce_then_rope_append():
    """CPU reference of rope_append_parts (the decode engine's qkv reduce-in-RoPE path)."""
    from service_account_auth_improvements_amd.ops import reference
    from service_account_auth_improvements_amd.ops.attention import rope_append_, rope_append_parts
    g = torch.Generator().manual_seed(4)
    Hq, Hkv, L = 4, 2, 16
    part = torch.randn(2, 3, (Hq + 2 * Hkv) * 128, generator=g)
    cos, sin = reference.rope_tables(L, 128)
    slots = torch.tensor([2, 0, 1], dtype=torch.int32)
    pos = torch.tensor([0, 5, 15], dtype=torch.int32)
    kc = torch.zeros(3, Hkv, L, 128, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    kc2, vc2 = kc.clone(), vc.clone()
    got = rope_append_parts(part, Hq, cos, sin, slots, pos, kc, vc)
    ref = (part[0] + part[1]).to(torch.bfloat16)
    rope_append_(ref, Hq, cos, sin, slots, pos, kc2, vc2)
    assert torch.equal(got, ref) and torch.equal(kc, kc2) and torch.equal(vc, vc2)
