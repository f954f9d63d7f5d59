"""The PyTorchJob worker loop (runtime/train_entry.py), its /metrics endpoint
(runtime/metrics.py) and periodic checkpoint-restart (runtime/checkpoint.py):

* the loop issues ONE device synchronisation (the first step) and otherwise reads step N-1's
  loss only after step N has been queued -- the benched loop (bench.py);
* a 2-rank gloo job serves every Prometheus series on rank 0, scraped over HTTP;
* the streaming safetensors writer round-trips through the safe loader;
* ``--ckpt-dir/--save-every`` publishes ``latest`` atomically and a restart resumes from it,
  bit-identical to an uninterrupted run; a changed data-parallel size re-shards ZeRO-1 state.
"""
import json
import os
import types
import urllib.request

import pytest
import torch

from dist_util import run_ranks


# ------------------------------------------------------------------ no per-step device sync

class _FakeEvent:
    def __init__(self, log, step):
        self.log, self.step = log, step

    def synchronize(self):
        self.log.append(("event_sync", self.step))

    def elapsed_time(self, other):
        return 250.0


def test_worker_loop_syncs_the_device_once_and_reads_losses_one_step_late(monkeypatch):
    from service_account_auth_improvements_amd.runtime import train_entry as te
    log = []
    made = []

    def end_event():
        ev = _FakeEvent(log, len(made))
        made.append(ev)
        return ev

    monkeypatch.setattr(te, "_device_sync", lambda: log.append(("device_sync", None)))
    monkeypatch.setattr(te, "_end_event", end_event)
    monkeypatch.setattr(te, "_host_scalar", lambda loss: loss.detach().clone())
    monkeypatch.delenv("KFAMD_METRICS_PORT", raising=False)
    monkeypatch.delenv("KFAMD_EVENTS_FILE", raising=False)

    class Tr:
        step_idx = 0

        def train_step(self, batch):
            log.append(("train_step", self.step_idx))
            self.step_idx += 1
            return torch.tensor(float(self.step_idx))

    class Data:
        def next(self):
            return None, None

    st = types.SimpleNamespace(device=types.SimpleNamespace(type="cuda"), rank=0, dp=1)
    a = types.SimpleNamespace(steps=6, grad_accum=1, ckpt_dir=None, save_every=0, save=None, keep_checkpoints=2)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    assert te._loop(a, Tr(), Data(), st, 0.0, 1024) == 0
    assert [e for e in log if e[0] == "device_sync"] == [("device_sync", None)]
    assert log.index(("device_sync", None)) == 1            # right after the first step, once
    for k in range(5):
        # step k's end is waited for only after step k+1 was handed to the device
        assert log.index(("event_sync", k)) > log.index(("train_step", k + 1)), log
    assert ("event_sync", 5) in log                          # the last step is read at the end


# ------------------------------------------------------------------ /metrics over HTTP

def _metrics_body(rank, world, tmp):
    from service_account_auth_improvements_amd.runtime import metrics as mm
    from service_account_auth_improvements_amd.runtime import train_entry
    os.environ["KFAMD_METRICS_PORT"] = "0"
    os.environ["KFAMD_METRICS_ADDR"] = "127.0.0.1"
    scraped = {}
    real_close = mm.TrainMetrics.close

    def close(self):          # scrape the live endpoint before the worker shuts it down
        with urllib.request.urlopen(f"http://127.0.0.1:{self.port}/metrics", timeout=10) as r:
            scraped["text"] = r.read().decode()
        real_close(self)

    mm.TrainMetrics.close = close
    argv = ["--model", "tiny", "--device", "cpu", "--seq-len", "32", "--micro-batch", "2", "--zero1",
            "--steps", "4"]
    assert train_entry.main(argv) == 0
    if rank == 0:
        with open(os.path.join(tmp, "metrics.txt"), "w") as f:
            f.write(scraped["text"])
    return "text" in scraped


def test_metrics_endpoint_serves_every_series_from_a_two_rank_job(tmp_path):
    served = run_ranks(_metrics_body, world=2, args=(str(tmp_path),))
    assert served == [True, False]                       # rank 0 serves, rank 1 does not
    text = (tmp_path / "metrics.txt").read_text()
    vals = {}
    for line in text.splitlines():
        if line and not line.startswith("#"):
            k, v = line.rsplit(" ", 1)
            vals[k] = float(v)

    def labels(k):
        body = k.partition("{")[2].rstrip("}")
        return dict(kv.split("=", 1) for kv in body.split(",")) if body else {}

    def val(name, **lab):
        want = {a: f'"{b}"' for a, b in lab.items()}
        hits = [v for k, v in vals.items() if k.split("{")[0] == name and labels(k) == want]
        assert hits, (name, lab, text)
        return hits[0]

    assert val("train_steps_total", rank="0") == 4
    assert val("train_tokens_total", rank="0") == 4 * 2 * 32
    assert val("train_step_seconds", rank="0") > 0
    assert val("train_tokens_per_second", rank="0") > 0
    assert val("train_loss", rank="0") > 0
    # ZeRO-1 with the fp32 reduction: bucket all-to-alls + parameter all-gathers
    for op in ("all_to_all", "all_gather"):
        assert val("train_collective_calls_total", rank="0", op=op) >= 4
        assert val("train_collective_bytes_total", rank="0", op=op) > 0
        assert val("train_collective_seconds_total", rank="0", op=op) > 0
        assert val("train_collective_bus_bandwidth_bytes_per_second", rank="0", op=op) > 0
    for name in ("hip_memory_allocated_bytes", "hip_memory_reserved_bytes", "hip_memory_peak_allocated_bytes",
                 "train_checkpoint_last_step", "train_checkpoint_save_seconds"):
        assert f"# TYPE {name} gauge" in text                # HBM series: values on a GPU job only


# ------------------------------------------------------------------ safetensors streaming writer

def test_streaming_safetensors_writer_round_trips_through_the_safe_loader(tmp_path):
    from safetensors.torch import load_file

    from service_account_auth_improvements_amd.runtime.checkpoint import write_safetensors
    g = torch.Generator().manual_seed(0)
    t = {"a/bf16": torch.randn(7, 13, generator=g).to(torch.bfloat16),
         "b/f32": torch.randn(1000, generator=g),
         "c/u8": torch.randint(0, 255, (37,), dtype=torch.uint8, generator=g),
         "d/i64": torch.arange(5),
         "e/empty": torch.zeros(0)}
    p = str(tmp_path / "x.safetensors")
    write_safetensors(p, t, metadata={"step": 3})
    back = load_file(p)
    assert back.keys() == t.keys()
    for k in t:
        assert back[k].dtype == t[k].dtype and torch.equal(back[k], t[k]), k
    assert not os.path.exists(p + ".tmp")


def test_streaming_writer_takes_a_tensor_as_page_locked_pieces(tmp_path):
    """A snapshot held as byte pieces (checkpoint.HostPieces: the GPU path's page-locked buffers)
    is written as the one tensor it came from."""
    from safetensors.torch import load_file

    from service_account_auth_improvements_amd.runtime.checkpoint import HostPieces, write_safetensors
    x = torch.randn(1000, 3).to(torch.bfloat16)
    raw = x.reshape(-1).view(torch.uint8)
    pieces = [raw[a:a + 777].clone() for a in range(0, raw.numel(), 777)]
    p = str(tmp_path / "p.safetensors")
    write_safetensors(p, {"x": HostPieces(x.shape, x.dtype, pieces), "y": torch.arange(3)})
    back = load_file(p)
    assert torch.equal(back["x"], x) and torch.equal(back["y"], torch.arange(3))


# ------------------------------------------------------------------ periodic checkpoint-restart

def _events(path):
    with open(path) as f:
        return [json.loads(x) for x in f]


def _run_entry(tmp, tag, argv):
    from service_account_auth_improvements_amd.runtime import train_entry
    ev = os.path.join(tmp, f"{tag}.events")
    os.environ["KFAMD_EVENTS_FILE"] = ev
    try:
        assert train_entry.main(argv) == 0
    finally:
        os.environ.pop("KFAMD_EVENTS_FILE", None)
    return _events(ev)


def test_periodic_checkpoints_publish_latest_and_a_restart_resumes_from_it(tmp_path):
    from service_account_auth_improvements_amd.runtime.checkpoint import latest_checkpoint
    base = ["--model", "tiny", "--device", "cpu", "--seq-len", "32", "--micro-batch", "2"]
    full = _run_entry(tmp_path, "full", base + ["--steps", "9"])
    ck = str(tmp_path / "ck")
    # first incarnation: total 9 steps, but it "dies" after 7 (only --steps 7 given)
    p1 = _run_entry(tmp_path, "p1", base + ["--steps", "7", "--ckpt-dir", ck, "--save-every", "3"])
    assert [e["step"] for e in p1 if e["event"] == "checkpoint_published"] == [3, 6]
    assert latest_checkpoint(ck).endswith("step-00000006")
    assert sorted(d for d in os.listdir(ck) if d.startswith("step-")) == ["step-00000003", "step-00000006"]
    # the restart: same command with the job's total; resumes from 'latest' (step 6)
    p2 = _run_entry(tmp_path, "p2", base + ["--steps", "9", "--ckpt-dir", ck, "--save-every", "3"])
    res = [e for e in p2 if e["event"] == "resumed"]
    assert res and res[0]["step"] == 6 and res[0]["auto"] is True
    steps = lambda ev: [(e["step"], e["loss"]) for e in ev if e["event"] == "step"]   # noqa: E731
    assert [s for s, _ in steps(p2)] == [6, 7, 8]
    assert steps(p2) == steps(full)[6:]


def test_a_killed_world_never_publishes_a_partial_checkpoint(tmp_path):
    """A save whose ranks did not all finish (a done marker missing, or one left by an earlier,
    killed world with another token) is never named by 'latest'."""
    from service_account_auth_improvements_amd.runtime import checkpoint as ckm
    root = tmp_path / "ck"
    root.mkdir()
    (root / "step-00000004").mkdir()
    (root / "step-00000004" / "meta.json").write_text("{}")
    (root / ckm.LATEST).write_text("step-00000002\n")
    pc = ckm.PeriodicCheckpointer.__new__(ckm.PeriodicCheckpointer)
    pc.root, pc.world, pc.token, pc.publish_timeout = str(root), 2, "new", 0.2
    (root / "step-00000004" / "rank0.done").write_text(json.dumps({"token": "new"}))
    (root / "step-00000004" / "rank1.done").write_text(json.dumps({"token": "old-world"}))
    with pytest.raises(TimeoutError):
        pc._publish(str(root / "step-00000004"), 4, 0.0)
    assert (root / ckm.LATEST).read_text().strip() == "step-00000002"


def _reshard_body(rank, world, tmp, phase):
    from service_account_auth_improvements_amd.runtime import train_entry
    argv = ["--model", "tiny", "--device", "cpu", "--seq-len", "32", "--micro-batch", "2", "--zero1"]
    if phase == "save":
        argv += ["--steps", "2", "--save", os.path.join(tmp, f"A{world}")]
    else:
        argv += ["--steps", "0", "--resume", os.path.join(tmp, "A2"), "--save", os.path.join(tmp, f"R{world}")]
    return train_entry.main(argv)


def _full_opt_state(path):
    """Every optimizer range of a checkpoint, re-assembled per (group, buffer) into full flat
    vectors -- independent of how many dp ranks wrote it."""
    from safetensors.torch import load_file

    from service_account_auth_improvements_amd.runtime.checkpoint import _OPT_KEY
    parts = {}
    for fn in os.listdir(path):
        if fn.startswith("tp") and fn.endswith(".safetensors"):
            for k, v in load_file(os.path.join(path, fn)).items():
                m = _OPT_KEY.match(k)
                if m:
                    parts.setdefault((m.group(1), m.group(4)), []).append((int(m.group(2)), v))
    out = {}
    for key, segs in parts.items():
        segs.sort(key=lambda x: x[0])
        out[key] = torch.cat([v for _, v in segs])
    return out


def test_periodic_saves_spread_the_optimizer_over_part_files_and_ignore_stale_ones(tmp_path, monkeypatch):
    """With small parts (KFAMD_CKPT_PART_MIN) a rank's optimizer state is cut into several part
    files written concurrently; the done marker lists them, and a part file of a killed earlier
    world left in the same step directory is never read on resume."""
    from service_account_auth_improvements_amd.runtime import checkpoint as ckm
    monkeypatch.setenv("KFAMD_CKPT_PART_MIN", "4096")
    base = ["--model", "tiny", "--device", "cpu", "--seq-len", "32", "--micro-batch", "2"]
    full = _run_entry(tmp_path, "full", base + ["--steps", "6"])
    ck = str(tmp_path / "ck")
    _run_entry(tmp_path, "p1", base + ["--steps", "4", "--ckpt-dir", ck, "--save-every", "3"])
    d = ckm.latest_checkpoint(ck)
    parts = sorted(f for f in os.listdir(d) if f.startswith("tp0-pp0-dp0"))
    assert len(parts) == ckm._writers() and "tp0-pp0-dp0.safetensors" in parts, parts
    with open(os.path.join(d, "rank0.done")) as f:
        assert sorted(json.load(f)["files"]) == parts
    # the main file keeps the parameters whole; every optimizer range is in exactly one part
    fi = ckm._FileIndex(os.path.join(d, "tp0-pp0-dp0.safetensors"))
    assert all(k.startswith("param/") for k in fi.keys())
    fi.close()
    srcs = ckm._opt_sources(d, type("St", (), {"tp_rank": 0, "pp_rank": 0})())
    assert len({s[0] for s in srcs}) == len(parts) - 1
    # a stale part of another world: the same ranges, garbage values
    stale = {}
    for f, g, lo, hi, pre in srcs:
        for suf in ("master", "m", "v"):
            stale[f"{pre}/{suf}"] = torch.full((hi - lo,), 1e9)
    ckm.write_safetensors(os.path.join(d, "tp0-pp0-dp0.part99.safetensors"), stale)
    p2 = _run_entry(tmp_path, "p2", base + ["--steps", "6", "--ckpt-dir", ck, "--save-every", "3"])
    steps = lambda ev: [(e["step"], e["loss"]) for e in ev if e["event"] == "step"]   # noqa: E731
    assert steps(p2) == steps(full)[3:]


def test_opt_parts_cut_the_ranges_into_equal_runs():
    from service_account_auth_improvements_amd.runtime.checkpoint import _opt_parts

    class Sh:
        def __init__(self, lo, hi):
            self.lo, self.hi = lo, hi
    shards = [Sh(0, 10), Sh(100, 100), Sh(40, 71)]
    out = _opt_parts(shards, 4, 1)
    assert [(a, b, j) for _, a, b, j in out] == [(0, 10, 1), (100, 100, 1), (40, 41, 1), (41, 52, 2), (52, 63, 3),
                                                 (63, 71, 4)]
    assert [(a, b, j) for _, a, b, j in _opt_parts(shards, 1, 0)] == [(0, 10, 0), (100, 100, 0), (40, 71, 0)]


@pytest.mark.parametrize("part_min", [None, "2048"])
def test_zero1_state_is_resharded_when_the_data_parallel_size_changes(tmp_path, monkeypatch, part_min):
    if part_min:
        monkeypatch.setenv("KFAMD_CKPT_PART_MIN", part_min)
    assert run_ranks(_reshard_body, world=2, args=(str(tmp_path), "save")) == [0, 0]
    for w in (1, 3):
        assert run_ranks(_reshard_body, world=w, args=(str(tmp_path), "load")) == [0] * w
        a, b = _full_opt_state(tmp_path / "A2"), _full_opt_state(tmp_path / f"R{w}")
        assert a.keys() == b.keys() and a
        for k in a:
            n = min(a[k].numel(), b[k].numel())          # the padded tails differ with dp
            assert torch.equal(a[k][:n], b[k][:n]), (w, k)
            assert not a[k][n:].any() and not b[k][n:].any()
        with open(tmp_path / f"R{w}" / "meta.json") as f:
            meta = json.load(f)
        assert meta["step"] == 2 and meta["parallel"]["dp"] == w


def test_hip_preinit_is_skipped_for_cpu_jobs_and_when_disabled(monkeypatch):
    """train_entry._hip_preinit: never for --device cpu or KFAMD_HIP_PREINIT=0 (and never where
    there is no GPU device node); otherwise one daemon thread that loads torch's own HIP runtime."""
    from service_account_auth_improvements_amd.runtime import train_entry as te
    assert te._hip_preinit("cpu") is None
    monkeypatch.setenv("KFAMD_HIP_PREINIT", "0")
    assert te._hip_preinit("auto") is None
    monkeypatch.setenv("KFAMD_HIP_PREINIT", "1")
    t = te._hip_preinit("auto")
    if not os.path.exists("/dev/kfd"):
        assert t is None
    else:
        assert t.daemon and t.name == "kfamd-hip-preinit"
        t.join(timeout=30)
