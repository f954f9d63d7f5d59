"""bench.py driver contract on the CPU (tiny model): one JSON line from rank 0 with the
required keys, 1 process and 2 processes under torch.distributed.run (gloo, 127.0.0.1)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
ARGS = ["--model", "tiny", "--seq-len", "64", "--micro-batch", "1", "--steps", "2", "--warmup", "1", "--crd-jobs", "0"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(rec, n):
    assert KEYS <= set(rec), KEYS - set(rec)
    assert rec["n_gpus"] == n and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["ms_per_step"] > 0 and rec["higher_is_better"] is True
    assert rec["scaling"] == "weak" and rec["dtype"] == "bf16"
    assert rec["config"]["global_batch"] == n and rec["config"]["parallelism"] == f"dp{n}"
    assert rec["metric"].startswith("tokens/sec PyTorchJob Llama-3-8B DDP")


def test_bench_single_process_json():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS], capture_output=True, text=True,
                       timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1
    _check(recs[0], 1)
    # one optimizer plan along the 1 -> N curve (ZeRO-1; one shard at N = 1)
    assert recs[0]["config"]["optimizer_sharding"] == "zero1" and recs[0]["config"]["optimizer_shards"] == 1


def test_bench_reports_crd_to_first_step():
    """The metric's second half: PyTorchJobs through the process-level control plane before the
    throughput run; p50 / p90 and the breakdown land in the same JSON line."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    args = [x for x in ARGS if x not in ("--crd-jobs", "0")] + ["--crd-jobs", "2"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=600, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    (rec,) = _json_lines(r.stdout)
    _check(rec, 1)
    crd = rec["crd_to_first_step"]
    assert "error" not in crd, crd
    assert crd["jobs"] == 2 and crd["control_plane"] == "processes over HTTP" and crd["model"] == "tiny"
    assert 0 < rec["crd_to_first_step_p50_s"] <= rec["crd_to_first_step_p90_s"] < 120
    b = crd["breakdown_p50_s"]
    assert b["cr_to_running"] < b["import"] + b["init_to_first_step"] + 5
    assert abs(sum(b[k] for k in ("cr_to_running", "running_to_process", "import", "dist_init", "model_init",
                                   "init_to_first_step")) - crd["p50_s"]) < 1.0
    # the same box's control: bare `import torch`, CPUs, load
    ctl = crd["box_control"]
    assert ctl["import_torch_s"] > 0 and len(ctl["import_torch_runs_s"]) == 3
    assert ctl["cpu_count"] >= 1 and ctl["cpus_usable"] >= 1 and ctl["loadavg_1m"] >= 0
    assert rec["crd_to_first_step_p50_minus_import_control_s"] == round(crd["p50_s"] - ctl["import_torch_s"], 3)


def test_bench_two_ranks_torchrun_json():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", *ARGS]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout          # rank 0 only
    _check(recs[0], 2)
    assert recs[0]["config"]["optimizer_sharding"] == "zero1" and recs[0]["config"]["optimizer_shards"] == 2


def test_bench_self_launches_ranks_without_torchrun():
    """``bench.py --gpus 2`` with no WORLD_SIZE starts its own 2 ranks (child torch.distributed.run)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *ARGS],
                       capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    _check(recs[0], 2)
    assert recs[0]["backend"] == "gloo" and recs[0]["world_size_seen"] == 2


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *ARGS],
                       capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode != 0
    recs = _json_lines(r.stdout)      # one diagnostic line, never a throughput number
    assert len(recs) == 1 and recs[0]["value"] is None and "WORLD_SIZE=1" in recs[0]["error"]


def test_bench_rehearsal_flag_marks_the_record():
    """``--force-collectives`` runs the ZeRO-1 / fp32-reduction path on a one-rank group and says so."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-collectives", *ARGS],
                       capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1
    _check(recs[0], 1)
    assert recs[0]["rehearsal"] and recs[0]["config"]["optimizer_sharding"] == "zero1"
    assert recs[0]["backend"] == "gloo"


def test_auto_micro_batch_memory_plan():
    """Micro-batch 4 at dp1 and for ZeRO-1 at every N; 3 when a full fp32 gradient buffer is added."""
    sys.path.insert(0, ROOT)
    import bench
    for dp in (1, 2, 4, 8):
        assert bench._auto_micro_batch(dp, dp > 1, "fp32", dp > 1) == 4
        assert bench._auto_micro_batch(dp, dp > 1, "bf16", dp > 1) == 4
    for dp in (2, 4, 8):
        assert bench._auto_micro_batch(dp, False, "fp32", True) == 3      # fp32 all-reduce staging
    assert bench._auto_micro_batch(1, True, "fp32", True) == 3            # one-rank rehearsal
    assert bench._auto_micro_batch(1, False, "fp32", False, grad_accum=4) == 3


def test_crd_device_release_wait_watches_only_our_cards(tmp_path):
    """The between-jobs wait reads amdgpu's sysfs VRAM counters and only waits for cards whose
    usage the job raised (other tenants' cards never delay the loop)."""
    import threading
    import time
    from service_account_auth_improvements_amd import crdbench

    gib = 1 << 30

    def card(n, used):
        d = tmp_path / f"card{n}" / "device"
        d.mkdir(parents=True, exist_ok=True)
        (d / "mem_info_vram_used").write_text(str(used))

    card(0, 1 * gib)
    card(1, 50 * gib)
    (tmp_path / "renderD128").mkdir()
    base = crdbench._vram_used(str(tmp_path))
    assert base == {"card0": gib, "card1": 50 * gib}
    card(0, 90 * gib)     # our job holds card0; card1 is another tenant that also grows a lot
    card(1, 60 * gib)
    held = crdbench._vram_used(str(tmp_path))
    threading.Timer(0.3, lambda: card(0, int(1.5 * gib))).start()
    t0 = time.time()
    waited = crdbench.wait_device_release(base, held, timeout=5.0, root=str(tmp_path), poll=0.01)
    assert 0.25 < waited < 2.0 and time.time() - t0 < 2.0
    # nothing of ours held -> no wait at all; a card that never drains -> bounded by timeout
    assert crdbench.wait_device_release(base, base, root=str(tmp_path)) < 0.05
    card(0, 90 * gib)
    assert 0.2 <= crdbench.wait_device_release(base, held, timeout=0.2, root=str(tmp_path), poll=0.01) < 1.0


def test_bench_pipeline_interleaved_two_ranks():
    """``--pp 2 --pp-virtual 2``: the interleaved 1F1B path end to end under torchrun (gloo)."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    args = [x for x in ARGS] + ["--pp", "2", "--pp-virtual", "2", "--grad-accum", "2", "--layers", "4"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    (rec,) = _json_lines(r.stdout)
    assert rec["config"]["parallelism"] == "dp1pp2" and rec["config"]["pp_virtual"] == 2
    assert rec["config"]["global_batch"] == 2 and rec["value"] > 0
    assert rec["loss_first"] > 0
