"""CRD-to-first-step latency -- the second half of BASELINE.json's headline metric
("... ; CRD-to-first-step p50", SURVEY.md §3.7: CR creationTimestamp -> the first step's log
line).

The platform runs as separate processes over HTTP (``cluster.ProcessCluster``: apiserver,
controller-manager with the training operator and scheduler, one kubelet per node with the
``amd.com/gpu`` device plugin); pods are real processes on this host.  Jobs are submitted one
after another; each job's workers are fresh processes (kfamd-launch -> ``python -m
service_account_auth_improvements_amd train``) that run one optimizer step and exit before
the next job's CR is created.  Per job the wall-clock time from the CR ``create`` call to rank
0's ``first_step`` event is measured, with a breakdown:

* ``cr_to_running``      CR create -> rank-0 pod Running (operator, scheduler, kubelet)
* ``running_to_process`` pod Running -> worker process start (kfamd-launch, interpreter)
* ``import``             worker start -> torch + runtime imported
* ``dist_init``          HIP runtime / device (+ process group when world > 1)
* ``model_init``         parameters, optimizer state
* ``init_to_first_step`` the first train step (first kernel / library loads included)

Used by ``bench.py`` (reported in its JSON line, measured before the bench process touches
the GPU) and by ``tools/bench_crd_to_step.py``.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import tempfile
import time
from typing import Callable, List, Optional

BREAKDOWN = ("cr_to_running", "running_to_process", "import", "dist_init", "model_init",
             "init_to_first_step", "process_to_init", "params_alloc_init", "optimizer_state")


def _events(path: str) -> list:
    try:
        with open(path) as f:
            return [json.loads(x) for x in f.read().splitlines() if x.strip()]
    except (OSError, ValueError):
        return []


def _vram_used(root: str = "/sys/class/drm") -> dict:
    """Per-card VRAM bytes in use, read from amdgpu's sysfs (no HIP call, so the measuring
    process stays off the GPU).  Empty when the node exposes no such files."""
    out = {}
    try:
        names = sorted(n for n in os.listdir(root) if n.startswith("card") and n[4:].isdigit())
    except OSError:
        return out
    for n in names:
        try:
            with open(os.path.join(root, n, "device", "mem_info_vram_used")) as f:
                out[n] = int(f.read().strip())
        except (OSError, ValueError):
            pass
    return out


def wait_device_release(base: dict, held: dict, n_devices: int = 1, timeout: float = 15.0,
                        slack: int = 1 << 30, root: str = "/sys/class/drm", poll: float = 0.05) -> float:
    """After a job's processes have exited, wait until the driver has given back the device
    memory they held.  The amdgpu driver tears a process's buffers down after the process is
    reaped; a next job that allocates during that teardown stalls for seconds in its first
    large allocations (seen as 2-3 s outliers in ``optimizer_state`` / the first step).
    Only the job's ``n_devices`` cards are watched: those whose usage rose most (by > 4 GiB)
    while the job ran (``held`` vs ``base``), so other tenants' cards on a shared node do not
    delay the loop.  Returns the seconds waited."""
    rise = sorted(((v - base.get(c, v), c) for c, v in held.items()), reverse=True)[:n_devices]
    ours = [c for d, c in rise if d > 4 * slack]
    t0 = time.time()
    while ours and time.time() - t0 < timeout:
        now = _vram_used(root)
        if all(now.get(c, 0) <= base.get(c, 0) + slack for c in ours):
            break
        time.sleep(poll)
    return time.time() - t0


def box_control(runs: int = 3, gpu: bool = False) -> dict:
    """The same box's own cost of the part of a worker start this repo does not control, measured
    right before the jobs in fresh interpreters: ``import_torch_s`` is the median time of
    ``import torch`` measured inside the child (the same span as a worker's ``import`` phase),
    ``python_import_torch_wall_s`` the child's whole wall time (interpreter start and exit
    included), with ``os.cpu_count()``, the CPUs this process may run on and the 1-minute load
    average.  ``gpu=True`` adds ``import torch`` + HIP runtime / device / context init
    (``torch.zeros(1, device='cuda')``), in-child.  ``p50 - import_torch_s`` then separates box
    speed from pipeline cost."""
    import subprocess

    def timed(code):
        inner, wall = [], []
        for _ in range(runs):
            t0 = time.perf_counter()
            r = subprocess.run([sys.executable, "-c", "import time; t0 = time.perf_counter(); " + code +
                                "; print(time.perf_counter() - t0)"],
                               check=True, capture_output=True, text=True)
            wall.append(time.perf_counter() - t0)
            inner.append(float(r.stdout.strip().splitlines()[-1]))
        return inner, wall
    imp, wall = timed("import torch")
    out = {"import_torch_s": round(statistics.median(imp), 3), "import_torch_runs_s": [round(x, 3) for x in imp],
           "python_import_torch_wall_s": round(statistics.median(wall), 3),
           "cpu_count": os.cpu_count(), "cpus_usable": len(os.sched_getaffinity(0)),
           "loadavg_1m": round(os.getloadavg()[0], 2)}
    if gpu:
        hip, _ = timed("import torch; torch.zeros(1, device='cuda'); torch.cuda.synchronize()")
        out["import_torch_hip_init_s"] = round(statistics.median(hip), 3)
        out["import_torch_hip_init_runs_s"] = [round(x, 3) for x in hip]
    return out


def measure(jobs: int = 3, model: str = "llama3-8b", gpus: int = 1, nodes: int = 1, seq_len: int = 8192,
            micro_batch: int = 1, layers: Optional[int] = None, device: str = "cuda", kind: str = "pytorchjob",
            processes: bool = True, gap: float = 0.0, release_wait: Optional[bool] = None,
            timeout: float = 300.0, port_base: int = 29700, poll: Optional[float] = None,
            control: bool = True,
            log: Callable[[str], None] = lambda s: print(s, file=sys.stderr, flush=True)) -> dict:
    """Submit ``jobs`` jobs one after another; returns p50 / p90 / min and the breakdown.

    ``poll`` is the measuring loop's period (default 0.05 s, ``KFAMD_CRD_POLL``).  The measured
    time comes from the worker's own ``first_step`` timestamp, so the period adds nothing to
    it; a short period only costs CPU that the worker's import competes for on a small box
    (0.01 vs 0.1 s A/B: profiles/crd_to_first_step_r6.md)."""
    if poll is None:
        poll = float(os.environ.get("KFAMD_CRD_POLL", "0.05"))
    ctl = box_control(gpu=device == "cuda") if control else None
    from .cluster import LocalCluster, ProcessCluster
    from .controlplane import training
    from .native import build_native
    build_native()
    if release_wait is None:
        release_wait = os.environ.get("KFAMD_CRD_RELEASE_WAIT", "1") != "0"
    tmp = tempfile.mkdtemp(prefix="crd2step-")
    events = os.path.join(tmp, "events.jsonl")
    env = {"KFAMD_EVENTS_FILE": events, "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS", "4")}
    t_up = time.time()
    if processes:
        cl = ProcessCluster(nodes=nodes, gpus_per_node=gpus, exec_pods=True, log_dir=tmp, extra_env=env).start()
        client, pod_log = cl.client, cl.pod_log
        client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "bench"}})
    else:
        cl = LocalCluster(n_gpus=gpus * nodes, exec_pods=True, api_port=None, log_dir=tmp, extra_env=env).start()
        client, pod_log = cl.client, cl.kubelet.pod_log
        cl.server.ensure_namespace("bench")
    t_up = time.time() - t_up
    cmd = [sys.executable, "-m", "service_account_auth_improvements_amd", "train", "--model", model,
           "--steps", "1", "--device", device]
    if model != "mnist":
        cmd += ["--seq-len", str(seq_len), "--micro-batch", str(micro_batch)]
    else:
        cmd += ["--micro-batch", "64"]
    if layers:
        cmd += ["--layers", str(layers)]
    rows: List[dict] = []
    try:
        for j in range(jobs):
            if j and gap:
                time.sleep(gap)
            name = f"job{j}"
            open(events, "w").close()
            port = port_base + 7 * j
            if kind == "mpijob":
                job = training.mpijob_manifest(name, "bench", "local", cmd, workers=nodes, gpus_per_worker=gpus,
                                               master_port=port)
                rank0_pod = f"{name}-worker-0"
            else:
                job = training.pytorchjob_manifest(name, "bench", "local", cmd, n_nodes=nodes, gpus_per_node=gpus,
                                                   master_port=port)
                if not gpus:
                    job["spec"]["nprocPerNode"] = "1"
                rank0_pod = f"{name}-master-0"
            base = _vram_used() if release_wait else {}
            t0 = time.time()
            client.create(job)
            t_running = None
            first = None
            evs: list = []
            deadline = t0 + timeout
            while time.time() < deadline:
                if t_running is None:
                    p = client.get_or_none("v1", "Pod", rank0_pod, "bench")
                    if p and (p.get("status") or {}).get("phase") == "Running":
                        t_running = time.time()
                evs = _events(events)
                fs = [e for e in evs if e["event"] == "first_step" and e.get("rank") == 0]
                if fs:
                    first = fs[0]
                    held = _vram_used() if release_wait else {}
                    break
                time.sleep(poll)
            if first is None:
                raise RuntimeError(f"{name}: no first_step within {timeout}s\n" + pod_log("bench", rank0_pod)[-3000:])
            r0 = [e for e in evs if e.get("rank") == 0]
            ps = next(e["ts"] for e in r0 if e["event"] == "process_start")
            ie = next(e for e in r0 if e["event"] == "init_done")
            imp = next((e["ts"] for e in r0 if e["event"] == "imported"), ps)
            dr = next((e["ts"] for e in r0 if e["event"] == "dist_ready"), imp)
            tr = t_running or ps
            rows.append({"total": first["ts"] - t0, "cr_to_running": tr - t0, "running_to_process": ps - tr,
                         "process_to_init": ie["ts"] - ps, "import": imp - ps, "dist_init": dr - imp,
                         "model_init": ie["ts"] - dr, "init_to_first_step": first["ts"] - ie["ts"],
                         "params_alloc_init": ie.get("params_alloc_init_s", 0.0),
                         "optimizer_state": ie.get("optimizer_state_s", 0.0)})
            # the job ends after its step; wait for it (and its pods' processes) so the devices
            # are free for the next job and for whatever runs after this measurement
            while time.time() < deadline:
                jb = client.get(job["apiVersion"], job["kind"], name, "bench")
                conds = (jb.get("status") or {}).get("conditions", [])
                if any(c["type"] in ("Succeeded", "Failed") and c["status"] == "True" for c in conds):
                    break
                time.sleep(0.05)
            if release_wait:
                rows[-1]["device_release"] = wait_device_release(base, held, n_devices=max(1, gpus * nodes))
            log(json.dumps({"crd_job": name, **{k: round(v, 3) for k, v in rows[-1].items()}}))
    finally:
        cl.stop()
    tot = sorted(r["total"] for r in rows)
    extra = {}
    if ctl is not None:
        p50 = statistics.median(tot)
        extra = {"box_control": ctl, "p50_minus_import_control_s": round(p50 - ctl["import_torch_s"], 3)}
        if "import_torch_hip_init_s" in ctl:
            extra["p50_minus_import_hip_control_s"] = round(p50 - ctl["import_torch_hip_init_s"], 3)
    return {**extra, "poll_s": poll, "jobs": len(rows), "kind": kind, "model": model, "gpus_per_node": gpus, "nodes": nodes,
            "control_plane": "processes over HTTP" if processes else "in-process",
            "p50_s": round(statistics.median(tot), 3),
            "p90_s": round(tot[min(len(tot) - 1, int(0.9 * len(tot)))], 3),
            "min_s": round(tot[0], 3), "max_s": round(tot[-1], 3),
            "per_job_s": [round(r["total"], 3) for r in rows],
            "cluster_up_s": round(t_up, 2),
            "device_release_wait_s": [round(r.get("device_release", 0.0), 3) for r in rows],
            "breakdown_p50_s": {k: round(statistics.median(r[k] for r in rows), 3) for k in BREAKDOWN}}
