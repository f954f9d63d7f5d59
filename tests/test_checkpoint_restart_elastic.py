"""Checkpoint-restart of an elastic PyTorchJob (runtime/checkpoint.py PeriodicCheckpointer,
runtime/train_entry.py --ckpt-dir/--save-every, kfamd-launch restarts):

3 workers (one rank each, gloo, ZeRO-1) train with a checkpoint every 4 steps.  One worker
process is SIGKILLed mid-run.  Its agent restarts it into a new rendezvous round, the other
agents see the membership change and restart theirs, and the new world of 3 resumes from the
atomically published ``latest``.  From the resumed step on, every rank's loss trajectory equals
an uninterrupted run's bit for bit, and the job ends Succeeded.

The reference analogue is level-triggered recovery: controller state kept in the API object
survives restarts (/root/reference/components/notebook-controller/controllers/culling_controller.go:50-52).
"""
import json
import os
import signal
import sys
import time

import pytest

from service_account_auth_improvements_amd.controlplane import training
from service_account_auth_improvements_amd.controlplane.apiserver import APIServer
from service_account_auth_improvements_amd.controlplane.client import InMemoryClient
from service_account_auth_improvements_amd.controlplane.kubelet import Kubelet
from service_account_auth_improvements_amd.controlplane.runtime import Manager

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = 60


def _events(path):
    if not os.path.exists(path):
        return []
    out = []
    with open(path) as f:
        for line in f:
            try:
                out.append(json.loads(line))
            except ValueError:
                pass          # a line being appended right now
    return out


def _state(c, name):
    conds = {x["type"] for x in (c.get(training.PT_API, "PyTorchJob", name, "team").get("status") or {})
             .get("conditions", []) if x["status"] == "True"}
    return "Succeeded" if "Succeeded" in conds else "Failed" if "Failed" in conds else None


def _run_job(tmp, name, port, kill_after_publish=None):
    srv = APIServer()
    training.register(srv)
    c = InMemoryClient(srv)
    srv.ensure_namespace("team")
    mgr = Manager(c)
    mgr.add(training.PyTorchJobReconciler(c))
    ev = os.path.join(tmp, f"{name}.events")
    kub = Kubelet(c, n_gpus=0, exec_pods=True, workdir=ROOT, log_dir=str(tmp),
                  extra_env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1", "KFAMD_EVENTS_FILE": ev})
    mgr.add(kub)
    ck = os.path.join(tmp, f"{name}-ckpt")
    cmd = [sys.executable, "-m", "service_account_auth_improvements_amd.runtime.train_entry", "--model", "tiny",
           "--device", "cpu", "--seq-len", "32", "--micro-batch", "2", "--zero1", "--steps", str(STEPS),
           "--ckpt-dir", ck, "--save-every", "4"]
    job = training.pytorchjob_manifest(name, "team", "local", cmd, n_nodes=1, gpus_per_node=0, master_port=port,
                                       restart_policy="OnFailure")
    specs = job["spec"]["pytorchReplicaSpecs"]
    specs["Worker"] = dict(specs.pop("Master"), replicas=3)
    job["spec"]["nprocPerNode"] = "1"
    job["spec"]["elasticPolicy"] = {"minReplicas": 2, "maxReplicas": 3, "maxRestarts": 3,
                                    "rdzvConf": [{"key": "last_call_timeout", "value": "1"}]}
    c.create(job)
    mgr.start(workers=2)
    killed = None
    try:
        deadline = time.time() + 240
        state = None
        while time.time() < deadline and state is None:
            if kill_after_publish is not None and killed is None:
                recs = _events(ev)
                pub = [e for e in recs if e["event"] == "checkpoint_published" and e["step"] >= kill_after_publish]
                r2 = [e for e in recs if e["event"] == "step" and e["rank"] == 2]
                if pub and r2 and r2[-1]["step"] >= pub[0]["step"] + 1:
                    killed = {"pid": r2[-1]["pid"], "at_step": r2[-1]["step"], "latest": pub[-1]["step"]}
                    os.kill(killed["pid"], signal.SIGKILL)       # one worker process dies mid-run
            state = _state(c, name)
            time.sleep(0.05)
        logs = "\n".join(kub.pod_log("team", f"{name}-worker-{i}")[-2000:] for i in range(3))
        assert state == "Succeeded", logs
    finally:
        mgr.stop()
        kub.shutdown()
    return _events(ev), killed


@pytest.mark.slow
def test_killed_worker_restarts_resume_from_latest_with_the_uninterrupted_trajectory(tmp_path):
    base, _ = _run_job(str(tmp_path), "ref", 29871)
    run, killed = _run_job(str(tmp_path), "kill", 29881, kill_after_publish=8)
    assert killed is not None, "the run finished before the kill"
    assert killed["at_step"] < STEPS - 1

    def losses(evs, rank):
        out = {}
        for e in evs:
            if e["event"] == "step" and e["rank"] == rank:
                out.setdefault(e["step"], []).append(e["loss"])
        return out

    resumed = [e for e in run if e["event"] == "resumed"]
    assert {e["rank"] for e in resumed} == {0, 1, 2}, resumed
    start = {e["step"] for e in resumed}
    assert len(start) == 1
    start = start.pop()
    assert start % 4 == 0 and 8 <= start <= killed["at_step"] + 1, (start, killed)
    assert all(e["auto"] for e in resumed)
    print("killed", killed, "resumed from step", start)
    for rank in range(3):
        ref, got = losses(base, rank), losses(run, rank)
        assert sorted(ref) == list(range(STEPS))
        assert sorted(got) == list(range(STEPS)), rank
        for s in range(STEPS):
            # every execution of a step (before the kill, and again after the resume) has the
            # uninterrupted run's loss
            assert all(v == ref[s][0] for v in got[s]), (rank, s, got[s], ref[s])
        # the new world re-ran only the steps after the checkpoint it resumed from
        assert all(len(got[s]) == 1 for s in range(start)), rank
    pids = {e["pid"] for e in run if e["event"] == "process_start"}
    assert len(pids) == 6                       # 3 workers, each started twice (the kill's round)
