"""PyTorchJob / MPIJob operators: object-level assertions, and one real end-to-end run
(CRD -> operator -> pods -> kfamd-launch -> gloo workers -> first step) on CPU."""
import json
import os
import time

import pytest

from service_account_auth_improvements_amd.controlplane import training
from service_account_auth_improvements_amd.controlplane.apiserver import APIServer
from service_account_auth_improvements_amd.controlplane.client import InMemoryClient
from service_account_auth_improvements_amd.controlplane.kubelet import Kubelet
from service_account_auth_improvements_amd.controlplane.runtime import Manager


@pytest.fixture
def cl():
    srv = APIServer()
    c = InMemoryClient(srv)
    srv.ensure_namespace("team")
    mgr = Manager(c)
    mgr.add(training.PyTorchJobReconciler(c))
    mgr.add(training.MPIJobReconciler(c))
    kub = Kubelet(c, n_gpus=8)
    mgr.add(kub)
    return srv, c, mgr, kub


def test_pytorchjob_pods_env_and_status(cl):
    srv, c, mgr, _ = cl
    c.create(training.pytorchjob_manifest("llama", "team", "kfamd/trainer:rocm", ["python", "-c", "pass"],
                                          n_nodes=2, gpus_per_node=8))
    mgr.run_until_idle()
    m = c.get("v1", "Pod", "llama-master-0", "team")
    w = c.get("v1", "Pod", "llama-worker-0", "team")
    env = {e["name"]: e["value"] for e in w["spec"]["containers"][0]["env"]}
    assert env["MASTER_ADDR"] == "llama-master-0" and env["WORLD_SIZE"] == "2" and env["RANK"] == "1"
    assert env["PET_NPROC_PER_NODE"] == "8" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert "CUDA_VISIBLE_DEVICES" not in env
    assert w["spec"]["containers"][0]["command"][0].endswith("kfamd_launch")
    assert m["metadata"]["labels"][training.LBL_ROLE] == "master"
    svc = c.get("v1", "Service", "llama-master-0", "team")
    assert svc["spec"]["clusterIP"] == "None"
    job = c.get(training.PT_API, "PyTorchJob", "llama", "team")
    types = {cd["type"] for cd in job["status"]["conditions"] if cd["status"] == "True"}
    assert {"Created", "Running"} <= types
    assert job["status"]["replicaStatuses"]["Master"]["active"] == 1
    # a third node does not fit: 16 GPUs are allocated on this 8-GPU node -> the second
    # pod stays Pending/Unschedulable (device plugin accounting)
    assert c.get("v1", "Pod", "llama-worker-0", "team")["status"]["phase"] == "Pending"


def test_pytorchjob_metrics_and_checkpoint_annotations_reach_the_workers(cl):
    """kfamd.io/metrics-port -> KFAMD_METRICS_PORT + prometheus.io scrape annotations on every
    pod; kfamd.io/checkpoint-dir / save-every -> the worker's periodic checkpoint-restart env."""
    srv, c, mgr, _ = cl
    c.create(training.pytorchjob_manifest("obs", "team", "kfamd/trainer:rocm", ["python", "-c", "pass"],
                                          n_nodes=1, gpus_per_node=1, metrics_port=9400,
                                          ckpt_dir="/mnt/ckpt/obs", save_every=50))
    mgr.run_until_idle()
    p = c.get("v1", "Pod", "obs-master-0", "team")
    env = {e["name"]: e["value"] for e in p["spec"]["containers"][0]["env"]}
    assert env["KFAMD_METRICS_PORT"] == "9400"
    assert env["KFAMD_CKPT_DIR"] == "/mnt/ckpt/obs" and env["KFAMD_SAVE_EVERY"] == "50"
    ann = p["metadata"]["annotations"]
    assert ann["prometheus.io/scrape"] == "true" and ann["prometheus.io/port"] == "9400"
    assert ann["prometheus.io/path"] == "/metrics"
    assert ann["sidecar.istio.io/inject"] == "false"          # the template's own annotation kept


def test_pytorchjob_failure_restart_and_backoff(cl):
    srv, c, mgr, _ = cl
    c.create(training.pytorchjob_manifest("j", "team", "img", ["x"], n_nodes=1, gpus_per_node=1, backoff_limit=1))
    mgr.run_until_idle()
    pod = c.get("v1", "Pod", "j-master-0", "team")
    pod["status"] = {"phase": "Failed", "containerStatuses": [{"name": "pytorch", "state": {"terminated": {"exitCode": 1}}}]}
    c.update_status(pod)
    mgr.run_until_idle()
    job = c.get(training.PT_API, "PyTorchJob", "j", "team")
    assert job["status"]["restartCount"] == 1
    assert any(cd["type"] == "Restarting" for cd in job["status"]["conditions"])
    pod = c.get("v1", "Pod", "j-master-0", "team")   # recreated
    pod["status"] = {"phase": "Failed", "containerStatuses": [{"name": "pytorch", "state": {"terminated": {"exitCode": 1}}}]}
    c.update_status(pod)
    mgr.run_until_idle()
    job = c.get(training.PT_API, "PyTorchJob", "j", "team")
    assert any(cd["type"] == "Failed" and cd["status"] == "True" for cd in job["status"]["conditions"])


def test_mpijob_hostfile_and_roles(cl):
    srv, c, mgr, _ = cl
    tpl = {"spec": {"containers": [{"name": "mpi", "image": "img", "command": ["true"]}]}}
    c.create({"apiVersion": training.MPI_API, "kind": "MPIJob",
              "metadata": {"name": "m70", "namespace": "team"},
              "spec": {"slotsPerWorker": 8, "mpiReplicaSpecs": {
                  "Launcher": {"replicas": 1, "template": tpl}, "Worker": {"replicas": 1, "template": tpl}}}})
    mgr.run_until_idle()
    cm = c.get("v1", "ConfigMap", "m70-config", "team")
    assert cm["data"]["hostfile"] == "m70-worker-0.m70.team.svc slots=8\n"
    assert c.get_or_none("v1", "Pod", "m70-launcher-0", "team") is not None
    assert c.get_or_none("v1", "Service", "m70-worker-0", "team") is not None
    assert c.get_or_none("v1", "Service", "m70-launcher-0", "team") is None


@pytest.mark.slow
def test_pytorchjob_end_to_end_cpu(tmp_path):
    """CR -> operator -> pod -> kfamd-launch (2 workers, gloo) -> trainer first step."""
    import sys
    srv = APIServer()
    c = InMemoryClient(srv)
    srv.ensure_namespace("team")
    mgr = Manager(c)
    mgr.add(training.PyTorchJobReconciler(c))
    ev = tmp_path / "events.jsonl"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    kub = Kubelet(c, n_gpus=0, exec_pods=True, workdir=root, log_dir=str(tmp_path),
                  extra_env={"KFAMD_EVENTS_FILE": str(ev), "PYTHONPATH": root, "OMP_NUM_THREADS": "1"})
    mgr.add(kub)
    cmd = [sys.executable, "-m", "service_account_auth_improvements_amd.runtime.train_entry", "--model", "tiny",
           "--seq-len", "32", "--steps", "2", "--device", "cpu"]
    job = training.pytorchjob_manifest("e2e", "team", "local", cmd, n_nodes=1, gpus_per_node=0, master_port=29613)
    job["spec"]["nprocPerNode"] = "2"
    created = c.create(job)
    t0 = time.time()
    mgr.start(workers=2)
    try:
        deadline = time.time() + 240
        while time.time() < deadline:
            j = c.get(training.PT_API, "PyTorchJob", "e2e", "team")
            if any(cd["type"] in ("Succeeded", "Failed") and cd["status"] == "True"
                   for cd in (j.get("status") or {}).get("conditions", [])):
                break
            time.sleep(0.5)
    finally:
        mgr.stop()
        kub.shutdown()
    j = c.get(training.PT_API, "PyTorchJob", "e2e", "team")
    log = kub.pod_log("team", "e2e-master-0")
    assert any(cd["type"] == "Succeeded" and cd["status"] == "True" for cd in j["status"]["conditions"]), log
    events = [json.loads(x) for x in ev.read_text().splitlines()]
    firsts = [e for e in events if e["event"] == "first_step"]
    assert {e["rank"] for e in firsts} == {0, 1}
    assert min(e["ts"] for e in firsts) - t0 < 240
