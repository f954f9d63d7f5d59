"""Multi-node local clusters: the scheduler (pods/binding, GPU-aware filter + bin-packing score,
Unschedulable status and retry), the pods/binding subresource over REST, and the platform split
into processes (apiserver / controller-manager / one kubelet per node) running a 2-node
PyTorchJob end to end on CPU."""
import json
import os
import sys
import time

import pytest

from service_account_auth_improvements_amd.cluster import LocalCluster, ProcessCluster
from service_account_auth_improvements_amd.controlplane import training
from service_account_auth_improvements_amd.controlplane.apiserver import ApiError
from service_account_auth_improvements_amd.controlplane.client import RestClient

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pod(name, gpus, **spec):
    c = {"name": "main", "image": "img"}
    if gpus:
        c["resources"] = {"limits": {"amd.com/gpu": str(gpus)}}
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "team"},
            "spec": dict({"containers": [c]}, **spec)}


def _node_of(c, name):
    return c.get("v1", "Pod", name, "team")["spec"].get("nodeName")


def test_scheduler_binpacks_gpus_and_retries_unschedulable():
    cl = LocalCluster(n_gpus=2, nodes=2, api_port=None)
    c, m = cl.client, cl.manager
    cl.server.ensure_namespace("team")
    for name, g in (("a", 2), ("b", 1), ("c", 1)):
        c.create(_pod(name, g))
        m.run_until_idle()
    assert _node_of(c, "a") == "node-0"                 # tie -> name order
    assert _node_of(c, "b") == "node-1" == _node_of(c, "c")   # most-allocated: c joins b
    c.create(_pod("d", 2))
    m.run_until_idle()
    d = c.get("v1", "Pod", "d", "team")
    assert not d["spec"].get("nodeName")
    cond = next(x for x in d["status"]["conditions"] if x["type"] == "PodScheduled")
    assert cond["status"] == "False" and cond["reason"] == "Unschedulable"
    assert cond["message"] == "0/2 nodes are available: 2 Insufficient amd.com/gpu."
    # a finishing pod frees its node's GPUs -> the pending pod is bound there
    a = c.get("v1", "Pod", "a", "team")
    a["status"] = dict(a["status"], phase="Succeeded")
    c.update_status(a)
    deadline = time.time() + 10
    while time.time() < deadline and _node_of(c, "d") is None:
        m.run_until_idle()
        time.sleep(0.05)
    assert _node_of(c, "d") == "node-0"
    assert c.get("v1", "Pod", "d", "team")["status"]["phase"] == "Running"
    ev = [e for e in c.list("v1", "Event", "team") if e["reason"] == "Scheduled"]
    assert any("team/d to node-0" in e["message"] for e in ev)


def test_scheduler_filters_taints_selectors_and_cpu_spread():
    cl = LocalCluster(n_gpus=1, nodes=3, api_port=None)
    c, m = cl.client, cl.manager
    cl.server.ensure_namespace("team")
    n1 = c.get("v1", "Node", "node-1")
    n1["spec"]["taints"] = [{"key": "amd.com/gpu", "value": "reserved", "effect": "NoSchedule"}]
    c.update(n1)
    n2 = c.get("v1", "Node", "node-2")
    n2["metadata"]["labels"]["pool"] = "mi355x"
    c.update(n2)
    c.create(_pod("sel", 1, nodeSelector={"pool": "mi355x"}))
    c.create(_pod("tol", 1, tolerations=[{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}]))
    m.run_until_idle()
    assert _node_of(c, "sel") == "node-2"
    assert _node_of(c, "tol") in ("node-0", "node-1")
    c.create(_pod("plain", 1))
    m.run_until_idle()
    free = {"node-0", "node-1"} - {_node_of(c, "tol")}
    if free == {"node-1"}:          # only the tainted node is left: no fit
        assert _node_of(c, "plain") is None
    else:
        assert _node_of(c, "plain") == "node-0"
    # CPU-only pods spread to the least loaded node
    c.create(_pod("cpu0", 0))
    m.run_until_idle()
    assert _node_of(c, "cpu0") is not None


def test_binding_subresource_over_rest():
    cl = LocalCluster(n_gpus=1, nodes=2, api_port=0)
    cl.http.start()
    try:
        rc = RestClient(cl.http.url)
        cl.server.ensure_namespace("team")
        rc.create(_pod("p", 0, schedulerName="other-scheduler"))   # the default scheduler leaves it alone
        rc.bind("team", "p", "node-1")
        assert rc.get("v1", "Pod", "p", "team")["spec"]["nodeName"] == "node-1"
        with pytest.raises(ApiError) as e:
            rc.bind("team", "p", "node-0")
        assert e.value.code == 409
    finally:
        cl.http.stop()


@pytest.mark.slow
def test_two_node_pytorchjob_across_processes(tmp_path):
    """apiserver, controller-manager and two kubelets as separate processes over HTTP; a
    2-replica PyTorchJob (1 CPU worker per node, gloo) reaches its first step and succeeds,
    its pods placed on different nodes by the scheduler."""
    ev = tmp_path / "events.jsonl"
    ev.write_text("")
    pc = ProcessCluster(nodes=2, gpus_per_node=0, exec_pods=True, log_dir=str(tmp_path),
                        extra_env={"KFAMD_EVENTS_FILE": str(ev), "OMP_NUM_THREADS": "1"}).start()
    try:
        c = pc.client
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
        cmd = [sys.executable, "-m", "service_account_auth_improvements_amd.runtime.train_entry", "--model", "tiny",
               "--seq-len", "32", "--steps", "2", "--device", "cpu"]
        job = training.pytorchjob_manifest("mp", "team", "local", cmd, n_nodes=2, gpus_per_node=0, master_port=29641)
        job["spec"]["nprocPerNode"] = "1"
        c.create(job)
        deadline = time.time() + 240
        done = None
        while time.time() < deadline:
            j = c.get(training.PT_API, "PyTorchJob", "mp", "team")
            done = next((cd["type"] for cd in (j.get("status") or {}).get("conditions", [])
                         if cd["type"] in ("Succeeded", "Failed") and cd["status"] == "True"), None)
            if done:
                break
            time.sleep(0.25)
        logs = pc.pod_log("team", "mp-master-0") + pc.component_log("controller-manager")[-2000:]
        assert done == "Succeeded", logs
        nodes = {_node_of(c, "mp-master-0"), _node_of(c, "mp-worker-0")}
        assert nodes == {"node-0", "node-1"}
        firsts = [json.loads(x) for x in ev.read_text().splitlines() if '"first_step"' in x]
        assert {e["rank"] for e in firsts} == {0, 1}
    finally:
        pc.stop()


def test_finished_pod_frees_its_gpus_for_the_next_binding():
    """The assume cache must let go of a binding once the view shows the pod bound -- also when
    the pod has already finished by then (short jobs on a 1-GPU node, back to back)."""
    cl = LocalCluster(n_gpus=1, nodes=2, api_port=None)
    c, m = cl.client, cl.manager
    cl.server.ensure_namespace("team")
    for i in range(4):
        c.create(_pod(f"p{i}", 1))
        m.run_until_idle()
        node = _node_of(c, f"p{i}")
        assert node is not None, i
        p = c.get("v1", "Pod", f"p{i}", "team")
        p["status"] = dict(p.get("status") or {}, phase="Succeeded")
        c.update_status(p)
        m.run_until_idle()
