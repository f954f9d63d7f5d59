"""Local workload plane: StatefulSet / Deployment controllers, a scheduler stand-in and a
kubelet that can really run pod containers as local processes.

The reference's integration tests assert on created objects only (envtest has no
kubelet).  To measure the north-star "CRD-to-first-step" latency and to run
PyTorchJob e2e tests, this module closes the loop on a single machine:

* ``StatefulSetController`` / ``DeploymentController`` create the template pods (owner
  references set, so GC works) and maintain ``status.readyReplicas``;
* ``Kubelet`` binds pending pods to a node (writing ``spec.nodeName`` -- how the reference
  fakes scheduling in pvcviewer tests), honours ``amd.com/gpu`` limits with a device
  plugin that assigns concrete GPU indices and injects ``HIP_VISIBLE_DEVICES``, and either
  marks pods Running/Ready (simulation) or, when ``exec_pods`` is set, executes the first
  container's command with its env as a subprocess and reports Succeeded / Failed from
  the exit code.
"""
from __future__ import annotations

import copy
import hashlib
import json
import logging
import os
import subprocess
import threading
import time
from typing import Dict, List, Optional

from .apiserver import ApiError, now_rfc3339, set_controller_reference
from .client import Client
from .runtime import Controller, Request, Result, for_kind, owns

log = logging.getLogger("kubelet")
GPU_RESOURCE = "amd.com/gpu"


def _pod_ready(pod: dict) -> bool:
    for c in (pod.get("status") or {}).get("conditions") or []:
        if c.get("type") == "Ready":
            return c.get("status") == "True"
    return False



_LAUNCHER_VARS = frozenset({"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                            "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"})


def _launcher_var(name: str) -> bool:
    """Process-launcher state of the kubelet's own parent (torchrun / the bench), not node state."""
    return name in _LAUNCHER_VARS or name.startswith(("TORCHELASTIC_", "KFAMD_BENCH_"))

class StatefulSetController(Controller):
    name = "statefulset-controller"

    def sources(self):
        return [for_kind("apps/v1", "StatefulSet"), owns("v1", "Pod", "StatefulSet")]

    def reconcile(self, req: Request) -> Result:
        c = self.client
        sts = c.get_or_none("apps/v1", "StatefulSet", req.name, req.namespace)
        if sts is None or sts["metadata"].get("deletionTimestamp"):
            return Result()
        want = int(sts["spec"].get("replicas", 1) or 0)
        tpl = sts["spec"]["template"]
        pods = [p for p in c.list("v1", "Pod", req.namespace)
                if any(r.get("uid") == sts["metadata"]["uid"] for r in p["metadata"].get("ownerReferences") or [])]
        have = {p["metadata"]["name"]: p for p in pods}
        for i in range(want):
            pn = f"{req.name}-{i}"
            if pn not in have:
                pod = {"apiVersion": "v1", "kind": "Pod",
                       "metadata": {"name": pn, "namespace": req.namespace,
                                    "labels": dict(tpl.get("metadata", {}).get("labels") or {},
                                                   **{"statefulset.kubernetes.io/pod-name": pn}),
                                    "annotations": dict(tpl.get("metadata", {}).get("annotations") or {})},
                       "spec": copy.deepcopy(tpl.get("spec", {}))}
                pod["spec"]["hostname"] = pn
                c.create(set_controller_reference(sts, pod))
        for pn, p in have.items():
            idx = pn.rsplit("-", 1)[-1]
            if not idx.isdigit() or int(idx) >= want:
                c.delete("v1", "Pod", pn, req.namespace)
        ready = sum(1 for p in have.values() if _pod_ready(p) and int(p["metadata"]["name"].rsplit("-", 1)[-1]) < want)
        st = {"replicas": min(len(have), want) if want else 0, "readyReplicas": ready}
        if sts.get("status") != st:
            sts["status"] = st
            c.update_status(sts)
        return Result()


class DeploymentController(Controller):
    name = "deployment-controller"

    def sources(self):
        return [for_kind("apps/v1", "Deployment"), owns("v1", "Pod", "Deployment")]

    def reconcile(self, req: Request) -> Result:
        c = self.client
        dep = c.get_or_none("apps/v1", "Deployment", req.name, req.namespace)
        if dep is None or dep["metadata"].get("deletionTimestamp"):
            return Result()
        want = int(dep["spec"].get("replicas", 1) if dep["spec"].get("replicas") is not None else 1)
        tpl = dep["spec"]["template"]
        h = hashlib.sha1(json.dumps(tpl, sort_keys=True).encode()).hexdigest()[:10]
        pods = [p for p in c.list("v1", "Pod", req.namespace)
                if any(r.get("uid") == dep["metadata"]["uid"] for r in p["metadata"].get("ownerReferences") or [])]
        current = [p for p in pods if (p["metadata"].get("labels") or {}).get("pod-template-hash") == h]
        for p in pods:   # template changed (Recreate / RollingUpdate collapsed): replace old pods
            if p not in current:
                c.delete("v1", "Pod", p["metadata"]["name"], req.namespace)
        for i in range(len(current), want):
            pod = {"apiVersion": "v1", "kind": "Pod",
                   "metadata": {"generateName": f"{req.name}-{h}-", "namespace": req.namespace,
                                "labels": dict(tpl.get("metadata", {}).get("labels") or {}, **{"pod-template-hash": h}),
                                "annotations": dict(tpl.get("metadata", {}).get("annotations") or {})},
                   "spec": copy.deepcopy(tpl.get("spec", {}))}
            c.create(set_controller_reference(dep, pod))
        for p in current[want:]:
            c.delete("v1", "Pod", p["metadata"]["name"], req.namespace)
        ready = sum(1 for p in current[:want] if _pod_ready(p))
        conds = [{"type": "Available", "status": "True" if ready >= want else "False",
                  "reason": "MinimumReplicasAvailable" if ready >= want else "MinimumReplicasUnavailable",
                  "lastTransitionTime": now_rfc3339()}]
        st = {"replicas": min(len(current), want), "readyReplicas": ready, "availableReplicas": ready,
              "conditions": conds}
        old = dep.get("status") or {}
        if {k: old.get(k) for k in ("replicas", "readyReplicas")} != {k: st[k] for k in ("replicas", "readyReplicas")} \
                or [x.get("status") for x in old.get("conditions") or []] != [x["status"] for x in conds]:
            dep["status"] = st
            c.update_status(dep)
        return Result()


class DevicePlugin:
    """amd.com/gpu allocator for one node: hands out concrete GPU indices."""

    def __init__(self, n_gpus: int, base: int = 0):
        self.free = list(range(base, base + n_gpus))
        self.owner: Dict[str, List[int]] = {}

    def allocate(self, pod_uid: str, n: int) -> Optional[List[int]]:
        if pod_uid in self.owner:
            return self.owner[pod_uid]
        if n > len(self.free):
            return None
        ids, self.free = self.free[:n], self.free[n:]
        self.owner[pod_uid] = ids
        return ids

    def release(self, pod_uid: str):
        ids = self.owner.pop(pod_uid, [])
        self.free = sorted(self.free + ids)


def pod_gpu_request(pod: dict) -> int:
    n = 0
    for c in pod.get("spec", {}).get("containers") or []:
        res = c.get("resources") or {}
        v = (res.get("limits") or {}).get(GPU_RESOURCE) or (res.get("requests") or {}).get(GPU_RESOURCE)
        if v:
            n += int(v)
    return n


class Kubelet(Controller):
    """Node agent for node ``node_name``.  ``exec_pods``: run containers for real."""
    name = "kubelet"

    def __init__(self, client: Client, node_name: str = "node-0", n_gpus: int = 8, exec_pods: bool = False,
                 extra_env: Optional[dict] = None, workdir: Optional[str] = None, log_dir: Optional[str] = None,
                 self_schedule: bool = True, gpu_base: int = 0):
        super().__init__(client)
        self.node = node_name
        self.name = "kubelet" if node_name == "node-0" else f"kubelet-{node_name}"
        # self_schedule: the single-node cluster's kubelet claims every unbound pod; with a
        # scheduler (multi-node clusters) it runs only the pods bound to its node
        self.self_schedule = self_schedule
        self.dp = DevicePlugin(n_gpus, gpu_base)
        self.exec_pods = exec_pods
        self.extra_env = extra_env or {}
        self.workdir = workdir
        self.log_dir = log_dir
        self.procs: Dict[str, subprocess.Popen] = {}
        self.uids: Dict[str, str] = {}      # ns/name -> uid holding devices (released when the pod goes)
        self.logs: Dict[str, str] = {}
        self._lock = threading.Lock()
        self._register_node(n_gpus)

    def _register_node(self, n_gpus):
        if self.client.get_or_none("v1", "Node", self.node) is None:
            self.client.create({"apiVersion": "v1", "kind": "Node",
                                "metadata": {"name": self.node, "labels": {"kubernetes.io/hostname": self.node}},
                                "spec": {"providerID": "local://" + self.node},
                                "status": {"capacity": {"cpu": str(os.cpu_count() or 8), "memory": "64Gi",
                                                        GPU_RESOURCE: str(n_gpus)},
                                           "allocatable": {GPU_RESOURCE: str(n_gpus)}}})

    def sources(self):
        return [for_kind("v1", "Pod")]

    def _status(self, phase, ready, state, reason="", message="", pod=None):
        t = now_rfc3339()
        conds = [{"type": "PodScheduled", "status": "True", "lastTransitionTime": t},
                 {"type": "Initialized", "status": "True", "lastTransitionTime": t},
                 {"type": "ContainersReady", "status": "True" if ready else "False", "lastTransitionTime": t},
                 {"type": "Ready", "status": "True" if ready else "False", "lastTransitionTime": t}]
        cs = [{"name": c["name"], "ready": ready, "restartCount": 0, "state": state, "image": c.get("image", "")}
              for c in (pod or {}).get("spec", {}).get("containers") or []]
        st = {"phase": phase, "conditions": conds, "containerStatuses": cs, "hostIP": "127.0.0.1",
              "podIP": "127.0.0.1", "startTime": t}
        if reason:
            st["reason"] = reason
        if message:
            st["message"] = message
        return st

    def reconcile(self, req: Request) -> Result:
        c = self.client
        pod = c.get_or_none("v1", "Pod", req.name, req.namespace)
        key = f"{req.namespace}/{req.name}"
        if pod is None or pod["metadata"].get("deletionTimestamp"):
            # the pod is gone (or going): stop its container and give its GPUs back
            with self._lock:
                p = self.procs.pop(key, None)
            if p and p.poll() is None:
                p.terminate()
            uid = self.uids.pop(key, None) or (pod or {}).get("metadata", {}).get("uid")
            if uid:
                self.dp.release(uid)
            return Result()
        uid = pod["metadata"]["uid"]
        phase = (pod.get("status") or {}).get("phase")
        if phase in ("Succeeded", "Failed"):
            self.dp.release(uid)
            self.uids.pop(key, None)
            return Result()
        bound = pod["spec"].get("nodeName")
        if not bound:
            if not self.self_schedule:
                return Result()
            pod["spec"]["nodeName"] = self.node
            pod = c.update(pod)
        elif bound != self.node:
            return Result()
        if phase in (None, "", "Pending"):
            ngpu = pod_gpu_request(pod)
            ids = self.dp.allocate(uid, ngpu) if ngpu else []
            if ngpu and ids is not None:
                self.uids[key] = uid
            if ids is None:
                st = self._status("Pending", False, {"waiting": {"reason": "Unschedulable"}},
                                  "Unschedulable", f"0/1 nodes are available: insufficient {GPU_RESOURCE}", pod)
                st["conditions"][0] = {"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                                       "message": f"insufficient {GPU_RESOURCE}"}
                pod["status"] = st
                c.update_status(pod)
                return Result(requeue_after=1.0)
            if self.exec_pods and (pod["spec"]["containers"][0].get("command") or
                                   pod["spec"]["containers"][0].get("args")):
                self._start(pod, ids)
                pod["status"] = self._status("Running", True, {"running": {"startedAt": now_rfc3339()}}, pod=pod)
                c.update_status(pod)
                return Result(requeue_after=0.2)
            pod["status"] = self._status("Running", True, {"running": {"startedAt": now_rfc3339()}}, pod=pod)
            c.update_status(pod)
            return Result()
        if phase == "Running" and key in self.procs:
            p = self.procs[key]
            rc = p.poll()
            if rc is None:
                return Result(requeue_after=0.2)
            term = {"terminated": {"exitCode": rc, "reason": "Completed" if rc == 0 else "Error",
                                   "finishedAt": now_rfc3339()}}
            pod["status"] = self._status("Succeeded" if rc == 0 else "Failed", False, term, pod=pod)
            c.update_status(pod)
            self.dp.release(uid)
            with self._lock:
                self.procs.pop(key, None)
        return Result()

    def _start(self, pod: dict, gpu_ids: List[int]):
        ctr = pod["spec"]["containers"][0]
        # a container gets the node's base environment, never the rank identity of whatever
        # launched this kubelet (a kubelet started by rank 0 of a torchrun job would otherwise
        # hand its RANK / MASTER_PORT / TORCHELASTIC_USE_AGENT_STORE to every pod, whose
        # rendezvous then waits on the outer job's store)
        env = {k: v for k, v in os.environ.items() if not _launcher_var(k)}
        env.update(self.extra_env)
        # single-host cluster DNS: a value naming a Service of the pod's namespace
        # (e.g. MASTER_ADDR=<job>-master-0) resolves to this host
        ns = pod["metadata"]["namespace"]
        svcs = {s["metadata"]["name"] for s in self.client.list("v1", "Service", ns)}
        for e in ctr.get("env") or []:
            if "value" in e:
                v = str(e["value"])
                host = v.split(".")[0]
                env[e["name"]] = "127.0.0.1" if (v in svcs or (host in svcs and ".svc" in v)) else v
        if gpu_ids:
            env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, gpu_ids))
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
        env["POD_NAME"] = pod["metadata"]["name"]
        env["POD_NAMESPACE"] = pod["metadata"]["namespace"]
        cmd = list(ctr.get("command") or []) + list(ctr.get("args") or [])
        if cmd and cmd[0] == "kfamd-launch":      # the image's /usr/local/bin launcher == our build
            from ..native import binary
            cmd[0] = binary("kfamd_launch")
        key = f'{pod["metadata"]["namespace"]}/{pod["metadata"]["name"]}'
        out = subprocess.DEVNULL
        if self.log_dir:
            os.makedirs(self.log_dir, exist_ok=True)
            path = os.path.join(self.log_dir, key.replace("/", "_") + ".log")
            self.logs[key] = path
            out = open(path, "w")
        # the image's filesystem is not on this host: a workingDir that only exists inside the
        # image (e.g. the notebook controller's /home/jovyan) falls back to the kubelet's workdir
        wd = ctr.get("workingDir")
        cwd = wd if wd and os.path.isdir(wd) else self.workdir
        p = subprocess.Popen(cmd, env=env, cwd=cwd, stdout=out, stderr=subprocess.STDOUT)
        with self._lock:
            self.procs[key] = p

    def pod_pids(self) -> Dict[str, int]:
        """Running pod processes (``ns/name`` -> pid), for the dashboard's metrics sampler."""
        with self._lock:
            return {k: p.pid for k, p in self.procs.items() if p.poll() is None}

    def pod_log(self, namespace: str, name: str) -> str:
        path = self.logs.get(f"{namespace}/{name}")
        if path and os.path.exists(path):
            return open(path).read()
        return ""

    def shutdown(self):
        with self._lock:
            for p in self.procs.values():
                if p.poll() is None:
                    p.terminate()
            for p in self.procs.values():
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    p.kill()
