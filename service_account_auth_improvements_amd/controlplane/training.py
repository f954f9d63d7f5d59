"""PyTorchJob (kubeflow.org/v1) and MPIJob (kubeflow.org/v2beta1) operators -- the
north-star job CRDs.  API-compatible with the training-operator /
mpi-operator shapes, MI355X-native in what they put into pods:

* every replica pod runs ``kfamd-launch`` (native/src/kfamd_launch.cpp) which spawns one
  worker per GPU (``nprocPerNode``, default = the pod's ``amd.com/gpu`` limit), performs
  the node-level rendezvous and supervises worker health;
* per-replica env: ``MASTER_ADDR`` / ``MASTER_PORT`` (the master replica's headless
  Service), ``WORLD_SIZE`` / ``RANK`` (node-level, training-operator convention) and the
  ``PET_*`` torchrun variables consumed by the launcher, plus ``HSA_ENABLE_IPC_MODE_LEGACY=0``
  for RCCL's dmabuf IPC.  ``HIP_VISIBLE_DEVICES`` is set by the node's device plugin from
  the ``amd.com/gpu`` allocation -- no ``CUDA_VISIBLE_DEVICES`` / NVIDIA assumptions;
* status: ``Created`` / ``Running`` / ``Restarting`` / ``Suspended`` / ``Succeeded`` /
  ``Failed`` conditions, ``replicaStatuses``, ``startTime`` / ``completionTime``.
* ``runPolicy`` (kubeflow.org/v1 RunPolicy): ``backoffLimit`` (pod restarts for ``OnFailure``
  / ``ExitCode``), ``cleanPodPolicy``, ``activeDeadlineSeconds`` (counted from ``startTime``;
  past it the job is Failed with reason ``DeadlineExceeded`` and its running pods are
  deleted -- a deadline that left them running would not bound anything), ``ttlSecondsAfter
  Finished`` (the finished job is deleted, its pods and services with it through owner
  references) and ``suspend`` (pods and services deleted, job kept with ``Suspended``;
  un-suspending recreates them with a fresh ``startTime``).  ``schedulingPolicy`` needs a gang
  scheduler this platform does not run and is rejected at admission (:func:`validate_job`),
  as is anything else the operator would otherwise silently ignore.
* PyTorchJob ``elasticPolicy``: ``minReplicas`` / ``maxReplicas`` / ``maxRestarts`` /
  ``rdzv*`` become the launcher's elastic rendezvous (``PET_NNODES=MIN:MAX``,
  ``PET_RDZV_ENDPOINT``, ``PET_MAX_RESTARTS``): when a node is lost the survivors restart and
  re-form the group at the smaller world size while at least ``minReplicas`` Workers remain;
  the job fails only below that.  HPA ``metrics`` are rejected at admission.
"""
from __future__ import annotations

import copy
import datetime as _dt
import logging
import os
import sys
import time
from typing import Dict, List, Optional

from .apiserver import ApiError, now_rfc3339, set_controller_reference
from .client import Client
from .runtime import Controller, Request, Result, for_kind, owns

log = logging.getLogger("training-operator")

PT_API, MPI_API = "kubeflow.org/v1", "kubeflow.org/v2beta1"
LBL_JOB = "training.kubeflow.org/job-name"
LBL_RTYPE = "training.kubeflow.org/replica-type"
LBL_RINDEX = "training.kubeflow.org/replica-index"
LBL_ROLE = "training.kubeflow.org/job-role"
DEFAULT_PORT = 23456
GPU = "amd.com/gpu"


def launcher_path() -> str:
    from ..native import binary
    return binary("kfamd_launch")


def _cond(ctype, reason, msg):
    t = now_rfc3339()
    return {"type": ctype, "status": "True", "reason": reason, "message": msg,
            "lastUpdateTime": t, "lastTransitionTime": t}


def _set_condition(status: dict, ctype: str, reason: str, msg: str):
    """Set condition ``ctype`` True (one entry per type, updated in place).  Running /
    Restarting / Suspended exclude each other and end at a terminal condition."""
    conds = status.setdefault("conditions", [])
    for c in conds:
        if c["type"] == ctype and c.get("status") == "True":
            return
    exclusive = {"Succeeded": ("Running", "Restarting"), "Failed": ("Running", "Restarting"),
                 "Running": ("Restarting",), "Restarting": ("Running",), "Suspended": ("Running", "Restarting")}
    t = now_rfc3339()
    for c in conds:
        if c["type"] in exclusive.get(ctype, ()) and c.get("status") == "True":
            c.update(status="False", lastUpdateTime=t, lastTransitionTime=t)
    for c in conds:
        if c["type"] == ctype:
            c.update(_cond(ctype, reason, msg))
            return
    conds.append(_cond(ctype, reason, msg))


def _has(status: dict, ctype: str) -> bool:
    return any(c["type"] == ctype and c.get("status") == "True" for c in status.get("conditions") or [])


def _parse_time(s: Optional[str]) -> Optional[float]:
    if not s:
        return None
    try:
        return _dt.datetime.fromisoformat(s.replace("Z", "+00:00")).timestamp()
    except ValueError:
        return None


def _elastic(job: dict) -> Optional[dict]:
    return job.get("spec", {}).get("elasticPolicy") if job.get("kind") == "PyTorchJob" else None


def _elastic_bounds(job: dict) -> tuple:
    """(minReplicas, maxReplicas) of an elastic PyTorchJob; both default to the Worker count."""
    ep = _elastic(job) or {}
    w = int(((job["spec"].get("pytorchReplicaSpecs") or {}).get("Worker") or {}).get("replicas", 1))
    mx = int(ep.get("maxReplicas") or w)
    return int(ep.get("minReplicas") or min(w, mx)), mx


def validate_job(job: dict) -> Optional[str]:
    """Admission check for PyTorchJob / MPIJob specs: what the operator cannot honour is refused
    here instead of being accepted and ignored (the training-operator validation webhook plus
    this platform's limits).  Returns the denial message, or None."""
    kind = job.get("kind")
    spec = job.get("spec") or {}
    key = "pytorchReplicaSpecs" if kind == "PyTorchJob" else "mpiReplicaSpecs"
    specs = spec.get(key) or {}
    if not specs:
        return f"{kind} needs spec.{key}"
    allowed = ("Master", "Worker") if kind == "PyTorchJob" else ("Launcher", "Worker")
    for rtype, rs in specs.items():
        if rtype not in allowed:
            return f"{kind} replica type {rtype!r} is not one of {', '.join(allowed)}"
        if not ((rs.get("template") or {}).get("spec") or {}).get("containers"):
            return f"{kind} {rtype} template needs at least one container"
    if kind == "PyTorchJob" and int((specs.get("Master") or {}).get("replicas", 1)) > 1:
        return "PyTorchJob Master replicas must be 1"
    if kind == "MPIJob" and int((specs.get("Launcher") or {}).get("replicas", 1)) != 1:
        return "MPIJob Launcher replicas must be 1"
    rp = spec.get("runPolicy") or {}
    if rp.get("schedulingPolicy"):
        return ("runPolicy.schedulingPolicy needs a gang scheduler (volcano / scheduler-plugins), which this "
                "platform does not run; remove it (pods are scheduled individually)")
    ep = spec.get("elasticPolicy")
    if ep is not None:
        if kind != "PyTorchJob":
            return "elasticPolicy is a PyTorchJob field"
        if ep.get("metrics"):
            return "elasticPolicy.metrics (HPA autoscaling of Workers) is not supported"
        if (ep.get("rdzvBackend") or "c10d") != "c10d":
            return f"elasticPolicy.rdzvBackend {ep.get('rdzvBackend')!r} is not supported (c10d only)"
        if "Master" in specs:
            return "an elastic PyTorchJob runs Worker replicas only (no Master)"
        if "Worker" not in specs:
            return "an elastic PyTorchJob needs Worker replicas"
        mn, mx = _elastic_bounds(job)
        w = int(specs["Worker"].get("replicas", 1))
        if mn > mx:
            return f"elasticPolicy.minReplicas {mn} > maxReplicas {mx}"
        if not mn <= w <= mx:
            return f"Worker replicas {w} outside elasticPolicy [{mn}, {mx}]"
    return None


def admission_review(request: dict) -> dict:
    """Validating webhook body (``/validate-kubeflow-org-v1-pytorchjob`` / ``-v2beta1-mpijob``)."""
    if request.get("operation") == "DELETE":
        return {"uid": request.get("uid"), "allowed": True}
    err = validate_job(request.get("object") or {})
    if err:
        return {"uid": request.get("uid"), "allowed": False,
                "status": {"code": 422, "reason": "Invalid", "message": err}}
    return {"uid": request.get("uid"), "allowed": True}


def register(server):
    from .apiserver import Webhook
    server.add_validating_webhook(Webhook("validator.pytorchjob.training-operator.kubeflow.org", "kubeflow.org",
                                          "PyTorchJob", ("CREATE", "UPDATE"), admission_review))
    server.add_validating_webhook(Webhook("validator.mpijob.training-operator.kubeflow.org", "kubeflow.org",
                                          "MPIJob", ("CREATE", "UPDATE"), admission_review))


def _gpus(tpl: dict) -> int:
    n = 0
    for c in tpl.get("spec", {}).get("containers") or []:
        v = ((c.get("resources") or {}).get("limits") or {}).get(GPU)
        n += int(v) if v else 0
    return n


class _JobBase(Controller):
    api = ""
    kind = ""
    specs_key = ""
    job_label_kind = ""

    def sources(self):
        return [for_kind(self.api, self.kind), owns("v1", "Pod", self.kind)]

    # --- pods / services
    def _replica_order(self, specs: dict) -> List[str]:
        raise NotImplementedError

    def _pod_env(self, job, rtype, index, specs, tpl) -> List[dict]:
        raise NotImplementedError

    def _desired_pods(self, job: dict) -> List[dict]:
        specs = job["spec"].get(self.specs_key) or {}
        name, ns = job["metadata"]["name"], job["metadata"]["namespace"]
        out = []
        for rtype in self._replica_order(specs):
            rs = specs[rtype]
            for i in range(int(rs.get("replicas", 1))):
                tpl = copy.deepcopy(rs["template"])
                pn = f"{name}-{rtype.lower()}-{i}"
                labels = dict(tpl.get("metadata", {}).get("labels") or {})
                labels.update({LBL_JOB: name, LBL_RTYPE: rtype.lower(), LBL_RINDEX: str(i)})
                if rtype in ("Master", "Launcher"):
                    labels[LBL_ROLE] = "master"
                spec = tpl.get("spec", {})
                restart = rs.get("restartPolicy", "OnFailure")
                spec["restartPolicy"] = "Never" if restart == "ExitCode" else (
                    "OnFailure" if restart == "OnFailure" else restart)
                env_add = self._pod_env(job, rtype, i, specs, tpl) + _worker_runtime_env(job)
                for c in spec.get("containers") or []:
                    if c.get("name") in ("pytorch", "mpi", "launcher", "worker") or len(spec["containers"]) == 1:
                        names = {e["name"] for e in c.get("env") or []}
                        c["env"] = list(c.get("env") or []) + [e for e in env_add if e["name"] not in names]
                ann = dict(tpl.get("metadata", {}).get("annotations") or {})
                ann.update(_scrape_annotations(job))
                pod = {"apiVersion": "v1", "kind": "Pod",
                       "metadata": {"name": pn, "namespace": ns, "labels": labels, "annotations": ann},
                       "spec": spec}
                out.append(set_controller_reference(job, pod))
        return out

    def _service(self, job, pod) -> dict:
        m = pod["metadata"]
        return set_controller_reference(job, {
            "apiVersion": "v1", "kind": "Service",
            "metadata": {"name": m["name"], "namespace": m["namespace"], "labels": dict(m["labels"])},
            "spec": {"clusterIP": "None", "selector": {LBL_JOB: m["labels"][LBL_JOB],
                                                       LBL_RTYPE: m["labels"][LBL_RTYPE],
                                                       LBL_RINDEX: m["labels"][LBL_RINDEX]},
                     "ports": [{"name": f"{self.kind.lower()}-port", "port": self._port(job)}]}})

    def _port(self, job) -> int:
        return int((job.get("metadata", {}).get("annotations") or {}).get("kfamd.io/master-port", DEFAULT_PORT))

    # --- reconcile
    def _delete_pods_and_services(self, pods: dict, ns: str, phases=None):
        c = self.client
        for p in pods.values():
            if phases is not None and p.get("status", {}).get("phase") not in phases:
                continue
            for kind in ("Pod", "Service"):
                try:
                    c.delete("v1", kind, p["metadata"]["name"], ns)
                except ApiError:
                    pass

    def reconcile(self, req: Request) -> Result:
        c = self.client
        job = c.get_or_none(self.api, self.kind, req.name, req.namespace)
        if job is None or job["metadata"].get("deletionTimestamp"):
            return Result()
        status = copy.deepcopy(job.get("status") or {})
        run_policy = job["spec"].get("runPolicy") or {}
        now = time.time()
        requeue = 0.0
        if not _has(status, "Created"):
            _set_condition(status, "Created", f"{self.kind}Created",
                           f'{self.kind} {req.name} is created.')
        terminal = _has(status, "Succeeded") or _has(status, "Failed")
        # runPolicy.ttlSecondsAfterFinished: the finished job goes (pods / services follow it
        # through their owner references)
        if terminal and run_policy.get("ttlSecondsAfterFinished") is not None:
            done_at = _parse_time(status.get("completionTime"))
            if done_at is not None:
                left = done_at + int(run_policy["ttlSecondsAfterFinished"]) - now
                if left <= 0:
                    try:
                        c.delete(self.api, self.kind, req.name, req.namespace)
                    except ApiError:
                        pass
                    return Result()
                requeue = left
        pods = {p["metadata"]["name"]: p for p in c.list("v1", "Pod", req.namespace,
                                                         label_selector=f"{LBL_JOB}={req.name}")}
        # runPolicy.suspend: no pods while suspended; resuming starts the clock again
        if run_policy.get("suspend") and not terminal:
            self._delete_pods_and_services(pods, req.namespace)
            if not _has(status, "Suspended"):
                _set_condition(status, "Suspended", f"{self.kind}Suspended", f"{self.kind} {req.name} is suspended.")
            status.pop("startTime", None)
            status["replicaStatuses"] = {rt: {"active": 0, "succeeded": 0, "failed": 0}
                                         for rt in (job["spec"].get(self.specs_key) or {})}
            self._write_status(job, status)
            return Result()
        if _has(status, "Suspended"):
            for cd in status["conditions"]:
                if cd["type"] == "Suspended" and cd.get("status") == "True":
                    cd.update(status="False", reason=f"{self.kind}Resumed", message=f"{self.kind} {req.name} is resumed.",
                              lastUpdateTime=now_rfc3339(), lastTransitionTime=now_rfc3339())
        desired = self._desired_pods(job)
        if not terminal:
            for pod in desired:
                pn = pod["metadata"]["name"]
                if pn not in pods:
                    pods[pn] = c.create(pod)
                if c.get_or_none("v1", "Service", pn, req.namespace) is None and self._wants_service(pod):
                    c.create(self._service(job, pod))
            status.setdefault("startTime", now_rfc3339())
        # replica statuses
        rstat: Dict[str, dict] = {}
        restarts = int(status.get("restartCount", 0))
        per_type = dict(status.get("replicaRestarts") or {})
        backoff = run_policy.get("backoffLimit")
        failed_msg = None
        specs = job["spec"].get(self.specs_key) or {}
        for pod in desired:
            rtype = next(k for k in specs if k.lower() == pod["metadata"]["labels"][LBL_RTYPE])
            live = pods.get(pod["metadata"]["name"])
            rs = rstat.setdefault(rtype, {"active": 0, "succeeded": 0, "failed": 0})
            phase = (live or {}).get("status", {}).get("phase")
            if phase == "Succeeded":
                rs["succeeded"] += 1
            elif phase == "Failed":
                policy = self._restart_policy(job, rtype, specs)
                code = self._exit_code(live)
                retryable = policy == "OnFailure" or (policy == "ExitCode" and code is not None and code >= 128)
                limit = self._backoff_limit(rtype, backoff)
                used = self._restarts_used(rtype, restarts, per_type)
                if retryable and not terminal and (limit is None or used < int(limit)):
                    restarts += 1
                    per_type[rtype] = per_type.get(rtype, 0) + 1
                    c.delete("v1", "Pod", live["metadata"]["name"], req.namespace)
                    _set_condition(status, "Restarting", f"{self.kind}Restarting",
                                   f'{self.kind} {req.name} is restarting because {rtype} replica(s) failed.')
                    rs["active"] += 1
                else:
                    rs["failed"] += 1
                    msg = self._failure_message(job, rtype, live)
                    if msg:
                        failed_msg = msg
            elif phase in ("Running", "Pending", None) and live is not None:
                rs["active"] += 1
        status["replicaStatuses"] = rstat
        status["restartCount"] = restarts
        if per_type:
            status["replicaRestarts"] = per_type
        if not terminal:
            failed_msg = failed_msg or self._job_failure(job, rstat)
            # runPolicy.activeDeadlineSeconds, counted from startTime
            ads = run_policy.get("activeDeadlineSeconds")
            started = _parse_time(status.get("startTime"))
            deadline_hit = False
            if ads is not None and started is not None and not failed_msg:
                left = started + int(ads) - now
                if left <= 0:
                    deadline_hit = True
                else:
                    requeue = min(requeue, left) if requeue else left
            if deadline_hit:
                _set_condition(status, "Failed", "DeadlineExceeded",
                               f"{self.kind} {req.name} is active more than {int(ads)} seconds.")
                status["completionTime"] = now_rfc3339()
                self._delete_pods_and_services(pods, req.namespace, phases=("Running", "Pending", None))
            elif failed_msg:
                _set_condition(status, "Failed", f"{self.kind}Failed", failed_msg)
                status["completionTime"] = now_rfc3339()
            elif self._succeeded(job, rstat, specs):
                _set_condition(status, "Succeeded", f"{self.kind}Succeeded",
                               f'{self.kind} {req.name} is successfully completed.')
                status["completionTime"] = now_rfc3339()
            elif self._running(pods, rstat):
                if not _has(status, "Running"):
                    _set_condition(status, "Running", f"{self.kind}Running", f'{self.kind} {req.name} is running.')
            if (_has(status, "Succeeded") or _has(status, "Failed")) and run_policy.get("ttlSecondsAfterFinished") is not None:
                requeue = max(0.05, float(run_policy["ttlSecondsAfterFinished"]))
        if _has(status, "Succeeded") or _has(status, "Failed"):
            clean = run_policy.get("cleanPodPolicy", "None")
            for p in pods.values():
                ph = p.get("status", {}).get("phase")
                if clean == "All" or (clean == "Running" and ph in ("Running", "Pending")):
                    try:
                        c.delete("v1", "Pod", p["metadata"]["name"], req.namespace)
                    except ApiError:
                        pass
        self._write_status(job, status)
        return Result(requeue_after=requeue) if requeue > 0 else Result()

    def _write_status(self, job: dict, status: dict):
        if status != (job.get("status") or {}):
            job["status"] = status
            self.client.update_status(job)

    def _restarts_used(self, rtype: str, total: int, per_type: dict) -> int:
        """Restarts counted against ``rtype``'s backoff limit (job-wide, as the training
        operator counts them)."""
        return total

    def _job_failure(self, job: dict, rstat: dict) -> Optional[str]:
        """A job-level failure decided from the replica counts (elastic PyTorchJobs), or None."""
        return None

    def _restart_policy(self, job, rtype, specs) -> str:
        return specs[rtype].get("restartPolicy", "OnFailure")

    def _backoff_limit(self, rtype: str, backoff):
        """How many restarts ``runPolicy.backoffLimit`` allows a replica of this type (None =
        unlimited)."""
        return backoff

    def _failure_message(self, job: dict, rtype: str, pod: dict) -> Optional[str]:
        """The Failed condition's message when a non-retried ``rtype`` pod failing ends the job,
        or None when that failure does not decide the job."""
        return f'{self.kind} {job["metadata"]["name"]} has failed because {rtype} replica(s) failed.'

    def _running(self, pods: dict, rstat: dict) -> bool:
        return any(p.get("status", {}).get("phase") == "Running" for p in pods.values())

    @staticmethod
    def _exit_code(pod):
        for cs in (pod or {}).get("status", {}).get("containerStatuses") or []:
            t = (cs.get("state") or {}).get("terminated")
            if t:
                return int(t.get("exitCode", 1))
        return None

    def _wants_service(self, pod) -> bool:
        return True

    def _succeeded(self, job, rstat, specs) -> bool:
        raise NotImplementedError


class PyTorchJobReconciler(_JobBase):
    name = "pytorchjob-controller"
    api, kind, specs_key = PT_API, "PyTorchJob", "pytorchReplicaSpecs"

    def _replica_order(self, specs):
        return [k for k in ("Master", "Worker") if k in specs]

    def _nproc(self, job, tpl) -> int:
        v = job["spec"].get("nprocPerNode")
        ep = _elastic(job) or {}
        if v is None and ep.get("nProcPerNode"):
            v = ep["nProcPerNode"]
        if v in (None, "auto", "gpu"):
            return max(1, _gpus(tpl))
        return int(v)

    def _pod_env(self, job, rtype, index, specs, tpl):
        name = job["metadata"]["name"]
        master = f"{name}-master-0" if "Master" in specs else f"{name}-worker-0"
        nnodes = sum(int(s.get("replicas", 1)) for s in specs.values())
        rank = index if rtype == "Master" else index + (1 if "Master" in specs else 0)
        port = self._port(job)
        nproc = self._nproc(job, tpl)
        env = [{"name": "MASTER_ADDR", "value": master}, {"name": "MASTER_PORT", "value": str(port)},
               {"name": "WORLD_SIZE", "value": str(nnodes)}, {"name": "RANK", "value": str(rank)},
               {"name": "PET_MASTER_ADDR", "value": master}, {"name": "PET_MASTER_PORT", "value": str(port)},
               {"name": "PET_NNODES", "value": str(nnodes)}, {"name": "PET_NODE_RANK", "value": str(rank)},
               {"name": "PET_NPROC_PER_NODE", "value": str(nproc)},
               {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
               {"name": "PYTHONUNBUFFERED", "value": "1"}]
        ep = _elastic(job)
        if ep is not None:
            # elastic rendezvous (kfamd-launch --nnodes MIN:MAX, hosted by worker 0's agent)
            mn, mx = _elastic_bounds(job)
            host = ep.get("rdzvHost") or master
            rport = int(ep.get("rdzvPort") or port + 1)
            over = {"PET_NNODES": f"{mn}:{mx}", "PET_RDZV_BACKEND": ep.get("rdzvBackend") or "c10d",
                    "PET_RDZV_ENDPOINT": f"{host}:{rport}", "PET_RDZV_ID": ep.get("rdzvId") or name,
                    "PET_MAX_RESTARTS": str(int(ep.get("maxRestarts") or 0))}
            for kv in ep.get("rdzvConf") or []:
                if kv.get("key") == "last_call_timeout":
                    over["KFAMD_RDZV_LAST_CALL"] = str(kv.get("value"))
                elif kv.get("key") == "join_timeout":       # torch elastic's name: how long an
                    over["KFAMD_RDZV_TIMEOUT"] = str(kv.get("value"))   # agent waits for a round
            env = [e for e in env if e["name"] not in over] + [{"name": k, "value": v} for k, v in over.items()]
        return env

    def _failure_message(self, job, rtype, pod):
        if _elastic(job) is not None and rtype == "Worker":
            return None          # decided by _job_failure: only below minReplicas
        return super()._failure_message(job, rtype, pod)

    def _job_failure(self, job, rstat):
        if _elastic(job) is None:
            return None
        w = rstat.get("Worker", {})
        mn, _ = _elastic_bounds(job)
        if w.get("failed", 0) and w.get("active", 0) + w.get("succeeded", 0) < mn:
            return (f'PyTorchJob {job["metadata"]["name"]} has failed because fewer than minReplicas={mn} '
                    f'Worker replicas remain ({w.get("failed", 0)} failed).')
        return None

    def _succeeded(self, job, rstat, specs):
        if _elastic(job) is not None:      # elastic: the surviving group finished
            w = rstat.get("Worker", {})
            return w.get("succeeded", 0) >= 1 and w.get("active", 0) == 0
        if "Master" in specs:
            return rstat.get("Master", {}).get("succeeded", 0) >= int(specs["Master"].get("replicas", 1))
        w = specs.get("Worker", {})
        return rstat.get("Worker", {}).get("succeeded", 0) >= int(w.get("replicas", 1))


class MPIJobReconciler(_JobBase):
    """MPIJob v2beta1: Launcher + Workers.  Workers run a kfamd-launch agent each (node
    rank = replica index); the Launcher runs node 0's agent over the job's hostfile.
    A ConfigMap ``<job>-config`` carries the ``hostfile`` (``slotsPerWorker`` slots each),
    as mpi-operator does.

    A Launcher whose command is ``mpirun ... program`` (upstream-style MPIJobs, workers running
    ``sshd``) is translated when the pods are built (``controlplane/mpi.py``): each Worker runs
    the program under kfamd-launch with mpirun's rank layout and ``-x`` exports, and the
    Launcher runs ``mpi-wait`` (mpirun's exit semantics over the Worker pods) under its own
    ServiceAccount with a read-only pods Role."""
    name = "mpijob-controller"
    api, kind, specs_key = MPI_API, "MPIJob", "mpiReplicaSpecs"

    @staticmethod
    def _main_container(tpl: dict) -> Optional[dict]:
        cs = tpl.get("spec", {}).get("containers") or []
        for c in cs:
            if c.get("name") in ("mpi", "launcher", "worker"):
                return c
        return cs[0] if cs else None

    def _mpirun(self, job) -> Optional[tuple]:
        """(MpirunSpec, ranks per worker, launcher container) when the Launcher runs mpirun."""
        from . import mpi
        specs = job["spec"].get(self.specs_key) or {}
        lt = (specs.get("Launcher") or {}).get("template") or {}
        lc = self._main_container(lt)
        argv = mpi.container_argv(lc) if lc else []
        if not mpi.is_mpirun(argv):
            return None
        sp = mpi.parse_mpirun(argv)
        workers = int((specs.get("Worker") or {}).get("replicas", 0))
        slots = int(job["spec"].get("slotsPerWorker", 1))
        return sp, mpi.rank_layout(sp, workers, slots), lc

    def _desired_pods(self, job: dict) -> List[dict]:
        pods = super()._desired_pods(job)
        try:
            mr = self._mpirun(job)
        except ValueError as e:
            log.warning("MPIJob %s: %s", job["metadata"]["name"], e)
            return pods
        if mr is None:
            return pods
        from . import mpi
        sp, layout, lc = mr
        name, ns = job["metadata"]["name"], job["metadata"]["namespace"]
        active = sum(1 for c in layout if c > 0)
        exports = mpi.export_env(sp, lc.get("env") or [])
        for pod in pods:
            rtype = pod["metadata"]["labels"][LBL_RTYPE]
            c = self._main_container({"spec": pod["spec"]})
            if rtype == "worker":
                pod["spec"]["restartPolicy"] = "Never"
                i = int(pod["metadata"]["labels"][LBL_RINDEX])
                if layout[i] == 0:            # more workers than mpirun places ranks on
                    c["command"], c["args"] = ["true"], []
                    continue
                # master address / port come from the PET_MASTER_* env (worker 0's Service)
                c["command"] = ["kfamd-launch", "--nnodes", str(active), "--node-rank", str(i),
                                "--nproc-per-node", str(layout[i]), "--"] + list(sp.program)
                c["args"] = []
                names = {e["name"] for e in c.get("env") or []}
                c["env"] = list(c.get("env") or []) + [e for e in exports if e["name"] not in names]
            elif rtype == "launcher":
                c["command"] = ["python3", "-m", "service_account_auth_improvements_amd", "mpi-wait",
                                "--job", name, "--namespace", ns, "--workers", str(active)]
                c["args"] = []
                pod["spec"]["serviceAccountName"] = f"{name}-launcher"
        return pods

    def _restart_policy(self, job, rtype, specs) -> str:
        # mpirun semantics: a failed rank fails the run (the Launcher's mpi-wait reports it and
        # the Launcher's own policy / backoffLimit decide); workers are not restarted behind it
        if rtype == "Worker":
            try:
                if self._mpirun(job) is not None:
                    return "Never"
            except ValueError:
                pass
        return super()._restart_policy(job, rtype, specs)

    def _launcher_rbac(self, job: dict):
        """ServiceAccount + Role (get/list/watch pods) + RoleBinding for the mpi-wait launcher."""
        name, ns = job["metadata"]["name"], job["metadata"]["namespace"]
        sa = f"{name}-launcher"
        objs = [
            {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": sa, "namespace": ns}},
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": sa, "namespace": ns},
             "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "list", "watch"]}]},
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
             "metadata": {"name": sa, "namespace": ns},
             "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": sa},
             "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": ns}]}]
        for o in objs:
            if self.client.get_or_none(o["apiVersion"], o["kind"], sa, ns) is None:
                self.client.create(set_controller_reference(job, o))

    def _replica_order(self, specs):
        return [k for k in ("Launcher", "Worker") if k in specs]

    def _pod_env(self, job, rtype, index, specs, tpl):
        name = job["metadata"]["name"]
        slots = int(job["spec"].get("slotsPerWorker", 1))
        nworkers = int(specs.get("Worker", {}).get("replicas", 0))
        port = self._port(job)
        base = [{"name": "OMPI_MCA_orte_default_hostfile", "value": "/etc/mpi/hostfile"},
                {"name": "K_MPI_JOB_ROLE", "value": rtype.lower()},
                {"name": "PET_MASTER_ADDR", "value": f"{name}-worker-0"},
                {"name": "PET_MASTER_PORT", "value": str(port)},
                {"name": "PET_NNODES", "value": str(max(nworkers, 1))},
                {"name": "PET_NPROC_PER_NODE", "value": str(slots)},
                {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
                {"name": "PYTHONUNBUFFERED", "value": "1"}]
        if rtype == "Worker":
            base.append({"name": "PET_NODE_RANK", "value": str(index)})
        return base

    def reconcile(self, req: Request) -> Result:
        job = self.client.get_or_none(self.api, self.kind, req.name, req.namespace)
        if job is not None and not job["metadata"].get("deletionTimestamp"):
            specs = job["spec"].get(self.specs_key) or {}
            slots = int(job["spec"].get("slotsPerWorker", 1))
            hosts = "".join(f"{req.name}-worker-{i}.{req.name}.{req.namespace}.svc slots={slots}\n"
                            for i in range(int(specs.get("Worker", {}).get("replicas", 0))))
            cm = set_controller_reference(job, {"apiVersion": "v1", "kind": "ConfigMap",
                                                "metadata": {"name": f"{req.name}-config", "namespace": req.namespace},
                                                "data": {"hostfile": hosts}})
            cur = self.client.get_or_none("v1", "ConfigMap", cm["metadata"]["name"], req.namespace)
            if cur is None:
                self.client.create(cm)
            elif cur.get("data") != cm["data"]:
                cur["data"] = cm["data"]
                self.client.update(cur)
            try:
                if self._mpirun(job) is not None:
                    self._launcher_rbac(job)
            except ValueError:
                pass
        return super().reconcile(req)

    def _wants_service(self, pod):
        return pod["metadata"]["labels"][LBL_RTYPE] == "worker"

    def _succeeded(self, job, rstat, specs):
        return rstat.get("Launcher", {}).get("succeeded", 0) >= 1

    # --- mpi-operator v2beta1 outcome semantics (pkg/controller/mpi_job_controller.go
    # updateMPIJobStatus): the Launcher decides the job.  It runs as a batch Job whose
    # backoffLimit is runPolicy.backoffLimit (the batch default, 6, when unset); a Worker that
    # fails is counted in replicaStatuses but reaches the job only through the Launcher's exit
    # code (mpirun / mpi-wait sees the rank die) -- except an evicted Worker, which fails the job.
    BATCH_BACKOFF_DEFAULT = 6

    def _backoff_limit(self, rtype, backoff):
        if rtype == "Launcher":
            return self.BATCH_BACKOFF_DEFAULT if backoff is None else backoff
        return backoff

    def _restarts_used(self, rtype, total, per_type):
        # the Launcher's batch Job counts its own failures only: Worker restarts (OnFailure
        # Workers without an mpirun Launcher) do not use up the Launcher's retries
        return per_type.get(rtype, 0) if rtype == "Launcher" else total

    def _failure_message(self, job, rtype, pod):
        name = job["metadata"]["name"]
        if rtype == "Launcher":
            return f"MPIJob {name} has failed because the launcher failed."
        if (pod.get("status") or {}).get("reason") == "Evicted":
            return f"MPIJob {name} has failed because a worker was evicted."
        return None

    def _running(self, pods, rstat):
        """Running once the Launcher runs and every Worker has started (upstream: launcher
        active and all workers Running; a Worker mpirun placed no rank on exits at once)."""
        phases = {p["metadata"]["labels"].get(LBL_RTYPE): [] for p in pods.values()}
        for p in pods.values():
            phases[p["metadata"]["labels"].get(LBL_RTYPE)].append(p.get("status", {}).get("phase"))
        return ("Running" in phases.get("launcher", []) and
                all(ph in ("Running", "Succeeded") for ph in phases.get("worker", [])))


# job annotations the operator turns into worker-runtime settings (runtime/train_entry.py):
#   kfamd.io/metrics-port    -> KFAMD_METRICS_PORT (rank 0 serves Prometheus /metrics there) and
#                               the prometheus.io/{scrape,port,path} pod annotations
#   kfamd.io/checkpoint-dir  -> KFAMD_CKPT_DIR (periodic checkpoints + auto-resume; a PVC path)
#   kfamd.io/save-every      -> KFAMD_SAVE_EVERY (steps between checkpoints)
ANN_METRICS_PORT = "kfamd.io/metrics-port"
ANN_CKPT_DIR = "kfamd.io/checkpoint-dir"
ANN_SAVE_EVERY = "kfamd.io/save-every"


def _worker_runtime_env(job: dict) -> List[dict]:
    ann = job.get("metadata", {}).get("annotations") or {}
    env = []
    for key, var in ((ANN_METRICS_PORT, "KFAMD_METRICS_PORT"), (ANN_CKPT_DIR, "KFAMD_CKPT_DIR"),
                     (ANN_SAVE_EVERY, "KFAMD_SAVE_EVERY")):
        if ann.get(key) not in (None, ""):
            env.append({"name": var, "value": str(ann[key])})
    return env


def _scrape_annotations(job: dict) -> dict:
    port = (job.get("metadata", {}).get("annotations") or {}).get(ANN_METRICS_PORT)
    if port in (None, ""):
        return {}
    return {"prometheus.io/scrape": "true", "prometheus.io/port": str(port), "prometheus.io/path": "/metrics"}


def pytorchjob_manifest(name: str, namespace: str, image: str, command: List[str], n_nodes: int = 1,
                        gpus_per_node: int = 8, master_port: Optional[int] = None,
                        restart_policy: str = "OnFailure", backoff_limit: int = 3,
                        metrics_port: Optional[int] = None, ckpt_dir: Optional[str] = None,
                        save_every: Optional[int] = None) -> dict:
    """A PyTorchJob for the kfamd trainer: each replica runs kfamd-launch over its GPUs.
    ``metrics_port`` / ``ckpt_dir`` / ``save_every`` become the job annotations above."""
    def tpl():
        return {"metadata": {"annotations": {"sidecar.istio.io/inject": "false"}},
                "spec": {"containers": [{"name": "pytorch", "image": image,
                                         "command": [launcher_path(), "--"] + list(command),
                                         "resources": {"limits": {GPU: str(gpus_per_node)}} if gpus_per_node else {}}]}}
    specs = {"Master": {"replicas": 1, "restartPolicy": restart_policy, "template": tpl()}}
    if n_nodes > 1:
        specs["Worker"] = {"replicas": n_nodes - 1, "restartPolicy": restart_policy, "template": tpl()}
    ann = {"kfamd.io/master-port": str(master_port)} if master_port else {}
    for key, v in ((ANN_METRICS_PORT, metrics_port), (ANN_CKPT_DIR, ckpt_dir), (ANN_SAVE_EVERY, save_every)):
        if v is not None:
            ann[key] = str(v)
    return {"apiVersion": PT_API, "kind": "PyTorchJob",
            "metadata": {"name": name, "namespace": namespace, "annotations": ann},
            "spec": {"nprocPerNode": str(gpus_per_node) if gpus_per_node else "1",
                     "runPolicy": {"backoffLimit": backoff_limit, "cleanPodPolicy": "None"},
                     "pytorchReplicaSpecs": specs}}


def mpijob_manifest(name: str, namespace: str, image: str, program: List[str], workers: int = 1,
                    gpus_per_worker: int = 8, master_port: Optional[int] = None) -> dict:
    """An MPIJob in the upstream mpi-operator shape: the Launcher runs ``mpirun -np N program``
    over the hostfile, the Workers run sshd (N = workers x slots).  The operator translates it
    (see MPIJobReconciler / controlplane/mpi.py)."""
    slots = max(gpus_per_worker, 1)
    wc = {"name": "worker", "image": image, "command": ["/usr/sbin/sshd", "-De"]}
    if gpus_per_worker:
        wc["resources"] = {"limits": {GPU: str(gpus_per_worker)}}
    lc = {"name": "launcher", "image": image,
          "command": ["mpirun", "--allow-run-as-root", "-np", str(workers * slots)] + list(program)}
    ann = {"kfamd.io/master-port": str(master_port)} if master_port else {}
    return {"apiVersion": MPI_API, "kind": "MPIJob",
            "metadata": {"name": name, "namespace": namespace, "annotations": ann},
            "spec": {"slotsPerWorker": slots, "runPolicy": {"cleanPodPolicy": "None"},
                     "mpiReplicaSpecs": {"Launcher": {"replicas": 1, "template": {"spec": {"containers": [lc]}}},
                                         "Worker": {"replicas": workers,
                                                    "template": {"spec": {"containers": [wc]}}}}}}
