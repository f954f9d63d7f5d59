"""Pod scheduler for multi-node local clusters (the kube-scheduler role of SURVEY.md §2.4 M3's
KinD harness: the reference's integration jobs run on a real cluster whose scheduler places
the job pods; here several node agents share one API server, so something has to).

Binds every pending, unbound pod to one node through the ``pods/binding`` subresource,
exactly what kube-scheduler does.  The plugin set is the one a GPU training cluster needs:

* filter -- ``spec.unschedulable`` nodes are skipped, ``nodeSelector`` must match the node's
  labels, ``NoSchedule`` / ``NoExecute`` taints need a matching toleration, and the node's
  allocatable ``amd.com/gpu`` minus the GPUs of the pods already bound there (and not finished)
  must cover the pod's request;
* score -- GPU pods go to the MOST allocated fitting node (bin-packing keeps whole 8-GPU
  nodes free for 8-GPU ranks; kube-scheduler's ``MostAllocated`` strategy for extended
  resources), CPU-only pods to the node running the fewest pods; ties break by node name;
* no fit -- the pod gets ``PodScheduled=False / Unschedulable`` with kube-scheduler's message
  form ("0/N nodes are available: ...") and is retried when a node changes or a pod finishes.

Bindings made but not yet visible in this scheduler's (informer-cached) view are kept in an
assume cache, so two pods reconciled back to back never over-commit a node.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Tuple

from .apiserver import ApiError, now_rfc3339
from .client import Client
from .kubelet import GPU_RESOURCE, pod_gpu_request
from .runtime import Controller, Request, Result, for_kind, watches

SCHEDULER_NAME = "default-scheduler"


def _unbound_pending(et, obj) -> bool:
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    return (not spec.get("nodeName") and st.get("phase") in (None, "", "Pending")
            and spec.get("schedulerName", SCHEDULER_NAME) == SCHEDULER_NAME)


def _tolerated(taint: dict, tolerations: List[dict]) -> bool:
    for t in tolerations or []:
        if t.get("effect") and t["effect"] != taint.get("effect"):
            continue
        if t.get("operator") == "Exists":
            if not t.get("key") or t["key"] == taint.get("key"):
                return True
        elif t.get("key") == taint.get("key") and t.get("value", "") == taint.get("value", ""):
            return True
    return False


class Scheduler(Controller):
    name = "kube-scheduler"

    def __init__(self, client: Client):
        super().__init__(client)
        self._lock = threading.Lock()
        self._assumed: Dict[str, Tuple[str, int]] = {}     # pod uid -> (node, gpus)

    def sources(self):
        def pending_pods(et, obj):
            # a node appearing / changing, or a pod finishing, can make room: retry every pending pod
            return [Request(p["metadata"]["namespace"], p["metadata"]["name"])
                    for p in self.client.list("v1", "Pod") if _unbound_pending("", p)]

        def finished(et, obj):
            ph = (obj.get("status") or {}).get("phase")
            return et == "DELETED" or ph in ("Succeeded", "Failed")

        return [for_kind("v1", "Pod", predicate=_unbound_pending),
                watches("v1", "Node", pending_pods),
                watches("v1", "Pod", pending_pods, predicate=finished)]

    # ------------------------------------------------------------------ accounting
    def _used(self, pods: List[dict]) -> Tuple[Dict[str, int], Dict[str, int]]:
        """-> (GPUs in use, running pod count) per node, assumed bindings included."""
        used: Dict[str, int] = {}
        count: Dict[str, int] = {}
        seen_bound = set()
        for p in pods:
            node = (p.get("spec") or {}).get("nodeName")
            if not node:
                continue
            seen_bound.add(p["metadata"].get("uid"))      # the view has the binding: drop the assumption
            if (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                continue
            used[node] = used.get(node, 0) + pod_gpu_request(p)
            count[node] = count.get(node, 0) + 1
        live = {p["metadata"].get("uid") for p in pods}
        for uid in list(self._assumed):
            if uid in seen_bound or uid not in live:
                del self._assumed[uid]           # the cache caught up (or the pod is gone)
                continue
            node, g = self._assumed[uid]
            used[node] = used.get(node, 0) + g
            count[node] = count.get(node, 0) + 1
        return used, count

    @staticmethod
    def _fits_static(pod: dict, node: dict) -> Optional[str]:
        spec = pod.get("spec") or {}
        nspec, labels = node.get("spec") or {}, node["metadata"].get("labels") or {}
        if nspec.get("unschedulable"):
            return "node(s) were unschedulable"
        for k, v in (spec.get("nodeSelector") or {}).items():
            if labels.get(k) != v:
                return "node(s) didn't match Pod's node affinity/selector"
        for taint in nspec.get("taints") or []:
            if taint.get("effect") in ("NoSchedule", "NoExecute") and not _tolerated(taint, spec.get("tolerations")):
                return "node(s) had untolerated taint"
        return None

    # ------------------------------------------------------------------ reconcile
    def reconcile(self, req: Request) -> Result:
        c = self.client
        pod = c.get_or_none("v1", "Pod", req.name, req.namespace)
        if pod is None or pod["metadata"].get("deletionTimestamp") or not _unbound_pending("", pod):
            return Result()
        need = pod_gpu_request(pod)
        with self._lock:
            nodes = sorted(c.list("v1", "Node"), key=lambda n: n["metadata"]["name"])
            used, count = self._used(c.list("v1", "Pod"))
            reasons: Dict[str, int] = {}
            fits = []
            for n in nodes:
                why = self._fits_static(pod, n)
                alloc = int(((n.get("status") or {}).get("allocatable") or {}).get(GPU_RESOURCE, 0) or 0)
                free = alloc - used.get(n["metadata"]["name"], 0)
                if why is None and free < need:
                    why = f"Insufficient {GPU_RESOURCE}"
                if why:
                    reasons[why] = reasons.get(why, 0) + 1
                else:
                    fits.append((n, alloc, free))
            if not fits:
                detail = ", ".join(f"{v} {k}" for k, v in sorted(reasons.items()))
                msg = f"0/{len(nodes)} nodes are available: {detail}." if nodes else "no nodes available to schedule pods"
                self._mark_unschedulable(pod, msg)
                return Result(requeue_after=1.0)
            pods_on = lambda f: count.get(f[0]["metadata"]["name"], 0)  # noqa: E731
            if need > 0:
                node = min(fits, key=lambda f: (f[2] - need, f[0]["metadata"]["name"]))[0]
            else:
                node = min(fits, key=lambda f: (pods_on(f), -f[2], f[0]["metadata"]["name"]))[0]
            name = node["metadata"]["name"]
            try:
                c.bind(pod["metadata"]["namespace"], pod["metadata"]["name"], name)
            except ApiError as e:
                if e.code == 409:          # bound meanwhile (by another scheduler or a retry)
                    return Result()
                raise
            self._assumed[pod["metadata"]["uid"]] = (name, need)
        c.record_event(pod, "Normal", "Scheduled",
                       f'Successfully assigned {pod["metadata"]["namespace"]}/{pod["metadata"]["name"]} to {name}',
                       source=SCHEDULER_NAME)
        return Result()

    def _mark_unschedulable(self, pod: dict, msg: str):
        st = dict(pod.get("status") or {})
        conds = [x for x in st.get("conditions") or [] if x.get("type") != "PodScheduled"]
        conds.append({"type": "PodScheduled", "status": "False", "reason": "Unschedulable", "message": msg,
                      "lastTransitionTime": now_rfc3339()})
        if st.get("conditions") and any(x.get("type") == "PodScheduled" and x.get("message") == msg
                                        for x in st["conditions"]):
            return
        st.update({"phase": "Pending", "conditions": conds})
        pod = dict(pod, status=st)
        try:
            self.client.update_status(pod)
        except ApiError:
            pass
