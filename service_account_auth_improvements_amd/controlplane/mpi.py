"""MPIJob launcher semantics without remote execution (SURVEY.md §2.9 "MPIJob CRD +
controller"; BASELINE configs[4]; upstream mpi-operator v2beta1).

Upstream, the Launcher pod runs ``mpirun ... program``; mpirun reads the hostfile ConfigMap and
starts the ranks on the Worker pods over ssh (the workers run ``sshd``).  Here nothing executes
commands received over the network.  The operator reads the Launcher's ``mpirun`` command line
when it builds the pods, and:

* every Worker pod runs the program itself under ``kfamd-launch`` (one process per slot / GPU,
  TCP rendezvous hosted by worker 0, the same agent as PyTorchJob replicas), with the rank
  layout mpirun would produce: ``-np N`` fills the hostfile's slots in order
  (``slotsPerWorker`` each), ``-npernode P`` / ``--map-by ppr:P:node`` places P per worker,
  ``-x VAR[=value]`` exports reach every rank (a bare ``VAR`` takes the Launcher container's
  value);
* the Launcher pod runs ``kfamd mpi-wait``: it follows the Worker pods through the API server
  (its own ServiceAccount with a read-only Role on pods, as mpi-operator gives its launcher)
  and exits like mpirun -- 0 once every worker succeeded, the first failing worker's exit code
  otherwise -- so the job's success stays the Launcher's, as upstream.

The commands therefore come only from the MPIJob's pod templates through the Kubernetes API and
its RBAC, exactly like a PyTorchJob's.
"""
from __future__ import annotations

import argparse
import os
import shlex
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

MPIRUN_NAMES = ("mpirun", "mpiexec", "orterun")
# mpirun options that take one value and do not change the rank layout
_ONE_ARG = {"--bind-to", "-bind-to", "--rank-by", "-rank-by", "--mca-param-file", "--prefix", "-prefix",
            "--output-filename", "-output-filename", "--report-bindings-file", "-wdir", "--wdir", "-cwd",
            "--cwd"}
_TWO_ARGS = {"--mca", "-mca", "--gmca", "-gmca"}
_FLAGS = {"--allow-run-as-root", "--oversubscribe", "-oversubscribe", "--tag-output", "-tag-output",
          "--report-bindings", "-report-bindings", "--display-map", "-display-map", "-v", "--verbose",
          "--timestamp-output", "--merge-stderr-to-stdout", "--quiet", "-q", "--nooversubscribe"}


@dataclass
class MpirunSpec:
    np: Optional[int] = None
    npernode: Optional[int] = None
    exports: List[str] = field(default_factory=list)
    program: List[str] = field(default_factory=list)


def is_mpirun(argv: List[str]) -> bool:
    return bool(argv) and os.path.basename(argv[0]) in MPIRUN_NAMES


def parse_mpirun(argv: List[str]) -> MpirunSpec:
    """The rank-layout-relevant subset of an OpenMPI ``mpirun`` command line."""
    if not is_mpirun(argv):
        raise ValueError(f"not an mpirun command: {argv[:1]}")
    sp = MpirunSpec()
    i, n = 1, len(argv)

    def val():
        nonlocal i
        if i + 1 >= n:
            raise ValueError(f"mpirun option {argv[i]} needs a value")
        i += 1
        return argv[i]
    while i < n:
        a = argv[i]
        if a in ("-np", "-n", "--np", "-c"):
            sp.np = int(val())
        elif a in ("-npernode", "--npernode", "-N"):
            sp.npernode = int(val())
        elif a in ("--map-by", "-map-by"):
            m = val()
            if m.startswith("ppr:") and m.endswith(":node"):
                sp.npernode = int(m.split(":")[1])
        elif a == "-x":
            sp.exports.append(val())
        elif a in ("--hostfile", "-hostfile", "--machinefile", "-machinefile", "-H", "--host", "-host"):
            val()                       # the operator's hostfile / worker list is authoritative
        elif a in _TWO_ARGS:
            val()
            val()
        elif a in _ONE_ARG:
            val()
        elif a in _FLAGS:
            pass
        elif a == "--":
            i += 1
            break
        elif a.startswith("-"):
            raise ValueError(f"unsupported mpirun option {a}")
        else:
            break
        i += 1
    sp.program = list(argv[i:])
    if not sp.program:
        raise ValueError("mpirun command without a program")
    return sp


def rank_layout(sp: MpirunSpec, workers: int, slots: int) -> List[int]:
    """Ranks per worker, as mpirun places them on a hostfile of ``workers`` x ``slots``."""
    if workers < 1:
        raise ValueError("an MPIJob with mpirun needs at least one Worker")
    if sp.npernode:
        if sp.np is not None and sp.np != sp.npernode * workers:
            raise ValueError(f"-np {sp.np} does not match {workers} workers x {sp.npernode} per node")
        return [sp.npernode] * workers
    total = sp.np if sp.np is not None else workers * slots
    if total > workers * slots:
        raise ValueError(f"-np {total} exceeds the {workers} x {slots} slots of the hostfile")
    out, left = [], total
    for _ in range(workers):
        c = min(left, slots)
        out.append(c)
        left -= c
    return out


def export_env(sp: MpirunSpec, launcher_env: List[dict]) -> List[dict]:
    """``-x VAR=value`` / ``-x VAR`` (value from the Launcher container's env) as pod env."""
    known = {e["name"]: e for e in launcher_env or [] if "name" in e}
    out = []
    for x in sp.exports:
        if "=" in x:
            k, v = x.split("=", 1)
            out.append({"name": k, "value": v})
        elif x in known:
            out.append(dict(known[x]))
    return out


def container_argv(c: dict) -> List[str]:
    argv = list(c.get("command") or []) + list(c.get("args") or [])
    # `bash -c "mpirun ..."` / `sh -c` launchers: look inside the script when it is a single command
    if len(argv) == 3 and os.path.basename(argv[0]) in ("bash", "sh") and argv[1] == "-c":
        inner = shlex.split(argv[2])
        if is_mpirun(inner):
            return inner
    return argv


# ------------------------------------------------------------------ launcher: mpi-wait
def _exit_code(pod: dict) -> int:
    for cs in (pod.get("status") or {}).get("containerStatuses") or []:
        t = (cs.get("state") or {}).get("terminated")
        if t:
            return int(t.get("exitCode", 1)) or 1
    return 1


def wait_workers(client, job: str, namespace: str, n_workers: int, timeout: float = 0.0,
                 period: float = 0.5, out=sys.stdout) -> int:
    """mpirun's exit semantics over the Worker pods: 0 when all ``n_workers`` succeeded, the
    first failing worker's exit code as soon as one fails."""
    from .training import LBL_JOB, LBL_RTYPE
    start = time.time()
    seen: Dict[str, str] = {}
    while True:
        pods = client.list("v1", "Pod", namespace, label_selector=f"{LBL_JOB}={job},{LBL_RTYPE}=worker")
        done = 0
        for p in sorted(pods, key=lambda p: p["metadata"]["name"]):
            name, ph = p["metadata"]["name"], (p.get("status") or {}).get("phase") or "Pending"
            if seen.get(name) != ph:
                print(f"[mpi-wait] {name}: {ph}", file=out, flush=True)
                seen[name] = ph
            if ph == "Failed":
                code = _exit_code(p)
                print(f"[mpi-wait] {name} failed with exit code {code}; the job fails", file=out, flush=True)
                return code
            done += ph == "Succeeded"
        if done >= n_workers:
            print(f"[mpi-wait] all {n_workers} workers succeeded", file=out, flush=True)
            return 0
        if timeout and time.time() - start > timeout:
            print(f"[mpi-wait] timed out after {timeout:.0f}s", file=out, flush=True)
            return 124
        time.sleep(period)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kfamd mpi-wait",
                                 description="MPIJob launcher: wait for the job's Worker pods like mpirun")
    ap.add_argument("--job", default=os.environ.get("KFAMD_MPI_JOB"))
    ap.add_argument("--namespace", default=os.environ.get("KFAMD_MPI_NAMESPACE") or os.environ.get("POD_NAMESPACE"))
    ap.add_argument("--workers", type=int, default=int(os.environ.get("KFAMD_MPI_WORKERS", "0") or 0))
    ap.add_argument("--timeout", type=float, default=0.0)
    ap.add_argument("--kube-api", default=os.environ.get("KUBE_API_URL"))
    a = ap.parse_args(argv)
    if not a.job or not a.namespace or a.workers < 1:
        ap.error("--job, --namespace and --workers are required")
    from .client import RestClient
    client = RestClient(a.kube_api) if a.kube_api else RestClient()
    return wait_workers(client, a.job, a.namespace, a.workers, timeout=a.timeout)


if __name__ == "__main__":
    sys.exit(main())
