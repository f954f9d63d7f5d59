"""M2: platform conformance run (counterpart of conformance/1.7: a kf-conformance Profile with
a resource quota, then the training-operator conformance workload).

Against a cluster's Kubernetes REST API (``--kube-api``) or an in-process LocalCluster
(default, pods executed as processes):

1. create Profile ``kf-conformance`` (owner, quota cpu 4 / memory 4Gi / storage 5Gi) and wait
   for its namespace, service accounts, role bindings and quota;
2. run the training conformance jobs -- a 2-replica MNIST PyTorchJob over gloo through the
   operator and the kfamd-launch launcher, and the same MNIST run as an upstream-shaped MPIJob
   (Launcher ``mpirun -np 2``, 2 Workers running sshd) -- and wait for ``Succeeded``;
3. (optional ``--gpu``) a 1-GPU Llama PyTorchJob step on MI355X;
4. write a JSON report (one record per check) and exit non-zero on any failure.

  python tools/conformance.py [--kube-api URL] [--gpu] [--report conformance.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NS = "kf-conformance"


def free_port_pair() -> int:
    """A port p with p and p + 1 both free (the job's MASTER_PORT and the launcher's rendezvous
    port): fixed ports collided with other jobs on a shared host, e.g. tests run in parallel."""
    import socket
    while True:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p >= 65000:
            continue
        t = socket.socket()
        try:
            t.bind(("127.0.0.1", p + 1))
            return p
        except OSError:
            continue
        finally:
            t.close()


def wait(fn, timeout):
    from service_account_auth_improvements_amd.controlplane.apiserver import ApiError
    end = time.time() + timeout
    while time.time() < end:
        try:
            v = fn()
            if v:
                return v
        except ApiError:
            pass
        time.sleep(0.1)
    return None


def job_done(c, name, api="kubeflow.org/v1", kind="PyTorchJob"):
    j = c.get(api, kind, name, NS)
    for cd in (j.get("status") or {}).get("conditions") or []:
        if cd["type"] in ("Succeeded", "Failed") and cd["status"] == "True":
            return cd["type"]
    return None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--kube-api", default=None)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--report", default=None)
    ap.add_argument("--timeout", type=float, default=240)
    a = ap.parse_args(argv)
    from service_account_auth_improvements_amd.controlplane import training
    from service_account_auth_improvements_amd.native import build_native
    cl = None
    if a.kube_api:
        from service_account_auth_improvements_amd.controlplane.client import RestClient
        c = RestClient(a.kube_api)
    else:
        from service_account_auth_improvements_amd.cluster import LocalCluster
        build_native()
        # the REST facade is up so the MPIJob launcher (mpi-wait) can follow its workers
        cl = LocalCluster(n_gpus=1 if a.gpu else 0, exec_pods=True, api_port=0,
                          extra_env={"OMP_NUM_THREADS": "2"}).start()
        c = cl.client
    results = []

    def check(name, ok, detail=""):
        results.append({"check": name, "passed": bool(ok), "detail": detail})
        print(("PASS " if ok else "FAIL ") + name + (f" -- {detail}" if detail and not ok else ""), flush=True)

    try:
        c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": NS},
                  "spec": {"owner": {"kind": "User", "name": "conformance@kubeflow.org"},
                           "resourceQuotaSpec": {"hard": {"cpu": "4", "memory": "4Gi", "requests.storage": "5Gi"}}}})
        check("profile namespace", wait(lambda: c.get("v1", "Namespace", NS), 30))
        check("profile service accounts", wait(lambda: c.get("v1", "ServiceAccount", "default-editor", NS) and
                                               c.get("v1", "ServiceAccount", "default-viewer", NS), 30))
        check("profile role bindings", wait(lambda: c.get("rbac.authorization.k8s.io/v1", "RoleBinding",
                                                          "namespaceAdmin", NS), 30))
        check("profile resource quota", wait(lambda: c.get("v1", "ResourceQuota", "kf-resource-quota", NS), 30))

        cmd = [sys.executable, "-m", "service_account_auth_improvements_amd", "train", "--model", "mnist",
               "--micro-batch", "32", "--steps", "20", "--device", "cpu"]
        job = training.pytorchjob_manifest("mnist-conformance", NS, "kfamd/trainer-rocm:latest", cmd, n_nodes=2,
                                           gpus_per_node=0, master_port=free_port_pair())
        job["spec"]["nprocPerNode"] = "1"
        c.create(job)
        res = wait(lambda: job_done(c, "mnist-conformance"), a.timeout)
        check("training: PyTorchJob 2-replica MNIST (gloo)", res == "Succeeded", f"result={res}")
        mj = training.mpijob_manifest("mnist-mpi-conformance", NS, "kfamd/trainer-rocm:latest", cmd, workers=2,
                                      gpus_per_worker=0, master_port=free_port_pair())
        c.create(mj)
        res = wait(lambda: job_done(c, "mnist-mpi-conformance", training.MPI_API, "MPIJob"), a.timeout)
        check("training: MPIJob mpirun -np 2 MNIST (gloo)", res == "Succeeded", f"result={res}")
        if a.gpu:
            cmd = [sys.executable, "-m", "service_account_auth_improvements_amd", "train", "--model", "llama3-8b",
                   "--seq-len", "2048", "--steps", "2", "--device", "cuda"]
            c.create(training.pytorchjob_manifest("llama-conformance", NS, "kfamd/trainer-rocm:latest", cmd,
                                                  n_nodes=1, gpus_per_node=1, master_port=free_port_pair()))
            res = wait(lambda: job_done(c, "llama-conformance"), a.timeout)
            check("training: PyTorchJob Llama-3-8B on MI355X", res == "Succeeded", f"result={res}")
        c.delete("kubeflow.org/v1", "Profile", NS)
        check("profile cleanup", wait(lambda: c.get_or_none("v1", "Namespace", NS) is None, 60))
    finally:
        if cl:
            cl.stop()
    if a.report:
        with open(a.report, "w") as f:
            json.dump({"results": results, "passed": all(r["passed"] for r in results)}, f, indent=1)
    return 0 if all(r["passed"] for r in results) else 1


if __name__ == "__main__":
    sys.exit(main())
