"""P9: notebook load test (counterpart of notebook-controller/loadtest/start_notebooks.py):
create N Notebooks (+ their workspace PVCs) in a namespace and report how long the
controller takes to bring every StatefulSet to readyReplicas == 1.

  python tools/loadtest_notebooks.py -n 50                          # in-process LocalCluster
  python tools/loadtest_notebooks.py -n 50 --kube-api http://127.0.0.1:8001 --namespace kubeflow-user
  python tools/loadtest_notebooks.py -n 3 --emit-yaml > notebooks.yaml   # kubectl apply -f
"""
import argparse
import json
import os
import sys
import time

import yaml

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def objects(i, ns, image, gpus):
    name = f"jupyter-test-{i}"
    pvc = {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": f"{name}-workspace", "namespace": ns},
           "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}}
    ctr = {"name": name, "image": image, "resources": {"requests": {"cpu": "0.5", "memory": "1Gi"}},
           "volumeMounts": [{"name": "workspace", "mountPath": "/home/jovyan"}]}
    if gpus:
        ctr["resources"]["limits"] = {"amd.com/gpu": str(gpus)}
    nb = {"apiVersion": "kubeflow.org/v1beta1", "kind": "Notebook", "metadata": {"name": name, "namespace": ns},
          "spec": {"template": {"spec": {"containers": [ctr], "volumes": [
              {"name": "workspace", "persistentVolumeClaim": {"claimName": f"{name}-workspace"}}]}}}}
    return [pvc, nb]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", type=int, default=3)
    ap.add_argument("--namespace", default="kubeflow-user")
    ap.add_argument("--image", default="kfamd/jupyter-pytorch-rocm:latest")
    ap.add_argument("--gpus", type=int, default=0)
    ap.add_argument("--kube-api", default=None)
    ap.add_argument("--emit-yaml", action="store_true")
    ap.add_argument("--timeout", type=float, default=300)
    a = ap.parse_args(argv)
    docs = [d for i in range(a.n) for d in objects(i, a.namespace, a.image, a.gpus)]
    if a.emit_yaml:
        yaml.safe_dump_all(docs, sys.stdout, sort_keys=False)
        return 0
    cl = None
    if a.kube_api:
        from service_account_auth_improvements_amd.controlplane.client import RestClient
        c = RestClient(a.kube_api)
    else:
        from service_account_auth_improvements_amd.cluster import LocalCluster
        cl = LocalCluster(n_gpus=max(8, a.n * a.gpus), api_port=None).start()
        cl.server.ensure_namespace(a.namespace)
        c = cl.client
    t0 = time.time()
    for d in docs:
        c.create(d)
    t_created = time.time()
    ready = 0
    while time.time() - t0 < a.timeout:
        ready = sum(1 for nb in c.list("kubeflow.org/v1beta1", "Notebook", a.namespace)
                    if (nb.get("status") or {}).get("readyReplicas") == 1)
        if ready >= a.n:
            break
        time.sleep(0.05)
    out = {"notebooks": a.n, "ready": ready, "create_s": round(t_created - t0, 3),
           "all_ready_s": round(time.time() - t0, 3)}
    print(json.dumps(out))
    if cl:
        cl.stop()
    return 0 if ready >= a.n else 1


if __name__ == "__main__":
    sys.exit(main())
