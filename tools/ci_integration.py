"""Per-component integration tests against a multi-process cluster (P6/P8: the reference's
``*_intergration_test.yaml`` workflows build a component image, deploy it into a KinD cluster,
apply a sample and wait for the result; e.g. .github/workflows/nb_controller_intergration_test.yaml,
profiles_kfam_intergration_test.yaml, poddefaults_intergration_test.yaml, jwa_intergration_test.yaml).

Here the cluster is ``cluster.ProcessCluster``: apiserver, controller-manager (+ scheduler) and
a kubelet as separate processes, everything over the Kubernetes REST API.  Web apps and KFAM run
in this process against that API (as their Deployments would), driven through their HTTP routes.

  python tools/ci_integration.py notebook-controller profile-controller ...   # or: all
Exit status 0 when every selected component passed; one line per component on stdout.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

USER = "ci@example.com"
H = {"kubeflow-userid": USER}
NS = "kf-ci"


def wait(fn, timeout=30.0, what=""):
    from service_account_auth_improvements_amd.controlplane.apiserver import ApiError
    end = time.time() + timeout
    last = None
    while time.time() < end:
        try:
            v = fn()
            if v:
                return v
        except (ApiError, KeyError, IndexError, TypeError) as e:
            last = e
        time.sleep(0.05)
    raise AssertionError(f"timed out waiting for {what or fn} ({last})")


def ensure_profile(c):
    """The user's namespace via a Profile (what every web-app test starts from)."""
    if c.get_or_none("kubeflow.org/v1", "Profile", NS) is None:
        c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": NS},
                  "spec": {"owner": {"kind": "User", "name": USER}}})
    wait(lambda: c.get("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin", NS), what="profile")
    if not c.list("storage.k8s.io/v1", "StorageClass"):
        c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass",
                  "metadata": {"name": "local", "annotations": {"storageclass.kubernetes.io/is-default-class": "true"}}})


def csrf(tc):
    r = tc.get("/", headers=H)
    tok = r.headers["Set-Cookie"].split(";")[0].split("=", 1)[1]
    return dict(H, **{"X-XSRF-TOKEN": tok})


# ------------------------------------------------------------------ components
def notebook_controller(c):
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "nb-ci"}})
    c.create({"apiVersion": "kubeflow.org/v1", "kind": "Notebook", "metadata": {"name": "nb", "namespace": "nb-ci"},
              "spec": {"template": {"spec": {"containers": [{"name": "nb", "image": "kfamd/jupyter:latest"}]}}}})
    wait(lambda: c.get("apps/v1", "StatefulSet", "nb", "nb-ci"), what="statefulset")
    wait(lambda: c.get("v1", "Service", "nb", "nb-ci"), what="service")
    wait(lambda: c.get("v1", "Pod", "nb-0", "nb-ci")["status"]["phase"] == "Running", what="pod running")
    wait(lambda: c.get("kubeflow.org/v1", "Notebook", "nb", "nb-ci")["status"]["readyReplicas"] == 1,
         what="notebook status")


def profile_controller(c):
    from service_account_auth_improvements_amd.controlplane.kfam import Kfam
    from prometheus_client import CollectorRegistry
    ensure_profile(c)
    for sa in ("default-editor", "default-viewer"):
        wait(lambda sa=sa: c.get("v1", "ServiceAccount", sa, NS), what=sa)
    wait(lambda: c.get("security.istio.io/v1beta1", "AuthorizationPolicy", "ns-owner-access-istio", NS),
         what="authorization policy")
    # KFAM (profiles_kfam_intergration_test): add and remove a contributor through its API
    tc = Kfam(c, user_id_header="kubeflow-userid", user_id_prefix="", cluster_admin="root@example.com",
              registry=CollectorRegistry()).app().test_client()
    body = {"user": {"kind": "User", "name": "bob@example.com"}, "referredNamespace": NS,
            "roleRef": {"kind": "ClusterRole", "name": "edit"}}
    r = tc.post("/kfam/v1/bindings", json=body, headers=H)
    assert r.status_code == 200, (r.status_code, r.data)
    wait(lambda: any(b["user"]["name"] == "bob@example.com" for b in
                     tc.get(f"/kfam/v1/bindings?namespace={NS}", headers=H).json["bindings"]), what="binding")
    assert tc.delete("/kfam/v1/bindings", json=body, headers=H).status_code == 200


def poddefaults(c):
    ensure_profile(c)
    c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PodDefault",
              "metadata": {"name": "add-rocm-env", "namespace": NS},
              "spec": {"selector": {"matchLabels": {"add-rocm-env": "true"}}, "desc": "ROCm env",
                       "env": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}]}})
    pod = c.create({"apiVersion": "v1", "kind": "Pod",
                    "metadata": {"name": "pd-ci", "namespace": NS, "labels": {"add-rocm-env": "true"}},
                    "spec": {"containers": [{"name": "main", "image": "img"}]}})
    env = {e["name"]: e.get("value") for e in pod["spec"]["containers"][0].get("env") or []}
    assert env.get("HSA_ENABLE_IPC_MODE_LEGACY") == "0", env
    ann = pod["metadata"].get("annotations") or {}
    assert any(k.startswith("poddefault.admission.kubeflow.org/poddefault-add-rocm-env") for k in ann), ann


def tensorboard_controller(c):
    ensure_profile(c)
    c.create({"apiVersion": "tensorboard.kubeflow.org/v1alpha1", "kind": "Tensorboard",
              "metadata": {"name": "tb-ci", "namespace": NS}, "spec": {"logspath": "gs://bucket/runs"}})
    wait(lambda: c.get("apps/v1", "Deployment", "tb-ci", NS), what="deployment")
    wait(lambda: c.get("v1", "Service", "tb-ci", NS), what="service")
    wait(lambda: c.get("networking.istio.io/v1alpha3", "VirtualService", "tb-ci", NS), what="virtualservice")


def pvcviewer_controller(c):
    ensure_profile(c)
    c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "data", "namespace": NS},
              "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}})
    c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer",
              "metadata": {"name": "pvc-ci", "namespace": NS}, "spec": {"pvc": "data"}})
    v = c.get("kubeflow.org/v1alpha1", "PVCViewer", "pvc-ci", NS)
    assert v["spec"].get("podSpec"), "the defaulting webhook did not fill spec.podSpec"
    wait(lambda: c.get("apps/v1", "Deployment", "pvcviewer-pvc-ci", NS), what="deployment")


def training_operator(c):
    from service_account_auth_improvements_amd.controlplane import training
    ensure_profile(c)
    cmd = [sys.executable, "-c", "import os; print('rank', os.environ['RANK'], 'of', os.environ['WORLD_SIZE'])"]
    job = training.pytorchjob_manifest("ci-job", NS, "local", cmd, n_nodes=2, gpus_per_node=0, master_port=29751)
    job["spec"]["nprocPerNode"] = "1"
    c.create(job)

    def done():
        j = c.get(training.PT_API, "PyTorchJob", "ci-job", NS)
        return next((x["type"] for x in (j.get("status") or {}).get("conditions", [])
                     if x["type"] in ("Succeeded", "Failed") and x["status"] == "True"), None)
    assert wait(done, timeout=120, what="job") == "Succeeded"


def jupyter_web_app(c):
    from service_account_auth_improvements_amd.webapps import jupyter
    ensure_profile(c)
    tc = jupyter.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    h = csrf(tc)
    body = {"name": "jwa-nb", "namespace": NS, "image": "kfamd/jupyter-pytorch-rocm:latest",
            "imagePullPolicy": "IfNotPresent", "serverType": "jupyter", "cpu": "1", "cpuLimit": "", "memory": "1Gi",
            "memoryLimit": "", "gpus": {"num": "none"}, "tolerationGroup": "none", "affinityConfig": "none",
            "configurations": [], "shm": True, "datavols": [],
            "workspace": {"mount": "/home/jovyan", "newPvc": {"metadata": {"name": "jwa-nb-ws"},
                                                              "spec": {"accessModes": ["ReadWriteOnce"],
                                                                       "resources": {"requests": {"storage": "1Gi"}}}}}}
    r = tc.post(f"/api/namespaces/{NS}/notebooks", json=body, headers=h)
    assert r.status_code == 200, r.data
    wait(lambda: [n for n in tc.get(f"/api/namespaces/{NS}/notebooks", headers=H).json["notebooks"]
                  if n["name"] == "jwa-nb" and n["status"]["phase"] == "ready"], timeout=30, what="ready notebook")
    assert tc.delete(f"/api/namespaces/{NS}/notebooks/jwa-nb", headers=h).status_code == 200


def volumes_web_app(c):
    from service_account_auth_improvements_amd.webapps import volumes
    ensure_profile(c)
    tc = volumes.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    h = csrf(tc)
    r = tc.post(f"/api/namespaces/{NS}/pvcs", json={"name": "vwa-pvc", "mode": "ReadWriteOnce", "class": "local",
                                                     "size": "1Gi", "type": "new"}, headers=h)
    assert r.status_code == 200, r.data
    assert any(p["name"] == "vwa-pvc" for p in tc.get(f"/api/namespaces/{NS}/pvcs", headers=H).json["pvcs"])
    assert tc.delete(f"/api/namespaces/{NS}/pvcs/vwa-pvc", headers=h).status_code == 200


def tensorboards_web_app(c):
    from service_account_auth_improvements_amd.webapps import tensorboards
    ensure_profile(c)
    tc = tensorboards.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    h = csrf(tc)
    r = tc.post(f"/api/namespaces/{NS}/tensorboards", json={"name": "twa-tb", "logspath": "gs://b/runs",
                                                             "configurations": []}, headers=h)
    assert r.status_code == 200, r.data
    wait(lambda: c.get("apps/v1", "Deployment", "twa-tb", NS), what="tensorboard deployment")
    assert any(t["name"] == "twa-tb" for t in
               tc.get(f"/api/namespaces/{NS}/tensorboards", headers=H).json["tensorboards"])


def centraldashboard(c):
    from prometheus_client import CollectorRegistry

    from service_account_auth_improvements_amd.controlplane.kfam import Kfam
    from service_account_auth_improvements_amd.webapps import dashboard
    from service_account_auth_improvements_amd.cluster import load_manifests
    ensure_profile(c)
    # the dashboard's links / settings ConfigMap, as its kustomize base deploys it
    for d in load_manifests(os.path.join(ROOT, "manifests", "centraldashboard")):
        if d["kind"] == "ConfigMap" and c.get_or_none("v1", "ConfigMap", d["metadata"]["name"],
                                                      d["metadata"].get("namespace", "kubeflow")) is None:
            d["metadata"].setdefault("namespace", "kubeflow")
            c.create(d)
    kf = Kfam(c, user_id_header="kubeflow-userid", user_id_prefix="", cluster_admin="root@example.com",
              registry=CollectorRegistry()).app().test_client()

    def transport(method, path, body, headers):
        r = kf.open("/kfam" + path, method=method, data=body, headers=headers)
        return r.status_code, r.data
    app = dashboard.create_app(c, dashboard.ProfilesService(transport),
                               dashboard.LocalMetricsService(start=False),
                               env={"USERID_HEADER": "kubeflow-userid", "USERID_PREFIX": ""}).test_client()
    r = app.get("/api/workgroup/exists", headers=H)
    assert r.status_code == 200 and r.json["hasWorkgroup"] is True, r.data
    r = app.get("/api/dashboard-links", headers=H)
    assert r.status_code == 200 and r.json.get("menuLinks"), r.data
    r = app.get(f"/api/workgroup/get-contributors/{NS}", headers=H)
    assert r.status_code == 200, r.data


COMPONENTS = {
    "notebook-controller": notebook_controller,
    "profile-controller": profile_controller,
    "poddefaults": poddefaults,
    "tensorboard-controller": tensorboard_controller,
    "pvcviewer-controller": pvcviewer_controller,
    "training-operator": training_operator,
    "jupyter-web-app": jupyter_web_app,
    "volumes-web-app": volumes_web_app,
    "tensorboards-web-app": tensorboards_web_app,
    "centraldashboard": centraldashboard,
}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("components", nargs="+", help=f"'all' or any of: {' '.join(COMPONENTS)}")
    a = ap.parse_args(argv)
    names = list(COMPONENTS) if a.components == ["all"] else a.components
    unknown = [n for n in names if n not in COMPONENTS]
    if unknown:
        ap.error(f"unknown component(s): {unknown}")
    from service_account_auth_improvements_amd.cluster import ProcessCluster
    from service_account_auth_improvements_amd.native import build_native
    build_native()
    pc = ProcessCluster(nodes=1, gpus_per_node=0, exec_pods=True).start()
    failed = 0
    try:
        for n in names:
            t0 = time.time()
            try:
                COMPONENTS[n](pc.client)
                print(f"PASS {n} ({time.time() - t0:.1f}s)", flush=True)
            except Exception:
                failed += 1
                print(f"FAIL {n}\n{traceback.format_exc()}", flush=True)
    finally:
        if failed:
            print(pc.component_log("controller-manager")[-3000:])
        pc.stop()
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
