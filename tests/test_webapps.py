"""CRUD web-app backends (crud_backend, JWA, TWA, VWA) against the in-memory API server.

Reference behaviour: components/crud-web-apps/*/backend (authn/csrf/authz, form
setters, status derivation, routes); the assertions mirror the reference's unit tests
(jupyter/backend/apps/common/{form,status}_test.py, volumes/backend/.../*_test.py)."""
import datetime as dt

import pytest

from service_account_auth_improvements_amd.controlplane.apiserver import APIServer
from service_account_auth_improvements_amd.controlplane.client import InMemoryClient
from service_account_auth_improvements_amd.controlplane.profile import default_cluster_roles
from service_account_auth_improvements_amd.webapps import crud_backend as cb
from service_account_auth_improvements_amd.webapps import jupyter

USER = {"kubeflow-userid": "alice@example.com"}


@pytest.fixture
def cluster():
    srv = APIServer()
    c = InMemoryClient(srv)
    for cr in default_cluster_roles():
        c.create(cr)
    for ns in ("alice", "bob"):
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
              "metadata": {"name": "namespaceAdmin", "namespace": "alice"},
              "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "kubeflow-admin"},
              "subjects": [{"apiGroup": "rbac.authorization.k8s.io", "kind": "User", "name": "alice@example.com"}]})
    c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "mi355x-0"},
              "status": {"capacity": {"amd.com/gpu": "8", "cpu": "256"}}})
    c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass",
              "metadata": {"name": "local", "annotations": {"storageclass.kubernetes.io/is-default-class": "true"}}})
    return srv, c


def _csrf(tc):
    r = tc.get("/", headers=USER)
    cookie = r.headers["Set-Cookie"].split(";")[0].split("=", 1)[1]
    return {"X-XSRF-TOKEN": cookie}


# ------------------------------------------------------------------ crud_backend
def test_authn_csrf_probes_and_base_routes(cluster):
    srv, c = cluster
    app = jupyter.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"})
    tc = app.test_client()
    assert tc.get("/healthz/liveness").json == "alive"
    r = tc.get("/api/namespaces/alice/notebooks")
    assert r.status_code == 401 and r.json["success"] is False and r.json["log"] == "No user detected."
    r = tc.get("/", headers=USER)
    assert b'<base href="/">' in r.data and "XSRF-TOKEN" in r.headers["Set-Cookie"]
    assert "no-store" in r.headers["Cache-Control"]
    # unsafe method without csrf -> 403
    r = tc.post("/api/namespaces/alice/notebooks", json={"name": "x"}, headers=USER)
    assert r.status_code == 403 and "CSRF" in r.json["log"]
    r = tc.get("/api/storageclasses/default", headers=USER)
    assert r.json == {"status": 200, "success": True, "user": "alice@example.com", "defaultStorageClass": "local"}
    assert tc.get("/api/storageclasses", headers=USER).json["storageClasses"] == ["local"]


def test_authz_denied_in_foreign_namespace(cluster):
    srv, c = cluster
    tc = jupyter.create_app(c).test_client()
    r = tc.get("/api/namespaces/bob/notebooks", headers=USER)
    assert r.status_code == 403
    assert r.json["log"] == ("User 'alice@example.com' is not authorized to list "
                             "kubeflow.org/v1beta1/notebooks in namespace 'bob'")
    assert tc.get("/api/namespaces/alice/notebooks", headers=USER).json["notebooks"] == []


def test_uptime():
    now = dt.datetime(2024, 1, 3, 12, 0, 0)
    assert cb.get_uptime("2024-01-03T12:00:00Z", now) == "just now"
    assert cb.get_uptime("2024-01-03T11:59:00Z", now) == "1 min ago"
    assert cb.get_uptime("2024-01-03T10:00:00Z", now) == "2 hours ago"
    assert cb.get_uptime("2024-01-01T12:00:00Z", now) == "2 days ago"


# ------------------------------------------------------------------ JWA
def _nb_body(**kw):
    b = {"name": "nb1", "namespace": "alice", "image": "kfamd/jupyter-pytorch-rocm:latest",
         "imagePullPolicy": "IfNotPresent", "serverType": "jupyter", "cpu": "2", "cpuLimit": "",
         "memory": "4Gi", "memoryLimit": "", "gpus": {"num": "1", "vendor": "amd.com/gpu"},
         "tolerationGroup": "none", "affinityConfig": "none", "configurations": ["add-gpu-env"], "shm": True,
         "datavols": [{"mount": "/data", "existingSource": {"persistentVolumeClaim": {"claimName": "data"}}}],
         "workspace": {"mount": "/home/jovyan", "newPvc": {"metadata": {"name": "nb1-workspace"},
                                                           "spec": {"accessModes": ["ReadWriteOnce"],
                                                                    "resources": {"requests": {"storage": "5Gi"}}}}}}
    b.update(kw)
    return b


def test_jwa_create_list_stop_delete(cluster):
    srv, c = cluster
    tc = jupyter.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    h = dict(USER, **_csrf(tc))
    assert tc.get("/api/gpus", headers=USER).json["vendors"] == ["amd.com/gpu"]
    assert tc.get("/api/config", headers=USER).json["config"]["gpus"]["value"]["vendor"] == "amd.com/gpu"
    r = tc.post("/api/namespaces/alice/notebooks", json=_nb_body(), headers=h)
    assert r.status_code == 200, r.json
    nb = c.get("kubeflow.org/v1beta1", "Notebook", "nb1", "alice")
    ctr = nb["spec"]["template"]["spec"]["containers"][0]
    assert ctr["resources"]["limits"] == {"cpu": "2.4", "memory": "4.8Gi", "amd.com/gpu": "1"}
    assert nb["metadata"]["labels"]["add-gpu-env"] == "true"
    assert nb["metadata"]["annotations"]["notebooks.kubeflow.org/creator"] == "alice@example.com"
    assert {m["mountPath"] for m in ctr["volumeMounts"]} == {"/dev/shm", "/data", "/home/jovyan"}
    assert c.get("v1", "PersistentVolumeClaim", "nb1-workspace", "alice")
    lst = tc.get("/api/namespaces/alice/notebooks", headers=USER).json["notebooks"]
    assert lst[0]["gpus"] == {"count": 1, "message": "1 AMD Instinct MI355X"}
    assert lst[0]["status"]["phase"] == "waiting"
    # stop / double stop / start
    assert tc.patch("/api/namespaces/alice/notebooks/nb1", json={"stopped": True}, headers=h).status_code == 200
    assert tc.patch("/api/namespaces/alice/notebooks/nb1", json={"stopped": True}, headers=h).status_code == 409
    nb = c.get("kubeflow.org/v1beta1", "Notebook", "nb1", "alice")
    nb["status"] = {"readyReplicas": 0, "containerState": {"terminated": {}}}
    c.update_status(nb)
    got = tc.get("/api/namespaces/alice/notebooks/nb1", headers=USER).json["notebook"]
    assert got["processed_status"]["phase"] == "stopped"
    assert tc.patch("/api/namespaces/alice/notebooks/nb1", json={"stopped": False}, headers=h).status_code == 200
    assert "kubeflow-resource-stopped" not in c.get("kubeflow.org/v1beta1", "Notebook", "nb1", "alice")[
        "metadata"].get("annotations", {})
    assert tc.get("/api/namespaces/alice/pvcs", headers=USER).json["pvcs"] == [
        {"name": "nb1-workspace", "size": "5Gi", "mode": "ReadWriteOnce"}]
    assert tc.delete("/api/namespaces/alice/notebooks/nb1", headers=h).status_code == 200


def test_jwa_form_validation(cluster):
    srv, c = cluster
    tc = jupyter.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    h = dict(USER, **_csrf(tc))
    r = tc.post("/api/namespaces/alice/notebooks", json=_nb_body(cpu="2", cpuLimit="1"), headers=h)
    assert r.status_code == 400 and r.json["log"] == "CPU limit must be greater than the request"
    r = tc.post("/api/namespaces/alice/notebooks", json=_nb_body(serverType="vscode"), headers=h)
    assert r.status_code == 400
    bad = _nb_body(datavols=[{"mount": "/d"}])
    assert tc.post("/api/namespaces/alice/notebooks", json=bad, headers=h).status_code == 400
    # nothing was created by the failed requests (dry-run first)
    assert c.list("kubeflow.org/v1beta1", "Notebook", "alice") == []
    assert c.list("v1", "PersistentVolumeClaim", "alice") == []


def test_get_form_value_readonly():
    d = {"image": {"value": "img", "readOnly": True}, "cpu": {"value": "1"}}
    assert jupyter.get_form_value({}, d, "image") == "img"
    with pytest.raises(Exception):
        jupyter.get_form_value({"image": "x"}, d, "image")
    assert jupyter.get_form_value({"cpu": "2"}, d, "cpu") == "2"
    assert jupyter.get_form_value({}, d, "foo", optional=True) is None


def test_notebook_status_derivation():
    base = {"metadata": {"name": "n", "namespace": "ns", "creationTimestamp": "2024-01-01T00:00:00Z"}}
    later = dt.datetime(2024, 1, 1, 0, 5, 0)
    st = jupyter.process_status(dict(base), now=dt.datetime(2024, 1, 1, 0, 0, 5))
    assert st["phase"] == "waiting"
    nb = dict(base, status={"readyReplicas": 1, "containerState": {"running": {}}})
    assert jupyter.process_status(nb, now=later)["phase"] == "ready"
    nb = dict(base, status={"containerState": {"waiting": {"reason": "ImagePullBackOff", "message": "no"}}})
    assert jupyter.process_status(nb, now=later) == {"phase": "warning", "message": "ImagePullBackOff: no",
                                                      "state": ""}
    nb = {"metadata": dict(base["metadata"], deletionTimestamp="x"), "status": {"conditions": [{"type": "x"}]}}
    assert jupyter.process_status(nb, now=later)["phase"] == "terminating"
    ev = [{"metadata": {"creationTimestamp": "2024-01-01T00:01:00Z"}, "type": "Warning",
           "message": "0/1 nodes are available: insufficient amd.com/gpu"}]
    nb = dict(base, status={"conditions": [{"type": "x"}]})
    st = jupyter.process_status(nb, events_fn=lambda n: ev, now=later)
    assert st["phase"] == "warning" and "amd.com/gpu" in st["message"]


# ------------------------------------------------------------------ TWA
def test_twa_crud(cluster):
    from service_account_auth_improvements_amd.webapps import tensorboards
    srv, c = cluster
    tc = tensorboards.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    h = dict(USER, **_csrf(tc))
    r = tc.post("/api/namespaces/alice/tensorboards", json={"name": "tb", "logspath": "pvc://runs/llama",
                                                            "configurations": ["add-gcp"]}, headers=h)
    assert r.status_code == 200, r.json
    tb = c.get("tensorboard.kubeflow.org/v1alpha1", "Tensorboard", "tb", "alice")
    assert tb["spec"]["logspath"] == "pvc://runs/llama" and tb["metadata"]["labels"] == {"add-gcp": "true"}
    lst = tc.get("/api/namespaces/alice/tensorboards", headers=USER).json["tensorboards"]
    assert lst[0]["status"]["phase"] == "unavailable"
    tb["status"] = {"readyReplicas": 1}
    c.update_status(tb)
    assert tc.get("/api/namespaces/alice/tensorboards", headers=USER).json["tensorboards"][0]["status"][
        "phase"] == "ready"
    r = tc.post("/api/namespaces/alice/tensorboards", json={"name": "tb2"}, headers=h)
    assert r.status_code == 400 and "logspath" in r.json["log"]
    assert tc.delete("/api/namespaces/alice/tensorboards/tb", headers=h).status_code == 200


# ------------------------------------------------------------------ VWA
def test_vwa_pvcs_viewers_and_delete_guard(cluster):
    from service_account_auth_improvements_amd.webapps import volumes
    srv, c = cluster
    tc = volumes.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    h = dict(USER, **_csrf(tc))
    body = {"name": "data", "mode": "ReadWriteOnce", "class": "{none}", "size": "10Gi", "type": "new"}
    assert tc.post("/api/namespaces/alice/pvcs", json=body, headers=h).status_code == 200
    pvc = c.get("v1", "PersistentVolumeClaim", "data", "alice")
    assert pvc["spec"]["storageClassName"] == "" and pvc["spec"]["resources"]["requests"]["storage"] == "10Gi"
    lst = tc.get("/api/namespaces/alice/pvcs", headers=USER).json["pvcs"]
    assert lst[0]["status"]["phase"] == "waiting" and lst[0]["viewer"]["status"] == "uninitialized"
    assert tc.post("/api/namespaces/alice/viewers", json={"name": "data"}, headers=h).status_code == 200
    v = c.get("kubeflow.org/v1alpha1", "PVCViewer", "data", "alice")
    assert v["spec"]["pvc"] == "data"
    assert v["spec"]["podSpec"]["containers"][0]["env"][4]["value"] == "/pvcviewers/alice/data/"
    # a training pod mounts it -> 409
    c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "trainer-0", "namespace": "alice"},
              "spec": {"containers": [{"name": "c", "image": "x"}],
                       "volumes": [{"name": "d", "persistentVolumeClaim": {"claimName": "data"}}]}})
    r = tc.delete("/api/namespaces/alice/pvcs/data", headers=h)
    assert r.status_code == 409 and "trainer-0" in r.json["log"]
    c.delete("v1", "Pod", "trainer-0", "alice")
    # only a viewer pod -> viewer deleted, then the PVC
    c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "viewer-0", "namespace": "alice",
                                                             "labels": {"app.kubernetes.io/name": "data"}},
              "spec": {"containers": [{"name": "c", "image": "x"}],
                       "volumes": [{"name": "d", "persistentVolumeClaim": {"claimName": "data"}}]}})
    assert tc.delete("/api/namespaces/alice/pvcs/data", headers=h).status_code == 200
    assert c.get_or_none("kubeflow.org/v1alpha1", "PVCViewer", "data", "alice") is None


def test_pvc_status_from_events():
    from service_account_auth_improvements_amd.webapps import volumes
    pvc = {"metadata": {"name": "p", "namespace": "n"}, "status": {"phase": "Pending"}}
    st = volumes.pvc_status(pvc, [{"reason": "WaitForFirstConsumer", "type": "Normal", "message": "m"}])
    assert st["phase"] == "unavailable" and st["state"] == "WaitForFirstConsumer"
    assert volumes.pvc_status(pvc, [{"reason": "FailedBinding", "type": "Warning", "message": "m"}])[
        "phase"] == "warning"
    assert volumes.pvc_status(dict(pvc, status={"phase": "Bound"}), [])["phase"] == "ready"


def test_spa_bundle_served_by_every_app(cluster):
    from service_account_auth_improvements_amd.webapps import tensorboards, volumes
    srv, c = cluster
    for mod in (jupyter, volumes, tensorboards):
        tc = mod.create_app(c).test_client()
        r = tc.get("/static/kfamd-ui.js", headers=USER)
        assert r.status_code == 200 and b"kfamd web UI" in r.data, mod
        assert b'data-app="' in tc.get("/", headers=USER).data
