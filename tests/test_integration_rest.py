"""P8-equivalent integration test against a running cluster over its Kubernetes REST API
(reference: py/kubeflow/kubeflow/ci/... profiles integration test: create Profile, check the
namespace, default-editor/default-viewer SAs and role bindings, delete, check cleanup).
Runs against the LocalCluster's REST facade through RestClient (no in-process shortcuts)."""
import time

from service_account_auth_improvements_amd.cluster import LocalCluster
from service_account_auth_improvements_amd.controlplane.apiserver import ApiError
from service_account_auth_improvements_amd.controlplane.client import RestClient


def _wait(fn, timeout=20.0):
    end = time.time() + timeout
    while time.time() < end:
        try:
            v = fn()
            if v:
                return v
        except ApiError:
            pass
        time.sleep(0.05)
    return None


def test_profile_lifecycle_over_rest():
    cl = LocalCluster(n_gpus=8, api_port=0).start()
    try:
        c = RestClient(cl.http.url)
        c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": "kf-integration"},
                  "spec": {"owner": {"kind": "User", "name": "ci@example.com"},
                           "resourceQuotaSpec": {"hard": {"cpu": "4", "memory": "4Gi", "requests.storage": "5Gi"}}}})
        ns = _wait(lambda: c.get("v1", "Namespace", "kf-integration"))
        assert ns["metadata"]["annotations"]["owner"] == "ci@example.com"
        for sa in ("default-editor", "default-viewer"):
            assert _wait(lambda sa=sa: c.get("v1", "ServiceAccount", sa, "kf-integration"))
        rbs = _wait(lambda: {r["metadata"]["name"] for r in c.list("rbac.authorization.k8s.io/v1", "RoleBinding",
                                                                      "kf-integration")} >= {"namespaceAdmin",
                                                                                             "default-editor",
                                                                                             "default-viewer"})
        assert rbs
        assert _wait(lambda: c.get("v1", "ResourceQuota", "kf-resource-quota", "kf-integration"))
        # label selector + watch over REST
        events = []
        stop = c.watch(lambda et, o: events.append((et, o["metadata"]["name"])), "kubeflow.org/v1", "Profile")
        c.delete("kubeflow.org/v1", "Profile", "kf-integration")
        assert _wait(lambda: c.get_or_none("kubeflow.org/v1", "Profile", "kf-integration") is None)
        assert _wait(lambda: c.get_or_none("v1", "Namespace", "kf-integration") is None)
        assert _wait(lambda: any(et == "DELETED" for et, _ in events))
        stop()
    finally:
        cl.stop()
