"""M1/M2: generated manifests are current, render with the kustomize-lite builder, name only
real component entrypoints; CRDs register kinds on the API server and enforce their schemas;
the sample CRs (one per BASELINE config) validate."""
import filecmp
import os

import pytest

from service_account_auth_improvements_amd import manifests
from service_account_auth_improvements_amd.cluster import load_manifests
from service_account_auth_improvements_amd.controlplane.apiserver import APIServer, ApiError, BUILTIN_TYPES
from service_account_auth_improvements_amd.controlplane.client import InMemoryClient

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAN = os.path.join(ROOT, "manifests")
CR_GROUPS = {"kubeflow.org", "tensorboard.kubeflow.org", "serving.kserve.io"}


def test_committed_manifests_are_current(tmp_path):
    manifests.generate(str(tmp_path))
    for root, _, files in os.walk(tmp_path):
        for f in files:
            rel = os.path.relpath(os.path.join(root, f), tmp_path)
            assert filecmp.cmp(os.path.join(root, f), os.path.join(MAN, rel), shallow=False), \
                f"{rel} is stale: run python -m service_account_auth_improvements_amd.manifests generate"


def test_overlay_renders_and_commands_exist():
    docs = manifests.build(os.path.join(MAN, "overlays", "kubeflow"))
    kinds = {d["kind"] for d in docs}
    assert {"CustomResourceDefinition", "Deployment", "Service", "ClusterRole", "VirtualService",
            "MutatingWebhookConfiguration", "ConfigMap"} <= kinds
    from service_account_auth_improvements_amd import __main__ as entry
    known = {"notebook-controller", "profile-controller", "kfam", "admission-webhook", "tensorboard-controller",
             "pvcviewer-controller", "training-operator", "inferenceservice-controller", "jupyter-web-app",
             "volumes-web-app", "tensorboards-web-app", "centraldashboard"}
    for d in docs:
        if d["kind"] == "Deployment":
            assert d["metadata"]["namespace"] == "kubeflow"
            for c in d["spec"]["template"]["spec"]["containers"]:
                assert c["command"] == ["python", "-m", "service_account_auth_improvements_amd"]
                assert c["args"][0] in known and c["args"][0] in entry.__doc__
                assert c["image"].startswith("kfamd/")


def test_crds_register_and_validate():
    srv = APIServer(types=[t for t in BUILTIN_TYPES if t.group not in CR_GROUPS])
    c = InMemoryClient(srv)
    with pytest.raises(ApiError):
        c.list("kubeflow.org/v1", "PyTorchJob")
    for d in load_manifests(os.path.join(MAN, "crds")):
        c.create(d)
    srv.ensure_namespace("kubeflow-user")
    for d in load_manifests(os.path.join(MAN, "samples")):
        c.create(d)
    assert c.get("kubeflow.org/v1", "PyTorchJob", "llama3-8b-ddp8", "kubeflow-user")
    assert c.get("kubeflow.org/v1beta1", "Notebook", "rocm-notebook", "kubeflow-user")
    # schema enforcement
    bad = [
        {"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": "p"}, "spec": {}},
        {"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer", "metadata": {"name": "v", "namespace": "kubeflow-user"},
         "spec": {"pvc": ""}},
        {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "j", "namespace": "kubeflow-user"},
         "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": -1, "restartPolicy": "Sometimes"}}}},
        {"apiVersion": "tensorboard.kubeflow.org/v1alpha1", "kind": "Tensorboard",
         "metadata": {"name": "t", "namespace": "kubeflow-user"}, "spec": {}},
    ]
    for b in bad:
        with pytest.raises(ApiError) as ei:
            c.create(b)
        assert ei.value.code == 422, b
    # served versions: v1alpha1 / v1 Notebook reachable, storage version v1beta1
    nb = c.get("kubeflow.org/v1", "Notebook", "rocm-notebook", "kubeflow-user")
    assert nb["metadata"]["name"] == "rocm-notebook"


def test_sample_jobs_reconcile_on_local_cluster():
    """Conformance-style smoke (M2): sample Profile + jobs reconcile into pods with GPUs."""
    from service_account_auth_improvements_amd.cluster import LocalCluster
    cl = LocalCluster(n_gpus=8, api_port=None).start()
    try:
        cl.apply(os.path.join(MAN, "samples", "profile.yaml"))
        assert cl.wait_for(lambda: cl.client.get_or_none("v1", "ResourceQuota", "kf-resource-quota", "kubeflow-user"), 20)
        cl.apply(os.path.join(MAN, "samples", "pytorchjob-llama3-8b-ddp8.yaml"))
        pod = cl.wait_for(lambda: cl.client.get_or_none("v1", "Pod", "llama3-8b-ddp8-master-0", "kubeflow-user"), 20)
        assert pod["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "8"
        cl.apply(os.path.join(MAN, "samples", "inferenceservice-llama3-8b.yaml"))
        assert cl.wait_for(lambda: cl.client.get_or_none("apps/v1", "Deployment", "llama3-8b-predictor",
                                                         "kubeflow-user"), 20)
    finally:
        cl.stop()


# ------------------------------------------------------------------ component overlays (M1)
def _by(docs, kind, name=None):
    return [d for d in docs if d["kind"] == kind and (name is None or d["metadata"]["name"] == name)]


@pytest.mark.parametrize("app,prefix", [("jupyter-web-app", "/jupyter"), ("volumes-web-app", "/volumes"),
                                        ("tensorboards-web-app", "/tensorboards")])
def test_istio_overlay_renders(app, prefix):
    """reference crud-web-apps/*/manifests/overlays/istio/{virtual-service,authorization-policy,destination-rule}.yaml"""
    docs = manifests.build(os.path.join(MAN, app, "overlays", "istio"))
    (vs,) = _by(docs, "VirtualService")
    http = vs["spec"]["http"][0]
    assert http["match"] == [{"uri": {"prefix": prefix + "/"}}] and http["rewrite"] == {"uri": "/"}
    assert http["headers"]["request"]["add"]["x-forwarded-prefix"] == prefix
    assert http["route"][0]["destination"]["host"] == f"{app}-service.kubeflow.svc.cluster.local"
    (ap,) = _by(docs, "AuthorizationPolicy")
    assert ap["spec"]["rules"][0]["from"][0]["source"]["principals"] == [manifests.INGRESS_GATEWAY_PRINCIPAL]
    assert ap["spec"]["selector"]["matchLabels"] == {"app": app}
    (dr,) = _by(docs, "DestinationRule")
    assert dr["spec"]["trafficPolicy"]["tls"]["mode"] == "ISTIO_MUTUAL"
    assert _by(docs, "Deployment") and all(d["metadata"]["namespace"] == "kubeflow" for d in docs
                                           if d["kind"] not in ("ClusterRole", "ClusterRoleBinding"))


def test_cert_manager_overlay_renders():
    docs = manifests.build(os.path.join(MAN, "admission-webhook", "overlays", "cert-manager"))
    (cert,) = _by(docs, "Certificate")
    assert cert["spec"]["dnsNames"] == ["admission-webhook-service.kubeflow.svc",
                                        "admission-webhook-service.kubeflow.svc.cluster.local"]
    assert cert["spec"]["secretName"] == "webhook-certs" and _by(docs, "Issuer", cert["spec"]["issuerRef"]["name"])
    (mw,) = _by(docs, "MutatingWebhookConfiguration")
    assert mw["metadata"]["annotations"]["cert-manager.io/inject-ca-from"] == "kubeflow/admission-webhook-cert"
    assert mw["webhooks"][0]["clientConfig"]["service"]["path"] == "/apply-poddefault"     # base kept
    (dep,) = _by(docs, "Deployment")
    ctr = dep["spec"]["template"]["spec"]["containers"][0]
    assert "--tls-cert-file=/etc/webhook/certs/tls.crt" in ctr["args"]
    assert any(v.get("secret", {}).get("secretName") == "webhook-certs" for v in dep["spec"]["template"]["spec"]["volumes"])


def test_kserve_overlay_adds_the_endpoints_link():
    import json
    base = json.loads(_by(manifests.build(os.path.join(MAN, "centraldashboard")), "ConfigMap",
                          "centraldashboard-config")[0]["data"]["links"])
    docs = manifests.build(os.path.join(MAN, "centraldashboard", "overlays", "kserve"))
    links = json.loads(_by(docs, "ConfigMap", "centraldashboard-config")[0]["data"]["links"])
    texts = [m["text"] for m in links["menuLinks"]]
    assert "KServe Endpoints" in texts and "KServe Endpoints" not in [m["text"] for m in base["menuLinks"]]
    assert set(m["text"] for m in base["menuLinks"]) <= set(texts)
    assert _by(docs, "VirtualService") and _by(docs, "AuthorizationPolicy")       # built on the istio overlay


def test_kubeflow_overlay_composes_the_component_overlays():
    docs = manifests.build(os.path.join(MAN, "overlays", "kubeflow"))
    assert len(_by(docs, "VirtualService")) == 4 and len(_by(docs, "DestinationRule")) == 3
    assert _by(docs, "Certificate") and _by(docs, "Issuer")
    names = [d["metadata"]["name"] for d in docs]
    assert len(names) == len(set((d["kind"], d["metadata"]["name"]) for d in docs)), "duplicate objects"
