"""M1: CRDs + per-component kustomize manifests, generated from this module, and a small
kustomize renderer (``build``) used by the local cluster and the manifest tests.

Reference layout: components/*/config/{crd,default,manager,rbac,overlays/{kubeflow,
standalone}} and components/*/manifests/{base,overlays/{istio,cert-manager,kserve}}.
The group / versions (in the reference's order) / served / storage / kind / plural / scope of
every reference CRD match the reference (tests/test_crd_compat.py pins them against a table
transcribed from the reference CRD files), e.g. Notebook serves v1 (storage), v1alpha1 and
v1beta1 (``notebook-controller/config/crd/bases/kubeflow.org_notebooks.yaml:18,3144,3147,6276``).
The schemas are this repo's own structural schemas: the core/v1 PodSpec subset the
controllers and web apps read (containers, initContainers, volumes, env/envFrom, resources,
ports, volumeMounts, tolerations, affinity, nodeSelector, securityContext, ...) is typed,
anything outside it is preserved (``x-kubernetes-preserve-unknown-fields``), and the
Notebook CRD carries the reference's ``config/crd/patches/validation_patches.yaml``
constraints (containers minItems 1; every container requires name and image).

CLI::

    python -m service_account_auth_improvements_amd.manifests generate [OUT=manifests]
    python -m service_account_auth_improvements_amd.manifests build DIR   # kustomize-lite
"""
from __future__ import annotations

import copy
import os
import sys
from typing import Dict, List

import yaml

PKG = "service_account_auth_improvements_amd"
IMAGE_PREFIX = "kfamd"
TAG = "latest"

class NoAliasDumper(yaml.SafeDumper):
    """Plain YAML: a schema node reused in several places is written out each time, never as an
    ``&anchor`` / ``*alias`` pair (manifest tools and kustomize patches edit nodes in place)."""

    def ignore_aliases(self, data):
        return True


# ------------------------------------------------------------------ schema helpers
OBJ_ANY = {"type": "object", "x-kubernetes-preserve-unknown-fields": True}


def obj(props=None, required=None, **kw):
    s = {"type": "object"}
    if props:
        s["properties"] = props
    if required:
        s["required"] = list(required)
    s.update(kw)
    return s


def arr(items):
    return {"type": "array", "items": items}


STR = {"type": "string"}
INT = {"type": "integer"}
BOOL = {"type": "boolean"}
CONDITIONS = arr(obj({"type": STR, "status": STR, "reason": STR, "message": STR,
                      "lastProbeTime": STR, "lastTransitionTime": STR, "lastUpdateTime": STR}))
INT_OR_STR = {"x-kubernetes-int-or-string": True}
STR_MAP = {"type": "object", "additionalProperties": STR}
QUANTITY_MAP = {"type": "object", "additionalProperties": INT_OR_STR}


def open_obj(props=None, required=None):
    """An object whose listed fields are typed and whose other fields are kept as-is."""
    o = obj(props, required)
    o["x-kubernetes-preserve-unknown-fields"] = True
    return o


# ---- core/v1 types: full structural schemas (corev1.py), no preserve-unknown holes
from . import corev1 as _core  # noqa: E402

ENV_VAR = _core.schema("EnvVar")
ENV_FROM = _core.schema("EnvFromSource")
VOLUME = _core.schema("Volume")
VOLUME_MOUNT = _core.schema("VolumeMount")
TOLERATION = _core.schema("Toleration")
AFFINITY = _core.schema("Affinity")
RESOURCES = _core.schema("ResourceRequirements")
LABEL_SELECTOR = _core.schema("LabelSelector")
LOCAL_REF = _core.schema("LocalObjectReference")
container = _core.container
pod_spec = _core.pod_spec


def _fresh(x):
    """A deep copy, so no two places of a generated CRD share one dict (alias-free YAML)."""
    return copy.deepcopy(x)


OBJECT_META = _core.schema("ObjectMeta")
POD_TEMPLATE = obj({"metadata": OBJECT_META, "spec": pod_spec(containers_min=1)})
REPLICA_SPEC = obj({"replicas": {"type": "integer", "minimum": 0},
                    "restartPolicy": {"type": "string", "enum": ["Always", "OnFailure", "Never", "ExitCode"]},
                    "template": POD_TEMPLATE})
REPLICA_STATUS = obj({"active": INT, "succeeded": INT, "failed": INT, "labelSelector": LABEL_SELECTOR,
                      "selector": STR})


def crd(group, kind, plural, scope, versions, short=None, categories=None, printer=None):
    """versions: list of (name, served, storage, schema_spec, schema_status)."""
    vs = []
    for name, served, storage, spec, status in versions:
        v = {"name": name, "served": served, "storage": storage,
             "schema": {"openAPIV3Schema": obj({"apiVersion": STR, "kind": STR, "metadata": {"type": "object"},
                                                "spec": spec, "status": status})},
             "subresources": {"status": {}}}
        if printer:
            v["additionalPrinterColumns"] = printer
        vs.append(v)
    names = {"kind": kind, "listKind": kind + "List", "plural": plural, "singular": kind.lower()}
    if short:
        names["shortNames"] = short
    if categories:
        names["categories"] = categories
    return {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
            "metadata": {"name": f"{plural}.{group}", "annotations": {"kfamd.io/generated": "true"}},
            "spec": {"group": group, "names": names, "scope": scope, "versions": vs}}


def crds() -> Dict[str, dict]:
    # Notebook: spec.template.spec is a full corev1.PodSpec plus the reference's validation
    # patches (containers minItems 1, name + image required per container)
    nb_spec = obj({"template": obj({"metadata": OBJECT_META,
                                    "spec": pod_spec(containers_min=1, container_required=("name", "image"))})})
    nb_status = obj({"conditions": CONDITIONS, "readyReplicas": INT, "containerState": _core.schema("ContainerState")})
    prof_spec = obj({"owner": obj({"kind": {"type": "string", "enum": ["User", "Group", "ServiceAccount"]},
                                   "name": STR, "apiGroup": STR, "namespace": STR}, ["kind", "name"]),
                     # a plugin's spec is a runtime.RawExtension: its shape is the plugin's own
                     "plugins": arr(obj({"kind": STR, "spec": OBJ_ANY}, ["kind"])),
                     "resourceQuotaSpec": obj({"hard": {"type": "object", "additionalProperties": INT_OR_STR},
                                               "scopes": arr(STR),
                                               "scopeSelector": obj({"matchExpressions": arr(obj(
                                                   {"operator": STR, "scopeName": STR, "values": arr(STR)},
                                                   ["operator", "scopeName"]))})})}, ["owner"])
    prof_status = obj({"conditions": CONDITIONS})
    pd_spec = obj({"selector": LABEL_SELECTOR, "desc": STR,
                   "serviceAccountName": STR, "automountServiceAccountToken": BOOL, "env": arr(ENV_VAR),
                   "envFrom": arr(ENV_FROM), "volumes": arr(VOLUME), "volumeMounts": arr(VOLUME_MOUNT),
                   "initContainers": arr(container()), "sidecars": arr(container()), "tolerations": arr(TOLERATION),
                   "imagePullSecrets": arr(LOCAL_REF), "annotations": STR_MAP, "labels": STR_MAP,
                   "args": arr(STR), "command": arr(STR)}, ["selector"])
    tb_spec = obj({"logspath": STR}, ["logspath"])
    tb_status = obj({"conditions": arr(obj({"deploymentState": STR, "lastProbeTime": STR})), "readyReplicas": INT})
    pv_spec = obj({"pvc": {"type": "string", "minLength": 1}, "podSpec": pod_spec(),
                   "networking": obj({"targetPort": {"x-kubernetes-int-or-string": True}, "basePrefix": STR,
                                      "rewrite": STR, "timeout": STR}, ["targetPort", "basePrefix"]),
                   "rwoScheduling": BOOL}, ["pvc"])
    pv_status = obj({"conditions": CONDITIONS, "ready": BOOL, "url": STR})
    # kubeflow.org/v1 RunPolicy: every field is declared (so none is pruned silently); the ones
    # this platform cannot honour (schedulingPolicy: no gang scheduler) are rejected at admission
    # by controlplane/training.py validate_job
    run_policy = obj({"cleanPodPolicy": {"type": "string", "enum": ["All", "Running", "None"]},
                      "backoffLimit": {"type": "integer", "minimum": 0},
                      "activeDeadlineSeconds": {"type": "integer", "minimum": 0},
                      "ttlSecondsAfterFinished": {"type": "integer", "minimum": 0},
                      "suspend": BOOL,
                      "schedulingPolicy": obj({"minAvailable": INT, "queue": STR, "minResources": QUANTITY_MAP,
                                               "priorityClass": STR, "scheduleTimeoutSeconds": INT})})
    job_status = obj({"conditions": CONDITIONS,
                      "replicaStatuses": {"type": "object", "additionalProperties": REPLICA_STATUS},
                      "restartCount": INT, "startTime": STR, "completionTime": STR, "lastReconcileTime": STR,
                      # restarts per replica type (an MPIJob Launcher's backoffLimit counts its own only)
                      "replicaRestarts": {"type": "object", "additionalProperties": INT}})
    pt_spec = obj({"pytorchReplicaSpecs": obj({"Master": REPLICA_SPEC, "Worker": REPLICA_SPEC}),
                   "nprocPerNode": {"x-kubernetes-int-or-string": True}, "runPolicy": run_policy,
                   "elasticPolicy": obj({"minReplicas": {"type": "integer", "minimum": 1},
                                         "maxReplicas": {"type": "integer", "minimum": 1},
                                         "rdzvBackend": STR, "rdzvHost": STR, "rdzvPort": INT, "rdzvId": STR,
                                         "rdzvConf": arr(obj({"key": STR, "value": STR})),
                                         "maxRestarts": {"type": "integer", "minimum": 0}, "nProcPerNode": INT,
                                         "standalone": BOOL,
                                         # autoscaling/v2 MetricSpec (declared; refused at admission)
                                         "metrics": arr(obj({"type": STR, "resource": obj({
                                             "name": STR, "target": obj({"type": STR, "averageUtilization": INT,
                                                                         "averageValue": INT_OR_STR,
                                                                         "value": INT_OR_STR})})}))})},
                  ["pytorchReplicaSpecs"])
    mpi_spec = obj({"mpiReplicaSpecs": obj({"Launcher": REPLICA_SPEC, "Worker": REPLICA_SPEC}),
                    "slotsPerWorker": {"type": "integer", "minimum": 1}, "runPolicy": run_policy,
                    "mpiImplementation": {"type": "string", "enum": ["OpenMPI", "Intel", "MPICH"]},
                    "sshAuthMountPath": STR}, ["mpiReplicaSpecs"])
    isvc_spec = obj({"predictor": obj({"model": obj({"modelFormat": obj({"name": STR, "version": STR}, ["name"]),
                                                     "storageUri": STR, "runtime": STR, "args": arr(STR),
                                                     "command": arr(STR), "env": arr(ENV_VAR),
                                                     "resources": RESOURCES, "image": STR,
                                                     "protocolVersion": STR}),
                                       "containers": arr(container()), "volumes": arr(VOLUME),
                                       "minReplicas": {"type": "integer", "minimum": 0}, "maxReplicas": INT,
                                       "serviceAccountName": STR, "nodeSelector": STR_MAP,
                                       "tolerations": arr(TOLERATION), "affinity": AFFINITY,
                                       "annotations": STR_MAP, "labels": STR_MAP})}, ["predictor"])
    isvc_status = obj({"conditions": CONDITIONS, "url": STR,
                       "address": obj({"url": STR}),
                       "components": {"type": "object", "additionalProperties": obj(
                           {"url": STR, "latestCreatedRevision": STR, "latestReadyRevision": STR,
                            "address": obj({"url": STR})})},
                       "modelStatus": obj({"states": obj({"activeModelState": STR, "targetModelState": STR}),
                                           "transitionStatus": STR, "copies": obj({"failedCopies": INT,
                                                                                    "totalCopies": INT})}),
                       "observedGeneration": INT})
    age = [{"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"}]
    return {
        "kubeflow.org_notebooks.yaml": crd("kubeflow.org", "Notebook", "notebooks", "Namespaced",
                                           [("v1", True, True, nb_spec, nb_status),
                                            ("v1alpha1", True, False, nb_spec, nb_status),
                                            ("v1beta1", True, False, nb_spec, nb_status)]),
        "kubeflow.org_profiles.yaml": crd("kubeflow.org", "Profile", "profiles", "Cluster",
                                          [("v1", True, True, prof_spec, prof_status),
                                           ("v1beta1", True, False, prof_spec, prof_status)]),
        "kubeflow.org_poddefaults.yaml": crd("kubeflow.org", "PodDefault", "poddefaults", "Namespaced",
                                             [("v1alpha1", True, True, pd_spec, obj({}))]),
        "kubeflow.org_pvcviewers.yaml": crd("kubeflow.org", "PVCViewer", "pvcviewers", "Namespaced",
                                            [("v1alpha1", True, True, pv_spec, pv_status)], printer=age),
        "tensorboard.kubeflow.org_tensorboards.yaml": crd("tensorboard.kubeflow.org", "Tensorboard", "tensorboards",
                                                          "Namespaced", [("v1alpha1", True, True, tb_spec, tb_status)]),
        "kubeflow.org_pytorchjobs.yaml": crd("kubeflow.org", "PyTorchJob", "pytorchjobs", "Namespaced",
                                             [("v1", True, True, pt_spec, job_status)],
                                             categories=["kubeflow-training"], printer=age),
        "kubeflow.org_mpijobs.yaml": crd("kubeflow.org", "MPIJob", "mpijobs", "Namespaced",
                                         [("v2beta1", True, True, mpi_spec, job_status)],
                                         categories=["kubeflow-training"], printer=age),
        "serving.kserve.io_inferenceservices.yaml": crd("serving.kserve.io", "InferenceService", "inferenceservices",
                                                        "Namespaced", [("v1beta1", True, True, isvc_spec, isvc_status)],
                                                        short=["isvc"], printer=[
                                                            {"name": "URL", "type": "string", "jsonPath": ".status.url"},
                                                            {"name": "Ready", "type": "string",
                                                             "jsonPath": ".status.conditions[?(@.type=='Ready')].status"}]
                                                        + age),
    }


# ------------------------------------------------------------------ component manifests
def _deployment(name, component, args, ports, env=None, sa=None, gpu=False, replicas=1, extra_ctr=None,
                volumes=None, mounts=None):
    ctr = {"name": "manager" if "controller" in component or component == "training-operator" else component,
           "image": f"{IMAGE_PREFIX}/{component}:{TAG}",
           "command": ["python", "-m", PKG], "args": args,
           "ports": [{"containerPort": p, "name": n} for n, p in ports.items()],
           "env": env or [],
           "resources": {"requests": {"cpu": "100m", "memory": "256Mi"}}}
    if "probe" in ports:
        ctr["livenessProbe"] = {"httpGet": {"path": "/healthz", "port": ports["probe"]}, "initialDelaySeconds": 15}
        ctr["readinessProbe"] = {"httpGet": {"path": "/readyz", "port": ports["probe"]}, "initialDelaySeconds": 5}
    if mounts:
        ctr["volumeMounts"] = mounts
    spec = {"serviceAccountName": sa or f"{component}-service-account", "containers": [ctr] + (extra_ctr or [])}
    if volumes:
        spec["volumes"] = volumes
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "labels": {"app": component}},
            "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": component}},
                     "template": {"metadata": {"labels": {"app": component},
                                               "annotations": {"sidecar.istio.io/inject": "false"}},
                                  "spec": spec}}}


def _service(name, component, ports):
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "labels": {"app": component}},
            "spec": {"selector": {"app": component},
                     "ports": [{"name": n, "port": p, "targetPort": t} for n, p, t in ports]}}


def _sa(component):
    return {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": f"{component}-service-account"}}


def _rbac(component, rules):
    return [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
             "metadata": {"name": f"{component}-role"}, "rules": rules},
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
             "metadata": {"name": f"{component}-role-binding"},
             "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": f"{component}-role"},
             "subjects": [{"kind": "ServiceAccount", "name": f"{component}-service-account", "namespace": "kubeflow"}]}]


def _rule(groups, resources, verbs=("get", "list", "watch", "create", "update", "patch", "delete")):
    return {"apiGroups": list(groups), "resources": list(resources), "verbs": list(verbs)}


def _vs(name, prefix, host, port=80, rewrite="/", forwarded_prefix=None, namespace="kubeflow",
        cluster_domain="cluster.local"):
    http = {"match": [{"uri": {"prefix": prefix}}], "rewrite": {"uri": rewrite},
            "route": [{"destination": {"host": f"{host}.{namespace}.svc.{cluster_domain}", "port": {"number": port}}}]}
    if forwarded_prefix:
        http = dict({"headers": {"request": {"add": {"x-forwarded-prefix": forwarded_prefix}}}}, **http)
    return {"apiVersion": "networking.istio.io/v1alpha3", "kind": "VirtualService", "metadata": {"name": name},
            "spec": {"gateways": ["kubeflow-gateway"], "hosts": ["*"], "http": [http]}}


INGRESS_GATEWAY_PRINCIPAL = "cluster.local/ns/istio-system/sa/istio-ingressgateway-service-account"


def _authz_ingress_only(name, app):
    """AuthorizationPolicy: only the Istio ingress gateway may call the app (reference
    crud-web-apps/*/manifests/overlays/istio/authorization-policy.yaml)."""
    return {"apiVersion": "security.istio.io/v1beta1", "kind": "AuthorizationPolicy", "metadata": {"name": name},
            "spec": {"action": "ALLOW", "rules": [{"from": [{"source": {"principals": [INGRESS_GATEWAY_PRINCIPAL]}}]}],
                     "selector": {"matchLabels": {"app": app}}}}


def _destination_rule(name, host, namespace="kubeflow"):
    return {"apiVersion": "networking.istio.io/v1alpha3", "kind": "DestinationRule", "metadata": {"name": name},
            "spec": {"host": f"{host}.{namespace}.svc.cluster.local", "trafficPolicy": {"tls": {"mode": "ISTIO_MUTUAL"}}}}


def _env(**kv):
    return [{"name": k, "value": str(v)} for k, v in kv.items()]


def components() -> Dict[str, Dict[str, List[dict]]]:
    """component -> {file name -> docs} for the base of each component."""
    ctrl_ports = {"metrics": 8080, "probe": 8081}
    out = {}
    out["notebook-controller"] = {
        "deployment.yaml": [_deployment("notebook-controller-deployment", "notebook-controller",
                                        ["notebook-controller", "--metrics-addr=:8080", "--probe-addr=:8081",
                                         "--enable-leader-election"], ctrl_ports,
                                        env=_env(USE_ISTIO="true", ISTIO_GATEWAY="kubeflow/kubeflow-gateway",
                                                 ISTIO_HOST="*", CLUSTER_DOMAIN="cluster.local", ENABLE_CULLING="false",
                                                 CULL_IDLE_TIME="1440", IDLENESS_CHECK_PERIOD="1", ADD_FSGROUP="true"))],
        "service.yaml": [_service("notebook-controller-service", "notebook-controller", [("metrics", 443, 8080)])],
        "rbac.yaml": [_sa("notebook-controller")] + _rbac("notebook-controller", [
            _rule(["kubeflow.org"], ["notebooks", "notebooks/status", "notebooks/finalizers"]),
            _rule(["apps"], ["statefulsets"]), _rule([""], ["services", "pods", "events"]),
            _rule(["networking.istio.io"], ["virtualservices"])]),
    }
    out["profile-controller"] = {
        "deployment.yaml": [_deployment(
            "profiles-deployment", "profile-controller",
            ["profile-controller", "--userid-header=kubeflow-userid", "--userid-prefix=",
             "--workload-identity=", "--namespace-labels-path=/etc/profile-controller/namespace-labels.yaml"],
            ctrl_ports, sa="profiles-controller-service-account",
            extra_ctr=[{"name": "kfam", "image": f"{IMAGE_PREFIX}/kfam:{TAG}", "command": ["python", "-m", PKG],
                        "args": ["kfam", "--userid-header=kubeflow-userid", "--userid-prefix=",
                                 "--cluster-admin=admin@kubeflow.org"],
                        "ports": [{"containerPort": 8081, "name": "kfam-http"}]}],
            volumes=[{"name": "namespace-labels", "configMap": {"name": "namespace-labels-data"}}],
            mounts=[{"name": "namespace-labels", "mountPath": "/etc/profile-controller", "readOnly": True}])],
        "service.yaml": [_service("profiles-kfam", "profile-controller", [("http", 8081, 8081)])],
        "rbac.yaml": [{"apiVersion": "v1", "kind": "ServiceAccount",
                       "metadata": {"name": "profiles-controller-service-account"}}] + [
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
             "metadata": {"name": "profiles-cluster-role-binding"},
             "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "cluster-admin"},
             "subjects": [{"kind": "ServiceAccount", "name": "profiles-controller-service-account",
                           "namespace": "kubeflow"}]}],
        "namespace-labels.yaml": [{"apiVersion": "v1", "kind": "ConfigMap",
                                   "metadata": {"name": "namespace-labels-data"},
                                   "data": {"namespace-labels.yaml": open(os.path.join(
                                       os.path.dirname(__file__), "config", "namespace-labels.yaml")).read()}}],
        "kubeflow-roles.yaml": _kubeflow_roles(),
    }
    out["admission-webhook"] = {
        "deployment.yaml": [_deployment("admission-webhook-deployment", "admission-webhook",
                                        ["admission-webhook", "--port=4443", "--tls-cert-file=/etc/webhook/certs/tls.crt",
                                         "--tls-key-file=/etc/webhook/certs/tls.key"], {"https-webhook": 4443},
                                        volumes=[{"name": "webhook-cert", "secret": {"secretName": "webhook-certs"}}],
                                        mounts=[{"name": "webhook-cert", "mountPath": "/etc/webhook/certs",
                                                 "readOnly": True}])],
        "service.yaml": [_service("admission-webhook-service", "admission-webhook", [("https-webhook", 443, 4443)])],
        "mutating-webhook-configuration.yaml": [{
            "apiVersion": "admissionregistration.k8s.io/v1", "kind": "MutatingWebhookConfiguration",
            "metadata": {"name": "admission-webhook-mutating-webhook-configuration"},
            "webhooks": [{"name": "admission-webhook-deployment.kubeflow.org", "admissionReviewVersions": ["v1"],
                          "sideEffects": "None", "failurePolicy": "Fail",
                          "clientConfig": {"service": {"name": "admission-webhook-service", "namespace": "kubeflow",
                                                       "path": "/apply-poddefault"}},
                          "namespaceSelector": {"matchLabels": {"app.kubernetes.io/part-of": "kubeflow-profile"}},
                          "rules": [{"apiGroups": [""], "apiVersions": ["v1"], "operations": ["CREATE"],
                                     "resources": ["pods"]}]}]}],
        "rbac.yaml": [_sa("admission-webhook")] + _rbac("admission-webhook", [
            _rule(["kubeflow.org"], ["poddefaults"], ("get", "list", "watch"))]),
    }
    out["tensorboard-controller"] = {
        "deployment.yaml": [_deployment("tensorboard-controller-deployment", "tensorboard-controller",
                                        ["tensorboard-controller", "--metrics-addr=:8080", "--probe-addr=:8081",
                                         "--enable-leader-election"], ctrl_ports,
                                        env=_env(ISTIO_GATEWAY="kubeflow/kubeflow-gateway", ISTIO_HOST="*",
                                                 TENSORBOARD_IMAGE=f"{IMAGE_PREFIX}/tensorboard:{TAG}",
                                                 RWO_PVC_SCHEDULING="true"))],
        "rbac.yaml": [_sa("tensorboard-controller")] + _rbac("tensorboard-controller", [
            _rule(["tensorboard.kubeflow.org"], ["tensorboards", "tensorboards/status"]),
            _rule(["apps"], ["deployments"]), _rule([""], ["services", "pods", "persistentvolumeclaims"]),
            _rule(["networking.istio.io"], ["virtualservices"])]),
    }
    out["pvcviewer-controller"] = {
        "deployment.yaml": [_deployment("pvcviewer-controller-manager", "pvcviewer-controller",
                                        ["pvcviewer-controller", "--metrics-addr=:8080", "--probe-addr=:8081",
                                         "--webhook-port=9443", "--enable-leader-election"],
                                        dict(ctrl_ports, **{"webhook-server": 9443}),
                                        env=_env(DEFAULT_POD_SPEC_PATH="/etc/config/default-viewer-podspec.yaml"))],
        "webhook.yaml": [
            {"apiVersion": "admissionregistration.k8s.io/v1", "kind": "MutatingWebhookConfiguration",
             "metadata": {"name": "pvcviewer-mutating-webhook-configuration"},
             "webhooks": [{"name": "mpvcviewer.kb.io", "admissionReviewVersions": ["v1"], "sideEffects": "None",
                           "failurePolicy": "Fail",
                           "clientConfig": {"service": {"name": "pvcviewer-webhook-service", "namespace": "kubeflow",
                                                        "path": "/mutate-kubeflow-org-v1alpha1-pvcviewer"}},
                           "rules": [{"apiGroups": ["kubeflow.org"], "apiVersions": ["v1alpha1"],
                                      "operations": ["CREATE", "UPDATE"], "resources": ["pvcviewers"]}]}]},
            {"apiVersion": "admissionregistration.k8s.io/v1", "kind": "ValidatingWebhookConfiguration",
             "metadata": {"name": "pvcviewer-validating-webhook-configuration"},
             "webhooks": [{"name": "vpvcviewer.kb.io", "admissionReviewVersions": ["v1"], "sideEffects": "None",
                           "failurePolicy": "Fail",
                           "clientConfig": {"service": {"name": "pvcviewer-webhook-service", "namespace": "kubeflow",
                                                        "path": "/validate-kubeflow-org-v1alpha1-pvcviewer"}},
                           "rules": [{"apiGroups": ["kubeflow.org"], "apiVersions": ["v1alpha1"],
                                      "operations": ["CREATE", "UPDATE"], "resources": ["pvcviewers"]}]}]}],
        "service.yaml": [_service("pvcviewer-webhook-service", "pvcviewer-controller", [("https", 443, 9443)])],
        "rbac.yaml": [_sa("pvcviewer-controller")] + _rbac("pvcviewer-controller", [
            _rule(["kubeflow.org"], ["pvcviewers", "pvcviewers/status", "pvcviewers/finalizers"]),
            _rule(["apps"], ["deployments"]), _rule([""], ["services", "pods", "persistentvolumeclaims"]),
            _rule(["networking.istio.io"], ["virtualservices"])]),
    }
    out["training-operator"] = {
        "deployment.yaml": [_deployment("training-operator", "training-operator",
                                        ["training-operator", "--metrics-addr=:8080", "--probe-addr=:8081",
                                         "--enable-leader-election"], ctrl_ports)],
        "rbac.yaml": [_sa("training-operator")] + _rbac("training-operator", [
            _rule(["kubeflow.org"], ["pytorchjobs", "pytorchjobs/status", "mpijobs", "mpijobs/status"]),
            _rule([""], ["pods", "services", "configmaps", "events"])]),
    }
    out["kserve-controller"] = {
        "deployment.yaml": [_deployment("kserve-controller-manager", "kserve-controller",
                                        ["inferenceservice-controller", "--metrics-addr=:8080", "--probe-addr=:8081"],
                                        ctrl_ports, env=_env(KFAMD_PREDICTOR_IMAGE=f"{IMAGE_PREFIX}/predictor-rocm:{TAG}"))],
        "rbac.yaml": [_sa("kserve-controller")] + _rbac("kserve-controller", [
            _rule(["serving.kserve.io"], ["inferenceservices", "inferenceservices/status"]),
            _rule(["apps"], ["deployments"]), _rule([""], ["services"]),
            _rule(["networking.istio.io"], ["virtualservices"])]),
    }
    for app, port, prefix in (("jupyter-web-app", 5000, "/jupyter/"), ("volumes-web-app", 5000, "/volumes/"),
                              ("tensorboards-web-app", 5000, "/tensorboards/")):
        env = _env(APP_PREFIX=prefix.rstrip("/"), USERID_HEADER="kubeflow-userid", USERID_PREFIX="",
                   APP_SECURE_COOKIES="true", APP_DISABLE_AUTH="false", CSRF_SAMESITE="Strict",
                   BACKEND_MODE="prod")
        docs = {"deployment.yaml": [_deployment(f"{app}-deployment", app, [app, f"--port={port}"], {"http": port},
                                                env=env)],
                "service.yaml": [_service(f"{app}-service", app, [("http", 80, port)])],
                "rbac.yaml": [_sa(app)] + _rbac(app, [
                    _rule(["authorization.k8s.io"], ["subjectaccessreviews"], ("create",)),
                    _rule([""], ["namespaces", "nodes"], ("get", "list")),
                    _rule(["storage.k8s.io"], ["storageclasses"], ("get", "list"))])}
        if app == "jupyter-web-app":
            docs["spawner-ui-config.yaml"] = [{"apiVersion": "v1", "kind": "ConfigMap",
                                               "metadata": {"name": "jupyter-web-app-config"},
                                               "data": {"spawner_ui_config.yaml": open(os.path.join(
                                                   os.path.dirname(__file__), "webapps", "config",
                                                   "spawner_ui_config.yaml")).read()}}]
        if app == "volumes-web-app":
            docs["viewer-spec.yaml"] = [{"apiVersion": "v1", "kind": "ConfigMap",
                                         "metadata": {"name": "volumes-web-app-viewer-spec"},
                                         "data": {"viewer-spec.yaml": open(os.path.join(
                                             os.path.dirname(__file__), "webapps", "config", "viewer-spec.yaml")).read()}}]
        out[app] = docs
    out["centraldashboard"] = {
        "deployment.yaml": [_deployment("centraldashboard", "centraldashboard", ["centraldashboard", "--port=8082"],
                                        {"http": 8082},
                                        env=_env(USERID_HEADER="kubeflow-userid", USERID_PREFIX="",
                                                 PROFILES_KFAM_SERVICE_HOST="profiles-kfam.kubeflow",
                                                 REGISTRATION_FLOW="true", DASHBOARD_CONFIGMAP="centraldashboard-config",
                                                 LOGOUT_URL="/oauth2/sign_out"))],
        "service.yaml": [_service("centraldashboard", "centraldashboard", [("http", 80, 8082)])],
        "configmap.yaml": [_dashboard_configmap()],
        "rbac.yaml": [_sa("centraldashboard")] + _rbac("centraldashboard", [
            _rule([""], ["namespaces", "events", "nodes", "configmaps"], ("get", "list", "watch")),
            _rule(["app.k8s.io"], ["applications"], ("get", "list", "watch"))]),
    }
    return out


def _kubeflow_roles():
    from .controlplane.profile import default_cluster_roles
    return default_cluster_roles()


def _dashboard_configmap(kserve: bool = False):
    """``kserve``: the kserve overlay's variant, adding the "KServe Endpoints" menu item
    (reference centraldashboard/manifests/overlays/kserve/patches/configmap.yaml)."""
    import json
    links = {"menuLinks": [
        {"type": "item", "link": "/jupyter/", "text": "Notebooks", "icon": "book"},
        {"type": "item", "link": "/tensorboards/", "text": "TensorBoards", "icon": "assessment"},
        {"type": "item", "link": "/volumes/", "text": "Volumes", "icon": "device:storage"},
        {"type": "item", "link": "/training/", "text": "Training Jobs (MI355X)", "icon": "kubeflow:katib"}],
        "externalLinks": [], "quickLinks": [
            {"text": "Create a new Notebook server", "desc": "Notebook Servers", "link": "/jupyter/new"},
            {"text": "Serve Llama-3 on MI355X", "desc": "InferenceService", "link": "/kserve-endpoints/"}],
        "documentationItems": []}
    if kserve:
        links["menuLinks"].insert(3, {"type": "item", "link": "/kserve-endpoints/", "text": "KServe Endpoints",
                                      "icon": "kubeflow:models"})
    settings = {"DASHBOARD_FORCE_IFRAME": True}
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "centraldashboard-config"},
            "data": {"links": json.dumps(links, indent=2), "settings": json.dumps(settings)}}


WEB_APPS = (("jupyter-web-app", "/jupyter/", "/jupyter"), ("volumes-web-app", "/volumes/", "/volumes"),
            ("tensorboards-web-app", "/tensorboards/", "/tensorboards"))


def component_overlays() -> Dict[str, dict]:
    """Per-component overlays (reference ``components/*/manifests/overlays/{istio,cert-manager,kserve}``):
    ``<component>/overlays/<name>`` -> {"kustomization": ..., "files": {file: [docs]}}."""
    out = {}
    for app, prefix, fwd in WEB_APPS:
        out[f"{app}/overlays/istio"] = {
            "kustomization": {"resources": ["../..", "virtual-service.yaml", "authorization-policy.yaml",
                                            "destination-rule.yaml"], "namespace": "kubeflow"},
            "files": {"virtual-service.yaml": [_vs(f"{app}-{app}", prefix, f"{app}-service", forwarded_prefix=fwd)],
                      "authorization-policy.yaml": [_authz_ingress_only(app, app)],
                      "destination-rule.yaml": [_destination_rule(app, f"{app}-service")]}}
    out["centraldashboard/overlays/istio"] = {
        "kustomization": {"resources": ["../..", "virtual-service.yaml", "authorizationpolicy.yaml"],
                          "namespace": "kubeflow"},
        "files": {"virtual-service.yaml": [_vs("centraldashboard", "/", "centraldashboard")],
                  "authorizationpolicy.yaml": [_authz_ingress_only("central-dashboard", "centraldashboard")]}}
    out["centraldashboard/overlays/kserve"] = {
        "kustomization": {"resources": ["../istio"], "patches": [{"path": "patches/configmap.yaml"}]},
        "files": {"patches/configmap.yaml": [_dashboard_configmap(kserve=True)]}}
    # cert-manager provisions the PodDefault webhook's serving certificate and injects its CA
    # into the MutatingWebhookConfiguration (reference admission-webhook/manifests/overlays/cert-manager)
    svc, ns = "admission-webhook-service", "kubeflow"
    out["admission-webhook/overlays/cert-manager"] = {
        "kustomization": {"resources": ["../..", "certificate.yaml"], "namespace": ns,
                          "patchesStrategicMerge": ["mutating-webhook-configuration.yaml", "deployment.yaml"]},
        "files": {
            "certificate.yaml": [
                {"apiVersion": "cert-manager.io/v1", "kind": "Certificate", "metadata": {"name": "admission-webhook-cert"},
                 "spec": {"isCA": True, "commonName": f"{svc}.{ns}.svc",
                          "dnsNames": [f"{svc}.{ns}.svc", f"{svc}.{ns}.svc.cluster.local"],
                          "issuerRef": {"kind": "Issuer", "name": "admission-webhook-selfsigned-issuer"},
                          "secretName": "webhook-certs"}},
                {"apiVersion": "cert-manager.io/v1", "kind": "Issuer",
                 "metadata": {"name": "admission-webhook-selfsigned-issuer"}, "spec": {"selfSigned": {}}}],
            "mutating-webhook-configuration.yaml": [
                {"apiVersion": "admissionregistration.k8s.io/v1", "kind": "MutatingWebhookConfiguration",
                 "metadata": {"name": "admission-webhook-mutating-webhook-configuration",
                              "annotations": {"cert-manager.io/inject-ca-from": f"{ns}/admission-webhook-cert"}}}],
            "deployment.yaml": [
                {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "admission-webhook-deployment"},
                 "spec": {"template": {"spec": {"containers": [
                     {"name": "admission-webhook",
                      "args": ["admission-webhook", "--port=4443", "--tls-cert-file=/etc/webhook/certs/tls.crt",
                               "--tls-key-file=/etc/webhook/certs/tls.key"]}]}}}}]}}
    return out


def overlays() -> Dict[str, dict]:
    """overlay dir -> kustomization (relative to manifests/)."""
    comps = sorted(components())
    via = {app: f"../../{app}/overlays/istio" for app, _, _ in WEB_APPS}
    via["centraldashboard"] = "../../centraldashboard/overlays/kserve"
    via["admission-webhook"] = "../../admission-webhook/overlays/cert-manager"
    return {
        "overlays/kubeflow": {"namespace": "kubeflow",
                              "resources": ["../../crds"] + [via.get(c, f"../../{c}") for c in comps],
                              "commonLabels": {"app.kubernetes.io/part-of": "kubeflow"}},
        "overlays/standalone": {"namespace": "kubeflow-standalone",
                                "resources": ["../../crds", "../../notebook-controller", "../../training-operator",
                                              "../../kserve-controller"]},
    }


def generate(out_dir: str):
    os.makedirs(os.path.join(out_dir, "crds"), exist_ok=True)
    cs = crds()
    for fn, doc in cs.items():
        # compact: leaf schema nodes as one-line flow mappings ({type: string}), block elsewhere
        _dump(os.path.join(out_dir, "crds", fn), [doc], flow=None)
    _dump(os.path.join(out_dir, "crds", "kustomization.yaml"),
          [{"apiVersion": "kustomize.config.k8s.io/v1beta1", "kind": "Kustomization", "resources": sorted(cs)}])
    for comp, files in components().items():
        d = os.path.join(out_dir, comp)
        os.makedirs(d, exist_ok=True)
        for fn, docs in files.items():
            _dump(os.path.join(d, fn), docs)
        _dump(os.path.join(d, "kustomization.yaml"),
              [{"apiVersion": "kustomize.config.k8s.io/v1beta1", "kind": "Kustomization",
                "resources": sorted(files),
                "images": [{"name": f"{IMAGE_PREFIX}/{comp}", "newName": f"{IMAGE_PREFIX}/{comp}", "newTag": TAG}]}])
    for rel, ov in component_overlays().items():
        d = os.path.join(out_dir, rel)
        for fn, docs in ov["files"].items():
            os.makedirs(os.path.dirname(os.path.join(d, fn)), exist_ok=True)
            _dump(os.path.join(d, fn), docs)
        _dump(os.path.join(d, "kustomization.yaml"),
              [dict({"apiVersion": "kustomize.config.k8s.io/v1beta1", "kind": "Kustomization"}, **ov["kustomization"])])
    for rel, k in overlays().items():
        d = os.path.join(out_dir, rel)
        os.makedirs(d, exist_ok=True)
        _dump(os.path.join(d, "kustomization.yaml"),
              [dict({"apiVersion": "kustomize.config.k8s.io/v1beta1", "kind": "Kustomization"}, **k)])


def _dump(path, docs, flow=False):
    with open(path, "w") as f:
        f.write("# Generated by `python -m service_account_auth_improvements_amd.manifests generate`; do not edit.\n")
        yaml.dump_all(docs, f, Dumper=NoAliasDumper, sort_keys=False, width=120, default_flow_style=flow)


# ------------------------------------------------------------------ kustomize-lite
def build(path: str, _seen=None) -> List[dict]:
    """Render a kustomization directory: resources (files / dirs), namespace, commonLabels,
    images, configMapGenerator (literals / files), patches (strategic-merge-like deep merge)."""
    _seen = _seen or set()
    path = os.path.abspath(path)
    if path in _seen:
        raise ValueError(f"kustomization cycle at {path}")
    _seen.add(path)
    with open(os.path.join(path, "kustomization.yaml")) as f:
        k = yaml.safe_load(f) or {}
    docs: List[dict] = []
    for r in k.get("resources") or []:
        p = os.path.join(path, r)
        if os.path.isdir(p):
            docs += build(p, _seen)
        else:
            with open(p) as f:
                docs += [d for d in yaml.safe_load_all(f) if d]
    for g in k.get("configMapGenerator") or []:
        data = {}
        for lit in g.get("literals") or []:
            kk, _, vv = lit.partition("=")
            data[kk] = vv
        for fn in g.get("files") or []:
            with open(os.path.join(path, fn)) as f:
                data[os.path.basename(fn)] = f.read()
        for envf in g.get("envs") or []:
            with open(os.path.join(path, envf)) as f:
                for line in f:
                    line = line.strip()
                    if line and not line.startswith("#") and "=" in line:
                        kk, _, vv = line.partition("=")
                        data[kk] = vv
        docs.append({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": g["name"]}, "data": data})
    for p in k.get("patchesStrategicMerge") or k.get("patches") or []:
        if isinstance(p, dict):
            p = p.get("path")
        with open(os.path.join(path, p)) as f:
            patch = yaml.safe_load(f)
        for d in docs:
            if d.get("kind") == patch.get("kind") and d["metadata"]["name"] == patch["metadata"]["name"]:
                _merge(d, patch)
    ns = k.get("namespace")
    labels = k.get("commonLabels") or {}
    images = {i["name"]: i for i in k.get("images") or []}
    for d in docs:
        if ns and d.get("kind") not in ("CustomResourceDefinition", "ClusterRole", "ClusterRoleBinding", "Namespace",
                                         "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"):
            d["metadata"]["namespace"] = ns
        if ns and d.get("kind") in ("ClusterRoleBinding",):
            for s in d.get("subjects") or []:
                if s.get("kind") == "ServiceAccount":
                    s["namespace"] = ns
        if labels:
            d["metadata"].setdefault("labels", {}).update(labels)
        for ctr in _containers(d):
            base, _, _ = ctr.get("image", "").partition(":")
            if base in images:
                im = images[base]
                ctr["image"] = f"{im.get('newName', base)}:{im.get('newTag', 'latest')}"
    return docs


def _containers(d):
    spec = ((d.get("spec") or {}).get("template") or {}).get("spec") or {}
    return list(spec.get("containers") or []) + list(spec.get("initContainers") or [])


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        elif isinstance(v, list) and isinstance(dst.get(k), list) and v and isinstance(v[0], dict) and "name" in v[0]:
            byname = {x.get("name"): x for x in dst[k] if isinstance(x, dict)}
            for item in v:
                if item.get("name") in byname:
                    _merge(byname[item["name"]], item)
                else:
                    dst[k].append(copy.deepcopy(item))
        else:
            dst[k] = copy.deepcopy(v)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in ("generate", "build"):
        print(__doc__)
        return 2
    if argv[0] == "generate":
        generate(argv[1] if len(argv) > 1 else "manifests")
        return 0
    yaml.dump_all(build(argv[1]), sys.stdout, Dumper=NoAliasDumper, sort_keys=False)
    return 0


if __name__ == "__main__":
    sys.exit(main())
