"""G2 / G2a / G2b / G2d: Profile controller with WorkloadIdentity and
AwsIamForServiceAccount plugins (multi-tenancy: one owned namespace per Profile).

Behavioural reference: components/profile-controller/controllers/profile_controller.go:105-798,
plugin_workload_identity.go:39-160, plugin_iam.go:30-305, main.go:41-127.

Per Profile: Namespace (annotation ``owner``, label ``istio-injection=enabled`` plus the
hot-reloaded default labels file: an empty value removes a key, existing keys are never
overwritten), Istio AuthorizationPolicy ``ns-owner-access-istio``, ServiceAccounts
``default-editor`` / ``default-viewer`` bound to ``kubeflow-edit`` / ``kubeflow-view``,
owner RoleBinding ``namespaceAdmin`` -> ``kubeflow-admin``, optional ResourceQuota
``kf-resource-quota`` (e.g. ``amd.com/gpu: 8``), plugins, finalizer ``profile-finalizer``.
A namespace owned by someone else is never taken over (a ``Failed`` condition is added).

Cloud IAM calls sit behind the small ``IamBackend`` interface; the policy-document
manipulation is implemented here exactly.  The deployed controller talks to the real clouds
through ``controlplane/cloud_iam.py`` (GCP IAM REST with ADC tokens, AWS IAM Query API with
SigV4); ``InMemoryIam`` models both for the local cluster and tests.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import re
import threading
import time
from typing import Dict, List, Optional

import yaml

from .apiserver import ApiError, set_controller_reference
from .client import Client
from .monitoring import SEVERITY_MAJOR, RequestMetrics
from .runtime import Controller, Request, Result, for_kind, get_env_default, owns

log = logging.getLogger("profile-controller")

PROFILE_API = "kubeflow.org/v1"
AUTHZPOLICYISTIO = "ns-owner-access-istio"
KFQUOTA = "kf-resource-quota"
PROFILEFINALIZER = "profile-finalizer"
USER, ROLE, ADMIN = "user", "role", "admin"
KUBEFLOW_ADMIN, KUBEFLOW_EDIT, KUBEFLOW_VIEW = "kubeflow-admin", "kubeflow-edit", "kubeflow-view"
ISTIO_INJECTION_LABEL = "istio-injection"
DEFAULT_EDITOR, DEFAULT_VIEWER = "default-editor", "default-viewer"
DEFAULT_LABELS_PATH = "/etc/profile-controller/namespace-labels.yaml"

KIND_WORKLOAD_IDENTITY = "WorkloadIdentity"
GCP_ANNOTATION_KEY = "iam.gke.io/gcp-service-account"
GCP_SA_SUFFIX = ".iam.gserviceaccount.com"
WORKLOAD_IDENTITY_ROLE = "roles/iam.workloadIdentityUser"
KIND_AWS_IAM_FOR_SERVICE_ACCOUNT = "AwsIamForServiceAccount"
AWS_ANNOTATION_KEY = "eks.amazonaws.com/role-arn"
AWS_TRUST_IDENTITY_SUBJECT = "system:serviceaccount:{}:{}"
AWS_DEFAULT_AUDIENCE = "sts.amazonaws.com"


def set_namespace_labels(ns: dict, new_labels: Dict[str, str]):
    labels = ns["metadata"].setdefault("labels", {})
    for k, v in (new_labels or {}).items():
        if not v:
            labels.pop(k, None)
        elif k not in labels:
            labels[k] = v


def read_default_labels(path: str) -> Dict[str, str]:
    with open(path) as f:
        data = yaml.safe_load(f) or {}
    return {str(k): ("" if v is None else str(v)) for k, v in data.items()}


# ----------------------------------------------------------------------------- IAM backends
class IamBackend:
    """GCP: get/set the IAM policy of a service account resource.
       AWS: get/update the assume-role policy document of a role."""

    def gcp_get_policy(self, resource: str) -> dict: raise NotImplementedError
    def gcp_set_policy(self, resource: str, policy: dict): raise NotImplementedError
    def gcp_default_project(self) -> str: return ""
    def aws_get_assume_role_policy(self, role_name: str) -> str: raise NotImplementedError
    def aws_update_assume_role_policy(self, role_name: str, doc: str): raise NotImplementedError


class InMemoryIam(IamBackend):
    def __init__(self, project: str = ""):
        self.gcp: Dict[str, dict] = {}
        self.aws: Dict[str, str] = {}
        self.project = project

    def gcp_get_policy(self, resource):
        return copy.deepcopy(self.gcp.setdefault(resource, {"bindings": []}))

    def gcp_set_policy(self, resource, policy):
        self.gcp[resource] = copy.deepcopy(policy)

    def gcp_default_project(self):
        return self.project

    def aws_get_assume_role_policy(self, role_name):
        return self.aws[role_name]

    def aws_update_assume_role_policy(self, role_name, doc):
        self.aws[role_name] = doc


class ConditionExistError(Exception):
    pass


def _issuer_from_provider_arn(arn: str) -> str:
    return arn[arn.index("/") + 1:]


def _role_name_from_arn(arn: str) -> str:
    return arn[arn.rindex("/") + 1:]


def _assume_role_doc(provider_arn: str, condition: dict) -> dict:
    return {"Version": "2012-10-17",
            "Statement": [{"Effect": "Allow", "Action": "sts:AssumeRoleWithWebIdentity",
                           "Principal": {"Federated": provider_arn}, "Condition": condition}]}


def add_sa_to_assume_role_policy(doc: str, ns: str, sa: str) -> str:
    old = json.loads(doc)
    st = old["Statement"][0]
    provider = st["Principal"]["Federated"]
    issuer = _issuer_from_provider_arn(provider)
    key = f"{issuer}:sub"
    ident = AWS_TRUST_IDENTITY_SUBJECT.format(ns, sa)
    cur = (st.get("Condition") or {}).get("StringEquals", {}).get(key, [])
    if isinstance(cur, str):
        cur = [cur]
    if ident in cur:
        raise ConditionExistError()
    new = list(cur) + [ident]
    return json.dumps(_assume_role_doc(provider, {"StringEquals": {f"{issuer}:aud": [AWS_DEFAULT_AUDIENCE],
                                                                   key: new}}))


def remove_sa_from_assume_role_policy(doc: str, ns: str, sa: str) -> str:
    old = json.loads(doc)
    st = old["Statement"][0]
    provider = st["Principal"]["Federated"]
    issuer = _issuer_from_provider_arn(provider)
    key = f"{issuer}:sub"
    ident = AWS_TRUST_IDENTITY_SUBJECT.format(ns, sa)
    cur = (st.get("Condition") or {}).get("StringEquals", {}).get(key, [])
    if isinstance(cur, str):
        cur = [cur]
    new = [x for x in cur if x != ident]
    cond = {f"{issuer}:aud": [AWS_DEFAULT_AUDIENCE]}
    if new:
        cond[key] = new
    return json.dumps(_assume_role_doc(provider, {"StringEquals": cond}))


class GcpWorkloadIdentity:
    def __init__(self, spec: dict, iam: IamBackend):
        self.gcp_sa = spec.get("gcpServiceAccount", "")
        self.iam = iam

    def project_id(self) -> str:
        if not self.gcp_sa.endswith(GCP_SA_SUFFIX):
            raise ValueError(f"{self.gcp_sa} is not a valid GCP service account.")
        m = re.search(r"@(.*?)\.", self.gcp_sa)
        if not m:
            raise ValueError(f"Cannot extract project id from {self.gcp_sa}.")
        return m.group(1)

    def _update(self, ns: str, ksa: str, add: bool):
        pid = self.project_id()
        res = f"projects/{pid}/serviceAccounts/{self.gcp_sa}"
        pol = self.iam.gcp_get_policy(res)
        member = f"serviceAccount:{self.iam.gcp_default_project() or pid}.svc.id.goog[{ns}/{ksa}]"
        if add:
            pol.setdefault("bindings", []).append({"role": WORKLOAD_IDENTITY_ROLE, "members": [member]})
        else:
            for b in pol.get("bindings", []):
                if b.get("role") == WORKLOAD_IDENTITY_ROLE:
                    b["members"] = [m for m in b.get("members", []) if m != member]
        self.iam.gcp_set_policy(res, pol)

    def apply(self, client: Client, profile: dict):
        ns = profile["metadata"]["name"]
        sa = client.get("v1", "ServiceAccount", DEFAULT_EDITOR, ns)
        sa["metadata"].setdefault("annotations", {})[GCP_ANNOTATION_KEY] = self.gcp_sa
        client.update(sa)
        self._update(ns, DEFAULT_EDITOR, True)

    def revoke(self, client: Client, profile: dict):
        self._update(profile["metadata"]["name"], DEFAULT_EDITOR, False)


class AwsIamForServiceAccount:
    def __init__(self, spec: dict, iam: IamBackend):
        self.role_arn = spec.get("awsIamRole", "")
        self.annotate_only = bool(spec.get("annotateOnly", False))
        self.iam = iam

    def _annotate(self, client, ns, add: bool):
        sa = client.get("v1", "ServiceAccount", DEFAULT_EDITOR, ns)
        if not self.role_arn:
            raise ValueError("failed to setup service account because awsIamRole is empty")
        ann = sa["metadata"].setdefault("annotations", {})
        if add:
            ann[AWS_ANNOTATION_KEY] = self.role_arn
        else:
            ann.pop(AWS_ANNOTATION_KEY, None)
        client.update(sa)

    def _update(self, ns, fn):
        if self.annotate_only:
            return
        role = _role_name_from_arn(self.role_arn)
        doc = self.iam.aws_get_assume_role_policy(role)
        try:
            new = fn(doc, ns, DEFAULT_EDITOR)
        except ConditionExistError:
            return
        self.iam.aws_update_assume_role_policy(role, new)

    def apply(self, client, profile):
        ns = profile["metadata"]["name"]
        self._annotate(client, ns, True)
        self._update(ns, add_sa_to_assume_role_policy)

    def revoke(self, client, profile):
        ns = profile["metadata"]["name"]
        self._annotate(client, ns, False)
        self._update(ns, remove_sa_from_assume_role_policy)


# ----------------------------------------------------------------------------- controller
class ProfileReconciler(Controller):
    name = "profile-controller"

    def __init__(self, client: Client, user_id_header: str = "x-goog-authenticated-user-email",
                 user_id_prefix: str = "accounts.google.com:", workload_identity: str = "",
                 labels_path: str = DEFAULT_LABELS_PATH, iam: Optional[IamBackend] = None,
                 metrics: Optional[RequestMetrics] = None, ns_wait_retries: int = 5, ns_wait_s: float = 3.0):
        super().__init__(client)
        self.user_id_header, self.user_id_prefix = user_id_header, user_id_prefix
        self.workload_identity = workload_identity
        self.labels_path = labels_path
        self.iam = iam or InMemoryIam()
        self.metrics = metrics or RequestMetrics("profile_controller")
        self.ns_wait_retries, self.ns_wait_s = ns_wait_retries, ns_wait_s
        self.manager = None

    def sources(self):
        return [for_kind(PROFILE_API, "Profile"), owns("v1", "Namespace", "Profile"),
                owns("security.istio.io/v1beta1", "AuthorizationPolicy", "Profile"),
                owns("v1", "ServiceAccount", "Profile"),
                owns("rbac.authorization.k8s.io/v1", "RoleBinding", "Profile")]

    # labels file hot reload (fsnotify equivalent: mtime poll) -> re-reconcile every profile
    def watch_labels_file(self, manager, period: float = 1.0):
        self.manager = manager

        def loop():
            last = None
            while True:
                try:
                    m = os.stat(self.labels_path).st_mtime
                except OSError:
                    m = None
                if last is not None and m != last:
                    manager.enqueue_all(self.name, PROFILE_API, "Profile")
                last = m
                time.sleep(period)
        threading.Thread(target=loop, daemon=True).start()

    def authorization_policy(self, profile: dict) -> dict:
        owner = profile["spec"]["owner"]["name"]
        nb_ctrl = get_env_default("NOTEBOOK_CONTROLLER_PRINCIPAL",
                                  "cluster.local/ns/kubeflow/sa/notebook-controller-service-account")
        igw = get_env_default("ISTIO_INGRESS_GATEWAY_PRINCIPAL",
                              "cluster.local/ns/istio-system/sa/istio-ingressgateway-service-account")
        kfp_ui = get_env_default("KFP_UI_PRINCIPAL", "cluster.local/ns/kubeflow/sa/ml-pipeline-ui")
        return {"action": "ALLOW", "rules": [
            {"when": [{"key": f"request.headers[{self.user_id_header}]", "values": [self.user_id_prefix + owner]}],
             "from": [{"source": {"principals": [igw, kfp_ui]}}]},
            {"when": [{"key": "source.namespace", "values": [profile["metadata"]["name"]]}]},
            {"to": [{"operation": {"paths": ["/healthz", "/metrics", "/wait-for-drain"]}}]},
            {"from": [{"source": {"principals": [nb_ctrl]}}],
             "to": [{"operation": {"methods": ["GET"], "paths": ["*/api/kernels"]}}]}]}

    def _plugins(self, profile: dict):
        out = []
        for p in profile["spec"].get("plugins") or []:
            if p.get("kind") == KIND_WORKLOAD_IDENTITY:
                out.append(GcpWorkloadIdentity(p.get("spec") or {}, self.iam))
            elif p.get("kind") == KIND_AWS_IAM_FOR_SERVICE_ACCOUNT:
                out.append(AwsIamForServiceAccount(p.get("spec") or {}, self.iam))
        return out

    def _fail(self, profile: dict, message: str) -> Result:
        st = profile.setdefault("status", {})
        conds = st.setdefault("conditions", [])
        cond = {"type": "Failed", "status": "True", "message": message}
        if not conds or conds[-1] != cond:   # a repeated failure is recorded once
            conds.append(cond)
            self.client.update_status(profile)
        return Result()

    def _upsert(self, profile: dict, obj: dict, same):
        c = self.client
        set_controller_reference(profile, obj)
        m = obj["metadata"]
        found = c.get_or_none(obj["apiVersion"], obj["kind"], m["name"], m.get("namespace"))
        if found is None:
            return c.create(obj)
        if not same(obj, found):
            for k in ("spec", "roleRef", "subjects"):
                if k in obj:
                    found[k] = copy.deepcopy(obj[k])
            return c.update(found)
        return found

    def reconcile(self, req: Request) -> Result:
        c = self.client
        labels = read_default_labels(self.labels_path) if os.path.exists(self.labels_path) else {}
        profile = c.get_or_none(PROFILE_API, "Profile", req.name)
        if profile is None:
            self.metrics.inc_request("profile deletion")
            return Result()
        name = profile["metadata"]["name"]
        owner = profile["spec"]["owner"]
        if profile["metadata"].get("deletionTimestamp"):
            if PROFILEFINALIZER in (profile["metadata"].get("finalizers") or []):
                for p in self._plugins(profile):
                    p.revoke(c, profile)
                profile["metadata"]["finalizers"] = [f for f in profile["metadata"]["finalizers"]
                                                     if f != PROFILEFINALIZER]
                c.update(profile)
            return Result()
        # namespace
        ns = {"apiVersion": "v1", "kind": "Namespace",
              "metadata": {"name": name, "annotations": {"owner": owner["name"]},
                           "labels": {ISTIO_INJECTION_LABEL: "enabled"}}}
        set_namespace_labels(ns, labels)
        set_controller_reference(profile, ns)
        found = c.get_or_none("v1", "Namespace", name)
        if found is None:
            c.create(ns)
            for _ in range(self.ns_wait_retries):
                if c.get_or_none("v1", "Namespace", name) is not None:
                    break
                time.sleep(self.ns_wait_s)
            else:
                self.metrics.inc_error("error namespace create completion", SEVERITY_MAJOR)
                return self._fail(profile, "Owning namespace failed to create within 15 seconds")
        else:
            if (found["metadata"].get("annotations") or {}).get("owner") == owner["name"]:
                old = dict(found["metadata"].get("labels") or {})
                set_namespace_labels(found, labels)
                if found["metadata"].get("labels") != old:
                    c.update(found)
            else:
                self.metrics.inc_request("reject profile taking over existing namespace")
                return self._fail(profile, f"namespace already exist, but not owned by profile creator {owner['name']}")
        # istio authorization policy
        self._upsert(profile, {"apiVersion": "security.istio.io/v1beta1", "kind": "AuthorizationPolicy",
                               "metadata": {"name": AUTHZPOLICYISTIO, "namespace": name,
                                            "annotations": {USER: owner["name"], ROLE: ADMIN}},
                               "spec": self.authorization_policy(profile)},
                     lambda a, b: a["spec"] == b.get("spec"))
        rb_same = lambda a, b: a["roleRef"] == b.get("roleRef") and a["subjects"] == b.get("subjects")  # noqa
        for sa, role in ((DEFAULT_EDITOR, KUBEFLOW_EDIT), (DEFAULT_VIEWER, KUBEFLOW_VIEW)):
            if c.get_or_none("v1", "ServiceAccount", sa, name) is None:
                c.create(set_controller_reference(profile, {"apiVersion": "v1", "kind": "ServiceAccount",
                                                            "metadata": {"name": sa, "namespace": name}}))
            self._upsert(profile, {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                                   "metadata": {"name": sa, "namespace": name},
                                   "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                               "name": role},
                                   "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": name}]}, rb_same)
        self._upsert(profile, {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                               "metadata": {"name": "namespaceAdmin", "namespace": name,
                                            "annotations": {USER: owner["name"], ROLE: ADMIN}},
                               "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                           "name": KUBEFLOW_ADMIN},
                               "subjects": [owner]}, rb_same)
        hard = ((profile["spec"].get("resourceQuotaSpec") or {}).get("hard")) or {}
        if hard:
            self._upsert(profile, {"apiVersion": "v1", "kind": "ResourceQuota",
                                   "metadata": {"name": KFQUOTA, "namespace": name},
                                   "spec": copy.deepcopy(profile["spec"]["resourceQuotaSpec"])},
                         lambda a, b: a["spec"] == b.get("spec"))
        else:
            if c.get_or_none("v1", "ResourceQuota", KFQUOTA, name) is not None:
                c.delete("v1", "ResourceQuota", KFQUOTA, name)
        # default plugin patch (+ Update, as the reference)
        if self.workload_identity and not any(p.get("kind") == KIND_WORKLOAD_IDENTITY
                                              for p in profile["spec"].get("plugins") or []):
            profile["spec"].setdefault("plugins", []).append(
                {"kind": KIND_WORKLOAD_IDENTITY, "spec": {"gcpServiceAccount": self.workload_identity}})
            profile = c.update(profile)
        for p in self._plugins(profile):
            p.apply(c, profile)
        if PROFILEFINALIZER not in (profile["metadata"].get("finalizers") or []):
            profile = c.get(PROFILE_API, "Profile", name)
            profile["metadata"].setdefault("finalizers", []).append(PROFILEFINALIZER)
            c.update(profile)
        self.metrics.inc_request("reconcile")
        return Result()


def default_cluster_roles() -> List[dict]:
    """kubeflow-admin/edit/view ClusterRoles (kubeflow-roles manifests), incl. the new job
    CRDs; installed by the local cluster so SubjectAccessReviews have something to match."""
    edit_rules = [{"apiGroups": ["kubeflow.org"], "resources": ["notebooks", "notebooks/status", "poddefaults",
                                                                "pvcviewers", "pytorchjobs", "mpijobs"],
                   "verbs": ["get", "list", "watch", "create", "delete", "deletecollection", "patch", "update"]},
                  {"apiGroups": ["tensorboard.kubeflow.org"], "resources": ["tensorboards"],
                   "verbs": ["get", "list", "watch", "create", "delete", "patch", "update"]},
                  {"apiGroups": ["serving.kserve.io"], "resources": ["inferenceservices"],
                   "verbs": ["get", "list", "watch", "create", "delete", "patch", "update"]},
                  {"apiGroups": [""], "resources": ["persistentvolumeclaims", "pods", "pods/log", "events",
                                                    "services", "configmaps", "secrets"],
                   "verbs": ["get", "list", "watch", "create", "delete", "patch", "update"]}]
    view_rules = [dict(r, verbs=["get", "list", "watch"]) for r in edit_rules]
    admin_rules = edit_rules + [{"apiGroups": ["rbac.authorization.k8s.io"], "resources": ["rolebindings"],
                                 "verbs": ["*"]}]
    mk = lambda n, rules: {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",  # noqa
                           "metadata": {"name": n}, "rules": rules}
    return [mk(KUBEFLOW_ADMIN, admin_rules), mk(KUBEFLOW_EDIT, edit_rules), mk(KUBEFLOW_VIEW, view_rules)]
