"""Kubernetes core/v1 types (the 1.24 API the reference's controller-runtime generations
target) as structural OpenAPI v3 schemas, for the CRDs that embed them: the Notebook's
``spec.template.spec`` is a full ``PodSpec`` (reference
components/notebook-controller/api/v1/notebook_types.go:26-30), the PodDefault spec
carries Containers, Volumes, EnvVars, Tolerations ... (components/admission-webhook/pkg/apis/
settings/v1alpha1/poddefault_types.go:27-125), and the job CRDs' replica templates are
PodTemplateSpecs.

Each type is a compact table: field -> type expression (``string``, ``int32``, ``int64``,
``bool``, ``number``, ``quantity`` / ``intstr`` (int-or-string), ``[]T`` for lists, ``{}T``
for string-keyed maps, or another type's name); ``!`` lists required fields, ``%`` holds
enums.  :func:`schema` expands a type into an alias-free schema tree (every node is a fresh
dict, so YAML dumps carry no anchors).  Nothing is left as ``x-kubernetes-preserve-unknown-
fields``: a misspelt pod field is rejected by the API server's schema validation
(controlplane/apiserver.py) as by a real one.
"""
from __future__ import annotations

import copy
from typing import Dict

PRIM = {
    "string": {"type": "string"},
    "int32": {"type": "integer", "format": "int32"},
    "int64": {"type": "integer", "format": "int64"},
    "bool": {"type": "boolean"},
    "number": {"type": "number"},
    "quantity": {"anyOf": [{"type": "integer"}, {"type": "string"}], "x-kubernetes-int-or-string": True},
    "intstr": {"anyOf": [{"type": "integer"}, {"type": "string"}], "x-kubernetes-int-or-string": True},
    "object": {"type": "object"},
}

_HANDLER = {"exec": "ExecAction", "httpGet": "HTTPGetAction", "tcpSocket": "TCPSocketAction"}
_KEY_TO_PATH = {"key": "string", "path": "string", "mode": "int32", "!": ["key", "path"]}
_SEC_REF = "LocalObjectReference"

TYPES: Dict[str, dict] = {
    # ---- references / selectors
    "LocalObjectReference": {"name": "string"},
    "SecretReference": {"name": "string", "namespace": "string"},
    "ObjectFieldSelector": {"apiVersion": "string", "fieldPath": "string", "!": ["fieldPath"]},
    "ResourceFieldSelector": {"containerName": "string", "divisor": "quantity", "resource": "string",
                              "!": ["resource"]},
    "ConfigMapKeySelector": {"key": "string", "name": "string", "optional": "bool", "!": ["key"]},
    "SecretKeySelector": {"key": "string", "name": "string", "optional": "bool", "!": ["key"]},
    "LabelSelectorRequirement": {"key": "string", "operator": "string", "values": "[]string",
                                 "!": ["key", "operator"]},
    "LabelSelector": {"matchExpressions": "[]LabelSelectorRequirement", "matchLabels": "{}string"},
    "NodeSelectorRequirement": {"key": "string", "operator": "string", "values": "[]string",
                                "!": ["key", "operator"]},
    "NodeSelectorTerm": {"matchExpressions": "[]NodeSelectorRequirement",
                         "matchFields": "[]NodeSelectorRequirement"},
    "NodeSelector": {"nodeSelectorTerms": "[]NodeSelectorTerm", "!": ["nodeSelectorTerms"]},
    "TypedLocalObjectReference": {"apiGroup": "string", "kind": "string", "name": "string",
                                  "!": ["kind", "name"]},
    # ---- env
    "EnvVarSource": {"configMapKeyRef": "ConfigMapKeySelector", "fieldRef": "ObjectFieldSelector",
                     "resourceFieldRef": "ResourceFieldSelector", "secretKeyRef": "SecretKeySelector"},
    "EnvVar": {"name": "string", "value": "string", "valueFrom": "EnvVarSource", "!": ["name"]},
    "ConfigMapEnvSource": {"name": "string", "optional": "bool"},
    "SecretEnvSource": {"name": "string", "optional": "bool"},
    "EnvFromSource": {"configMapRef": "ConfigMapEnvSource", "prefix": "string", "secretRef": "SecretEnvSource"},
    # ---- container
    "ExecAction": {"command": "[]string"},
    "HTTPHeader": {"name": "string", "value": "string", "!": ["name", "value"]},
    "HTTPGetAction": {"host": "string", "httpHeaders": "[]HTTPHeader", "path": "string", "port": "intstr",
                      "scheme": "string", "!": ["port"]},
    "TCPSocketAction": {"host": "string", "port": "intstr", "!": ["port"]},
    "GRPCAction": {"port": "int32", "service": "string", "!": ["port"]},
    "LifecycleHandler": dict(_HANDLER),
    "Lifecycle": {"postStart": "LifecycleHandler", "preStop": "LifecycleHandler"},
    "Probe": dict(_HANDLER, grpc="GRPCAction", failureThreshold="int32", initialDelaySeconds="int32",
                  periodSeconds="int32", successThreshold="int32", terminationGracePeriodSeconds="int64",
                  timeoutSeconds="int32"),
    "ContainerPort": {"containerPort": "int32", "hostIP": "string", "hostPort": "int32", "name": "string",
                      "protocol": "string", "!": ["containerPort"], "%": {"protocol": ["TCP", "UDP", "SCTP"]}},
    "ResourceRequirements": {"limits": "{}quantity", "requests": "{}quantity"},
    "Capabilities": {"add": "[]string", "drop": "[]string"},
    "SELinuxOptions": {"level": "string", "role": "string", "type": "string", "user": "string"},
    "SeccompProfile": {"localhostProfile": "string", "type": "string", "!": ["type"]},
    "WindowsSecurityContextOptions": {"gmsaCredentialSpec": "string", "gmsaCredentialSpecName": "string",
                                      "hostProcess": "bool", "runAsUserName": "string"},
    "SecurityContext": {"allowPrivilegeEscalation": "bool", "capabilities": "Capabilities", "privileged": "bool",
                        "procMount": "string", "readOnlyRootFilesystem": "bool", "runAsGroup": "int64",
                        "runAsNonRoot": "bool", "runAsUser": "int64", "seLinuxOptions": "SELinuxOptions",
                        "seccompProfile": "SeccompProfile", "windowsOptions": "WindowsSecurityContextOptions"},
    "VolumeDevice": {"devicePath": "string", "name": "string", "!": ["devicePath", "name"]},
    "VolumeMount": {"mountPath": "string", "mountPropagation": "string", "name": "string", "readOnly": "bool",
                    "subPath": "string", "subPathExpr": "string", "!": ["mountPath", "name"]},
    "Container": {"args": "[]string", "command": "[]string", "env": "[]EnvVar", "envFrom": "[]EnvFromSource",
                  "image": "string", "imagePullPolicy": "string", "lifecycle": "Lifecycle",
                  "livenessProbe": "Probe", "name": "string", "ports": "[]ContainerPort",
                  "readinessProbe": "Probe", "resources": "ResourceRequirements",
                  "securityContext": "SecurityContext", "startupProbe": "Probe", "stdin": "bool",
                  "stdinOnce": "bool", "terminationMessagePath": "string", "terminationMessagePolicy": "string",
                  "tty": "bool", "volumeDevices": "[]VolumeDevice", "volumeMounts": "[]VolumeMount",
                  "workingDir": "string", "!": ["name"],
                  "%": {"imagePullPolicy": ["Always", "Never", "IfNotPresent"]}},
    # ---- volumes
    "KeyToPath": dict(_KEY_TO_PATH),
    "DownwardAPIVolumeFile": {"fieldRef": "ObjectFieldSelector", "mode": "int32", "path": "string",
                              "resourceFieldRef": "ResourceFieldSelector", "!": ["path"]},
    "ConfigMapProjection": {"items": "[]KeyToPath", "name": "string", "optional": "bool"},
    "SecretProjection": {"items": "[]KeyToPath", "name": "string", "optional": "bool"},
    "DownwardAPIProjection": {"items": "[]DownwardAPIVolumeFile"},
    "ServiceAccountTokenProjection": {"audience": "string", "expirationSeconds": "int64", "path": "string",
                                      "!": ["path"]},
    "VolumeProjection": {"configMap": "ConfigMapProjection", "downwardAPI": "DownwardAPIProjection",
                         "secret": "SecretProjection", "serviceAccountToken": "ServiceAccountTokenProjection"},
    "PersistentVolumeClaimSpec": {"accessModes": "[]string", "dataSource": "TypedLocalObjectReference",
                                  "dataSourceRef": "TypedLocalObjectReference",
                                  "resources": "ResourceRequirements", "selector": "LabelSelector",
                                  "storageClassName": "string", "volumeMode": "string", "volumeName": "string"},
    "PersistentVolumeClaimTemplate": {"metadata": "object", "spec": "PersistentVolumeClaimSpec", "!": ["spec"]},
    "Volume": {
        "name": "string", "!": ["name"],
        "awsElasticBlockStore": {"fsType": "string", "partition": "int32", "readOnly": "bool", "volumeID": "string",
                                 "!": ["volumeID"]},
        "azureDisk": {"cachingMode": "string", "diskName": "string", "diskURI": "string", "fsType": "string",
                      "kind": "string", "readOnly": "bool", "!": ["diskName", "diskURI"]},
        "azureFile": {"readOnly": "bool", "secretName": "string", "shareName": "string",
                      "!": ["secretName", "shareName"]},
        "cephfs": {"monitors": "[]string", "path": "string", "readOnly": "bool", "secretFile": "string",
                   "secretRef": _SEC_REF, "user": "string", "!": ["monitors"]},
        "cinder": {"fsType": "string", "readOnly": "bool", "secretRef": _SEC_REF, "volumeID": "string",
                   "!": ["volumeID"]},
        "configMap": {"defaultMode": "int32", "items": "[]KeyToPath", "name": "string", "optional": "bool"},
        "csi": {"driver": "string", "fsType": "string", "nodePublishSecretRef": _SEC_REF, "readOnly": "bool",
                "volumeAttributes": "{}string", "!": ["driver"]},
        "downwardAPI": {"defaultMode": "int32", "items": "[]DownwardAPIVolumeFile"},
        "emptyDir": {"medium": "string", "sizeLimit": "quantity"},
        "ephemeral": {"volumeClaimTemplate": "PersistentVolumeClaimTemplate"},
        "fc": {"fsType": "string", "lun": "int32", "readOnly": "bool", "targetWWNs": "[]string", "wwids": "[]string"},
        "flexVolume": {"driver": "string", "fsType": "string", "options": "{}string", "readOnly": "bool",
                       "secretRef": _SEC_REF, "!": ["driver"]},
        "flocker": {"datasetName": "string", "datasetUUID": "string"},
        "gcePersistentDisk": {"fsType": "string", "partition": "int32", "pdName": "string", "readOnly": "bool",
                              "!": ["pdName"]},
        "gitRepo": {"directory": "string", "repository": "string", "revision": "string", "!": ["repository"]},
        "glusterfs": {"endpoints": "string", "path": "string", "readOnly": "bool", "!": ["endpoints", "path"]},
        "hostPath": {"path": "string", "type": "string", "!": ["path"]},
        "iscsi": {"chapAuthDiscovery": "bool", "chapAuthSession": "bool", "fsType": "string",
                  "initiatorName": "string", "iqn": "string", "iscsiInterface": "string", "lun": "int32",
                  "portals": "[]string", "readOnly": "bool", "secretRef": _SEC_REF, "targetPortal": "string",
                  "!": ["iqn", "lun", "targetPortal"]},
        "nfs": {"path": "string", "readOnly": "bool", "server": "string", "!": ["path", "server"]},
        "persistentVolumeClaim": {"claimName": "string", "readOnly": "bool", "!": ["claimName"]},
        "photonPersistentDisk": {"fsType": "string", "pdID": "string", "!": ["pdID"]},
        "portworxVolume": {"fsType": "string", "readOnly": "bool", "volumeID": "string", "!": ["volumeID"]},
        "projected": {"defaultMode": "int32", "sources": "[]VolumeProjection"},
        "quobyte": {"group": "string", "readOnly": "bool", "registry": "string", "tenant": "string",
                    "user": "string", "volume": "string", "!": ["registry", "volume"]},
        "rbd": {"fsType": "string", "image": "string", "keyring": "string", "monitors": "[]string", "pool": "string",
                "readOnly": "bool", "secretRef": _SEC_REF, "user": "string", "!": ["image", "monitors"]},
        "scaleIO": {"fsType": "string", "gateway": "string", "protectionDomain": "string", "readOnly": "bool",
                    "secretRef": _SEC_REF, "sslEnabled": "bool", "storageMode": "string", "storagePool": "string",
                    "system": "string", "volumeName": "string", "!": ["gateway", "secretRef", "system"]},
        "secret": {"defaultMode": "int32", "items": "[]KeyToPath", "optional": "bool", "secretName": "string"},
        "storageos": {"fsType": "string", "readOnly": "bool", "secretRef": _SEC_REF, "volumeName": "string",
                      "volumeNamespace": "string"},
        "vsphereVolume": {"fsType": "string", "storagePolicyID": "string", "storagePolicyName": "string",
                          "volumePath": "string", "!": ["volumePath"]},
    },
    # ---- scheduling
    "Toleration": {"effect": "string", "key": "string", "operator": "string", "tolerationSeconds": "int64",
                   "value": "string",
                   "%": {"operator": ["Exists", "Equal"], "effect": ["NoSchedule", "PreferNoSchedule", "NoExecute", ""]}},
    "PreferredSchedulingTerm": {"preference": "NodeSelectorTerm", "weight": "int32", "!": ["preference", "weight"]},
    "NodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": "[]PreferredSchedulingTerm",
                     "requiredDuringSchedulingIgnoredDuringExecution": "NodeSelector"},
    "PodAffinityTerm": {"labelSelector": "LabelSelector", "namespaceSelector": "LabelSelector",
                        "namespaces": "[]string", "topologyKey": "string", "!": ["topologyKey"]},
    "WeightedPodAffinityTerm": {"podAffinityTerm": "PodAffinityTerm", "weight": "int32",
                                "!": ["podAffinityTerm", "weight"]},
    "PodAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": "[]WeightedPodAffinityTerm",
                    "requiredDuringSchedulingIgnoredDuringExecution": "[]PodAffinityTerm"},
    "Affinity": {"nodeAffinity": "NodeAffinity", "podAffinity": "PodAffinity", "podAntiAffinity": "PodAffinity"},
    "TopologySpreadConstraint": {"labelSelector": "LabelSelector", "maxSkew": "int32", "topologyKey": "string",
                                 "whenUnsatisfiable": "string", "!": ["maxSkew", "topologyKey", "whenUnsatisfiable"]},
    # ---- pod
    "PodDNSConfigOption": {"name": "string", "value": "string"},
    "PodDNSConfig": {"nameservers": "[]string", "options": "[]PodDNSConfigOption", "searches": "[]string"},
    "HostAlias": {"hostnames": "[]string", "ip": "string"},
    "PodOS": {"name": "string", "!": ["name"]},
    "PodReadinessGate": {"conditionType": "string", "!": ["conditionType"]},
    "Sysctl": {"name": "string", "value": "string", "!": ["name", "value"]},
    "PodSecurityContext": {"fsGroup": "int64", "fsGroupChangePolicy": "string", "runAsGroup": "int64",
                           "runAsNonRoot": "bool", "runAsUser": "int64", "seLinuxOptions": "SELinuxOptions",
                           "seccompProfile": "SeccompProfile", "supplementalGroups": "[]int64",
                           "sysctls": "[]Sysctl", "windowsOptions": "WindowsSecurityContextOptions"},
    "PodSpec": {"activeDeadlineSeconds": "int64", "affinity": "Affinity", "automountServiceAccountToken": "bool",
                "containers": "[]Container", "dnsConfig": "PodDNSConfig", "dnsPolicy": "string",
                "enableServiceLinks": "bool", "ephemeralContainers": "[]EphemeralContainer",
                "hostAliases": "[]HostAlias", "hostIPC": "bool", "hostNetwork": "bool", "hostPID": "bool",
                "hostname": "string", "imagePullSecrets": "[]LocalObjectReference", "initContainers": "[]Container",
                "nodeName": "string", "nodeSelector": "{}string", "os": "PodOS", "overhead": "{}quantity",
                "preemptionPolicy": "string", "priority": "int32", "priorityClassName": "string",
                "readinessGates": "[]PodReadinessGate", "restartPolicy": "string", "runtimeClassName": "string",
                "schedulerName": "string", "securityContext": "PodSecurityContext", "serviceAccount": "string",
                "serviceAccountName": "string", "setHostnameAsFQDN": "bool", "shareProcessNamespace": "bool",
                "subdomain": "string", "terminationGracePeriodSeconds": "int64", "tolerations": "[]Toleration",
                "topologySpreadConstraints": "[]TopologySpreadConstraint", "volumes": "[]Volume",
                "!": ["containers"], "%": {"restartPolicy": ["Always", "OnFailure", "Never"]}},
    "ObjectMeta": {"annotations": "{}string", "labels": "{}string", "name": "string", "namespace": "string",
                   "generateName": "string"},
    "PodTemplateSpec": {"metadata": "ObjectMeta", "spec": "PodSpec"},
    # ---- status types
    "ContainerStateRunning": {"startedAt": "string"},
    "ContainerStateTerminated": {"containerID": "string", "exitCode": "int32", "finishedAt": "string",
                                 "message": "string", "reason": "string", "signal": "int32", "startedAt": "string",
                                 "!": ["exitCode"]},
    "ContainerStateWaiting": {"message": "string", "reason": "string"},
    "ContainerState": {"running": "ContainerStateRunning", "terminated": "ContainerStateTerminated",
                       "waiting": "ContainerStateWaiting"},
}
# an ephemeral container is a Container with the container it targets
TYPES["EphemeralContainer"] = dict(TYPES["Container"], targetContainerName="string")


def _expand(expr, overrides: dict):
    if isinstance(expr, dict):                      # an inline anonymous type
        return _object(expr, overrides)
    if expr.startswith("[]"):
        return {"type": "array", "items": _expand(expr[2:], overrides)}
    if expr.startswith("{}"):
        return {"type": "object", "additionalProperties": _expand(expr[2:], overrides)}
    if expr in PRIM:
        return copy.deepcopy(PRIM[expr])
    if expr in overrides:
        return copy.deepcopy(overrides[expr])
    return _object(TYPES[expr], overrides)


def _object(t: dict, overrides: dict) -> dict:
    props = {}
    enums = t.get("%", {})
    for k, v in t.items():
        if k in ("!", "%"):
            continue
        props[k] = _expand(v, overrides)
        if k in enums:
            props[k]["enum"] = list(enums[k])
    out = {"type": "object", "properties": props}
    if t.get("!"):
        out["required"] = list(t["!"])
    return out


def schema(type_name: str, required=None, **overrides) -> dict:
    """The structural schema of ``type_name``.  ``overrides`` replace a named type wherever it
    occurs (e.g. ``Container=`` a stricter container schema); ``required`` replaces the
    top-level required list."""
    s = _expand(type_name, overrides)
    if required is not None:
        if required:
            s["required"] = list(required)
        else:
            s.pop("required", None)
    return s


def container(required=("name",)) -> dict:
    return schema("Container", required=required)


def pod_spec(containers_min: int = 0, container_required=("name",)) -> dict:
    """PodSpec with the reference Notebook CRD's validation patches expressible here:
    ``containers`` minItems and per-container required fields
    (components/notebook-controller/config/crd/patches/validation_patches.yaml)."""
    s = schema("PodSpec", Container=container(container_required))
    if containers_min:
        s["properties"]["containers"]["minItems"] = containers_min
    else:
        s.pop("required", None)     # template pod specs may be filled in by a controller
    return s


def paths(s: dict, pre: str = "") -> set:
    """Every property path of a schema: ``.a.b``, ``[]`` for array items, ``{}`` for map values."""
    out = set()
    if not isinstance(s, dict):
        return out
    for k, v in (s.get("properties") or {}).items():
        p = f"{pre}.{k}"
        out.add(p)
        out |= paths(v, p)
    if isinstance(s.get("items"), dict):
        out |= paths(s["items"], pre + "[]")
    if isinstance(s.get("additionalProperties"), dict):
        out |= paths(s["additionalProperties"], pre + "{}")
    return out
