"""G7: idempotent get-or-create-then-diff-update helpers and field copiers
(reference: components/common/reconcilehelper/util.go:18-219).

``copy_*_fields(desired, found)`` copy the fields a controller owns from the desired
object onto the live one and return True when an update is required; everything else on
the live object (e.g. a Service's clusterIP, server-set metadata) is preserved.
"""
from __future__ import annotations

import copy
import logging
from typing import Callable

from .apiserver import ApiError
from .client import Client

log = logging.getLogger("reconcilehelper")


def _copy_meta_maps(desired: dict, found: dict) -> bool:
    upd = False
    dm, fm = desired.get("metadata", {}), found.setdefault("metadata", {})
    for key in ("labels", "annotations"):
        want = dm.get(key) or {}
        have = fm.get(key) or {}
        # like the reference: only changes/removals of keys already on the live object
        # force an update; the desired map is always assigned
        for k, v in have.items():
            if want.get(k) != v:
                upd = True
        fm[key] = copy.deepcopy(want)
    return upd


def copy_statefulset_fields(desired: dict, found: dict) -> bool:
    upd = _copy_meta_maps(desired, found)
    ds, fs = desired.get("spec", {}), found.setdefault("spec", {})
    if ds.get("replicas") != fs.get("replicas"):
        fs["replicas"] = ds.get("replicas")
        upd = True
    dt, ft = ds.get("template", {}).get("spec"), fs.setdefault("template", {}).get("spec")
    if dt != ft:
        upd = True
    fs["template"]["spec"] = copy.deepcopy(dt)
    return upd


def copy_deployment_fields(desired: dict, found: dict) -> bool:
    upd = _copy_meta_maps(desired, found)
    ds, fs = desired.get("spec", {}), found.setdefault("spec", {})
    if ds.get("replicas") != fs.get("replicas"):
        fs["replicas"] = ds.get("replicas")
        upd = True
    dt, ft = ds.get("template", {}).get("spec"), fs.setdefault("template", {}).get("spec")
    if dt != ft:
        upd = True
    fs["template"]["spec"] = copy.deepcopy(dt)
    if "strategy" in ds and ds["strategy"] != fs.get("strategy"):
        fs["strategy"] = copy.deepcopy(ds["strategy"])
        upd = True
    return upd


def copy_service_fields(desired: dict, found: dict) -> bool:
    """Selector and ports only -- never clusterIP (assigned by the apiserver)."""
    upd = _copy_meta_maps(desired, found)
    ds, fs = desired.get("spec", {}), found.setdefault("spec", {})
    if ds.get("selector") != fs.get("selector"):
        fs["selector"] = copy.deepcopy(ds.get("selector"))
        upd = True
    if ds.get("ports") != fs.get("ports"):
        fs["ports"] = copy.deepcopy(ds.get("ports"))
        upd = True
    return upd


def copy_virtual_service(desired: dict, found: dict) -> bool:
    """The whole spec."""
    if desired.get("spec") != found.get("spec"):
        found["spec"] = copy.deepcopy(desired.get("spec"))
        return True
    return False


def copy_generic_spec(desired: dict, found: dict) -> bool:
    upd = _copy_meta_maps(desired, found)
    if desired.get("spec") != found.get("spec"):
        found["spec"] = copy.deepcopy(desired.get("spec"))
        upd = True
    return upd


def reconcile_object(client: Client, desired: dict, copier: Callable[[dict, dict], bool]) -> dict:
    """Create ``desired`` if absent, else copy owned fields and update when they differ."""
    m = desired["metadata"]
    found = client.get_or_none(desired["apiVersion"], desired["kind"], m["name"], m.get("namespace"))
    if found is None:
        log.info("Creating %s %s/%s", desired["kind"], m.get("namespace"), m["name"])
        return client.create(desired)
    if copier(desired, found):
        log.info("Updating %s %s/%s", desired["kind"], m.get("namespace"), m["name"])
        return client.update(found)
    return found


def deployment(client: Client, desired: dict) -> dict:
    return reconcile_object(client, desired, copy_deployment_fields)


def service(client: Client, desired: dict) -> dict:
    return reconcile_object(client, desired, copy_service_fields)


def virtual_service(client: Client, desired: dict) -> dict:
    return reconcile_object(client, desired, copy_virtual_service)


def statefulset(client: Client, desired: dict) -> dict:
    return reconcile_object(client, desired, copy_statefulset_fields)
