"""Property-based tests (hypothesis) for the control plane's core algebra -- the SURVEY §5
"race detection / sanitizers" row: the reference has none; here the patch / selector / naming
logic every controller relies on is checked on generated inputs."""
import copy

from hypothesis import given, settings, strategies as st

from service_account_auth_improvements_amd.controlplane.apiserver import (create_json_patch, json_patch,
                                                                          labels_match, merge_patch)
from service_account_auth_improvements_amd.controlplane.kfam import binding_name

keys = st.text(alphabet="abcxyz/~-_.", min_size=1, max_size=6)
scalars = st.one_of(st.none(), st.booleans(), st.integers(-5, 5), st.text(max_size=4))
json_docs = st.recursive(scalars, lambda ch: st.one_of(st.lists(ch, max_size=3),
                                                       st.dictionaries(keys, ch, max_size=4)), max_leaves=12)
objects = st.dictionaries(keys, json_docs, max_size=5)


@settings(max_examples=300, deadline=None)
@given(objects, objects)
def test_json_patch_roundtrip(a, b):
    """apply(diff(a, b), a) == b for any two documents (the webhook response path)."""
    assert json_patch(a, create_json_patch(a, b)) == b


@settings(max_examples=300, deadline=None)
@given(objects, objects)
def test_merge_patch_rfc7386(target, patch):
    out = merge_patch(copy.deepcopy(target), patch)
    for k, v in patch.items():
        if v is None:
            assert k not in out                         # null deletes
        elif not isinstance(v, dict):
            assert out[k] == v                          # non-objects replace
    for k in target:
        if k not in patch:
            assert out[k] == target[k]                  # untouched keys survive
    assert merge_patch(copy.deepcopy(out), patch) == out   # idempotent


label_keys = st.sampled_from(["app", "tier", "notebook-name", "team"])
label_vals = st.sampled_from(["a", "b", "c"])


@settings(max_examples=300, deadline=None)
@given(st.dictionaries(label_keys, label_vals, max_size=4), st.dictionaries(label_keys, label_vals, max_size=3))
def test_equality_selector_semantics(labels, sel):
    s = ",".join(f"{k}={v}" for k, v in sel.items())
    assert labels_match(labels, s) == all(labels.get(k) == v for k, v in sel.items())
    # set-based forms agree with their definitions
    for k, v in sel.items():
        assert labels_match(labels, f"{k} in ({v})") == (labels.get(k) == v)
        assert labels_match(labels, f"{k} notin ({v})") == (labels.get(k) != v)
        assert labels_match(labels, k) == (k in labels)
        assert labels_match(labels, f"!{k}") == (k not in labels)


@settings(max_examples=300, deadline=None)
@given(st.emails(), st.sampled_from(["admin", "edit", "view"]), st.sampled_from(["User", "Group"]))
def test_kfam_binding_name_is_a_valid_k8s_name(user, role, kind):
    n = binding_name({"user": {"kind": kind, "name": user}, "referredNamespace": "ns",
                      "roleRef": {"kind": "ClusterRole", "name": role}})
    assert n == n.lower() and len(n) > 0
    assert all(ch.isalnum() or ch == "-" for ch in n)
    assert n.endswith(role)
