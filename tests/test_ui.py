"""Web UI (T2-T7): the JavaScript sources parse (node --check), every app's pages render and behave in a
small DOM (tests/js/dom_shim.js + ui_pages.js: tables, forms, dialogs, routes, errors), the common-lib logic
(static/lib/kf-logic.js) behaves as the reference kubeflow-common-lib / JWA / VWA frontends do
(run under node), and the JWA create body the UI generates is accepted by the real JWA backend."""
import json
import os
import shutil
import subprocess

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STATIC = os.path.join(ROOT, "service_account_auth_improvements_amd", "webapps", "static")
pytestmark = pytest.mark.skipif(shutil.which("node") is None, reason="node not available")


@pytest.fixture(scope="module")
def out():
    r = subprocess.run(["node", os.path.join(ROOT, "tests", "js", "kf_logic_cases.js")], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


@pytest.mark.parametrize("f", ["kfamd-ui.js", "dashboard-ng.js", "lib/kf-common.js", "lib/kf-logic.js"])
def test_js_sources_parse(f):
    r = subprocess.run(["node", "--check", os.path.join(STATIC, f)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr


def test_every_app_page_loads_the_shared_libs():
    for app in ("jupyter", "volumes", "tensorboards", "dashboard"):
        html = open(os.path.join(STATIC, app, "index.html")).read()
        i, j, k = (html.index(s) for s in ("lib/kf-logic.js", "lib/kf-common.js", "kfamd-ui.js\""))
        assert i < j < k and f'data-app="{app}"' in html


def test_poller_and_backoff(out):
    assert out["poll"] == [1000, 2000, 4000, 8000, 8000, 1000, 2000]     # PollerService.exponential
    assert out["backoff"] == [1000, 2000, 4000, 8000, 16000, 16000] and out["backoffReset"] == 1000


def test_validators_and_env(out):
    assert out["names"][0] == "" and out["names"][5] == ""
    assert all(out["names"][i] for i in (1, 2, 3, 4))
    assert [bool(x) for x in out["quantities"]] == [False, False, False, True, False]
    assert out["env"] == {"A": "1", "B": " two=2"} and "not KEY=VALUE" in out["envErr"]
    assert out["route"] == [{"page": "details", "args": ["ns1", "nb 1"]}, {"page": "index", "args": []},
                            {"page": "new", "args": []}]


def test_form_body_shape(out):
    b = out["body"]
    assert "shm" not in b                       # readOnly in the spawner config: never sent
    assert b["gpus"] == {"num": "1", "vendor": "amd.com/gpu"} and b["environment"] == {"HIP_VISIBLE_DEVICES": "0"}
    assert b["workspace"]["newPvc"]["metadata"]["name"] == "nb1-workspace"
    assert b["datavols"][0] == {"mount": "/data", "existingSource": {"persistentVolumeClaim": {"claimName": "data"}}}
    assert b["datavols"][1]["newPvc"]["spec"]["resources"]["requests"]["storage"] == "20Gi"
    assert out["formErrors"] == []
    errs = " | ".join(out["badFormErrors"])
    for want in ("lower case", "CPU limit must be greater", "memory: Invalid quantity", "mount path used twice",
                 "needs a name"):
        assert want in errs, errs
    cb = out["customBody"]
    assert cb["customImage"] == "rocm/pytorch:latest" and "image" not in cb and cb["gpus"] == {"num": "none"}
    assert "workspace" not in cb


def test_ui_generated_bodies_are_accepted_by_the_jwa_backend(out):
    from test_webapps import USER, _csrf, cluster  # noqa: F401
    from service_account_auth_improvements_amd.controlplane.apiserver import APIServer
    from service_account_auth_improvements_amd.controlplane.client import InMemoryClient
    from service_account_auth_improvements_amd.controlplane.profile import default_cluster_roles
    from service_account_auth_improvements_amd.webapps import jupyter
    c = InMemoryClient(APIServer())
    for cr in default_cluster_roles():
        c.create(cr)
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "alice"}})
    c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
              "metadata": {"name": "namespaceAdmin", "namespace": "alice"},
              "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "kubeflow-admin"},
              "subjects": [{"apiGroup": "rbac.authorization.k8s.io", "kind": "User", "name": "alice@example.com"}]})
    c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "data", "namespace": "alice"},
              "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}})
    tc = jupyter.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    h = dict(USER, **_csrf(tc))
    body = dict(out["body"])
    body["shm"] = True         # the dev spawner config is not readOnly for shm: the form sends it there
    r = tc.post("/api/namespaces/alice/notebooks", json=body, headers=h)
    assert r.status_code == 200, r.json
    nb = c.get("kubeflow.org/v1beta1", "Notebook", "nb1", "alice")
    ctr = nb["spec"]["template"]["spec"]["containers"][0]
    assert ctr["resources"]["limits"]["amd.com/gpu"] == "1"
    assert {"name": "HIP_VISIBLE_DEVICES", "value": "0"} in ctr["env"]
    assert {m["mountPath"] for m in ctr["volumeMounts"]} == {"/dev/shm", "/data", "/scratch", "/home/jovyan"}
    assert c.get("v1", "PersistentVolumeClaim", "scratch", "alice")
    r = tc.post("/api/namespaces/alice/notebooks", json=out["customBody"], headers=h)
    assert r.status_code == 200, r.json
    assert c.get("kubeflow.org/v1beta1", "Notebook", "nb2", "alice")["spec"]["template"]["spec"]["containers"][0][
        "image"] == "rocm/pytorch:latest"


def test_volume_details_groups_pods_by_owner(out):
    assert out["groups"] == [
        {"name": "Notebooks", "links": [{"name": "nb1", "url": "https://kf.example.com/jupyter/notebook/details/alice/nb1/"}]},
        {"name": "InferenceService", "links": [
            {"name": "llm (predictor)", "url": "https://kf.example.com/models/details/alice/llm/"},
            {"name": "old (transformer)", "url": "https://kf.example.com/models/details/alice/old/"}]}]


def test_details_overview_conditions_and_yaml(out):
    o = out["overview"]
    assert o["gpus"] == ["1 x amd.com/gpu"] and o["configurations"] == ["add-gpu-env"]
    assert o["cpu"] == "2" and o["cpuLimit"] == "2.4" and o["creator"] == "alice@example.com"
    assert {"name": "dshm", "source": "emptyDir (Memory)", "mount": "/dev/shm"} in o["volumes"]
    assert out["conditions"][0]["lastTransitionTime"] == "2024-01-01T00:00:00Z"
    assert yaml.safe_load(out["yaml"]) == out["yamlInput"]          # the YAML tab round-trips
    assert out["age"] == ["30s", "2d"]


# ---------------------------------------------------------------- the pages themselves
# tests/js/ui_pages.js renders every app's pages in a small DOM (tests/js/dom_shim.js) against
# fixtures shaped like the reference Cypress fixtures, clicks and types like a user, and reports
# what the DOM shows and what the page sent.  The cases mirror
# crud-web-apps/jupyter/frontend/cypress/e2e/{main-page,form-page}.cy.ts and the central
# dashboard's guard / interceptor / 404 behaviour (centraldashboard-angular/frontend/src/app).
@pytest.fixture(scope="module")
def pages(tmp_path_factory):
    cfg = yaml.safe_load(open(os.path.join(ROOT, "service_account_auth_improvements_amd", "webapps", "config",
                                           "spawner_ui_config.yaml")))["spawnerFormDefaults"]
    p = tmp_path_factory.mktemp("ui") / "config.json"
    p.write_text(json.dumps(cfg))
    r = subprocess.run(["node", os.path.join(ROOT, "tests", "js", "ui_pages.js"), str(p)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_jwa_main_table(pages):
    o = pages["jwaIndex"]
    assert o["title"] == "Notebooks" and o["errorSnacks"] == []
    assert o["names"] == sorted(o["names"]) == ["alpha-analysis", "mid-codeserver", "zeta-trainer"]   # by Name
    assert o["statusClasses"] == ["st st-stopped", "st st-warning", "st st-ready"]
    assert o["gpus"] == ["-", "-", "1 AMD"] and not o["namespaceColumn"]
    assert o["requested"][-1] == "GET api/namespaces/kubeflow-user/notebooks"


def test_jwa_all_namespaces_and_sorting(pages):
    o = pages["jwaAll"]
    assert o["namespaceColumn"] and "beta-decode" in o["names"]
    assert dict(zip(o["names"], o["namespaces"]))["beta-decode"] == "team-b"
    assert o["namesDesc"] == sorted(o["names"], reverse=True)


def test_app_takes_namespace_only_from_its_parent_frame_origin(pages):
    """kf-common.js iframe protocol: a namespace-selected message from another origin, with an
    empty origin, or from a window that is not the embedding dashboard is ignored."""
    o = pages["jwaIframeNs"]
    assert o["ignored"] == "kubeflow-user" and o["accepted"] == "team-b"


def test_delete_goes_through_the_confirm_dialog(pages):
    d = pages["jwaDelete"]
    assert d["dialogTitle"] == "Delete Notebook zeta-trainer?" and d["afterCancel"] == 0
    assert d["deletes"] == ["api/namespaces/kubeflow-user/notebooks/zeta-trainer"] and not d["dialogOpen"]
    v = pages["vwa"]         # a failed delete keeps the dialog open with the backend's message
    assert v["names"] == ["checkpoints", "datasets"] and v["usedBy"] == ["-", "zeta-trainer"]
    assert v["dialogStillOpen"] and "used by pod zeta-trainer-0" in v["dialogError"]
    assert v["buttons"][:2] == ["Browse", "Delete"] and "Open viewer" in v["buttons"]


def test_vwa_form_storage_classes_and_existing_names(pages):
    """Volume form (ref volumes/frontend pages/form/form-default): the cluster's storage classes
    with the backend's default preselected and "None" as {none}; an existing name is refused in
    the page (no request); a new one POSTs the body the VWA backend takes."""
    v = pages["vwa"]
    assert v["classOptions"] == ["{empty}", "{none}", "fast-nvme", "standard"] and v["classSelected"] == "standard"
    assert v["dupPosts"] == 0 and any("already exists" in s[1] for s in v["dupSnacks"])
    assert v["posts"] == [{"name": "scratch", "mode": "ReadWriteOnce", "class": "standard", "size": "10Gi", "type": "new"}]


def test_jwa_form_drives_names_and_mounts_and_posts_the_body(pages):
    f = pages["jwaForm"]
    assert f["title"] == "New notebook"
    # '{notebook-name}-workspace' from the spawner config, following the name field
    assert f["workspaceInitial"] == "-workspace" and f["workspaceFollowsName"] == "nb1-workspace"
    assert f["workspaceHeader"] == "nb1-workspace"
    assert f["mountAuto"] == "/home/jovyan/new-volume-name" and f["mountDirty"] == "/data/dirty"
    assert f["gpuVendors"] == ["AMD Instinct MI355X"]
    assert f["posts"] == ["api/namespaces/kubeflow-user/notebooks"] and f["hashAfter"] == "#/"
    b = f["body"]
    assert b["name"] == "nb1" and b["gpus"] == {"num": "1", "vendor": "amd.com/gpu"}
    assert b["configurations"] == ["rccl-debug"]
    assert b["workspace"]["newPvc"]["metadata"]["name"] == "nb1-workspace"
    assert [d["mount"] for d in b["datavols"]] == ["/home/jovyan/new-volume-name", "/data/dirty"]
    assert f["snacks"] == [["SUCCESS", "Notebook nb1 created"]]
    assert "lower case" in f["badNameError"] and f["badNamePosts"] == 0


def test_page_built_body_creates_the_notebook_in_the_backend(pages):
    from test_webapps import USER, _csrf  # noqa: F401
    from service_account_auth_improvements_amd.controlplane.apiserver import APIServer
    from service_account_auth_improvements_amd.controlplane.client import InMemoryClient
    from service_account_auth_improvements_amd.controlplane.profile import default_cluster_roles
    from service_account_auth_improvements_amd.webapps import jupyter
    c = InMemoryClient(APIServer())
    for cr in default_cluster_roles():
        c.create(cr)
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "kubeflow-user"}})
    c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
              "metadata": {"name": "namespaceAdmin", "namespace": "kubeflow-user"},
              "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "kubeflow-admin"},
              "subjects": [{"apiGroup": "rbac.authorization.k8s.io", "kind": "User", "name": "alice@example.com"}]})
    tc = jupyter.create_app(c, settings_env={"APP_SECURE_COOKIES": "false"}).test_client()
    r = tc.post("/api/namespaces/kubeflow-user/notebooks", json=pages["jwaForm"]["body"], headers=dict(USER, **_csrf(tc)))
    assert r.status_code == 200, r.json
    nb = c.get("kubeflow.org/v1beta1", "Notebook", "nb1", "kubeflow-user")
    ctr = nb["spec"]["template"]["spec"]["containers"][0]
    assert ctr["resources"]["limits"]["amd.com/gpu"] == "1"
    assert nb["metadata"]["labels"]["rccl-debug"] == "true"
    assert {"/home/jovyan/new-volume-name", "/data/dirty", "/home/jovyan"} <= {m["mountPath"] for m in ctr["volumeMounts"]}


def test_error_interceptor_snack(pages):
    (snack,) = pages["jwaError"]["snacks"]
    assert snack[0] == "ERROR" and snack[1].startswith("[500] Kubernetes API is unreachable\n")
    assert snack[1].endswith("/api/namespaces/kubeflow-user/notebooks")


def test_jwa_details_page_widgets(pages):
    d = pages["jwaDetails"]
    assert d["tabs"] == ["Overview", "Logs", "Events", "YAML"]
    assert d["gpuChips"] == ["1 x amd.com/gpu"] and d["configChips"] == ["rccl-debug"]     # details-list chips
    assert d["envRows"][0] == ["container", "HIP_VISIBLE_DEVICES", "0"]                   # variables-groups-table
    assert d["helpButtons"] == 2 and d["eventReasons"] == ["Created"] and d["yamlHasGpu"]


def test_twa_form_posts_the_tensorboard(pages):
    assert pages["twa"]["posts"] == [{"name": "tb1", "logspath": "pvc://datasets/runs/llama3",
                                      "configurations": ["access-ml-pipeline"]}]


# ------------------------------------------------------------------ central dashboard (T2)
# tests/js/centraldashboard.js drives static/centraldashboard.js like the reference's
# centraldashboard/public/components/*_test.js drive the Polymer components.
@pytest.fixture(scope="module")
def cd():
    r = subprocess.run(["node", os.path.join(ROOT, "tests", "js", "centraldashboard.js")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_cd_registration_validates_and_surfaces_backend_errors(cd):
    """registration-page_test.js: the default name from the user id, validateNamespace's message
    (no request sent), the backend's error in the form, then exists polled until the workgroup
    appears and the app reloads."""
    r = cd["registration"]
    assert r["welcome"] and r["nsPageHidden"]
    assert r["defaultName"] == "alice-smith-example-com"
    assert r["invalidError"].startswith("Name can only start and end with alpha-num characters")
    assert r["postsAfterInvalid"] == 0
    assert r["backendError"] == "namespace alice already exists"
    assert r["createBodies"] == [{"namespace": "alice"}, {"namespace": "alice"}]
    assert r["existsPolls"] == 3 and r["reloaded"] == 1


def test_cd_navigation_iframe_guard_and_logout(cd):
    h = cd["home"]
    nav = dict(h["nav"])
    assert nav["Notebooks"] == "#/_/jupyter/?ns=kubeflow-user" and nav["Manage Contributors"] == "#/manage-users"
    assert nav["Grafana"] == "https://grafana.example/"
    assert h["quick"] == ["#/_/jupyter/new?ns=kubeflow-user"] and h["docs"] == ["https://www.kubeflow.org/docs/"]
    assert h["iframeSrc"] == "/jupyter/?ns=kubeflow-user"
    # namespace messages go to the dashboard's own origin only, and the choice is stored per user
    assert h["messages"] == [[{"type": "namespace-selected", "value": "team-b"}, "http://localhost"]]
    assert h["stored"] == "team-b"
    # a protocol-relative or backslash path from the URL hash stays on this origin
    assert h["hostile"]["iframe"] and h["hostileSrc"] == "/evil.example/steal"
    assert h["hostile2"]["iframe"] and h["hostile2Src"] == "/evil.example/x"
    assert h["notFound"].startswith("404Sorry, /no/such/page is not a valid page.")
    assert h["activity"][:2] and "Created pod nb1-0" in h["activity"]
    assert h["logout"] == {"method": "POST", "auth": "Bearer sess42", "replaced": ["/dex/auth?loggedout=1"]}


def test_cd_resource_charts_from_metrics(cd):
    """resource-chart_test.js: series per label, the 5 highest means when more (title "(Top 5)"),
    a % axis for CPU, the interval menu re-queries."""
    c = {x["metric"]: x for x in cd["home"]["charts"]}
    assert c["node"]["title"] == "Cluster CPU Utilization (Top 5)" and c["node"]["lines"] == 5
    assert c["node"]["legend"] == ["n7", "n6", "n5", "n4", "n3"]
    assert c["podcpu"]["title"] == "Pod CPU Utilization" and c["podcpu"]["legend"] == ["kubeflow-user", "team-b"]
    assert c["node"]["ymax"].endswith("%") and c["node"]["link"] == "https://grafana.example/d/cluster"
    assert cd["home"]["metricRequests"] == ["api/metrics/node?interval=Last60m", "api/metrics/podcpu?interval=Last60m"]
    assert cd["home"]["intervalRequest"] == "api/metrics/node?interval=Last5m"
    assert cd["noNs"]["charts"] == 0           # /api/metrics 405: no charts


def test_cd_notebooks_and_pipelines_cards(cd):
    h = cd["home"]
    assert [n[0] for n in h["notebooks"]] == ["d.ipynb", "b.ipynb", "f.ipynb", "c.ipynb", "a.ipynb"]   # newest 5
    assert h["notebooks"][0][1] == "#/_/notebook/kubeflow-user/nb2/notebooks/d.ipynb"
    assert h["pipelines"][0] == ["train-llama", "#/_/pipeline/?ns=kubeflow-user#/pipelines/details/p1"]
    assert h["runs"] == [["run-ok", "success"], ["run-bad", "error"], ["run-now", "pending"]]
    assert "resource_reference_key.id=kubeflow-user" in h["runsQuery"][0]
    assert cd["noNs"]["notebooksMsg"] == "Choose a namespace to see Notebooks"
    assert cd["pipelinesError"] == "Error retrieving Pipeline Runs"
    assert cd["noNs"]["hash"] == "#/namespace-needed" and cd["noNs"]["page"].startswith("This page requires a namespace")


def test_cd_manage_contributors_surfaces_every_failure(cd):
    """manage-users-view(-contributor)_test.js: account info, the role table, the cluster-admin
    overview, chips per contributor; add / remove update the chips, a failed add or remove shows
    the backend error under the field, a failed fetch shows a toast."""
    m = cd["manage"]
    assert m["account"].endswith("alice@example.com (Cluster Admin)")
    assert m["roles"][1:] == ["Ownerkubeflow-user", "Contributorteam-b", "Viewerteam-c"]
    assert m["overview"][1] == "kubeflow-useralice@example.combob@example.com"
    assert m["sections"] == ["kubeflow-user"] and m["chips0"] == ["bob@example.com"]
    assert m["afterAdd"] == {"chips": ["bob@example.com", "carol@example.com"], "input": "", "error": ""}
    assert m["badAdd"]["error"] == "Contributor doesn't look like a valid email address"
    assert m["badAdd"]["chips"] == ["bob@example.com", "carol@example.com"] and m["badAdd"]["input"] == "not-an-email"
    assert m["afterRemove"] == {"chips": ["carol@example.com"], "error": ""}
    assert cd["removeError"] == {"error": "Unable to remove contributor", "chips": ["dave@example.com"]}
    assert cd["fetchError"] == [["ERROR", "Failed to fetch contributor list for kubeflow-user, because: KFAM is down"]]


# ------------------------------------------------------------------ second dashboard frontend (T3)
@pytest.fixture(scope="module")
def ng():
    r = subprocess.run(["node", os.path.join(ROOT, "tests", "js", "dashboard_ng.js")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_ng_namespace_resolution_and_persistence(ng):
    """namespace.service.ts: owned namespace first time, written back as ?ns and stored per user;
    the stored choice beats ownership, the query beats the stored choice, and a disabled
    "All namespaces" in the query falls back."""
    f = ng["first"]
    assert f["hash"] == "#/?ns=kubeflow-user" and f["selected"] == "kubeflow-user" and f["home"]
    assert f["stored"] == '"kubeflow-user"'
    assert f["options"][0] == ["All namespaces", True]          # disabled outside the allowed apps
    assert ng["restored"] == {"hash": "#/?ns=team-b", "selected": "team-b"}
    assert ng["queryWins"] == {"hash": "#/?ns=kubeflow-user", "selected": "kubeflow-user"}
    assert ng["allNsHome"]["selected"] == "team-b"
    assert f["build"].startswith("Build version v1.8-mi355x")


def test_ng_menu_links_and_all_namespaces(ng):
    menu = dict(ng["first"]["menu"])
    assert menu["Notebooks"] == "#/_/jupyter/?ns=kubeflow-user"
    assert menu["Runs"] == "#/_/pipeline/#/runs?ns=kubeflow-user"     # link's own ?ns={ns} resolved, fragment kept
    assert ng["first"]["quick"][0] == "#/_/jupyter/new?ns=kubeflow-user"
    assert ng["jupyter"]["options"][0] == ["All namespaces", False]   # allowed for jupyter
    assert ng["allNs"]["last"] == {"type": "all-namespaces"} and "ns=All+namespaces" in ng["allNs"]["hash"]


def test_ng_iframe_wrapper_protocol_and_mirroring(ng):
    assert ng["jupyter"]["src"] == "/jupyter/?ns=team-b" and ng["jupyter"]["stored"] == '"team-b"'
    assert ng["connected"] == [{"type": "namespace-selected", "value": "team-b"}]
    sw = ng["switched"]
    assert sw["hash"] == "#/_/jupyter/?ns=kubeflow-user" and sw["sameFrame"]
    assert sw["messages"] == [{"type": "namespace-selected", "value": "kubeflow-user"}]
    # the app navigated inside the iframe: the dashboard URL follows, with ?ns added
    assert ng["mirrored"]["hash"] == "#/_/jupyter/new?ns=kubeflow-user"


def test_ng_guard_404_and_error_interceptor(ng):
    assert ng["guard"]["page"] and ng["guard"]["hash"].startswith("#/namespace-needed?path=")
    assert ng["noNs"]["page"] and ng["noNs"]["after"].startswith("#/namespace-needed")
    assert ng["notFound"]["page"] and "/no-such-page" in ng["notFound"]["text"]
    # "#/_//evil.example/..." loads a path of this origin, never the other host; a frame whose
    # location throws (cross-origin) does not stop the URL-mirroring poll
    assert ng["hostile"] == {"src": "/evil.example/steal/?ns=team-b", "refused": False}
    assert ng["pollAlive"]["before"] >= 1 and ng["pollAlive"]["after"] >= 1
    assert ng["error"] == [["ERROR", "[500] kfam unreachable\nhttp://localhost/app/api/workgroup/env-info"]]
