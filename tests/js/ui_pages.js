// Renders the web apps' pages (static/kfamd-ui.js on lib/kf-common.js + lib/kf-logic.js) in
// the DOM shim against fixture responses shaped like the reference frontends' Cypress fixtures
// (the central dashboard has its own driver: centraldashboard.js)
// (crud-web-apps/jupyter/frontend/cypress/fixtures), drives them like a user, and prints one
// JSON object of observations for tests/test_ui.py.   usage: node ui_pages.js CONFIG_JSON
"use strict";
var fs = require("fs"), path = require("path"), vm = require("vm");
var shim = require("./dom_shim.js");
var STATIC = path.join(__dirname, "..", "..", "service_account_auth_improvements_amd", "webapps", "static");
var FIX = path.join(__dirname, "fixtures");
var SRC = ["lib/kf-logic.js", "lib/kf-common.js", "kfamd-ui.js"].map(function (f) {
  return [f, fs.readFileSync(path.join(STATIC, f), "utf8")];
});
var fx = function (n) { return JSON.parse(fs.readFileSync(path.join(FIX, n + ".json"), "utf8")); };
var CONFIG = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));

function boot(app, routes, opts) {
  opts = opts || {};
  var env = shim.makeEnv({ app: app, routes: routes, hash: opts.hash || "", search: opts.search || "" });
  var ctx = vm.createContext(env.ctx);
  SRC.forEach(function (s) { vm.runInContext(s[1], ctx, { filename: s[0] }); });
  env.q = function (sel) { return env.document.querySelector(sel); };
  env.qa = function (sel) { return env.document.querySelectorAll(sel); };
  env.text = function (sel) { var e = env.q(sel); return e ? e.textContent : null; };
  env.snacks = function () { return env.qa("[data-cy-snack-status]").map(function (s) { return [s.getAttribute("data-cy-snack-status"), s.textContent]; }); };
  env.go = function (h) { env.window.location.hash = h; return shim.flush(); };
  return shim.flush().then(function () { return env; });
}

var jwaRoutes = function (extra) {
  var r = {
    "GET api/config": { config: CONFIG, success: true, status: 200 },
    "GET api/namespaces": fx("namespaces"),
    "GET api/namespaces/kubeflow-user/notebooks": fx("notebooks"),
    "GET api/namespaces/team-b/notebooks": fx("notebooks_team_b"),
    "GET api/namespaces/default/notebooks": { notebooks: [], success: true },
    "GET api/namespaces/kubeflow/notebooks": { notebooks: [], success: true },
    "GET api/namespaces/kubeflow-user/poddefaults": fx("poddefaults"),
    "GET api/namespaces/kubeflow-user/pvcs": fx("pvcs"),
    "GET api/gpus": { vendors: ["amd.com/gpu"], success: true },
    "POST api/namespaces/kubeflow-user/notebooks": { success: true, status: 200 },
    "DELETE api/namespaces/kubeflow-user/notebooks/zeta-trainer": { success: true, status: 200 },
  };
  Object.keys(extra || {}).forEach(function (k) { r[k] = extra[k]; });
  return r;
};

var out = {};
function col(env, name) { return env.qa('[data-cy-resource-table-row="' + name + '"]').map(function (e) { return e.textContent; }); }

Promise.resolve()
  // ---------------------------------------------------------------- JWA main table (main-page.cy.ts)
  .then(function () { return boot("jupyter", jwaRoutes(), { search: "?ns=kubeflow-user" }); })
  .then(function (env) {
    out.jwaIndex = {
      title: env.text("[data-cy-toolbar-title]"),
      names: col(env, "Name"),
      statusClasses: env.qa('[data-cy-resource-table-row="Status"] span').map(function (s) { return s.className; }),
      gpus: col(env, "GPUs"),
      namespaceColumn: !!env.q('[data-cy-table-header-row="Namespace"]'),
      errorSnacks: env.snacks().filter(function (s) { return s[0] === "ERROR"; }),
      requested: env.requests.map(function (r) { return r.method + " " + r.path; }),
    };
    // all namespaces (cy.selectAllNamespaces): a Namespace column and every namespace's notebooks
    var sel = env.q("select#ns");
    sel.select_("*");
    return shim.flush().then(function () {
      out.jwaAll = { namespaceColumn: !!env.q('[data-cy-table-header-row="Namespace"]'), names: col(env, "Name"),
                     namespaces: col(env, "Namespace") };
      // sorting: click the Name header twice -> descending
      var th = env.q('[data-cy-table-header-row="Name"]');
      th.click();                                   // already sorted by Name: one click reverses
      out.jwaAll.namesDesc = col(env, "Name");
      // delete through the confirm dialog: cancel sends nothing, accept sends the DELETE
      sel.select_("kubeflow-user");
      return shim.flush();
    }).then(function () {
      var del = env.qa('[data-cy="delete"]')[col(env, "Name").indexOf("zeta-trainer")];
      del.click();
      var title = env.text('[data-cy="dialog-title"]');
      env.q('[data-cy="dialog-cancel"]').click();
      var afterCancel = env.requests.filter(function (r) { return r.method === "DELETE"; }).length;
      del.click();
      env.q('[data-cy="dialog-accept"]').click();
      return shim.flush().then(function () {
        out.jwaDelete = { dialogTitle: title, afterCancel: afterCancel, dialogOpen: !!env.q('[role="dialog"]'),
                          deletes: env.requests.filter(function (r) { return r.method === "DELETE"; }).map(function (r) { return r.path; }) };
      });
    }).then(function () {
      // the dashboard's iframe protocol: only the parent frame, on this origin, switches the namespace
      env.message({ type: "namespace-selected", value: "team-b" }, "https://evil.example");
      env.message({ type: "namespace-selected", value: "team-b" }, "");
      env.message({ type: "namespace-selected", value: "team-b" }, undefined, { postMessage: function () {} });
      var ignored = env.q("select#ns").value;
      env.message({ type: "namespace-selected", value: "team-b" });
      return shim.flush().then(function () { out.jwaIframeNs = { ignored: ignored, accepted: env.q("select#ns").value }; });
    });
  })
  // ---------------------------------------------------------------- JWA form (form-page.cy.ts)
  .then(function () { return boot("jupyter", jwaRoutes(), { search: "?ns=kubeflow-user", hash: "#/new" }); })
  .then(function (env) {
    var o = out.jwaForm = { title: env.text("[data-cy-toolbar-title]") };
    var ws = env.q('[data-cy="workspace volume"] [data-cy="volume name input"]');
    o.workspaceInitial = ws.value;                                   // '{notebook-name}-workspace' with no name yet
    env.q('input[name="name"]').type_("nb1");
    o.workspaceFollowsName = ws.value;
    o.workspaceHeader = env.text('[data-cy="volume name header"]');
    // data volume: mount follows the name until the mount path is edited
    env.q('[data-cy="add new volume"]').click();
    var last = env.q('.last[data-cy="data volumes"]');
    last.q = function (s) { return last.querySelector(s); };
    last.q('[data-cy="volume name input"]').type_("new-volume-name");
    o.mountAuto = env.q('.last[data-cy="data volumes"] [data-cy="mount path"]').value;
    env.q('[data-cy="add new volume"]').click();
    var last2 = env.q('.last[data-cy="data volumes"]');
    last2.querySelector('[data-cy="mount path"]').type_("/data/dirty");
    last2.querySelector('[data-cy="volume name input"]').type_("second");
    o.mountDirty = env.q('.last[data-cy="data volumes"] [data-cy="mount path"]').value;
    // GPUs + a configuration, then submit
    env.q('select[name="gpus"]').select_("1");
    var cfg = env.qa('input[type="checkbox"]').filter(function (i) { return i.value === "rccl-debug"; })[0];
    cfg.click();
    o.gpuVendors = env.q('select[name="gpuVendor"]').querySelectorAll("option").map(function (x) { return x.textContent; });
    env.q('button[type="submit"]').click();
    return shim.flush().then(function () {
      var post = env.requests.filter(function (r) { return r.method === "POST"; });
      o.posts = post.map(function (r) { return r.path; });
      o.body = post.length ? post[0].body : null;
      o.hashAfter = env.window.location.hash;
      o.snacks = env.snacks();
      // a second form with a bad name shows the validation error and sends nothing
      return boot("jupyter", jwaRoutes(), { search: "?ns=kubeflow-user", hash: "#/new" });
    }).then(function (env2) {
      env2.q('input[name="name"]').type_("Bad_Name");
      env2.q('button[type="submit"]').click();
      return shim.flush().then(function () {
        o.badNameError = env2.q("form .err").textContent;
        o.badNamePosts = env2.requests.filter(function (r) { return r.method === "POST"; }).length;
      });
    });
  })
  // ---------------------------------------------------------------- backend error -> interceptor snack
  .then(function () {
    return boot("jupyter", jwaRoutes({ "GET api/namespaces/kubeflow-user/notebooks":
      { status: 500, body: { success: false, status: 500, log: "Kubernetes API is unreachable" } } }), { search: "?ns=kubeflow-user" });
  })
  .then(function (env) { out.jwaError = { snacks: env.snacks() }; })
  // ---------------------------------------------------------------- JWA details page
  .then(function () {
    var nb = { apiVersion: "kubeflow.org/v1", kind: "Notebook",
               metadata: { name: "zeta-trainer", namespace: "kubeflow-user", creationTimestamp: "2026-10-15T10:00:00Z",
                           labels: { "rccl-debug": "true" }, annotations: { "notebooks.kubeflow.org/creator": "alice@example.com" } },
               spec: { template: { spec: { containers: [{ name: "zeta-trainer", image: "kfamd/jupyter-pytorch-rocm:latest",
                 resources: { requests: { cpu: "4", memory: "32Gi" }, limits: { "amd.com/gpu": "1" } },
                 env: [{ name: "HIP_VISIBLE_DEVICES", value: "0" }, { name: "NB_PREFIX", value: "/notebook/kubeflow-user/zeta-trainer" }],
                 volumeMounts: [{ name: "dshm", mountPath: "/dev/shm" }] }],
                 volumes: [{ name: "dshm", emptyDir: { medium: "Memory" } }] } } },
               status: { conditions: [{ type: "Ready", status: "True", lastTransitionTime: "2026-10-15T10:01:00Z" }] },
               processed_status: { phase: "ready", message: "Running" } };
    return boot("jupyter", jwaRoutes({
      "GET api/namespaces/kubeflow-user/notebooks/zeta-trainer": { notebook: nb, success: true },
      "GET api/namespaces/kubeflow-user/notebooks/zeta-trainer/events": { events: [{ type: "Normal", reason: "Created",
        message: "Created pod zeta-trainer-0", involvedObject: { kind: "Pod", name: "zeta-trainer-0" }, lastTimestamp: "2026-10-15T10:00:05Z" }], success: true },
    }), { search: "?ns=kubeflow-user", hash: "#/details/kubeflow-user/zeta-trainer" });
  })
  .then(function (env) {
    var o = out.jwaDetails = {};
    o.detailKeys = env.qa("[data-cy-details-key]").map(function (e) { return e.getAttribute("data-cy-details-key"); });
    o.gpuChips = env.qa('[data-cy-details-value="GPUs"] .chip').map(function (e) { return e.textContent; });
    o.configChips = env.qa('[data-cy-details-value="Configurations"] .chip').map(function (e) { return e.textContent; });
    o.envRows = env.qa("table.vgt tbody tr").map(function (tr) { return tr.querySelectorAll("td").map(function (td) { return td.textContent; }); });
    o.helpButtons = env.qa("button.help").length;
    var tabs = env.qa('[role="tab"]');
    o.tabs = tabs.map(function (t) { return t.textContent; });
    tabs[2].click();
    return shim.flush().then(function () {
      o.eventReasons = col(env, "Reason");
      tabs[3].click();
      return shim.flush();
    }).then(function () {
      o.yamlHasGpu = /amd\.com\/gpu/.test(env.text("pre.code") || "");
    });
  })
  // ---------------------------------------------------------------- VWA: index + delete dialog
  .then(function () {
    return boot("volumes", { "GET api/namespaces": fx("namespaces"), "GET api/namespaces/kubeflow-user/pvcs": fx("pvcs"),
                             "GET api/storageclasses": { storageClasses: ["fast-nvme", "standard"], success: true },
                             "GET api/storageclasses/default": { defaultStorageClass: "standard", success: true },
                             "POST api/namespaces/kubeflow-user/pvcs": { success: true, status: 200 },
                             "DELETE api/namespaces/kubeflow-user/pvcs/datasets": { status: 409, body: { success: false, status: 409,
                               log: "PVC datasets is used by pod zeta-trainer-0" } } }, { search: "?ns=kubeflow-user" });
  })
  .then(function (env) {
    var o = out.vwa = { names: col(env, "Name"), usedBy: col(env, "Used by") };
    o.buttons = env.qa('[data-cy-resource-table-row=""] button').map(function (b) { return b.textContent; });
    env.qa('[data-cy="delete"]')[col(env, "Name").indexOf("datasets")].click();
    env.q('[data-cy="dialog-accept"]').click();
    return shim.flush().then(function () {
      o.dialogStillOpen = !!env.q('[role="dialog"]');
      o.dialogError = env.text('[data-cy="dialog-error"]');
      // the create form: storage classes from the backend, its default preselected
      var sc = env.q('[data-cy="storage class"]');
      o.classOptions = sc.children.map(function (c) { return c.getAttribute("value"); });
      o.classSelected = sc.value;
      var newBtn = env.qa("button").filter(function (b) { return b.textContent === "+ New volume"; })[0];
      env.q('input[placeholder="name"]').type_("datasets");          // an existing volume's name
      newBtn.click();
      return shim.flush().then(function () {
        o.dupSnacks = env.snacks();
        o.dupPosts = env.requests.filter(function (r) { return r.method === "POST"; }).length;
        env.q('input[placeholder="name"]').value = "";
        env.q('input[placeholder="name"]').type_("scratch");
        newBtn.click();
        return shim.flush();
      }).then(function () {
        o.posts = env.requests.filter(function (r) { return r.method === "POST"; }).map(function (r) { return r.body; });
      });
    });
  })
  // ---------------------------------------------------------------- TWA: create
  .then(function () {
    return boot("tensorboards", { "GET api/namespaces": fx("namespaces"), "GET api/namespaces/kubeflow-user/pvcs": fx("pvcs"),
                                  "GET api/namespaces/kubeflow-user/poddefaults": fx("poddefaults"),
                                  "GET api/namespaces/kubeflow-user/tensorboards": { tensorboards: [], success: true },
                                  "POST api/namespaces/kubeflow-user/tensorboards": { success: true } }, { search: "?ns=kubeflow-user" });
  })
  .then(function (env) {
    env.q('input[placeholder="name"]').type_("tb1");
    env.q('input[placeholder="sub/path"]').type_("/runs/llama3");
    env.qa('input[type="checkbox"]')[0].click();
    env.qa("button").filter(function (b) { return b.textContent === "+ New TensorBoard"; })[0].click();
    return shim.flush().then(function () {
      out.twa = { posts: env.requests.filter(function (r) { return r.method === "POST"; }).map(function (r) { return r.body; }) };
    });
  })
  .then(function () { process.stdout.write(JSON.stringify(out)); },
        function (e) { process.stderr.write((e && e.stack) || String(e)); process.exit(1); });
