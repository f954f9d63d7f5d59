// Drives the central dashboard (static/centraldashboard.js, the Polymer centraldashboard/public
// components) in the DOM shim, the way the reference's *_test.js files drive theirs:
// registration-page (default name, validateNamespace, backend error, exists polling), main-page
// (navigation, iframe-container with the same-origin guard and the namespace message protocol,
// 404, namespace-needed), dashboard-view (quick links, resource charts from fixture metrics,
// notebooks card, pipelines cards), manage-users-view (roles, cluster-admin overview,
// contributor add / remove incl. failures) and logout-button.  Prints one JSON object for
// tests/test_ui.py.   usage: node centraldashboard.js
"use strict";
var fs = require("fs"), path = require("path"), vm = require("vm");
var shim = require("./dom_shim.js");
var STATIC = path.join(__dirname, "..", "..", "service_account_auth_improvements_amd", "webapps", "static");
var SRC = ["lib/kf-logic.js", "lib/kf-common.js", "centraldashboard.js", "kfamd-ui.js"].map(function (f) {
  return [f, fs.readFileSync(path.join(STATIC, f), "utf8")];
});

var USER = "alice@example.com";
var ENV = { user: USER, isClusterAdmin: true,
            platform: { kubeflowVersion: "v1.8-mi355x", provider: "other", providerName: "other", logoutUrl: "/authservice/logout" },
            namespaces: [{ namespace: "kubeflow-user", role: "owner", user: USER },
                         { namespace: "team-b", role: "contributor", user: USER },
                         { namespace: "team-c", role: "viewer", user: USER }] };
var LINKS = { menuLinks: [{ type: "item", link: "/jupyter/", text: "Notebooks" },
                          { type: "item", link: "/pipeline/#/runs", text: "Runs" }],
              externalLinks: [{ link: "https://grafana.example/", text: "Grafana" }],
              quickLinks: [{ link: "/jupyter/new", text: "Create a new Notebook server", desc: "Notebook Servers" }],
              documentationItems: [{ link: "https://www.kubeflow.org/docs/", text: "Getting Started", desc: "docs" }] };
var T0 = 1760000000;
function series(labels, n) {       // n points per label, label i has mean ~ (i + 1) / 10
  var pts = [];
  labels.forEach(function (l, i) {
    for (var k = 0; k < n; ++k) pts.push({ timestamp: T0 + 10 * k, label: l, value: (i + 1) / 10 + 0.01 * k });
  });
  return pts;
}
function contents(files) {
  return { content: files.map(function (f) { return { name: f[0], last_modified: f[1], type: "notebook" }; }) };
}

function boot(routes, opts) {
  opts = opts || {};
  var env = shim.makeEnv({ app: "dashboard", routes: routes, hash: opts.hash || "" });
  env.document.cookie = "XSRF-TOKEN=tok123; authservice_session=sess42";
  var ctx = vm.createContext(env.ctx);
  SRC.forEach(function (s) { vm.runInContext(s[1], ctx, { filename: s[0] }); });
  env.q = function (sel) { return env.document.querySelector(sel); };
  env.qa = function (sel) { return env.document.querySelectorAll(sel); };
  env.text = function (sel) { var e = env.q(sel); return e ? e.textContent : null; };
  env.go = function (h) { env.window.location.hash = h; return shim.flush(); };
  env.snacks = function () { return env.qa("[data-cy-snack-status]").map(function (s) { return [s.getAttribute("data-cy-snack-status"), s.textContent]; }); };
  env.tick = function () { var t = env.timers.splice(0); t.forEach(function (x) { x.f(); }); return shim.flush(); };
  env.click = function (sel) { env.q(sel).click(); return shim.flush(); };
  return shim.flush(10).then(function () { return env; });
}

function mainRoutes(extra) {
  var contribs = ["bob@example.com"];
  var r = {
    "GET api/workgroup/exists": { hasWorkgroup: true, hasAuth: true, registrationFlowAllowed: true, user: USER },
    "GET api/workgroup/env-info": ENV,
    "GET api/dashboard-links": LINKS,
    "GET api/metrics": { resourceChartsLink: "https://grafana.example/d/cluster", resourceChartsLinkText: "View in Grafana" },
    "GET api/metrics/node": series(["n1", "n2", "n3", "n4", "n5", "n6", "n7"], 4),
    "GET api/metrics/podcpu": series(["kubeflow-user", "team-b"], 3),
    "GET api/activities/team-b": [{ type: "Normal", message: "Created pod nb1-0", lastTimestamp: "2026-10-17T10:00:00Z",
                                          involvedObject: { kind: "Pod", name: "nb1-0" } }],
    "GET jupyter/api/namespaces/kubeflow-user/notebooks": { notebooks: [{ name: "nb1", namespace: "kubeflow-user" },
                                                                          { name: "nb2", namespace: "kubeflow-user" }] },
    "GET notebook/kubeflow-user/nb1/api/contents": contents([["a.ipynb", "2026-10-01T00:00:00Z"], ["b.ipynb", "2026-10-05T00:00:00Z"],
                                                             ["c.ipynb", "2026-10-03T00:00:00Z"]]),
    "GET notebook/kubeflow-user/nb2/api/contents": contents([["d.ipynb", "2026-10-06T00:00:00Z"], ["e.ipynb", "2026-09-01T00:00:00Z"],
                                                             ["f.ipynb", "2026-10-04T00:00:00Z"]]),
    "GET pipeline/apis/v1beta1/pipelines": { pipelines: [{ id: "p1", name: "train-llama", created_at: "2026-10-02T00:00:00Z" },
                                                          { id: "p2", name: "eval", created_at: "2026-10-03T00:00:00Z" }] },
    "GET pipeline/apis/v1beta1/runs": { runs: [{ id: "r1", name: "run-ok", status: "Succeeded", created_at: "2026-10-02T00:00:00Z" },
                                               { id: "r2", name: "run-bad", status: "Failed", created_at: "2026-10-02T00:00:00Z" },
                                               { id: "r3", name: "run-now", status: "Running", created_at: "2026-10-02T00:00:00Z" }] },
    "GET api/workgroup/get-all-namespaces": [["kubeflow-user", USER, "bob@example.com"], ["team-b", "carol@example.com", USER]],
    "GET api/workgroup/get-contributors/kubeflow-user": function () { return contribs.slice(); },
    "POST api/workgroup/add-contributor/kubeflow-user": function (b) {
      if (b.contributor.indexOf("@") < 0) return { status: 400, body: { success: false, log: "Contributor doesn't look like a valid email address" } };
      contribs.push(b.contributor);
      return contribs.slice();
    },
    "DELETE api/workgroup/remove-contributor/kubeflow-user": function (b) {
      if (b.contributor === "dave@example.com") return { status: 500, body: { success: false, log: "Unable to remove contributor" } };
      contribs = contribs.filter(function (c) { return c !== b.contributor; });
      return contribs.slice();
    },
    "POST authservice/logout": { afterLogoutURL: "/dex/auth?loggedout=1" },
  };
  Object.keys(extra || {}).forEach(function (k) { r[k] = extra[k]; });
  return r;
}

var out = {};
Promise.resolve()
  // ---------------------------------------------------------------- registration-page
  .then(function () {
    var exists = 0, creates = 0;
    return boot({
      "GET api/workgroup/exists": function () {
        exists++;
        return { hasWorkgroup: exists > 2, hasAuth: true, registrationFlowAllowed: true, user: "Alice.Smith@example.com" };
      },
      "POST api/workgroup/create": function () {
        creates++;
        return creates === 1 ? { status: 409, body: { success: false, log: "namespace alice already exists" } }
                             : { message: "Created namespace alice" };
      },
    }).then(function (env) {
      var o = out.registration = { welcome: !!env.q('[data-cy="registration-welcome"]'),
                                   nsPageHidden: env.q('[data-cy="registration-namespace-page"]').getAttribute("hidden") !== null };
      return env.click('[data-cy="registration-start"]').then(function () {
        var inp = env.q('[data-cy="registration-namespace"]');
        o.defaultName = inp.value;
        inp.value = "-Bad_Name-";
        return env.click('[data-cy="registration-finish"]');
      }).then(function () {
        o.invalidError = env.text('[data-cy="registration-error"]');
        o.postsAfterInvalid = env.requests.filter(function (r) { return r.method === "POST"; }).length;
        env.q('[data-cy="registration-namespace"]').value = "alice";
        return env.click('[data-cy="registration-finish"]');
      }).then(function () {
        o.backendError = env.text('[data-cy="registration-error"]');
        return env.click('[data-cy="registration-finish"]');
      }).then(function () {
        return env.tick();         // the exists poll's 300 ms sleeps
      }).then(function () { return env.tick(); }).then(function () {
        o.createBodies = env.requests.filter(function (r) { return r.method === "POST"; }).map(function (r) { return r.body; });
        o.existsPolls = exists;
        o.reloaded = env.window.location.reloaded;
      });
    });
  })
  // ---------------------------------------------------------------- main-page + dashboard-view
  .then(function () { return boot(mainRoutes()); })
  .then(function (env) {
    var o = out.home = {
      nav: env.qa('[data-cy="sidenav"] a').map(function (a) { return [a.textContent, a.getAttribute("href")]; }),
      user: env.text('[data-cy="user"]'),
      selector: env.qa('[data-cy="namespace-selector"] option').map(function (x) { return x.value; }),
      quick: env.qa('[data-cy="quick-link"]').map(function (a) { return a.getAttribute("href"); }),
      docs: env.qa('[data-cy="documentation"] a').map(function (a) { return a.getAttribute("href"); }),
      charts: env.qa('[data-cy="resource-chart"]').map(function (c) {
        return { metric: c.getAttribute("data-metric"), title: c.querySelector('[data-cy="chart-title"]').textContent,
                 lines: c.querySelectorAll("polyline").length,
                 legend: c.querySelectorAll('[data-cy="chart-legend"] li').map(function (li) { return li.textContent; }),
                 ymax: (c.querySelector('[data-cy="chart-ymax"]') || { textContent: "" }).textContent,
                 link: (c.querySelector('[data-cy="chart-link"]') || { getAttribute: function () { return null; } }).getAttribute("href") };
      }),
      notebooks: env.qa('[data-cy="notebook-link"]').map(function (a) { return [a.textContent, a.getAttribute("href")]; }),
      pipelines: env.qa('[data-kind="pipelines"] [data-cy="pipeline-link"]').map(function (a) { return [a.textContent, a.getAttribute("href")]; }),
      runs: env.qa('[data-kind="runs"] li').map(function (li) { return [li.querySelector("a").textContent, li.getAttribute("data-status")]; }),
      runsQuery: env.requests.filter(function (r) { return r.path.indexOf("pipeline/apis/v1beta1/runs") === 0; }).map(function (r) { return r.path; }),
      metricRequests: env.requests.filter(function (r) { return r.path.indexOf("api/metrics/") === 0; }).map(function (r) { return r.path; }),
    };
    // a chart's interval menu re-queries with the new interval
    var chartSel = env.q('[data-cy="chart-interval"]');
    chartSel.value = "Last5m";
    chartSel.dispatchEvent({ type: "change" });
    return shim.flush().then(function () {
      o.intervalRequest = env.requests.filter(function (r) { return r.path.indexOf("api/metrics/node") === 0; }).pop().path;
      // iframe-container: an app, then a hostile protocol-relative path
      return env.go("#/_/jupyter/?ns=kubeflow-user");
    }).then(function () {
      var frame = env.q('[data-cy="iframe"]');
      o.iframeSrc = frame.src;
      var got = [];
      frame.contentWindow = { postMessage: function (m, target) { got.push([m, target]); } };
      env.window.__listeners = null;
      var sel = env.q('[data-cy="namespace-selector"]');
      sel.value = "team-b";
      sel.dispatchEvent({ type: "change" });
      return shim.flush().then(function () {
        o.messages = got;
        o.stored = env.localStorage["/centraldashboard/selectedNamespace/" + USER];
        return env.go("#/_//evil.example/steal");
      });
    }).then(function () {
      o.hostile = { refused: env.text('[data-cy="refused"]'), iframe: !!env.q('[data-cy="iframe"]') };
      o.hostileSrc = (env.q('[data-cy="iframe"]') || {}).src;
      return env.go("#/_/\\\\evil.example/x");
    }).then(function () {
      o.hostile2 = { refused: !!env.q('[data-cy="refused"]'), iframe: !!env.q('[data-cy="iframe"]') };
      o.hostile2Src = (env.q('[data-cy="iframe"]') || {}).src;
      return env.go("#/no/such/page");
    }).then(function () {
      o.notFound = env.text('[data-cy="not-found"]');
      return env.go("#/activity");
    }).then(function () {
      o.activity = env.qa('[data-cy="activity-view"] td').map(function (td) { return td.textContent; });
      // logout-button: POST logoutUrl with the session as a bearer token, then location.replace
      return env.click('[data-cy="logout-button"]');
    }).then(function () {
      var req = env.requests.filter(function (r) { return r.path === "authservice/logout"; })[0];
      o.logout = { method: req && req.method, auth: req && req.headers.Authorization, replaced: env.window.location.replaced };
    });
  })
  // ---------------------------------------------------------------- manage-users-view
  .then(function () { return boot(mainRoutes(), { hash: "#/manage-users" }); })
  .then(function (env) {
    var chips = function () { return env.qa('[data-cy="contributor"]').map(function (c) { return c.childNodes[0].textContent; }); };
    var o = out.manage = {
      account: env.text('[data-cy="account-info"]'),
      roles: env.qa('[data-cy="memberships"] tr').map(function (tr) { return tr.textContent; }),
      overview: env.qa('[data-cy="cluster-namespaces"] tr').map(function (tr) { return tr.textContent; }),
      sections: env.qa('[data-cy="contributors"]').map(function (s) { return s.getAttribute("data-namespace"); }),
      chips0: chips(),
    };
    var input = env.q('[data-cy="contributor-input"]');
    input.value = "carol@example.com";
    return env.click('[data-cy="contributor-add"]').then(function () {
      o.afterAdd = { chips: chips(), input: input.value, error: env.text('[data-cy="contributor-error"]') };
      input.value = "not-an-email";
      return env.click('[data-cy="contributor-add"]');
    }).then(function () {
      o.badAdd = { chips: chips(), error: env.text('[data-cy="contributor-error"]'), input: input.value };
      env.qa('[data-cy="contributor-remove"]')[0].click();     // bob
      return shim.flush();
    }).then(function () {
      o.afterRemove = { chips: chips(), error: env.text('[data-cy="contributor-error"]') };
    });
  })
  // a failing contributor fetch surfaces as a toast; a failing removal under the field
  .then(function () {
    return boot(mainRoutes({ "GET api/workgroup/get-contributors/kubeflow-user": { status: 500, body: { success: false, log: "KFAM is down" } } }),
                { hash: "#/manage-users" });
  })
  .then(function (env) {
    out.fetchError = env.snacks();
  })
  .then(function () {
    return boot(mainRoutes({ "GET api/workgroup/get-contributors/kubeflow-user": ["dave@example.com"] }), { hash: "#/manage-users" });
  })
  .then(function (env) {
    env.qa('[data-cy="contributor-remove"]')[0].click();
    return shim.flush().then(function () {
      out.removeError = { error: env.text('[data-cy="contributor-error"]'),
                          chips: env.qa('[data-cy="contributor"]').map(function (c) { return c.childNodes[0].textContent; }) };
    });
  })
  // no namespace at all: an app path holding {ns} goes to namespace-needed; no metrics service
  .then(function () {
    return boot(mainRoutes({ "GET api/workgroup/env-info": { user: "bob@example.com", namespaces: [], platform: {} },
                             "GET api/metrics": { status: 405, body: { success: false, log: "Operation not supported" } } }),
                { hash: "#/_/pipeline/?ns={ns}" });
  })
  .then(function (env) {
    return shim.flush(10).then(function () {
      out.noNs = { hash: env.window.location.hash, page: env.text('[data-cy="namespace-needed"]'),
                   charts: env.qa('[data-cy="resource-chart"]').length };
      return env.go("#/");
    }).then(function () {
      out.noNs.charts = env.qa('[data-cy="resource-chart"]').length;
      out.noNs.notebooksMsg = env.text('[data-cy="notebooks-card"] [data-cy="card-message"]');
    });
  })
  // pipelines error path
  .then(function () { return boot(mainRoutes({ "GET pipeline/apis/v1beta1/runs": { status: 503, body: {} } })); })
  .then(function (env) {
    out.pipelinesError = env.text('[data-kind="runs"] [data-cy="card-message"]');
  })
  .then(function () { process.stdout.write(JSON.stringify(out)); },
        function (e) { process.stderr.write((e && e.stack) || String(e)); process.exit(1); });
