// Drives the second central-dashboard frontend (static/dashboard-ng.js, the centraldashboard-angular
// behaviour) in the DOM shim: namespace resolution order and persistence, the "All namespaces"
// option, the iframe guard, the iframe wrapper's src / message protocol / URL mirroring, the 404
// and namespace-needed pages, and the error interceptor.  Prints one JSON object for
// tests/test_ui.py.   usage: node dashboard_ng.js
"use strict";
var fs = require("fs"), path = require("path"), vm = require("vm");
var shim = require("./dom_shim.js");
var STATIC = path.join(__dirname, "..", "..", "service_account_auth_improvements_amd", "webapps", "static");
var SRC = ["lib/kf-logic.js", "lib/kf-common.js", "dashboard-ng.js"].map(function (f) {
  return [f, fs.readFileSync(path.join(STATIC, f), "utf8")];
});

var ENV = { user: "alice@example.com", isClusterAdmin: false,
            platform: { kubeflowVersion: "v1.8-mi355x", provider: "other", providerName: "other" },
            namespaces: [{ namespace: "team-b", role: "contributor", user: "alice@example.com" },
                         { namespace: "kubeflow-user", role: "owner", user: "alice@example.com" }] };
var LINKS = { menuLinks: [{ type: "item", link: "/jupyter/", text: "Notebooks" },
                          { type: "item", link: "/volumes/", text: "Volumes" },
                          { type: "item", link: "/pipeline/#/runs?ns={ns}", text: "Runs" }],
              quickLinks: [{ link: "/jupyter/new?ns={ns}", text: "Create a new Notebook server", desc: "Notebook Servers" }],
              documentationItems: [{ link: "https://www.kubeflow.org/docs/", text: "Getting Started" }] };

function boot(opts) {
  opts = opts || {};
  var routes = { "GET api/workgroup/env-info": opts.envInfo || ENV, "GET api/dashboard-links": LINKS };
  var env = shim.makeEnv({ app: "dashboard-ng", routes: routes, hash: opts.hash || "", localStorage: opts.store });
  var ctx = vm.createContext(env.ctx);
  SRC.forEach(function (s) { vm.runInContext(s[1], ctx, { filename: s[0] }); });
  env.q = function (sel) { return env.document.querySelector(sel); };
  env.qa = function (sel) { return env.document.querySelectorAll(sel); };
  env.hash = function () { return env.window.location.hash; };
  env.go = function (h) { env.window.location.hash = h; return shim.flush(); };
  env.options = function () {
    return env.qa("[data-cy-namespace-selector] option").map(function (o) { return [o.value, o.getAttribute("disabled") !== null]; });
  };
  env.selected = function () { return env.q("[data-cy-namespace-selector]").value; };
  env.tick = function () { var t = env.timers.splice(0); t.forEach(function (x) { x.f(); }); return shim.flush(); };
  return shim.flush().then(function () { return env; });
}

var out = {};
Promise.resolve()
  // owned namespace when nothing else says otherwise; ?ns written back; choice stored
  .then(function () { return boot({ hash: "" }); })
  .then(function (env) {
    out.first = { hash: env.hash(), home: !!env.q('[data-cy="home"]'), options: env.options(), selected: env.selected(),
                  stored: env.localStorage["selectedNamespace/.alice@example.com"],
                  menu: env.qa("[data-cy-sidenav-menu-item]").map(function (a) { return [a.getAttribute("data-cy-sidenav-menu-item"), a.getAttribute("href")]; }),
                  quick: env.qa('[data-cy="home"] li a').map(function (a) { return a.getAttribute("href"); }),
                  build: env.q('[data-cy="build"]').textContent };
    // an app in the iframe: src without "/_", trailing "/", ?ns; "All namespaces" enabled for jupyter
    return env.go("#/_/jupyter/?ns=team-b").then(function () {
      var frame = env.q('[data-cy="iframe"]');
      out.jupyter = { src: frame.src, selected: env.selected(), options: env.options(),
                      stored: env.localStorage["selectedNamespace/.alice@example.com"] };
      var got = [];
      frame.contentWindow = { postMessage: function (m) { got.push(m); }, location: {} };
      env.message({ type: "iframe-connected" }, "https://evil.example");   // ignored: foreign origin
      env.message({ type: "iframe-connected" }, "");                       // ignored: no origin
      env.message({ type: "iframe-connected" });
      out.connected = got.slice();
      // the namespace selector: new ?ns, the iframe is told
      var sel = env.q("[data-cy-namespace-selector]");
      sel.value = "kubeflow-user";
      sel.dispatchEvent({ type: "change" });
      return shim.flush().then(function () {
        out.switched = { hash: env.hash(), messages: got.slice(1), sameFrame: env.q('[data-cy="iframe"]') === frame };
        // the app navigates inside the iframe: the dashboard URL follows, ?ns kept
        frame.contentWindow.location = { pathname: "/jupyter/new", search: "", hash: "" };
        return env.tick();
      }).then(function () {
        out.mirrored = { hash: env.hash(), src: env.q('[data-cy="iframe"]').src };
        // "All namespaces" on an app that allows it
        var sel2 = env.q("[data-cy-namespace-selector]");
        sel2.value = "All namespaces";
        sel2.dispatchEvent({ type: "change" });
        return shim.flush();
      }).then(function () {
        out.allNs = { hash: env.hash(), last: got[got.length - 1] };
        // guard: an app path still holding {ns}
        return env.go("#/_/jupyter/{ns}/details");
      }).then(function () {
        out.guard = { hash: env.hash(), page: !!env.q('[data-cy="namespace-needed"]') };
        return env.go("#/no-such-page");
      }).then(function () {
        out.notFound = { page: !!env.q('[data-cy="not-found"]'), text: env.q('[data-cy="not-found"]').textContent };
        // a protocol-relative app path stays on this origin; a cross-origin frame (its location
        // throws SecurityError) does not stop the URL-mirroring poll
        return env.go("#/_//evil.example/steal?ns=team-b");
      }).then(function () {
        var frame = env.q('[data-cy="iframe"]');
        out.hostile = { src: frame && frame.src, refused: !!env.q('[data-cy="refused"]') };
        frame.contentWindow = { postMessage: function () {} };
        Object.defineProperty(frame.contentWindow, "location", { get: function () { throw new Error("SecurityError"); } });
        var polls = function () { return env.timers.filter(function (t) { return t.ms === 100; }).length; };
        var before = polls();
        return env.tick().then(function () { return env.tick(); }).then(function () {
          out.pollAlive = { before: before, after: polls() };
        });
      });
    });
  })
  // the stored choice beats ownership; the query beats the stored choice; a disabled
  // "All namespaces" in the query falls back
  .then(function () { return boot({ hash: "", store: { "selectedNamespace/.alice@example.com": "\"team-b\"" } }); })
  .then(function (env) { out.restored = { hash: env.hash(), selected: env.selected() }; })
  .then(function () { return boot({ hash: "#/?ns=kubeflow-user", store: { "selectedNamespace/.alice@example.com": "\"team-b\"" } }); })
  .then(function (env) { out.queryWins = { hash: env.hash(), selected: env.selected() }; })
  .then(function () { return boot({ hash: "#/?ns=All%20namespaces", store: { "selectedNamespace/.alice@example.com": "\"team-b\"" } }); })
  .then(function (env) { out.allNsHome = { hash: env.hash(), selected: env.selected() }; })
  // a user with no namespace: links keep {ns} -> the guard sends them to namespace-needed
  .then(function () { return boot({ hash: "", envInfo: { user: "bob@example.com", namespaces: [], platform: {} } }); })
  .then(function (env) {
    var items = env.qa("[data-cy-sidenav-menu-item]");
    if (!items.length) { out.noNs = { hash: env.hash(), items: 0, snacks: env.qa("[data-cy-snack-status]").map(function (s) { return s.textContent; }) }; return; }
    var runs = items.filter(function (a) { return a.getAttribute("data-cy-sidenav-menu-item") === "Runs"; })[0];
    out.noNs = { hash: env.hash(), runsHref: runs.getAttribute("href") };
    return env.go(runs.getAttribute("href")).then(function () {
      out.noNs.after = env.hash();
      out.noNs.page = !!env.q('[data-cy="namespace-needed"]');
    });
  })
  // error interceptor: a failing env-info call
  .then(function () { return boot({ hash: "", envInfo: { status: 500, body: { success: false, log: "kfam unreachable" } } }); })
  .then(function (env) {
    out.error = env.qa("[data-cy-snack-status]").map(function (s) { return [s.getAttribute("data-cy-snack-status"), s.textContent]; });
  })
  .then(function () { console.log(JSON.stringify(out)); })
  .catch(function (e) { console.error(e && e.stack || e); process.exit(1); });
