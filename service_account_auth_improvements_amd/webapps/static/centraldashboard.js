// Central dashboard frontend (T2): the Polymer app of centraldashboard/public/components
// re-expressed dependency-free on the kubeflow-common-lib DOM helpers (lib/kf-common.js).
//
//   main-page            toolbar (namespace selector, user, logout-button), side navigation from
//                        /api/dashboard-links, routes #/ home, #/activity, #/manage-users,
//                        #/_/<app path> (iframe-container), #/namespace-needed, 404
//   registration-page    two-step namespace setup: name derived from the user id, validated
//                        (validateNamespace), POST /api/workgroup/create, backend errors shown
//                        in the form, then /api/workgroup/exists polled (66 x 300 ms)
//   dashboard-view       quick shortcuts (?ns= added), two resource-charts (when /api/metrics
//                        says charts are available), notebooks-card, two pipelines-cards,
//                        documentation
//   resource-chart       SVG line chart of /api/metrics/<node|podcpu|podmem>?interval=..., top 5
//                        series by mean ("(Top 5)"), % axis for CPU, interval menu + refresh
//   notebooks-card       the 5 most recently modified notebooks over the namespace's servers
//   pipelines-card       recent pipelines / runs (status icons for runs)
//   activity-view        the namespace's events
//   manage-users-view    account info, role table, cluster-admin profile overview, and per
//                        owned namespace the contributor chips with remove, an add field, and
//                        every add / remove / fetch failure surfaced
//   logout-button        POST logoutUrl with the authservice session as a bearer token, then
//                        location.replace(afterLogoutURL)
// The iframe only ever loads same-origin paths (CD.safeSrc) and namespace messages go to the
// dashboard's own origin.
(function (root) {
  "use strict";
  var KF = root.KF, el = KF.el;
  var SVGNS = "http://www.w3.org/2000/svg";
  var ALL = "kubeflow-all-namespaces";

  // ---------------------------------------------------------------- pure helpers (exported)
  function origin() {
    var l = root.location;
    return l.origin || new URL(l.href).origin;
  }
  // an app path from the URL hash -> a same-origin "/path?query#frag", or null: leading slashes
  // are collapsed (no protocol-relative "//host"), and anything resolving elsewhere is refused
  function safeSrc(path) {
    if (typeof path !== "string") return null;
    var p = "/" + path.replace(/^[\s\/\\]+/, "");
    var u;
    try { u = new URL(p, origin()); } catch (e) { return null; }
    if (u.origin !== origin()) return null;
    return u.pathname + u.search + u.hash;
  }
  // registration-page _onUserDetails: the default namespace for a user id
  function defaultNamespace(user) {
    return String(user || "").replace(/[^\w]|\./g, "-").replace(/^-+|-+$|_/g, "").toLowerCase();
  }
  var NS_ERROR = "Name can only start and end with alpha-num characters, dashes are only permitted between start " +
                 "and end. (minlength >= 1)";
  function validateNamespace(name) {
    return /^[a-z0-9]([-a-z0-9]*[a-z0-9])?$/.test(name || "") ? null : NS_ERROR;
  }
  // utilities-mixin buildHref: set the known query parameters (ns) on an app link; the link's
  // fragment stays after the query, as URL.searchParams.set leaves it
  function buildHref(href, params) {
    var u = new URL(href, origin());
    ["ns"].forEach(function (k) { if (params && params[k]) u.searchParams.set(k, params[k]); });
    return u.href.slice(u.origin.length);
  }
  // resource-chart _buildDatasets: series by label, truncated to the 5 highest means
  var MAX_SERIES = 5, METRICS = ["node", "podcpu", "podmem"],
      INTERVALS = [["Last5m", "5m"], ["Last15m", "15m"], ["Last30m", "30m"], ["Last60m", "1h"], ["Last180m", "3h"]];
  function buildSeries(points) {
    var by = {}, order = [];
    (points || []).forEach(function (p) {
      if (!by[p.label]) { by[p.label] = { label: p.label, mean: 0, data: [] }; order.push(p.label); }
      var s = by[p.label];
      s.data.push({ t: p.timestamp, y: p.value });
      s.mean = (s.mean * (s.data.length - 1) + p.value) / s.data.length;
    });
    var series = order.map(function (k) { return by[k]; });
    var truncated = series.length > MAX_SERIES;
    if (truncated) series = series.slice().sort(function (a, b) { return b.mean - a.mean; }).slice(0, MAX_SERIES);
    return { series: series, truncated: truncated };
  }
  function metricUrl(metric, interval) {
    var m = METRICS.indexOf(metric) >= 0 ? metric : "node";
    var i = INTERVALS.some(function (x) { return x[0] === interval; }) ? interval : "Last15m";
    return "api/metrics/" + m + "?interval=" + i;
  }
  // manage-users-view nsBreakdown: [role, "ns1, ns2"] rows
  function nsBreakdown(namespaces) {
    var rows = [];
    [["owner", "Owner"], ["contributor", "Contributor"], ["viewer", "Viewer"]].forEach(function (r) {
      var names = (namespaces || []).filter(function (n) { return n.role === r[0]; }).map(function (n) { return n.namespace; });
      if (names.length) rows.push([r[1], names.join(", ")]);
    });
    return rows;
  }
  function errText(e) { return (e && e.message) || String(e); }
  function cookie(name) {
    var m = ("; " + document.cookie).split("; " + name + "=");
    return m.length > 1 ? m.pop().split(";")[0] : "";
  }

  // ---------------------------------------------------------------- resource-chart (SVG)
  function svg(tag, attrs) {
    var e = document.createElementNS ? document.createElementNS(SVGNS, tag) : document.createElement(tag);
    Object.keys(attrs || {}).forEach(function (k) { e.setAttribute(k, attrs[k]); });
    Array.prototype.slice.call(arguments, 2).forEach(function (c) { if (c) e.append(c); });
    return e;
  }
  var COLORS = ["#1e88e5", "#00acc1", "#e91e63", "#ff9800", "#9ccc65"];
  function resourceChart(opts) {
    var interval = opts.interval || "Last60m";
    var title = el("h2", { "data-cy": "chart-title" }, opts.header);
    var body = el("div", { class: "chart", "data-cy": "chart-body" });
    var sel = el("select", { "data-cy": "chart-interval", title: "Select interval" },
      INTERVALS.map(function (x) { return el("option", { value: x[0], selected: x[0] === interval }, x[1]); }));
    sel.value = interval;
    var card = el("section", { class: "card", "data-cy": "resource-chart", "data-metric": opts.metric },
      el("header", { class: "title-toolbar" }, title, el("span", { class: "spacer" }), sel,
         el("button", { "data-cy": "chart-refresh", title: "Refresh chart", onclick: function () { load(); } }, "Refresh")),
      body,
      opts.link ? el("footer", {}, el("a", { href: opts.link, target: "_blank", "data-cy": "chart-link" }, opts.linkText || "Charts")) : null);
    sel.addEventListener("change", function () { interval = sel.value; load(); });
    function draw(points) {
      var b = buildSeries(points), pct = opts.metric !== "podmem";
      title.textContent = opts.header + (b.truncated ? " (Top " + MAX_SERIES + ")" : "");
      if (!b.series.length) return body.replaceChildren(el("div", { class: "hint" }, "No data"));
      var W = 400, H = 200, P = 30, all = [];
      b.series.forEach(function (s) { all = all.concat(s.data); });
      var t0 = Math.min.apply(null, all.map(function (d) { return d.t; })), t1 = Math.max.apply(null, all.map(function (d) { return d.t; }));
      var ymax = Math.max.apply(null, all.map(function (d) { return d.y; }).concat([pct ? 1 : 0]));
      var x = function (t) { return P + (t1 > t0 ? (t - t0) / (t1 - t0) : 0) * (W - 2 * P); };
      var y = function (v) { return H - P - (ymax > 0 ? v / ymax : 0) * (H - 2 * P); };
      var lines = b.series.map(function (s, i) {
        return svg("polyline", { fill: "none", stroke: COLORS[i % COLORS.length], "stroke-width": "2", "data-label": s.label,
                                 points: s.data.map(function (d) { return x(d.t).toFixed(1) + "," + y(d.y).toFixed(1); }).join(" ") });
      });
      var axis = svg("text", { x: "2", y: String(P), "data-cy": "chart-ymax" }, document.createTextNode(pct ? (ymax * 100).toFixed(0) + "%" : String(ymax)));
      body.replaceChildren(svg.apply(null, ["svg", { viewBox: "0 0 " + W + " " + H, width: "100%", "data-cy": "chart-svg" }, axis].concat(lines)),
        el("ul", { class: "legend", "data-cy": "chart-legend" }, b.series.map(function (s, i) {
          return el("li", { style: "color:" + COLORS[i % COLORS.length] }, s.label);
        })));
    }
    function load() {
      return KF.api("GET", metricUrl(opts.metric, interval), null, { quiet: true })
        .then(function (pts) { draw(Array.isArray(pts) ? pts : []); },
              function (e) { body.replaceChildren(el("div", { class: "err" }, "Could not load metrics: " + errText(e))); });
    }
    card.load = load;
    load();
    return card;
  }

  // ---------------------------------------------------------------- notebooks-card / pipelines-card
  var MAX_ITEMS = 5;
  function notebooksCard(ns) {
    var card = el("section", { class: "card", "data-cy": "notebooks-card" }, el("h2", {}, "Recent Notebooks"));
    var msg = el("div", { class: "hint", "data-cy": "card-message" });
    card.append(msg);
    if (!ns || ns === ALL) { msg.textContent = "Choose a namespace to see Notebooks"; return card; }
    msg.textContent = "Loading...";
    KF.api("GET", "/jupyter/api/namespaces/" + ns + "/notebooks", null, { quiet: true }).then(function (r) {
      return Promise.all((r.notebooks || []).map(function (n) {
        return KF.api("GET", "/notebook/" + n.namespace + "/" + n.name + "/api/contents", null, { quiet: true })
          .then(function (c) {
            return (c.content || []).map(function (f) {
              var d = new Date(f.last_modified);
              return { name: f.name, server: n.name, sort: d.getTime(), when: d.toLocaleString(),
                       href: "/notebook/" + n.namespace + "/" + n.name + "/notebooks/" + f.name };
            });
          }, function () { return []; });
      }));
    }).then(function (lists) {
      var items = [].concat.apply([], lists).sort(function (a, b) { return b.sort - a.sort; }).slice(0, MAX_ITEMS);
      msg.textContent = items.length ? "" : "No Notebooks in namespace " + ns;
      card.append(el("ul", { class: "links" }, items.map(function (n) {
        return el("li", {}, el("a", { href: "#/_" + n.href, "data-cy": "notebook-link" }, n.name),
                  el("span", { class: "hint" }, " Accessed " + n.when));
      })));
    }, function () { msg.textContent = "Error retrieving Notebooks"; });
    return card;
  }
  function pipelinesCard(heading, kind, ns) {
    var card = el("section", { class: "card", "data-cy": "pipelines-card", "data-kind": kind }, el("h2", {}, heading));
    var msg = el("div", { class: "hint", "data-cy": "card-message" }, "Loading...");
    card.append(msg);
    var url = "/pipeline/apis/v1beta1/" + kind + "?page_size=5&sort_by=created_at%20desc";
    if (kind === "runs") url += "&resource_reference_key.type=NAMESPACE&resource_reference_key.id=" + encodeURIComponent(ns || "");
    KF.api("GET", url, null, { quiet: true }).then(function (r) {
      var items = (r[kind] || []).slice(0, MAX_ITEMS).map(function (p) {
        var cls = kind === "runs" ? (p.status === "Succeeded" ? "success" : (p.status === "Error" || p.status === "Failed") ? "error" : "pending") : "pipeline";
        return el("li", { "data-status": cls }, el("span", { class: "status-" + cls, title: p.status || "" },
                  cls === "success" ? "✔ " : cls === "error" ? "✖ " : cls === "pending" ? "⏲ " : ""),
                  el("a", { href: "#/_" + buildHref("/pipeline/#/" + kind + "/details/" + p.id, { ns: ns }), "data-cy": "pipeline-link" }, p.name),
                  el("span", { class: "hint" }, " Created " + new Date(p.created_at).toLocaleString()));
      });
      msg.textContent = items.length ? "" : "None Found";
      card.append(el("ul", { class: "links" }, items));
    }, function () { msg.textContent = kind === "pipelines" ? "Error retrieving Pipelines" : "Error retrieving Pipeline Runs"; });
    return card;
  }

  // ---------------------------------------------------------------- main page
  function start(app) {
    var j = function (p, quiet) { return KF.api("GET", p, null, { quiet: quiet }); };
    return j("api/workgroup/exists").then(function (ex) {
      if (ex.registrationFlowAllowed && ex.hasAuth && !ex.hasWorkgroup) return registration(app, ex);
      return Promise.all([j("api/workgroup/env-info"), j("api/dashboard-links", true).catch(function () { return {}; }),
                          j("api/metrics", true).catch(function () { return null; })]).then(function (r) {
        mainPage(app, r[0], r[1] || {}, r[2]);
      });
    });
  }

  function registration(app, ex) {
    var name = el("input", { "data-cy": "registration-namespace", maxlength: "253", value: defaultNamespace(ex.user) });
    var error = el("div", { class: "err", "data-cy": "registration-error" });
    var finish = el("button", { "data-cy": "registration-finish" }, "Finish");
    var back = el("button", { "data-cy": "registration-back" }, "Go back");
    var page0 = el("div", { "data-cy": "registration-welcome" }, el("h2", {}, "Welcome"),
      el("p", {}, "In order to use Kubeflow, a namespace for your account must be created. Follow the steps to get started"),
      el("button", { "data-cy": "registration-start", onclick: function () { show(1); } }, "Start Setup"));
    var page1 = el("div", { "data-cy": "registration-namespace-page", hidden: true }, el("h2", {}, "Namespace"),
      el("p", {}, "A namespace is a collection of Kubeflow services. Resources created within a namespace are isolated to " +
                  "that namespace. By default, a namespace will be created for you."),
      KF.field("Namespace Name", name), error, el("div", { class: "actions" }, finish, back));
    function show(i) { page0.hidden = i !== 0; page1.hidden = i !== 1; }
    name.addEventListener("input", function () { error.textContent = ""; });
    back.addEventListener("click", function () { show(0); });
    function poll(times) {
      return j0().then(function (r) {
        if (r && r.hasWorkgroup) return true;
        if (times <= 1) return false;
        return new Promise(function (res) { setTimeout(res, 300); }).then(function () { return poll(times - 1); });
      });
    }
    function j0() { return KF.api("GET", "api/workgroup/exists", null, { quiet: true }).catch(function () { return null; }); }
    finish.addEventListener("click", function () {
      var v = validateNamespace(name.value);
      if (v) { error.textContent = v; return; }
      finish.disabled = back.disabled = name.disabled = true;
      KF.api("POST", "api/workgroup/create", { namespace: name.value }, { quiet: true }).then(function () {
        return poll(66).then(function (ok) {
          if (ok) { app.dataset.flowComplete = "true"; root.location.reload(); }
          else error.textContent = "The namespace is not ready yet; press Finish to check again.";
        });
      }, function (e) { error.textContent = errText(e); }).then(function () {
        finish.disabled = back.disabled = name.disabled = false;
      });
    });
    app.replaceChildren(el("div", { class: "card registration", "data-cy": "registration-page" }, page0, page1));
  }

  function mainPage(app, env, links, metrics) {
    var nsList = env.namespaces || [];
    var platform = env.platform || {};
    var logoutUrl = platform.logoutUrl || "/logout";
    var stored = null;
    try { stored = root.localStorage.getItem("/centraldashboard/selectedNamespace/" + (env.user || "")); } catch (e) { stored = null; }
    var sel = el("select", { "data-cy": "namespace-selector" }, nsList.map(function (b) {
      return el("option", { value: b.namespace }, b.namespace + " (" + b.role + ")");
    }));
    var q = new URLSearchParams((root.location.hash.split("?")[1] || ""));
    var want = q.get("ns") || stored;
    if (want && nsList.some(function (b) { return b.namespace === want; })) sel.value = want;
    var logout = el("button", { "data-cy": "logout-button", title: "Logout", onclick: function () {
      fetch(new URL(logoutUrl, origin()).href, { method: "POST", credentials: "same-origin",
                         headers: { Authorization: "Bearer " + cookie("authservice_session") } })
        .then(function (r) { return r.json(); })
        .then(function (b) { root.location.replace(b.afterLogoutURL || "/"); },
              function (e) { KF.snack("Logout failed: " + errText(e), true); });
    } }, "Logout");
    var main = el("div", { class: "dash-main", "data-cy": "outlet" });
    var nav = el("nav", { "data-cy": "sidenav" });
    app.replaceChildren(el("header", { "data-cy": "toolbar" }, el("h1", {}, "Kubeflow on MI355X"), sel,
                           el("span", { "data-cy": "user" }, env.user || ""), logout),
                        el("div", { class: "dash" }, nav, main));
    var frame = null;
    function ns() { return sel.value || ""; }
    function post() {
      if (frame && frame.contentWindow) {
        frame.contentWindow.postMessage(ns() === ALL ? { type: "all-namespaces" } : { type: "namespace-selected", value: ns() },
                                        origin());
      }
    }
    root.addEventListener("message", function (ev) {          // library.js protocol, own origin only
      if (ev.origin !== origin()) return;                    // an empty origin is not ours either
      if (ev.data && ev.data.type === "iframe-connected") post();
    });
    sel.addEventListener("change", function () {
      try { root.localStorage.setItem("/centraldashboard/selectedNamespace/" + (env.user || ""), ns()); } catch (e) { /* private mode */ }
      post();
      route();
    });
    function renderNav() {
      var items = [el("a", { href: "#/" }, "Home")];
      (links.menuLinks || []).forEach(function (l) {
        items.push(el("a", { href: "#/_" + buildHref(l.link.split("{ns}").join(ns() || "{ns}"), { ns: ns() }), "data-cy-menu": l.text }, l.text));
      });
      items.push(el("a", { href: "#/activity" }, "Activity"), el("a", { href: "#/manage-users", "data-cy-menu": "manage-users" }, "Manage Contributors"));
      (links.externalLinks || []).forEach(function (l) { items.push(el("a", { href: l.link, target: "_blank" }, l.text)); });
      nav.replaceChildren.apply(nav, items);
    }
    function route() {
      renderNav();
      var h = (root.location.hash || "#/").slice(1).split("?")[0] || "/";
      if (h === "/") return home();
      if (h === "/activity") return activity();
      if (h === "/manage-users") return manageUsers();
      if (h === "/namespace-needed") return namespaceNeeded();
      if (h.indexOf("/_/") === 0) return iframe(decodeURIComponent((root.location.hash || "").slice(3)));
      return notFound(h);
    }
    function iframe(path) {
      if (path.indexOf("{ns}") >= 0) {
        if (!nsList.length) { root.location.hash = "#/namespace-needed"; return; }
        path = path.split("{ns}").join(ns());
      }
      var src = safeSrc(path);
      if (src === null) return main.replaceChildren(el("div", { class: "error-page", "data-cy": "refused" }, "Refusing to load ", el("b", {}, path),
                                                      ": not a path of this site."));
      if (!frame) {
        frame = el("iframe", { name: "content", "data-cy": "iframe" });
        frame.addEventListener("load", post);
      }
      frame.src = src;
      main.replaceChildren(frame);
    }
    function home() {
      var quick = (links.quickLinks || []).map(function (l) {
        return el("li", {}, el("a", { href: "#/_" + buildHref(l.link, { ns: ns() }), "data-cy": "quick-link" }, l.text),
                  l.desc ? el("span", { class: "hint" }, " " + l.desc) : null);
      });
      var charts = metrics && metrics.resourceChartsLinkText ? [
        resourceChart({ header: "Cluster CPU Utilization", metric: "node", interval: "Last60m", link: metrics.resourceChartsLink,
                        linkText: metrics.resourceChartsLinkText }),
        resourceChart({ header: "Pod CPU Utilization", metric: "podcpu", interval: "Last60m", link: metrics.resourceChartsLink,
                        linkText: metrics.resourceChartsLinkText })] : [];
      var docs = (links.documentationItems || []).map(function (d) {
        return el("li", {}, el("a", { href: d.link, target: "_blank" }, d.text), d.desc ? el("span", { class: "hint" }, " " + d.desc) : null);
      });
      main.replaceChildren(el("div", { class: "grid", "data-cy": "dashboard-view" },
        el("div", { class: "column" }, el("section", { class: "card", "data-cy": "quick-links" }, el("h2", {}, "Quick shortcuts"),
                                          el("ul", { class: "links" }, quick)), charts),
        el("div", { class: "column" }, notebooksCard(ns()), pipelinesCard("Recent Pipelines", "pipelines", ns()),
           pipelinesCard("Recent Pipeline Runs", "runs", ns())),
        el("div", { class: "column" }, el("section", { class: "card", "data-cy": "documentation" }, el("h2", {}, "Documentation"),
                                          el("ul", { class: "links" }, docs)))));
    }
    function activity() {
      var box = el("div", { class: "card", "data-cy": "activity-view" }, el("h2", {}, "Activity in " + ns()));
      main.replaceChildren(box);
      KF.api("GET", "api/activities/" + ns(), null, { quiet: true }).then(function (evs) {
        box.append(KF.table([["Time", function (e) { return KF.dateTime(e.lastTimestamp || e.eventTime); }],
                             ["Type", function (e) { return e.type; }],
                             ["Object", function (e) { return (e.involvedObject || {}).kind + "/" + (e.involvedObject || {}).name; }],
                             ["Message", function (e) { return e.message; }]], (Array.isArray(evs) ? evs : []).slice(0, 50),
                            { empty: "No recent activity." }));
      }, function (e) { box.append(el("div", { class: "err" }, "Could not load activities: " + errText(e))); });
    }
    function manageUsers() {
      var owned = nsList.filter(function (n) { return n.role === "owner"; });
      var rows = nsBreakdown(nsList);
      var view = el("div", { "data-cy": "manage-users-view" }, el("h2", { class: "page-title" }, "Manage Contributors"),
        el("section", { class: "card", "data-cy": "account-info" }, el("h3", {}, "Account Information"), el("span", {}, env.user || ""),
           env.isClusterAdmin ? el("b", { style: "color:red" }, " (Cluster Admin)") : null),
        el("section", { class: "card", "data-cy": "memberships" }, el("h3", {}, "Profile Memberships"),
           rows.length ? KF.table([["Your Role", function (r) { return r[0]; }], ["Namespaces", function (r) { return r[1]; }]], rows)
                       : el("span", {}, "You don't have any namespace memberships.")));
      main.replaceChildren(view);
      if (env.isClusterAdmin) {
        var all = el("section", { class: "card", "data-cy": "cluster-namespaces" }, el("h3", {}, "Profiles Overview (Cluster Admin)"));
        view.append(all);
        KF.api("GET", "api/workgroup/get-all-namespaces", null, { quiet: true }).then(function (list) {
          all.append(KF.table([["Namespace", function (r) { return r[0]; }], ["Owner", function (r) { return r[1]; }],
                               ["Contributors", function (r) { return r[2]; }]], list || []));
        }, function (e) { KF.snack("Failed to fetch all namespaces, because: " + errText(e), true); });
      }
      owned.forEach(function (o) { view.append(contributors(o.namespace)); });
    }
    // manage-users-view-contributor: chips with remove, an add field; a failed add / remove shows
    // the backend error under the field (contribCreateError), a failed fetch a toast
    function contributors(namespace) {
      var box = el("section", { class: "card", "data-cy": "contributors", "data-namespace": namespace },
                   el("h3", {}, "Contributors for - ", el("code", {}, namespace)));
      var chips = el("div", { class: "chips", "data-cy": "contributor-chips" });
      var input = el("input", { placeholder: "Add by email address", "data-cy": "contributor-input" });
      var error = el("div", { class: "err", "data-cy": "contributor-error" });
      function render(list) {
        chips.replaceChildren.apply(chips, (list || []).map(function (u) {
          return el("span", { class: "chip", "data-cy": "contributor" }, u,
                    el("button", { "data-cy": "contributor-remove", title: "Remove " + u, onclick: function () { change("DELETE", u); } }, "×"));
        }));
      }
      function change(method, who) {
        return KF.api(method, "api/workgroup/" + (method === "POST" ? "add" : "remove") + "-contributor/" + namespace,
                      { contributor: who }, { quiet: true })
          .then(function (list) { error.textContent = ""; if (method === "POST") input.value = ""; render(list); },
                function (e) { error.textContent = errText(e); });
      }
      input.addEventListener("keydown", function (ev) { if (ev.key === "Enter" && input.value) change("POST", input.value); });
      box.append(chips, input, el("button", { "data-cy": "contributor-add", onclick: function () { if (input.value) change("POST", input.value); } }, "Add"), error);
      KF.api("GET", "api/workgroup/get-contributors/" + namespace, null, { quiet: true }).then(render, function (e) {
        KF.snack("Failed to fetch contributor list for " + namespace + ", because: " + errText(e), true);
      });
      return box;
    }
    function namespaceNeeded() {
      main.replaceChildren(el("div", { class: "error-page", "data-cy": "namespace-needed" },
        el("div", {}, "This page requires a namespace to be selected but no namespaces are currently available."),
        el("a", { href: "#/" }, "back to home")));
    }
    function notFound(h) {
      main.replaceChildren(el("div", { class: "error-page", "data-cy": "not-found" }, el("div", { class: "headline" }, "404"),
        el("div", {}, "Sorry, ", el("b", {}, h), " is not a valid page."), el("a", { href: "#/" }, "back to home")));
    }
    root.addEventListener("hashchange", route);
    route();
  }

  root.CD = { start: start, safeSrc: safeSrc, defaultNamespace: defaultNamespace, validateNamespace: validateNamespace,
              buildHref: buildHref, buildSeries: buildSeries, metricUrl: metricUrl, nsBreakdown: nsBreakdown, NS_ERROR: NS_ERROR };
})(self);
