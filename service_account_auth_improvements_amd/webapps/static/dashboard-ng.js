// Central dashboard, second frontend (T3): the behaviour of
// components/centraldashboard-angular/frontend/src/app as its own single-page app, on the shared
// kubeflow-common-lib port (lib/kf-common.js) and the same /api backend (webapps/dashboard.py).
//
//   services/environment.service.ts  -> Env          env-info (user, namespaces, platform) + dashboard links
//   services/local-storage.service.ts-> Store        JSON values in localStorage
//   services/namespace.service.ts    -> Namespaces   option list with "All namespaces", the current
//                                                    namespace: ?ns= > stored choice > owned > first
//   guards/iframe.guard.ts           -> iframeGuard  "{ns}" in an app path -> #/namespace-needed
//   interceptors/error.interceptor.ts-> KF.api       (kf-common.js: "[status] log" snacks)
//   app-routing.module.ts            -> ROUTES       "" home, "_/**" app in the iframe, namespace-needed, 404
//   pages/main-page (+ namespace-selector), home-page, iframe-wrapper, namespace-needed-page,
//   not-found-page                   -> the page functions below
//
// Routing is hash based: #/<path>?ns=<namespace>.  The iframe protocol is the dashboard
// library's (public/library.js): the app posts "iframe-connected", the dashboard answers with
// "namespace-selected"; the dashboard mirrors the iframe's own navigation into its URL.
(function (root) {
  "use strict";
  function ownOrigin() {
    return root.location.origin || new URL(root.location.href).origin;
  }
  var KF = root.KF, el = KF.el;
  var ALL_NAMESPACES = "All namespaces";
  // apps whose index pages can list every namespace at once (namespace.service.ts)
  var ALL_NAMESPACES_ALLOWED_LIST = ["jupyter", "volumes", "tensorboards", "katib", "models"];

  // ------------------------------------------------------------------ services
  var Store = {
    get: function (k) {
      var v = root.localStorage.getItem(k);
      if (v === null || v === undefined) return null;
      try { return JSON.parse(v); } catch (e) { return null; }
    },
    set: function (k, v) { root.localStorage.setItem(k, JSON.stringify(v === undefined ? null : v)); }
  };

  function parseHash(h) {
    h = (h || "").replace(/^#/, "") || "/";
    var q = h.indexOf("?"), path = q >= 0 ? h.slice(0, q) : h, query = {};
    new URLSearchParams(q >= 0 ? h.slice(q + 1) : "").forEach(function (v, k) { query[k] = v; });
    return { path: path || "/", query: query };
  }
  function buildHash(path, query) {
    var qs = new URLSearchParams();
    Object.keys(query || {}).forEach(function (k) { if (query[k] !== undefined && query[k] !== null) qs.set(k, query[k]); });
    var s = qs.toString();
    return "#" + path + (s ? "?" + s : "");
  }

  function Namespaces(env) {
    var self = this;
    this.user = env.user || "";
    this.base = (env.namespaces || []).map(function (n) {
      return { namespace: n.namespace, role: n.role, user: n.user, disabled: false };
    });
    this.current = null;
    this.listeners = [];
    this.key = function () { return "selectedNamespace/" + (self.user ? "." + self.user : ""); };
  }
  Namespaces.prototype.allowedAll = function (path) {
    var p = path.indexOf("/_/") === 0 ? path.slice(3) : path.replace(/^\//, "");
    return ALL_NAMESPACES_ALLOWED_LIST.some(function (a) { return p.indexOf(a) === 0; });
  };
  Namespaces.prototype.options = function (path) {
    return [{ namespace: ALL_NAMESPACES, role: "", user: "", disabled: !this.allowedAll(path) }].concat(this.base);
  };
  Namespaces.prototype.valid = function (n) { return !!n && !(n.namespace === ALL_NAMESPACES && n.disabled); };
  Namespaces.prototype.find = function (name, opts) {
    return name ? opts.filter(function (n) { return n.namespace === name; })[0] : undefined;
  };
  // the namespace a navigation to `route` should show: query > stored choice > owned > first valid
  Namespaces.prototype.resolve = function (route) {
    var opts = this.options(route.path);
    var fromQuery = this.find(route.query.ns, opts);
    if (this.valid(fromQuery)) return fromQuery;
    var stored = this.find(Store.get(this.key()), opts);
    if (this.valid(stored)) return stored;
    var owned = opts.filter(function (n) { return n.role === "owner"; })[0];
    if (owned) return owned;
    return opts.filter(this.valid.bind(this))[0];
  };
  Namespaces.prototype.select = function (n) {
    var changed = !this.current || this.current.namespace !== n.namespace;
    this.current = n;
    Store.set(this.key(), n.namespace);
    if (changed) this.listeners.forEach(function (f) { f(n); });
  };

  // guards/iframe.guard.ts
  function iframeGuard(route) {
    var decoded = decodeURIComponent(buildHash(route.path, route.query).slice(1));
    if (decoded.indexOf("{ns}") >= 0) return buildHash("/namespace-needed", { path: decoded });
    return null;
  }

  // ------------------------------------------------------------------ app
  function start() {
    var app = document.getElementById("app");
    var j = function (p, quiet) { return KF.api("GET", p, null, { quiet: quiet }); };
    Promise.all([j("api/workgroup/env-info"),
                 j("api/dashboard-links", true).catch(function () { return { menuLinks: [] }; })]).then(function (r) {
      var env = r[0], links = r[1] || {};
      var ns = new Namespaces(env);
      var iframed = root.self !== root.top && root.top !== undefined && root.parent !== root;
      var selector = el("select", { "data-cy-namespace-selector": "" });
      var outlet = el("div", { class: "dash-main", "data-cy": "outlet" });
      var menu = el("nav", { "data-cy": "sidenav" });
      var platform = env.platform || {};
      var footer = el("div", { class: "hint", "data-cy": "build" },
        platform.kubeflowVersion ? "Build version " + platform.kubeflowVersion : "",
        platform.providerName ? " · " + platform.providerName : "");
      var toolbar = el("header", { "data-cy": "toolbar" }, el("h1", {}, "Kubeflow"), selector, el("span", {}, env.user || ""));
      app.replaceChildren(iframed ? el("span") : toolbar, el("div", { class: "dash" }, el("div", {}, menu, footer), outlet));

      var frame = null, frameSeen = null, mode = null;
      function post() {
        if (frame && frame.contentWindow && ns.current) {
          var n = ns.current.namespace;
          frame.contentWindow.postMessage(n === ALL_NAMESPACES ? { type: "all-namespaces" }
                                                              : { type: "namespace-selected", value: n }, ownOrigin());
        }
      }
      ns.listeners.push(post);
      root.addEventListener("message", function (ev) {
        if (ev.origin !== ownOrigin()) return;               // an empty origin is not ours either
        if (ev.data && ev.data.type === "iframe-connected") post();
      });

      // main-page getUrlPath / getNamespaceParams: an app link as a dashboard route -- the {ns}
      // placeholder resolved (kept when no namespace is selected, for the iframe guard), ?ns added
      // unless the link carries its own, an in-app fragment (#/runs) kept
      function appHash(link) {
        var n = ns.current && ns.current.namespace !== ALL_NAMESPACES ? ns.current.namespace : "{ns}";
        var resolved = link.split("{ns}").join(n);
        if (/[?&]ns=/.test(link) || !ns.current) return "#/_" + resolved;
        var at = resolved.indexOf("#"), head = at >= 0 ? resolved.slice(0, at) : resolved, frag = at >= 0 ? resolved.slice(at) : "";
        return "#/_" + head + (head.indexOf("?") >= 0 ? "&" : "?") + "ns=" + encodeURIComponent(ns.current.namespace) + frag;
      }
      function renderMenu(route) {
        var q = ns.current ? { ns: ns.current.namespace } : {};
        var items = [el("a", { href: buildHash("/", q), "data-cy-sidenav-menu-item": "Home",
                               class: route.path === "/" ? "active" : "" }, "Home")];
        (links.menuLinks || []).forEach(function (l) {
          items.push(el("a", { href: appHash(l.link), "data-cy-sidenav-menu-item": l.text,
                               class: route.path.indexOf("/_" + l.link.split("{ns}")[0].split("#")[0]) === 0 ? "active" : "" }, l.text));
        });
        menu.replaceChildren.apply(menu, items);
      }
      function renderSelector(route) {
        selector.replaceChildren.apply(selector, ns.options(route.path).map(function (n) {
          return el("option", { value: n.namespace, disabled: n.disabled, selected: ns.current && n.namespace === ns.current.namespace },
                    n.namespace);
        }));
        if (ns.current) selector.value = ns.current.namespace;
      }
      selector.addEventListener("change", function () {
        var route = parseHash(location.hash);
        var n = ns.find(selector.value, ns.options(route.path));
        if (!ns.valid(n)) return;
        route.query.ns = n.namespace;
        ns.select(n);
        location.hash = buildHash(route.path, route.query);
      });

      // ---------------------------------------------------------------- pages
      function home() {
        mode = "home";
        var quick = links.quickLinks || [], docs = links.documentationItems || [];
        outlet.replaceChildren(el("div", { class: "card", "data-cy": "home" },
          el("h2", {}, "Welcome" + (env.user ? ", " + env.user : "")),
          el("h3", {}, "Quick shortcuts"),
          el("ul", {}, quick.map(function (l) {
            return el("li", {}, el("a", { href: appHash(l.link) }, l.text),
                      l.desc ? el("span", { class: "hint" }, " " + l.desc) : null);
          })),
          el("h3", {}, "Documentation"),
          el("ul", {}, docs.map(function (d) { return el("li", {}, el("a", { href: d.link, target: "_blank" }, d.text)); }))));
      }
      function notFound(route) {
        mode = "404";
        outlet.replaceChildren(el("div", { class: "error-page", "data-cy": "not-found" }, el("div", { class: "headline" }, "404"),
          el("div", {}, "Sorry, ", el("b", {}, route.path), " is not a valid page."), el("a", { href: "#/" }, "back to home")));
      }
      function namespaceNeeded(route) {
        mode = "namespace-needed";
        outlet.replaceChildren(el("div", { class: "error-page", "data-cy": "namespace-needed" },
          el("div", {}, "This page requires a namespace to be selected but no namespaces are currently available."),
          route.query.path ? el("div", { class: "hint" }, route.query.path) : null,
          el("a", { href: "#/" }, "back to home")));
      }
      // iframe-wrapper: the app path without the "/_" prefix, with a trailing "/" (Istio-exported
      // services expect one), and the namespace as ?ns=; the iframe is only reloaded when the
      // browser URL and the iframe's own location differ
      // (the upstream wrapper prefixes window.location.origin: leading slashes are collapsed and a
      // src that still resolves to another origin is refused -- "#/_//evil.example/" loads nothing)
      function srcFor(route) {
        var p = "/" + (route.path.slice(2) || "/").replace(/^[\s\/\\]+/, "");
        var hashAt = p.indexOf("#"), frag = "";
        if (hashAt >= 0) { frag = p.slice(hashAt); p = p.slice(0, hashAt); }
        if (p[p.length - 1] !== "/" && p.split("/").pop().indexOf(".") < 0) p += "/";
        var q = {};
        Object.keys(route.query).forEach(function (k) { q[k] = route.query[k]; });
        var qs = new URLSearchParams(q).toString();
        var u;
        try { u = new URL(p + (qs ? "?" + qs : "") + frag, ownOrigin()); } catch (e) { return null; }
        return u.origin === ownOrigin() ? u.pathname + u.search + u.hash : null;
      }
      function iframeWrapper(route) {
        var src = srcFor(route);
        if (src === null) {
          mode = "refused";
          outlet.replaceChildren(el("div", { class: "error-page", "data-cy": "refused" }, "Refusing to load ",
                                    el("b", {}, route.path.slice(2)), ": not a path of this site."));
          return;
        }
        if (mode !== "iframe" || !frame) {
          frame = el("iframe", { name: "content", "data-cy": "iframe" });
          frame.addEventListener("load", post);
          outlet.replaceChildren(frame);
        }
        mode = "iframe";
        if (frameSeen !== src) {
          frame.src = src;
          frameSeen = src;
        }
      }
      // mirror the iframe's own navigation into the dashboard URL (the wrapper's 100 ms poll)
      function pollFrame() {
        try {   // a cross-origin frame throws on .location: skip this tick, keep polling
          if (mode === "iframe" && frame && frame.contentWindow && frame.contentWindow.location) {
            var l = frame.contentWindow.location, now = l.pathname + (l.search || "") + (l.hash || "");
            if (l.pathname && now !== frameSeen) {
              frameSeen = now;
              var q = {};
              new URLSearchParams(l.search || "").forEach(function (v, k) { q[k] = v; });
              if (!q.ns && ns.current) q.ns = ns.current.namespace;
              location.hash = buildHash("/_" + l.pathname + (l.hash || ""), q);
            }
          }
        } catch (e) {
          /* SecurityError on a cross-origin document */
        } finally {
          root.setTimeout(pollFrame, 100);
        }
      }

      function navigate() {
        var route = parseHash(location.hash);
        if (route.path.indexOf("/_/") === 0 || route.path === "/_") {
          var redirect = iframeGuard(route);
          if (redirect) { location.hash = redirect; return; }
        }
        var want = ns.resolve(route);
        if (want) {
          ns.select(want);
          if (route.query.ns !== want.namespace && route.path !== "/namespace-needed") {   // keep ?ns in the URL
            route.query.ns = want.namespace;
            location.hash = buildHash(route.path, route.query);
            return;
          }
        }
        renderSelector(route);
        renderMenu(route);
        if (route.path === "/") return home();
        if (route.path === "/namespace-needed") return namespaceNeeded(route);
        if (route.path.indexOf("/_/") === 0) return iframeWrapper(route);
        return notFound(route);
      }
      root.addEventListener("hashchange", navigate);
      navigate();
      root.setTimeout(pollFrame, 100);
    }).catch(function () {});          // KF.api (the error interceptor) has shown the snack
  }

  root.CDB = { parseHash: parseHash, buildHash: buildHash, Namespaces: Namespaces, iframeGuard: iframeGuard,
               ALL_NAMESPACES: ALL_NAMESPACES, Store: Store };
  if (document.getElementById("app") && document.getElementById("app").getAttribute("data-app") === "dashboard-ng") start();
})(self);
