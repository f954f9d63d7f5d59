// kubeflow-common-lib components for the kfamd web UI (DOM side; the logic is kf-logic.js).
// Reference: crud-web-apps/common/frontend/kubeflow-common-lib/projects/kubeflow/src/lib/
// {resource-table, status-icon, namespace-select, snack-bar, editor, conditions-table,
//  logs-viewer, details-list, title-actions-toolbar, confirm-dialog, help-popover, date-time,
//  variables-groups-table, services/backend, services/poller} and the central dashboard's
// error interceptor (centraldashboard-angular/frontend/src/app/interceptors).
(function (root) {
  "use strict";
  var L = root.KFL;
  var base = (document.querySelector("base") || {}).href || "/";

  function el(tag, attrs) {
    var e = document.createElement(tag);
    var a = attrs || {};
    Object.keys(a).forEach(function (k) {
      var v = a[k];
      if (v === undefined || v === null || v === false) return;
      if (k.indexOf("on") === 0) e.addEventListener(k.slice(2), v);
      else if (k === "class") e.className = v;
      else if (k === "value") e.value = v;
      else if (k === "checked") e.checked = !!v;
      else e.setAttribute(k, v === true ? "" : v);
    });
    var kids = Array.prototype.slice.call(arguments, 2);
    (function add(list) {
      list.forEach(function (k) {
        if (Array.isArray(k)) add(k);
        else if (k !== undefined && k !== null && k !== false) e.append(k instanceof Node ? k : document.createTextNode(String(k)));
      });
    })(kids);
    return e;
  }

  function cookie(name) {
    var m = document.cookie.match(new RegExp("(?:^|; )" + name + "=([^;]*)"));
    return m ? decodeURIComponent(m[1]) : "";
  }

  // error interceptor (centraldashboard-angular interceptors/error.interceptor.ts): the snack
  // text for a failed request -- [status] backend log + URL, or "could not connect" -- while the
  // rejected promise carries the backend's log line itself
  function backendLog(status, j, statusText) {
    if (j && j.log) return j.log;
    if (j && j.error) return typeof j.error === "string" ? j.error : JSON.stringify(j.error);
    return status + ": " + (statusText || "error");
  }
  function snackErrorMessage(e) {
    if (typeof e === "string") return "An error occurred: " + e;
    if (e && e.status !== undefined) {
      if (e.status <= 0) return "Could not connect to the backend.";
      return "[" + e.status + "] " + e.message + "\n" + (e.url || "");
    }
    return (e && e.message) || "Unexpected error encountered";
  }
  function HttpError(status, message, url) {
    var e = new Error(message);
    e.status = status;
    e.url = url;
    return e;
  }

  // backend service: the crud_backend response envelope {success, status, log, <payload>};
  // failures go through the error interceptor (snack unless opts.quiet) and reject
  function api(method, path, body, opts) {
    opts = opts || {};
    var headers = { "Content-Type": "application/json" };
    if (["GET", "HEAD"].indexOf(method) < 0) headers["X-XSRF-TOKEN"] = cookie("XSRF-TOKEN");
    var url = new URL(path, base);
    return fetch(url, { method: method, headers: headers, credentials: "same-origin",
                        body: body ? JSON.stringify(body) : undefined })
      .then(function (r) {
        return r.json().catch(function () { return {}; }).then(function (j) {
          if (!r.ok || j.success === false) throw HttpError(r.status || j.status || 500, backendLog(r.status, j, r.statusText), url.href);
          return j;
        });
      }, function () { throw HttpError(0, "Could not connect to the backend.", url.href); })
      .catch(function (e) {
        if (!opts.quiet) snack(snackErrorMessage(e), true);
        throw e;
      });
  }

  function snack(msg, err) {
    var s = el("div", { class: "snack" + (err ? " err" : ""), role: "status",
                        "data-cy-snack-status": err ? "ERROR" : "SUCCESS" }, msg);
    document.body.append(s);
    setTimeout(function () { s.remove(); }, 5000);
  }

  // confirm-dialog (kubeflow-common-lib confirm-dialog): a modal with a title, a message and
  // accept / cancel; resolves true on accept.  The accept button shows the "applying" text while
  // opts.onAccept's promise runs; an error there stays in the dialog.
  function confirmDialog(opts) {
    return new Promise(function (resolve) {
      var err = el("div", { class: "err", "data-cy": "dialog-error" });
      var accept = el("button", { class: "accept", "data-cy": "dialog-accept" }, opts.accept || "DELETE");
      var cancel = el("button", { "data-cy": "dialog-cancel" }, opts.cancel || "CANCEL");
      var box = el("div", { class: "dialog-backdrop", role: "dialog", "aria-modal": "true" },
        el("div", { class: "dialog" }, el("h3", { "data-cy": "dialog-title" }, opts.title || "Are you sure?"),
          el("p", { "data-cy": "dialog-message" }, opts.message || ""), err, el("div", { class: "actions" }, cancel, accept)));
      function close(v) { box.remove(); resolve(v); }
      cancel.addEventListener("click", function () { close(false); });
      accept.addEventListener("click", function () {
        if (!opts.onAccept) return close(true);
        accept.disabled = true;
        accept.textContent = opts.applying || "DELETING";
        Promise.resolve().then(opts.onAccept).then(function () { close(true); }, function (e) {
          accept.disabled = false;
          accept.textContent = opts.accept || "DELETE";
          err.textContent = (e && e.message) || String(e);
        });
      });
      document.body.append(box);
    });
  }

  // help-popover (kubeflow-common-lib help-popover): a "?" that toggles a short help text
  function helpPopover(text) {
    var pop = el("div", { class: "popover", role: "tooltip", hidden: true }, text);
    var btn = el("button", { type: "button", class: "help", "aria-label": "help", onclick: function () {
      pop.hidden = !pop.hidden;
      if (pop.hidden) pop.setAttribute("hidden", ""); else pop.removeAttribute("hidden");
    } }, "?");
    pop.hidden = true;
    return el("span", { class: "help-popover" }, btn, pop);
  }

  // date-time (kubeflow-common-lib date-time): the relative age, the absolute time on hover
  function dateTime(ts) {
    if (!ts) return el("span", { class: "muted" }, "-");
    var d = new Date(ts);
    return el("span", { class: "date-time", title: isNaN(d) ? String(ts) : d.toISOString() }, L.age(ts));
  }

  // title-actions-toolbar (kubeflow-common-lib title-actions-toolbar): back link, title, buttons
  function titleToolbar(title, actions, backHref) {
    return el("div", { class: "toolbar title-toolbar" },
      backHref ? el("a", { href: backHref, class: "back", "aria-label": "back" }, "←") : null,
      el("h2", { "data-cy-toolbar-title": "" }, title), el("span", { class: "spacer" }), actions || null);
  }

  // variables-groups-table (kubeflow-common-lib variables-groups-table): groups of
  // key / value variables (a PodDefault's env, a notebook's configurations)
  function variablesGroupsTable(groups) {
    var rows = [];
    (groups || []).forEach(function (g) {
      var vars = g.variables || [];
      if (!vars.length) rows.push(el("tr", {}, el("td", { class: "group" }, g.name), el("td", { colspan: 2, class: "muted" }, "-")));
      vars.forEach(function (v, i) {
        rows.push(el("tr", {}, el("td", { class: "group" }, i === 0 ? g.name : ""), el("td", { class: "key" }, v[0]),
                     el("td", { class: "value" }, v[1] === undefined ? "" : v[1])));
      });
    });
    return el("table", { class: "rt vgt" }, el("thead", {}, el("tr", {}, el("th", {}, "Group"), el("th", {}, "Name"),
                                                                 el("th", {}, "Value"))), el("tbody", {}, rows));
  }

  var ICON = { ready: "✔", waiting: "⏳", warning: "⚠", error: "✖", stopped: "⏹",
               terminating: "✖", unavailable: "⚠", uninitialized: "•" };
  function status(st) {
    st = st || {};
    return el("span", { class: "st st-" + (st.phase || ""), title: st.message || "" }, ICON[st.phase] || "?", " ",
              st.phase || "");
  }

  // resource table: cols = [[title, render(row), sortKey(row)?], ...]; click a sortable header;
  // opts.sortBy = the title of the column sorted (ascending) on first render
  function table(cols, rows, opts) {
    opts = opts || {};
    var first = -1;
    cols.forEach(function (c, i) { if (c[0] === opts.sortBy && c[2]) first = i; });
    var state = { col: first, dir: 1 };
    var body = el("tbody");
    function render() {
      var rs = rows.slice();
      if (state.col >= 0) {
        var key = cols[state.col][2];
        rs.sort(function (a, b) { var x = key(a), y = key(b); return (x > y ? 1 : x < y ? -1 : 0) * state.dir; });
      }
      body.replaceChildren.apply(body, rs.length ? rs.map(function (r) {
        return el("tr", { onclick: opts.onRow ? function (ev) { if (ev.target.tagName !== "BUTTON" && ev.target.tagName !== "A") opts.onRow(r); } : null,
                          class: opts.onRow ? "clickable" : null },
                  cols.map(function (c) { return el("td", { "data-cy-resource-table-row": c[0] }, c[1](r)); }));
      }) : [el("tr", {}, el("td", { colspan: cols.length, class: "empty" }, opts.empty || "No resources found."))]);
    }
    var head = el("tr", {}, cols.map(function (c, i) {
      return el("th", { class: c[2] ? "sortable" : null, "data-cy-table-header-row": c[0], onclick: c[2] ? function () {
        state.dir = state.col === i ? -state.dir : 1; state.col = i; render();
      } : null }, c[0]);
    }));
    render();
    return el("table", { class: "rt" }, el("thead", {}, head), body);
  }

  // PollerService.exponential
  function poll(fn) {
    var delay = 0, last = "", timer = null, stopped = false;
    function tick() {
      Promise.resolve().then(fn).then(function (data) {
        var sig = JSON.stringify(data);
        delay = L.nextPollDelay(delay, sig !== last);
        last = sig;
      }, function (e) { snack(e.message, true); delay = L.nextPollDelay(delay, false); })
        .then(function () { if (!stopped) timer = setTimeout(tick, delay); });
    }
    tick();
    return { reset: function () { delay = 0; clearTimeout(timer); tick(); },
             stop: function () { stopped = true; clearTimeout(timer); } };
  }

  // namespace-select; opts.all adds the "All namespaces" entry (value ALL_NS)
  var ALL_NS = "*";
  function namespaceSelect(onChange, opts) {
    opts = opts || {};
    var sel = el("select", { id: "ns", "aria-label": "namespace" });
    var qs = new URLSearchParams(location.search).get("ns") || sessionStorage.getItem("kf-ns");
    return api("GET", "api/namespaces").then(function (j) { return j.namespaces || []; }, function () {
      return [];
    }).then(function (nss) {
      sel.namespaces = nss.slice();
      nss.forEach(function (n) { sel.append(el("option", { value: n }, n)); });
      if (opts.all) sel.append(el("option", { value: ALL_NS, "data-cy": "all-namespaces" }, "All namespaces"));
      if (qs && (nss.indexOf(qs) >= 0 || (opts.all && qs === ALL_NS))) sel.value = qs;
      sel.addEventListener("change", function () { sessionStorage.setItem("kf-ns", sel.value); onChange(sel.value); });
      window.addEventListener("message", function (ev) {        // central dashboard iframe protocol:
        // only the embedding dashboard (our parent frame, our own origin) may switch the namespace
        if (ev.source !== window.parent || ev.origin !== (location.origin || new URL(location.href).origin)) return;
        if (ev.data && ev.data.type === "namespace-selected") { sel.value = ev.data.value; onChange(sel.value); }
      });
      // the dashboard and the apps share one origin (behind the gateway): never post elsewhere
      if (window.parent !== window) window.parent.postMessage({ type: "iframe-connected" }, location.origin || new URL(location.href).origin);
      return sel;
    });
  }

  // tabs: [[title, render() -> Node | Promise<Node>], ...]
  function tabs(list) {
    var bar = el("div", { class: "tabs", role: "tablist" }), pane = el("div", { class: "tabpane" });
    var btns = list.map(function (t, i) {
      return el("button", { role: "tab", onclick: function () { show(i); } }, t[0]);
    });
    btns.forEach(function (b) { bar.append(b); });
    function show(i) {
      btns.forEach(function (b, j) { b.className = j === i ? "active" : ""; });
      pane.replaceChildren(el("div", { class: "muted" }, "Loading..."));
      Promise.resolve().then(list[i][1]).then(function (n) { pane.replaceChildren(n); },
                                               function (e) { pane.replaceChildren(el("div", { class: "err" }, e.message)); });
    }
    show(0);
    return el("div", {}, bar, pane);
  }

  // editor: read-only YAML view with line numbers, copy and download (the JWA YAML tab)
  function yamlView(obj, filename) {
    var text = L.yamlDump(obj);
    var lines = text.split("\n");
    var gutter = el("pre", { class: "gutter" }, lines.map(function (_, i) { return (i + 1) + "\n"; }).join(""));
    var code = el("pre", { class: "code" }, text);
    return el("div", { class: "editor" },
      el("div", { class: "toolbar" },
        el("button", { onclick: function () { navigator.clipboard.writeText(text).then(function () { snack("Copied"); }); } }, "Copy"),
        el("a", { href: URL.createObjectURL(new Blob([text], { type: "text/yaml" })), download: filename || "object.yaml" }, "Download")),
      el("div", { class: "editor-body" }, gutter, code));
  }

  function conditionsTable(conds) {
    return table([["Type", function (c) { return c.type; }, function (c) { return c.type; }],
                  ["Status", function (c) { return c.status; }], ["Reason", function (c) { return c.reason; }],
                  ["Message", function (c) { return c.message; }],
                  ["Last transition", function (c) { return c.lastTransitionTime; }, function (c) { return c.lastTransitionTime; }]],
                 L.conditionRows(conds), { empty: "No conditions." });
  }

  // logs viewer: polls fetchLines() every 3 s while attached, follow-tail, download
  function logsViewer(fetchLines, filename) {
    var pre = el("pre", { class: "logs" }), follow = el("input", { type: "checkbox", checked: true });
    var text = "";
    var box = el("div", { class: "logbox" },
      el("div", { class: "toolbar" }, el("label", {}, follow, " follow"),
        el("button", { onclick: function () {
          var a = el("a", { href: URL.createObjectURL(new Blob([text], { type: "text/plain" })), download: filename || "logs.txt" });
          a.click();
        } }, "Download")), pre);
    function refresh() {
      if (!document.body.contains(box) && text) return;        // detached: stop polling
      Promise.resolve().then(fetchLines).then(function (lines) {
        text = (lines || []).join("\n");
        pre.replaceChildren.apply(pre, (lines || []).map(function (l, i) {
          return el("div", { class: "logline" }, el("span", { class: "ln" }, i + 1), l);
        }));
        if (follow.checked) pre.scrollTop = pre.scrollHeight;
      }, function (e) { pre.replaceChildren(el("div", { class: "err" }, e.message)); })
        .then(function () { setTimeout(refresh, 3000); });
    }
    refresh();
    return box;
  }

  // details-list (kubeflow-common-lib details-list): rows of [key, value, help?]; an array
  // value renders as chips, an empty one as "-"
  function details(rows) {
    return el("dl", { class: "details" }, rows.map(function (r) {
      var v = r[1];
      if (Array.isArray(v) && !(v[0] instanceof Node)) {
        v = v.length ? v.map(function (x) { return el("span", { class: "chip" }, x); }) : "-";
      }
      return [el("dt", { "data-cy-details-key": r[0] }, r[0], r[2] ? helpPopover(r[2]) : null),
              el("dd", { "data-cy-details-value": r[0] }, v === "" || v === undefined || v === null ? "-" : v)];
    }));
  }

  function field(label, input, hint) {
    return [el("label", {}, label), el("div", {}, input, hint ? el("div", { class: "hint" }, hint) : null)];
  }

  var css = [
    "body{font-family:system-ui,sans-serif;margin:0;background:#fafafa;color:#222}",
    "header{background:#ed1c24;color:#fff;padding:10px 16px;display:flex;gap:12px;align-items:center}",
    "header h1{font-size:18px;margin:0;flex:1} header a{color:#fff} main{padding:16px}",
    "table.rt{border-collapse:collapse;width:100%;background:#fff} .rt th,.rt td{border-bottom:1px solid #ddd;padding:6px 8px;text-align:left;font-size:13px}",
    ".rt th.sortable{cursor:pointer;text-decoration:underline dotted} .rt tr.clickable:hover{background:#f3f6fb;cursor:pointer} td.empty{color:#777}",
    ".st-ready{color:#188038}.st-warning,.st-error{color:#c5221f} .muted{color:#777} .err{color:#c5221f} .hint{color:#777;font-size:12px}",
    ".snack{position:fixed;bottom:16px;left:16px;background:#323232;color:#fff;padding:10px 16px;border-radius:4px;z-index:9}",
    ".snack.err{background:#c5221f} form.card,div.card{background:#fff;padding:12px;margin:12px 0;display:grid;grid-template-columns:200px 1fr;gap:8px 12px;max-width:880px}",
    "fieldset{grid-column:1/3;border:1px solid #ddd} button{margin-right:4px}",
    ".tabs{display:flex;gap:4px;border-bottom:1px solid #ccc;margin:8px 0} .tabs button{border:0;background:none;padding:8px 12px;cursor:pointer}",
    ".tabs button.active{border-bottom:2px solid #ed1c24;font-weight:600} .tabpane{background:#fff;padding:12px}",
    "dl.details{display:grid;grid-template-columns:220px 1fr;gap:4px 12px} dt{color:#555}",
    ".editor{border:1px solid #ddd} .editor .toolbar,.logbox .toolbar{display:flex;gap:8px;padding:4px;background:#f3f3f3}",
    ".editor-body{display:flex;max-height:70vh;overflow:auto} .gutter{color:#999;text-align:right;padding:0 6px;margin:0;border-right:1px solid #eee}",
    ".code{margin:0;padding:0 8px} pre.logs{max-height:70vh;overflow:auto;background:#111;color:#ddd;margin:0;padding:8px;font-size:12px}",
    ".ln{color:#777;display:inline-block;width:4em} .group h4{margin:8px 0 4px}",
    "nav a{display:block;padding:8px 12px;color:#222;text-decoration:none} nav a:hover{background:#eee}",
    ".dash{display:grid;grid-template-columns:220px 1fr;height:calc(100vh - 44px)} iframe{border:0;width:100%;height:100%}",
    ".dialog-backdrop{position:fixed;inset:0;background:rgba(0,0,0,.35);display:flex;align-items:center;justify-content:center;z-index:10}",
    ".dialog{background:#fff;padding:16px 20px;min-width:320px;border-radius:4px} .dialog .actions{text-align:right}",
    ".dialog .accept{color:#c5221f} .help{border-radius:50%;border:1px solid #999;background:#fff;padding:0 6px;margin-left:4px}",
    ".popover{position:absolute;background:#333;color:#fff;padding:6px 8px;font-size:12px;max-width:320px} .chip{background:#eee;border-radius:10px;padding:1px 8px;margin-right:4px}",
    ".title-toolbar{display:flex;align-items:center;gap:8px} .title-toolbar .spacer{flex:1} .error-page{padding:32px;text-align:center}"
  ].join("\n");
  document.head.append(el("style", {}, css));

  root.KF = { el: el, api: api, snack: snack, status: status, table: table, poll: poll,
              namespaceSelect: namespaceSelect, ALL_NS: ALL_NS, tabs: tabs, yamlView: yamlView,
              conditionsTable: conditionsTable, logsViewer: logsViewer, details: details, field: field, base: base,
              confirmDialog: confirmDialog, helpPopover: helpPopover, dateTime: dateTime, titleToolbar: titleToolbar,
              variablesGroupsTable: variablesGroupsTable, snackErrorMessage: snackErrorMessage };
})(self);
