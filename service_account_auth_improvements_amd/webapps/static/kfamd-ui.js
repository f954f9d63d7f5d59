// kfamd web UI (T2-T7): the Notebooks, Volumes and TensorBoards web apps and the central
// dashboard, dependency-free, against the same REST APIs the reference Angular/Polymer
// frontends use (crud-web-apps/*/frontend, centraldashboard/public).  Shared components are
// lib/kf-common.js (DOM) and lib/kf-logic.js (pure logic, unit-tested under node).
//
// Routes (hash): #/ index, #/new create form, #/details/<ns>/<name> details page.
//  * Notebooks (jupyter/frontend/src/app/pages): index with status/GPUs/volumes, the full
//    new-notebook form (image or custom image, server type, CPU/memory + limits, GPUs with
//    vendor availability, workspace + data volumes (new or existing PVCs), affinity,
//    tolerations, PodDefault configurations, shm, environment; readOnly spawner fields are
//    shown disabled and never sent), and the details page with Overview / Logs / Events /
//    YAML tabs (pages/notebook-page/{overview,logs,events,yaml}).
//  * Volumes: index with viewer buttons, details page with the pods using the volume grouped
//    by owner kind (Notebooks, InferenceService: volume-details-page/overview), events, YAML.
//  * TensorBoards: index + form (logs path, PodDefault configurations).
(function () {
  "use strict";
  var KF = self.KF, L = self.KFL, el = KF.el, api = KF.api, snack = KF.snack;
  var root = document.getElementById("app");
  var APP = root ? root.dataset.app : "dashboard";
  var VIEWER_BASE = "";     // links into sibling apps (same origin behind the dashboard)

  function header(title, extra) {
    return el("header", {}, el("h1", {}, title), extra);
  }
  // delete through the common-lib confirm dialog (the reference's DELETE / CANCEL dialog)
  function confirmDelete(kind, name, doDelete) {
    return KF.confirmDialog({ title: "Delete " + kind + " " + name + "?",
                              message: "Warning: All data in this " + kind.toLowerCase() + " will be lost.",
                              accept: "DELETE", applying: "DELETING", onAccept: doDelete });
  }
  // (re-)render the page of the current hash; the hashchange listener is registered once per app
  function router(pages) {
    if (!pages._go) {
      pages._go = function () {
        var r = L.route(location.hash);
        (pages[r.page] || pages.index).apply(null, r.args);
      };
      window.addEventListener("hashchange", pages._go);
    }
    pages._go();
  }
  function back(label) { return el("a", { href: "#/" }, "← " + (label || "back")); }

  // ==================================================================== Notebooks (T4)
  function jupyter() {
    var ns = "", config = {}, poller = null, sel = null;
    var main = el("main"), headerExtra = el("span");
    root.append(header("Notebooks", headerExtra), main);
    api("GET", "api/config").then(function (j) { config = j.config || {}; }, function (e) { snack(e.message, true); })
      .then(function () { return KF.namespaceSelect(function (v) { ns = v; router(pages); }, { all: true }); })
      .then(function (s) { sel = s; ns = s.value; headerExtra.replaceChildren(sel); router(pages); });

    var pages = {
      index: function () {
        if (poller) poller.stop();
        var list = el("div");
        main.replaceChildren(KF.titleToolbar("Notebooks", el("a", { href: "#/new" }, el("button", {}, "+ New notebook"))), list);
        poller = KF.poll(function () {
          if (!ns) return [];
          var all = ns === KF.ALL_NS;
          // all namespaces: the union of every namespace's list (the reference frontend does
          // the same over its namespace list)
          var nsList = all ? (sel && sel.namespaces) || [] : [ns];
          return Promise.all(nsList.map(function (n) {
            return api("GET", "api/namespaces/" + n + "/notebooks", null, { quiet: all }).then(function (j) { return j.notebooks || []; },
                                                                                    function () { return []; });
          })).then(function (parts) {
            var nbs = [].concat.apply([], parts);
            list.replaceChildren(KF.table([
              ["Status", function (n) { return KF.status(n.status); }, function (n) { return n.status.phase; }],
              ["Name", function (n) { return el("a", { href: "#/details/" + n.namespace + "/" + n.name }, n.name); },
               function (n) { return n.name; }],
            ].concat(all ? [["Namespace", function (n) { return n.namespace; }, function (n) { return n.namespace; }]] : [], [
              ["Type", function (n) { return n.serverType || "jupyter"; }],
              ["Age", function (n) { return KF.dateTime(n.age); }, function (n) { return n.age; }],
              ["Image", function (n) { return n.shortImage; }],
              ["GPUs", function (n) { return (n.gpus && n.gpus.message) || "-"; }],
              ["CPU", function (n) { return n.cpu; }], ["Memory", function (n) { return n.memory; }],
              ["Volumes", function (n) { return (n.volumes || []).join(", "); }],
              ["", function (n) {
                return [el("a", { href: "/notebook/" + n.namespace + "/" + n.name + "/", target: "_blank" },
                           el("button", { disabled: n.status.phase !== "ready" }, "Connect")),
                        el("button", { onclick: function () { act("PATCH", n.name, { stopped: n.status.phase !== "stopped" }, n.namespace); } },
                           n.status.phase === "stopped" ? "Start" : "Stop"),
                        el("button", { "data-cy": "delete", onclick: function () {
                          confirmDelete("Notebook", n.name, function () { return act("DELETE", n.name, undefined, n.namespace); });
                        } }, "Delete")];
              }]]), nbs, { empty: "No notebooks in this namespace.", sortBy: "Name" }));
            return nbs;
          });
        });
      },
      new: function () { if (poller) poller.stop(); form(); },
      details: function (dns, name) { if (poller) poller.stop(); notebookDetails(dns || ns, name); }
    };

    function act(method, name, body, where) {
      return api(method, "api/namespaces/" + (where || ns) + "/notebooks/" + name, body)
        .then(function () { if (poller) poller.reset(); });
    }

    // ------------------------------------------------------------ new notebook form
    function form() {
      var ro = function (f) { return L.readOnly(config, f); };
      var v = function (f, d) { return L.cfgValue(config, f, d); };
      var vendorsInstalled = [], pvcs = [], poddefaults = [];
      var f = el("form", { class: "card", novalidate: true });
      main.replaceChildren(KF.titleToolbar("New notebook", null, "#/"), f);
      Promise.all([api("GET", "api/gpus").then(function (j) { vendorsInstalled = j.vendors || []; }, function () {}),
                   api("GET", "api/namespaces/" + ns + "/pvcs").then(function (j) { pvcs = j.pvcs || []; }, function () {}),
                   api("GET", "api/namespaces/" + ns + "/poddefaults").then(function (j) { poddefaults = j.poddefaults || []; }, function () {})])
        .then(render);

      function opt(value, text, selected) { return el("option", { value: value, selected: selected ? true : null }, text); }
      function render() {
        var imgCfg = config.image || {}, gpu = v("gpus", {}) || {};
        var name = el("input", { name: "name", required: true, placeholder: "my-notebook" });
        var serverType = el("select", { name: "serverType", disabled: ro("serverType") },
          opt("jupyter", "JupyterLab"), opt("group-one", "VS Code (code-server)"), opt("group-two", "RStudio"));
        var imageSel = el("select", { name: "image", disabled: ro("image") });
        function images() {
          var key = { "jupyter": "image", "group-one": "imageGroupOne", "group-two": "imageGroupTwo" }[serverType.value];
          var c = config[key] || imgCfg;
          imageSel.replaceChildren.apply(imageSel, (c.options || []).map(function (o) { return opt(o, o, o === c.value); }));
        }
        serverType.addEventListener("change", images);
        images();
        var custom = el("input", { type: "checkbox", name: "customImageCheck", disabled: ro("image") });
        var customImg = el("input", { name: "customImage", placeholder: "registry/image:tag", disabled: true });
        custom.addEventListener("change", function () { customImg.disabled = !custom.checked; imageSel.disabled = custom.checked || ro("image"); });
        var pull = el("select", { name: "imagePullPolicy", disabled: ro("imagePullPolicy") },
          ["IfNotPresent", "Always", "Never"].map(function (p) { return opt(p, p, p === v("imagePullPolicy", "IfNotPresent")); }));
        var cpu = el("input", { name: "cpu", value: v("cpu", "0.5"), disabled: ro("cpu") });
        var cpuLimit = el("input", { name: "cpuLimit", value: v("cpuLimit", ""), placeholder: "auto (limit factor)", disabled: ro("cpu") });
        var mem = el("input", { name: "memory", value: v("memory", "1.0Gi"), disabled: ro("memory") });
        var memLimit = el("input", { name: "memoryLimit", value: v("memoryLimit", ""), placeholder: "auto (limit factor)", disabled: ro("memory") });
        var gpuNum = el("select", { name: "gpus", disabled: ro("gpus") },
          ["none", "1", "2", "4", "8"].map(function (o) { return opt(o, o, o === String(gpu.num || "none")); }));
        var gpuVendor = el("select", { name: "gpuVendor", disabled: ro("gpus") }, (gpu.vendors || []).map(function (x) {
          var missing = vendorsInstalled.indexOf(x.limitsKey) < 0;
          return el("option", { value: x.limitsKey, title: missing ? "There are no " + x.uiName + " GPUs in the cluster" : null,
                                selected: x.limitsKey === gpu.vendor ? true : null }, x.uiName + (missing ? " (not installed)" : ""));
        }));
        // workspace volume
        var wsType = el("select", { disabled: ro("workspaceVolume") }, opt("new", "New volume"), opt("existing", "Existing volume"), opt("none", "None"));
        var wsTpl = ((((v("workspaceVolume", {}) || {}).newPvc || {}).metadata || {}).name) || "{notebook-name}-workspace";
        var wsDirty = false;
        var wsName = el("input", { "data-cy": "volume name input", value: wsTpl.replace("{notebook-name}", ""),
                                   oninput: function () { wsDirty = true; wsHeader.textContent = wsName.value; } });
        var wsHeader = el("span", { "data-cy": "volume name header" }, wsName.value);
        name.addEventListener("input", function () {
          if (!wsDirty) { wsName.value = wsTpl.replace("{notebook-name}", name.value); wsHeader.textContent = wsName.value; }
        });
        var wsSize = el("input", { value: "5Gi" });
        var wsMount = el("input", { value: "/home/jovyan" });
        var wsExisting = el("select", {}, pvcs.map(function (p) { return opt(p.name, p.name + " (" + p.size + ")"); }));
        var wsBox = el("div", { "data-cy": "workspace volume" });
        function wsRender() {
          wsBox.replaceChildren.apply(wsBox, wsType.value === "new" ? ["name ", wsName, " size ", wsSize, " mount ", wsMount]
            : wsType.value === "existing" ? ["claim ", wsExisting, " mount ", wsMount] : []);
        }
        wsType.addEventListener("change", wsRender);
        wsRender();
        // data volumes
        var dvList = el("div"), datavols = [];
        function dvRender() {
          dvList.replaceChildren.apply(dvList, datavols.map(function (d, i) {
            var t = el("select", { onchange: function (ev) { d.type = ev.target.value; dvRender(); } },
                       opt("new", "New", d.type === "new"), opt("existing", "Existing", d.type === "existing"));
            var mount = el("input", { value: d.mount, "data-cy": "mount path",
                                      oninput: function (ev) { d.mount = ev.target.value; d.mountDirty = true; } });
            // a new data volume mounts at /home/jovyan/<name> until its mount path is edited
            var follow = function (v) { d.name = v; if (!d.mountDirty) { d.mount = "/home/jovyan/" + v; mount.value = d.mount; } };
            var nm = d.type === "existing"
              ? el("select", { "data-cy": "volume name input", onchange: function (ev) { follow(ev.target.value); } },
                   pvcs.map(function (p) { return opt(p.name, p.name, p.name === d.name); }))
              : el("input", { value: d.name, placeholder: "volume name", "data-cy": "volume name input",
                              oninput: function (ev) { follow(ev.target.value); } });
            if (d.type === "existing" && !d.name && pvcs.length) follow(pvcs[0].name);
            return el("div", { class: "dv" + (i === datavols.length - 1 ? " last" : ""), "data-cy": "data volumes" }, t, " ", nm,
              d.type === "new" ? [" size ", el("input", { value: d.size, size: 6, oninput: function (ev) { d.size = ev.target.value; } })] : null,
              " mount ", mount,
              el("button", { type: "button", onclick: function () { datavols.splice(i, 1); dvRender(); } }, "✖"));
          }));
        }
        var addDv = el("button", { type: "button", "data-cy": "add new volume", disabled: ro("dataVolumes"), onclick: function () {
          datavols.push({ type: "new", name: "", size: "10Gi", mount: "/home/jovyan/data-" + (datavols.length + 1) }); dvRender();
        } }, "+ Add volume");
        // scheduling + configurations
        var aff = el("select", { name: "affinityConfig", disabled: ro("affinityConfig") }, opt("none", "None"),
          ((config.affinityConfig || {}).options || []).map(function (o) { return opt(o.configKey, o.displayName || o.configKey); }));
        var tol = el("select", { name: "tolerationGroup", disabled: ro("tolerationGroup") }, opt("none", "None"),
          ((config.tolerationGroup || {}).options || []).map(function (o) { return opt(o.groupKey, o.displayName || o.groupKey); }));
        var cfgBoxes = poddefaults.map(function (pd) {
          return el("label", { title: pd.desc }, el("input", { type: "checkbox", value: pd.label, disabled: ro("configurations"),
                                                                checked: (v("configurations", []) || []).indexOf(pd.label) >= 0 }), " ", pd.desc);
        });
        var shm = el("input", { type: "checkbox", name: "shm", checked: v("shm", true), disabled: ro("shm") });
        var env = el("textarea", { rows: 3, cols: 50, placeholder: "KEY=VALUE per line", disabled: ro("environment") });
        var errBox = el("div", { class: "err" });
        f.replaceChildren.apply(f, [].concat(
          KF.field("Name", name, "lower-case letters, digits and '-'"),
          KF.field("Server type", serverType),
          KF.field("Image", [imageSel, el("label", {}, " ", custom, " custom image "), customImg]),
          KF.field("Image pull policy", pull),
          KF.field("CPU request / limit", [cpu, " / ", cpuLimit]),
          KF.field("Memory request / limit", [mem, " / ", memLimit]),
          KF.field("GPUs", [gpuNum, " ", gpuVendor]),
          KF.field(["Workspace volume ", wsHeader], [wsType, " ", wsBox]),
          KF.field("Data volumes", [dvList, addDv]),
          KF.field("Affinity", aff), KF.field("Tolerations", tol),
          KF.field("Configurations", cfgBoxes.length ? cfgBoxes : el("span", { class: "muted" }, "no PodDefaults in this namespace")),
          KF.field(["Shared memory (/dev/shm)", KF.helpPopover("Mounts an in-memory /dev/shm: PyTorch DataLoader workers and RCCL use it.")], shm),
          KF.field("Environment", env),
          [el("span"), el("div", {}, errBox, el("button", { type: "submit" }, "Launch"), el("a", { href: "#/" }, el("button", { type: "button" }, "Cancel")))]));
        f.onsubmit = function (ev) {
          ev.preventDefault();
          var vals;
          try {
            vals = { name: name.value, serverType: serverType.value, image: imageSel.value, customImageCheck: custom.checked,
                     customImage: customImg.value, imagePullPolicy: pull.value, cpu: cpu.value, cpuLimit: cpuLimit.value,
                     memory: mem.value, memoryLimit: memLimit.value, gpus: gpuNum.value, gpuVendor: gpuVendor.value,
                     affinityConfig: aff.value, tolerationGroup: tol.value, shm: shm.checked,
                     configurations: cfgBoxes.map(function (l) { return l.querySelector("input"); })
                       .filter(function (i) { return i.checked; }).map(function (i) { return i.value; }),
                     environment: L.parseEnv(env.value),
                     workspace: { type: wsType.value, name: wsType.value === "existing" ? wsExisting.value : (wsName.value || name.value + "-workspace"),
                                  size: wsSize.value, mount: wsMount.value },
                     datavols: datavols };
          } catch (e) { errBox.textContent = e.message; return; }
          var errs = L.jwaFormErrors(vals);
          if (errs.length) { errBox.textContent = errs.join("; "); return; }
          api("POST", "api/namespaces/" + ns + "/notebooks", L.jwaFormBody(vals, config, ns))
            .then(function () { snack("Notebook " + vals.name + " created"); location.hash = "#/"; },
                  function (e) { errBox.textContent = e.message; });
        };
      }
    }

    // ------------------------------------------------------------ notebook details page
    function notebookDetails(dns, name) {
      var p = "api/namespaces/" + dns + "/notebooks/" + name;
      var title = el("h2", {}, name), st = el("span");
      main.replaceChildren(back("Notebooks"), el("div", {}, title, " ", st,
        el("a", { href: "/notebook/" + dns + "/" + name + "/", target: "_blank" }, el("button", {}, "Connect")),
        el("button", { "data-cy": "delete", onclick: function () {
          confirmDelete("Notebook", name, function () { return act("DELETE", name, undefined, dns); })
            .then(function (ok) { if (ok) location.hash = "#/"; });
        } }, "Delete")),
        KF.tabs([
          ["Overview", function () {
            return api("GET", p).then(function (j) {
              var nb = j.notebook, o = L.notebookOverview(nb);
              st.replaceChildren(KF.status(nb.processed_status));
              return el("div", {}, KF.details([
                ["Status", KF.status(nb.processed_status)], ["Server type", o.serverType], ["Image", o.image],
                ["Creator", o.creator], ["CPU (request / limit)", o.cpu + " / " + (o.cpuLimit || "-")],
                ["Memory (request / limit)", o.memory + " / " + (o.memoryLimit || "-")],
                ["GPUs", o.gpus.length ? o.gpus : ["none"], "amd.com/gpu devices allocated to the notebook's pod"],
                ["Configurations", o.configurations, "PodDefaults applied by label"],
                ["Tolerations / affinity", o.tolerations + " / " + (o.affinity ? "set" : "none")],
                ["Age", KF.dateTime(nb.metadata.creationTimestamp)]]),
                el("h4", {}, "Environment"),
                KF.variablesGroupsTable([{ name: "container", variables: o.environment.map(function (e) {
                  var i = e.indexOf("="); return [e.slice(0, i), e.slice(i + 1)]; }) }]),
                el("h4", {}, "Volumes"),
                KF.table([["Name", function (x) { return x.name; }], ["Source", function (x) { return x.source; }],
                          ["Mount path", function (x) { return x.mount; }]], o.volumes),
                el("h4", {}, "Conditions"), KF.conditionsTable((nb.status || {}).conditions));
            });
          }],
          ["Logs", function () {
            return api("GET", p + "/pod").then(function (j) {
              var pod = j.pod.metadata.name;
              return KF.logsViewer(function () {
                return api("GET", p + "/pod/" + pod + "/logs").then(function (r) { return r.logs; });
              }, name + ".log");
            }, function () { return el("div", { class: "muted" }, "No pod for this notebook (stopped or starting)."); });
          }],
          ["Events", function () {
            return api("GET", p + "/events").then(function (j) {
              return KF.table([["Type", function (e) { return e.type; }, function (e) { return e.type; }],
                               ["Reason", function (e) { return e.reason; }], ["Message", function (e) { return e.message; }],
                               ["Object", function (e) { return (e.involvedObject || {}).kind + "/" + (e.involvedObject || {}).name; }],
                               ["Last seen", function (e) { return e.lastTimestamp || e.eventTime || ""; },
                                function (e) { return e.lastTimestamp || ""; }]], j.events, { empty: "No events." });
            });
          }],
          ["YAML", function () {
            return api("GET", p).then(function (j) {
              var nb = j.notebook; delete nb.processed_status;
              return KF.yamlView(nb, name + ".yaml");
            });
          }]]));
    }
  }

  // ==================================================================== Volumes (T5)
  function volumes() {
    var ns = "", poller = null;
    var main = el("main"), headerExtra = el("span");
    root.append(header("Volumes", headerExtra), main);
    KF.namespaceSelect(function (v) { ns = v; router(pages); }).then(function (s) { ns = s.value; headerExtra.replaceChildren(s); router(pages); });
    var pages = {
      index: function () {
        if (poller) poller.stop();
        var list = el("div"), names = [];
        var name = el("input", { placeholder: "name" }), size = el("input", { value: "10Gi", size: 6 });
        var mode = el("select", {}, ["ReadWriteOnce", "ReadOnlyMany", "ReadWriteMany"].map(function (m) { return el("option", { value: m }, m); }));
        // storage class (form-default: "None" = {none}, the cluster's classes, the default one
        // preselected; until the backend answers, {empty} leaves the class to the cluster default)
        var sclass = el("select", { "data-cy": "storage class" }, el("option", { value: "{empty}" }, "(cluster default)"),
                        el("option", { value: "{none}" }, "None"));
        api("GET", "api/storageclasses").then(function (j) {
          (j.storageClasses || []).forEach(function (c) { sclass.append(el("option", { value: c }, c)); });
          return api("GET", "api/storageclasses/default");
        }).then(function (j) { if (j && j.defaultStorageClass) sclass.value = j.defaultStorageClass; }, function () {});
        var create = el("button", { onclick: function () {
          var err = L.dns1123Name(name.value) || L.quantity(size.value) ||
                    (names.indexOf(name.value) >= 0 ? "Volume " + name.value + " already exists" : "");
          if (err) { snack(err, true); return; }
          api("POST", "api/namespaces/" + ns + "/pvcs", { name: name.value, mode: mode.value, class: sclass.value,
                                                          size: size.value, type: "new" })
            .then(function () { poller.reset(); }, function (e) { snack(e.message, true); });
        } }, "+ New volume");
        main.replaceChildren(el("div", { class: "card" }, el("label", {}, "New volume"),
                                el("div", {}, name, " ", size, " ", mode, " ", sclass, " ", create)), list);
        poller = KF.poll(function () {
          if (!ns) return [];
          return api("GET", "api/namespaces/" + ns + "/pvcs").then(function (j) {
            var pvcs = j.pvcs;
            names = pvcs.map(function (p) { return p.name; });
            list.replaceChildren(KF.table([
              ["Status", function (p) { return KF.status(p.status); }],
              ["Name", function (p) { return el("a", { href: "#/details/" + p.namespace + "/" + p.name }, p.name); }, function (p) { return p.name; }],
              ["Age", function (p) { return L.age(p.age); }, function (p) { return p.age; }],
              ["Size", function (p) { return p.capacity; }], ["Access", function (p) { return (p.modes || []).join(","); }],
              ["Class", function (p) { return p.class || "-"; }],
              ["Used by", function (p) { return (p.notebooks || []).join(", ") || "-"; }],
              ["", function (p) {
                return [p.viewer.status === "ready" && p.viewer.url ? el("a", { href: p.viewer.url, target: "_blank" }, el("button", {}, "Browse"))
                  : el("button", { onclick: function () { api("POST", "api/namespaces/" + ns + "/viewers", { name: p.name })
                      .then(function () { poller.reset(); }, function (e) { snack(e.message, true); }); } }, "Open viewer"),
                  el("button", { "data-cy": "delete", onclick: function () {
                    confirmDelete("Volume", p.name, function () {
                      return api("DELETE", "api/namespaces/" + ns + "/pvcs/" + p.name).then(function () { poller.reset(); });
                    }); } }, "Delete")];
              }]], pvcs, { empty: "No volumes in this namespace.", sortBy: "Name" }));
            return pvcs;
          });
        });
      },
      details: function (dns, name) {
        if (poller) poller.stop();
        var p = "api/namespaces/" + dns + "/pvcs/" + name;
        main.replaceChildren(back("Volumes"), el("h2", {}, name), KF.tabs([
          ["Overview", function () {
            return Promise.all([api("GET", p), api("GET", p + "/pods")]).then(function (r) {
              var pvc = r[0].pvc, pods = r[1].pods, s = pvc.spec || {}, stt = pvc.status || {};
              var groups = L.groupPodsByOwner(pods, VIEWER_BASE);
              return el("div", {}, KF.details([
                ["Status", stt.phase], ["Size", ((stt.capacity || {}).storage) || ((s.resources || {}).requests || {}).storage],
                ["Access modes", (stt.accessModes || s.accessModes || []).join(", ")],
                ["Storage class", s.storageClassName], ["Volume", s.volumeName],
                ["Age", L.age(pvc.metadata.creationTimestamp)]]),
                el("h4", {}, "Used by"),
                groups.length ? groups.map(function (g) {
                  return el("div", { class: "group" }, el("h4", {}, g.name),
                            el("ul", {}, g.links.map(function (l) { return el("li", {}, el("a", { href: l.url, target: "_top" }, l.name)); })));
                }) : el("div", { class: "muted" }, "No Notebook or InferenceService pods use this volume."),
                el("h4", {}, "Conditions"), KF.conditionsTable(stt.conditions));
            });
          }],
          ["Events", function () {
            return api("GET", p + "/events").then(function (j) {
              return KF.table([["Type", function (e) { return e.type; }], ["Reason", function (e) { return e.reason; }],
                               ["Message", function (e) { return e.message; }],
                               ["Last seen", function (e) { return e.lastTimestamp || ""; }]], j.events, { empty: "No events." });
            });
          }],
          ["YAML", function () { return api("GET", p).then(function (j) { return KF.yamlView(j.pvc, name + ".yaml"); }); }]]));
      }
    };
  }

  // ==================================================================== TensorBoards (T6)
  function tensorboards() {
    var ns = "", poller = null;
    var main = el("main"), headerExtra = el("span");
    root.append(header("TensorBoards", headerExtra), main);
    KF.namespaceSelect(function (v) { ns = v; render(); }).then(function (s) { ns = s.value; headerExtra.replaceChildren(s); render(); });
    function render() {
      if (poller) poller.stop();
      var list = el("div");
      var name = el("input", { placeholder: "name" });
      var kind = el("select", {}, el("option", { value: "pvc" }, "PVC"), el("option", { value: "cloud" }, "Object store (gs:// s3://)"));
      var claim = el("select"), sub = el("input", { placeholder: "sub/path" }), uri = el("input", { placeholder: "gs://bucket/logs" });
      var cfgs = el("span");
      Promise.all([api("GET", "api/namespaces/" + ns + "/pvcs").then(function (j) {
        claim.replaceChildren.apply(claim, (j.pvcs || []).map(function (p) { return el("option", { value: p.name || p }, p.name || p); }));
      }, function () {}), api("GET", "api/namespaces/" + ns + "/poddefaults").then(function (j) {
        cfgs.replaceChildren.apply(cfgs, (j.poddefaults || []).map(function (pd) {
          return el("label", { title: pd.desc }, el("input", { type: "checkbox", value: pd.label }), " ", pd.desc, " ");
        }));
      }, function () {})]);
      var create = el("button", { onclick: function () {
        var err = L.dns1123Name(name.value);
        if (err) { snack(err, true); return; }
        var logspath = kind.value === "pvc" ? "pvc://" + claim.value + "/" + sub.value.replace(/^\//, "") : uri.value;
        var configurations = Array.prototype.map.call(cfgs.querySelectorAll("input:checked"), function (i) { return i.value; });
        api("POST", "api/namespaces/" + ns + "/tensorboards", { name: name.value, logspath: logspath, configurations: configurations })
          .then(function () { poller.reset(); }, function (e) { snack(e.message, true); });
      } }, "+ New TensorBoard");
      main.replaceChildren(el("div", { class: "card" }, KF.field("Name", name), KF.field("Logs", [kind, " ", claim, " ", sub, " ", uri]),
                              KF.field("Configurations", cfgs), el("span"), create), list);
      poller = KF.poll(function () {
        if (!ns) return [];
        return api("GET", "api/namespaces/" + ns + "/tensorboards").then(function (j) {
          var tbs = j.tensorboards;
          list.replaceChildren(KF.table([
            ["Status", function (t) { return KF.status(t.status); }],
            ["Name", function (t) { return el("a", { href: "/tensorboard/" + t.namespace + "/" + t.name + "/", target: "_blank" }, t.name); }, function (t) { return t.name; }],
            ["Logs", function (t) { return t.logspath; }], ["Age", function (t) { return L.age(t.age); }],
            ["", function (t) { return el("button", { "data-cy": "delete", onclick: function () {
              confirmDelete("TensorBoard", t.name, function () {
                return api("DELETE", "api/namespaces/" + ns + "/tensorboards/" + t.name).then(function () { poller.reset(); });
              }); } }, "Delete"); }]],
            tbs, { empty: "No TensorBoards in this namespace.", sortBy: "Name" }));
          return tbs;
        });
      });
    }
  }

  // ==================================================================== Central dashboard (T2)
  // centraldashboard.js (the Polymer main-page / registration / dashboard-view / manage-users
  // components); failed calls of its shell go through the error interceptor (KF.api snack)
  function dashboard() {
    self.CD.start(root).catch(function () {});
  }

  var apps = { jupyter: jupyter, volumes: volumes, tensorboards: tensorboards, dashboard: dashboard };
  try { (apps[APP] || dashboard)(); } catch (e) { snack(e.message, true); }
})();
