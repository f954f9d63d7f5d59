// kubeflow-common-lib logic for the kfamd web UI (T4-T7): the pure, DOM-free parts, shared by
// the browser apps (window.KFL) and unit-tested under node (module.exports; tests/test_ui.py).
//
// Reference behaviour:
//  * PollerService.exponential -- crud-web-apps/common/frontend/kubeflow-common-lib/projects/
//    kubeflow/src/lib/services/poller.service.ts:12-39 (1 s, doubling to an 8 s cap, reset to
//    1 s when the polled data changes);
//  * ExponentialBackoff -- .../lib/polling/exponential-backoff.ts:10-95 (1 s doubling to 16 s);
//  * the JWA form -> POST body -- jupyter/frontend/src/app/pages/form/form-new (fields of
//    jupyter/backend/apps/common/form.py), readOnly fields are never sent;
//  * the volume details "used by" groups -- volumes/frontend/src/app/pages/volume-details-page/
//    overview/overview.component.ts:60-128 (InferenceService pods labelled
//    serving.kubeflow.org/inferenceservice, Notebook pods labelled notebook-name);
//  * the details pages' YAML tab (a YAML rendering of the object) and conditions table.
(function (root, factory) {
  var lib = factory();
  if (typeof module === "object" && module.exports) module.exports = lib;
  else root.KFL = lib;
})(typeof self !== "undefined" ? self : this, function () {
  "use strict";

  // ------------------------------------------------------------------ polling
  var POLL_START = 1000, POLL_MAX = 8000;
  function nextPollDelay(prev, changed) {
    if (changed || !prev) return POLL_START;
    return Math.min(prev * 2, POLL_MAX);
  }

  function ExponentialBackoff(opts) {
    opts = opts || {};
    this.interval = opts.interval || 1000;
    this.maxInterval = opts.maxInterval || 16000;
    this.current = this.interval;
  }
  ExponentialBackoff.prototype.next = function () {
    var d = this.current;
    this.current = Math.min(this.current * 2, this.maxInterval);
    return d;
  };
  ExponentialBackoff.prototype.reset = function () { this.current = this.interval; };

  // ------------------------------------------------------------------ validators
  var DNS1123 = /^[a-z0-9]([-a-z0-9]*[a-z0-9])?$/;
  function dns1123Name(v) {
    if (!v) return "Name is required";
    if (v.length > 52) return "Name must be at most 52 characters";   // STS + pod suffixes fit in 63
    if (!DNS1123.test(v)) return "Name must consist of lower case alphanumeric characters or '-', and start and end with an alphanumeric character";
    return "";
  }
  var QTY = /^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$/;
  function quantity(v) {
    if (v === "" || v === undefined || v === null) return "";
    if (!QTY.test(String(v)) || isNaN(parseFloat(v))) return "Invalid quantity: " + v;
    return "";
  }
  function parseEnv(text) {
    var out = {}, lines = String(text || "").split("\n");
    for (var i = 0; i < lines.length; i++) {
      var l = lines[i].trim();
      if (!l || l.charAt(0) === "#") continue;
      var j = l.indexOf("=");
      if (j <= 0) throw new Error("Environment line " + (i + 1) + " is not KEY=VALUE: " + l);
      out[l.slice(0, j).trim()] = l.slice(j + 1);
    }
    return out;
  }

  // ------------------------------------------------------------------ JWA form
  function readOnly(config, field) {
    return !!(config && config[field] && config[field].readOnly);
  }
  function cfgValue(config, field, dflt) {
    return config && config[field] && config[field].value !== undefined ? config[field].value : dflt;
  }
  // form values (flat, as the form holds them) -> the JWA POST body (form.py field names)
  function jwaFormBody(v, config, namespace) {
    var body = { name: v.name, namespace: namespace };
    function put(field, value) { if (!readOnly(config, field)) body[field] = value; }
    if (v.customImageCheck) { if (!readOnly(config, "image")) body.customImage = v.customImage; }
    else put("image", v.image);
    put("imagePullPolicy", v.imagePullPolicy || cfgValue(config, "imagePullPolicy", "IfNotPresent"));
    put("serverType", v.serverType || "jupyter");
    put("cpu", String(v.cpu));
    put("cpuLimit", v.cpuLimit ? String(v.cpuLimit) : "");
    put("memory", String(v.memory));
    put("memoryLimit", v.memoryLimit ? String(v.memoryLimit) : "");
    put("gpus", !v.gpus || v.gpus === "none" ? { num: "none" } : { num: String(v.gpus), vendor: v.gpuVendor });
    put("tolerationGroup", v.tolerationGroup || "none");
    put("affinityConfig", v.affinityConfig || "none");
    put("configurations", v.configurations || []);
    put("shm", !!v.shm);
    if (v.environment && Object.keys(v.environment).length) put("environment", v.environment);
    if (!readOnly(config, "workspaceVolume")) {
      if (v.workspace && v.workspace.type === "new") {
        body.workspace = { mount: v.workspace.mount || "/home/jovyan", newPvc: {
          metadata: { name: v.workspace.name || (v.name + "-workspace") },
          spec: { accessModes: [v.workspace.mode || "ReadWriteOnce"],
                  resources: { requests: { storage: v.workspace.size || "5Gi" } },
                  storageClassName: v.workspace.storageClass || undefined } } };
      } else if (v.workspace && v.workspace.type === "existing") {
        body.workspace = { mount: v.workspace.mount || "/home/jovyan",
                           existingSource: { persistentVolumeClaim: { claimName: v.workspace.name } } };
      }
    }
    if (!readOnly(config, "dataVolumes")) {
      body.datavols = (v.datavols || []).map(function (d) {
        if (d.type === "existing") {
          return { mount: d.mount, existingSource: { persistentVolumeClaim: { claimName: d.name } } };
        }
        return { mount: d.mount, newPvc: { metadata: { name: d.name },
          spec: { accessModes: [d.mode || "ReadWriteOnce"], resources: { requests: { storage: d.size || "10Gi" } },
                  storageClassName: d.storageClass || undefined } } };
      });
    }
    return JSON.parse(JSON.stringify(body));   // drops undefined fields
  }
  function jwaFormErrors(v) {
    var errs = [];
    var e = dns1123Name(v.name); if (e) errs.push(e);
    ["cpu", "cpuLimit", "memory", "memoryLimit"].forEach(function (f) { var q = quantity(v[f]); if (q) errs.push(f + ": " + q); });
    if (v.cpuLimit && parseFloat(v.cpuLimit) < parseFloat(v.cpu)) errs.push("CPU limit must be greater than the request");
    if (v.memoryLimit && parseFloat(v.memoryLimit) < parseFloat(v.memory)) errs.push("Memory limit must be greater than the request");
    var mounts = {};
    (v.datavols || []).concat(v.workspace && v.workspace.type !== "none" ? [v.workspace] : []).forEach(function (d) {
      if (!d.mount) errs.push("every volume needs a mount path");
      else if (mounts[d.mount]) errs.push("mount path used twice: " + d.mount);
      mounts[d.mount] = 1;
      if (!d.name) errs.push("every volume needs a name");
    });
    return errs;
  }

  // ------------------------------------------------------------------ details pages
  function groupPodsByOwner(pods, viewerUrl) {
    var groups = [];
    (pods || []).forEach(function (pod) {
      var labels = (pod.metadata && pod.metadata.labels) || {}, ns = pod.metadata.namespace, item = null;
      var isvc = labels["serving.kubeflow.org/inferenceservice"] || labels["serving.kserve.io/inferenceservice"];
      if (isvc) {
        item = { group: "InferenceService", name: isvc + " (" + (labels.component || "predictor") + ")",
                 url: (viewerUrl || "") + "/models/details/" + ns + "/" + isvc + "/" };
      } else if (labels["notebook-name"]) {
        item = { group: "Notebooks", name: labels["notebook-name"],
                 url: (viewerUrl || "") + "/jupyter/notebook/details/" + ns + "/" + labels["notebook-name"] + "/" };
      }
      if (!item) return;
      var g = null;
      for (var i = 0; i < groups.length; i++) if (groups[i].name === item.group) g = groups[i];
      if (!g) { g = { name: item.group, links: [] }; groups.push(g); }
      if (!g.links.some(function (l) { return l.name === item.name; })) g.links.push({ name: item.name, url: item.url });
    });
    return groups;
  }

  function conditionRows(conds) {
    return (conds || []).map(function (c) {
      return { type: c.type || "", status: c.status || "", reason: c.reason || "", message: c.message || "",
               lastTransitionTime: c.lastTransitionTime || c.lastProbeTime || c.lastUpdateTime || "" };
    });
  }

  // Notebook -> the fields of the details page's overview tab
  function notebookOverview(nb) {
    var spec = (((nb || {}).spec || {}).template || {}).spec || {};
    var ctr = (spec.containers || [])[0] || {};
    var res = ctr.resources || {}, req = res.requests || {}, lim = res.limits || {};
    var gpus = Object.keys(lim).filter(function (k) { return /\/gpu$/.test(k); })
      .map(function (k) { return lim[k] + " x " + k; });
    var labels = (nb.metadata || {}).labels || {};
    var cfgs = Object.keys(labels).filter(function (k) { return labels[k] === "true"; });
    var mounts = {};
    (ctr.volumeMounts || []).forEach(function (m) { mounts[m.name] = m.mountPath; });
    var vols = (spec.volumes || []).map(function (v) {
      var src = v.persistentVolumeClaim ? "PVC " + v.persistentVolumeClaim.claimName
        : v.emptyDir ? "emptyDir" + (v.emptyDir.medium ? " (" + v.emptyDir.medium + ")" : "")
        : Object.keys(v).filter(function (k) { return k !== "name"; })[0] || "";
      return { name: v.name, source: src, mount: mounts[v.name] || "" };
    });
    var env = (ctr.env || []).map(function (e) { return e.name + "=" + (e.value !== undefined ? e.value : "(ref)"); });
    var ann = (nb.metadata || {}).annotations || {};
    return { image: ctr.image || "", serverType: ann["notebooks.kubeflow.org/server-type"] || "jupyter",
             creator: ann["notebooks.kubeflow.org/creator"] || "", cpu: req.cpu || "", cpuLimit: lim.cpu || "",
             memory: req.memory || "", memoryLimit: lim.memory || "", gpus: gpus, configurations: cfgs,
             volumes: vols, environment: env, tolerations: (spec.tolerations || []).length,
             affinity: !!spec.affinity };
  }

  // ------------------------------------------------------------------ YAML view
  function yamlScalar(v) {
    if (v === null || v === undefined) return "null";
    if (typeof v === "number" || typeof v === "boolean") return String(v);
    var s = String(v);
    if (s === "" || /^[\s]|[\s]$|^[-?:,\[\]{}#&*!|>'"%@`]|: |\s#|^(true|false|null|yes|no|on|off|~)$|^[+-]?[0-9.]+([eE][+-]?[0-9]+)?$|\n/i.test(s)) {
      return JSON.stringify(s);
    }
    return s;
  }
  function yamlDump(v, indent) {
    indent = indent || "";
    if (Array.isArray(v)) {
      if (!v.length) return "[]";
      return v.map(function (x) {
        if (x !== null && typeof x === "object" && !Array.isArray(x) && Object.keys(x).length) {
          var inner = yamlDump(x, indent + "  ");
          return indent + "- " + inner.slice(indent.length + 2);
        }
        return indent + "- " + (x !== null && typeof x === "object" ? yamlDump(x, indent + "  ").trim() : yamlScalar(x));
      }).join("\n");
    }
    if (v !== null && typeof v === "object") {
      var keys = Object.keys(v);
      if (!keys.length) return "{}";
      return keys.map(function (k) {
        var x = v[k], key = indent + yamlScalar(k) + ":";
        if (x !== null && typeof x === "object" && (Array.isArray(x) ? x.length : Object.keys(x).length)) {
          return key + "\n" + yamlDump(x, Array.isArray(x) ? indent : indent + "  ");
        }
        return key + " " + (x !== null && typeof x === "object" ? (Array.isArray(x) ? "[]" : "{}") : yamlScalar(x));
      }).join("\n");
    }
    return indent + yamlScalar(v);
  }

  // ------------------------------------------------------------------ misc
  function age(ts, now) {
    if (!ts) return "";
    var s = Math.max(0, Math.floor(((now || Date.now()) - Date.parse(ts)) / 1000));
    if (s < 60) return s + "s";
    if (s < 3600) return Math.floor(s / 60) + "m";
    if (s < 86400) return Math.floor(s / 3600) + "h";
    return Math.floor(s / 86400) + "d";
  }
  // "#/details/ns/name" -> {page: "details", args: ["ns", "name"]}
  function route(hash) {
    var parts = String(hash || "").replace(/^#\/?/, "").split("/").filter(Boolean).map(decodeURIComponent);
    return { page: parts[0] || "index", args: parts.slice(1) };
  }

  return { nextPollDelay: nextPollDelay, ExponentialBackoff: ExponentialBackoff, dns1123Name: dns1123Name,
           quantity: quantity, parseEnv: parseEnv, readOnly: readOnly, cfgValue: cfgValue, jwaFormBody: jwaFormBody,
           jwaFormErrors: jwaFormErrors, groupPodsByOwner: groupPodsByOwner, conditionRows: conditionRows,
           notebookOverview: notebookOverview, yamlDump: yamlDump, age: age, route: route,
           POLL_START: POLL_START, POLL_MAX: POLL_MAX };
});
