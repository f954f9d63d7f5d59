// kfamd web UI (T2-T7): one dependency-free script that renders the Notebooks, Volumes and
// TensorBoards web apps and the central dashboard against the same REST APIs the reference
// Angular/Polymer frontends use (crud-web-apps/*/frontend, centraldashboard/public).
//
// Shared pieces (kubeflow-common-lib equivalents): namespace selector, resource table with
// status icons, exponential-backoff poller (1 s doubling to 8 s, reset on change), snack
// bar errors, CSRF double-submit header (X-XSRF-TOKEN from the XSRF-TOKEN cookie).
(function () {
  "use strict";
  const root = document.getElementById("app");
  const APP = root ? root.dataset.app : "dashboard";
  const base = (document.querySelector("base") || {}).href || "/";

  // ------------------------------------------------------------------ helpers
  function el(tag, attrs, ...kids) {
    const e = document.createElement(tag);
    for (const [k, v] of Object.entries(attrs || {})) {
      if (k.startsWith("on")) e.addEventListener(k.slice(2), v);
      else if (k === "class") e.className = v;
      else e.setAttribute(k, v);
    }
    for (const k of kids.flat()) e.append(k instanceof Node ? k : document.createTextNode(String(k == null ? "" : k)));
    return e;
  }
  function cookie(name) {
    const m = document.cookie.match(new RegExp("(?:^|; )" + name + "=([^;]*)"));
    return m ? decodeURIComponent(m[1]) : "";
  }
  async function api(method, path, body) {
    const headers = { "Content-Type": "application/json" };
    if (!["GET", "HEAD"].includes(method)) headers["X-XSRF-TOKEN"] = cookie("XSRF-TOKEN");
    const r = await fetch(new URL(path, base), { method, headers, body: body ? JSON.stringify(body) : undefined,
                                                  credentials: "same-origin" });
    const j = await r.json().catch(() => ({}));
    if (!r.ok || j.success === false) throw new Error(j.log || j.error || r.statusText);
    return j;
  }
  function snack(msg, err) {
    const s = el("div", { class: "snack" + (err ? " err" : "") }, msg);
    document.body.append(s);
    setTimeout(() => s.remove(), 5000);
  }
  const ICON = { ready: "✔", waiting: "⏳", warning: "⚠", error: "✖", stopped: "⏹",
                 terminating: "✖", unavailable: "⚠", uninitialized: "•" };
  function status(st) {
    st = st || {};
    return el("span", { class: "st st-" + (st.phase || ""), title: st.message || "" }, ICON[st.phase] || "?", " ",
              st.phase || "");
  }
  function table(cols, rows) {
    return el("table", { class: "rt" }, el("thead", {}, el("tr", {}, cols.map((c) => el("th", {}, c[0])))),
              el("tbody", {}, rows.map((r) => el("tr", {}, cols.map((c) => el("td", {}, c[1](r)))))));
  }
  // exponential poller (common-lib PollerService.exponential)
  function poll(fn) {
    let delay = 1000, last = "", timer = null, stopped = false;
    async function tick() {
      try {
        const sig = JSON.stringify(await fn());
        delay = sig !== last ? 1000 : Math.min(delay * 2, 8000);
        last = sig;
      } catch (e) { snack(e.message, true); delay = Math.min(delay * 2, 8000); }
      if (!stopped) timer = setTimeout(tick, delay);
    }
    tick();
    return { reset() { delay = 1000; clearTimeout(timer); tick(); }, stop() { stopped = true; clearTimeout(timer); } };
  }
  async function namespaceSelect(onChange) {
    const sel = el("select", { id: "ns" });
    const qs = new URLSearchParams(location.search).get("ns");
    let nss = [];
    try { nss = (await api("GET", "api/namespaces")).namespaces || []; } catch (e) { snack(e.message, true); }
    for (const n of nss) sel.append(el("option", { value: n }, n));
    if (qs) sel.value = qs;
    sel.addEventListener("change", () => onChange(sel.value));
    window.addEventListener("message", (ev) => {            // dashboard iframe protocol
      if (ev.data && ev.data.type === "namespace-selected") { sel.value = ev.data.value; onChange(sel.value); }
    });
    return sel;
  }
  const style = el("style", {}, `
    body{font-family:system-ui,sans-serif;margin:0;background:#fafafa;color:#222}
    header{background:#ed1c24;color:#fff;padding:10px 16px;display:flex;gap:16px;align-items:center}
    header h1{font-size:18px;margin:0;flex:1} main{padding:16px}
    table.rt{border-collapse:collapse;width:100%;background:#fff} .rt th,.rt td{border-bottom:1px solid #ddd;
    padding:6px 8px;text-align:left;font-size:13px} .st-ready{color:#188038}.st-warning,.st-error{color:#c5221f}
    .snack{position:fixed;bottom:16px;left:16px;background:#323232;color:#fff;padding:10px 16px;border-radius:4px}
    .snack.err{background:#c5221f} form.card{background:#fff;padding:12px;margin:12px 0;display:grid;
    grid-template-columns:160px 1fr;gap:6px 12px;max-width:720px} button{margin-right:4px}
    nav a{display:block;padding:8px 12px;color:#222;text-decoration:none} nav a:hover{background:#eee}
    .dash{display:grid;grid-template-columns:220px 1fr;height:calc(100vh - 44px)} iframe{border:0;width:100%;height:100%}`);
  document.head.append(style);

  // ------------------------------------------------------------------ Jupyter (T4)
  async function jupyter() {
    let ns = "", config = {};
    const list = el("div"), form = el("div");
    const sel = await namespaceSelect((v) => { ns = v; poller.reset(); });
    ns = sel.value;
    root.append(el("header", {}, el("h1", {}, "Notebooks"), sel,
                   el("button", { onclick: () => showForm() }, "+ New notebook")), el("main", {}, form, list));
    try { config = (await api("GET", "api/config")).config; } catch (e) { snack(e.message, true); }
    async function refresh() {
      if (!ns) return [];
      const nbs = (await api("GET", `api/namespaces/${ns}/notebooks`)).notebooks;
      list.replaceChildren(table([
        ["Status", (n) => status(n.status)], ["Name", (n) => el("a", { href: `/notebook/${n.namespace}/${n.name}/`,
                                                                       target: "_blank" }, n.name)],
        ["Type", (n) => n.serverType || "jupyter"], ["Age", (n) => n.age], ["Image", (n) => n.shortImage],
        ["GPUs", (n) => n.gpus.message || "-"], ["CPU", (n) => n.cpu], ["Memory", (n) => n.memory],
        ["", (n) => [
          el("button", { onclick: () => act("PATCH", n, { stopped: n.status.phase !== "stopped" }) },
             n.status.phase === "stopped" ? "Start" : "Stop"),
          el("button", { onclick: () => confirm(`Delete ${n.name}?`) && act("DELETE", n) }, "Delete")]],
      ], nbs));
      return nbs;
    }
    async function act(method, n, body) {
      try { await api(method, `api/namespaces/${ns}/notebooks/${n.name}`, body); poller.reset(); }
      catch (e) { snack(e.message, true); }
    }
    async function showForm() {
      let vendors = [];
      try { vendors = (await api("GET", "api/gpus")).vendors; } catch (e) { /* optional */ }
      const g = config.gpus || { value: {} };
      const f = el("form", { class: "card" },
        el("label", {}, "Name"), el("input", { name: "name", required: "" }),
        el("label", {}, "Image"), el("select", { name: "image" },
          ((config.image || {}).options || []).map((o) => el("option", { value: o }, o))),
        el("label", {}, "CPU"), el("input", { name: "cpu", value: (config.cpu || {}).value || "0.5" }),
        el("label", {}, "Memory"), el("input", { name: "memory", value: (config.memory || {}).value || "1.0Gi" }),
        el("label", {}, "GPUs"), el("select", { name: "gpus" },
          ["none", "1", "2", "4", "8"].map((o) => el("option", { value: o }, o))),
        el("label", {}, "GPU vendor"), el("select", { name: "vendor" },
          (g.value.vendors || []).map((v) => el("option", { value: v.limitsKey },
            v.uiName + (vendors.includes(v.limitsKey) ? "" : " (not installed)")))),
        el("label", {}, "Workspace size"), el("input", { name: "ws", value: "5Gi" }),
        el("span"), el("div", {}, el("button", { type: "submit" }, "Launch"),
                        el("button", { type: "button", onclick: () => form.replaceChildren() }, "Cancel")));
      f.addEventListener("submit", async (ev) => {
        ev.preventDefault();
        const d = Object.fromEntries(new FormData(f));
        const body = { name: d.name, namespace: ns, image: d.image, imagePullPolicy: "IfNotPresent",
                       serverType: "jupyter", cpu: d.cpu, cpuLimit: "", memory: d.memory, memoryLimit: "",
                       gpus: { num: d.gpus, vendor: d.vendor }, tolerationGroup: "none", affinityConfig: "none",
                       configurations: [], shm: true, datavols: [],
                       workspace: { mount: "/home/jovyan", newPvc: { metadata: { name: `${d.name}-workspace` },
                         spec: { accessModes: ["ReadWriteOnce"], resources: { requests: { storage: d.ws } } } } } };
        try { await api("POST", `api/namespaces/${ns}/notebooks`, body); form.replaceChildren(); poller.reset(); }
        catch (e) { snack(e.message, true); }
      });
      form.replaceChildren(f);
    }
    const poller = poll(refresh);
  }

  // ------------------------------------------------------------------ Volumes (T5)
  async function volumes() {
    let ns = "";
    const list = el("div");
    const sel = await namespaceSelect((v) => { ns = v; poller.reset(); });
    ns = sel.value;
    const name = el("input", { placeholder: "name" }), size = el("input", { value: "10Gi" });
    const create = el("button", { onclick: async () => {
      try {
        await api("POST", `api/namespaces/${ns}/pvcs`, { name: name.value, mode: "ReadWriteOnce", class: "{empty}",
                                                        size: size.value, type: "new" });
        poller.reset();
      } catch (e) { snack(e.message, true); }
    } }, "+ New volume");
    root.append(el("header", {}, el("h1", {}, "Volumes"), sel, name, size, create), el("main", {}, list));
    async function refresh() {
      if (!ns) return [];
      const pvcs = (await api("GET", `api/namespaces/${ns}/pvcs`)).pvcs;
      list.replaceChildren(table([
        ["Status", (p) => status(p.status)], ["Name", (p) => p.name], ["Size", (p) => p.capacity],
        ["Access", (p) => (p.modes || []).join(",")], ["Class", (p) => p.class || "-"],
        ["Used by", (p) => (p.notebooks || []).join(", ") || "-"],
        ["", (p) => [
          p.viewer.status === "ready" && p.viewer.url ? el("a", { href: p.viewer.url, target: "_blank" }, "Browse")
            : el("button", { onclick: () => api("POST", `api/namespaces/${ns}/viewers`, { name: p.name })
                .then(() => poller.reset(), (e) => snack(e.message, true)) }, "Open viewer"),
          el("button", { onclick: () => confirm(`Delete ${p.name}?`) &&
            api("DELETE", `api/namespaces/${ns}/pvcs/${p.name}`).then(() => poller.reset(),
                                                                     (e) => snack(e.message, true)) }, "Delete")]],
      ], pvcs));
      return pvcs;
    }
    const poller = poll(refresh);
  }

  // ------------------------------------------------------------------ TensorBoards (T6)
  async function tensorboards() {
    let ns = "";
    const list = el("div");
    const sel = await namespaceSelect((v) => { ns = v; poller.reset(); });
    ns = sel.value;
    const name = el("input", { placeholder: "name" }), logs = el("input", { placeholder: "pvc://claim/path" });
    const create = el("button", { onclick: () => api("POST", `api/namespaces/${ns}/tensorboards`,
        { name: name.value, logspath: logs.value, configurations: [] }).then(() => poller.reset(),
                                                                           (e) => snack(e.message, true)) },
      "+ New TensorBoard");
    root.append(el("header", {}, el("h1", {}, "TensorBoards"), sel, name, logs, create), el("main", {}, list));
    async function refresh() {
      if (!ns) return [];
      const tbs = (await api("GET", `api/namespaces/${ns}/tensorboards`)).tensorboards;
      list.replaceChildren(table([
        ["Status", (t) => status(t.status)],
        ["Name", (t) => el("a", { href: `/tensorboard/${t.namespace}/${t.name}/`, target: "_blank" }, t.name)],
        ["Logs", (t) => t.logspath], ["Age", (t) => t.age],
        ["", (t) => el("button", { onclick: () => confirm(`Delete ${t.name}?`) &&
          api("DELETE", `api/namespaces/${ns}/tensorboards/${t.name}`).then(() => poller.reset(),
                                                                           (e) => snack(e.message, true)) },
          "Delete")]], tbs));
      return tbs;
    }
    const poller = poll(refresh);
  }

  // ------------------------------------------------------------------ Central dashboard (T2/T3)
  async function dashboard() {
    const j = (p) => fetch(new URL(p, base)).then((r) => r.json());
    const env = await j("api/workgroup/env-info");
    const exists = await j("api/workgroup/exists");
    const links = await j("api/dashboard-links").catch(() => ({ menuLinks: [] }));
    const nsSel = el("select", {}, (env.namespaces || []).map((b) =>
      el("option", { value: b.namespace }, `${b.namespace} (${b.role})`)));
    const frame = el("iframe", { name: "content" });
    const post = () => frame.contentWindow &&
      frame.contentWindow.postMessage({ type: "namespace-selected", value: nsSel.value }, "*");
    nsSel.addEventListener("change", post);
    frame.addEventListener("load", post);
    const nav = el("nav", {}, (links.menuLinks || []).map((l) =>
      el("a", { href: "#", onclick: (ev) => { ev.preventDefault(); frame.src = `${l.link}?ns=${nsSel.value}`; } },
         l.text)),
      el("a", { href: "#", onclick: (ev) => { ev.preventDefault(); manage(); } }, "Manage contributors"));
    const main = el("div", {}, frame);
    root.append(el("header", {}, el("h1", {}, "Kubeflow on MI355X"), nsSel, el("span", {}, env.user || "")),
                el("div", { class: "dash" }, nav, main));
    if (!exists.hasWorkgroup && exists.registrationFlowAllowed && exists.hasAuth) {
      const inp = el("input", { value: exists.user });
      main.replaceChildren(el("div", { class: "card" }, el("h2", {}, "Create your namespace"), inp,
        el("button", { onclick: () => fetch(new URL("api/workgroup/create", base), {
          method: "POST", headers: { "Content-Type": "application/json" },
          body: JSON.stringify({ namespace: inp.value }) }).then(() => location.reload()) }, "Finish")));
      return;
    }
    async function manage() {
      const ns = nsSel.value;
      const users = await j(`api/workgroup/get-contributors/${ns}`).catch(() => []);
      const who = el("input", { placeholder: "user@example.com" });
      const call = (m) => fetch(new URL(`api/workgroup/${m === "POST" ? "add" : "remove"}-contributor/${ns}`, base),
        { method: m, headers: { "Content-Type": "application/json" }, body: JSON.stringify({ contributor: who.value }) })
        .then(async (r) => { if (!r.ok) snack((await r.json()).error, true); manage(); });
      main.replaceChildren(el("div", { class: "card" }, el("h2", {}, `Contributors of ${ns}`),
        el("ul", {}, users.map((u) => el("li", {}, u))), who,
        el("button", { onclick: () => call("POST") }, "Add"), el("button", { onclick: () => call("DELETE") }, "Remove")));
    }
  }

  ({ jupyter, volumes, tensorboards, dashboard }[APP] || dashboard)().catch((e) => snack(e.message, true));
})();
