// A small DOM for running the web UI's page code under node (no packages): elements with
// attributes, classes, children, text, form values and events; a selector engine for the
// compound selectors the tests use (tag, #id, .class, [attr], [attr="v"], :checked, and the
// descendant combinator); document / window / location (hash routing + hashchange) / cookies /
// sessionStorage; fetch answered from fixture routes, every request recorded; timers recorded,
// not run (pollers stay at their first tick unless a test runs them).
"use strict";

class Node_ {
  constructor() { this.parentNode = null; this.childNodes = []; }
  get children() { return this.childNodes.filter(function (c) { return c instanceof Element_; }); }
  get firstChild() { return this.childNodes[0] || null; }
  _adopt(c) {
    if (typeof c === "string" || typeof c === "number") c = new Text_(String(c));
    if (c.parentNode) c.parentNode._remove(c);
    c.parentNode = this;
    return c;
  }
  _remove(c) { var i = this.childNodes.indexOf(c); if (i >= 0) this.childNodes.splice(i, 1); c.parentNode = null; }
  append() { for (var i = 0; i < arguments.length; i++) this.childNodes.push(this._adopt(arguments[i])); }
  appendChild(c) { this.append(c); return c; }
  replaceChildren() {
    this.childNodes.slice().forEach(function (c) { c.parentNode = null; });
    this.childNodes = [];
    this.append.apply(this, arguments);
  }
  remove() { if (this.parentNode) this.parentNode._remove(this); }
  contains(n) { for (; n; n = n.parentNode) if (n === this) return true; return false; }
  get textContent() { return this.childNodes.map(function (c) { return c.textContent; }).join(""); }
  set textContent(v) { this.replaceChildren(); if (v !== "" && v !== null && v !== undefined) this.append(String(v)); }
}

class Text_ extends Node_ {
  constructor(t) { super(); this.data = t; }
  get textContent() { return this.data; }
  set textContent(v) { this.data = String(v); }
}

var BOOL_ATTRS = ["disabled", "checked", "selected", "required", "novalidate"];

class Element_ extends Node_ {
  constructor(tag) {
    super();
    this.tagName = tag.toUpperCase();
    this.attributes = {};
    this.listeners = {};
    this.style = {};
    this._value = undefined;
    this.checked = false;
    this.disabled = false;
    this.scrollTop = 0;
    this.scrollHeight = 0;
  }
  setAttribute(k, v) {
    v = String(v);
    if (k === "checked") { this.checked = true; return; }
    if (k === "disabled") { this.disabled = true; return; }
    if (k === "selected") { this.selected = true; return; }
    this.attributes[k] = v;
  }
  getAttribute(k) {
    if (BOOL_ATTRS.indexOf(k) >= 0 && this[k]) return "";
    return Object.prototype.hasOwnProperty.call(this.attributes, k) ? this.attributes[k] : null;
  }
  hasAttribute(k) { return this.getAttribute(k) !== null; }
  removeAttribute(k) { delete this.attributes[k]; if (BOOL_ATTRS.indexOf(k) >= 0) this[k] = false; }
  get id() { return this.attributes.id || ""; }
  get className() { return this.attributes["class"] || ""; }
  set className(v) { this.attributes["class"] = v; }
  get classList() {
    var self = this;
    return { contains: function (c) { return self.className.split(/\s+/).indexOf(c) >= 0; },
             add: function (c) { if (!this.contains(c)) self.className = (self.className + " " + c).trim(); },
             remove: function (c) { self.className = self.className.split(/\s+/).filter(function (x) { return x !== c; }).join(" "); } };
  }
  get dataset() {
    var out = {};
    var a = this.attributes;
    Object.keys(a).forEach(function (k) {
      if (k.indexOf("data-") === 0) out[k.slice(5).replace(/-([a-z])/g, function (_, c) { return c.toUpperCase(); })] = a[k];
    });
    return out;
  }
  get href() { return this.attributes.href || ""; }
  set href(v) { this.attributes.href = v; }
  get src() { return this.attributes.src || ""; }
  set src(v) { this.attributes.src = v; }
  get type() { return this.attributes.type || (this.tagName === "BUTTON" ? "submit" : "text"); }
  get name() { return this.attributes.name || ""; }
  get options() { return this.querySelectorAll("option"); }
  get value() {
    if (this.tagName === "SELECT") {
      var opts = this.querySelectorAll("option");
      if (this._value !== undefined && opts.some(function (o) { return o.value === this._value; }, this)) return this._value;
      var sel = opts.filter(function (o) { return o.selected; })[0] || opts[0];
      return sel ? sel.value : "";
    }
    if (this.tagName === "OPTION") return this.attributes.value !== undefined ? this.attributes.value : this.textContent;
    if (this._value !== undefined) return this._value;
    if (this.tagName === "TEXTAREA") return this.textContent;
    return this.attributes.value !== undefined ? this.attributes.value : (this.type === "checkbox" ? "on" : "");
  }
  set value(v) {
    if (this.tagName === "OPTION") this.attributes.value = String(v);    // reflects to the attribute
    else this._value = String(v);
  }
  addEventListener(t, fn) { (this.listeners[t] = this.listeners[t] || []).push(fn); }
  removeEventListener(t, fn) { this.listeners[t] = (this.listeners[t] || []).filter(function (f) { return f !== fn; }); }
  dispatchEvent(ev) {
    ev.target = ev.target || this;
    ev.defaultPrevented = false;
    ev.preventDefault = function () { ev.defaultPrevented = true; };
    var stop = false;
    ev.stopPropagation = function () { stop = true; };
    for (var n = this; n && !stop; n = n.parentNode) {
      ev.currentTarget = n;
      (n.listeners ? (n.listeners[ev.type] || []).slice() : []).forEach(function (fn) { fn.call(n, ev); });
      if (n["on" + ev.type]) n["on" + ev.type].call(n, ev);
      if (ev.bubbles === false) break;
    }
    return !ev.defaultPrevented;
  }
  click() {
    if (this.disabled) return;
    if (this.tagName === "INPUT" && this.type === "checkbox") {
      this.checked = !this.checked;
      this.dispatchEvent({ type: "click" });
      this.dispatchEvent({ type: "change" });
      return;
    }
    var ok = this.dispatchEvent({ type: "click" });
    // a submit button submits its form; a link follows its hash
    if (ok && this.tagName === "BUTTON" && this.type === "submit") {
      for (var f = this.parentNode; f; f = f.parentNode) if (f.tagName === "FORM") { f.dispatchEvent({ type: "submit" }); break; }
    }
    if (ok && this.tagName === "A" && this.href.indexOf("#") === 0) global.__shim.location.hash = this.href;
  }
  // user typing / picking: set the value, then fire input + change
  type_(v) { this.value = v; this.dispatchEvent({ type: "input" }); this.dispatchEvent({ type: "change" }); }
  select_(v) { this.value = v; this.dispatchEvent({ type: "change" }); }
  querySelectorAll(sel) { return selectAll(this, sel); }
  querySelector(sel) { return selectAll(this, sel)[0] || null; }
  get outerText() { return this.textContent; }
}

// ---- selectors
function parseCompound(s) {
  var re = /([a-zA-Z0-9*-]+)|#([\w-]+)|\.([\w-]+)|\[([\w-]+)(?:="([^"]*)")?\]|:(checked|disabled)/g, m, out = { attrs: [] };
  while ((m = re.exec(s))) {
    if (m[1]) out.tag = m[1].toUpperCase();
    else if (m[2]) out.id = m[2];
    else if (m[3]) (out.cls = out.cls || []).push(m[3]);
    else if (m[4]) out.attrs.push([m[4], m[5]]);
    else if (m[6]) out.pseudo = m[6];
  }
  return out;
}
function matches(e, c) {
  if (!(e instanceof Element_)) return false;
  if (c.tag && c.tag !== "*" && e.tagName !== c.tag) return false;
  if (c.id && e.id !== c.id) return false;
  if (c.cls && !c.cls.every(function (k) { return e.classList.contains(k); })) return false;
  if (!c.attrs.every(function (a) { var v = e.getAttribute(a[0]); return v !== null && (a[1] === undefined || v === a[1]); })) return false;
  if (c.pseudo === "checked" && !e.checked) return false;
  if (c.pseudo === "disabled" && !e.disabled) return false;
  return true;
}
function descendants(n, out) {
  n.childNodes.forEach(function (c) { if (c instanceof Element_) { out.push(c); descendants(c, out); } });
  return out;
}
function selectAll(root, sel) {
  var res = [];
  sel.split(",").forEach(function (one) {
    var parts = one.trim().match(/(?:[^\s"\[]|\[[^\]]*\])+/g).map(parseCompound);
    var cur = [root];
    parts.forEach(function (p) {
      var next = [];
      cur.forEach(function (n) { descendants(n, []).forEach(function (d) { if (matches(d, p) && next.indexOf(d) < 0) next.push(d); }); });
      cur = next;
    });
    cur.forEach(function (e) { if (res.indexOf(e) < 0) res.push(e); });
  });
  return res;
}

// ---- the page environment
function makeEnv(opts) {
  opts = opts || {};
  var routes = opts.routes || {};
  var requests = [], timers = [], winListeners = {}, posted = [];
  var document = new Element_("#document");
  var html = new Element_("html"), head = new Element_("head"), body = new Element_("body");
  document.append(html);
  html.append(head, body);
  document.body = body;
  document.head = head;
  document.cookie = "XSRF-TOKEN=tok123";
  document.createElement = function (t) { return new Element_(t); };
  document.createElementNS = function (ns, t) { var e = new Element_(t); e.namespaceURI = ns; return e; };
  document.createTextNode = function (t) { return new Text_(t); };
  document.getElementById = function (id) { return selectAll(document, "#" + id)[0] || null; };
  var baseHref = opts.base || "http://localhost/app/";
  var app = new Element_("div");
  app.setAttribute("id", "app");
  app.setAttribute("data-app", opts.app || "dashboard");
  body.append(app);
  var realQS = document.querySelector.bind(document);
  document.querySelector = function (s) { return s === "base" ? { href: baseHref } : realQS(s); };
  var loc = { _hash: opts.hash || "", search: opts.search || "", pathname: "/app/", href: baseHref,
              reloaded: 0, reload: function () { this.reloaded++; },
              replaced: [], replace: function (u) { this.replaced.push(u); } };
  Object.defineProperty(loc, "hash", {
    get: function () { return this._hash; },
    set: function (v) {
      v = String(v);
      if (v && v[0] !== "#") v = "#" + v;
      if (v === this._hash) return;
      this._hash = v;
      Promise.resolve().then(function () { (winListeners.hashchange || []).forEach(function (f) { f({ type: "hashchange" }); }); });
    }
  });
  var store = {}, lstore = opts.localStorage || {};
  var window = {
    document: document, location: loc,
    addEventListener: function (t, f) { (winListeners[t] = winListeners[t] || []).push(f); },
    removeEventListener: function () {},
    postMessage: function (data) { posted.push(data); }
  };
  window.parent = opts.inIframe ? { postMessage: function (d) { posted.push(d); } } : window;
  window.self = window;
  function respond(method, url, body, headers) {
    var u = new URL(url);
    var path = u.pathname.replace(/^\/app\//, "").replace(/^\//, "") + u.search;
    requests.push({ method: method, path: path, body: body === undefined ? undefined : JSON.parse(body), headers: headers || {} });
    var key = method + " " + path, h = routes[key] !== undefined ? routes[key] : routes[method + " " + path.split("?")[0]];
    if (typeof h === "function") h = h(body === undefined ? undefined : JSON.parse(body), path);
    if (h === undefined) h = { status: 404, body: { success: false, status: 404, log: "not found: " + key } };
    if (h === "NETWORK") return Promise.reject(new TypeError("Failed to fetch"));
    var st = h.status || 200, b = h.body !== undefined ? h.body : h;
    if (h.status === undefined) st = 200;
    return Promise.resolve({ ok: st >= 200 && st < 300, status: st, statusText: st === 200 ? "OK" : "Error", url: u.href,
                             json: function () { return Promise.resolve(JSON.parse(JSON.stringify(b))); } });
  }
  var ctx = {
    window: window, self: window, document: document, location: loc, Node: Node_,
    console: console, URL: URL, URLSearchParams: URLSearchParams, Promise: Promise, JSON: JSON, Math: Math, Date: Date,
    Array: Array, Object: Object, String: String, Number: Number, RegExp: RegExp, Error: Error, TypeError: TypeError,
    encodeURIComponent: encodeURIComponent, decodeURIComponent: decodeURIComponent, parseInt: parseInt, parseFloat: parseFloat,
    isNaN: isNaN,
    Blob: function (parts, o) { this.parts = parts; this.type = (o || {}).type; },
    sessionStorage: { getItem: function (k) { return store[k] === undefined ? null : store[k]; },
                      setItem: function (k, v) { store[k] = String(v); } },
    localStorage: { getItem: function (k) { return lstore[k] === undefined ? null : lstore[k]; },
                    setItem: function (k, v) { lstore[k] = String(v); },
                    removeItem: function (k) { delete lstore[k]; } },
    navigator: { clipboard: { writeText: function () { return Promise.resolve(); } } },
    fetch: function (url, init) { init = init || {}; return respond(init.method || "GET", String(url), init.body, init.headers); },
    setTimeout: function (f, ms) { timers.push({ f: f, ms: ms }); return timers.length; },
    clearTimeout: function () {},
    confirm: function () { throw new Error("window.confirm used: pages must use KF.confirmDialog"); },
  };
  ctx.URL.createObjectURL = ctx.URL.createObjectURL || function () { return "blob:x"; };
  Object.keys(ctx).forEach(function (k) { if (!(k in window)) window[k] = ctx[k]; });
  global.__shim = { location: loc };
  return { ctx: ctx, document: document, window: window, app: app, requests: requests, timers: timers, posted: posted,
           localStorage: lstore,
           winListeners: winListeners,
           // a postMessage arriving here: from this origin and the parent frame unless a test says otherwise
           message: function (data, origin, source) {
             var ev = { data: data, origin: origin === undefined ? new URL(loc.href).origin : origin,
                        source: source === undefined ? window.parent : source };
             (winListeners.message || []).forEach(function (f) { f(ev); });
           } };
}

function flush(n) {
  var p = Promise.resolve();
  for (var i = 0; i < (n || 30); i++) p = p.then(function () { return new Promise(function (r) { setImmediate(r); }); });
  return p;
}

module.exports = { makeEnv: makeEnv, flush: flush, Element: Element_, Text: Text_ };
