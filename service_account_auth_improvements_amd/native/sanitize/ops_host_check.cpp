// Host-side sanitizer harness for the op library (VERDICT r1 hygiene: "an ASan+UBSan build and
// run of the host side of ops/csrc/bindings.cpp").
//
// Built by native/sanitize.py together with bindings.cpp and every ops/csrc/*.hip file, all
// with AddressSanitizer + UndefinedBehaviorSanitizer on the HOST side only (device code is
// ordinary gfx950 code), and linked against libtorch.  It drives every registered
// torch.ops.kfamd operator through the dispatcher (boxed calls, exactly the path Python uses):
//
//   * argument validation: CPU tensors, wrong dtypes, wrong shapes, out-of-range slots must be
//     rejected with c10::Error before any kernel launch (runs on CPU-only hosts);
//   * with a GPU (--gpu): every op on small shapes, checked against an fp32 ATen reference of
//     the same math, so the host launch code (grid sizing, workspace sizing, the flash
//     backward's side-stream fork/join, the decode split choice, the embedding sort) runs under
//     the sanitizers with real launches.
//
// Exit status 0 = all checks passed and no sanitizer report (reports abort the process).
#include <ATen/ATen.h>
#include <ATen/core/dispatch/Dispatcher.h>
#include <ATen/core/stack.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

namespace {

using Stack = std::vector<c10::IValue>;
int g_fail = 0, g_pass = 0;

Stack call(const char* op, Stack s) {
  auto h = c10::Dispatcher::singleton().findSchemaOrThrow(op, "");
  h.callBoxed(&s);
  return s;
}

void expect_reject(const char* what, const char* op, Stack s) {
  try {
    call(op, std::move(s));
    std::printf("FAIL reject %-40s (accepted)\n", what);
    ++g_fail;
  } catch (const c10::Error&) {
    ++g_pass;
  }
}

void expect_close(const char* what, const at::Tensor& got, const at::Tensor& ref, double atol, double rtol) {
  auto g = got.detach().to(at::kCPU, at::kFloat).reshape({-1});
  auto r = ref.detach().to(at::kCPU, at::kFloat).reshape({-1});
  if (g.numel() != r.numel()) {
    std::printf("FAIL %-44s numel %lld vs %lld\n", what, (long long)g.numel(), (long long)r.numel());
    ++g_fail;
    return;
  }
  auto err = (g - r).abs();
  auto tol = r.abs() * rtol + atol;
  const double maxerr = err.max().item<double>();
  const long bad = (err > tol).sum().item<long>();
  const bool finite = at::isfinite(g).all().item<bool>();
  if (bad == 0 && finite) {
    std::printf("PASS %-44s max|err| %.3e\n", what, maxerr);
    ++g_pass;
  } else {
    std::printf("FAIL %-44s max|err| %.3e, %ld of %lld outside tolerance, finite=%d\n", what, maxerr, bad,
                (long long)g.numel(), (int)finite);
    ++g_fail;
  }
}

// ------------------------------------------------------------------ validation (CPU-only hosts too)
void check_rejections_cpu() {
  auto bf = at::TensorOptions().dtype(at::kBFloat16);
  auto f32 = at::TensorOptions().dtype(at::kFloat);
  auto i64 = at::TensorOptions().dtype(at::kLong);
  auto x = at::randn({4, 256}, bf), w = at::randn({256}, bf);
  expect_reject("rmsnorm_fwd cpu tensor", "kfamd::rmsnorm_fwd", {x, c10::IValue(), w, 1e-5});
  expect_reject("rmsnorm_fwd fp32 input", "kfamd::rmsnorm_fwd", {x.to(at::kFloat), c10::IValue(), w, 1e-5});
  expect_reject("swiglu_fwd cpu tensor", "kfamd::swiglu_fwd", {x});
  expect_reject("swiglu_bwd cpu tensor", "kfamd::swiglu_bwd", {x, at::randn({4, 128}, bf)});
  auto p = at::zeros({64}, bf), m = at::zeros({64}, f32);
  expect_reject("adamw_ cpu tensor", "kfamd::adamw_",
                {p, m, m.clone(), m.clone(), p.clone(), 32, 1e-3, 0.9, 0.95, 1e-8, 0.1, 1, 1.0, c10::IValue(), 0.0});
  expect_reject("sumsq cpu tensor", "kfamd::sumsq", {p, at::zeros({1}, f32), false});
  expect_reject("shard_sum_ cpu tensor", "kfamd::shard_sum_", {at::zeros({16}, bf), 2, at::zeros({8}, f32), false});
  expect_reject("grad_accum_ cpu tensor", "kfamd::grad_accum_", {at::zeros({8}, f32), at::zeros({8}, bf), 1});
  auto lg = at::randn({4, 512}, bf);
  auto lab = at::zeros({4}, i64);
  expect_reject("cross_entropy_ cpu tensor", "kfamd::cross_entropy_",
                {lg, lab, 0, -100, c10::IValue(), 1.0, 0, at::zeros({4}, f32), at::zeros({4}, f32), c10::IValue(),
                 c10::IValue(), c10::IValue()});
  auto qkv = at::randn({128, 3 * 128}, bf);
  expect_reject("flash_fwd cpu tensor", "kfamd::flash_fwd", {qkv, 1, 128, 1, 1, 128, 0.08, true});
  expect_reject("transpose_bf16 cpu tensor", "kfamd::transpose_bf16", {at::randn({64, 64}, bf)});
  expect_reject("skinny_gemm cpu tensor", "kfamd::skinny_gemm", {at::randn({1, 256}, bf), at::randn({16, 256}, bf), false});
  expect_reject("embed_fwd cpu tensor", "kfamd::embed_fwd", {at::zeros({4}, i64), at::randn({16, 64}, bf), 0});
  expect_reject("car_open short handle", "kfamd::car_open", {at::zeros({8}, at::TensorOptions().dtype(at::kByte))});
  expect_reject("gemm_tn_ cpu tensor", "kfamd::gemm_tn_",
                {at::randn({128, 256}, bf), at::randn({128, 256}, bf), at::zeros({256, 256}, bf), false});
  // the gemm_tn_ok predicate answers false (never throws) for non-GPU operands
  auto ok = call("kfamd::gemm_tn_ok", {at::randn({128, 256}, bf), at::randn({128, 256}, bf), at::zeros({256, 256}, bf)});
  if (ok.at(0).toBool()) { std::printf("FAIL gemm_tn_ok accepted CPU tensors\n"); ++g_fail; } else { ++g_pass; }
  std::printf("validation (CPU): %d checks\n", g_pass);
}

// ------------------------------------------------------------------ GPU runs
at::Tensor attn_ref(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale) {
  // q [B,Hq,S,D], k/v [B,Hkv,S,D] fp32, causal
  const int64_t rep = q.size(1) / k.size(1), S = q.size(2);
  auto kf = k.repeat_interleave(rep, 1), vf = v.repeat_interleave(rep, 1);
  auto s = at::matmul(q, kf.transpose(-1, -2)) * scale;
  auto mask = at::ones({S, S}, q.options().dtype(at::kBool)).triu(1);
  s = s.masked_fill(mask, -INFINITY);
  return at::matmul(at::softmax(s, -1), vf);
}

void check_gpu() {
  at::manual_seed(7);
  auto dev = at::TensorOptions().device(at::kCUDA);
  auto bf = dev.dtype(at::kBFloat16), f32 = dev.dtype(at::kFloat), i64 = dev.dtype(at::kLong),
       i32 = dev.dtype(at::kInt);

  // RMSNorm with the fused residual add
  {
    auto a = at::randn({64, 1024}, bf), b = at::randn({64, 1024}, bf), w = at::randn({1024}, bf);
    auto r = call("kfamd::rmsnorm_fwd", {a, b, w, 1e-5});
    auto hf = a.to(at::kFloat) + b.to(at::kFloat);
    auto yref = hf * at::rsqrt(hf.pow(2).mean(-1, true) + 1e-5) * w.to(at::kFloat);
    expect_close("rmsnorm_fwd y", r[0].toTensor(), yref, 2e-2, 2e-2);
    expect_close("rmsnorm_fwd h", r[1].toTensor(), hf, 1e-2, 1e-2);
    auto h = r[1].toTensor(), rstd = r[2].toTensor();
    auto dy = at::randn({64, 1024}, bf), dw = at::zeros({1024}, bf);
    auto dh = call("kfamd::rmsnorm_bwd", {dy, h, rstd, w, c10::IValue(), dw, false})[0].toTensor();
    auto hv = h.to(at::kFloat).detach().requires_grad_(true);
    auto wv = w.to(at::kFloat).detach().requires_grad_(true);
    auto y = hv * at::rsqrt(hv.pow(2).mean(-1, true) + 1e-5) * wv;
    y.backward(dy.to(at::kFloat));
    expect_close("rmsnorm_bwd dh", dh, hv.grad(), 3e-2, 3e-2);
    expect_close("rmsnorm_bwd dw", dw, wv.grad(), 0.5, 3e-2);
    expect_reject("rmsnorm_fwd weight mismatch", "kfamd::rmsnorm_fwd", {a, c10::IValue(), at::randn({512}, bf), 1e-5});
  }
  // SwiGLU
  {
    auto gu = at::randn({32, 2 * 512}, bf);
    auto out = call("kfamd::swiglu_fwd", {gu})[0].toTensor();
    auto g = gu.narrow(1, 0, 512).to(at::kFloat), u = gu.narrow(1, 512, 512).to(at::kFloat);
    expect_close("swiglu_fwd", out, at::silu(g) * u, 2e-2, 2e-2);
    auto dout = at::randn({32, 512}, bf);
    auto dgu = call("kfamd::swiglu_bwd", {gu, dout})[0].toTensor();
    auto gv = gu.to(at::kFloat).detach().requires_grad_(true);
    auto o = at::silu(gv.narrow(1, 0, 512)) * gv.narrow(1, 512, 512);
    o.backward(dout.to(at::kFloat));
    expect_close("swiglu_bwd", dgu, gv.grad(), 3e-2, 3e-2);
  }
  // AdamW with bf16 and fp32 gradients, clip from the device sum of squares
  {
    const int64_t n = 4096, n_decay = 2048;
    auto w0 = at::randn({n}, f32), g32 = at::randn({n}, f32).to(at::kBFloat16).to(at::kFloat);
    for (int gfp32 = 0; gfp32 < 2; ++gfp32) {
      auto p = w0.to(at::kBFloat16), w = w0.clone(), m = at::zeros({n}, f32), v = at::zeros({n}, f32);
      auto g = gfp32 ? g32 : g32.to(at::kBFloat16);
      auto ss = at::zeros({1}, f32);
      call("kfamd::sumsq", {g, ss, false});
      expect_close(gfp32 ? "sumsq fp32 grad" : "sumsq bf16 grad", ss, g32.pow(2).sum().reshape({1}), 1e-2, 1e-4);
      const double lr = 1e-2, b1 = 0.9, b2 = 0.95, eps = 1e-8, wd = 0.1, max_norm = 1.0;
      call("kfamd::adamw_", {p, w, m, v, g, n_decay, lr, b1, b2, eps, wd, 1, 1.0, ss, max_norm});
      const double nrm = std::sqrt(g32.pow(2).sum().item<double>());
      auto gc = g32 * std::min(1.0, max_norm / (nrm + 1e-6));
      auto mr = gc * (1 - b1), vr = gc * gc * (1 - b2);
      auto upd = (mr / (1 - b1)) / (at::sqrt(vr) / std::sqrt(1 - b2) + eps);
      auto decay = at::ones({n}, f32);
      decay.narrow(0, 0, n_decay).fill_(1 - lr * wd);
      auto wref = w0 * decay - lr * upd;
      expect_close(gfp32 ? "adamw_ fp32 grad master" : "adamw_ bf16 grad master", w, wref, 1e-5, 1e-5);
      expect_close(gfp32 ? "adamw_ fp32 grad compute copy" : "adamw_ bf16 grad compute copy", p, wref, 1e-2, 1e-2);
    }
  }
  // fp32 DP reduction pieces
  {
    const int64_t R = 4, n = 2048;
    auto recv = at::randn({R * n}, bf), out = at::randn({n}, f32);
    auto ref = out + recv.to(at::kFloat).view({R, n}).sum(0);
    call("kfamd::shard_sum_", {recv, R, out, true});
    expect_close("shard_sum_ accumulate", out, ref, 1e-5, 1e-5);
    expect_reject("shard_sum_ size mismatch", "kfamd::shard_sum_", {recv, 3, out, false});
    auto main_ = at::zeros({n}, f32), g1 = at::randn({n}, bf), g2 = at::randn({n}, bf);
    call("kfamd::grad_accum_", {main_, g1, 0});
    call("kfamd::grad_accum_", {main_, g2, 1});
    expect_close("grad_accum_ set+add", main_, g1.to(at::kFloat) + g2.to(at::kFloat), 1e-6, 1e-6);
    auto g3 = at::randn({n}, bf);
    auto fold = (main_ + g3.to(at::kFloat));
    call("kfamd::grad_accum_", {main_, g3, 2});
    expect_close("grad_accum_ fold", g3, fold, 1e-2, 1e-2);
  }
  // fused cross entropy (loss rows, lse, dlogits in place)
  {
    const int64_t T = 16, V = 4096;
    auto logits = at::randn({T, V}, bf) * 3;
    logits = logits.to(at::kBFloat16).contiguous();
    auto labels = at::randint(0, V, {T}, i64);
    labels.index_put_({at::indexing::Slice(0, 1)}, -100);
    auto lf = logits.to(at::kFloat);
    auto loss = at::empty({T}, f32), lse = at::empty({T}, f32);
    const double sc = 1.0 / (T - 1);
    call("kfamd::cross_entropy_", {logits, labels, 0, -100, c10::IValue(), sc, 0, loss, lse, c10::IValue(),
                                   c10::IValue(), c10::IValue()});
    auto lse_ref = at::logsumexp(lf, -1);
    auto valid = labels.ne(-100);
    auto xy = lf.gather(1, labels.clamp_min(0).unsqueeze(1)).squeeze(1);
    expect_close("cross_entropy_ lse", lse, lse_ref, 1e-3, 1e-4);
    expect_close("cross_entropy_ loss", loss, at::where(valid, lse_ref - xy, at::zeros_like(xy)), 1e-3, 1e-4);
    auto pr = at::softmax(lf, -1);
    pr.scatter_add_(1, labels.clamp_min(0).unsqueeze(1), -at::ones({T, 1}, f32));
    pr = pr * sc * valid.unsqueeze(1).to(at::kFloat);
    expect_close("cross_entropy_ dlogits", logits, pr, 1e-4, 2e-2);
  }
  // flash attention fwd + bwd (GQA 4:2, causal, two sequences) against fp32 autograd
  {
    const int64_t B = 2, S = 256, Hq = 4, Hkv = 2, D = 128;
    const double scale = 1.0 / std::sqrt((double)D);
    auto qkv = at::randn({B * S, (Hq + 2 * Hkv) * D}, bf);
    auto r = call("kfamd::flash_fwd", {qkv, B, S, Hq, Hkv, D, scale, true});
    auto o = r[0].toTensor(), lse = r[1].toTensor();
    auto split = [&](const at::Tensor& t, int64_t off, int64_t H) {
      return t.narrow(1, off * D, H * D).reshape({B, S, H, D}).permute({0, 2, 1, 3}).to(at::kFloat).contiguous();
    };
    auto q = split(qkv, 0, Hq).requires_grad_(true), k = split(qkv, Hq, Hkv).requires_grad_(true),
         v = split(qkv, Hq + Hkv, Hkv).requires_grad_(true);
    auto oref = attn_ref(q, k, v, scale);
    expect_close("flash_fwd o", o, oref.permute({0, 2, 1, 3}).reshape({B * S, Hq * D}), 2e-2, 2e-2);
    auto dout = at::randn({B * S, Hq * D}, bf);
    auto dqkv = call("kfamd::flash_bwd", {qkv, o, lse, dout, B, S, Hq, Hkv, D, scale, true, true})[0].toTensor();
    auto dqkv_atomic = call("kfamd::flash_bwd", {qkv, o, lse, dout, B, S, Hq, Hkv, D, scale, true, false})[0].toTensor();
    oref.backward(dout.to(at::kFloat).reshape({B, S, Hq, D}).permute({0, 2, 1, 3}));
    auto back = [&](const at::Tensor& gr, int64_t H) { return gr.permute({0, 2, 1, 3}).reshape({B * S, H * D}); };
    expect_close("flash_bwd dq", dqkv.narrow(1, 0, Hq * D), back(q.grad(), Hq), 5e-2, 5e-2);
    expect_close("flash_bwd dk", dqkv.narrow(1, Hq * D, Hkv * D), back(k.grad(), Hkv), 5e-2, 5e-2);
    expect_close("flash_bwd dv", dqkv.narrow(1, (Hq + Hkv) * D, Hkv * D), back(v.grad(), Hkv), 5e-2, 5e-2);
    expect_close("flash_bwd atomic vs deterministic", dqkv_atomic, dqkv, 2e-2, 2e-2);
    expect_reject("flash_fwd head dim 64", "kfamd::flash_fwd", {qkv, B, S, Hq, Hkv, (int64_t)64, scale, true});
    expect_reject("flash_fwd S % 128", "kfamd::flash_fwd",
                  {at::randn({B * 200, (Hq + 2 * Hkv) * D}, bf), B, (int64_t)200, Hq, Hkv, D, scale, true});
    expect_reject("flash_bwd lse size", "kfamd::flash_bwd",
                  {qkv, o, lse.narrow(2, 0, 128).contiguous(), dout, B, S, Hq, Hkv, D, scale, true, true});
  }
  // embedding fwd / bwd (sorted scatter-add), one vocab shard starting at 100
  {
    const int64_t Vl = 200, H = 256, T = 64, vstart = 100;
    auto E = at::randn({Vl, H}, bf);
    auto tok = at::randint(0, 400, {T}, i64);
    auto out = call("kfamd::embed_fwd", {tok, E, vstart})[0].toTensor();
    auto loc = tok - vstart;
    auto inr = loc.ge(0).logical_and(loc.lt(Vl));
    auto ref = E.to(at::kFloat).index_select(0, loc.clamp(0, Vl - 1)) * inr.unsqueeze(1).to(at::kFloat);
    expect_close("embed_fwd", out, ref, 0, 0);
    auto g = at::randn({T, H}, bf), dE = at::zeros({Vl, H}, bf);
    call("kfamd::embed_bwd_", {tok, g, dE, vstart, false});
    auto dref = at::zeros({Vl, H}, f32);
    dref.index_add_(0, loc.clamp(0, Vl - 1), g.to(at::kFloat) * inr.unsqueeze(1).to(at::kFloat));
    expect_close("embed_bwd_", dE, dref, 3e-2, 2e-2);
  }
  // transpose, weight-gradient GEMM, decode GEMMs
  {
    auto x = at::randn({128, 192}, bf);
    expect_close("transpose_bf16", call("kfamd::transpose_bf16", {x})[0].toTensor(), x.t(), 0, 0);
    expect_reject("transpose_bf16 dims % 64", "kfamd::transpose_bf16", {at::randn({100, 64}, bf)});
    auto a = at::randn({256, 256}, bf), b = at::randn({256, 512}, bf), c = at::randn({256, 512}, bf);
    auto cref = c.to(at::kFloat) + at::matmul(a.to(at::kFloat).t(), b.to(at::kFloat));
    call("kfamd::gemm_tn_", {a, b, c, true});
    expect_close("gemm_tn_ accumulate", c, cref, 0.5, 2e-2);
    expect_reject("gemm_tn_ M % 256", "kfamd::gemm_tn_", {at::randn({256, 128}, bf), b, at::zeros({128, 512}, bf), false});
    for (int64_t M : {1, 3, 16}) {
      auto xs = at::randn({M, 1024}, bf), ws = at::randn({512, 1024}, bf);
      auto y = call("kfamd::skinny_gemm", {xs, ws, false})[0].toTensor();
      std::string nm = "skinny_gemm M=" + std::to_string(M);
      expect_close(nm.c_str(), y, at::matmul(xs.to(at::kFloat), ws.to(at::kFloat).t()), 0.5, 2e-2);
    }
    expect_reject("skinny_gemm K mismatch", "kfamd::skinny_gemm", {at::randn({2, 1024}, bf), at::randn({64, 512}, bf), false});
  }
  // prefill a KV cache slot, then single-token decode attention over it
  {
    const int64_t Hq = 8, Hkv = 2, D = 128, S = 300, slots_n = 3, Lmax = 512, slot = 1;
    auto qkv = at::randn({S, (Hq + 2 * Hkv) * D}, bf);
    auto kc = at::zeros({slots_n, Hkv, Lmax, D}, bf), vc = at::zeros({slots_n, Hkv, Lmax, D}, bf);
    call("kfamd::kv_fill_", {qkv, S, Hq, slot, kc, vc});
    auto kref = qkv.narrow(1, Hq * D, Hkv * D).reshape({S, Hkv, D}).permute({1, 0, 2});
    expect_close("kv_fill_ k", kc.select(0, slot).narrow(1, 0, S), kref, 0, 0);
    expect_reject("kv_fill_ slot out of range", "kfamd::kv_fill_", {qkv, S, Hq, slots_n, kc, vc});
    auto q = at::randn({1, Hq * D}, bf);
    auto slots = at::full({1}, slot, i32), lens = at::full({1}, S, i32);
    const double scale = 1.0 / std::sqrt((double)D);
    auto o = call("kfamd::decode_attn", {q, kc, vc, slots, lens, Hq, scale})[0].toTensor();
    auto qf = q.to(at::kFloat).reshape({Hq, 1, D});
    auto kf = kref.to(at::kFloat).repeat_interleave(Hq / Hkv, 0);
    auto vf = qkv.narrow(1, (Hq + Hkv) * D, Hkv * D).reshape({S, Hkv, D}).permute({1, 0, 2}).to(at::kFloat)
                  .repeat_interleave(Hq / Hkv, 0);
    auto oref = at::matmul(at::softmax(at::matmul(qf, kf.transpose(1, 2)) * scale, -1), vf).reshape({1, Hq * D});
    expect_close("decode_attn", o, oref, 2e-2, 2e-2);
    expect_reject("decode_attn lengths dtype", "kfamd::decode_attn", {q, kc, vc, slots, lens.to(at::kLong), Hq, scale});
  }
}

}  // namespace

int main(int argc, char** argv) {
  bool gpu = argc > 1 && std::strcmp(argv[1], "--gpu") == 0;
  check_rejections_cpu();
  if (gpu) {
    if (!at::hasCUDA()) {
      std::printf("FAIL --gpu given but no GPU is visible\n");
      return 1;
    }
    check_gpu();
  }
  std::printf("%s: %d passed, %d failed\n", gpu ? "host-sanitized ops (GPU)" : "host-sanitized ops (CPU)", g_pass,
              g_fail);
  return g_fail == 0 ? 0 : 1;
}
