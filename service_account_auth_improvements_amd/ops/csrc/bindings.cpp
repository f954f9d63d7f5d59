// Torch operator registrations for the gfx950 kernels (namespace torch.ops.kfamd).
//
// The .hip translation units expose plain `extern "C"` launchers taking raw pointers and
// a hipStream_t; only this file sees libtorch.  Every op launches on the caller's current
// HIP stream, allocates scratch through the caching allocator (capturable in hipGraphs)
// and validates shapes/dtypes on the host BEFORE any kernel is launched: a kernel is
// never started on operands whose shape it does not support.
#include <cstdlib>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <map>
#include <tuple>

extern "C" {
int kf_rmsnorm_fwd_parts(const void*, const float*, int, void*, void*, float*, const void*, int, int, float,
                         hipStream_t);
int kf_rmsnorm_fwd(const void*, const void*, void*, void*, float*, const void*, int, int, float,
                   hipStream_t);
int kf_rmsnorm_bwd(const void*, const void*, const float*, const void*, const void*, void*, float*,
                   int, void*, int, int, int, hipStream_t);
int kf_rope(void*, long, int, int, int, const float*, const float*, const int*, int, int,
            hipStream_t);
int kf_swiglu_fwd(const void*, void*, int, int, hipStream_t);
int kf_swiglu_bwd(const void*, const void*, void*, int, int, hipStream_t);
int kf_adamw(void*, float*, float*, float*, const void*, int, size_t, size_t, float, float, float, float,
             float, int, float, const float*, float, hipStream_t);
int kf_sumsq(const void*, int, size_t, float*, float*, int, hipStream_t);
int kf_shard_sum(const void*, int, size_t, float*, int, hipStream_t);
int kf_grad_accum(float*, void*, size_t, int, hipStream_t);
int kf_cross_entropy(void*, long, int, int, const long*, long, long, float*, float*, float*, float*,
                     float*, const float*, float, int, hipStream_t);
int kf_flash_fwd(const void*, long, void*, long, float*, int, int, int, int, int, float, int,
                 hipStream_t);
int kf_flash_bwd(const void*, long, const void*, long, const void*, long, const float*, float*,
                 float*, float*, void*, long, int, int, int, int, int, float, int, int, hipStream_t);
long kf_flash_bwd_acc_floats(int, int, int, int, int);
int kf_decode_splits(int, int, int);
int kf_decode_splits1(int, int, int);
int kf_decode_attn_fused(const void*, long, const void*, const void*, const int*, const int*, void*, long, float*,
                         float*, int*, int, int, int, int, int, int, float, hipStream_t);
int kf_decode_attn(const void*, long, const void*, const void*, const int*, const int*, void*, long,
                   float*, float*, int, int, int, int, int, int, float, hipStream_t);
int kf_rope_append_parts(const float*, int, void*, int, int, int, int, const float*, const float*, const int*,
                         const int*, void*, void*, int, hipStream_t);
int kf_rope_append(void*, long, int, int, int, int, const float*, const float*, const int*, const int*, void*,
                   void*, int, hipStream_t);
int kf_kv_append(const void*, long, int, int, int, int, const int*, const int*, void*, void*, int,
                 hipStream_t);
int kf_kv_fill(const void*, long, int, int, int, int, int, void*, void*, int, hipStream_t);
int kf_embed_fwd(const long*, const void*, void*, int, int, long, long, hipStream_t);
int kf_embed_bwd(const long*, const long*, const void*, void*, int, int, long, long, int, hipStream_t);
int kf_skinny_gemm(const void*, long, int, const void*, int, int, void*, long, int, int, hipStream_t);
int kf_bgemm_splits(int, int, int);
int kf_bgemm(const void*, long, int, const void*, int, int, void*, long, int, int, int, float*, hipStream_t);
int kf_gemv(const void*, long, int, const void*, const void*, float, void*, long, const void*, int, int, void*, long,
            int, int, hipStream_t);
int kf_gemv_norm_rope(const void*, long, int, const void*, const void*, float, void*, long, const void*, int, int,
                      void*, long, const float*, const float*, const int*, const int*, void*, void*, int, int, int,
                      hipStream_t);
int kf_skinny_gemm_norm(const void*, long, int, const void*, const void*, float, void*, long, const void*, int, int,
                        void*, long, int, int, hipStream_t);
int kf_gemm_tn(const void*, long, const void*, long, void*, long, int, int, int, int, hipStream_t);
int kf_gemm_tn2(const void*, long, const void*, long, void*, long, int, int, const void*, long, const void*, long, void*,
                long, int, int, int, int, hipStream_t);
int kf_transpose_bf16(const void*, long, void*, long, int, int, hipStream_t);
long kf_car_header_bytes();
int kf_car_alloc(long, void**, void*);
int kf_car_open(const void*, void**);
int kf_car_close(void*);
int kf_car_free(void*);
int kf_car_allreduce(void* const*, int, int, const void*, void*, long, long, int, double, hipStream_t);
int kf_car_error(void*, hipStream_t);
long kf_ts_header_bytes();
int kf_ts_alloc(long, int, void**, void*);
int kf_ts_run(int, void* const*, int, int, const void*, void*, long, long, int, double, hipStream_t);
int kf_ts_error(void*, hipStream_t);
int kf_ts_error_async(void*, int*, hipStream_t);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_bf16_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}
void check_rc(int rc, const char* op) { TORCH_CHECK(rc == 0, op, ": unsupported shape (rc=", rc, ")"); }

// ---------------- RMSNorm ----------------
std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& a,
                                                           const std::optional<at::Tensor>& b,
                                                           const at::Tensor& w, double eps) {
  check_bf16_cuda(a, "a");
  check_bf16_cuda(w, "w");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous(), "rmsnorm: contiguous inputs required");
  const int64_t H = a.size(-1);
  TORCH_CHECK(w.numel() == H, "rmsnorm: weight size mismatch");
  const int64_t rows = a.numel() / H;
  c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  auto y = at::empty_like(a);
  auto rstd = at::empty({rows}, a.options().dtype(at::kFloat));
  at::Tensor h;
  const void* bp = nullptr;
  void* hp = nullptr;
  if (b.has_value()) {
    check_bf16_cuda(*b, "b");
    TORCH_CHECK(b->is_contiguous() && b->sizes() == a.sizes(), "rmsnorm: residual shape mismatch");
    h = at::empty_like(a);
    bp = b->data_ptr();
    hp = h.data_ptr();
  } else {
    h = at::empty({0}, a.options());
  }
  check_rc(kf_rmsnorm_fwd(a.data_ptr(), bp, hp, y.data_ptr(), rstd.data_ptr<float>(), w.data_ptr(),
                          (int)rows, (int)H, (float)eps, cur_stream()),
           "rmsnorm_fwd");
  return {y, h, rstd};
}

// h = a + bf16(sum_s part[s]); y = rmsnorm(h) * w with part the fp32 K-split partials [S, rows, H]
// of the batched-decode GEMM (bgemm_parts): the reduce launch folded into the norm
std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_fwd_parts(const at::Tensor& a, const at::Tensor& part,
                                                                 const at::Tensor& w, double eps) {
  check_bf16_cuda(a, "a");
  check_bf16_cuda(w, "w");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3,
              "rmsnorm_fwd_parts: fp32 [S, rows, H] partials");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous() && a.dim() == 2, "rmsnorm_fwd_parts: contiguous [rows, H] input");
  const int64_t rows = a.size(0), H = a.size(1);
  TORCH_CHECK(part.size(1) == rows && part.size(2) == H && w.numel() == H, "rmsnorm_fwd_parts: shape mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  auto y = at::empty_like(a);
  auto h = at::empty_like(a);
  auto rstd = at::empty({rows}, a.options().dtype(at::kFloat));
  check_rc(kf_rmsnorm_fwd_parts(a.data_ptr(), part.data_ptr<float>(), (int)part.size(0), h.data_ptr(), y.data_ptr(),
                                rstd.data_ptr<float>(), w.data_ptr(), (int)rows, (int)H, (float)eps, cur_stream()),
           "rmsnorm_fwd_parts");
  return {y, h, rstd};
}

at::Tensor rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& rstd,
                       const at::Tensor& w, const std::optional<at::Tensor>& dres, at::Tensor dw,
                       bool accumulate) {
  check_bf16_cuda(dy, "dy");
  check_bf16_cuda(h, "h");
  check_bf16_cuda(dw, "dw");
  TORCH_CHECK(dy.is_contiguous() && h.is_contiguous() && dy.sizes() == h.sizes(), "rmsnorm_bwd: shapes");
  TORCH_CHECK(dw.is_contiguous() && dw.numel() == h.size(-1), "rmsnorm_bwd: dw shape");
  const int64_t H = h.size(-1), rows = h.numel() / H;
  TORCH_CHECK(rstd.numel() == rows, "rmsnorm_bwd: rstd shape");
  c10::hip::HIPGuardMasqueradingAsCUDA g(h.device());
  auto dh = at::empty_like(h);
  const void* dr = nullptr;
  if (dres.has_value()) {
    TORCH_CHECK(dres->sizes() == h.sizes() && dres->is_contiguous(), "rmsnorm_bwd: dres shape");
    dr = dres->data_ptr();
  }
  // one block per row at a time; ~4 blocks per CU keep HBM busy, 1024 dW partial rows (16 MB at H=4096)
  int nblocks = (int)std::min<int64_t>(1024, rows);
  if (nblocks < 1) nblocks = 1;
  auto part = at::empty({(int64_t)nblocks, H}, h.options().dtype(at::kFloat));
  check_rc(kf_rmsnorm_bwd(dy.data_ptr(), h.data_ptr(), rstd.data_ptr<float>(), w.data_ptr(), dr,
                          dh.data_ptr(), part.data_ptr<float>(), nblocks, dw.data_ptr(),
                          accumulate ? 1 : 0, (int)rows, (int)H, cur_stream()),
           "rmsnorm_bwd");
  return dh;
}

// ---------------- RoPE (in place) ----------------
void rope_(at::Tensor x, int64_t nheads, int64_t head_dim, const at::Tensor& cos_t,
           const at::Tensor& sin_t, const std::optional<at::Tensor>& pos, int64_t seq_len,
           bool inverse) {
  check_bf16_cuda(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "rope: x must be [T, C] with unit inner stride");
  TORCH_CHECK(nheads * head_dim <= x.size(1), "rope: heads exceed row");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat &&
                  cos_t.is_contiguous() && sin_t.is_contiguous() && cos_t.size(-1) == head_dim / 2,
              "rope: cos/sin must be contiguous fp32 [P, D/2]");
  const int* pp = nullptr;
  if (pos.has_value()) {
    TORCH_CHECK(pos->scalar_type() == at::kInt && pos->numel() == x.size(0), "rope: pos int32 [T]");
    pp = pos->data_ptr<int>();
  } else {
    TORCH_CHECK(seq_len > 0 && seq_len <= cos_t.size(0), "rope: seq_len exceeds table");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(kf_rope(x.data_ptr(), x.stride(0), (int)x.size(0), (int)nheads, (int)head_dim,
                   cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), pp, (int)seq_len,
                   inverse ? 1 : 0, cur_stream()),
           "rope");
}

// ---------------- SwiGLU ----------------
at::Tensor swiglu_fwd(const at::Tensor& gu) {
  check_bf16_cuda(gu, "gu");
  TORCH_CHECK(gu.is_contiguous() && gu.size(-1) % 2 == 0, "swiglu: [.., 2F] contiguous");
  const int64_t F = gu.size(-1) / 2, rows = gu.numel() / gu.size(-1);
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto out = at::empty(sizes, gu.options());
  check_rc(kf_swiglu_fwd(gu.data_ptr(), out.data_ptr(), (int)rows, (int)F, cur_stream()), "swiglu_fwd");
  return out;
}

at::Tensor swiglu_bwd(const at::Tensor& gu, const at::Tensor& dout) {
  check_bf16_cuda(gu, "gu");
  check_bf16_cuda(dout, "dout");
  const int64_t F = gu.size(-1) / 2, rows = gu.numel() / gu.size(-1);
  TORCH_CHECK(gu.is_contiguous() && dout.is_contiguous() && dout.numel() == rows * F, "swiglu_bwd: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto dgu = at::empty_like(gu);
  check_rc(kf_swiglu_bwd(gu.data_ptr(), dout.data_ptr(), dgu.data_ptr(), (int)rows, (int)F, cur_stream()),
           "swiglu_bwd");
  return dgu;
}

// ---------------- AdamW (flat) ----------------
void adamw_(at::Tensor p, at::Tensor w, at::Tensor m, at::Tensor v, const at::Tensor& g,
            int64_t n_decay, double lr, double b1, double b2, double eps, double wd, int64_t step,
            double gscale, const std::optional<at::Tensor>& sumsq, double max_norm) {
  check_bf16_cuda(p, "p");
  TORCH_CHECK(g.is_cuda() && (g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat),
              "adamw: g must be a bf16 or fp32 GPU tensor");
  const int64_t n = p.numel();
  TORCH_CHECK(w.numel() == n && m.numel() == n && v.numel() == n && g.numel() == n, "adamw: sizes");
  TORCH_CHECK(w.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "adamw: master/m/v must be fp32");
  TORCH_CHECK(p.is_contiguous() && w.is_contiguous() && m.is_contiguous() && v.is_contiguous() &&
                  g.is_contiguous(), "adamw: contiguous flat buffers required");
  const float* sp = nullptr;
  if (sumsq.has_value()) sp = sumsq->data_ptr<float>();
  c10::hip::HIPGuardMasqueradingAsCUDA gd(p.device());
  check_rc(kf_adamw(p.data_ptr(), w.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                    g.data_ptr(), g.scalar_type() == at::kFloat ? 1 : 0, (size_t)n, (size_t)n_decay, (float)lr, (float)b1, (float)b2,
                    (float)eps, (float)wd, (int)step, (float)gscale, sp, (float)max_norm, cur_stream()),
           "adamw");
}

void sumsq(const at::Tensor& g, at::Tensor out, bool accumulate) {
  TORCH_CHECK(g.is_cuda() && (g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat),
              "sumsq: g must be a bf16 or fp32 GPU tensor");
  TORCH_CHECK(g.is_contiguous() && out.scalar_type() == at::kFloat, "sumsq: args");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(g.device());
  auto part = at::empty({2048}, g.options().dtype(at::kFloat));
  check_rc(kf_sumsq(g.data_ptr(), g.scalar_type() == at::kFloat ? 1 : 0, (size_t)g.numel(), part.data_ptr<float>(), out.data_ptr<float>(),
                    accumulate ? 1 : 0, cur_stream()),
           "sumsq");
}

// ---------------- Cross entropy (grad in place) ----------------
void cross_entropy_(at::Tensor logits, const at::Tensor& labels, int64_t vocab_start,
                    int64_t ignore_index, const std::optional<at::Tensor>& scale, double scale_h,
                    int64_t mode, at::Tensor loss, at::Tensor lse, const std::optional<at::Tensor>& sm,
                    const std::optional<at::Tensor>& ss, const std::optional<at::Tensor>& sxy) {
  check_bf16_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "ce: logits [T, V]");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0) && labels.is_contiguous(),
              "ce: labels int64 [T]");
  const int64_t rows = logits.size(0);
  TORCH_CHECK(loss.numel() == rows && lse.numel() == rows && loss.scalar_type() == at::kFloat &&
                  lse.scalar_type() == at::kFloat, "ce: loss/lse fp32 [T]");
  float *pm = nullptr, *ps = nullptr, *pxy = nullptr;
  if (mode == 1) {
    TORCH_CHECK(sm.has_value() && ss.has_value() && sxy.has_value(), "ce: stats outputs required");
    pm = sm->data_ptr<float>(); ps = ss->data_ptr<float>(); pxy = sxy->data_ptr<float>();
  }
  const float* scp = scale.has_value() ? scale->data_ptr<float>() : nullptr;
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  check_rc(kf_cross_entropy(logits.data_ptr(), logits.stride(0), (int)rows, (int)logits.size(1),
                            labels.data_ptr<int64_t>(), vocab_start, ignore_index, loss.data_ptr<float>(),
                            lse.data_ptr<float>(), pm, ps, pxy, scp, (float)scale_h, (int)mode, cur_stream()),
           "cross_entropy");
}

// ---------------- Flash attention (K3) ----------------
std::tuple<at::Tensor, at::Tensor> flash_fwd(const at::Tensor& qkv, int64_t B, int64_t S, int64_t Hq,
                                             int64_t Hkv, int64_t D, double scale, bool causal) {
  check_bf16_cuda(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(0) == B * S &&
                  qkv.size(1) >= (Hq + 2 * Hkv) * D, "flash_fwd: qkv must be [B*S, >=(Hq+2Hkv)*D]");
  TORCH_CHECK(D == 128 && S % 128 == 0 && Hq % Hkv == 0, "flash_fwd: needs D=128, S%128==0, Hq%Hkv==0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  auto o = at::empty({B * S, Hq * D}, qkv.options());
  auto lse = at::empty({B, Hq, S}, qkv.options().dtype(at::kFloat));
  check_rc(kf_flash_fwd(qkv.data_ptr(), qkv.stride(0), o.data_ptr(), o.stride(0), lse.data_ptr<float>(),
                        (int)B, (int)S, (int)Hq, (int)Hkv, (int)D, (float)scale, causal ? 1 : 0, cur_stream()),
           "flash_fwd");
  return {o, lse};
}

at::Tensor flash_bwd(const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                     const at::Tensor& dout, int64_t B, int64_t S, int64_t Hq, int64_t Hkv, int64_t D,
                     double scale, bool causal, bool deterministic) {
  check_bf16_cuda(qkv, "qkv");
  check_bf16_cuda(o, "o");
  check_bf16_cuda(dout, "dout");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(0) == B * S &&
                  qkv.size(1) >= (Hq + 2 * Hkv) * D, "flash_bwd: qkv shape");
  TORCH_CHECK(o.dim() == 2 && o.stride(1) == 1 && o.size(0) == B * S && o.size(1) == Hq * D, "flash_bwd: o shape");
  TORCH_CHECK(dout.sizes() == o.sizes() && dout.stride(1) == 1, "flash_bwd: dout shape");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * Hq * S, "flash_bwd: lse");
  TORCH_CHECK(D == 128 && S % 128 == 0 && Hq % Hkv == 0, "flash_bwd: needs D=128, S%128==0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  auto f32 = qkv.options().dtype(at::kFloat);
  auto delta = at::empty({B, Hq, S}, f32);
  // zeroed by kf_flash_bwd on its dK/dV stream (atomic mode) or fully stored (deterministic slots)
  const long nacc = kf_flash_bwd_acc_floats((int)B, (int)S, (int)Hkv, causal ? 1 : 0, deterministic ? 1 : 0);
  auto acc = at::empty({2 * nacc}, f32);
  float* dk = acc.data_ptr<float>();
  float* dv = dk + nacc;
  auto dqkv = at::empty({B * S, (Hq + 2 * Hkv) * D}, qkv.options());
  check_rc(kf_flash_bwd(qkv.data_ptr(), qkv.stride(0), o.data_ptr(), o.stride(0), dout.data_ptr(),
                        dout.stride(0), lse.data_ptr<float>(), delta.data_ptr<float>(), dk, dv,
                        dqkv.data_ptr(), dqkv.stride(0), (int)B, (int)S, (int)Hq, (int)Hkv, (int)D,
                        (float)scale, causal ? 1 : 0, deterministic ? 1 : 0, cur_stream()),
           "flash_bwd");
  return dqkv;
}

// ---------------- decode attention + KV cache (InferenceService) ----------------
void check_cache(const at::Tensor& kc, const at::Tensor& vc, int64_t Hkv, int64_t D) {
  check_bf16_cuda(kc, "k_cache");
  check_bf16_cuda(vc, "v_cache");
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.sizes() == kc.sizes() && vc.is_contiguous(),
              "kv cache must be contiguous [slots, Hkv, Lmax, D]");
  TORCH_CHECK(kc.size(1) == Hkv && kc.size(3) == D && D == 128, "kv cache: head shape mismatch (D=128)");
}
void check_rows_i32(const at::Tensor& t, int64_t B, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous() && t.numel() == B, name,
              " must be int32 [B] on the GPU");
}

// Per-device arrival tickets of the fused decode attention (4096 int32, zeroed once).  Returns
// nullptr while the current stream is capturing a graph and the buffer does not exist yet (the
// caller then takes the two-kernel path); the serving engine's warm-up runs before capture.
int* decode_tickets(int dev) {
  static std::mutex mu;
  static int* buf[64] = {nullptr};
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (buf[dev] == nullptr) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(cur_stream(), &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    int* p = nullptr;
    if (hipMalloc(&p, 4096 * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, 4096 * sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    buf[dev] = p;
  }
  return buf[dev];
}

// q2d: [B, >=Hq*D] rows (e.g. the q columns of fused qkv rows). Returns o [B, Hq*D].
at::Tensor decode_attn(const at::Tensor& q2d, const at::Tensor& kc, const at::Tensor& vc,
                       const at::Tensor& slots, const at::Tensor& lengths, int64_t Hq, double scale) {
  check_bf16_cuda(q2d, "q");
  TORCH_CHECK(q2d.dim() == 2 && q2d.stride(1) == 1, "decode_attn: q must be 2-D row-major");
  const int64_t B = q2d.size(0), Hkv = kc.size(1), D = kc.size(3), Lmax = kc.size(2);
  check_cache(kc, vc, Hkv, D);
  TORCH_CHECK(q2d.size(1) >= Hq * D && Hq % Hkv == 0 && Hq / Hkv <= 8, "decode_attn: q heads");
  check_rows_i32(slots, B, "slots");
  check_rows_i32(lengths, B, "lengths");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q2d.device());
  static const int splits_env = [] {
    const char* v = std::getenv("KFAMD_DECODE_SPLITS");   // tuning override (tools/bench_decode_splits.py)
    return v ? std::atoi(v) : 0;
  }();
  auto f32 = q2d.options().dtype(at::kFloat);
  // small batches, opt-in (KFAMD_DECODE_FUSED=1): split-K + merge in one launch
  // (kf_decode_attn_fused), whose arrival tickets live in a per-device zeroed buffer that every
  // launch leaves zero (allocated on first use, outside any graph capture).  Measured slower than
  // the two kernels on MI355X -- 13.6 vs 10.1 us at batch 1 / 1024 keys, decode step 3.14 vs
  // 3.06 ms (profiles/serve_decode_attn_fused_ab_r4.txt): the last arriver's merge is a serial
  // tail inside the launch, the combine kernel's boundary costs less
  const char* fv = std::getenv("KFAMD_DECODE_FUSED");      // read per call (tests compare both forms)
  const bool fused_on = fv && fv[0] == '1';
  if (fused_on && B <= 4 && B * Hkv <= 4096 && Hq / Hkv <= 8) {
    int* tickets = decode_tickets(q2d.device().index());
    if (tickets != nullptr) {
      const int splits1 = kf_decode_splits1((int)B, (int)Hkv, (int)Lmax);
      const int64_t slots_per = B * Hkv * 64;                        // MAX_SPLITS1 = 64
      auto po = at::empty({slots_per * (Hq / Hkv) * D}, f32);
      auto pml = at::empty({slots_per * (Hq / Hkv) * 2}, f32);
      auto out = at::empty({B, Hq * D}, q2d.options());
      check_rc(kf_decode_attn_fused(q2d.data_ptr(), q2d.stride(0), kc.data_ptr(), vc.data_ptr(),
                                    slots.data_ptr<int>(), lengths.data_ptr<int>(), out.data_ptr(), out.stride(0),
                                    po.data_ptr<float>(), pml.data_ptr<float>(), tickets, (int)B, (int)Hq, (int)Hkv,
                                    (int)D, (int)Lmax, splits1, (float)scale, cur_stream()),
               "decode_attn_fused");
      return out;
    }
  }
  const int splits = splits_env > 0 ? splits_env : kf_decode_splits((int)B, (int)Hkv, (int)Lmax);
  auto po = at::empty({B * Hq * splits * D}, f32);
  auto pml = at::empty({B * Hq * splits * 2}, f32);
  auto out = at::empty({B, Hq * D}, q2d.options());
  check_rc(kf_decode_attn(q2d.data_ptr(), q2d.stride(0), kc.data_ptr(), vc.data_ptr(), slots.data_ptr<int>(),
                          lengths.data_ptr<int>(), out.data_ptr(), out.stride(0), po.data_ptr<float>(),
                          pml.data_ptr<float>(), (int)B, (int)Hq, (int)Hkv, (int)D, (int)Lmax, splits,
                          (float)scale, cur_stream()),
           "decode_attn");
  return out;
}

// Append one token per row (K/V columns of fused qkv rows) at pos[b] of slot slots[b].
void kv_append_(const at::Tensor& qkv, int64_t Hq, const at::Tensor& slots, const at::Tensor& pos,
                at::Tensor& kc, at::Tensor& vc) {
  check_bf16_cuda(qkv, "qkv");
  const int64_t B = qkv.size(0), Hkv = kc.size(1), D = kc.size(3);
  check_cache(kc, vc, Hkv, D);
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(1) >= (Hq + 2 * Hkv) * D, "kv_append: qkv");
  check_rows_i32(slots, B, "slots");
  check_rows_i32(pos, B, "pos");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  check_rc(kf_kv_append(qkv.data_ptr(), qkv.stride(0), (int)B, (int)Hq, (int)Hkv, (int)D, slots.data_ptr<int>(),
                        pos.data_ptr<int>(), kc.data_ptr(), vc.data_ptr(), (int)kc.size(2), cur_stream()),
           "kv_append");
}

// Decode prologue: RoPE on q/k heads of each fused qkv row at pos[b] + append k, v to the cache.
void rope_append_(at::Tensor& qkv, int64_t Hq, const at::Tensor& cos_t, const at::Tensor& sin_t,
                  const at::Tensor& slots, const at::Tensor& pos, at::Tensor& kc, at::Tensor& vc) {
  check_bf16_cuda(qkv, "qkv");
  const int64_t B = qkv.size(0), Hkv = kc.size(1), D = kc.size(3);
  check_cache(kc, vc, Hkv, D);
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(1) >= (Hq + 2 * Hkv) * D, "rope_append: qkv");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                  sin_t.is_contiguous() && cos_t.size(-1) == D / 2 && cos_t.size(0) >= kc.size(2),
              "rope_append: cos/sin tables must be fp32 [>=Lmax, D/2]");
  check_rows_i32(slots, B, "slots");
  check_rows_i32(pos, B, "pos");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  check_rc(kf_rope_append(qkv.data_ptr(), qkv.stride(0), (int)B, (int)Hq, (int)Hkv, (int)D, cos_t.data_ptr<float>(),
                          sin_t.data_ptr<float>(), slots.data_ptr<int>(), pos.data_ptr<int>(), kc.data_ptr(),
                          vc.data_ptr(), (int)kc.size(2), cur_stream()),
           "rope_append");
}

// rope_append_ on the qkv projection's fp32 K-split partials [S, B, (Hq + 2 Hkv) * D] (bgemm_parts):
// the reduce launch folded in.  Returns the rotated bf16 qkv rows.
at::Tensor rope_append_parts(const at::Tensor& part, int64_t Hq, const at::Tensor& cos_t, const at::Tensor& sin_t,
                             const at::Tensor& slots, const at::Tensor& pos, at::Tensor& kc, at::Tensor& vc) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3,
              "rope_append_parts: fp32 [S, B, N] partials");
  const int64_t B = part.size(1), Hkv = kc.size(1), D = kc.size(3);
  check_cache(kc, vc, Hkv, D);
  TORCH_CHECK(part.size(2) == (Hq + 2 * Hkv) * D, "rope_append_parts: row width");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                  sin_t.is_contiguous() && cos_t.size(-1) == D / 2 && cos_t.size(0) >= kc.size(2),
              "rope_append_parts: cos/sin tables must be fp32 [>=Lmax, D/2]");
  check_rows_i32(slots, B, "slots");
  check_rows_i32(pos, B, "pos");
  c10::hip::HIPGuardMasqueradingAsCUDA g(part.device());
  auto qkv = at::empty({B, part.size(2)}, kc.options());
  check_rc(kf_rope_append_parts(part.data_ptr<float>(), (int)part.size(0), qkv.data_ptr(), (int)B, (int)Hq, (int)Hkv,
                                (int)D, cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), slots.data_ptr<int>(),
                                pos.data_ptr<int>(), kc.data_ptr(), vc.data_ptr(), (int)kc.size(2), cur_stream()),
           "rope_append_parts");
  return qkv;
}

// Decode qkv projection, fused: h = x (+ res); qkv = (rmsnorm(h) * nw) . w^T; RoPE at pos[b] on
// the q/k heads; rotated k and v appended to the cache at (slots[b], pos[b]).  Returns (qkv, h);
// == skinny_gemm_norm + rope_append_ bit for bit.  1 <= B <= 4 rows, head dim 128.
std::tuple<at::Tensor, at::Tensor> gemv_norm_rope(const at::Tensor& x, const std::optional<at::Tensor>& res,
                                                  const at::Tensor& nw, double eps, const at::Tensor& w, int64_t Hq,
                                                  const at::Tensor& cos_t, const at::Tensor& sin_t,
                                                  const at::Tensor& slots, const at::Tensor& pos, at::Tensor& kc,
                                                  at::Tensor& vc) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(nw, "norm weight");
  const int64_t B = x.size(0), K = x.size(1), N = w.size(0), Hkv = kc.size(1), D = kc.size(3);
  check_cache(kc, vc, Hkv, D);
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && w.dim() == 2 && w.is_contiguous() && w.size(1) == K &&
                  nw.numel() == K && nw.is_contiguous(), "gemv_norm_rope: operands");
  TORCH_CHECK(D == 128 && N == (Hq + 2 * Hkv) * D, "gemv_norm_rope: w must be the fused [q; k; v] projection, D = 128");
  TORCH_CHECK(B >= 1 && B <= 4 && B * K * 2 <= 64 * 1024 && K % 8 == 0, "gemv_norm_rope: 1 <= B <= 4, B*K*2 <= 64 KB");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                  sin_t.is_contiguous() && cos_t.size(-1) == D / 2 && cos_t.size(0) >= kc.size(2),
              "gemv_norm_rope: cos/sin tables must be fp32 [>=Lmax, D/2]");
  check_rows_i32(slots, B, "slots");
  check_rows_i32(pos, B, "pos");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor h = x;
  const void* rp = nullptr;
  if (res.has_value()) {
    check_bf16_cuda(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous(), "gemv_norm_rope: res shape");
    h = at::empty_like(x);
    rp = res->data_ptr();
  }
  auto y = at::empty({B, N}, x.options());
  check_rc(kf_gemv_norm_rope(x.data_ptr(), x.stride(0), (int)B, rp, nw.data_ptr(), (float)eps,
                             rp ? h.data_ptr() : nullptr, h.stride(0), w.data_ptr(), (int)N, (int)K, y.data_ptr(),
                             y.stride(0), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), slots.data_ptr<int>(),
                             pos.data_ptr<int>(), kc.data_ptr(), vc.data_ptr(), (int)Hq, (int)Hkv, (int)kc.size(2),
                             cur_stream()),
           "gemv_norm_rope");
  return {y, h};
}

// Prefill: rows [0, S) of one sequence's fused qkv -> positions [0, S) of `slot`.
void kv_fill_(const at::Tensor& qkv, int64_t S, int64_t Hq, int64_t slot, at::Tensor& kc, at::Tensor& vc) {
  check_bf16_cuda(qkv, "qkv");
  const int64_t Hkv = kc.size(1), D = kc.size(3);
  check_cache(kc, vc, Hkv, D);
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(0) >= S && qkv.size(1) >= (Hq + 2 * Hkv) * D,
              "kv_fill: qkv");
  TORCH_CHECK(slot >= 0 && slot < kc.size(0) && S <= kc.size(2), "kv_fill: slot/length out of range");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  check_rc(kf_kv_fill(qkv.data_ptr(), qkv.stride(0), (int)S, (int)Hq, (int)Hkv, (int)D, (int)slot, kc.data_ptr(),
                      vc.data_ptr(), (int)kc.size(2), cur_stream()),
           "kv_fill");
}

// 1-2 decode rows (and 3-4 rows on the large matrices) stream W faster through the VALU GEMV
// (ops/csrc/gemv.hip, 1 KB contiguous per row and instruction) than through the MFMA skinny
// kernel: tools/kbench/gemv_bench.hip, e.g. gate/up 59 -> 41 us, LM head 199 -> 154 us at M = 1.
static bool use_gemv(int64_t M, int64_t Nw, int64_t K) {
  if (M > 4) return false;
  const bool mfma_fits = K % 256 == 0 && Nw % 16 == 0;   // else the GEMV is the only kernel for it
  return M <= 2 || !mfma_fits || Nw * K > (int64_t)20 * 1024 * 1024;
}

// Decode GEMM: x [M<=64, K] (unit inner stride) . w[N, K]^T -> [M, N]; swiglu: w = [gate; up]
// (2F rows) -> silu(x.gate^T) * (x.up^T), [M, F].
at::Tensor skinny_gemm(const at::Tensor& x, const at::Tensor& w, bool swiglu) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.dim() == 2 && w.is_contiguous(), "skinny_gemm: 2-D operands");
  const int64_t M = x.size(0), K = x.size(1), Nw = w.size(0);
  TORCH_CHECK(w.size(1) == K, "skinny_gemm: K mismatch");
  TORCH_CHECK(!swiglu || Nw % 2 == 0, "skinny_gemm: swiglu needs an even number of rows");
  const int64_t N = swiglu ? Nw / 2 : Nw;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto y = at::empty({M, N}, x.options());
  if (M >= 1 && use_gemv(M, Nw, K) &&
      kf_gemv(x.data_ptr(), x.stride(0), (int)M, nullptr, nullptr, 0.f, nullptr, 0, w.data_ptr(), (int)N, (int)K,
              y.data_ptr(), y.stride(0), swiglu ? 1 : 0, (int)N, cur_stream()) == 0)
    return y;
  TORCH_CHECK(M >= 1 && M <= 64 && K % 256 == 0, "skinny_gemm: needs 1 <= M <= 64, K % 256 == 0");
  TORCH_CHECK(N % 16 == 0, "skinny_gemm: N % 16 != 0");
  check_rc(kf_skinny_gemm(x.data_ptr(), x.stride(0), (int)M, w.data_ptr(), (int)N, (int)K, y.data_ptr(), y.stride(0),
                          swiglu ? 1 : 0, (int)N, cur_stream()),
           "skinny_gemm");
  return y;
}

// Batched-decode GEMM (17..256 rows): y = x . w^T, or silu(x . gate^T) * (x . up^T) with
// w = [gate; up] when swiglu.  splits = 0 picks the K split (kf_bgemm_splits); the fp32
// partials of a split launch live in a workspace from the caching allocator.
at::Tensor bgemm(const at::Tensor& x, const at::Tensor& w, bool swiglu, int64_t splits) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.dim() == 2 && w.is_contiguous(), "bgemm: 2-D operands");
  const int64_t M = x.size(0), K = x.size(1), Nw = w.size(0);
  TORCH_CHECK(w.size(1) == K, "bgemm: K mismatch");
  TORCH_CHECK(M >= 1 && M <= 256 && K % 256 == 0 && Nw % 64 == 0, "bgemm: needs 1 <= M <= 256, K % 256 == 0, N % 64 == 0");
  const int64_t N = swiglu ? Nw / 2 : Nw;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto y = at::empty({M, N}, x.options());
  const int S = splits > 0 ? (int)splits : kf_bgemm_splits((int)M, (int)Nw, (int)K);
  at::Tensor part;
  if (S > 1) part = at::empty({(int64_t)S * M * Nw}, x.options().dtype(at::kFloat));
  check_rc(kf_bgemm(x.data_ptr(), x.stride(0), (int)M, w.data_ptr(), (int)Nw, (int)K, y.data_ptr(), y.stride(0),
                    swiglu ? 1 : 0, (int)N, S, S > 1 ? part.data_ptr<float>() : nullptr, cur_stream()),
           "bgemm");
  return y;
}

// bgemm whose K-split partials are left for the consumer: fp32 [S, M, N] when the automatic split
// is S > 1 (no reduce launch; rmsnorm_fwd_parts sums them), else the bf16 [M, N] product
at::Tensor bgemm_parts(const at::Tensor& x, const at::Tensor& w) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.dim() == 2 && w.is_contiguous(), "bgemm_parts: 2-D operands");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "bgemm_parts: K mismatch");
  TORCH_CHECK(M >= 1 && M <= 256 && K % 256 == 0 && N % 64 == 0, "bgemm_parts: needs 1 <= M <= 256, K % 256 == 0, N % 64 == 0");
  const int S = kf_bgemm_splits((int)M, (int)N, (int)K);
  if (S == 1) return bgemm(x, w, false, 1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto part = at::empty({(int64_t)S, M, N}, x.options().dtype(at::kFloat));
  check_rc(kf_bgemm(x.data_ptr(), x.stride(0), (int)M, w.data_ptr(), (int)N, (int)K, nullptr, N, 0, (int)N, S,
                    part.data_ptr<float>(), cur_stream()),
           "bgemm_parts");
  return part;
}

// Decode GEMM with the residual-add + RMSNorm fused in as a prologue:
//   h = x (+ res);  y = (rmsnorm(h) * nw) . w^T  [SwiGLU epilogue when swiglu].
// Returns (y, h); h aliases x when res is None.  Needs M <= 8 and M * K <= 32768.
std::tuple<at::Tensor, at::Tensor> skinny_gemm_norm(const at::Tensor& x, const std::optional<at::Tensor>& res,
                                                    const at::Tensor& nw, double eps, const at::Tensor& w,
                                                    bool swiglu) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(nw, "norm weight");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && w.dim() == 2 && w.is_contiguous(), "skinny_gemm_norm: 2-D operands");
  const int64_t M = x.size(0), K = x.size(1), Nw = w.size(0);
  TORCH_CHECK(w.size(1) == K && nw.numel() == K && nw.is_contiguous(), "skinny_gemm_norm: K mismatch");
  TORCH_CHECK(M >= 1 && M <= 8 && (M <= 4 ? 4 : 8) * K <= 32768 && K % 256 == 0,
              "skinny_gemm_norm: needs M <= 8, K % 256 == 0 and K <= 8192 (M <= 4) / 4096 (M <= 8)");
  TORCH_CHECK(!swiglu || Nw % 2 == 0, "skinny_gemm_norm: swiglu needs an even number of rows");
  const int64_t N = swiglu ? Nw / 2 : Nw;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor h = x;
  const void* rp = nullptr;
  if (res.has_value()) {
    check_bf16_cuda(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous(), "skinny_gemm_norm: res shape");
    h = at::empty_like(x);
    rp = res->data_ptr();
  }
  auto y = at::empty({M, N}, x.options());
  if (use_gemv(M, Nw, K) &&
      kf_gemv(x.data_ptr(), x.stride(0), (int)M, rp, nw.data_ptr(), (float)eps, rp ? h.data_ptr() : nullptr,
              h.stride(0), w.data_ptr(), (int)N, (int)K, y.data_ptr(), y.stride(0), swiglu ? 1 : 0, (int)N,
              cur_stream()) == 0)
    return {y, h};
  TORCH_CHECK(N % 16 == 0, "skinny_gemm_norm: N % 16 != 0");
  check_rc(kf_skinny_gemm_norm(x.data_ptr(), x.stride(0), (int)M, rp, nw.data_ptr(), (float)eps,
                               rp ? h.data_ptr() : nullptr, h.stride(0), w.data_ptr(), (int)N, (int)K, y.data_ptr(),
                               y.stride(0), swiglu ? 1 : 0, (int)N, cur_stream()),
           "skinny_gemm_norm");
  return {y, h};
}

// out = in^T for a bf16 [R, C] matrix (R, C % 64 == 0; unit inner stride)
at::Tensor transpose_bf16(const at::Tensor& x) {
  check_bf16_cuda(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(0) % 64 == 0 && x.size(1) % 64 == 0,
              "transpose_bf16: 2-D, unit inner stride, dims % 64 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto out = at::empty({x.size(1), x.size(0)}, x.options());
  check_rc(kf_transpose_bf16(x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0), (int)x.size(0), (int)x.size(1),
                             cur_stream()),
           "transpose_bf16");
  return out;
}

// ---- one-shot IPC all-reduce (ops/csrc/custom_ar.hip). Device pointers travel as int64.
std::tuple<int64_t, at::Tensor> car_alloc(int64_t slot_bytes) {
  void* p = nullptr;
  auto h = at::empty({64}, at::TensorOptions().dtype(at::kByte));
  TORCH_CHECK(kf_car_alloc(slot_bytes, &p, h.data_ptr()) == 0, "car_alloc: uncached IPC allocation failed");
  return {reinterpret_cast<int64_t>(p), h};
}

int64_t car_open(const at::Tensor& handle) {
  TORCH_CHECK(handle.numel() == 64 && handle.scalar_type() == at::kByte && !handle.is_cuda(), "car_open: 64-byte handle");
  void* p = nullptr;
  TORCH_CHECK(kf_car_open(handle.contiguous().data_ptr(), &p) == 0, "car_open: hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}

void car_close(int64_t p) { kf_car_close(reinterpret_cast<void*>(p)); }
void car_free(int64_t p) { kf_car_free(reinterpret_cast<void*>(p)); }

// in place, like dist.all_reduce (the engine's TP code relies on all-reduce being in place)
void car_allreduce_(const std::vector<int64_t>& ptrs, int64_t rank, at::Tensor& x, int64_t slot_bytes, int64_t blocks,
                    double timeout_s) {
  check_bf16_cuda(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 8 == 0 && 2 * x.numel() <= slot_bytes,
              "car_allreduce: contiguous bf16 with numel % 8 == 0 that fits the slot");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  std::vector<void*> pv;
  for (auto v : ptrs) pv.push_back(reinterpret_cast<void*>(v));
  check_rc(kf_car_allreduce(pv.data(), (int)pv.size(), (int)rank, x.data_ptr(), x.data_ptr(), x.numel(), slot_bytes,
                            (int)blocks, timeout_s, cur_stream()),
           "car_allreduce");
}

int64_t car_error(int64_t own) { return kf_car_error(reinterpret_cast<void*>(own), cur_stream()); }

// ---- two-shot reduce-scatter / all-gather / all-reduce (ops/csrc/custom_ar.hip, namespace ts);
// open / close / free are the one-shot ones (plain IPC handles).
std::tuple<int64_t, at::Tensor> ts_alloc(int64_t slot_bytes, int64_t world) {
  void* p = nullptr;
  auto h = at::empty({64}, at::TensorOptions().dtype(at::kByte));
  TORCH_CHECK(kf_ts_alloc(slot_bytes, (int)world, &p, h.data_ptr()) == 0, "ts_alloc: uncached IPC allocation failed");
  return {reinterpret_cast<int64_t>(p), h};
}

// mode 0: all-reduce x in place (out is x); 1: reduce-scatter x[n] -> out[n / world];
// 2: all-gather x[n / world] -> out[n].  Runs on the current stream.
void ts_run(int64_t mode, const std::vector<int64_t>& ptrs, int64_t rank, const at::Tensor& x, at::Tensor& out,
            int64_t slot_bytes, int64_t blocks, double timeout_s) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(out, "out");
  const long w = (long)ptrs.size();
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous(), "ts_run: contiguous tensors");
  const long n = mode == 2 ? x.numel() * w : x.numel();
  const long n_out = mode == 1 ? n / w : n;
  TORCH_CHECK(out.numel() == n_out, "ts_run: out has ", out.numel(), " elements, expected ", n_out);
  TORCH_CHECK(n % (8 * w) == 0 && 2 * n <= slot_bytes, "ts_run: numel % (8 world) == 0 that fits the slot");
  TORCH_CHECK(mode != 0 || x.data_ptr() == out.data_ptr(), "ts_run: all-reduce is in place");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  std::vector<void*> pv;
  for (auto v : ptrs) pv.push_back(reinterpret_cast<void*>(v));
  check_rc(kf_ts_run((int)mode, pv.data(), (int)w, (int)rank, x.data_ptr(), out.data_ptr(), n, slot_bytes,
                     (int)blocks, timeout_s, cur_stream()),
           "ts_run");
}

int64_t ts_error(int64_t own) { return kf_ts_error(reinterpret_cast<void*>(own), cur_stream()); }
// queue a copy of the error word into `host` (a pinned int32 CPU tensor) on the current stream
void ts_error_async(int64_t own, at::Tensor& host) {
  TORCH_CHECK(!host.is_cuda() && host.scalar_type() == at::kInt && host.numel() >= 1 && host.is_pinned(),
              "ts_error_async: pinned int32 host tensor");
  check_rc(kf_ts_error_async(reinterpret_cast<void*>(own), host.data_ptr<int>(), cur_stream()), "ts_error_async");
}

// Weight-gradient GEMM: C[M, N] (+)= a^T . b with a = [K, M], b = [K, N] (row stride may
// exceed the width: views into fused activations); C may be a view into the flat grad buffer.
bool gemm_tn_ok(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c) {
  if (!a.is_cuda() || a.scalar_type() != at::kBFloat16 || b.scalar_type() != at::kBFloat16 ||
      c.scalar_type() != at::kBFloat16)
    return false;
  if (a.dim() != 2 || b.dim() != 2 || c.dim() != 2 || a.stride(1) != 1 || b.stride(1) != 1 || c.stride(1) != 1)
    return false;
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  return b.size(0) == K && c.size(0) == M && c.size(1) == N && M % 256 == 0 && N % 256 == 0 && K % 128 == 0 &&
         a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && c.stride(0) % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(a.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(b.data_ptr()) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(c.data_ptr()) & 7) == 0 && K < (1l << 31) && M < (1l << 31);
}

void gemm_tn_(const at::Tensor& a, const at::Tensor& b, at::Tensor& c, bool accumulate) {
  TORCH_CHECK(gemm_tn_ok(a, b, c), "gemm_tn: unsupported shapes/strides (needs M, N % 256, K % 128, bf16)");
  c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  check_rc(kf_gemm_tn(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(), c.stride(0), (int)a.size(1),
                      (int)b.size(1), (int)a.size(0), accumulate ? 1 : 0, cur_stream()),
           "gemm_tn");
}

// Two weight-gradient products over the same K in one launch (their tiles share one grid).
void gemm_tn2_(const at::Tensor& a0, const at::Tensor& b0, at::Tensor& c0, const at::Tensor& a1, const at::Tensor& b1,
               at::Tensor& c1, bool accumulate) {
  TORCH_CHECK(gemm_tn_ok(a0, b0, c0) && gemm_tn_ok(a1, b1, c1) && a0.size(0) == a1.size(0),
              "gemm_tn2: unsupported shapes/strides");
  c10::hip::HIPGuardMasqueradingAsCUDA g(a0.device());
  check_rc(kf_gemm_tn2(a0.data_ptr(), a0.stride(0), b0.data_ptr(), b0.stride(0), c0.data_ptr(), c0.stride(0),
                       (int)a0.size(1), (int)b0.size(1), a1.data_ptr(), a1.stride(0), b1.data_ptr(), b1.stride(0),
                       c1.data_ptr(), c1.stride(0), (int)a1.size(1), (int)b1.size(1), (int)a0.size(0),
                       accumulate ? 1 : 0, cur_stream()),
           "gemm_tn2");
}

// K7 embedding: tokens int64 [T]; E [vl, H] (this rank's vocab shard starting at vstart).
at::Tensor embed_fwd(const at::Tensor& tok, const at::Tensor& E, int64_t vstart) {
  check_bf16_cuda(E, "E");
  TORCH_CHECK(tok.is_cuda() && tok.scalar_type() == at::kLong && tok.is_contiguous(), "embed: tokens int64");
  TORCH_CHECK(E.dim() == 2 && E.is_contiguous() && E.size(1) % 8 == 0, "embed: E [V, H], H % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(E.device());
  auto out = at::empty({tok.numel(), E.size(1)}, E.options());
  check_rc(kf_embed_fwd(tok.data_ptr<int64_t>(), E.data_ptr(), out.data_ptr(), (int)tok.numel(), (int)E.size(1),
                        vstart, E.size(0), cur_stream()),
           "embed_fwd");
  return out;
}

// dE (bf16 [vl, H], e.g. a view into the flat gradient buffer) <- scatter-add of g [T, H] by token.
void embed_bwd_(const at::Tensor& tok, const at::Tensor& g, at::Tensor& dE, int64_t vstart, bool accumulate) {
  check_bf16_cuda(g, "g");
  check_bf16_cuda(dE, "dE");
  TORCH_CHECK(tok.is_cuda() && tok.scalar_type() == at::kLong, "embed_bwd: tokens int64");
  TORCH_CHECK(g.dim() == 2 && g.is_contiguous() && g.size(0) == tok.numel() && dE.dim() == 2 && dE.is_contiguous() &&
                  dE.size(1) == g.size(1) && g.size(1) % 8 == 0, "embed_bwd: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  if (!accumulate) dE.zero_();
  auto sorted = at::sort(tok.reshape({-1}));
  auto keys = std::get<0>(sorted).contiguous();
  auto perm = std::get<1>(sorted).contiguous();
  check_rc(kf_embed_bwd(keys.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), g.data_ptr(), dE.data_ptr(),
                        (int)tok.numel(), (int)g.size(1), vstart, dE.size(0), accumulate ? 1 : 0, cur_stream()),
           "embed_bwd");
}

}  // namespace

// ---------------- fp32 DP gradient reduction / accumulation (grad_reduce.hip) ----------------
// out (+)= sum of the R equal bf16 shards of `recv` (fp32, rank order)
void shard_sum_(const at::Tensor& recv, int64_t R, at::Tensor out, bool accumulate) {
  check_bf16_cuda(recv, "recv");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && recv.is_contiguous(),
              "shard_sum: out must be contiguous fp32 on the GPU");
  TORCH_CHECK(R >= 1 && recv.numel() == R * out.numel() && out.numel() % 8 == 0, "shard_sum: sizes");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(recv.device());
  check_rc(kf_shard_sum(recv.data_ptr(), (int)R, (size_t)out.numel(), out.data_ptr<float>(), accumulate ? 1 : 0,
                        cur_stream()),
           "shard_sum");
}

// mode 0: main = g; 1: main += g; 2: g = bf16(main + g)
void grad_accum_(at::Tensor main_, at::Tensor g, int64_t mode) {
  check_bf16_cuda(g, "g");
  TORCH_CHECK(main_.is_cuda() && main_.scalar_type() == at::kFloat && main_.is_contiguous() && g.is_contiguous(),
              "grad_accum: main must be contiguous fp32 on the GPU");
  TORCH_CHECK(main_.numel() == g.numel() && g.numel() % 8 == 0, "grad_accum: sizes");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(g.device());
  check_rc(kf_grad_accum(main_.data_ptr<float>(), g.data_ptr(), (size_t)g.numel(), (int)mode, cur_stream()),
           "grad_accum");
}

TORCH_LIBRARY(kfamd, m) {
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_fwd_parts", &rmsnorm_fwd_parts);
  m.def("bgemm_parts", &bgemm_parts);
  m.def("rope_append_parts", &rope_append_parts);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("rope_", &rope_);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("adamw_", &adamw_);
  m.def("sumsq", &sumsq);
  m.def("shard_sum_(Tensor recv, int R, Tensor(a!) out, bool accumulate) -> ()", &shard_sum_);
  m.def("grad_accum_(Tensor(a!) main, Tensor(b!) g, int mode) -> ()", &grad_accum_);
  m.def("cross_entropy_", &cross_entropy_);
  m.def("flash_fwd", &flash_fwd);
  m.def("flash_bwd", &flash_bwd);
  m.def("decode_attn", &decode_attn);
  m.def("skinny_gemm", &skinny_gemm);
  m.def("bgemm(Tensor x, Tensor w, bool swiglu, int splits) -> Tensor", &bgemm);
  m.def("skinny_gemm_norm", &skinny_gemm_norm);
  m.def("transpose_bf16", &transpose_bf16);
  m.def("car_alloc", &car_alloc);
  m.def("car_open", &car_open);
  m.def("car_close", &car_close);
  m.def("car_free", &car_free);
  m.def("car_allreduce_(int[] ptrs, int rank, Tensor(a!) x, int slot_bytes, int blocks, float timeout_s) -> ()",
        &car_allreduce_);
  m.def("car_error", &car_error);
  m.def("ts_alloc", &ts_alloc);
  m.def("ts_run(int mode, int[] ptrs, int rank, Tensor x, Tensor(a!) out, int slot_bytes, int blocks, float timeout_s) -> ()",
        &ts_run);
  m.def("ts_error", &ts_error);
  m.def("ts_error_async(int own, Tensor(a!) host) -> ()", &ts_error_async);
  m.def("gemm_tn_ok", &gemm_tn_ok);
  m.def("gemm_tn_(Tensor a, Tensor b, Tensor(a!) c, bool accumulate) -> ()", &gemm_tn_);
  m.def("gemm_tn2_(Tensor a0, Tensor b0, Tensor(a!) c0, Tensor a1, Tensor b1, Tensor(b!) c1, bool accumulate) -> ()",
        &gemm_tn2_);
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd_(Tensor tok, Tensor g, Tensor(a!) dE, int vstart, bool accumulate) -> ()", &embed_bwd_);
  m.def("rope_append_(Tensor(a!) qkv, int Hq, Tensor cos, Tensor sin, Tensor slots, Tensor pos, Tensor(b!) kc, "
        "Tensor(c!) vc) -> ()", &rope_append_);
  m.def("gemv_norm_rope(Tensor x, Tensor? res, Tensor nw, float eps, Tensor w, int Hq, Tensor cos, Tensor sin, "
        "Tensor slots, Tensor pos, Tensor(a!) kc, Tensor(b!) vc) -> (Tensor, Tensor)", &gemv_norm_rope);
  m.def("kv_append_(Tensor qkv, int Hq, Tensor slots, Tensor pos, Tensor(a!) kc, Tensor(b!) vc) -> ()", &kv_append_);
  m.def("kv_fill_(Tensor qkv, int S, int Hq, int slot, Tensor(a!) kc, Tensor(b!) vc) -> ()", &kv_fill_);
}
