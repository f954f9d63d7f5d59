// K6: fused AdamW over FLAT parameter storage.
//
// MI355X-first layout: every trainable parameter of the model lives in ONE contiguous
// bf16 buffer (the compute copy), with matching flat fp32 master / exp_avg / exp_avg_sq
// buffers and a flat bf16 gradient buffer (whose slices are the DDP buckets). The whole
// optimizer step is therefore a single streaming kernel over N elements -- no
// multi-tensor-apply pointer lists -- moving 30 B/param (bf16 g, fp32 w/m/v r+w, bf16 w).
// For Llama-3-8B that is ~240 GB -> ~40 ms at the measured ~6 TB/s HBM roof.
//
// The gradient operand is bf16 (the flat gradient buffer, single-rank or bf16-reduced) or
// fp32 (the fp32 DP reduction's shard / the fp32 micro-batch accumulator, see
// grad_reduce.hip); the element loop is the same template.
//
// Gradient clipping never syncs with the host: the global sum of squares is produced on
// device (kf_sumsq, deterministic two-level reduce) and the AdamW kernel derives the clip
// coefficient from it.  Elements [0, n_decay) receive decoupled weight decay; the tail
// (norm gains, by the packer's ordering) does not.
#include "common.h"

using namespace kf;

template <bool G32>
__device__ __forceinline__ void load_grad8(const void* g, size_t e, float* gf) {
  if constexpr (G32) {
    const float* gp = reinterpret_cast<const float*>(g) + e;
    f32x4 a = ldf4(gp), b = ldf4(gp + 4);
    gf[0] = a[0]; gf[1] = a[1]; gf[2] = a[2]; gf[3] = a[3];
    gf[4] = b[0]; gf[5] = b[1]; gf[6] = b[2]; gf[7] = b[3];
  } else {
    unpack8(ld16(reinterpret_cast<const bf16_t*>(g) + e), gf);
  }
}

template <bool G32>
__global__ __launch_bounds__(256) void adamw_kernel(
    bf16_t* __restrict__ p, float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
    const void* __restrict__ g, size_t nvec, size_t n_decay, float lr, float b1, float b2,
    float eps, float wd, float inv_bc1, float inv_sqrt_bc2, float gscale,
    const float* __restrict__ sumsq, float max_norm) {
  float coef = gscale;
  if (sumsq != nullptr && max_norm > 0.f) {
    const float nrm = sqrtf(sumsq[0]) * gscale;
    coef = gscale * fminf(1.f, max_norm / (nrm + 1e-6f));
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t e = i * 8;
    float gf[8];
    load_grad8<G32>(g, e, gf);
    f32x4 w0 = ldf4(w + e), w1 = ldf4(w + e + 4);
    f32x4 m0 = ldf4(m + e), m1 = ldf4(m + e + 4);
    f32x4 v0 = ldf4(v + e), v1 = ldf4(v + e + 4);
    float wa[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
    float ma[8] = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
    float va[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    const float decay = (e < n_decay) ? (1.f - lr * wd) : 1.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gj = gf[j] * coef;
      ma[j] = b1 * ma[j] + (1.f - b1) * gj;
      va[j] = b2 * va[j] + (1.f - b2) * gj * gj;
      const float denom = sqrtf(va[j]) * inv_sqrt_bc2 + eps;
      wa[j] = wa[j] * decay - lr * (ma[j] * inv_bc1) / denom;
    }
    stf4(w + e, f32x4{wa[0], wa[1], wa[2], wa[3]}); stf4(w + e + 4, f32x4{wa[4], wa[5], wa[6], wa[7]});
    stf4(m + e, f32x4{ma[0], ma[1], ma[2], ma[3]}); stf4(m + e + 4, f32x4{ma[4], ma[5], ma[6], ma[7]});
    stf4(v + e, f32x4{va[0], va[1], va[2], va[3]}); stf4(v + e + 4, f32x4{va[4], va[5], va[6], va[7]});
    st16(p + e, pack8(wa));
  }
}

// Sum of squares of a bf16 or fp32 vector: per-block partials, then one block folds them
// in a fixed order (bitwise reproducible, no float atomics).
template <bool G32>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const void* __restrict__ g, size_t nvec,
                                                            float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec;
       i += (size_t)gridDim.x * blockDim.x) {
    float f[8];
    load_grad8<G32>(g, i * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[j] * f[j];
  }
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void sum_final_kernel(const float* __restrict__ part, int n,
                                                        float* __restrict__ out, int accumulate) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + s : s;
}

extern "C" {

int kf_adamw(void* p, float* w, float* m, float* v, const void* g, int g_fp32, size_t n, size_t n_decay,
             float lr, float b1, float b2, float eps, float wd, int step, float gscale,
             const float* sumsq, float max_norm, hipStream_t s) {
  if (n % 8) return 1;
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  const size_t nvec = n / 8;
  size_t grid = (nvec + 255) / 256;
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  if (g_fp32)
    adamw_kernel<true><<<(int)grid, 256, 0, s>>>((bf16_t*)p, w, m, v, g, nvec, n_decay, lr, b1, b2, eps, wd,
                                                 1.f / bc1, 1.f / sqrtf(bc2), gscale, sumsq, max_norm);
  else
    adamw_kernel<false><<<(int)grid, 256, 0, s>>>((bf16_t*)p, w, m, v, g, nvec, n_decay, lr, b1, b2, eps, wd,
                                                  1.f / bc1, 1.f / sqrtf(bc2), gscale, sumsq, max_norm);
  return 0;
}

// part must hold 2048 floats. out[0] = sum(g^2) (+ out[0] if accumulate).
int kf_sumsq(const void* g, int g_fp32, size_t n, float* part, float* out, int accumulate, hipStream_t s) {
  if (n % 8) return 1;
  const size_t nvec = n / 8;
  size_t grid = (nvec + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  if (g_fp32)
    sumsq_partial_kernel<true><<<(int)grid, 256, 0, s>>>(g, nvec, part);
  else
    sumsq_partial_kernel<false><<<(int)grid, 256, 0, s>>>(g, nvec, part);
  sum_final_kernel<<<1, 256, 0, s>>>(part, (int)grid, out, accumulate);
  return 0;
}
}
