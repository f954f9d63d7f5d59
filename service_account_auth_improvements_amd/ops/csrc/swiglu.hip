// K4: SwiGLU on the fused gate/up projection.
//
// gu = x @ [Wg; Wu]^T is one [T, 2F] bf16 buffer (gate columns [0,F), up columns [F,2F)).
//   fwd: out = silu(g) * u                                  -> [T, F]
//   bwd: dg  = dout * u * sig(g) * (1 + g * (1 - sig(g)))
//        du  = dout * silu(g)                               -> [T, 2F] (same layout as gu)
// 16-byte vectors (8 x bf16) per lane; purely HBM-bound.
#include "common.h"

using namespace kf;

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu,
                                                         bf16_t* __restrict__ out, int rows, int F) {
  const int vpr = F >> 3;
  const int total = rows * vpr;
  for (int it = blockIdx.x * blockDim.x + threadIdx.x; it < total; it += gridDim.x * blockDim.x) {
    const int r = it / vpr, c = (it - r * vpr) * 8;
    const bf16_t* pg = gu + (size_t)r * 2 * F + c;
    float g[8], u[8], o[8];
    unpack8(ld16(pg), g);
    unpack8(ld16(pg + F), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] * sigmoidf_(g[j]) * u[j];
    st16(out + (size_t)r * F + c, pack8(o));
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ gu,
                                                         const bf16_t* __restrict__ dout,
                                                         bf16_t* __restrict__ dgu, int rows, int F) {
  const int vpr = F >> 3;
  const int total = rows * vpr;
  for (int it = blockIdx.x * blockDim.x + threadIdx.x; it < total; it += gridDim.x * blockDim.x) {
    const int r = it / vpr, c = (it - r * vpr) * 8;
    const size_t gbase = (size_t)r * 2 * F + c;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(ld16(gu + gbase), g);
    unpack8(ld16(gu + gbase + F), u);
    unpack8(ld16(dout + (size_t)r * F + c), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigmoidf_(g[j]);
      const float silu = g[j] * s;
      du[j] = d[j] * silu;
      dg[j] = d[j] * u[j] * s * (1.f + g[j] * (1.f - s));
    }
    st16(dgu + gbase, pack8(dg));
    st16(dgu + gbase + F, pack8(du));
  }
}

// Row-tiled kernels (default): grid (ceil(F/8/256), rows), one 16-byte vector per lane, no
// index division and no grid-stride loop. Measured 4-6 % faster than the grid-stride loop at
// T=16384, F=14336 (profiles/swiglu_unroll_ab.md). KFAMD_SWIGLU_2D=0 selects the grid-stride
// loop, which also serves rows > 65535.
__global__ __launch_bounds__(256) void swiglu_fwd_2d_kernel(const bf16_t* __restrict__ gu,
                                                            bf16_t* __restrict__ out, int F) {
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (c >= F) return;
  const size_t r = blockIdx.y;
  const bf16_t* pg = gu + r * 2 * F + c;
  float g[8], u[8], o[8];
  unpack8(ld16(pg), g);
  unpack8(ld16(pg + F), u);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = g[j] * sigmoidf_(g[j]) * u[j];
  st16(out + r * F + c, pack8(o));
}

__global__ __launch_bounds__(256) void swiglu_bwd_2d_kernel(const bf16_t* __restrict__ gu,
                                                            const bf16_t* __restrict__ dout,
                                                            bf16_t* __restrict__ dgu, int F) {
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (c >= F) return;
  const size_t r = blockIdx.y;
  const size_t gbase = r * 2 * F + c;
  float g[8], u[8], d[8], dg[8], du[8];
  unpack8(ld16(gu + gbase), g);
  unpack8(ld16(gu + gbase + F), u);
  unpack8(ld16(dout + r * F + c), d);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float s = sigmoidf_(g[j]);
    du[j] = d[j] * g[j] * s;
    dg[j] = d[j] * u[j] * s * (1.f + g[j] * (1.f - s));
  }
  st16(dgu + gbase, pack8(dg));
  st16(dgu + gbase + F, pack8(du));
}

static bool use_2d(int rows) {
  static const bool on = [] {
    const char* e = getenv("KFAMD_SWIGLU_2D");
    return !(e && atoi(e) == 0);
  }();
  return on && rows > 0 && rows <= 65535;
}

static int grid_for(long total) {
  long g = (total + 255) / 256;
  if (g > 16384) g = 16384;
  return g < 1 ? 1 : (int)g;
}

extern "C" {
int kf_swiglu_fwd(const void* gu, void* out, int rows, int F, hipStream_t s) {
  if (F % 8 || (long)rows * F / 8 >= (1L << 31)) return 1;
  if (use_2d(rows)) {
    swiglu_fwd_2d_kernel<<<dim3((F / 8 + 255) / 256, rows), 256, 0, s>>>((const bf16_t*)gu,
                                                                         (bf16_t*)out, F);
    return 0;
  }
  swiglu_fwd_kernel<<<grid_for((long)rows * F / 8), 256, 0, s>>>((const bf16_t*)gu, (bf16_t*)out,
                                                                  rows, F);
  return 0;
}
int kf_swiglu_bwd(const void* gu, const void* dout, void* dgu, int rows, int F, hipStream_t s) {
  if (F % 8 || (long)rows * F / 8 >= (1L << 31)) return 1;
  if (use_2d(rows)) {
    swiglu_bwd_2d_kernel<<<dim3((F / 8 + 255) / 256, rows), 256, 0, s>>>(
        (const bf16_t*)gu, (const bf16_t*)dout, (bf16_t*)dgu, F);
    return 0;
  }
  swiglu_bwd_kernel<<<grid_for((long)rows * F / 8), 256, 0, s>>>(
      (const bf16_t*)gu, (const bf16_t*)dout, (bf16_t*)dgu, rows, F);
  return 0;
}
}
