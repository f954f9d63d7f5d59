// K1: fused residual-add + RMSNorm forward / backward for gfx950.
//
// Layout: rows of H bf16 values (the [T, hidden] activation of a Llama block).
// One wave64 owns one row: lane l holds 16-byte vectors l, l+64, ... of the row in
// registers, so the row is read from HBM exactly once in the forward (sum of
// squares + normalise from registers) and once in the backward.
//
//   fwd:  h = a (+ b);  r = rsqrt(mean(h^2) + eps);  y = h * r * w
//   bwd:  g = dy * w;   dh = r*g - h * r^3 * mean(g*h)  (+ dres);  dw = sum_rows dy*h*r
//
// dw is reduced in two steps (per-wave partial rows, then a column reduce kernel)
// so no float atomics are needed and the result is bitwise reproducible.
#include "common.h"

using namespace kf;

// Every load of the row (a, b and w) is issued up front and unconditionally (a chunk past the
// row re-reads its last chunk and counts nothing): with the loads under per-chunk branches hipcc
// waited for each one in turn, 16 dependent round trips per row -- invisible on a training-sized
// launch, but 10 us for the 8 rows of a decode step.
template <int VPT>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(
    const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, bf16_t* __restrict__ h_out,
    bf16_t* __restrict__ y, float* __restrict__ rstd, const bf16_t* __restrict__ w,
    int rows, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = H >> 3;
  const size_t base = (size_t)row * H;
  const bool has_b = b != nullptr;
  const bf16_t* bp = has_b ? b : a;
  u32x4 av[VPT], bv[VPT], wv[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int v = min(i * 64 + lane, nv - 1);
    av[i] = ld16(a + base + v * 8);
    bv[i] = ld16(bp + base + v * 8);
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) wv[i] = ld16(w + min(i * 64 + lane, nv - 1) * 8);
  u32x4 hq[VPT];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int v = i * 64 + lane;
    float x[8], t[8];
    unpack8(av[i], x);
    unpack8(bv[i], t);
    // the residual sum rounded to bf16 exactly as it is stored, so fwd/bwd agree (without a
    // residual h = a, which the round trip leaves unchanged)
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += has_b ? t[j] : 0.f;
    hq[i] = pack8(x);
    if (has_b && v < nv) st16(h_out + base + v * 8, hq[i]);
    unpack8(hq[i], x);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * x[j];
    ss += v < nv ? s : 0.f;
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)H + eps);
  if (lane == 0) rstd[row] = r;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int v = i * 64 + lane;
    if (v < nv) {
      float x[8], wf[8], o[8];
      unpack8(hq[i], x);
      unpack8(wv[i], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = x[j] * r * wf[j];
      st16(y + base + v * 8, pack8(o));
    }
  }
}

// Backward, one 256-thread block per row at a time (blocks stride over rows).  Each thread
// owns VPT fixed 16-B column chunks of the row, so the weight and the dW partial stay in ~4*VPT*8
// registers whatever H is (the wave-per-row form needed 312 VGPRs at H = 4096 and ran at
// one wave per SIMD, half of HBM bandwidth).  dot(g, h) is reduced across the block.
template <int VPT>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h, const float* __restrict__ rstd,
    const bf16_t* __restrict__ w, const bf16_t* __restrict__ dres, bf16_t* __restrict__ dh,
    float* __restrict__ dw_part, int rows, int H) {
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nv = H >> 3;
  float wf[VPT][8], dwacc[VPT][8];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int v = i * 256 + tid;
    if (v < nv) unpack8(ld16(w + v * 8), wf[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = 0.f;
  }
  int parity = 0;
  for (int row = blockIdx.x; row < rows; row += gridDim.x, parity ^= 1) {
    const size_t base = (size_t)row * H;
    const float r = rstd[row];
    float g[VPT][8], hx[VPT][8];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int v = i * 256 + tid;
      if (v < nv) {
        float d[8];
        unpack8(ld16(dy + base + v * 8), d);
        unpack8(ld16(h + base + v * 8), hx[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          g[i][j] = d[j] * wf[i][j];
          dot += g[i][j] * hx[i][j];
          dwacc[i][j] += d[j] * hx[i][j] * r;
        }
      }
    }
    dot = wave_sum(dot);
    if (lane == 0) red[parity][wv] = dot;      // double-buffered: no second barrier per row
    __syncthreads();
    dot = red[parity][0] + red[parity][1] + red[parity][2] + red[parity][3];
    const float c = r * r * r * dot / (float)H;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int v = i * 256 + tid;
      if (v < nv) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = r * g[i][j] - hx[i][j] * c;
        if (dres) {
          float t[8];
          unpack8(ld16(dres + base + v * 8), t);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += t[j];
        }
        st16(dh + base + v * 8, pack8(o));
      }
    }
  }
  float* out = dw_part + (size_t)blockIdx.x * H;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int v = i * 256 + tid;
    if (v < nv) {
      stf4(out + v * 8, f32x4{dwacc[i][0], dwacc[i][1], dwacc[i][2], dwacc[i][3]});
      stf4(out + v * 8 + 4, f32x4{dwacc[i][4], dwacc[i][5], dwacc[i][6], dwacc[i][7]});
    }
  }
}

// Column-sum P partial rows of length H (fp32) into a bf16 vector, optionally
// accumulating into the existing value (gradient accumulation into the flat grad buffer).
// Block = 16 waves x 64 columns; wave k sums rows k, k+16, ... (256-B coalesced row
// segments, 8 loads in flight per lane), then the 16 wave sums meet in LDS.
__global__ __launch_bounds__(1024) void colsum_to_bf16_kernel(const float* __restrict__ part, int P,
                                                              int H, bf16_t* __restrict__ out,
                                                              int accumulate) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < H) {
    int p = wv;
    for (; p + 16 * 7 < P; p += 16 * 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = part[(size_t)(p + 16 * u) * H + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += t[u];
    }
    for (; p < P; p += 16) s += part[(size_t)p * H + c];
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && c < H) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lane];
    if (accumulate) t += bf2f(out[c]);
    out[c] = f2bf(t);
  }
}

// Decode: h = a + bf16(sum_s part[s]); y = rmsnorm(h) * w, where part [S, rows, H] holds the fp32
// K-split partial sums of the batched-decode GEMM that produced the residual branch
// (ops/csrc/bgemm.hip with its reduce launch skipped).  The partials are summed in slice order
// and rounded to bf16 exactly as bgemm_reduce_kernel rounds them, so h is bitwise the unfused
// path's h.  One 256-thread block per row: a decode step has only 33-256 rows, so the row's
// CPT x S partial loads are spread over four waves and all issued before the first use.
template <int CPT, int S>
__global__ __launch_bounds__(256) void rmsnorm_fwd_parts_kernel(
    const bf16_t* __restrict__ a, const float* __restrict__ part, bf16_t* __restrict__ h_out,
    bf16_t* __restrict__ y, float* __restrict__ rstd, const bf16_t* __restrict__ w, int rows, int H, float eps) {
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int row = blockIdx.x;
  if (row >= rows) return;
  const int nv = H >> 3;
  const size_t base = (size_t)row * H, pstride = (size_t)rows * H;
  u32x4 av[CPT], wq[CPT];
  f32x4 pv[CPT][S][2];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int v = min(i * 256 + tid, nv - 1);
    av[i] = ld16(a + base + v * 8);
    wq[i] = ld16(w + v * 8);
#pragma unroll
    for (int t = 0; t < S; ++t) {
      pv[i][t][0] = ldf4(part + t * pstride + base + v * 8);
      pv[i][t][1] = ldf4(part + t * pstride + base + v * 8 + 4);
    }
  }
  u32x4 hq[CPT];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int v = i * 256 + tid;
    f32x4 d0 = f32x4{0.f, 0.f, 0.f, 0.f}, d1 = d0;
#pragma unroll
    for (int t = 0; t < S; ++t) {
      d0 += pv[i][t][0];
      d1 += pv[i][t][1];
    }
    float x[8], dr[8];
    unpack8(u32x4{pack2(d0[0], d0[1]), pack2(d0[2], d0[3]), pack2(d1[0], d1[1]), pack2(d1[2], d1[3])}, dr);
    unpack8(av[i], x);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += dr[j];
    hq[i] = pack8(x);
    if (v < nv) st16(h_out + base + v * 8, hq[i]);
    unpack8(hq[i], x);
    float sq = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) sq += x[j] * x[j];
    ss += v < nv ? sq : 0.f;
  }
  ss = wave_sum(ss);
  if (lane == 0) red[wv] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  const float r = rsqrtf(ss / (float)H + eps);
  if (tid == 0) rstd[row] = r;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int v = i * 256 + tid;
    if (v < nv) {
      float x[8], wf[8], o[8];
      unpack8(hq[i], x);
      unpack8(wq[i], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = x[j] * r * wf[j];
      st16(y + base + v * 8, pack8(o));
    }
  }
}

#define DISPATCH_VPT(nv, ...)                 \
  do {                                        \
    int _v = ((nv) + 63) / 64;                \
    if (_v <= 1) { constexpr int VPT = 1; __VA_ARGS__; }        \
    else if (_v <= 2) { constexpr int VPT = 2; __VA_ARGS__; }   \
    else if (_v <= 4) { constexpr int VPT = 4; __VA_ARGS__; }   \
    else if (_v <= 8) { constexpr int VPT = 8; __VA_ARGS__; }   \
    else if (_v <= 12) { constexpr int VPT = 12; __VA_ARGS__; } \
    else { constexpr int VPT = 16; __VA_ARGS__; }               \
  } while (0)

extern "C" {

int kf_rmsnorm_fwd(const void* a, const void* b, void* h_out, void* y, float* rstd, const void* w,
                   int rows, int H, float eps, hipStream_t s) {
  if (H % 8 != 0 || H > 8192) return 1;
  dim3 grid(cdiv(rows, 4));
  DISPATCH_VPT(H / 8, rmsnorm_fwd_kernel<VPT><<<grid, 256, 0, s>>>(
                          (const bf16_t*)a, (const bf16_t*)b, (bf16_t*)h_out, (bf16_t*)y, rstd,
                          (const bf16_t*)w, rows, H, eps));
  return 0;
}

// dw_part must hold nblocks * H floats (one dW partial row per block).
int kf_rmsnorm_bwd(const void* dy, const void* h, const float* rstd, const void* w,
                   const void* dres, void* dh, float* dw_part, int nblocks, void* dw_out,
                   int accumulate, int rows, int H, hipStream_t s) {
  if (H % 8 != 0 || H > 8192) return 1;
  const int nv = H / 8;
  if (nv <= 256) {
    rmsnorm_bwd_kernel<1><<<nblocks, 256, 0, s>>>((const bf16_t*)dy, (const bf16_t*)h, rstd, (const bf16_t*)w,
                                                 (const bf16_t*)dres, (bf16_t*)dh, dw_part, rows, H);
  } else if (nv <= 512) {
    rmsnorm_bwd_kernel<2><<<nblocks, 256, 0, s>>>((const bf16_t*)dy, (const bf16_t*)h, rstd, (const bf16_t*)w,
                                                 (const bf16_t*)dres, (bf16_t*)dh, dw_part, rows, H);
  } else {
    rmsnorm_bwd_kernel<4><<<nblocks, 256, 0, s>>>((const bf16_t*)dy, (const bf16_t*)h, rstd, (const bf16_t*)w,
                                                 (const bf16_t*)dres, (bf16_t*)dh, dw_part, rows, H);
  }
  colsum_to_bf16_kernel<<<cdiv(H, 64), 1024, 0, s>>>(dw_part, nblocks, H, (bf16_t*)dw_out, accumulate);
  return 0;
}

// part: fp32 [S, rows, H] (S = 2, 4 or 8; H a multiple of 8, at most 4096 -- two chunks per thread)
int kf_rmsnorm_fwd_parts(const void* a, const float* part, int S, void* h_out, void* y, float* rstd, const void* w,
                         int rows, int H, float eps, hipStream_t s) {
  if (H % 8 != 0 || H > 4096 || rows < 1) return 1;
  const int cpt = (H / 8 + 255) / 256;
#define RN_PARTS(C, SV)                                                                                       \
  rmsnorm_fwd_parts_kernel<C, SV><<<rows, 256, 0, s>>>((const bf16_t*)a, part, (bf16_t*)h_out, (bf16_t*)y, rstd, \
                                                       (const bf16_t*)w, rows, H, eps)
  if (cpt == 1) {
    if (S == 2) RN_PARTS(1, 2); else if (S == 4) RN_PARTS(1, 4); else if (S == 8) RN_PARTS(1, 8); else return 1;
  } else {
    if (S == 2) RN_PARTS(2, 2); else if (S == 4) RN_PARTS(2, 4); else if (S == 8) RN_PARTS(2, 8); else return 1;
  }
#undef RN_PARTS
  return 0;
}

}  // extern "C"
