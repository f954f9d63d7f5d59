// Skinny GEMM for decode: Y[M, N] = X[M, K] . W[N, K]^T with M <= 64 (one decode row per
// sequence), bf16 in / bf16 out, fp32 accumulate.  Decode is weight-streaming-bound: every
// weight byte is read once per token, so the kernel is built to keep HBM busy, not MFMA:
//
//  * one workgroup = 16 rows of W (one v_mfma_f32_16x16x32_bf16 A tile) x all of K, split
//    over 8 waves (split-K inside the workgroup, reduced through LDS) -> N/16 workgroups,
//    8 waves each: 2048 waves for N = 4096, enough loads in flight to cover HBM latency.
//  * each lane streams 16 B of W per MFMA (4 lanes x 16 B = 64 B contiguous per row),
//    UNROLL loads issued back to back before their MFMAs.
//  * X (<= 64 x K bf16, L2-resident, shared by every workgroup) is the B operand; M is
//    covered by NT column tiles of 16 (rows >= M are predicated off, not read).
//  * epilogues: plain bf16 store, or SwiGLU -- the workgroup also computes the matching
//    "up" rows (W row n + F) and writes silu(gate) * up, so the decode MLP's gate/up GEMM
//    and the activation are one kernel.
// MFMA 16x16x32 bf16 layout (guide §3): lane l holds A[row l&15][k 8(l>>4)+j] and
// B[k 8(l>>4)+j][col l&15]; D: col = l&15, row = 4(l>>4) + reg.
#include "common.h"

using namespace kf;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int WAVES = 8;
constexpr int NT_MAX = 4;

__device__ __forceinline__ bf16x8 as_bf(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int NT, bool SWIGLU, int UNROLL>
__global__ __launch_bounds__(64 * WAVES) void skinny_gemm_kernel(const bf16_t* __restrict__ x, long ldx, int M,
                                                                 const bf16_t* __restrict__ w, int K,
                                                                 bf16_t* __restrict__ y, long ldy, int up_off) {
  __shared__ float red[WAVES][SWIGLU ? 2 : 1][NT][16 * 16];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63;
  const int r = l & 15, q = l >> 4;
  const int n0 = blockIdx.x * 16;
  const int kw = K / WAVES;                 // host guarantees K % (WAVES * 32 * UNROLL) == 0
  const int kbeg = wave * kw;
  const bf16_t* wp = w + (long)(n0 + r) * K + kbeg + 8 * q;
  const bf16_t* wu = SWIGLU ? wp + (long)up_off * K : nullptr;
  f32x4 acc[SWIGLU ? 2 : 1][NT];
#pragma unroll
  for (int e = 0; e < (SWIGLU ? 2 : 1); ++e)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[e][t] = f32x4{};

  for (int k = 0; k < kw; k += 32 * UNROLL) {
    u32x4 a[UNROLL], au[UNROLL];
#pragma unroll
    for (int i = 0; i < UNROLL; ++i) {
      a[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wp + k + 32 * i));
      if (SWIGLU) au[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wu + k + 32 * i));
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int row = 16 * t + r;
      u32x4 bx[UNROLL];
#pragma unroll
      for (int i = 0; i < UNROLL; ++i)
        bx[i] = row < M ? ld16(x + (long)row * ldx + kbeg + k + 32 * i + 8 * q) : u32x4{0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < UNROLL; ++i) {
        acc[0][t] = mfma16(as_bf(a[i]), as_bf(bx[i]), acc[0][t]);
        if (SWIGLU) acc[SWIGLU ? 1 : 0][t] = mfma16(as_bf(au[i]), as_bf(bx[i]), acc[SWIGLU ? 1 : 0][t]);
      }
    }
  }
  // D[n_local = 4q + j][m_local = r] -> LDS, reduce over the 8 waves
#pragma unroll
  for (int e = 0; e < (SWIGLU ? 2 : 1); ++e)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wave][e][t][(4 * q + j) * 16 + r] = acc[e][t][j];
  __syncthreads();
  for (int o = tid; o < NT * 256; o += 64 * WAVES) {
    const int t = o >> 8, nl = (o >> 4) & 15, ml = o & 15;
    const int m = 16 * t + ml;
    if (m >= M) continue;
    float g = 0.f;
#pragma unroll
    for (int v = 0; v < WAVES; ++v) g += red[v][0][t][nl * 16 + ml];
    if (SWIGLU) {
      float u = 0.f;
#pragma unroll
      for (int v = 0; v < WAVES; ++v) u += red[v][SWIGLU ? 1 : 0][t][nl * 16 + ml];
      g = g * sigmoidf_(g) * u;
    }
    y[(long)m * ldy + n0 + nl] = f2bf(g);
  }
}

template <int NT, bool SWIGLU>
int launch(const bf16_t* x, long ldx, int M, const bf16_t* w, int N, int K, bf16_t* y, long ldy, int up_off,
           hipStream_t st) {
  dim3 grid(N / 16), block(64 * WAVES);
  if (K % (WAVES * 32 * 8) == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<NT, SWIGLU, 8>), grid, block, 0, st, x, ldx, M, w, K, y, ldy, up_off);
  else if (K % (WAVES * 32 * 4) == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<NT, SWIGLU, 4>), grid, block, 0, st, x, ldx, M, w, K, y, ldy, up_off);
  else if (K % (WAVES * 32 * 2) == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<NT, SWIGLU, 2>), grid, block, 0, st, x, ldx, M, w, K, y, ldy, up_off);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<NT, SWIGLU, 1>), grid, block, 0, st, x, ldx, M, w, K, y, ldy, up_off);
  KF_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// swiglu: W holds [gate (up_off rows); up (up_off rows)], N = up_off, Y = silu(X.Wg^T) * (X.Wu^T)
extern "C" int kf_skinny_gemm(const void* x, long ldx, int M, const void* w, int N, int K, void* y, long ldy,
                              int swiglu, int up_off, hipStream_t st) {
  if (M <= 0 || M > 16 * NT_MAX || N % 16 != 0 || K % (WAVES * 32) != 0) return 1;
  auto X = (const bf16_t*)x;
  auto W = (const bf16_t*)w;
  auto Y = (bf16_t*)y;
  const int nt = (M + 15) / 16;
  if (swiglu) {
    switch (nt) {
      case 1: return launch<1, true>(X, ldx, M, W, N, K, Y, ldy, up_off, st);
      case 2: return launch<2, true>(X, ldx, M, W, N, K, Y, ldy, up_off, st);
      default: return launch<4, true>(X, ldx, M, W, N, K, Y, ldy, up_off, st);
    }
  }
  switch (nt) {
    case 1: return launch<1, false>(X, ldx, M, W, N, K, Y, ldy, 0, st);
    case 2: return launch<2, false>(X, ldx, M, W, N, K, Y, ldy, 0, st);
    default: return launch<4, false>(X, ldx, M, W, N, K, Y, ldy, 0, st);
  }
}
