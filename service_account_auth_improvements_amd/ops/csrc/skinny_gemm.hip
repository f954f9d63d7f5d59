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
//  * optional fused residual-add + RMSNorm PROLOGUE (the decode layer's two norms): every
//    workgroup forms h = bf16(x + res) for its <= 8 rows, reduces sum(h^2) over K, and stages
//    y = bf16(h * rstd * w_norm) in LDS as the X operand; workgroup 0 also stores h (the new
//    residual stream).  The first W loads are issued before the prologue, so its latency
//    hides under the weight stream, and two launches (+ their graph gaps) per layer vanish.
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

// residual-add + RMSNorm prologue operands (NORM kernels only)
struct NormArgs {
  const bf16_t* res;   // added to x (nullable)
  const bf16_t* w;     // norm weight [K]
  bf16_t* h_out;       // h = bf16(x + res), written by workgroup 0 (nullable when res is null)
  long ldh;
  float eps;
};
constexpr int NORM_MAX_ROWS = 8;
constexpr int NORM_LDS = 64 * 1024;   // staged normalised X: rows * K * 2 bytes

// MR: row slots of the norm prologue's LDS image (0 = no prologue; 4 or 8, >= M)
template <int NT, bool SWIGLU, int UNROLL, int MR>
__global__ __launch_bounds__(64 * WAVES) void skinny_gemm_kernel(const bf16_t* __restrict__ x, long ldx, int M,
                                                                 const bf16_t* __restrict__ w, int K,
                                                                 bf16_t* __restrict__ y, long ldy, int up_off,
                                                                 NormArgs na) {
  constexpr bool NORM = MR > 0;
  __shared__ float red[WAVES][SWIGLU ? 2 : 1][NT][16 * 16];
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];   // NORM: staged X, M * K (dynamic)
  __shared__ float ssq[NORM ? WAVES * NORM_MAX_ROWS : 1];
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

  u32x4 a[UNROLL], au[UNROLL];
  auto load_w = [&](int k) {
#pragma unroll
    for (int i = 0; i < UNROLL; ++i) {
      a[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wp + k + 32 * i));
      if (SWIGLU) au[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wu + k + 32 * i));
    }
  };
  if constexpr (NORM) {
    // h = bf16(x + res) -> sum of squares per row -> y = bf16(h * rstd * w) into LDS.  The first
    // pass's x, residual and gain chunks are loaded AHEAD of the weight stream and
    // unconditionally (rows past M repeat row M - 1, a chunk past the row its last chunk; none
    // of them is stored), so the prologue waits for them alone while the weights stream in; under
    // per-row branches hipcc waited for every load in flight.
    const int nch = K / 8;                   // 16-byte chunks per row
    const bool has_res = na.res != nullptr;
    const bf16_t* resp = has_res ? na.res : x;
    u32x4 xq[MR], rq[MR];
    const int c0 = min(tid, nch - 1);
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      // row offsets in VGPRs: 16 wave-uniform row pointers held in SGPRs spilled
      long off = (long)min(m, M - 1) * ldx + 8 * c0;
      asm volatile("" : "+v"(off));
      xq[m] = ld16(x + off);
      rq[m] = ld16(resp + off);
    }
    const u32x4 wn0 = ld16(na.w + 8 * c0);
    load_w(0);
    float ss[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) ss[m] = 0.f;
    auto absorb = [&](int c, const u32x4* xc, const u32x4* rc, bool valid) {
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        float hv[8], tv[8];
        unpack8(xc[m], hv);
        unpack8(rc[m], tv);
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] += has_res ? tv[j] : 0.f;
        const u32x4 hb = pack8(hv);          // the residual stream is stored (and normed) as bf16
        if (has_res && valid && m < M && blockIdx.x == 0) st16(na.h_out + (long)m * na.ldh + 8 * c, hb);
        unpack8(hb, hv);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += hv[j] * hv[j];
        ss[m] += valid ? s : 0.f;
        // (the LDS image has MR >= M row slots: rows past M hold duplicates, never read)
        if (valid) *reinterpret_cast<u32x4*>(xs + (long)m * K + 8 * c) = hb;   // un-normalised h for now
      }
    };
    absorb(c0, xq, rq, tid < nch);
    for (int c = tid + 64 * WAVES; c < nch; c += 64 * WAVES) {
      u32x4 xc[MR], rc[MR];
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        long off = (long)min(m, M - 1) * ldx + 8 * c;
        asm volatile("" : "+v"(off));
        xc[m] = ld16(x + off);
        rc[m] = ld16(resp + off);
      }
      absorb(c, xc, rc, true);
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const float v = wave_sum(ss[m]);
      if (l == 0) ssq[wave * MR + m] = v;
    }
    __syncthreads();
    float rs[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      float tot = 0.f;
#pragma unroll
      for (int v = 0; v < WAVES; ++v) tot += ssq[v * MR + m];
      rs[m] = rsqrtf(tot / (float)K + na.eps);
    }
    // in place, so only the owner of a chunk reads and writes it
    auto apply = [&](int c, u32x4 wq) {
      float wf[8];
      unpack8(wq, wf);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        float hv[8];
        unpack8(*reinterpret_cast<const u32x4*>(xs + (long)m * K + 8 * c), hv);
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = hv[j] * rs[m] * wf[j];
        *reinterpret_cast<u32x4*>(xs + (long)m * K + 8 * c) = pack8(hv);
      }
    };
    if (tid < nch) apply(tid, wn0);
    for (int c = tid + 64 * WAVES; c < nch; c += 64 * WAVES) apply(c, ld16(na.w + 8 * c));
    __syncthreads();
  } else {
    load_w(0);
  }

  for (int k = 0; k < kw; k += 32 * UNROLL) {
    if (k > 0) load_w(k);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int row = 16 * t + r;
      u32x4 bx[UNROLL];
#pragma unroll
      for (int i = 0; i < UNROLL; ++i) {
        if constexpr (NORM)
          bx[i] = row < M ? *reinterpret_cast<const u32x4*>(xs + (long)row * K + kbeg + k + 32 * i + 8 * q)
                          : u32x4{0, 0, 0, 0};
        else
          bx[i] = row < M ? ld16(x + (long)row * ldx + kbeg + k + 32 * i + 8 * q) : u32x4{0, 0, 0, 0};
      }
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

template <int NT, bool SWIGLU, int MR = 0>
int launch(const bf16_t* x, long ldx, int M, const bf16_t* w, int N, int K, bf16_t* y, long ldy, int up_off,
           hipStream_t st, NormArgs na = NormArgs{}) {
  dim3 grid(N / 16), block(64 * WAVES);
  const size_t dyn = (size_t)MR * K * 2;   // the norm prologue's staged X (MR row slots)
  if (K % (WAVES * 32 * 8) == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<NT, SWIGLU, 8, MR>), grid, block, dyn, st, x, ldx, M, w, K, y, ldy, up_off, na);
  else if (K % (WAVES * 32 * 4) == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<NT, SWIGLU, 4, MR>), grid, block, dyn, st, x, ldx, M, w, K, y, ldy, up_off, na);
  else if (K % (WAVES * 32 * 2) == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<NT, SWIGLU, 2, MR>), grid, block, dyn, st, x, ldx, M, w, K, y, ldy, up_off, na);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<NT, SWIGLU, 1, MR>), grid, block, dyn, st, x, ldx, M, w, K, y, ldy, up_off, na);
  KF_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// y = (rmsnorm(x + res) * w_norm) . W^T  [SwiGLU epilogue when swiglu]; h_out = x + res.
// Needs M <= NORM_MAX_ROWS and the staged X (4 row slots up to M = 4, else 8) x K x 2 bytes
// <= NORM_LDS; returns 1 otherwise.
extern "C" int kf_skinny_gemm_norm(const void* x, long ldx, int M, const void* res, const void* nw, float eps,
                                   void* h_out, long ldh, const void* w, int N, int K, void* y, long ldy,
                                   int swiglu, int up_off, hipStream_t st) {
  const int mr = M <= 4 ? 4 : NORM_MAX_ROWS;
  if (M <= 0 || M > NORM_MAX_ROWS || (long)mr * K * 2 > NORM_LDS || N % 16 != 0 || K % (WAVES * 32) != 0) return 1;
  if (res && !h_out) return 1;
  const NormArgs na{(const bf16_t*)res, (const bf16_t*)nw, (bf16_t*)h_out, ldh, eps};
  auto X = (const bf16_t*)x;
  auto W = (const bf16_t*)w;
  auto Y = (bf16_t*)y;
  if (mr == 4)
    return swiglu ? launch<1, true, 4>(X, ldx, M, W, N, K, Y, ldy, up_off, st, na)
                  : launch<1, false, 4>(X, ldx, M, W, N, K, Y, ldy, 0, st, na);
  return swiglu ? launch<1, true, NORM_MAX_ROWS>(X, ldx, M, W, N, K, Y, ldy, up_off, st, na)
                : launch<1, false, NORM_MAX_ROWS>(X, ldx, M, W, N, K, Y, ldy, 0, st, na);
}

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
