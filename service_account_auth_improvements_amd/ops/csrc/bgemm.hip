// Decode GEMM for 17 <= M <= 256 rows (batched decode): Y[M, N] = X[M, K] . W[N, K]^T, bf16
// in / out, fp32 accumulate.  At these batches the narrow projections of a decoder layer
// (N = 4096-6144) are still a weight stream (M flops per weight byte against ~300 at the
// MFMA/HBM balance point), but hipBLASLt's 128x128-class tiles leave most of the 256 CUs idle
// and stream them at 1.2-2.5 TB/s (profiles/serve_large_batch.md).  This kernel is laid out
// for the stream:
//
//  * one workgroup = 64 WT W rows (4 waves x 16 WT, WT = 1, or 2 above 128 rows: the A operand
//    of v_mfma_f32_16x16x32_bf16, every X fragment shared by the wave's WT tiles) x all
//    M (X is the B operand, MT = M/16 padded to 4, 8, 12, 16 column tiles) x one K slice.
//    K is split S ways (S chosen so the grid fills the CUs in one round); S > 1 writes fp32
//    partials [S][M][N] that bgemm_reduce_kernel sums (and rounds, or SwiGLUs) in a second launch.
//  * W goes straight from HBM into registers (lane (row l&15, k-chunk l>>4): 64 B per row per
//    k-step, KS k-steps per stage back to back); X, re-read by every workgroup, is staged by
//    LDS-DMA into a ring of stages, [16 MT rows][64 KS B] each, 16-B chunks XOR-swizzled so
//    that the four 16-lane groups of every ds_read_b128 hit 64 distinct banks.  W and X of a
//    stage are issued WD - 1 stages ahead in one in-order stream, so one counted vmcnt per stage
//    covers both (vmcnt retires in issue order: a shallower X ring would drag the W lookahead
//    down).  See BgCfg for the per-MT stage depth / ring depth.
//  * SwiGLU epilogue (decode gate/up projection): a workgroup owns 32 gate rows and the 32
//    matching up rows (W = [gate; up], up rows at +up_off) and writes silu(gate) * up.
#include "common.h"

#include <cstdlib>
#include <type_traits>

using namespace kf;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int BG_WAVES = 4;
constexpr int BG_BN = 16 * BG_WAVES;   // W rows per workgroup
constexpr int BG_KQ = 256;             // K granularity (the deepest stage)

// per MT: KS = 32-k MFMA steps per stage (a W row streams 64 KS contiguous bytes per stage:
// HBM wants long runs per row -- 128 B runs streamed at ~3.8 TB/s), WD = ring depth (stages),
// OCC = workgroups per CU.  X stage = 16 MT rows x 64 KS B.
// WT = 16-row W tiles per wave: 2 shares every X fragment read from LDS between two W tiles
// (half the LDS read traffic per weight byte; at M = 128 a one-tile wave reads 8 KB of X per
// KB of W), at twice the W and accumulator registers.
template <int MT, int WT> struct BgCfg;
template <> struct BgCfg<4, 1> { static constexpr int KS = 8, WD = 4, OCC = 1; };
template <> struct BgCfg<8, 1> { static constexpr int KS = 4, WD = 4, OCC = 1; };
template <> struct BgCfg<12, 1> { static constexpr int KS = 2, WD = 6, OCC = 1; };
template <> struct BgCfg<16, 1> { static constexpr int KS = 2, WD = 5, OCC = 1; };
template <> struct BgCfg<4, 2> { static constexpr int KS = 4, WD = 4, OCC = 1; };
template <> struct BgCfg<8, 2> { static constexpr int KS = 4, WD = 3, OCC = 1; };
template <> struct BgCfg<12, 2> { static constexpr int KS = 2, WD = 4, OCC = 1; };
template <> struct BgCfg<16, 2> { static constexpr int KS = 2, WD = 4, OCC = 1; };

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ u32 lds_u32(const void* p) {
  return (u32)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}
// X row reads in inline asm: hipcc would otherwise order every LDS read after all in-flight
// LDS-DMA (vmcnt(0)); the counted waits below tie the destination registers instead
__device__ __forceinline__ bf16x8 lds_row16(u32 addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}
template <int N>
__device__ __forceinline__ void lgkm_wait4(bf16x8* f) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
// W into registers by inline asm: hipcc's vmcnt bookkeeping for compiler-visible loads that stay
// in flight across the ring's loop back-edge degrades to vmcnt(0) before the first MFMA block of
// every revolution (a pipeline drain); the kernel's own counted waits cover these loads instead
__device__ __forceinline__ u32x4 gload16_nt(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ int xcd_remap(int bid, int total) {
  const int q = total / 8, r = total % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}
// 16-B chunk XOR swizzle of a staged X row: conflict-free for the fragment reads (lane: row l&15,
// chunk 4 ks + l>>4) -- 128-B rows pair up in the 64 banks, so they swizzle by row >> 1
template <int KS>
__device__ __forceinline__ int bg_swz(int row) { return KS == 2 ? (row >> 1) & 7 : row & 15; }

template <int MT, int WT, bool SWIGLU>
__global__ __launch_bounds__(64 * BG_WAVES, (BgCfg<MT, WT>::OCC)) void bgemm_kernel(
    const bf16_t* __restrict__ x, long ldx, int M, const bf16_t* __restrict__ w, long ldw, int kslice, int S,
    int NB, bf16_t* __restrict__ y, long ldy, float* __restrict__ part, int NP, int up_off) {
  constexpr int WD = BgCfg<MT, WT>::WD, KS = BgCfg<MT, WT>::KS;
  constexpr int BK = 32 * KS, ROWB = 2 * BK;        // k and X row bytes per stage
  constexpr int XST = 16 * MT * ROWB;               // bytes per X stage
  constexpr int RPI = 1024 / ROWB, LPR = 64 / RPI;  // X rows per DMA wave-instruction, lanes per row
  constexpr int XPW = XST / 1024 / BG_WAVES;        // X DMA wave-instructions per wave per stage
  constexpr int C = XPW + KS * WT;                  // VMEM instructions per wave per stage
  static_assert((WD - 2) * C <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[WD * XST];

  const int tid = threadIdx.x, l = tid & 63, wave = tid >> 6;
  const int lid = xcd_remap(blockIdx.x, NB * S);
  const int s = lid % S, nb = lid / S;
  const int kb = s * kslice, nst = kslice / BK;

  // this wave's 16 WT W rows (SwiGLU: waves 0-1 gate rows, waves 2-3 the matching up rows)
  const int wrow0 = SWIGLU ? (wave < 2 ? nb * 32 * WT + 16 * WT * wave : nb * 32 * WT + 16 * WT * (wave - 2) + up_off)
                           : nb * BG_BN * WT + 16 * WT * wave;
  const bf16_t* wp = w + (long)(wrow0 + (l & 15)) * ldw + kb + 8 * (l >> 4);   // tile t: + 16 t rows
  // X DMA: wave-instruction i (= wave + 4 t) fills rows RPI i ..; lane l -> row RPI i + l / LPR,
  // physical chunk l % LPR, i.e. logical chunk (l % LPR) ^ swz(row); rows >= M read row M-1
  const bf16_t* xp[XPW];
#pragma unroll
  for (int t = 0; t < XPW; ++t) {
    const int row = RPI * (wave + 4 * t) + l / LPR;
    xp[t] = x + (long)min(row, M - 1) * ldx + kb + 8 * ((l % LPR) ^ bg_swz<KS>(row));
  }
  char* const xdst = smem + 1024 * wave;            // + slot * XST + 4096 t

  u32x4 wv[WD][KS][WT];
  // Stage j's X DMA then its W loads, into ring slot SL (a compile-time register index).  Every
  // step issues exactly C instructions -- stages past the slice re-read L2-resident X rows into
  // a dead slot -- so one constant vmcnt per step is exact.
  const bf16_t* const wdummy = x + 8 * (l >> 4);
  auto issue = [&](auto slotc, int j) {
    constexpr int SL = decltype(slotc)::value;
    const bool live = j < nst;
#pragma unroll
    for (int t = 0; t < XPW; ++t) glds16(live ? xp[t] + BK * j : xp[t], xdst + SL * XST + 4096 * t);
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      const bf16_t* src = live ? wp + (long)16 * t * ldw + BK * j : wdummy;
#pragma unroll
      for (int q = 0; q < KS; ++q) wv[SL][q][t] = gload16_nt(src + 32 * q);
    }
  };

  f32x4 acc[WT][MT];
#pragma unroll
  for (int t = 0; t < WT; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  // lane's X fragment address in a stage: row 16 m + (l & 15), logical chunk 4 ks + (l >> 4)
  const int xr = l & 15;
  const u32 xrd = lds_u32(smem) + xr * ROWB;
  const int sw = bg_swz<KS>(xr);                    // swz(16 m + xr) == swz(xr)

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1 % WD>;
  using I2 = std::integral_constant<int, 2 % WD>;
  using I3 = std::integral_constant<int, 3 % WD>;
  using I4 = std::integral_constant<int, 4 % WD>;
  using I5 = std::integral_constant<int, 5 % WD>;
  using I6 = std::integral_constant<int, 6 % WD>;
  using I7 = std::integral_constant<int, 7 % WD>;
  // prologue: stages 0 .. WD-2 in flight
  issue(I0(), 0);
  if constexpr (WD > 2) issue(I1(), 1);
  if constexpr (WD > 3) issue(I2(), 2);
  if constexpr (WD > 4) issue(I3(), 3);
  if constexpr (WD > 5) issue(I4(), 4);
  if constexpr (WD > 6) issue(I5(), 5);
  if constexpr (WD > 7) issue(I6(), 6);

  auto stage = [&](auto slotc, int j) {
    constexpr int U = decltype(slotc)::value;
    vm_wait<(WD - 2) * C>();                        // stage j landed (WD - 2 later stages in flight)
    barrier();                                      // ... for every wave; the slot of j - 1 is free
    issue(std::integral_constant<int, (U + WD - 1) % WD>(), j + WD - 1);
    // Stage j's W registers have landed (the wait above): hand them back to the compiler on EVERY
    // path.  It believes an asm load wrote its register at issue, so a def left without a use
    // (a dead step) frees the register while the load is still in flight, and a value placed
    // there meanwhile is overwritten when the load lands.
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int t = 0; t < WT; ++t) asm volatile("" : "+v"(wv[U][q][t]));
    if (j >= nst) return;                           // a dead step of the last revolution
    const u32 base = xrd + U * XST;
    bf16x8 xf[2][4];
    // groups of four X fragments: (ks, m0..m0+3); the next group is read before this one's MFMAs
    constexpr int G = KS * MT / 4;
    auto rd = [&](int g, bf16x8* f) {
      const int ks = g / (MT / 4), m0 = 4 * (g % (MT / 4));
#pragma unroll
      for (int i = 0; i < 4; ++i) f[i] = lds_row16(base + (m0 + i) * 16 * ROWB + 16 * ((4 * ks + (l >> 4)) ^ sw));
    };
    rd(0, xf[0]);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (g + 1 < G) {
        rd(g + 1, xf[(g + 1) & 1]);
        lgkm_wait4<4>(xf[g & 1]);
      } else {
        lgkm_wait4<0>(xf[g & 1]);
      }
      const int ks = g / (MT / 4), m0 = 4 * (g % (MT / 4));
#pragma unroll
      for (int t = 0; t < WT; ++t) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, wv[U][ks][t]);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[t][m0 + i] = mfma16(a, xf[g & 1][i], acc[t][m0 + i]);
      }
    }
  };
  // whole ring revolutions; the last one's steps past nst only keep the load count uniform
  for (int j = 0; j < nst; j += WD) {
    stage(I0(), j);
    if constexpr (WD > 1) stage(I1(), j + 1);
    if constexpr (WD > 2) stage(I2(), j + 2);
    if constexpr (WD > 3) stage(I3(), j + 3);
    if constexpr (WD > 4) stage(I4(), j + 4);
    if constexpr (WD > 5) stage(I5(), j + 5);
    if constexpr (WD > 6) stage(I6(), j + 6);
    if constexpr (WD > 7) stage(I7(), j + 7);
  }
  vm_wait<0>();                                     // drain the dummy loads before LDS reuse / exit
#pragma unroll
  for (int u = 0; u < WD; ++u)                      // ... and only then release their registers
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int t = 0; t < WT; ++t) asm volatile("" : "+v"(wv[u][q][t]));

  // acc[t][m]: lane l, reg r -> W row (n) 16 t + 4 (l >> 4) + r of this wave's 16 WT, X row (m)
  // 16 m + (l & 15)
  const int nr = 4 * (l >> 4);
  if constexpr (SWIGLU) {
    // waves 2-3 hand their up-row sums to waves 0-1 through LDS (the ring is idle now)
    __syncthreads();
    float* up = reinterpret_cast<float*>(smem);     // [2 waves][WT][MT][64 lanes][4]
    if (wave >= 2) {
#pragma unroll
      for (int t = 0; t < WT; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m)
          *reinterpret_cast<f32x4*>(up + ((((wave - 2) * WT + t) * MT + m) * 64 + l) * 4) = acc[t][m];
    }
    __syncthreads();
    if (wave >= 2) return;
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      const int col0 = nb * 32 * WT + 16 * (WT * wave + t) + nr;   // output (gate) column of reg 0
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int row = 16 * m + (l & 15);
        const f32x4 u = *reinterpret_cast<const f32x4*>(up + (((wave * WT + t) * MT + m) * 64 + l) * 4);
        if (S == 1) {
          if (row < M) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = acc[t][m][r] * sigmoidf_(acc[t][m][r]) * u[r];
            *reinterpret_cast<u32x2*>(y + (long)row * ldy + col0) = u32x2{pack2(o[0], o[1]), pack2(o[2], o[3])};
          }
        } else if (row < M) {   // partials in 64-wide [32 gate | 32 up] blocks (bgemm_reduce_kernel)
          float* p = part + ((long)s * M + row) * NP + (col0 / 32) * 64 + col0 % 32;
          *reinterpret_cast<f32x4*>(p) = acc[t][m];
          *reinterpret_cast<f32x4*>(p + 32) = u;
        }
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      const int col0 = nb * BG_BN * WT + 16 * (WT * wave + t) + nr;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int row = 16 * m + (l & 15);
        if (row >= M) continue;
        if (S == 1) {
          *reinterpret_cast<u32x2*>(y + (long)row * ldy + col0) =
              u32x2{pack2(acc[t][m][0], acc[t][m][1]), pack2(acc[t][m][2], acc[t][m][3])};
        } else {
          *reinterpret_cast<f32x4*>(part + ((long)s * M + row) * NP + col0) = acc[t][m];
        }
      }
    }
  }
}

// y[m, n] = bf16(sum_s part[s, m, n]) (SwiGLU: silu(gate) * up from 64-wide [gate | up] blocks)
template <bool SWIGLU>
__global__ __launch_bounds__(256) void bgemm_reduce_kernel(const float* __restrict__ part, int S, int M, int NP,
                                                           bf16_t* __restrict__ y, long ldy) {
  const int Nout = SWIGLU ? NP / 2 : NP;
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;   // 4 output columns per thread
  if (i >= (long)M * Nout) return;
  const int m = (int)(i / Nout), n = (int)(i % Nout);
  const long stride = (long)M * NP;
  if constexpr (SWIGLU) {
    const int pc = (n / 32) * 64 + n % 32;
    f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f}, u = g;
    for (int t = 0; t < S; ++t) {
      const float* p = part + t * stride + (long)m * NP + pc;
      g += *reinterpret_cast<const f32x4*>(p);
      u += *reinterpret_cast<const f32x4*>(p + 32);
    }
    float o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = g[r] * sigmoidf_(g[r]) * u[r];
    *reinterpret_cast<u32x2*>(y + (long)m * ldy + n) = u32x2{pack2(o[0], o[1]), pack2(o[2], o[3])};
  } else {
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < S; ++t) a += *reinterpret_cast<const f32x4*>(part + t * stride + (long)m * NP + n);
    *reinterpret_cast<u32x2*>(y + (long)m * ldy + n) = u32x2{pack2(a[0], a[1]), pack2(a[2], a[3])};
  }
}

template <int MT, int WT, bool SWIGLU>
void bg_launch(int grid, hipStream_t st, const bf16_t* x, long ldx, int M, const bf16_t* w, long ldw, int kslice,
               int S, int NB, bf16_t* y, long ldy, float* part, int NP, int up_off) {
  hipLaunchKernelGGL((bgemm_kernel<MT, WT, SWIGLU>), dim3(grid), dim3(64 * BG_WAVES), 0, st, x, ldx, M, w, ldw,
                     kslice, S, NB, y, ldy, part, NP, up_off);
}

int bg_mt(int M) { return M <= 64 ? 4 : M <= 128 ? 8 : M <= 192 ? 12 : 16; }

}  // namespace

// W tiles per wave for an (M, N, K) problem; N must split into 64 WT-row blocks.  Two tiles above
// 128 rows, where the X reads dominate: wd 59.4 -> 53.1 us and wqkv 37.9 -> 33.7 us at 256 rows;
// at 64-128 rows the doubled registers cost more than the halved LDS reads (wo at 128 rows
// 19.8 -> 25.2 us; profiles/serve_bgemm_wt_r5.md).  KFAMD_BGEMM_WT = 1 / 2 overrides (A/Bs).
extern "C" int kf_bgemm_wt(int M, int N, int K) {
  static const int force = [] {
    const char* e = std::getenv("KFAMD_BGEMM_WT");
    return e ? std::atoi(e) : 0;
  }();
  const int wt = force == 1 || force == 2 ? force : (M > 128 ? 2 : 1);
  return N % (BG_BN * wt) == 0 ? wt : 1;
}

// K split for an (M, N, K) problem: enough workgroups for one full round of the CUs, K slices a
// whole number of 64-k stages.  KFAMD_BGEMM_SPLIT overrides (tools/bench_bgemm.py sweeps).
// N = rows of W (SwiGLU: gate + up), so the grid has N / (64 WT) column blocks either way.
extern "C" int kf_bgemm_splits(int M, int N, int K) {
  static const int force = [] {
    const char* e = std::getenv("KFAMD_BGEMM_SPLIT");
    return e ? std::atoi(e) : 0;
  }();
  const int wt = kf_bgemm_wt(M, N, K);
  const int NB = N / (BG_BN * wt);
  const int stages = K / BG_KQ;
  if (force > 0) return (stages % force == 0) ? force : 1;
  int S = 1;   // one workgroup per CU: fill the 256 CUs, slices of >= 4 (WT 2: 2) 256-k quanta
  const int min_q = wt == 2 ? 2 : 4;
  while (S < 8 && NB * S * 2 <= 256 && stages % (S * 2) == 0 && stages / (S * 2) >= min_q) S *= 2;
  return S;
}

// Y[M, N] = X[M, K] . W^T with W [N, K] (SwiGLU: W = [gate; up] with up rows at +up_off, Y
// [M, up_off] = silu(X gate^T) * (X up^T)).  part: fp32 workspace of S * M * NP floats (NP = N,
// or 2 * up_off for SwiGLU) when S > 1.  y = nullptr with S > 1 (not SwiGLU): only the partials
// are written and the reduce launch is left to the consumer (kf_rmsnorm_fwd_parts sums them in
// its prologue).  Returns 1 (nothing launched) outside the kernel's range.
extern "C" int kf_bgemm(const void* x, long ldx, int M, const void* w, int N, int K, void* y, long ldy, int swiglu,
                        int up_off, int S, float* part, hipStream_t st) {
  if (M < 1 || M > 256 || K % BG_KQ || ldx % 8 || ldy % 4 || S < 1 || (K / BG_KQ) % S) return 1;
  if ((((uintptr_t)x) | ((uintptr_t)w)) & 15 || ((uintptr_t)y) & 7) return 1;
  const int wt = kf_bgemm_wt(M, N, K);
  if (swiglu ? (up_off % (32 * wt) || N != 2 * up_off) : N % (BG_BN * wt)) return 1;
  if (S > 1 && !part) return 1;
  if (!y && (S == 1 || swiglu)) return 1;
  const int NB = swiglu ? up_off / (32 * wt) : N / (BG_BN * wt), NP = swiglu ? 2 * up_off : N;
  const int kslice = K / S, grid = NB * S;
  auto X = (const bf16_t*)x;
  auto W = (const bf16_t*)w;
  auto Y = (bf16_t*)y;
  const int mt = bg_mt(M);
#define BG_CASE(MTV)                                                                                           \
  case MTV:                                                                                                    \
    if (wt == 2) {                                                                                             \
      if (swiglu) bg_launch<MTV, 2, true>(grid, st, X, ldx, M, W, (long)K, kslice, S, NB, Y, ldy, part, NP, up_off); \
      else bg_launch<MTV, 2, false>(grid, st, X, ldx, M, W, (long)K, kslice, S, NB, Y, ldy, part, NP, 0);       \
    } else {                                                                                                   \
      if (swiglu) bg_launch<MTV, 1, true>(grid, st, X, ldx, M, W, (long)K, kslice, S, NB, Y, ldy, part, NP, up_off); \
      else bg_launch<MTV, 1, false>(grid, st, X, ldx, M, W, (long)K, kslice, S, NB, Y, ldy, part, NP, 0);       \
    }                                                                                                          \
    break;
  switch (mt) {
    BG_CASE(4)
    BG_CASE(8)
    BG_CASE(12)
    BG_CASE(16)
    default: return 1;
  }
#undef BG_CASE
  KF_CHECK_LAUNCH();
  if (S > 1 && y) {
    const long threads = (long)M * (swiglu ? up_off : N) / 4;
    const int blocks = (int)((threads + 255) / 256);
    if (swiglu) hipLaunchKernelGGL(bgemm_reduce_kernel<true>, dim3(blocks), dim3(256), 0, st, part, S, M, NP, Y, ldy);
    else hipLaunchKernelGGL(bgemm_reduce_kernel<false>, dim3(blocks), dim3(256), 0, st, part, S, M, NP, Y, ldy);
    KF_CHECK_LAUNCH();
  }
  return 0;
}
