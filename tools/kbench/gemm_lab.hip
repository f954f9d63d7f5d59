// Lab copy for the dW GEMM: the production kernel (ops/csrc/gemm.hip) plus candidate variants,
// selected in gemm_bench by KF_GEMM_IMPL (8 = production 8-wave kernel, 4 = variant below).
//
// Variant "tn4": 4 waves (one per SIMD), 256 x 256 workgroup tile, each wave 128 x 128 =
// 8 x 8 v_mfma_f32_16x16x32_bf16 accumulators (256 registers, AGPR half of the unified file).
// Per 32-k stage and SIMD it issues 32 transposed LDS reads for 64 MFMAs (the 8-wave kernel:
// 48), one barrier per 1024 MFMA cycles, and its 8 LDS-DMA pieces two per MFMA group after the
// barrier instead of in one burst.  B fragments ping-pong between two register sets across
// stages (no copies); a 4-deep ring keeps the buffer index and the register parity aligned over
// a 4-stage unroll.  Past the last stage the "next stage" reads and DMA are issued anyway from
// valid addresses (results unused) so every wait count stays a compile-time constant.
#include "gemm_prod_lab.hip"   // the production kernel with its anatomy / tuning knobs

namespace g4 {
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    static_for<I + 1, N>(f);
  }
}
// acc += a.b with the accumulator pinned to AGPRs (the builtin keeps the VGPR form and copies
// all 256 accumulators through v_accvgpr moves); operands come straight from LDS reads
__device__ __forceinline__ void mfma16a(f32x4& acc, bf16x8 a, bf16x8 b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
#ifndef KF_G4_NB
#define KF_G4_NB 4
#endif
constexpr int NB4 = KF_G4_NB;                  // ring depth (stages of 32 k-rows): 4 = 128 KB, 5 = 160 KB
constexpr int IMG4 = gm::IMG;                  // [32][128] bf16 image, 8 KB
constexpr int SMEM4 = 4 * NB4 * IMG4;            // 128 KB: [image A lo, A hi, B lo, B hi][buffer]

template <int N>
__device__ __forceinline__ void lgkm(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_all(bf16x8& a, bf16x8* b) {
  asm volatile("s_waitcnt lgkmcnt(%9)"
               : "+v"(a), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7])
               : "i"(N)
               : "memory");
}
// KF_G4_V: 1 = first form (next-stage reads nb 2i, 2i+1, na i in group 4+i; the 8 DMA pieces
// two per group in groups 4-7); 2 = B fragments first (groups 4-6 read nb 0-7 + na0, group 7
// na1-3: the wait before a stage's first MFMA group covers reads two groups old, not one) and
// one DMA piece per MFMA group (groups 4-7 the first half of this stage's refill, groups 0-3 of
// the next stage the second half)
#ifndef KF_G4_V
#define KF_G4_V 2
#endif
// wait before MFMA group t (see the issue order in the kernel)
template <int T> struct W;
template <> struct W<0> { static constexpr int v = KF_G4_V == 1 ? 2 : 6; };
template <> struct W<1> { static constexpr int v = KF_G4_V == 1 ? 14 : 6; };
template <> struct W<2> { static constexpr int v = KF_G4_V == 1 ? 10 : 6; };
template <> struct W<3> { static constexpr int v = 6; };
template <> struct W<4> { static constexpr int v = 6; };
template <> struct W<5> { static constexpr int v = 10; };
template <> struct W<6> { static constexpr int v = 14; };
template <> struct W<7> { static constexpr int v = 15; };   // 18 issued after a7: any wait <= 15 covers it
}  // namespace g4

__global__ __launch_bounds__(256, 1) void gemm_tn4_kernel(TnGroup grp, int K) {
  using namespace g4;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int lid = xcd_remap(blockIdx.x, grp.total);
  const int pi = (grp.n > 1 && lid >= grp.p[0].tiles) ? 1 : 0;
  if (pi) lid -= grp.p[0].tiles;
  const TnProblem& P = grp.p[pi];
  const bf16_t* __restrict__ A = P.A;
  const bf16_t* __restrict__ Bm = P.B;
  bf16_t* __restrict__ C = P.C;
  const long lda = P.lda, ldb = P.ldb, ldc = P.ldc;
  const int M = P.M, N = P.N;
  const bool ACC = P.acc != 0;
  const int mt_n = M / gm::BM, nt_n = N / gm::BN;
  const int per_group = GROUP_M * nt_n;
  const int gid = lid / per_group, first_m = gid * GROUP_M;
  const int gsize = min(mt_n - first_m, GROUP_M);
  const int mt = first_m + (lid % per_group) % gsize, nt = (lid % per_group) / gsize;
  const long m0 = (long)mt * gm::BM, n0 = (long)nt * gm::BN;
  const int wm = wave & 1, wn = wave >> 1;          // wave sub-tile: rows 128 wm.., cols 128 wn..

  f32x4 acc[8][8];                                  // [n tile u][m tile t], C^T fragments
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32 aad[8], bad[8];
  {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, row = 8 * g + q;
    const u32 rb = lds_addr(smem) + row * 256 + 8 * p;
    const int f = blk_x(row);
#pragma unroll
    for (int t = 0; t < 8; ++t) aad[t] = rb + wm * NB4 * IMG4 + 32 * (t ^ f);
#pragma unroll
    for (int u = 0; u < 8; ++u) bad[u] = rb + (2 + wn) * NB4 * IMG4 + 32 * (u ^ f);
  }
  // DMA: wave w fills rows 4w..4w+3 (piece j = 0) and 16+4w.. (j = 1) of each of the 4 images;
  // the j = 1 piece reuses the lane offset with the panel base 16 rows further (SGPR)
  u32 dmo[4];
  {
    const int row = 4 * wave + (lane >> 4), pc = lane & 15;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int col = 16 * ((pc >> 1) ^ blk_x(row)) + 8 * (pc & 1) + 128 * (k & 1);
      dmo[k] = (u32)(((k < 2 ? lda : ldb) * row + col) * 2);
    }
  }
  const int nk = K / gm::BK;
  const char* Ap = reinterpret_cast<const char*>(A + m0);
  const char* Bp = reinterpret_cast<const char*>(Bm + n0);
  const long astep = (long)gm::BK * lda * 2, bstep = (long)gm::BK * ldb * 2;
  const long a16 = 16 * lda * 2, b16 = 16 * ldb * 2;
  const u32 lds_w = __builtin_amdgcn_readfirstlane(lds_addr(smem) + 1024 * wave);
  // anatomy switches (numerics broken): KF_G4_ABL_DMA=1 no loop DMA, =2 loop DMA always from the
  // first (L2-resident) panel rows; KF_G4_ABL_BAR=1 no loop vmcnt wait + barrier
  auto piece = [&](int k, int j, const char* a, const char* b, u32 buf) {
#if defined(KF_G4_ABL_DMA) && KF_G4_ABL_DMA == 2
    a = Ap;
    b = Bp;
#endif
    const char* base = k < 2 ? a + j * a16 : b + j * b16;
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                 :
                 : "s"(lds_w + k * NB4 * IMG4 + buf * IMG4 + j * 4096), "v"(dmo[k]), "s"(uniform_ptr(base))
                 : "memory", "m0");
  };
  auto stage_all = [&](int s, u32 buf) {
    const char* a = Ap + (long)s * astep;
    const char* b = Bp + (long)s * bstep;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      piece(k, 0, a, b, buf);
      piece(k, 1, a, b, buf);
    }
  };
  // prologue: stages 0..3 in flight (V2: the second half of stage 3 comes from stage 0's groups
  // 0-3, as every later refill's second half does), publish stage 0
  if (KF_G4_V == 1) {
#pragma unroll
    for (int s = 0; s < NB4; ++s) stage_all(min(s, nk - 1), s);
    vm_wait<8 * (NB4 - 1)>();
  } else {
#pragma unroll
    for (int s = 0; s < NB4 - 1; ++s) stage_all(min(s, nk - 1), s);
    {
      const int s3 = min(NB4 - 1, nk - 1);
      const char* a3 = Ap + (long)s3 * astep;
      const char* b3 = Bp + (long)s3 * bstep;
#pragma unroll
      for (int k = 0; k < 4; ++k) piece(k, 0, a3, b3, NB4 - 1);
    }
    vm_wait<8 * (NB4 - 2) + 4>();
  }
  barrier();

  bf16x8 a[8], bs[2][8];
  // the reads a virtual stage -1 would have issued in its groups 4..7 (same order, same counts)
  if (KF_G4_V == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bs[0][2 * i] = tr_frag<0>(bad[2 * i]);
      bs[0][2 * i + 1] = tr_frag<0>(bad[2 * i + 1]);
      a[i] = tr_frag<0>(aad[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) bs[0][i] = tr_frag<0>(bad[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = tr_frag<0>(aad[i]);
  }

  auto stage = [&](auto bufc, auto parc, int s) {
    constexpr int CB = decltype(bufc)::value, PAR = decltype(parc)::value, NX = (CB + 1) % NB4;
    constexpr int PB = (CB + NB4 - 1) % NB4;
    constexpr int OC = CB * IMG4, ON = NX * IMG4;
    bf16x8* b = bs[PAR];
    bf16x8* nb = bs[PAR ^ 1];
    // DMA sources (stage indices are scalar; past the end the last stage is re-read, unused)
    const int s4 = min(s + NB4, nk - 1), s3 = min(s + NB4 - 1, nk - 1);
    const char* da = Ap + (long)s4 * astep;
    const char* db = Bp + (long)s4 * bstep;
    const char* pa = Ap + (long)s3 * astep;
    const char* pbb = Bp + (long)s3 * bstep;
    static_for<0, 8>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t == 0) lgkm_all<W<0>::v>(a[0], b);
      else lgkm<W<t>::v>(a[t]);
#pragma unroll
      for (int u = 0; u < 8; ++u) mfma16a(acc[u][t], b[u], a[t]);
      if constexpr (t < 4) {
        a[t + 4] = tr_frag<OC>(aad[t + 4]);
        // V2: second half of the previous stage's refill (buffer PB <- stage s+3)
#if !(defined(KF_G4_ABL_DMA) && KF_G4_ABL_DMA == 1)
        if (KF_G4_V == 2) piece(t, 1, pa, pbb, PB);
#endif
      } else {
        constexpr int i = t - 4;
        if constexpr (KF_G4_V == 1) {
          nb[2 * i] = tr_frag<ON>(bad[2 * i]);
          nb[2 * i + 1] = tr_frag<ON>(bad[2 * i + 1]);
          a[i] = tr_frag<ON>(aad[i]);
          // refill this stage's buffer (every wave has issued all its reads of it) with stage s+4
          piece(i, 0, da, db, CB);
          piece(i, 1, da, db, CB);
        } else {
          if constexpr (i < 3) {
            nb[3 * i] = tr_frag<ON>(bad[3 * i]);
            nb[3 * i + 1] = tr_frag<ON>(bad[3 * i + 1]);
            if constexpr (i < 2) nb[3 * i + 2] = tr_frag<ON>(bad[3 * i + 2]);
            else a[0] = tr_frag<ON>(aad[0]);
          } else {
            a[1] = tr_frag<ON>(aad[1]);
            a[2] = tr_frag<ON>(aad[2]);
            a[3] = tr_frag<ON>(aad[3]);
          }
#if !(defined(KF_G4_ABL_DMA) && KF_G4_ABL_DMA == 1)
          piece(i, 0, da, db, CB);      // first half of this stage's refill (stage s+4)
#endif
        }
      }
#if !defined(KF_G4_ABL_BAR)
      if constexpr (t == 3) {
        vm_wait<8 * (NB4 - 2)>();      // stage s+1 landed: only s+2, s+3 may be in flight
        barrier();
      }
#endif
    });
  };
  // buffer index s % NB4 and register parity s % 2 repeat every UN stages
  constexpr int UN = NB4 % 2 ? 2 * NB4 : NB4;
  int s = 0;
  for (; s + UN <= nk; s += UN)
    static_for<0, UN>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      stage(std::integral_constant<int, j % NB4>(), std::integral_constant<int, j % 2>(), s + j);
    });
  // (a remainder of nk % UN stages is not supported: a per-stage switch here spilled ~400-570
  // VGPRs; kf_gemm_tn4 refuses such K)
  // no LDS-DMA may outlive the workgroup; the last MFMAs drain before their AGPRs are read
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const long m = m0 + 128 * wm + 16 * t + (lane & 15);
    bf16_t* crow = C + m * ldc + n0 + 128 * wn + 4 * (lane >> 4);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      bf16_t* p = crow + 16 * u;
      float v0 = acc[u][t][0], v1 = acc[u][t][1], v2 = acc[u][t][2], v3 = acc[u][t][3];
      if (ACC) {
        const u32x2 old = *reinterpret_cast<const u32x2*>(p);
        v0 += bflo(old[0]);
        v1 += bfhi(old[0]);
        v2 += bflo(old[1]);
        v3 += bfhi(old[1]);
      }
      *reinterpret_cast<u32x2*>(p) = u32x2{pack2(v0, v1), pack2(v2, v3)};
    }
  }
}

extern "C" int kf_gemm_tn4(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                           int accumulate, hipStream_t s) {
  constexpr int UN = g4::NB4 % 2 ? 2 * g4::NB4 : g4::NB4;
  if (!tn_shape_ok(A, lda, B, ldb, C, ldc, M, N, K) || K % (gm::BK * UN)) return 1;
  if (M == 0 || N == 0) return 0;
  TnGroup g{};
  g.p[0] = TnProblem{(const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, lda, ldb, ldc, M, N, accumulate,
                     (M / gm::BM) * (N / gm::BN)};
  g.n = 1;
  g.total = g.p[0].tiles;
  hipLaunchKernelGGL(gemm_tn4_kernel, dim3(g.total), dim3(256), 0, s, g, K);
  KF_CHECK_LAUNCH();
  return 0;
}
