// LAB COPY of ops/csrc/gemm.hip with the measured tuning knobs (KF_GEMM_NBUF, KF_GEMM_GROUP_M,
// KF_GEMM_DMA_STAGGER) and the anatomy switches (KF_ABL_*: numerics deliberately broken) that the
// shipped source no longer carries.  Defaults reproduce the shipped kernel.
//
// Weight-gradient GEMM for gfx950: C[M,N] (+)= A^T . B with A = [K, M] and B = [K, N], both
// row-major with the REDUCTION index K on the rows (dW = dY^T . X, K = tokens).
//
// hipBLASLt's TN ("Alik_Bljk") solutions for these shapes run at 1.0-1.2 PF against
// 1.45-1.55 PF for the NT forward GEMMs of the same size (tools/bench_gemm.py).  The
// layout is native to the gfx950 hardware-transpose LDS read: both operands are staged
// as k-row images and read column-wise with ds_read_b64_tr_b16 -- no transpose pass.
//
//  * 256 x 256 output tile per workgroup, 8 waves (2 along M x 4 along N), each wave a
//    128 x 64 sub-tile = 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators (128 VGPRs).  The
//    16x16x32 form holds a higher clock than 32x32x16 on random data (guide: DVFS).
//  * K is staged 32 rows at a time into a 5-deep LDS ring (5 x 32 KB = all 160 KB): each stage is four
//    [32][128 x bf16] images (A lo/hi, B lo/hi) with 256-B rows whose 32-byte blocks are
//    XOR-permuted by f(row) = (row & 3) | ((row >> 1) & 4): the two 16-lane groups of a
//    transposed read (rows r..r+3 and r+8..r+11, 16 columns) then hit 8 distinct blocks,
//    i.e. all 64 banks once, and the per-tile address is base ^ 32 t (one VGPR per tile).
//  * LDS-DMA (global_load_lds_dwordx4) runs four stages ahead; each stage's data is
//    published by ONE counted vmcnt + s_barrier in the middle of the previous stage, so the
//    operand reads can run four MFMA groups ahead across the stage seam.
//  * Operand reads are inline asm with hand-counted lgkmcnt waits (<= 15 in flight): hipcc
//    treats every compiler-visible LDS read as aliasing an in-flight LDS-DMA and would
//    insert vmcnt(0) before it.  The waits tie the destination registers, so no MFMA can be
//    hoisted above the wait for its operands.
//  * Products are computed as C^T tiles (operands swapped): each lane holds 4 consecutive
//    output columns -> 8-byte stores (and loads when accumulating).
//  * XCD-aware bijective block remap + grouped (4 M-tiles) raster: the workgroups of one
//    XCD share A and B panels in its L2.
//  * The four DMA pieces of a stage go out as one burst: one piece per MFMA group measured
//    0.5 % slower, and additionally staggering the two waves of a SIMD 4 % slower
//    (profiles/gemm_dw_raster_group.txt).
//  * s_setprio(1/0) around each MFMA group measured null (tools/kbench/gemm_bench: 1276 vs
//    1279 TF over the step's dW shapes), so the schedule is left to the counted waits.
//  * A 4-wave variant (2 x 2 waves of 128 x 128, 256 accumulators pinned to AGPRs with
//    inline-asm MFMAs, two-group-ahead operand reads) halves the LDS read rate but ran at
//    1210 TF vs 1275: at one wave per SIMD every wait/barrier bubble reaches the MFMA pipe.
//  * Anatomy (round 3, tools/kbench anatomy builds, K = 32768): removing the DMA pieces lifts the
//    loop from 1273 to 1645 TF, removing the barrier + vmcnt wait to 1383, removing the operand
//    reads to 1454, all three 1945; pieces that always hit L2 1453.  So the stage fetch is the
//    cost -- its issue and its memory latency, not LDS bandwidth.  Register staging (global
//    loads + ds_write_b128 one stage ahead) measured 1220 TF, i.e. worse; a fifth ring buffer
//    (one more stage of DMA lookahead) +4.6 %; staggering the two halves' DMA issue +1 % alone
//    and -2 % on top of the fifth buffer (profiles/gemm_dw_r3.md).
#include "common.h"   // (tools/kbench/build.sh puts ops/csrc on the include path)

using namespace kf;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace gm {
// K rows are staged BK at a time into an NBUF-deep LDS ring (KF_GEMM_NBUF: 4 = 128 KB, 5 = the
// full 160 KB with the DMA one stage further ahead: 1,316-1,319 vs 1,256-1,262 TF over the
// step's dW shapes at K = 32768 on one box, bit-identical output; profiles/gemm_dw_r3.md)
#ifndef KF_GEMM_NBUF
#define KF_GEMM_NBUF 5
#endif
constexpr int BM = 256, BN = 256, BK = 32, NBUF = KF_GEMM_NBUF;
static_assert(NBUF == 4 || NBUF == 5, "ring depth");
constexpr int IMG = BK * 256;               // one [32][128] bf16 image: 8 KB
constexpr int SMEM = 4 * NBUF * IMG;        // images laid out [image][buffer]: 128 / 160 KB
// M-tiles per raster group: 4 measured 1.0-1.3 % faster than 8 over the step's dW shapes on
// two boxes (16 / 32: -3 % / -6 %; tools/gpu_r2_gemm.sh); -DKF_GEMM_GROUP_M overrides
#ifndef KF_GEMM_GROUP_M
#define KF_GEMM_GROUP_M 4
#endif
constexpr int GROUP_M = KF_GEMM_GROUP_M;
// 1 = waves 4-7 issue their stage's DMA pieces four MFMA groups after waves 0-3 (see kernel)
#ifndef KF_GEMM_DMA_STAGGER
#define KF_GEMM_DMA_STAGGER 0
#endif

__device__ __forceinline__ int blk_x(int row) { return (row & 3) | ((row >> 1) & 4); }

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ u32 lds_addr(const char* p) { return (u32)(uintptr_t)LDS_PTR(char, p); }

// one 16x16x32 operand: two transposed reads, k-rows 8g..8g+3 and 8g+4..8g+7 (+1024 B)
template <int OFF>
__device__ __forceinline__ bf16x8 tr_frag(u32 addr) {
  u32x2 x, y;
  asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
               : "=&v"(x), "=v"(y)
               : "v"(addr), "i"(OFF), "i"(OFF + 1024));
  return __builtin_bit_cast(bf16x8, u32x4{x[0], x[1], y[0], y[1]});
}
// wait until at most N LDS operations are outstanding; ties the registers that become valid
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& a, bf16x8* b) {
  asm volatile("s_waitcnt lgkmcnt(%5)" : "+v"(a), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ int xcd_remap(int bid, int total) {
  const int q = total / 8, r = total % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// DMA one stage (32 k-rows of the A and B panels) into ring buffer `buf`.  32 wave-
// instructions of 1 KB (4 rows of 256 B); wave w issues w, w+8, w+16, w+24 = image
// (A lo, A hi, B lo, B hi) x 4 rows.  Lane L writes physical 16-B chunk L%16 of row
// 4j + L/16, i.e. block (L%16)/2, half L%2 -> it fetches logical block block ^ f(row).
// The per-lane source is a 32-bit byte offset from a wave-uniform panel pointer (SGPR
// base + VGPR offset addressing), precomputed once.
__device__ __forceinline__ void dma_offsets(long lda, long ldb, int wave, int lane, u32* off) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {          // instruction k of wave w: image k, rows 4w..4w+3
    const int row = 4 * wave + (lane >> 4), pc = lane & 15;
    const int col = 16 * ((pc >> 1) ^ blk_x(row)) + 8 * (pc & 1) + 128 * (k & 1);
    off[k] = (u32)(((k < 2 ? lda : ldb) * row + col) * 2);
  }
}
__device__ __forceinline__ const char* uniform_ptr(const char* p) {
  const uint64_t v = (uint64_t)p;
  return (const char*)(((uint64_t)__builtin_amdgcn_readfirstlane((u32)(v >> 32)) << 32) |
                       (u32)__builtin_amdgcn_readfirstlane((u32)v));
}
// m0 is set and consumed inside one asm statement (no other m0 user in this kernel)
#pragma clang diagnostic ignored "-Winline-asm"
// `lds` = wave-uniform LDS byte address of image 0 / buffer `buf` / this wave's 1 KB slot
__device__ __forceinline__ void stage_dma(const char* a, const char* b, const u32* off, u32 lds) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                 :
                 : "s"(lds + k * NBUF * IMG), "v"(off[k]), "s"(uniform_ptr(k < 2 ? a : b))
                 : "memory", "m0");
}
}  // namespace gm

using namespace gm;

// Wait counts before MFMA group t (reads issued after the youngest one group t needs; see
// the issue order in the kernel): nb0 a0 nb1 a1 nb2 a2 nb3 a3 | a4 a5 a6 a7 | nb0' a0' ...
template <int T> struct Cnt;
template <> struct Cnt<0> { static constexpr int v = 2; };
template <> struct Cnt<1> { static constexpr int v = 10; };
template <> struct Cnt<2> { static constexpr int v = 8; };
template <> struct Cnt<3> { static constexpr int v = 6; };
template <> struct Cnt<4> { static constexpr int v = 6; };
template <> struct Cnt<5> { static constexpr int v = 8; };
template <> struct Cnt<6> { static constexpr int v = 10; };
template <> struct Cnt<7> { static constexpr int v = 12; };

// Up to two independent products with the same K (the two weight gradients of one half of a
// decoder layer) share one launch: their tiles form one grid, so the partial last wave of
// one product is filled by tiles of the other (e.g. wo 256 + wqkv 384 tiles = 2.5 waves of
// 256 CUs instead of 1 + 1.5 rounded up to 3).
struct TnProblem {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  long lda, ldb, ldc;
  int M, N, acc, tiles;
};
struct TnGroup {
  TnProblem p[2];
  int n, total;
};

__global__ __launch_bounds__(512, 1) void gemm_tn_kernel(TnGroup grp, int K) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
  const int mt_n = M / BM, nt_n = N / BN;
  const int per_group = GROUP_M * nt_n;
  const int gid = lid / per_group, first_m = gid * GROUP_M;
  const int gsize = min(mt_n - first_m, GROUP_M);
  const int mt = first_m + (lid % per_group) % gsize, nt = (lid % per_group) / gsize;
  const long m0 = (long)mt * BM, n0 = (long)nt * BN;
  const int wm = wave & 1, wn = wave >> 1;          // wave sub-tile: rows 128 wm.., cols 64 wn..

  f32x4 acc[4][8];                                  // [n tile u][m tile t], C^T fragments
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addresses (buffer 0): lane 4q+p of 16-lane group g reads row 8g+q,
  // columns 16 t + 4p..4p+3 -> byte 256 row + 32 (t ^ f(row)) + 8p
  u32 aad[8], bad[4];
  {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, row = 8 * g + q;
    const u32 rb = lds_addr(smem) + row * 256 + 8 * p;
    const int f = blk_x(row);
#pragma unroll
    for (int t = 0; t < 8; ++t) aad[t] = rb + wm * NBUF * IMG + 32 * (t ^ f);
#pragma unroll
    for (int u = 0; u < 4; ++u) bad[u] = rb + (2 + (wn >> 1)) * NBUF * IMG + 32 * ((4 * (wn & 1) + u) ^ f);
  }

  const int nk = K / BK;
  const char* Ap = reinterpret_cast<const char*>(A + m0);
  const char* Bp = reinterpret_cast<const char*>(Bm + n0);
  const long astep = (long)BK * lda * 2, bstep = (long)BK * ldb * 2;
  u32 dmo[4];
  dma_offsets(lda, ldb, wave, lane, dmo);
  const u32 lds_w = __builtin_amdgcn_readfirstlane(lds_addr(smem) + 1024 * wave);
  // DMA issue point (KF_GEMM_DMA_STAGGER): waves 4-7 issue four MFMA groups after waves 0-3,
  // so the two waves sharing a SIMD do not stall on DMA issue at the same time
  const bool late = KF_GEMM_DMA_STAGGER && __builtin_amdgcn_readfirstlane(wave) >= 4;
  // prologue: stages 0..NBUF-2 in flight, publish stage 0, first operand reads
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < nk) stage_dma(Ap + s * astep, Bp + s * bstep, dmo, lds_w + s * IMG);
  if (nk >= NBUF - 1) vm_wait<4 * (NBUF - 2)>(); else vm_wait<0>();
  barrier();

  const char* dA = Ap + (NBUF - 1) * astep;   // next stage to DMA (loop-carried, wave-uniform)
  const char* dB = Bp + (NBUF - 1) * bstep;
  bf16x8 a[8], b[4], nb[4];
  nb[0] = tr_frag<0>(bad[0]);  a[0] = tr_frag<0>(aad[0]);
  nb[1] = tr_frag<0>(bad[1]);  a[1] = tr_frag<0>(aad[1]);
  nb[2] = tr_frag<0>(bad[2]);  a[2] = tr_frag<0>(aad[2]);
  nb[3] = tr_frag<0>(bad[3]);  a[3] = tr_frag<0>(aad[3]);

  // One ring revolution = NBUF stages, buffer index a compile-time immediate.
  auto stage = [&](auto bufc, int s) {
    constexpr int CB = decltype(bufc)::value, NX = (CB + 1) % NBUF;
    constexpr int OC = CB * IMG, ON = NX * IMG, OF = ((CB + NBUF - 1) % NBUF) * IMG;
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = nb[u];
    auto group = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t == 0) lgkm_wait<Cnt<0>::v>(a[0], b);
      else lgkm_wait<Cnt<t>::v>(a[t]);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u][t] = mfma16(b[u], a[t], acc[u][t]);
      if constexpr (t == 3) {
        // publish stage s+1 (its DMA went out NBUF-2 stages ago): wait until only the pieces
        // of the stages after it that exist are outstanding
        // (KF_ABL_* : anatomy builds for tools/kbench only -- numerics deliberately broken)
#ifndef KF_ABL_NOVMW
        if constexpr (NBUF == 5) {
          if (s + 3 < nk) vm_wait<8>(); else if (s + 2 < nk) vm_wait<4>(); else vm_wait<0>();
        } else {
          if (s + 2 < nk) vm_wait<4>(); else vm_wait<0>();
        }
#endif
#ifndef KF_ABL_NOBAR
        barrier();
#endif
      }
      // refill the buffer every wave has finished with (stage s-1's) with stage s+NBUF-1
      if constexpr (t == 3 || t == 7) {
        if ((t == 3) != late && s + NBUF - 1 < nk) {
#ifndef KF_ABL_NODMA
#ifdef KF_ABL_DMASAME
          stage_dma(Ap, Bp, dmo, lds_w + OF);   // always the (L2-resident) first panel rows
#else
          stage_dma(dA, dB, dmo, lds_w + OF);
#endif
#endif
          dA += astep;
          dB += bstep;
        }
      }
#ifndef KF_ABL_NOREAD
      if constexpr (t >= 4) nb[t - 4] = tr_frag<ON>(bad[t - 4]);
      if constexpr (t < 4) a[t + 4] = tr_frag<OC>(aad[t + 4]);
      else a[t - 4] = tr_frag<ON>(aad[t - 4]);
#endif
    };
    group(std::integral_constant<int, 0>());
    group(std::integral_constant<int, 1>());
    group(std::integral_constant<int, 2>());
    group(std::integral_constant<int, 3>());
    group(std::integral_constant<int, 4>());
    group(std::integral_constant<int, 5>());
    group(std::integral_constant<int, 6>());
    group(std::integral_constant<int, 7>());
  };
  // the ring revolution is unrolled; a K that is not a multiple of NBUF stages leaves the
  // last revolution early (wave-uniform)
  int s = 0;
  for (; s + NBUF <= nk; s += NBUF) {
    stage(std::integral_constant<int, 0>(), s);
    stage(std::integral_constant<int, 1>(), s + 1);
    stage(std::integral_constant<int, 2>(), s + 2);
    stage(std::integral_constant<int, 3>(), s + 3);
    if constexpr (NBUF == 5) stage(std::integral_constant<int, 4 % NBUF>(), s + 4);
  }
  if constexpr (NBUF == 5) {
    const int rem = nk - s;
    if (rem >= 1) stage(std::integral_constant<int, 0>(), s);
    if (rem >= 2) stage(std::integral_constant<int, 1>(), s + 1);
    if (rem >= 3) stage(std::integral_constant<int, 2>(), s + 2);
    if (rem >= 4) stage(std::integral_constant<int, 3>(), s + 3);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // acc[u][t] = C^T fragment: lane l, reg r -> n = 16u + 4(l>>4) + r, m = 16t + (l&15)
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const long m = m0 + 128 * wm + 16 * t + (lane & 15);
    bf16_t* crow = C + m * ldc + n0 + 64 * wn + 4 * (lane >> 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
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

static bool tn_shape_ok(const void* A, long lda, const void* B, long ldb, const void* C, long ldc, int M, int N,
                        int K) {
  if (M % BM || N % BN || K % (NBUF == 4 ? BK * NBUF : BK) || K < BK || lda % 8 || ldb % 8 || ldc % 4) return false;
  return !(((uintptr_t)A | (uintptr_t)B) & 15) && !((uintptr_t)C & 7);
}

extern "C" int kf_gemm_tn(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                          int accumulate, hipStream_t s) {
  if (!tn_shape_ok(A, lda, B, ldb, C, ldc, M, N, K)) return 1;
  if (M == 0 || N == 0) return 0;
  TnGroup g{};
  g.p[0] = TnProblem{(const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, lda, ldb, ldc, M, N, accumulate, (M / BM) * (N / BN)};
  g.n = 1;
  g.total = g.p[0].tiles;
  hipLaunchKernelGGL(gemm_tn_kernel, dim3(g.total), dim3(512), 0, s, g, K);
  KF_CHECK_LAUNCH();
  return 0;
}

// two products C_i (+)= A_i^T B_i over the same K in one launch (see TnGroup)
extern "C" int kf_gemm_tn2(const void* A0, long lda0, const void* B0, long ldb0, void* C0, long ldc0, int M0, int N0,
                           const void* A1, long lda1, const void* B1, long ldb1, void* C1, long ldc1, int M1, int N1,
                           int K, int accumulate, hipStream_t s) {
  if (!tn_shape_ok(A0, lda0, B0, ldb0, C0, ldc0, M0, N0, K) || !tn_shape_ok(A1, lda1, B1, ldb1, C1, ldc1, M1, N1, K))
    return 1;
  TnGroup g{};
  g.p[0] = TnProblem{(const bf16_t*)A0, (const bf16_t*)B0, (bf16_t*)C0, lda0, ldb0, ldc0, M0, N0, accumulate,
                     (M0 / BM) * (N0 / BN)};
  g.p[1] = TnProblem{(const bf16_t*)A1, (const bf16_t*)B1, (bf16_t*)C1, lda1, ldb1, ldc1, M1, N1, accumulate,
                     (M1 / BM) * (N1 / BN)};
  g.n = 2;
  g.total = g.p[0].tiles + g.p[1].tiles;
  if (g.total == 0) return 0;
  hipLaunchKernelGGL(gemm_tn_kernel, dim3(g.total), dim3(512), 0, s, g, K);
  KF_CHECK_LAUNCH();
  return 0;
}
