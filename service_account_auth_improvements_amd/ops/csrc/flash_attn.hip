// K3: causal GQA flash attention for gfx950 (MI355X), head_dim 128, bf16 in/out.
//
// Reads q/k/v straight from the fused QKV activation [B*S, (Hq + 2*Hkv)*128] (row stride
// `ld`), writes O as [B*S, Hq*128] and the per-row natural log-sum-exp [B, Hq, S].
//
// Shared building blocks (all kernels):
//  * v_mfma_f32_32x32x16_bf16 everywhere.  The "swapped" products keep the QUERY on the
//    MFMA lane (S^T = K.Q^T, O^T = V^T.P^T, dQ^T = K^T.dS^T) so softmax statistics,
//    rescales and row constants are lane-local; an accumulator whose rows are the
//    reduction index of the next product is fed to it as the B operand unchanged
//    (converted pairwise to bf16), and the matching A operand is read with the gfx950
//    hardware-transpose ds_read_b64_tr_b16.
//  * Every [rows x 128] bf16 tile lives in LDS as 256-B rows with the XOR chunk swizzle
//    `swz` that is conflict-free for both row reads (ds_read_b128) and transposed reads.
//  * Tiles are staged by LDS-DMA (global_load_lds_dwordx4, no VGPRs): the destination
//    of a wave-instruction is lane-linear, so the swizzle is applied to the per-lane
//    SOURCE address (the XOR is an involution).  The next tile's DMA is issued before
//    the current tile's MFMAs; one vmcnt(0)+barrier per tile publishes it.
//  * XCD-aware bijective block remap: blocks resident on one XCD share one (batch,
//    kv-head), so its K/V (fwd, dQ) or Q/dO (dK/dV) stay in that XCD's 4 MB L2; causal
//    work is launched heaviest-first.
//
// Forward: 1 workgroup = 8 waves x 32 query rows, 128-key tiles in a 2-deep LDS-DMA ring,
// online softmax (exp2) with the running max folded into the MFMA chain (see the kernel).
// Backward, two kernels, no dQ atomics:
//  * dQ kernel (forward-shaped, per 128 query rows): S^T, dP^T = V.dO^T, P^T, dS^T,
//    dQ^T += K^T.dS^T; dQ written once as bf16 into the dqkv buffer.
//  * dK/dV kernel (per 128-key block x query chunk, all G query heads of the GQA group):
//    S = Q.K^T and dP = dO.V^T with the KEY on the lane (accumulators pre-loaded with
//    -lse/scale and -delta, the "row constants"), dV^T += dO^T.P, dK^T += Q^T.dS; each
//    wave keeps its 32 keys' dK^T/dV^T (128 registers) across the chunk; chunk partial
//    sums are transposed through LDS and added row-contiguously in fp32.
//  * The two kernels run concurrently: dQ on the caller's stream, the accumulator memset and
//    dK/dV on a per-device side stream (event fork/join, see kf_flash_bwd).
// Measured alternatives (round 5, profiles/fa_dkdv2_r5.md, profiles/dq_atomic_r5.md): a one-wave-
// per-SIMD dK/dV with 64-row iterations and the next S/dP chain under the softmax (15 % slower),
// a fused dK/dV + dQ (its fp32 dQ atomics alone take 6.7 ms per layer at B4 S8192, more than
// this whole backward), the forward's next-tile S chain under the current softmax (2 % slower),
// and one stream for both backward kernels (same step time).  The matrix pipe is 50-60 % busy
// in all three kernels (PMC, same file).
#include "common.h"

#include <mutex>

#include <cstdlib>

using namespace kf;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace fa {
constexpr int D = 128;
constexpr int BQ = 128;           // sequence-length granule the launchers require (S % BQ == 0)
constexpr int BK = 64;            // keys per dQ half-stage (stages hold BKF = 128)
constexpr int BKV = 128;          // keys per dK/dV workgroup (4 waves x 32)
constexpr int QT = 32;            // query rows per dK/dV iteration
constexpr int QCH = 1536;         // query rows per dK/dV work item: 1536 is 1.1 % faster than 1024 and 1280-2048
                                  // (profiles/fa_fwd128_r5.md; 512: 6 % slower in round 3)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ int swz_x(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
// byte offset of 16-byte chunk `ch` (0..15) of row `row` in a [rows][128 x bf16] LDS image
__device__ __forceinline__ int swz(int row, int ch) { return row * 256 + 16 * (ch ^ swz_x(row)); }
// byte offset of the 8 bytes at column `col` (multiple of 4) of row `row`
__device__ __forceinline__ int swz8(int row, int col) { return swz(row, col >> 3) + 8 * ((col >> 2) & 1); }

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 as_bf16x8(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// LDS-DMA of one 16-B piece per lane; `lds` must be wave-uniform (lands at lds + 16*lane)
__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}
// One LDS-DMA wave-instruction (16 B per lane) from a wave-uniform panel base (SGPRs) plus a
// 32-bit lane byte offset, landing at the wave-uniform LDS byte address `lds` (m0)
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ const char* uniform_ptr(const char* p) {
  const uint64_t v = (uint64_t)p;
  return (const char*)(((uint64_t)__builtin_amdgcn_readfirstlane((u32)(v >> 32)) << 32) |
                       (u32)__builtin_amdgcn_readfirstlane((u32)v));
}
__device__ __forceinline__ void dma_sv(const char* base, u32 off, u32 lds) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(off), "s"(uniform_ptr(base))
               : "memory", "m0");
}
// Stage `nrows` rows of 128 bf16 (global row stride ld) into the swizzled image at `tile`.
// Wave-instruction i fills LDS bytes [1024 i, 1024 i + 1024) = rows 4i..4i+3; lane L of it
// writes physical chunk L%16 of row 4i + L/16 and therefore fetches logical chunk
// (L%16) ^ swz_x(row).
__device__ __forceinline__ void stage_rows(const bf16_t* g, long ld, char* tile, int nrows, int wave,
                                           int nwaves, int lane) {
  for (int i = wave; i < nrows / 4; i += nwaves) {
    const int row = 4 * i + (lane >> 4);
    const int ch = (lane & 15) ^ swz_x(row);
    glds16(g + (long)row * ld + ch * 8, tile + 1024 * i);
  }
}
__device__ __forceinline__ void wait_dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// Bijective XCD remap: blocks b and b+8 share an XCD; give each XCD a contiguous range
// of logical ids (guide §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int bid, int total) {
  const int q = total / 8, r = total % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

struct QBlock {
  int b, h, hkv, qb;
};
// forward / dQ block decode: logical order [b][hkv][q-block (heavy first)][g]
__device__ __forceinline__ QBlock decode_qblock(int S, int Hq, int Hkv, int B, bool causal) {
  const int nqb = S / BQ, G = Hq / Hkv;
  const int lid = xcd_remap(blockIdx.x, B * Hq * nqb);
  QBlock r;
  const int g = lid % G;
  int t1 = lid / G;
  r.qb = t1 % nqb;
  t1 /= nqb;
  r.hkv = t1 % Hkv;
  r.b = t1 / Hkv;
  if (causal) r.qb = nqb - 1 - r.qb;
  r.h = r.hkv * G + g;
  return r;
}
}  // namespace fa

using namespace fa;

// xor-32 lane reductions by v_permlane32_swap (no LDS round trip on the softmax path)
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float bf16_round(float x) { return (float)(__bf16)x; }
__device__ __forceinline__ u32 lds_addr(const void* p) { return (u32)(uintptr_t)LDS_PTR(const char, p); }
// one MFMA operand fragment = two transposed 4x16 reads, in inline asm: hipcc treats every
// compiler-visible LDS read as aliasing an in-flight LDS-DMA and would wait vmcnt(0) first
__device__ __forceinline__ bf16x8 tr_pair_asm(u32 a0, u32 a1) {
  u32x2 x, y;
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3" : "=&v"(x), "=v"(y) : "v"(a0), "v"(a1) : "memory");
  return as_bf16x8(u32x4{x[0], x[1], y[0], y[1]});
}
// wait until at most N LDS operations are outstanding; ties the fragments that become valid
template <int N>
__device__ __forceinline__ void lgkm_wait_tie(bf16x8* f) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]) : "i"(N) : "memory");
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
// Inline-asm LDS reads with an immediate offset (the per-lane part in one VGPR); the caller
// waits for them with counted, register-tying lgkmcnt waits (lgkm_tie*)
template <int OFF>
__device__ __forceinline__ bf16x8 rd_b128(u32 a) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return as_bf16x8(r);
}
template <int OFF>
__device__ __forceinline__ bf16x8 rd_tr2(u32 a0, u32 a1) {
  u32x2 x, y;
  asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%4\n\tds_read_b64_tr_b16 %1, %3 offset:%4"
               : "=&v"(x), "=v"(y)
               : "v"(a0), "v"(a1), "i"(OFF)
               : "memory");
  return as_bf16x8(u32x4{x[0], x[1], y[0], y[1]});
}
template <int OFF>
__device__ __forceinline__ float rd_b32(u32 a) {
  float r;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}
template <int OFF>
__device__ __forceinline__ f32x4 rd_f4(u32 a) {
  f32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}
// transposed pair from one address: rows at OFF and OFF + 4096 (16 rows of 256 B further)
template <int OFF>
__device__ __forceinline__ bf16x8 rd_tr2i(u32 a) {
  u32x2 x, y;
  asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
               : "=&v"(x), "=v"(y)
               : "v"(a), "i"(OFF), "i"(OFF + 4096)
               : "memory");
  return as_bf16x8(u32x4{x[0], x[1], y[0], y[1]});
}
template <int N>
__device__ __forceinline__ void lgkm_tie1(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_tie3(bf16x8& a, bf16x8& b, bf16x8& c) {
  asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_tie_f2(float& a, float& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N) : "memory");
}
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    static_for<I + 1, N>(f);
  }
}
template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
// Row constant folded into an MFMA chain as one extra k-chunk: A holds a ones column at
// k = 0, 1 and B the (hi, lo) bf16 split of -c for this lane's row, so the product adds
// -c (to ~2^-16 relative) to every accumulator element of the row.
__device__ __forceinline__ bf16x8 fold_ones(int hh) {
  return hh ? bf16x8{} : bf16x8{(__bf16)1.f, (__bf16)1.f, 0, 0, 0, 0, 0, 0};
}
__device__ __forceinline__ bf16x8 fold_const(float c, int hh) {
  const __bf16 hi = (__bf16)(-c);
  const __bf16 lo = (__bf16)(-c - (float)hi);
  return hh ? bf16x8{} : bf16x8{hi, lo, 0, 0, 0, 0, 0, 0};
}

// ====================================================================================
// Forward
// ====================================================================================
// 1 workgroup = 8 waves x 32 query rows (256 rows), one workgroup per CU (2 waves per SIMD).
//  * K/V 128-key tiles arrive by LDS-DMA in a 2-deep ring of K+V stages (2 x 64 KB): the DMA
//    runs one tile ahead, and each tile is published by a vmcnt + raw s_barrier.  Each staged
//    tile feeds 8 waves.  128-key tiles measured 4.6 % faster than 64-key tiles in a 4-deep
//    ring (2.14 vs 2.24 ms at B4 S8192, same numerics): one barrier, one max / sum exchange and
//    one threshold ballot per 128 keys (profiles/fa_fwd128_r5.md).
//  * The loop is VALU-issue bound (two waves share a SIMD's vector issue; an MFMA holds it
//    for 8 of its 32 cycles), so the softmax is put on a diet: the running row max m
//    (bf16-exact) rides in the S^T MFMA chain as a folded row constant, so p = exp2(c S')
//    needs no subtraction.  m only moves (rescaling O, l and the tile) when a row's tile max
//    exceeds it by > 2^8, which after the first tiles is rare -- the per-tile rescale of the
//    usual online softmax is gone.  (Measured: +10 % over the FMA form; an MFMA row sum
//    instead of the VALU adds and static younger-half priority were both slower or null.)
//  * V^T fragments for PV group g+1 are read while group g's MFMAs run.
// The dQ kernel stages K/V the same way but computes each 128-key stage as two 64-key halves
// (its S and dP chains hold twice the forward's accumulators): 2.81 vs 2.86 ms, the same
// numerics (profiles/fa_fwd128_r5.md).
constexpr int BQ8 = 256;                            // query rows per forward / dQ workgroup
constexpr float FOLD_T = 8.f;                       // tolerated growth of p above 1 (log2)

// lane id from v_mbcnt in asm volatile: recomputed where used, never kept live in a VGPR
__device__ __forceinline__ u32 lane_id_opaque() {
  u32 x;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(x));
  return x;
}
// K row fragments are read by inline asm FP MFMA steps ahead; tiles staged by SGPR-base DMA
// (the compiler-scheduled form waited lgkmcnt(0) before every MFMA: profiles/fa_fwd_pipe_ab.txt;
// 2 / 4 / 5 steps ahead measured the same in the 128-key forward)
constexpr int FP = 3;
// (measured and removed: ping-pong wave roles -- waves 4-7 taking each tile's barrier after their
// S chain -- 2.31-2.36 vs 2.23-2.25 ms, profiles/fa_fwd_pingpong_ab.txt)
constexpr int BKF = 128;                 // keys per K/V stage (forward and dQ)
constexpr int TILEF = BKF * D * 2;       // 32 KB
constexpr int NSF = 2;                   // ring depth (stages of K + V)
constexpr int STGF = 2 * TILEF;
constexpr int NKT = BKF / 32;            // 32-key chunks per tile
static_assert(NSF * STGF <= 163840, "LDS");
// Epilogue of the forward and dQ kernels: a wave's 32 x 128 output tile (the O^T-layout
// accumulators, already scaled) goes through 8 KB of the ring buffer the last stage did not use
// (swizzled 16-B chunks, wave-local, so no workgroup barrier), then out as whole 256-B rows: 16 B
// per lane, 4 rows per store instruction.  The per-lane 8-B stores it replaces touched 32 rows per
// instruction; 0.5-1.2 % faster kernels (profiles/fa_fwd128_r5.md).
__device__ __forceinline__ void store_rows_via_lds(const f32x16 (&v)[4], float mul, char* ob, bf16_t* orow,
                                                   long ldr) {
  // the lane id is recomputed here (v_mbcnt), not kept live across the main loop
  const int l = (int)lane_id_opaque(), lr = l & 31, hh = l >> 5;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      u32x2 p;
      p[0] = pack2(v[t][4 * gq] * mul, v[t][4 * gq + 1] * mul);
      p[1] = pack2(v[t][4 * gq + 2] * mul, v[t][4 * gq + 3] * mul);
      // row lr, output columns 32 t + 8 gq + 4 hh .. + 3: 16-B chunk 4 t + gq, half hh
      *reinterpret_cast<u32x2*>(ob + swz(lr, 4 * t + gq) + 8 * hh) = p;
    }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 4 * i + (l >> 4), ch = l & 15;
    st16(orow + (long)row * ldr + 8 * ch, *reinterpret_cast<const u32x4*>(ob + swz(row, ch)));
  }
}
// NW waves per workgroup: 8 (256 query rows, 128-key K/V stages, one workgroup per CU) or 4 (128
// rows, 64-key stages in 64 KB of LDS, two workgroups per CU with independent stage barriers)
template <int NW> struct FwdCfg {
  static constexpr int RW = 32 * NW;              // query rows per workgroup
  static constexpr int BKS = NW == 8 ? 128 : 64;  // keys per K/V stage
  static constexpr int KT = BKS / 32;             // 32-key chunks per stage
  static constexpr int HF = BKS / 64;             // 64-key halves per stage (PV groups: 4 HF)
  static constexpr int TILE = BKS * D * 2;
  static constexpr int STG = 2 * TILE;
  static constexpr int NDI = BKS / (4 * NW);      // DMA wave-instructions per wave per tile
};
template <bool CAUSAL, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void flash_fwd_kernel(
    const bf16_t* __restrict__ qkv, long ld, bf16_t* __restrict__ out, long ldo,
    float* __restrict__ lse_out, int B, int S, int Hq, int Hkv, float scale_log2) {
  using C = FwdCfg<NW>;
  constexpr int RW = C::RW, BKS = C::BKS, NKTL = C::KT, HF = C::HF, TILE = C::TILE, STG = C::STG;
  static_assert(NSF * STG <= 163840 && C::NDI * 4 * NW == BKS, "forward stage layout");
  __shared__ __attribute__((aligned(1024))) char smem[NSF * STG];
  const int nqb = (S + RW - 1) / RW, G = Hq / Hkv;
  // logical order [b][hkv][q-block][g]: an XCD's contiguous range shares one K/V panel
  int lid = xcd_remap(blockIdx.x, B * Hq * nqb);
  const int g = lid % G;
  lid /= G;
  int qb = lid % nqb;
  lid /= nqb;
  const int hkv = lid % Hkv, b = lid / Hkv, h = hkv * G + g;
  if (CAUSAL) qb = nqb - 1 - qb;   // heaviest blocks first

  const int tid = threadIdx.x, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = qb * RW + w * 32 + lr;
  const int qmin_w = qb * RW + w * 32, qmax_w = qmin_w + 31;
  const bool live = qmin_w < S;   // the last block of S % 256 == 128 has 4 idle waves

  bf16x8 qf[8];  // B operand of S^T = K Q^T: Q[q][16ks + 8hh .. +8]
  {
    const bf16_t* qp = qkv + ((long)b * S + min(q, S - 1)) * ld + (long)h * D + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = as_bf16x8(ld16(qp + 16 * ks));
  }
  const bf16_t* kp = qkv + (long)b * S * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + (long)b * S * ld + (long)(Hq + Hkv + hkv) * D;
  u32 dma_kv;   // see the dQ kernel: one lane offset for the K and V panels
  {
    const int row = 4 * w + (l >> 4), ch = (l & 15) ^ swz_x(row);
    dma_kv = (u32)((row * ld + ch * 8) * 2);
  }
  const u32 lds_w = lds_addr(smem) + 1024 * w;
  // 8 DMA wave-instructions per wave per stage: the 32-row segments i of the K and V tiles
  auto stage = [&](int j) {
    const u32 st = lds_w + (j % NSF) * STG;
    const char* kb_ = reinterpret_cast<const char*>(kp + (long)j * BKS * ld);
    const char* vb_ = reinterpret_cast<const char*>(vp + (long)j * BKS * ld);
#pragma unroll
    for (int i = 0; i < C::NDI; ++i) dma_sv(kb_ + (long)8 * NW * ld * i, dma_kv, st + 1024 * NW * i);
#pragma unroll
    for (int i = 0; i < C::NDI; ++i) dma_sv(vb_ + (long)8 * NW * ld * i, dma_kv, st + TILE + 1024 * NW * i);
  };
  const int ntiles = CAUSAL ? min(S, qb * RW + RW) / BKS : S / BKS;
  if (ntiles > 0) stage(0);

  // retire the Q loads HERE (the compiler's wait counts only them, the DMA stays in flight):
  // a first use inside the loop would make hipcc wait vmcnt(0) on every tile
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) asm volatile("" : "+v"(qf[ks]));
  const bf16x8 ones = fold_ones(hh);
  bf16x8 mref = bf16x8{};    // folded -m (m bf16-exact: the hi part carries it, lo = 0)
  bool first = true;
  const float thresh = FOLD_T / scale_log2;   // m and S' are in raw score units
  float m = 0.f, lsum = 0.f;
  f32x16 o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = f32x16{};
  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

  // S'^T = K Q^T - m of tile j: key on the accumulator rows, query on the lane; K row fragments
  // by inline asm, FP steps ahead, the four 32-key chains alternating
  auto s_chain = [&](int j, f32x16 (&sc)[NKTL]) {
    const u32 ln = lane_id_opaque(), lr_ = ln & 31;
    const u32 a_t = (lds_addr(smem) + (u32)((j % NSF) * STG)) + lr_ * 256 + 16 * ((ln >> 5) ^ swz_x(lr_));
    bf16x8 fk[FP + 1];
    auto rdK = [&](auto ic) {
      constexpr int i = decltype(ic)::value, kt = i % NKTL, ks = i / NKTL;
      fk[i % (FP + 1)] = rd_b128<8192 * kt>(a_t ^ (32 * ks));
    };
    static_for<0, FP>([&](auto ic) { rdK(ic); });
#pragma unroll
    for (int kt = 0; kt < NKTL; ++kt) sc[kt] = mfma32(ones, mref, f32x16{});
    static_for<0, 8 * NKTL>([&](auto ic) {
      constexpr int i = decltype(ic)::value, kt = i % NKTL, ks = i / NKTL, NI = 8 * NKTL;
      if constexpr (i + FP < NI) rdK(std::integral_constant<int, i + FP>());
      lgkm_tie1<(i + FP < NI ? FP : NI - 1 - i)>(fk[i % (FP + 1)]);
      sc[kt] = mfma32(fk[i % (FP + 1)], qf[ks], sc[kt]);
    });
  };
  // causal mask, online softmax, O^T += V^T P^T of tile j
  auto soft_pv = [&](int j, f32x16 (&sc)[NKTL]) {
    const int k0 = j * BKS;
    const char* Vs = smem + (j % NSF) * STG + TILE;
    if (CAUSAL && k0 + BKS - 1 > qmin_w) {   // a wave's diagonal tiles only (uniform branch)
#pragma unroll
      for (int kt = 0; kt < NKTL; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
          sc[kt][r] = key > q ? -INFINITY : sc[kt][r];
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKTL; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kt][r]);
    mx = xor32_max(mx);
    if (__ballot(first || mx > thresh)) {
      // move the reference: m' = bf16(m + max(mx, 0)); rescale O, l and this tile's S'
      const float mnew = first ? bf16_round(mx) : bf16_round(m + fmaxf(mx, 0.f));
      const float shift = first ? mnew : mnew - m;
      const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-shift * scale_log2);
      lsum *= alpha;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
#pragma unroll
      for (int kt = 0; kt < NKTL; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[kt][r] -= shift;
      m = mnew;
      first = false;
      mref = fold_const(m, hh);
    }
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKTL; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(sc[kt][r] * scale_log2);
        sc[kt][r] = p;
        rs += p;
      }
    lsum += xor32_sum(rs);
    bf16x8 pf[NKTL][2];
#pragma unroll
    for (int kt = 0; kt < NKTL; ++kt)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        u32x4 u;
#pragma unroll
        for (int i = 0; i < 4; ++i) u[i] = pack2(sc[kt][8 * ss + 2 * i], sc[kt][8 * ss + 2 * i + 1]);
        pf[kt][ss] = as_bf16x8(u);
      }
    // O^T += V^T P^T in 8 groups (output block t, key half hf); group g+1's V^T fragments are
    // read while group g's MFMAs run
    const u32 vbase = lds_addr(Vs);
    bf16x8 vf[2][4];
    auto v_read = [&](int gi, bf16x8* f) {
      const int t = gi / HF, hf = gi % HF;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int row = 32 * (2 * hf + kk) + 16 * ss + vrow, col = 32 * t + vcol;
          f[2 * kk + ss] = tr_pair_asm(vbase + swz8(row, col), vbase + swz8(row + 8, col));
        }
    };
    v_read(0, vf[0]);
#pragma unroll
    for (int gi = 0; gi < 4 * HF; ++gi) {
      if (gi < 4 * HF - 1) {
        v_read(gi + 1, vf[(gi + 1) & 1]);
        lgkm_wait_tie<8>(vf[gi & 1]);
      } else {
        lgkm_wait_tie<0>(vf[gi & 1]);
      }
      const int t = gi / HF, hf = gi % HF;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) o[t] = mfma32(vf[gi & 1][2 * kk + ss], pf[2 * hf + kk][ss], o[t]);
    }
  };
  auto live_tile = [&](int j) { return live && (!CAUSAL || j * BKS <= qmax_w); };

  vm_wait<0>();
  barrier();
  f32x16 scp[NKTL];
  for (int j = 0; j < ntiles; ++j) {
    if (j + 1 < ntiles) stage(j + 1);   // into the buffer every wave finished with (tile j-1)
    if (live_tile(j)) {
      s_chain(j, scp);
      soft_pv(j, scp);
    }
    if (j + 1 < ntiles) {
      vm_wait<0>();
      barrier();
    }
  }
  if (!live) return;
  const float inv = 1.f / lsum;
  store_rows_via_lds(o, inv, smem + (ntiles % NSF) * STG + 8192 * w, out + ((long)b * S + qmin_w) * ldo + (long)h * D,
                     ldo);
  if (hh == 0) lse_out[((long)b * Hq + h) * S + q] = (m * scale_log2 + log2f(lsum)) * LN2;
}

// ====================================================================================
// Backward: delta = rowsum(dO * O)
// ====================================================================================
__global__ __launch_bounds__(256) void flash_bwd_pre_kernel(const bf16_t* __restrict__ o, long ldo,
                                                            const bf16_t* __restrict__ dout, long lddo,
                                                            float* __restrict__ delta, int B, int S,
                                                            int Hq) {
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);   // over B*S*Hq, 16 lanes per row
  const int sub = threadIdx.x & 15;
  const int total = B * S * Hq;
  float acc = 0.f;
  int t = 0, h = 0;
  if (row < total) {
    t = row / Hq;
    h = row - t * Hq;
    float a[8], bb[8];
    unpack8(ld16(o + (long)t * ldo + h * 128 + sub * 8), a);
    unpack8(ld16(dout + (long)t * lddo + h * 128 + sub * 8), bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * bb[j];
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < total && sub == 0) {
    const int bidx = t / S, q = t - bidx * S;
    delta[((long)bidx * Hq + h) * S + q] = acc;
  }
}

// ====================================================================================
// Backward: dQ (forward-shaped)
// ====================================================================================
// Same skeleton as the forward (8 waves x 32 query rows, 128-key K+V stages in a 2-deep LDS-DMA
// ring, one vmcnt + raw barrier per stage, each stage computed as two 64-key halves).  Per 64-key
// half: S'^T = K Q^T - lse/scale and dP'^T = V dO^T - delta
// come out of the MFMA chains with both row constants folded in (hi/lo bf16 split, no
// accumulator-initialising moves), so dS^T = exp2(c S') * dP' per element; dQ^T += K^T dS^T
// with the K^T fragments read (inline asm, counted waits) one output block ahead.
// K/V row fragments by inline asm, QP k-steps ahead; -lse enters through the exp's FMA (a
// per-lane constant) instead of a folded MFMA per 32-key chain (profiles/fa_dq_lsefma_ab.txt)
constexpr int QP = 1;
template <int N>
__device__ __forceinline__ void lgkm_tie2(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N) : "memory");
}
// NW waves per workgroup: 8 (256 query rows, 128-key stages computed as two 64-key halves, one
// workgroup per CU) or 4 (128 rows, 64-key stages, 64 KB of LDS: two workgroups per CU whose
// stage barriers are independent, so the two waves sharing a SIMD are not phase-locked)
template <int NW> struct DqCfg {
  static constexpr int RW = 32 * NW;              // query rows per workgroup
  static constexpr int BKS = NW == 8 ? 128 : 64;  // keys per K/V stage
  static constexpr int TILE = BKS * D * 2;        // one K (or V) tile
  static constexpr int STG = 2 * TILE;
  static constexpr int NH = BKS / BK;             // 64-key halves per stage
  static constexpr int NI = BKS / (4 * NW);       // DMA wave-instructions per wave per tile
};
template <bool CAUSAL, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void flash_bwd_dq_kernel(
    const bf16_t* __restrict__ qkv, long ld, const bf16_t* __restrict__ dout, long lddo,
    const float* __restrict__ lse, const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    long lddq, int B, int S, int Hq, int Hkv, float scale_log2, float scale) {
  using C = DqCfg<NW>;
  constexpr int RW = C::RW, BKS = C::BKS, TILE = C::TILE, STG = C::STG;
  static_assert(NSF * STG <= 163840 && C::NI * 4 * NW == BKS, "dQ stage layout");
  __shared__ __attribute__((aligned(1024))) char smem[NSF * STG];
  const int nqb = (S + RW - 1) / RW, G = Hq / Hkv;
  int lid = xcd_remap(blockIdx.x, B * Hq * nqb);
  const int g = lid % G;
  lid /= G;
  int qb = lid % nqb;
  lid /= nqb;
  const int hkv = lid % Hkv, b = lid / Hkv, h = hkv * G + g;
  if (CAUSAL) qb = nqb - 1 - qb;

  const int tid = threadIdx.x, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = qb * RW + w * 32 + lr, qc = min(q, S - 1);
  const int qmin_w = qb * RW + w * 32, qmax_w = qmin_w + 31;
  const bool live = qmin_w < S;

  bf16x8 qf[8], df[8];
  {
    const bf16_t* qp = qkv + ((long)b * S + qc) * ld + (long)h * D + 8 * hh;
    const bf16_t* dp_ = dout + ((long)b * S + qc) * lddo + (long)h * D + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      qf[ks] = as_bf16x8(ld16(qp + 16 * ks));
      df[ks] = as_bf16x8(ld16(dp_ + 16 * ks));
    }
  }
  float lse_s = lse[((long)b * Hq + h) * S + qc] / scale;   // lse in raw score units
  float dl = delta[((long)b * Hq + h) * S + qc];
  const bf16_t* kp = qkv + (long)b * S * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + (long)b * S * ld + (long)(Hq + Hkv + hkv) * D;
  // wave w fills rows 4w.., 4w+4NW.. of the K and V images: SGPR panel base + one 32-bit lane
  // offset shared by K and V (same row stride; rows 16 apart share the chunk swizzle)
  u32 dma_kv;
  {
    const int row = 4 * w + (l >> 4), ch = (l & 15) ^ swz_x(row);
    dma_kv = (u32)((row * ld + ch * 8) * 2);
  }
  const u32 lds_w = lds_addr(smem) + 1024 * w;
  // a stage is 128 keys of K and V (the forward's staging: 8 DMA wave-instructions per wave,
  // 2-deep ring), computed as two 64-key halves under one barrier
  auto stage = [&](int j) {
    const u32 st = lds_w + (j % NSF) * STG;
    const char* kb_ = reinterpret_cast<const char*>(kp + (long)j * BKS * ld);
    const char* vb_ = reinterpret_cast<const char*>(vp + (long)j * BKS * ld);
#pragma unroll
    for (int i = 0; i < C::NI; ++i) dma_sv(kb_ + (long)8 * NW * ld * i, dma_kv, st + 1024 * NW * i);
#pragma unroll
    for (int i = 0; i < C::NI; ++i) dma_sv(vb_ + (long)8 * NW * ld * i, dma_kv, st + TILE + 1024 * NW * i);
  };
  const int ntiles = CAUSAL ? min(S, qb * RW + RW) / BKS : S / BKS;
  if (ntiles > 0) stage(0);
  // retire the register loads before the loop (see the forward)
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) asm volatile("" : "+v"(qf[ks]), "+v"(df[ks]));
  asm volatile("" : "+v"(lse_s), "+v"(dl));
  const bf16x8 ones = fold_ones(hh), dl_b = fold_const(dl, hh);
  const float nlse = -lse_s * scale_log2;
  f32x16 dq[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dq[t] = f32x16{};
  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

  vm_wait<0>();
  barrier();
  for (int j = 0; j < ntiles; ++j) {
    if (j + 1 < ntiles) stage(j + 1);   // into the buffer every wave finished with (stage j-1)
#pragma unroll
    for (int hf = 0; hf < C::NH; ++hf) {
    const int k0 = j * BKS + BK * hf;
    if (live && (!CAUSAL || k0 <= qmax_w)) {
      const u32 hoff = (u32)((j % NSF) * STG + BK * 256 * hf);   // this half's K rows (V: + TILE)
      const char* Ks = smem + hoff;
      // non-causal: an opaque false keeps the causal loop's shape (folded away, hipcc spilled)
      int nm = CAUSAL ? (k0 + BK - 1 > qmin_w) : 0;
      if (!CAUSAL) asm volatile("" : "+v"(nm));
      const bool need_mask = __builtin_amdgcn_readfirstlane(nm) != 0;
      bf16x8 sf[2][2];
      // K and V row fragments by inline asm, QP k-steps ahead across both 32-key halves
      // (the compiler-scheduled form waited lgkmcnt(0) before every MFMA pair); this tile's
      // lane base is opaque so the 16 XOR-ed addresses are formed next to their reads
      // rematerialised from the lane id per tile (a long-lived copy spilled, and its reload
      // waited vmcnt(0) -- i.e. for every DMA stage in flight)
      const u32 ln = lane_id_opaque(), lr_ = ln & 31;
      const u32 a_t = (lds_addr(smem) + hoff) + lr_ * 256 + 16 * ((ln >> 5) ^ swz_x(lr_));
      bf16x8 fk[QP + 1], fv[QP + 1];
      auto rdS = [&](auto ic) {
        constexpr int i = decltype(ic)::value, kt = i >> 3, ks = i & 7, sl = i % (QP + 1);
        fk[sl] = rd_b128<8192 * kt>(a_t ^ (32 * ks));
        fv[sl] = rd_b128<TILE + 8192 * kt>(a_t ^ (32 * ks));
      };
      static_for<0, QP>([&](auto ic) { rdS(ic); });
      // s_setprio 1 over the MFMA chains, 0 over the exp / pack VALU: the SIMD's other wave then
      // keeps the matrix pipe fed through this wave's softmax (2.72 vs 2.76 ms,
      // profiles/fa_fwd128_r5.md; the forward measured null)
      __builtin_amdgcn_s_setprio(1);
      f32x16 s, dp;
      static_for<0, 16>([&](auto ic) {
        constexpr int i = decltype(ic)::value, kt = i >> 3, ks = i & 7, sl = i % (QP + 1);
        if constexpr (ks == 0) {
          // -lse is a per-LANE constant here (query on the lane): it goes into the exp's FMA
          // below instead of a folded MFMA; -delta stays folded (dS needs dP' = dP - delta)
          s = f32x16{};
          dp = mfma32(ones, dl_b, f32x16{});
        }
        if constexpr (i + QP < 16) rdS(std::integral_constant<int, i + QP>());
        lgkm_tie2<2 * (i + QP < 16 ? QP : 15 - i)>(fk[sl], fv[sl]);
        s = mfma32(fk[sl], qf[ks], s);
        dp = mfma32(fv[sl], df[ks], dp);
        if constexpr (ks == 7) {
          __builtin_amdgcn_s_setprio(0);
          if (need_mask) {
            const int ln = (int)lane_id_opaque(), qq = qmin_w + (ln & 31), h4 = 4 * (ln >> 5);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int key = k0 + 32 * kt + (r & 3) + 8 * (r >> 2) + h4;
              s[r] = key > qq ? -INFINITY : s[r];
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) s[r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r], scale_log2, nlse)) * dp[r];   // dS^T (unscaled)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            u32x4 u;
#pragma unroll
            for (int e = 0; e < 4; ++e) u[e] = pack2(s[8 * ss + 2 * e], s[8 * ss + 2 * e + 1]);
            sf[kt][ss] = as_bf16x8(u);
          }
          __builtin_amdgcn_s_setprio(1);
        }
      });
      const u32 kbase = lds_addr(Ks);
      bf16x8 kf[2][4];
      auto k_read = [&](int t, bf16x8* f) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            const int row = 32 * kt + 16 * ss + vrow, col = 32 * t + vcol;
            f[2 * kt + ss] = tr_pair_asm(kbase + swz8(row, col), kbase + swz8(row + 8, col));
          }
      };
      k_read(0, kf[0]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < 3) {
          k_read(t + 1, kf[(t + 1) & 1]);
          lgkm_wait_tie<8>(kf[t & 1]);
        } else {
          lgkm_wait_tie<0>(kf[t & 1]);
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) dq[t] = mfma32(kf[t & 1][2 * kt + ss], sf[kt][ss], dq[t]);
      }
      __builtin_amdgcn_s_setprio(0);
    }
    }
    if (j + 1 < ntiles) {
      vm_wait<0>();
      barrier();
    }
  }
  if (!live) return;
  store_rows_via_lds(dq, scale, smem + (ntiles % NSF) * STG + 8192 * w,
                     dqkv + ((long)b * S + qmin_w) * lddq + (long)h * D, lddq);
}

// ====================================================================================
// Backward: dK / dV
// ====================================================================================
namespace fb {
// waves per dK/dV workgroup (32 keys each): 4 = 128 keys, 66 KB LDS, 2 workgroups per CU (8 waves
// = 256 keys, 1 workgroup per CU, measured 4.30 vs 4.10-4.21 ms: profiles/fa_dkdv_w8_ab.txt)
constexpr int NWK = 4;
constexpr int BKVW = 32 * NWK;                 // keys per workgroup
// the per-iteration buffers sit first so their ds_read immediates (buffer + tile offsets)
// stay below the 16-bit offset field; K (read through a per-wave VGPR base) follows
constexpr int OFF_Q = 0;                       // [2][32 x 256 B]
constexpr int OFF_DO = OFF_Q + 16384;          // [2][32 x 256 B]
constexpr int OFF_LD = OFF_DO + 16384;         // [2][lse 32 f32 | delta 32 f32]
constexpr int OFF_K = OFF_LD + 512;            // [BKVW keys x 256 B] = 32 / 64 KB (256-B aligned)
constexpr int SMEM = OFF_K + BKVW * 256;       // 66048 B (2 WG per CU)
// read-ahead of the software-pipelined iteration: S/dP k-steps (3 row reads each) and dV/dK
// transposed fragments (a fourth fragment measured no better: profiles/fa_dkdv_pt_ab.txt)
constexpr int PA = 1, PT = 3;
// (measured and removed: a split S / dP chain with the softmax beside the dP MFMAs, and a
// v_mfma_f32_16x16x32_bf16 form with the row constants as the first MFMA's C operand --
// 4.38 and 4.39-4.44 ms vs 4.10-4.21 ms, profiles/fa_dkdv_split_ab.txt, fa_dkdv_mfma16_ab.txt)
// transposed fragment j of the dV/dK chain: column block t, row half ss (column block major; the
// row-half-major order measured 8 % slower, profiles/fa_dkdv_prio_ab.txt)
template <int J> struct FragJ {
  static constexpr int t = (J & 7) >> 1;
  static constexpr int ss = J & 1;
};
// s_setprio 1 over the MFMA chains, 0 over the softmax VALU and the DMA issue
__device__ __forceinline__ void prio(int p) {
  if (p) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

__host__ __device__ inline int n_chunks(int kb, int S, bool causal) {
  const int q0 = causal ? kb * BKVW : 0;
  return (S - q0 + QCH - 1) / QCH;
}
}  // namespace fb

// DET (deterministic mode) is a template parameter, not a run-time flag: the atomic
// instantiation compiles to round 5's instruction stream, whose main loop is hand-scheduled
template <bool CAUSAL, bool DET>
__global__ __launch_bounds__(64 * fb::NWK, 8 / fb::NWK) void flash_bwd_dkdv_kernel(
    const bf16_t* __restrict__ qkv, long ld, const bf16_t* __restrict__ dout, long lddo,
    const float* __restrict__ lse, const float* __restrict__ delta, float* __restrict__ dk_acc,
    float* __restrict__ dv_acc, int B, int S, int Hq, int Hkv, float scale, int items_per_head) {
  using namespace fb;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  const int G = Hq / Hkv;
  const int lid = xcd_remap(blockIdx.x, B * Hkv * items_per_head);
  int item = lid % items_per_head;
  const int slot = item;            // this work item's partial-sum slot (DET)
  const int bh = lid / items_per_head;
  const int hkv = bh % Hkv, b = bh / Hkv;
  const int nkb = S / BKVW;
  int kb = 0;
  for (; kb < nkb; ++kb) {
    const int n = n_chunks(kb, S, CAUSAL);
    if (item < n) break;
    item -= n;
  }
  const int kv0 = kb * BKVW;
  const int qs = (CAUSAL ? kv0 : 0) + item * QCH;
  const int qe = min(S, qs + QCH);
  const int ntq = (qe - qs) / QT;
  const int niter = ntq * G;

  const int tid = threadIdx.x, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kw0 = kv0 + 32 * w;
  const float c = scale * LOG2E, inv_scale = 1.f / scale;
  const long rowB = (long)b * S;
  const bf16_t* kp = qkv + rowB * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + rowB * ld + (long)(Hq + Hkv + hkv) * D;

  stage_rows(kp + (long)kv0 * ld, ld, smem + OFF_K, BKVW, w, NWK, l);
  bf16x8 vf[8];  // B operand of dP = dO V^T: V[key][16ks + 8hh .. +8]
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) vf[ks] = as_bf16x8(ld16(vp + (long)(kw0 + lr) * ld + 16 * ks + 8 * hh));
  const u32 sbase = lds_addr(smem);
  u32 dma_q, dma_do;   // byte offset of this lane's 16-B piece of row 4w + l/16 in a Q / dO panel
  {
    const int row = 4 * w + (l >> 4), ch = (l & 15) ^ swz_x(row);
    dma_q = (u32)((row * ld + ch * 8) * 2);
    dma_do = (u32)((row * lddo + ch * 8) * 2);
  }

  // iteration it = (head hq, query tile qt) is carried incrementally (no runtime division)
  auto stage = [&](int hq, int qt, int buf) {
    const int h = hkv * G + hq;
    const int q0 = qs + qt * QT;
    // wave w fills rows 4w.. and 4w+16.. of the Q and dO images: SGPR panel base + one 32-bit
    // lane offset per tensor (rows 16 apart share the lane's chunk swizzle)
    const char* qb_ = reinterpret_cast<const char*>(qkv + (rowB + q0) * ld + (long)h * D);
    const char* db_ = reinterpret_cast<const char*>(dout + (rowB + q0) * lddo + (long)h * D);
    const u32 lq = sbase + OFF_Q + buf * 8192 + 1024 * w, ldo_ = sbase + OFF_DO + buf * 8192 + 1024 * w;
    dma_sv(qb_, dma_q, lq);
    dma_sv(db_, dma_do, ldo_);
    if (NWK == 4) {
      dma_sv(qb_ + 32 * ld, dma_q, lq + 4096);
      dma_sv(db_ + 32 * lddo, dma_do, ldo_ + 4096);
    }
    if (w == 0) {
      // lse/delta select from an opaque lane id: hoisted, the per-lane 64-bit pointer lived
      // across the loop and was the kernel's only scratch spill
      int lo = l;
      asm volatile("" : "+v"(lo));
      const float* src = (lo < 32 ? lse : delta) + ((long)b * Hq + h) * S + q0 + (lo & 31);
      glds4(src, smem + OFF_LD + buf * 256);
    }
  };

  f32x16 dK[4], dV[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) { dK[t] = f32x16{}; dV[t] = f32x16{}; }
  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

  if (niter > 0) stage(0, 0, 0);
  wait_dma_barrier();
  const bf16x8 ones = fold_ones(hh);
  int nx_hq = 0, nx_qt = 0;   // (head, tile) of the NEXT iteration to stage
  auto adv = [&]() {
    if (++nx_qt == ntq) { nx_qt = 0; ++nx_hq; }
  };
  // Software-pipelined iteration.  Every LDS read is inline asm with an immediate buffer
  // offset and a counted, register-tying wait: the compiler-scheduled form issued each
  // operand right before its MFMA behind an lgkmcnt(0) (one read latency exposed per MFMA)
  // and waited vmcnt(0) for the NEXT tile's DMA before the transposed reads.
  //  * S/dP chain: Q, K and dO row fragments two k-steps ahead (3-slot ring);
  //  * dV^T/dK^T chain: the 16 transposed fragments (dO^T, then Q^T) three ahead (4-slot ring),
  //    the first three issued before the softmax VALU work.
  // Lane address parts: smem is 1024-aligned, so the k-step / column-block terms are XORs that
  // never carry (row chunk 2ks+hh -> a_row ^ 32ks; transposed column block t -> a_tr ^ 64t).
  const u32 a_row0 = sbase + lr * 256 + 16 * (hh ^ swz_x(lr));
  const u32 a_k0 = a_row0 + 8192 * w + OFF_K;
  const u32 a_ls = sbase + OFF_LD + 4 * lr;
  u32 a_tr[2][2];
#pragma unroll
  for (int ss = 0; ss < 2; ++ss)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int row = 16 * ss + vrow + 8 * hf;
      a_tr[ss][hf] = sbase + row * 256 + 16 * ((vcol >> 3) ^ swz_x(row)) + 8 * (l & 1);
    }
  auto iter = [&](auto curc, int it) {
    constexpr int CUR = decltype(curc)::value;
    constexpr int OQ = OFF_Q + CUR * 8192, OD = OFF_DO + CUR * 8192, OL = CUR * 256;
    const int q0 = qs + nx_qt * QT;   // this iteration's tile (advanced below to the next)
    adv();
    if (it + 1 < niter) stage(nx_hq, nx_qt, CUR ^ 1);
    // opaque per iteration: keeps the 32 XOR-ed per-read addresses from being hoisted out of
    // the loop as invariants (they would pin ~30 VGPRs and spill)
    u32 a_row = a_row0, a_k = a_k0, a_t00 = a_tr[0][0], a_t01 = a_tr[0][1], a_t10 = a_tr[1][0], a_t11 = a_tr[1][1];
    asm volatile("" : "+v"(a_row), "+v"(a_k), "+v"(a_t00), "+v"(a_t01), "+v"(a_t10), "+v"(a_t11));
    const u32 a_t[2][2] = {{a_t00, a_t01}, {a_t10, a_t11}};
    if (!CAUSAL || kw0 <= q0 + QT - 1) {
      prio(1);
      float lse_v = rd_b32<OL>(a_ls), dl_v = rd_b32<OL + 128>(a_ls);
      bf16x8 fq[PA + 1], fk[PA + 1], fd[PA + 1];
      auto rdA = [&](auto kc) {
        constexpr int ks = decltype(kc)::value, sl = ks % (PA + 1);
        fq[sl] = rd_b128<OQ>(a_row ^ (32 * ks));
        fk[sl] = rd_b128<0>(a_k ^ (32 * ks));
        fd[sl] = rd_b128<OD>(a_row ^ (32 * ks));
      };
      static_for<0, PA>([&](auto kc) { rdA(kc); });
      lgkm_tie_f2<3 * PA>(lse_v, dl_v);
      // row constants -lse/scale and -delta of query row lr folded into the chains
      f32x16 s = mfma32(fold_const(lse_v * inv_scale, hh), ones, f32x16{});
      f32x16 dp = mfma32(fold_const(dl_v, hh), ones, f32x16{});
      static_for<0, 8>([&](auto kc) {
        constexpr int ks = decltype(kc)::value, sl = ks % (PA + 1);
        if constexpr (ks + PA < 8) rdA(std::integral_constant<int, ks + PA>());
        // outstanding after this k-step's reads: the later k-steps already issued
        lgkm_tie3<3 * (ks + PA < 8 ? PA : 7 - ks)>(fq[sl], fk[sl], fd[sl]);
        s = mfma32(fq[sl], fk[sl], s);
        dp = mfma32(fd[sl], vf[ks], dp);
      });
      // transposed fragment j: j < 8 -> dO^T (dV), else Q^T (dK); column block t, row half ss
      bf16x8 ft[PT + 1];
      auto rdT = [&](auto jc) {
        constexpr int j = decltype(jc)::value, t = FragJ<j>::t, ss = FragJ<j>::ss;
        ft[j % (PT + 1)] = rd_tr2<(j < 8 ? OD : OQ)>(a_t[ss][0] ^ (64 * t), a_t[ss][1] ^ (64 * t));
      };
      static_for<0, PT>([&](auto jc) { rdT(jc); });
      prio(0);
      const int key = kw0 + lr;
      // non-causal: an opaque false keeps the causal loop's shape (with the masked path folded
      // away hipcc scheduled the loop differently and spilled 12 VGPRs)
      int nm = CAUSAL ? (kw0 + 31 > q0) : 0;
      if (!CAUSAL) asm volatile("" : "+v"(nm));
      const bool need_mask = __builtin_amdgcn_readfirstlane(nm) != 0;
      if (need_mask) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(s[r] * c);
          s[r] = key > q0 + (r & 3) + 8 * (r >> 2) + 4 * hh ? 0.f : p;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = __builtin_amdgcn_exp2f(s[r] * c);
      }
      bf16x8 pf[2], sf[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        u32x4 u, v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          u[i] = pack2(s[8 * ss + 2 * i], s[8 * ss + 2 * i + 1]);
          v[i] = pack2(s[8 * ss + 2 * i] * dp[8 * ss + 2 * i], s[8 * ss + 2 * i + 1] * dp[8 * ss + 2 * i + 1]);
        }
        pf[ss] = as_bf16x8(u);
        sf[ss] = as_bf16x8(v);
      }
      prio(1);
      static_for<0, 16>([&](auto jc) {
        constexpr int j = decltype(jc)::value, t = FragJ<j>::t, ss = FragJ<j>::ss, sl = j % (PT + 1);
        if constexpr (j + PT < 16) rdT(std::integral_constant<int, j + PT>());
        lgkm_tie1<2 * (j + PT < 16 ? PT : 15 - j)>(ft[sl]);
        if constexpr (j < 8) dV[t] = mfma32(ft[sl], pf[ss], dV[t]);
        else dK[t] = mfma32(ft[sl], sf[ss], dK[t]);
      });
      prio(0);
    }
    wait_dma_barrier();
  };
  {
    int it = 0;
    for (; it + 1 < niter; it += 2) {
      iter(std::integral_constant<int, 0>(), it);
      iter(std::integral_constant<int, 1>(), it + 1);
    }
    if (it < niter) iter(std::integral_constant<int, 0>(), it);
  }
  // ---- chunk partial sums: transpose [d][key] accumulators through LDS, row-contiguous adds,
  // 128 keys (4 waves' accumulators) per pass
  float* T = reinterpret_cast<float*>(smem);   // [128 keys][128 d] fp32 = 64 KB
  auto flush = [&](const f32x16(&acc)[4], float mul, float* dst_base) {
#pragma unroll
    for (int pass = 0; pass < NWK / 4; ++pass) {
      if (w / 4 == pass) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int d = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const int key = 32 * (w & 3) + lr;
            T[key * 128 + (d ^ ((key & 31) << 2))] = acc[t][r] * mul;
          }
      }
      __syncthreads();
      // atomics: every work item of a key block adds into one [T, Hkv*D] accumulator (fp32 sum
      // order varies run to run); deterministic mode: each item stores its partial into its own
      // slot rows, and flash_bwd_post_kernel sums a key block's slots in item order
      float* dst = DET ? dst_base + ((long)(b * items_per_head + slot) * BKVW + 128 * pass) * (long)(Hkv * D) + (long)hkv * D
                       : dst_base + (rowB + kv0 + 128 * pass) * (long)(Hkv * D) + (long)hkv * D;
      if constexpr (DET) {
        for (int e = tid; e < 128 * 128; e += 64 * NWK) {
          const int key = e >> 7, d = e & 127;
          dst[(long)key * Hkv * D + d] = T[key * 128 + (d ^ ((key & 31) << 2))];
        }
      } else {
        for (int e = tid; e < 128 * 128; e += 64 * NWK) {
          const int key = e >> 7, d = e & 127;
          atomicAdd(dst + (long)key * Hkv * D + d, T[key * 128 + (d ^ ((key & 31) << 2))]);
        }
      }
      __syncthreads();
    }
  };
  flush(dK, scale, dk_acc);
  flush(dV, 1.f, dv_acc);
}

// fp32 dK/dV accumulators -> bf16 k/v columns of the fused dqkv [T, (Hq + 2Hkv) * 128].
// Deterministic mode (ns > 0): the accumulators are per-work-item slots [B][ns][BKVW][Hkv * 128],
// and each key's value is the sum of its key block's slots in item order.
__global__ __launch_bounds__(256) void flash_bwd_post_kernel(const float* __restrict__ dk,
                                                             const float* __restrict__ dv,
                                                             bf16_t* __restrict__ dqkv, long ld, int T,
                                                             int Hq, int Hkv, int S, int ns, int causal) {
  const int ck = Hkv * 16, per_row = 2 * ck;   // 8-element chunks
  const long total = (long)T * per_row;
  const long row_f = (long)Hkv * 128;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int t = (int)(i / per_row), c = (int)(i - (long)t * per_row);
    const float* base = c < ck ? dk : dv;
    const int col = (c < ck ? c : c - ck) * 8;
    float f[8];
    if (ns == 0) {
      const float* src = base + (long)t * row_f + col;
      const f32x4 a = ldf4(src), bb = ldf4(src + 4);
      f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3]; f[4] = bb[0]; f[5] = bb[1]; f[6] = bb[2]; f[7] = bb[3];
    } else {
      using namespace fb;
      const int b = t / S, key = t - b * S, kb = key / BKVW, kl = key - kb * BKVW;
      int slot0 = 0;
      for (int k = 0; k < kb; ++k) slot0 += n_chunks(k, S, causal != 0);
      const int nc = n_chunks(kb, S, causal != 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = 0.f;
      for (int cc = 0; cc < nc; ++cc) {
        const float* src = base + ((long)(b * ns + slot0 + cc) * BKVW + kl) * row_f + col;
        const f32x4 a = ldf4(src), bb = ldf4(src + 4);
        f[0] += a[0]; f[1] += a[1]; f[2] += a[2]; f[3] += a[3];
        f[4] += bb[0]; f[5] += bb[1]; f[6] += bb[2]; f[7] += bb[3];
      }
    }
    st16(dqkv + (long)t * ld + Hq * 128 + (c < ck ? 0 : Hkv * 128) + col, pack8(f));
  }
}

extern "C" {

// waves per forward workgroup (FwdCfg)
constexpr int FWD_NW = 8;

int kf_flash_fwd(const void* qkv, long ld, void* out, long ldo, float* lse, int B, int S, int Hq,
                 int Hkv, int D_, float scale, int causal, hipStream_t st) {
  if (D_ != D || S % BQ != 0 || Hq % Hkv != 0 || ld % 8 || ldo % 8) return 1;
  const int grid = B * Hq * ((S + FwdCfg<FWD_NW>::RW - 1) / FwdCfg<FWD_NW>::RW);
  const float sl2 = scale * LOG2E;
  if (causal)
    flash_fwd_kernel<true, FWD_NW><<<grid, 64 * FWD_NW, 0, st>>>((const bf16_t*)qkv, ld, (bf16_t*)out, ldo, lse, B, S,
                                                 Hq, Hkv, sl2);
  else
    flash_fwd_kernel<false, FWD_NW><<<grid, 64 * FWD_NW, 0, st>>>((const bf16_t*)qkv, ld, (bf16_t*)out, ldo, lse, B,
                                                  S, Hq, Hkv, sl2);
  return 0;
}

// dQ || dK/dV fork: the two backward kernels only share read-only inputs, so the dK/dV
// chain (zero its fp32 accumulators -> dK/dV kernel) runs on a side stream (event fork/join,
// legal under hipGraph capture): the accumulator memset overlaps the delta pre-pass and the
// dQ blocks fill CUs as dK/dV blocks retire instead of waiting for that grid's tail.  One
// side stream and its events per device (one process per GPU).  KFAMD_FA_BWD_FORK=0 serialises.
// The lazy per-device init and every use of the shared events run under the device's mutex
// (two host threads may call backward on one device), and every exit after the fork joins the
// side stream back, so an error return never leaves forked work dangling (which would also
// invalidate a hipGraph capture).
namespace {
struct BwdFork {
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, pre = nullptr, join = nullptr;
  std::mutex mu;
};
bool bwd_fork_enabled() {
  static const bool on = [] {
    const char* e = getenv("KFAMD_FA_BWD_FORK");
    return !(e && e[0] == '0');
  }();
  return on;
}
BwdFork* bwd_fork() {
  static BwdFork per_dev[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  BwdFork& f = per_dev[dev];
  std::lock_guard<std::mutex> lk(f.mu);
  if (!f.side) {
    // the dK/dV chain (the longer kernel) on the device's highest-priority stream: its workgroups are
    // dispatched ahead of dQ's, which fill the CUs around them (backward 7.370-7.376 vs 7.451-7.461
    // ms at B4 S8192, alternating builds on one box: profiles/fa_structure_r6.md)
    int lo_prio = 0, hi_prio = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio);
    if (hipStreamCreateWithPriority(&f.side, hipStreamNonBlocking, hi_prio) != hipSuccess ||
        hipEventCreateWithFlags(&f.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&f.pre, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&f.join, hipEventDisableTiming) != hipSuccess) {
      f.side = nullptr;
      return nullptr;
    }
  }
  return &f;
}
}  // namespace

// waves per dQ workgroup (DqCfg)
constexpr int DQ_NW = 8;
// dK/dV work items per (batch, kv head): one per key block and query chunk
static int dkdv_items(int S, int causal) {
  int items = 0;
  for (int kb = 0; kb < S / fb::BKVW; ++kb) items += fb::n_chunks(kb, S, causal);
  return items;
}
// floats of ONE of the two dK / dV scratch buffers kf_flash_bwd needs: [B*S, Hkv*128] for the
// atomic accumulation, [B][items][BKVW][Hkv*128] partial slots in deterministic mode
long kf_flash_bwd_acc_floats(int B, int S, int Hkv, int causal, int deterministic) {
  if (deterministic) return (long)B * dkdv_items(S, causal) * fb::BKVW * Hkv * D;
  return (long)B * S * Hkv * D;
}

// dk_acc/dv_acc: fp32 scratch of kf_flash_bwd_acc_floats each (zeroed here in the atomic mode);
// delta: fp32 [B, Hq, S] scratch.  deterministic = 1: bitwise run-to-run reproducible dK/dV
// (per-item partial slots summed in a fixed order by the post kernel instead of fp32 atomics).
int kf_flash_bwd(const void* qkv, long ld, const void* o, long ldo, const void* dout, long lddo,
                 const float* lse, float* delta, float* dk_acc, float* dv_acc, void* dqkv,
                 long lddqkv, int B, int S, int Hq, int Hkv, int D_, float scale, int causal,
                 int deterministic, hipStream_t st) {
  using namespace fb;
  if (D_ != D || S % BKVW != 0 || S % BQ != 0 || Hq % Hkv != 0) return 1;
  const int T = B * S;
  const int det = deterministic ? 1 : 0;
  const size_t acc_bytes = (size_t)T * Hkv * D * sizeof(float);
  BwdFork* fk = bwd_fork_enabled() ? bwd_fork() : nullptr;
  std::unique_lock<std::mutex> lk;
  if (fk) lk = std::unique_lock<std::mutex>(fk->mu);
  hipStream_t skv = st;
  if (fk && hipEventRecord(fk->fork, st) == hipSuccess &&
      hipStreamWaitEvent(fk->side, fk->fork, 0) == hipSuccess)
    skv = fk->side;
  // error exit after the fork: join the side stream back before returning
  auto fail = [&](int rc) {
    if (skv != st && hipEventRecord(fk->join, skv) == hipSuccess) (void)hipStreamWaitEvent(st, fk->join, 0);
    return rc;
  };
  // deterministic mode: every slot row is stored by its work item, nothing to zero
  if (!det && (hipMemsetAsync(dk_acc, 0, acc_bytes, skv) != hipSuccess ||
               hipMemsetAsync(dv_acc, 0, acc_bytes, skv) != hipSuccess))
    return fail(2);
  flash_bwd_pre_kernel<<<(T * Hq + 15) / 16, 256, 0, st>>>((const bf16_t*)o, ldo, (const bf16_t*)dout,
                                                           lddo, delta, B, S, Hq);
  if (skv != st &&
      (hipEventRecord(fk->pre, st) != hipSuccess || hipStreamWaitEvent(skv, fk->pre, 0) != hipSuccess))
    return fail(2);
  const int items = dkdv_items(S, causal);
  const int g_kv = B * Hkv * items, g_q = B * Hq * ((S + DqCfg<DQ_NW>::RW - 1) / DqCfg<DQ_NW>::RW);
  const float sl2 = scale * LOG2E;
  const bf16_t* q_ = (const bf16_t*)qkv;
  const bf16_t* do_ = (const bf16_t*)dout;
  auto dkdv = [&](auto kern) {
    kern<<<g_kv, 64 * NWK, 0, skv>>>(q_, ld, do_, lddo, lse, delta, dk_acc, dv_acc, B, S, Hq, Hkv, scale, items);
  };
  if (causal) {
    if (det) dkdv(flash_bwd_dkdv_kernel<true, true>);
    else dkdv(flash_bwd_dkdv_kernel<true, false>);
    flash_bwd_dq_kernel<true, DQ_NW><<<g_q, 64 * DQ_NW, 0, st>>>(q_, ld, do_, lddo, lse, delta, (bf16_t*)dqkv, lddqkv, B,
                                                                 S, Hq, Hkv, sl2, scale);
  } else {
    if (det) dkdv(flash_bwd_dkdv_kernel<false, true>);
    else dkdv(flash_bwd_dkdv_kernel<false, false>);
    flash_bwd_dq_kernel<false, DQ_NW><<<g_q, 64 * DQ_NW, 0, st>>>(q_, ld, do_, lddo, lse, delta, (bf16_t*)dqkv, lddqkv, B,
                                                                  S, Hq, Hkv, sl2, scale);
  }
  if (skv != st &&
      (hipEventRecord(fk->join, skv) != hipSuccess || hipStreamWaitEvent(st, fk->join, 0) != hipSuccess))
    return 2;
  const long chunks = (long)T * Hkv * 32;
  const int pg = (int)std::min<long>((chunks + 255) / 256, 16384);
  flash_bwd_post_kernel<<<pg, 256, 0, st>>>(dk_acc, dv_acc, (bf16_t*)dqkv, lddqkv, T, Hq, Hkv, S,
                                            det ? items : 0, causal);
  return 0;
}
}
