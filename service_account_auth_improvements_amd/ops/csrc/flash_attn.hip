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
// Forward: 1 workgroup = 4 waves x 32 query rows, 64-key tiles, online softmax (exp2).
// Backward, two kernels, no dQ atomics:
//  * dQ kernel (forward-shaped, per 128 query rows): S^T, dP^T = V.dO^T, P^T, dS^T,
//    dQ^T += K^T.dS^T; dQ written once as bf16 into the dqkv buffer.
//  * dK/dV kernel (per 128-key block x query chunk, all G query heads of the GQA group):
//    S = Q.K^T and dP = dO.V^T with the KEY on the lane (accumulators pre-loaded with
//    -lse/scale and -delta, the "row constants"), dV^T += dO^T.P, dK^T += Q^T.dS; each
//    wave keeps its 32 keys' dK^T/dV^T (128 registers) across the chunk; chunk partial
//    sums are transposed through LDS and added row-contiguously in fp32.
#include "common.h"

using namespace kf;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f4;
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace fa {
constexpr int D = 128;
constexpr int BQ = 128;           // query rows per forward / dQ workgroup (4 waves x 32)
constexpr int BK = 64;            // keys per tile (forward / dQ)
constexpr int TILE = BK * D * 2;  // 16 KB
constexpr int BKV = 128;          // keys per dK/dV workgroup (4 waves x 32)
constexpr int QT = 32;            // query rows per dK/dV iteration
constexpr int QCH = 1024;         // query rows per dK/dV work item
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
__device__ __forceinline__ u32x2 tr_read(const char* p) {
  s16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p));
  return __builtin_bit_cast(u32x2, t);
}
__device__ __forceinline__ bf16x8 tr_pair(const char* base, int o0, int o1) {
  const u32x2 a = tr_read(base + o0), b = tr_read(base + o1);
  return as_bf16x8(u32x4{a[0], a[1], b[0], b[1]});
}
__device__ __forceinline__ bf16x8 row_read(const char* base, int off) {
  return as_bf16x8(*reinterpret_cast<const u32x4*>(base + off));
}

// LDS-DMA of one 16-B piece per lane; `lds` must be wave-uniform (lands at lds + 16*lane)
__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
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

// ====================================================================================
// Forward
// ====================================================================================
template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) void flash_fwd_kernel(
    const bf16_t* __restrict__ qkv, long ld, bf16_t* __restrict__ out, long ldo,
    float* __restrict__ lse_out, int B, int S, int Hq, int Hkv, float scale_log2) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // K0 K1 V0 V1
  const QBlock blk = decode_qblock(S, Hq, Hkv, B, CAUSAL);
  const int b = blk.b, h = blk.h, hkv = blk.hkv, qb = blk.qb;
  const int tid = threadIdx.x, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = qb * BQ + w * 32 + lr;
  const int qmin_w = qb * BQ + w * 32, qmax_w = qmin_w + 31;

  bf16x8 qf[8];  // B operand of S^T = K Q^T: Q[q][16ks + 8hh .. +8]
  {
    const bf16_t* qp = qkv + ((long)b * S + q) * ld + (long)h * D + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = as_bf16x8(ld16(qp + 16 * ks));
  }
  const bf16_t* kp = qkv + (long)b * S * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + (long)b * S * ld + (long)(Hq + Hkv + hkv) * D;
  auto stage = [&](int j, int buf) {
    stage_rows(kp + (long)j * BK * ld, ld, smem + buf * TILE, BK, w, 4, l);
    stage_rows(vp + (long)j * BK * ld, ld, smem + (2 + buf) * TILE, BK, w, 4, l);
  };

  f32x16 o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = f32x16{};
  float m = -INFINITY, lsum = 0.f;
  const int ntiles = CAUSAL ? (qb * BQ + BQ) / BK : S / BK;
  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

  stage(0, 0);
  wait_dma_barrier();
  for (int j = 0; j < ntiles; ++j) {
    const int cur = j & 1;
    if (j + 1 < ntiles) stage(j + 1, cur ^ 1);
    const int k0 = j * BK;
    if (!CAUSAL || k0 <= qmax_w) {
      const char* Ks = smem + cur * TILE;
      const char* Vs = smem + (2 + cur) * TILE;
      f32x16 s[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) s[kt] = mfma32(row_read(Ks, swz(32 * kt + lr, 2 * ks + hh)), qf[ks], s[kt]);
      }
      // scores stay unscaled; the running max m lives in the scaled log2 domain so each
      // p = exp2(s*c - m) is one FMA + one raw v_exp_f32 (argument <= 0: exp2f's
      // denormal fix-up is dead weight).  Only a wave's diagonal tiles mask (uniform branch).
      if (CAUSAL && k0 + BK - 1 > qmin_w) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
            s[kt][r] = key > q ? -INFINITY : s[kt][r];
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx * scale_log2);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = __builtin_amdgcn_exp2f(m - msafe);
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[kt][r], scale_log2, -msafe));
          s[kt][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32, 64);
      lsum = lsum * alpha + rs;
      m = mnew;
      if (__ballot(alpha != 1.f)) {   // skip the O rescale when no row's max moved
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
      }
      bf16x8 pf[2][2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          u32x4 u;
#pragma unroll
          for (int i = 0; i < 4; ++i) u[i] = pack2(s[kt][8 * ss + 2 * i], s[kt][8 * ss + 2 * i + 1]);
          pf[kt][ss] = as_bf16x8(u);
        }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            const int row = 32 * kt + 16 * ss + vrow, col = 32 * t + vcol;
            o[t] = mfma32(tr_pair(Vs, swz8(row, col), swz8(row + 8, col)), pf[kt][ss], o[t]);
          }
    }
    wait_dma_barrier();
  }
  const float inv = 1.f / lsum;
  bf16_t* op = out + ((long)b * S + q) * ldo + (long)h * D;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int d = 32 * t + 8 * gq + 4 * hh;
      u32x2 v;
      v[0] = pack2(o[t][4 * gq] * inv, o[t][4 * gq + 1] * inv);
      v[1] = pack2(o[t][4 * gq + 2] * inv, o[t][4 * gq + 3] * inv);
      *reinterpret_cast<u32x2*>(op + d) = v;
    }
  if (hh == 0) lse_out[((long)b * Hq + h) * S + q] = (m + log2f(lsum)) * LN2;
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
template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) void flash_bwd_dq_kernel(
    const bf16_t* __restrict__ qkv, long ld, const bf16_t* __restrict__ dout, long lddo,
    const float* __restrict__ lse, const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    long lddq, int B, int S, int Hq, int Hkv, float scale_log2, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // K0 K1 V0 V1
  const QBlock blk = decode_qblock(S, Hq, Hkv, B, CAUSAL);
  const int b = blk.b, h = blk.h, hkv = blk.hkv, qb = blk.qb;
  const int tid = threadIdx.x, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = qb * BQ + w * 32 + lr;
  const int qmin_w = qb * BQ + w * 32, qmax_w = qmin_w + 31;

  bf16x8 qf[8], df[8];
  {
    const bf16_t* qp = qkv + ((long)b * S + q) * ld + (long)h * D + 8 * hh;
    const bf16_t* dp_ = dout + ((long)b * S + q) * lddo + (long)h * D + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      qf[ks] = as_bf16x8(ld16(qp + 16 * ks));
      df[ks] = as_bf16x8(ld16(dp_ + 16 * ks));
    }
  }
  const float lse2 = lse[((long)b * Hq + h) * S + q] * LOG2E;
  const float dl = delta[((long)b * Hq + h) * S + q];
  const bf16_t* kp = qkv + (long)b * S * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + (long)b * S * ld + (long)(Hq + Hkv + hkv) * D;
  auto stage = [&](int j, int buf) {
    stage_rows(kp + (long)j * BK * ld, ld, smem + buf * TILE, BK, w, 4, l);
    stage_rows(vp + (long)j * BK * ld, ld, smem + (2 + buf) * TILE, BK, w, 4, l);
  };
  f32x16 dq[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dq[t] = f32x16{};
  const int ntiles = CAUSAL ? (qb * BQ + BQ) / BK : S / BK;
  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

  stage(0, 0);
  wait_dma_barrier();
  for (int j = 0; j < ntiles; ++j) {
    const int cur = j & 1;
    if (j + 1 < ntiles) stage(j + 1, cur ^ 1);
    const int k0 = j * BK;
    if (!CAUSAL || k0 <= qmax_w) {
      const char* Ks = smem + cur * TILE;
      const char* Vs = smem + (2 + cur) * TILE;
      const bool need_mask = CAUSAL && (k0 + BK - 1 > qmin_w);
      bf16x8 sf[2][2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          s = mfma32(row_read(Ks, swz(32 * kt + lr, 2 * ks + hh)), qf[ks], s);
          dp = mfma32(row_read(Vs, swz(32 * kt + lr, 2 * ks + hh)), df[ks], dp);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = __builtin_amdgcn_exp2f(s[r] * scale_log2 - lse2);
          if (need_mask) {
            const int key = k0 + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (key > q) p = 0.f;
          }
          s[r] = p * (dp[r] - dl);   // dS^T (unscaled)
        }
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          u32x4 u;
#pragma unroll
          for (int i = 0; i < 4; ++i) u[i] = pack2(s[8 * ss + 2 * i], s[8 * ss + 2 * i + 1]);
          sf[kt][ss] = as_bf16x8(u);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            const int row = 32 * kt + 16 * ss + vrow, col = 32 * t + vcol;
            dq[t] = mfma32(tr_pair(Ks, swz8(row, col), swz8(row + 8, col)), sf[kt][ss], dq[t]);
          }
    }
    wait_dma_barrier();
  }
  bf16_t* op = dqkv + ((long)b * S + q) * lddq + (long)h * D;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int d = 32 * t + 8 * gq + 4 * hh;
      u32x2 v;
      v[0] = pack2(dq[t][4 * gq] * scale, dq[t][4 * gq + 1] * scale);
      v[1] = pack2(dq[t][4 * gq + 2] * scale, dq[t][4 * gq + 3] * scale);
      *reinterpret_cast<u32x2*>(op + d) = v;
    }
}

// ====================================================================================
// Backward: dK / dV
// ====================================================================================
namespace fb {
constexpr int OFF_K = 0;                       // [128 keys x 256 B] = 32 KB
constexpr int OFF_Q = 32768;                   // [2][32 x 256 B]
constexpr int OFF_DO = OFF_Q + 16384;          // [2][32 x 256 B]
constexpr int OFF_LD = OFF_DO + 16384;         // [2][lse 32 f32 | delta 32 f32]
constexpr int SMEM = OFF_LD + 512;             // 66048 B -> 2 workgroups per CU

__device__ __forceinline__ int n_chunks(int kb, int S, bool causal) {
  const int q0 = causal ? kb * BKV : 0;
  return (S - q0 + QCH - 1) / QCH;
}
}  // namespace fb

template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) void flash_bwd_dkdv_kernel(
    const bf16_t* __restrict__ qkv, long ld, const bf16_t* __restrict__ dout, long lddo,
    const float* __restrict__ lse, const float* __restrict__ delta, float* __restrict__ dk_acc,
    float* __restrict__ dv_acc, int B, int S, int Hq, int Hkv, float scale, int items_per_head) {
  using namespace fb;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int G = Hq / Hkv;
  const int lid = xcd_remap(blockIdx.x, B * Hkv * items_per_head);
  int item = lid % items_per_head;
  const int bh = lid / items_per_head;
  const int hkv = bh % Hkv, b = bh / Hkv;
  const int nkb = S / BKV;
  int kb = 0;
  for (; kb < nkb; ++kb) {
    const int n = n_chunks(kb, S, CAUSAL);
    if (item < n) break;
    item -= n;
  }
  const int kv0 = kb * BKV;
  const int qs = (CAUSAL ? kv0 : 0) + item * QCH;
  const int qe = min(S, qs + QCH);
  const int ntq = (qe - qs) / QT;
  const int niter = ntq * G;

  const int tid = threadIdx.x, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kw0 = kv0 + 32 * w;
  const float c = scale * LOG2E;
  const float inv_scale = 1.f / scale;
  const long rowB = (long)b * S;
  const bf16_t* kp = qkv + rowB * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + rowB * ld + (long)(Hq + Hkv + hkv) * D;

  stage_rows(kp + (long)kv0 * ld, ld, smem + OFF_K, BKV, w, 4, l);
  bf16x8 vf[8];  // B operand of dP = dO V^T: V[key][16ks + 8hh .. +8]
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) vf[ks] = as_bf16x8(ld16(vp + (long)(kw0 + lr) * ld + 16 * ks + 8 * hh));

  auto stage = [&](int it, int buf) {
    const int hq = it / ntq, qt = it - hq * ntq;
    const int h = hkv * G + hq;
    const int q0 = qs + qt * QT;
    stage_rows(qkv + (rowB + q0) * ld + (long)h * D, ld, smem + OFF_Q + buf * 8192, QT, w, 4, l);
    stage_rows(dout + (rowB + q0) * lddo + (long)h * D, lddo, smem + OFF_DO + buf * 8192, QT, w, 4, l);
    if (w == 0) {
      const float* src = (l < 32 ? lse : delta) + ((long)b * Hq + h) * S + q0 + (l & 31);
      glds4(src, smem + OFF_LD + buf * 256);
    }
  };

  f32x16 dK[4], dV[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) { dK[t] = f32x16{}; dV[t] = f32x16{}; }
  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

  if (niter > 0) stage(0, 0);
  wait_dma_barrier();
  for (int it = 0; it < niter; ++it) {
    const int cur = it & 1;
    const int qt = it % ntq;
    const int q0 = qs + qt * QT;
    if (it + 1 < niter) stage(it + 1, cur ^ 1);
    const char* Qs = smem + OFF_Q + cur * 8192;
    const char* dOs = smem + OFF_DO + cur * 8192;
    const float* Ls = reinterpret_cast<const float*>(smem + OFF_LD + cur * 256);
    if (!CAUSAL || kw0 <= q0 + QT - 1) {
      // row constants, q(r) = (r&3) + 8(r>>2) + 4hh
      f32x16 s, dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f4 L4 = *reinterpret_cast<const f4*>(Ls + 8 * g + 4 * hh);
        const f4 D4 = *reinterpret_cast<const f4*>(Ls + 32 + 8 * g + 4 * hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) { s[4 * g + i] = -L4[i] * inv_scale; dp[4 * g + i] = -D4[i]; }
      }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        s = mfma32(row_read(Qs, swz(lr, 2 * ks + hh)), row_read(smem + OFF_K, swz(32 * w + lr, 2 * ks + hh)), s);
      const int key = kw0 + lr;
      const bool need_mask = CAUSAL && (kw0 + 31 > q0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = __builtin_amdgcn_exp2f(s[r] * c);
        if (need_mask && key > q0 + (r & 3) + 8 * (r >> 2) + 4 * hh) p = 0.f;
        s[r] = p;
      }
      bf16x8 pf[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        u32x4 u;
#pragma unroll
        for (int i = 0; i < 4; ++i) u[i] = pack2(s[8 * ss + 2 * i], s[8 * ss + 2 * i + 1]);
        pf[ss] = as_bf16x8(u);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int row = 16 * ss + vrow, col = 32 * t + vcol;
          dV[t] = mfma32(tr_pair(dOs, swz8(row, col), swz8(row + 8, col)), pf[ss], dV[t]);
        }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) dp = mfma32(row_read(dOs, swz(lr, 2 * ks + hh)), vf[ks], dp);
      bf16x8 sf[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        u32x4 u;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          u[i] = pack2(s[8 * ss + 2 * i] * dp[8 * ss + 2 * i], s[8 * ss + 2 * i + 1] * dp[8 * ss + 2 * i + 1]);
        sf[ss] = as_bf16x8(u);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int row = 16 * ss + vrow, col = 32 * t + vcol;
          dK[t] = mfma32(tr_pair(Qs, swz8(row, col), swz8(row + 8, col)), sf[ss], dK[t]);
        }
    }
    wait_dma_barrier();
  }
  // ---- chunk partial sums: transpose [d][key] accumulators through LDS, row-contiguous adds
  float* T = reinterpret_cast<float*>(smem);   // [128 keys][128 d] fp32 = 64 KB
  auto flush = [&](const f32x16(&acc)[4], float mul, float* dst_base) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const int key = 32 * w + lr;
        T[key * 128 + (d ^ ((key & 31) << 2))] = acc[t][r] * mul;
      }
    __syncthreads();
    float* dst = dst_base + (rowB + kv0) * (long)(Hkv * D) + (long)hkv * D;
    for (int e = tid; e < BKV * 128; e += 256) {
      const int key = e >> 7, d = e & 127;
      atomicAdd(dst + (long)key * Hkv * D + d, T[key * 128 + (d ^ ((key & 31) << 2))]);
    }
    __syncthreads();
  };
  flush(dK, scale, dk_acc);
  flush(dV, 1.f, dv_acc);
}

// fp32 dK/dV accumulators -> bf16 k/v columns of the fused dqkv [T, (Hq + 2Hkv) * 128]
__global__ __launch_bounds__(256) void flash_bwd_post_kernel(const float* __restrict__ dk,
                                                             const float* __restrict__ dv,
                                                             bf16_t* __restrict__ dqkv, long ld, int T,
                                                             int Hq, int Hkv) {
  const int ck = Hkv * 16, per_row = 2 * ck;   // 8-element chunks
  const long total = (long)T * per_row;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int t = (int)(i / per_row), c = (int)(i - (long)t * per_row);
    const float* src = c < ck ? dk + (long)t * Hkv * 128 + c * 8 : dv + (long)t * Hkv * 128 + (c - ck) * 8;
    const f32x4 a = ldf4(src), bb = ldf4(src + 4);
    const float f[8] = {a[0], a[1], a[2], a[3], bb[0], bb[1], bb[2], bb[3]};
    st16(dqkv + (long)t * ld + Hq * 128 + c * 8, pack8(f));
  }
}

extern "C" {

int kf_flash_fwd(const void* qkv, long ld, void* out, long ldo, float* lse, int B, int S, int Hq,
                 int Hkv, int D_, float scale, int causal, hipStream_t st) {
  if (D_ != D || S % BQ != 0 || Hq % Hkv != 0 || ld % 8 || ldo % 8) return 1;
  const int grid = B * Hq * (S / BQ);
  const float sl2 = scale * LOG2E;
  if (causal)
    flash_fwd_kernel<true><<<grid, 256, 0, st>>>((const bf16_t*)qkv, ld, (bf16_t*)out, ldo, lse, B, S,
                                                 Hq, Hkv, sl2);
  else
    flash_fwd_kernel<false><<<grid, 256, 0, st>>>((const bf16_t*)qkv, ld, (bf16_t*)out, ldo, lse, B,
                                                  S, Hq, Hkv, sl2);
  return 0;
}

// dk_acc/dv_acc: zeroed fp32 [B*S, Hkv*128]; delta: fp32 [B, Hq, S] scratch.
int kf_flash_bwd(const void* qkv, long ld, const void* o, long ldo, const void* dout, long lddo,
                 const float* lse, float* delta, float* dk_acc, float* dv_acc, void* dqkv,
                 long lddqkv, int B, int S, int Hq, int Hkv, int D_, float scale, int causal,
                 hipStream_t st) {
  using namespace fb;
  if (D_ != D || S % BKV != 0 || S % BQ != 0 || Hq % Hkv != 0) return 1;
  const int T = B * S;
  flash_bwd_pre_kernel<<<(T * Hq + 15) / 16, 256, 0, st>>>((const bf16_t*)o, ldo, (const bf16_t*)dout,
                                                           lddo, delta, B, S, Hq);
  int items = 0;
  for (int kb = 0; kb < S / BKV; ++kb) items += (S - (causal ? kb * BKV : 0) + QCH - 1) / QCH;
  const int g_kv = B * Hkv * items, g_q = B * Hq * (S / BQ);
  const float sl2 = scale * LOG2E;
  if (causal) {
    flash_bwd_dkdv_kernel<true><<<g_kv, 256, 0, st>>>((const bf16_t*)qkv, ld, (const bf16_t*)dout, lddo,
                                                      lse, delta, dk_acc, dv_acc, B, S, Hq, Hkv, scale, items);
    flash_bwd_dq_kernel<true><<<g_q, 256, 0, st>>>((const bf16_t*)qkv, ld, (const bf16_t*)dout, lddo, lse,
                                                   delta, (bf16_t*)dqkv, lddqkv, B, S, Hq, Hkv, sl2, scale);
  } else {
    flash_bwd_dkdv_kernel<false><<<g_kv, 256, 0, st>>>((const bf16_t*)qkv, ld, (const bf16_t*)dout, lddo,
                                                       lse, delta, dk_acc, dv_acc, B, S, Hq, Hkv, scale, items);
    flash_bwd_dq_kernel<false><<<g_q, 256, 0, st>>>((const bf16_t*)qkv, ld, (const bf16_t*)dout, lddo, lse,
                                                    delta, (bf16_t*)dqkv, lddqkv, B, S, Hq, Hkv, sl2, scale);
  }
  const long chunks = (long)T * Hkv * 32;
  const int pg = (int)std::min<long>((chunks + 255) / 256, 16384);
  flash_bwd_post_kernel<<<pg, 256, 0, st>>>(dk_acc, dv_acc, (bf16_t*)dqkv, lddqkv, T, Hq, Hkv);
  return 0;
}
}
