// K3: causal GQA flash attention for gfx950 (MI355X), head_dim 128, bf16 in/out.
//
// Reads q/k/v straight from the fused QKV activation [B*S, (Hq + 2*Hkv)*128] (row stride
// `ld`), writes O as [B*S, Hq*128] (row stride `ldo`) and the per-row log-sum-exp.
//
// Forward structure (one workgroup = 4 waves = 128 query rows of one (b, q-head)):
//  * S^T = K . Q^T on v_mfma_f32_32x32x16_bf16 ("swapped" QK^T): the accumulator keeps the
//    QUERY on the lane, so every lane owns one query row's scores, max, sum and rescale
//    factor -- the online softmax needs a single cross-half exchange (lane ^ 32), no LDS.
//  * O^T = V^T . P^T: the S^T accumulator, converted pairwise to bf16, IS the B operand
//    of the next MFMA (no lane movement), and V^T comes from the LDS tile through the
//    gfx950 hardware-transpose read ds_read_b64_tr_b16.  O^T's accumulator again keeps the
//    query on the lane, so the alpha rescale and the final 1/l are lane-local.
//  * K and V tiles (64 keys x 128 d, 16 KB each) are double-buffered in LDS with the
//    256-B-row XOR image that is conflict-free for both the row reads (K, ds_read_b128)
//    and the transposed reads (V); register-staged: the next tile's global loads are
//    issued before this tile's MFMAs and written to LDS after them (one barrier/tile).
//  * Grid: XCD-aware bijective remap so the workgroups resident on one XCD share one
//    (batch, kv-head) -> its K/V stay in that XCD's 4 MB L2; causal blocks run heaviest
//    (last q-block) first.
#include "common.h"

using namespace kf;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace fa {
constexpr int D = 128;
constexpr int BQ = 128;     // query rows per workgroup (4 waves x 32)
constexpr int BK = 64;      // keys per tile
constexpr int TILE = BK * D * 2;  // 16 KB
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// byte offset of 16-byte chunk `ch` (0..15) of row `row` in a [rows][128 x bf16] LDS image
__device__ __forceinline__ int swz(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 as_bf16x8(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ u32x2 tr_read(const char* p) {
  s16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p));
  return __builtin_bit_cast(u32x2, t);
}

// Bijective XCD remap: blocks b and b+8 share an XCD; give each XCD a contiguous range
// of logical ids (guide §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int bid, int total) {
  const int q = total / 8, r = total % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}
}  // namespace fa

using namespace fa;

template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) void flash_fwd_kernel(
    const bf16_t* __restrict__ qkv, long ld, bf16_t* __restrict__ out, long ldo,
    float* __restrict__ lse_out, int B, int S, int Hq, int Hkv, float scale_log2) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // K0 K1 V0 V1
  const int nqb = S / BQ;
  const int G = Hq / Hkv;
  const int total = B * Hq * nqb;
  const int lid = xcd_remap(blockIdx.x, total);
  const int g = lid % G;
  int t1 = lid / G;
  int qb = t1 % nqb;
  t1 /= nqb;
  const int hkv = t1 % Hkv;
  const int b = t1 / Hkv;
  if (CAUSAL) qb = nqb - 1 - qb;
  const int h = hkv * G + g;

  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int q = qb * BQ + w * 32 + lr;          // this lane's query (within the sequence)
  const int qmin_w = qb * BQ + w * 32, qmax_w = qmin_w + 31;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16ks + 8hh .. +8]
  bf16x8 qf[8];
  {
    const bf16_t* qp = qkv + ((long)b * S + q) * ld + (long)h * D + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = as_bf16x8(ld16(qp + 16 * ks));
  }
  const bf16_t* kp = qkv + (long)b * S * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + (long)b * S * ld + (long)(Hq + Hkv + hkv) * D;

  u32x4 kr[4], vr[4];
  auto gload = [&](int j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i, row = idx >> 4, ch = idx & 15;
      const long off = (long)(j * BK + row) * ld + ch * 8;
      kr[i] = ld16(kp + off);
      vr[i] = ld16(vp + off);
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i, row = idx >> 4, ch = idx & 15;
      *reinterpret_cast<u32x4*>(smem + buf * TILE + swz(row, ch)) = kr[i];
      *reinterpret_cast<u32x4*>(smem + (2 + buf) * TILE + swz(row, ch)) = vr[i];
    }
  };

  f32x16 o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = f32x16{};
  float m = -INFINITY, lsum = 0.f;
  const int ntiles = CAUSAL ? (qb * BQ + BQ) / BK : S / BK;

  // per-lane constant parts of the LDS addresses
  const int vrow = 4 * hh + ((l & 15) >> 2);           // + 32kt + 16ss (+8)
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);  // + 32t

  gload(0);
  swrite(0);
  __syncthreads();
  for (int j = 0; j < ntiles; ++j) {
    const int cur = j & 1;
    if (j + 1 < ntiles) gload(j + 1);
    const int k0 = j * BK;
    if (!CAUSAL || k0 <= qmax_w) {
      const char* Ks = smem + cur * TILE;
      const char* Vs = smem + (2 + cur) * TILE;
      f32x16 s[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          const bf16x8 kf = as_bf16x8(*reinterpret_cast<const u32x4*>(Ks + swz(32 * kt + lr, 2 * ks + hh)));
          s[kt] = mfma32(kf, qf[ks], s[kt]);
        }
      }
      const bool need_mask = CAUSAL && (k0 + BK - 1 > qmin_w);
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = s[kt][r] * scale_log2;
          if (need_mask) {
            const int key = k0 + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (key > q) v = -INFINITY;
          }
          s[kt][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = exp2f(m - msafe);
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = exp2f(s[kt][r] - msafe);
          s[kt][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32, 64);
      lsum = lsum * alpha + rs;
      m = mnew;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
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
            const int row = 32 * kt + 16 * ss + vrow;
            const int col = 32 * t + vcol;
            const u32x2 a0 = tr_read(Vs + swz(row, col >> 3) + 8 * ((col >> 2) & 1));
            const u32x2 a1 = tr_read(Vs + swz(row + 8, col >> 3) + 8 * ((col >> 2) & 1));
            const bf16x8 vf = as_bf16x8(u32x4{a0[0], a0[1], a1[0], a1[1]});
            o[t] = mfma32(vf, pf[kt][ss], o[t]);
          }
    }
    if (j + 1 < ntiles) swrite(cur ^ 1);
    __syncthreads();
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

extern "C" int kf_flash_fwd(const void* qkv, long ld, void* out, long ldo, float* lse, int B, int S,
                            int Hq, int Hkv, int D_, float scale, int causal, hipStream_t st) {
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

// ====================================================================================
// Backward.
//
// One workgroup = 8 waves = a 256-key block of one (batch, kv-head) x a chunk of up to
// QCH query rows, swept for all G query heads of the GQA group (so dK/dV of the block
// accumulate in registers across the group).  Per 32-row query tile:
//   S   = Q K^T   (key on the lane; accumulator initialised to -lse/c, so p = exp2(c*S'))
//   dP  = dO V^T  (accumulator initialised to -delta, delta = rowsum(dO*O))
//   P, dS = P*(dP-delta) never leave registers for dV/dK: as 32x32 accumulators with the
//   query on the register axis they ARE the B operands of
//   dV^T += dO^T P  and  dK^T += Q^T dS  (A operands via ds_read_b64_tr_b16 of the staged
//   Q/dO tiles).  Each wave owns 32 keys: dK^T+dV^T = 128 accumulator registers.
//   dQ  = dS K: dS^T crosses LDS once (XOR-swizzled 64-B rows), every wave computes two
//   16x16 dQ tiles over all 256 keys on v_mfma_f32_16x16x32_bf16 (both operands by
//   transposed reads) and adds them to an fp32 dQ accumulator with no-return float
//   atomics (Guideline 12: 256 keys/WG -> 640 FLOP per atomic byte).
// dK/dV partial sums are transposed through LDS at the end and added row-contiguously.
// Work list: for every 256-key block, query chunks of QCH rows (causal: only q >= k0),
// so the causal triangle is cut into near-equal work items.
// ====================================================================================
namespace fb {
constexpr int BKV = 256;
constexpr int QT = 32;
constexpr int QCH = 512;
constexpr int OFF_K = 0;                   // 256 x 256 B
constexpr int OFF_Q = 65536;               // [2][32 x 256 B]
constexpr int OFF_DO = OFF_Q + 16384;      // [2][32 x 256 B]
constexpr int OFF_DS = OFF_DO + 16384;     // [2][256 keys x 64 B]
constexpr int OFF_LD = OFF_DS + 32768;     // [2][lse2 32 f32 | delta 32 f32]
constexpr int SMEM = OFF_LD + 512;         // 131584 B
typedef __attribute__((ext_vector_type(4))) float f4;

__device__ __forceinline__ f4 mfma16(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// dS^T image: row = key (64 B = 32 q), 8-byte chunk c (4 q) XOR-swizzled by row
__device__ __forceinline__ int ds_off(int key, int c) { return key * 64 + ((c ^ (key & 7)) << 3); }

// number of query chunks for key block kb
__device__ __forceinline__ int n_chunks(int kb, int S, bool causal) {
  const int q0 = causal ? kb * BKV : 0;
  return (S - q0 + QCH - 1) / QCH;
}
}  // namespace fb

template <bool CAUSAL>
__global__ __launch_bounds__(512, 2) void flash_bwd_kernel(
    const bf16_t* __restrict__ qkv, long ld, const bf16_t* __restrict__ dout, long lddo,
    const float* __restrict__ lse, const float* __restrict__ delta, float* __restrict__ dq_acc,
    float* __restrict__ dk_acc, float* __restrict__ dv_acc, int B, int S, int Hq, int Hkv,
    float scale, int items_per_head) {
  using namespace fb;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int G = Hq / Hkv;
  const int total = B * Hkv * items_per_head;
  const int lid = xcd_remap(blockIdx.x, total);
  int item = lid % items_per_head;
  const int bh = lid / items_per_head;
  const int hkv = bh % Hkv, b = bh / Hkv;
  // decode (kb, chunk) from the flat item index
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

  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int kw0 = kv0 + 32 * w;          // this wave's first key
  const float c = scale * LOG2E;         // S -> log2 domain
  const float inv_c = 1.f / c;
  const long rowK = (long)b * S;
  const bf16_t* kp = qkv + rowK * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + rowK * ld + (long)(Hq + Hkv + hkv) * D;

  // K block -> LDS (swizzled 256-B rows), V fragments -> registers (B operand of dP)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int idx = tid + 512 * i, row = idx >> 4, ch = idx & 15;
    *reinterpret_cast<u32x4*>(smem + OFF_K + swz(row, ch)) = ld16(kp + (long)(kv0 + row) * ld + ch * 8);
  }
  bf16x8 vf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) vf[ks] = as_bf16x8(ld16(vp + (long)(kw0 + lr) * ld + 16 * ks + 8 * hh));

  f32x16 dK[4], dV[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) { dK[t] = f32x16{}; dV[t] = f32x16{}; }

  // staging of one (head, q-tile): Q row chunk, dO row chunk, lse/delta scalar
  u32x4 sq, sdo;
  float sld = 0.f;
  auto gload = [&](int it) {
    const int hq = it / ntq, qt = it - hq * ntq;
    const int h = hkv * G + hq;
    const int q0 = qs + qt * QT;
    const int row = tid >> 4, ch = tid & 15;
    sq = ld16(qkv + (rowK + q0 + row) * ld + (long)h * D + ch * 8);
    sdo = ld16(dout + (rowK + q0 + row) * lddo + (long)h * D + ch * 8);
    if (tid < 32) sld = lse[((long)b * Hq + h) * S + q0 + tid] * LOG2E;
    else if (tid < 64) sld = delta[((long)b * Hq + h) * S + q0 + tid - 32];
  };
  auto swrite = [&](int buf) {
    const int row = tid >> 4, ch = tid & 15;
    *reinterpret_cast<u32x4*>(smem + OFF_Q + buf * 8192 + swz(row, ch)) = sq;
    *reinterpret_cast<u32x4*>(smem + OFF_DO + buf * 8192 + swz(row, ch)) = sdo;
    if (tid < 64) reinterpret_cast<float*>(smem + OFF_LD + buf * 256)[tid] = sld;
  };

  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);
  // dQ tiling: wave -> q half (16 rows) and two 16-wide d tiles
  const int qh = w & 1, dt0 = 2 * (w >> 1);
  const int g16 = l >> 4, i16 = l & 15;

  if (niter > 0) {
    gload(0);
    swrite(0);
  }
  __syncthreads();
  for (int it = 0; it < niter; ++it) {
    const int cur = it & 1;
    const int hq = it / ntq, qt = it - hq * ntq;
    const int h = hkv * G + hq;
    const int q0 = qs + qt * QT;
    if (it + 1 < niter) gload(it + 1);
    const char* Qs = smem + OFF_Q + cur * 8192;
    const char* dOs = smem + OFF_DO + cur * 8192;
    const float* Ls = reinterpret_cast<const float*>(smem + OFF_LD + cur * 256);
    char* dSt = smem + OFF_DS + cur * 16384;
    const bool active = !CAUSAL || (kw0 <= q0 + QT - 1);
    if (active) {
      // row constants: q(r) = (r&3) + 8(r>>2) + 4hh
      f32x16 s, dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f4 L4 = *reinterpret_cast<const f4*>(Ls + 8 * g + 4 * hh);
        const f4 D4 = *reinterpret_cast<const f4*>(Ls + 32 + 8 * g + 4 * hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) { s[4 * g + i] = -L4[i] * inv_c; dp[4 * g + i] = -D4[i]; }
      }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const bf16x8 qa = as_bf16x8(*reinterpret_cast<const u32x4*>(Qs + swz(lr, 2 * ks + hh)));
        const bf16x8 kb_ = as_bf16x8(*reinterpret_cast<const u32x4*>(smem + OFF_K + swz(32 * w + lr, 2 * ks + hh)));
        s = mfma32(qa, kb_, s);
      }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const bf16x8 da = as_bf16x8(*reinterpret_cast<const u32x4*>(dOs + swz(lr, 2 * ks + hh)));
        dp = mfma32(da, vf[ks], dp);
      }
      const int key = kw0 + lr;
      const bool need_mask = CAUSAL && (kw0 + 31 > q0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = exp2f(s[r] * c);
        if (need_mask) {
          const int qq = q0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (key > qq) p = 0.f;
        }
        s[r] = p;             // P
        dp[r] = p * dp[r];    // dS (unscaled)
      }
      bf16x8 pf[2], sf[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        u32x4 u, v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          u[i] = pack2(s[8 * ss + 2 * i], s[8 * ss + 2 * i + 1]);
          v[i] = pack2(dp[8 * ss + 2 * i], dp[8 * ss + 2 * i + 1]);
        }
        pf[ss] = as_bf16x8(u);
        sf[ss] = as_bf16x8(v);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int row = 16 * ss + vrow, col = 32 * t + vcol;
          const int o0 = swz(row, col >> 3) + 8 * ((col >> 2) & 1);
          const int o1 = swz(row + 8, col >> 3) + 8 * ((col >> 2) & 1);
          const u32x2 a0 = tr_read(dOs + o0), a1 = tr_read(dOs + o1);
          dV[t] = mfma32(as_bf16x8(u32x4{a0[0], a0[1], a1[0], a1[1]}), pf[ss], dV[t]);
          const u32x2 b0 = tr_read(Qs + o0), b1 = tr_read(Qs + o1);
          dK[t] = mfma32(as_bf16x8(u32x4{b0[0], b0[1], b1[0], b1[1]}), sf[ss], dK[t]);
        }
      // dS^T[key][q] (bf16): 4 consecutive q per register group
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 v;
        v[0] = pack2(dp[4 * g], dp[4 * g + 1]);
        v[1] = pack2(dp[4 * g + 2], dp[4 * g + 3]);
        *reinterpret_cast<u32x2*>(dSt + ds_off(32 * w + lr, 2 * g + hh)) = v;
      }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<u32x2*>(dSt + ds_off(32 * w + lr, 2 * g + hh)) = u32x2{0u, 0u};
    }
    if (it + 1 < niter) swrite(cur ^ 1);
    __syncthreads();
    // dQ[q0 + 16qh + ..][16(dt0+e) + ..] = sum_k dS[q][k] K[k][d]
    {
      f4 dq0 = f4{}, dq1 = f4{};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int krow = 32 * ks + 8 * g16 + (i16 >> 2);
        const int qcol = 16 * qh + 4 * (i16 & 3);
        const u32x2 a0 = tr_read(dSt + ds_off(krow, qcol >> 2));
        const u32x2 a1 = tr_read(dSt + ds_off(krow + 4, qcol >> 2));
        const bf16x8 af = as_bf16x8(u32x4{a0[0], a0[1], a1[0], a1[1]});
        const int dc0 = 16 * dt0 + 4 * (i16 & 3), dc1 = dc0 + 16;
        const u32x2 b0 = tr_read(smem + OFF_K + swz(krow, dc0 >> 3) + 8 * ((dc0 >> 2) & 1));
        const u32x2 b1 = tr_read(smem + OFF_K + swz(krow + 4, dc0 >> 3) + 8 * ((dc0 >> 2) & 1));
        dq0 = mfma16(af, as_bf16x8(u32x4{b0[0], b0[1], b1[0], b1[1]}), dq0);
        const u32x2 e0 = tr_read(smem + OFF_K + swz(krow, dc1 >> 3) + 8 * ((dc1 >> 2) & 1));
        const u32x2 e1 = tr_read(smem + OFF_K + swz(krow + 4, dc1 >> 3) + 8 * ((dc1 >> 2) & 1));
        dq1 = mfma16(af, as_bf16x8(u32x4{e0[0], e0[1], e1[0], e1[1]}), dq1);
      }
      // C(16x16): col = d = lane&15, row = 4*(lane>>4) + i
      float* dqp = dq_acc + (rowK + q0 + 16 * qh + 4 * g16) * (long)(Hq * D) + (long)h * D + 16 * dt0 + i16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        atomicAdd(dqp + (long)i * Hq * D, dq0[i] * scale);
        atomicAdd(dqp + (long)i * Hq * D + 16, dq1[i] * scale);
      }
    }
  }
  // ---- dK / dV: transpose the [d][key] accumulators through LDS, then row-contiguous adds
  __syncthreads();
  float* T = reinterpret_cast<float*>(smem);   // [256 keys][128 d] fp32 = 128 KB
  auto flush = [&](const f32x16 (&acc)[4], float mul, float* dst_base) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const int key = 32 * w + lr;
        T[key * 128 + (d ^ ((key & 31) << 2))] = acc[t][r] * mul;
      }
    __syncthreads();
    float* dst = dst_base + (rowK + kv0) * (long)(Hkv * D) + (long)hkv * D;
    for (int e = tid; e < BKV * 128; e += 512) {
      const int key = e >> 7, d = e & 127;
      atomicAdd(dst + (long)key * Hkv * D + d, T[key * 128 + (d ^ ((key & 31) << 2))]);
    }
    __syncthreads();
  };
  flush(dK, scale, dk_acc);
  flush(dV, 1.f, dv_acc);
}

// delta[b, h, q] = sum_d dO[q, h, d] * O[q, h, d]   (16 lanes per row, 8 elems per lane)
__global__ __launch_bounds__(256) void flash_bwd_pre_kernel(const bf16_t* __restrict__ o, long ldo,
                                                            const bf16_t* __restrict__ dout, long lddo,
                                                            float* __restrict__ delta, int B, int S,
                                                            int Hq) {
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);   // over B*S*Hq
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

// fp32 accumulators -> bf16 fused dqkv [T, (Hq + 2Hkv) * 128]
__global__ __launch_bounds__(256) void flash_bwd_post_kernel(const float* __restrict__ dq,
                                                             const float* __restrict__ dk,
                                                             const float* __restrict__ dv,
                                                             bf16_t* __restrict__ dqkv, long ld, int T,
                                                             int Hq, int Hkv) {
  const int cq = Hq * 16, ck = Hkv * 16, per_row = cq + 2 * ck;   // 8-element chunks
  const long total = (long)T * per_row;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int t = (int)(i / per_row), c = (int)(i - (long)t * per_row);
    const float* src;
    if (c < cq) src = dq + (long)t * Hq * 128 + c * 8;
    else if (c < cq + ck) src = dk + (long)t * Hkv * 128 + (c - cq) * 8;
    else src = dv + (long)t * Hkv * 128 + (c - cq - ck) * 8;
    const f32x4 a = ldf4(src), bb = ldf4(src + 4);
    const float f[8] = {a[0], a[1], a[2], a[3], bb[0], bb[1], bb[2], bb[3]};
    st16(dqkv + (long)t * ld + c * 8, pack8(f));
  }
}

extern "C" int kf_flash_bwd(const void* qkv, long ld, const void* o, long ldo, const void* dout,
                            long lddo, const float* lse, float* delta, float* dq_acc, float* dk_acc,
                            float* dv_acc, void* dqkv, long lddqkv, int B, int S, int Hq, int Hkv,
                            int D_, float scale, int causal, hipStream_t st) {
  using namespace fb;
  if (D_ != D || S % BKV != 0 || Hq % Hkv != 0) return 1;
  const int T = B * S;
  flash_bwd_pre_kernel<<<(T * Hq + 15) / 16, 256, 0, st>>>((const bf16_t*)o, ldo, (const bf16_t*)dout,
                                                           lddo, delta, B, S, Hq);
  int items = 0;
  for (int kb = 0; kb < S / BKV; ++kb) {
    const int q0 = causal ? kb * BKV : 0;
    items += (S - q0 + QCH - 1) / QCH;
  }
  const int grid = B * Hkv * items;
  if (causal)
    flash_bwd_kernel<true><<<grid, 512, 0, st>>>((const bf16_t*)qkv, ld, (const bf16_t*)dout, lddo,
                                                 lse, delta, dq_acc, dk_acc, dv_acc, B, S, Hq, Hkv,
                                                 scale, items);
  else
    flash_bwd_kernel<false><<<grid, 512, 0, st>>>((const bf16_t*)qkv, ld, (const bf16_t*)dout, lddo,
                                                  lse, delta, dq_acc, dk_acc, dv_acc, B, S, Hq, Hkv,
                                                  scale, items);
  long chunks = (long)T * (Hq + 2 * Hkv) * 16;
  int pg = (int)std::min<long>((chunks + 255) / 256, 16384);
  flash_bwd_post_kernel<<<pg, 256, 0, st>>>(dq_acc, dk_acc, dv_acc, (bf16_t*)dqkv, lddqkv, T, Hq, Hkv);
  return 0;
}
