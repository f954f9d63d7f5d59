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
