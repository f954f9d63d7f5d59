// LAB (shipped in round 5 as ops/csrc/flash_attn.hip flash_fwd_kernel, profiles/fa_fwd128_r5.md):
// the forward with 128-key tiles (round-4 review: "a 128-key forward tile").  Included by
// fa_bench.hip after flash_attn_lab.hip; KFAMD_FA_FWD=128 times it instead of the production
// forward.  Same structure as ops/csrc/flash_attn.hip's flash_fwd_kernel (8 waves x 32 query
// rows, swapped products, the folded running max), with each K/V stage twice as deep:
//  * a stage is a 128-key K tile + V tile (64 KB); the ring holds two (128 KB), so the DMA runs
//    one tile (128 keys) ahead instead of three 64-key tiles;
//  * per tile and wave: 4 S-chain accumulators (32 MFMAs + 4 fold MFMAs), one softmax pass over
//    64 scores per lane, 32 PV MFMAs -- one barrier, one max/sum exchange and one threshold
//    ballot per 128 keys instead of per 64.
namespace f128 {
constexpr int BKF = 128;
constexpr int TILEF = BKF * D * 2;    // 32 KB
constexpr int NS = 2;                 // ring depth (stages)
constexpr int STGF = 2 * TILEF;       // K + V
constexpr int NKT = BKF / 32;         // 32-key chunks per tile
static_assert(NS * STGF <= 163840, "LDS");
#ifndef KF_F128_FP
#define KF_F128_FP FP
#endif
constexpr int FPK = KF_F128_FP;
#ifndef KF_F128_LATE
#define KF_F128_LATE 0
#endif
// 1 = O staged through LDS and stored as whole rows (16 B per lane) instead of 8-B pieces
#ifndef KF_F128_OST
#define KF_F128_OST 0
#endif
// s_setprio 1 over the S chain (bit 0) and / or the PV MFMAs (bit 1), 0 over the softmax
#ifndef KF_F128_PRIO
#define KF_F128_PRIO 0
#endif       // K row fragments read this many MFMA steps ahead
}  // namespace f128

template <bool CAUSAL>
__global__ __launch_bounds__(512, 1) void flash_fwd128_kernel(
    const bf16_t* __restrict__ qkv, long ld, bf16_t* __restrict__ out, long ldo,
    float* __restrict__ lse_out, int B, int S, int Hq, int Hkv, float scale_log2) {
  using namespace f128;
  __shared__ __attribute__((aligned(1024))) char smem[NS * STGF];
  const int nqb = (S + BQ8 - 1) / BQ8, G = Hq / Hkv;
  int lid = xcd_remap(blockIdx.x, B * Hq * nqb);
  const int g = lid % G;
  lid /= G;
  int qb = lid % nqb;
  lid /= nqb;
  const int hkv = lid % Hkv, b = lid / Hkv, h = hkv * G + g;
  if (CAUSAL) qb = nqb - 1 - qb;

  const int tid = threadIdx.x, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = qb * BQ8 + w * 32 + lr;
  const int qmin_w = qb * BQ8 + w * 32, qmax_w = qmin_w + 31;
  const bool live = qmin_w < S;

  bf16x8 qf[8];
  {
    const bf16_t* qp = qkv + ((long)b * S + min(q, S - 1)) * ld + (long)h * D + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = as_bf16x8(ld16(qp + 16 * ks));
  }
  const bf16_t* kp = qkv + (long)b * S * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + (long)b * S * ld + (long)(Hq + Hkv + hkv) * D;
  u32 dma_kv;
  {
    const int row = 4 * w + (l >> 4), ch = (l & 15) ^ swz_x(row);
    dma_kv = (u32)((row * ld + ch * 8) * 2);
  }
  const u32 lds_w = lds_addr(smem) + 1024 * w;
  // 8 DMA wave-instructions per wave per stage: 32-row segments i of the K and V tiles
  auto stage = [&](int j) {
    const u32 st = lds_w + (j % NS) * STGF;
    const char* kb_ = reinterpret_cast<const char*>(kp + (long)j * BKF * ld);
    const char* vb_ = reinterpret_cast<const char*>(vp + (long)j * BKF * ld);
#pragma unroll
    for (int i = 0; i < NKT; ++i) dma_sv(kb_ + (long)64 * ld * i, dma_kv, st + 8192 * i);
#pragma unroll
    for (int i = 0; i < NKT; ++i) dma_sv(vb_ + (long)64 * ld * i, dma_kv, st + TILEF + 8192 * i);
  };
  const int ntiles = CAUSAL ? min(S, qb * BQ8 + BQ8) / BKF : S / BKF;
  if (ntiles > 0) stage(0);
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) asm volatile("" : "+v"(qf[ks]));
  const bf16x8 ones = fold_ones(hh);
  bf16x8 mref = bf16x8{};
  bool first = true;
  const float thresh = FOLD_T / scale_log2;
  float m = 0.f, lsum = 0.f;
  f32x16 o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = f32x16{};
  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

  auto s_chain = [&](int j, f32x16 (&sc)[NKT]) {
    const u32 ln = lane_id_opaque(), lr_ = ln & 31;
    const u32 a_t = (lds_addr(smem) + (u32)((j % NS) * STGF)) + lr_ * 256 + 16 * ((ln >> 5) ^ swz_x(lr_));
    bf16x8 fk[FPK + 1];
    auto rdK = [&](auto ic) {
      constexpr int i = decltype(ic)::value, kt = i % NKT, ks = i / NKT;
      fk[i % (FPK + 1)] = rd_b128<8192 * kt>(a_t ^ (32 * ks));
    };
    static_for<0, FPK>([&](auto ic) { rdK(ic); });
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) sc[kt] = mfma32(ones, mref, f32x16{});
    static_for<0, 8 * NKT>([&](auto ic) {
      constexpr int i = decltype(ic)::value, kt = i % NKT, ks = i / NKT, NI = 8 * NKT;
      if constexpr (i + FPK < NI) rdK(std::integral_constant<int, i + FPK>());
      lgkm_tie1<(i + FPK < NI ? FPK : NI - 1 - i)>(fk[i % (FPK + 1)]);
      sc[kt] = mfma32(fk[i % (FPK + 1)], qf[ks], sc[kt]);
    });
  };
  auto soft_pv = [&](int j, f32x16 (&sc)[NKT]) {
    const int k0 = j * BKF;
    const char* Vs = smem + (j % NS) * STGF + TILEF;
    if (CAUSAL && k0 + BKF - 1 > qmin_w) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
          sc[kt][r] = key > q ? -INFINITY : sc[kt][r];
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kt][r]);
    mx = xor32_max(mx);
    if (__ballot(first || mx > thresh)) {
      const float mnew = first ? bf16_round(mx) : bf16_round(m + fmaxf(mx, 0.f));
      const float shift = first ? mnew : mnew - m;
      const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-shift * scale_log2);
      lsum *= alpha;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[kt][r] -= shift;
      m = mnew;
      first = false;
      mref = fold_const(m, hh);
    }
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(sc[kt][r] * scale_log2);
        sc[kt][r] = p;
        rs += p;
      }
    lsum += xor32_sum(rs);
    bf16x8 pf[NKT][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
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
      const int t = gi >> 1, hf = gi & 1;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int row = 32 * (2 * hf + kk) + 16 * ss + vrow, col = 32 * t + vcol;
          f[2 * kk + ss] = tr_pair_asm(vbase + swz8(row, col), vbase + swz8(row + 8, col));
        }
    };
    v_read(0, vf[0]);
    if (KF_F128_PRIO & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int gi = 0; gi < 8; ++gi) {
      if (gi < 7) {
        v_read(gi + 1, vf[(gi + 1) & 1]);
        lgkm_wait_tie<8>(vf[gi & 1]);
      } else {
        lgkm_wait_tie<0>(vf[gi & 1]);
      }
      const int t = gi >> 1, hf = gi & 1;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) o[t] = mfma32(vf[gi & 1][2 * kk + ss], pf[2 * hf + kk][ss], o[t]);
    }
    if (KF_F128_PRIO & 2) __builtin_amdgcn_s_setprio(0);
  };
  auto live_tile = [&](int j) { return live && (!CAUSAL || j * BKF <= qmax_w); };

  vm_wait<0>();
  barrier();
  f32x16 scp[NKT];
  for (int j = 0; j < ntiles; ++j) {
    // into the buffer every wave finished with (tile j-1); KF_F128_LATE=1: after this tile's S chain
    if (!KF_F128_LATE && j + 1 < ntiles) stage(j + 1);
    if (live_tile(j)) {
      if (KF_F128_PRIO & 1) __builtin_amdgcn_s_setprio(1);
      s_chain(j, scp);
      if (KF_F128_PRIO & 1) __builtin_amdgcn_s_setprio(0);
      if (KF_F128_LATE && j + 1 < ntiles) stage(j + 1);
      soft_pv(j, scp);
    } else if (KF_F128_LATE && j + 1 < ntiles) {
      stage(j + 1);
    }
    if (j + 1 < ntiles) {
      vm_wait<0>();
      barrier();
    }
  }
  if (!live) return;
  const float inv = 1.f / lsum;
#if KF_F128_OST
  {
    // O staged through the ring buffer the last tile did not use, [32 rows][256 B] per wave
    // (swizzled 16-B chunks), then stored as whole rows: 16 B per lane, 4 rows per instruction
    char* ob = smem + (ntiles % NS) * STGF + 8192 * w;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        u32x2 v;
        v[0] = pack2(o[t][4 * gq] * inv, o[t][4 * gq + 1] * inv);
        v[1] = pack2(o[t][4 * gq + 2] * inv, o[t][4 * gq + 3] * inv);
        *reinterpret_cast<u32x2*>(ob + swz(lr, 4 * t + gq) + 8 * hh) = v;
      }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    bf16_t* orow = out + ((long)b * S + qmin_w) * ldo + (long)h * D;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 4 * i + (l >> 4), ch = l & 15;
      st16(orow + (long)row * ldo + 8 * ch, *reinterpret_cast<const u32x4*>(ob + swz(row, ch)));
    }
  }
#else
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
#endif
  if (hh == 0) lse_out[((long)b * Hq + h) * S + q] = (m * scale_log2 + log2f(lsum)) * LN2;
}
