// LAB: the dQ kernel with 128-key stages (two 64-key halves per stage, one barrier per stage,
// 2-deep ring of 64 KB stages) -- the staging of the shipped 128-key forward applied to dQ.
// Included by fa_bench.hip; KFAMD_FA_DQ=128 times it instead of the production dQ kernel.
#ifndef KF_DQ128_UNROLL
#define KF_DQ128_UNROLL 0
#endif
#ifndef KF_DQ128_OST
#define KF_DQ128_OST 0
#endif
// 1 = s_setprio 1 over the S/dP and dQ MFMA chains, 0 over the exp / pack VALU
#ifndef KF_DQ128_PRIO
#define KF_DQ128_PRIO 0
#endif
namespace d128 {
constexpr int BK2 = 128, TILE2 = BK2 * D * 2, NS2 = 2, STG2 = 2 * TILE2;
static_assert(NS2 * STG2 <= 163840, "LDS");
}  // namespace d128

template <bool CAUSAL>
__global__ __launch_bounds__(512, 1) void flash_bwd_dq128_kernel(
    const bf16_t* __restrict__ qkv, long ld, const bf16_t* __restrict__ dout, long lddo,
    const float* __restrict__ lse, const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    long lddq, int B, int S, int Hq, int Hkv, float scale_log2, float scale) {
  __shared__ __attribute__((aligned(1024))) char smem[d128::NS2 * d128::STG2];
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
  const int q = qb * BQ8 + w * 32 + lr, qc = min(q, S - 1);
  const int qmin_w = qb * BQ8 + w * 32, qmax_w = qmin_w + 31;
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
  // wave w fills rows 4w.. and 4w+32.. of the K and V images: SGPR panel base + one 32-bit lane
  // offset shared by K and V (same row stride; rows 32 apart share the chunk swizzle)
  u32 dma_kv;
  {
    const int row = 4 * w + (l >> 4), ch = (l & 15) ^ swz_x(row);
    dma_kv = (u32)((row * ld + ch * 8) * 2);
  }
  const u32 lds_w = lds_addr(smem) + 1024 * w;
  // a stage is 128 keys of K and V (8 DMA wave-instructions per wave); 2-deep ring
  auto stage = [&](int j) {
    const u32 st = lds_w + (j % d128::NS2) * d128::STG2;
    const char* kb_ = reinterpret_cast<const char*>(kp + (long)j * d128::BK2 * ld);
    const char* vb_ = reinterpret_cast<const char*>(vp + (long)j * d128::BK2 * ld);
#pragma unroll
    for (int i = 0; i < 4; ++i) dma_sv(kb_ + (long)64 * ld * i, dma_kv, st + 8192 * i);
#pragma unroll
    for (int i = 0; i < 4; ++i) dma_sv(vb_ + (long)64 * ld * i, dma_kv, st + d128::TILE2 + 8192 * i);
  };
  const int ntiles = CAUSAL ? min(S, qb * BQ8 + BQ8) / d128::BK2 : S / d128::BK2;
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
    if (j + 1 < ntiles) stage(j + 1);
#if KF_DQ128_UNROLL
#pragma unroll
#else
#pragma nounroll
#endif
    for (int hf = 0; hf < 2; ++hf) {   // the stage's two 64-key halves, one barrier per stage
    const int k0 = j * d128::BK2 + BK * hf;
    if (live && (!CAUSAL || k0 <= qmax_w)) {
      const u32 hoff = (u32)((j % d128::NS2) * d128::STG2 + 16384 * hf);
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
        fv[sl] = rd_b128<d128::TILE2 + 8192 * kt>(a_t ^ (32 * ks));
      };
      static_for<0, QP>([&](auto ic) { rdS(ic); });
      if (KF_DQ128_PRIO) __builtin_amdgcn_s_setprio(1);
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
          if (KF_DQ128_PRIO) __builtin_amdgcn_s_setprio(0);
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
          if (KF_DQ128_PRIO) __builtin_amdgcn_s_setprio(1);
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
      if (KF_DQ128_PRIO) __builtin_amdgcn_s_setprio(0);
    }
    }
    if (j + 1 < ntiles) {
      vm_wait<0>();
      barrier();
    }
  }
  if (!live) return;
#if KF_DQ128_OST
  {
    // dQ staged through the ring buffer the last stage did not use, then whole-row stores
    char* ob = smem + (ntiles % d128::NS2) * d128::STG2 + 8192 * w;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        u32x2 v;
        v[0] = pack2(dq[t][4 * gq] * scale, dq[t][4 * gq + 1] * scale);
        v[1] = pack2(dq[t][4 * gq + 2] * scale, dq[t][4 * gq + 3] * scale);
        *reinterpret_cast<u32x2*>(ob + swz(lr, 4 * t + gq) + 8 * hh) = v;
      }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    bf16_t* orow = dqkv + ((long)b * S + qmin_w) * lddq + (long)h * D;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 4 * i + (l >> 4), ch = l & 15;
      st16(orow + (long)row * lddq + 8 * ch, *reinterpret_cast<const u32x4*>(ob + swz(row, ch)));
    }
  }
#else
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
#endif
}

