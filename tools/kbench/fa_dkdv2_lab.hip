// LAB: dK/dV backward at ONE wave per SIMD with a software-pipelined iteration (candidate for
// ops/csrc/flash_attn.hip).  Includes the production kernels (helpers, reference dK/dV kernel).
//
// Geometry: 1 workgroup = 4 waves = 256 keys of one (batch, kv head); wave w owns keys
// kv0 + 64w .. +63 as two 32-key groups g0 / g1, and keeps their dK^T / dV^T (4 column blocks
// x 2 groups x 2 = 16 accumulators = 256 registers) in AGPRs across its work item (a query
// chunk, all G query heads).  Per iteration (32 query rows of one head) 68 MFMAs: the row-
// constant folds (2 per group), S = Q K'^T and dP = dO V^T (16 per group), dV^T += dO^T P and
// dK^T += Q^T dS (16 per group).
//
// The iteration is four steps whose MFMA chains each run beside the VALU work of ANOTHER chain
// (one wave per SIMD: nothing else hides the softmax):
//   A  S/dP(g0, it)          | softmax(g1, it-1): P, dS, bf16 packing
//   B  dV/dK(g1, it-1)       | P(g0, it)
//   C  S/dP(g1, it)          | dS(g0, it)
//   D  dV/dK(g0, it)         | --
// so g1's dV/dK lag one iteration and read the previous iteration's Q/dO buffer: a 4-deep
// LDS ring of Q / dO / (lse, delta) tiles, staged by LDS-DMA two iterations ahead, one counted
// vmcnt + barrier per iteration.  K' = c K (c = scale log2 e) is pre-scaled in LDS once per
// work item, so p = exp2(S' - lse log2 e) costs one v_exp (the row constant is folded).
// Causally masked iterations (the first 256 query rows of a key block's first chunk) are a
// separate instantiation of the body, run first (query tiles are the outer index).
#include "flash_attn.hip"

namespace f2 {
constexpr int NW2 = 4, KPW = 64, BKV2 = NW2 * KPW;   // 256 keys per workgroup
constexpr int QT2 = 32;
#ifndef KF2_QCH
#define KF2_QCH 1024
#endif
constexpr int QCH2 = KF2_QCH;
constexpr int NBUF = 4;
#ifndef KF2_NOPIPE
#define KF2_NOPIPE 0
#endif
#ifndef KF2_PA
#define KF2_PA 2
#endif
#ifndef KF2_PT
#define KF2_PT 3
#endif
// per-iteration buffer b = [Q tile | dO tile] at OFF_BUF + 16 KB b (the buffer base is in the
// lane address VGPR; only the Q / dO split is a ds_read immediate: immediates stay < 32 KB --
// a transposed read at offset 0x8400 measured wrong dV, row reads there were fine); K after
constexpr int OFF_LD = 0;                             // [4][lse 32 f32 | delta 32 f32]
constexpr int OFF_BUF = 1024;                         // [4][Q 32 x 256 B | dO 32 x 256 B]
constexpr int BUFB = 16384;
constexpr int IQ = 0, IDO = 8192;                     // immediates inside a buffer
constexpr int OFF_K = OFF_BUF + NBUF * BUFB;          // [256 keys x 256 B]
constexpr int SMEM = OFF_K + BKV2 * 256;               // 132096 B
static_assert(SMEM >= BKV2 * 128 * 4, "flush transpose fits");

__host__ __device__ inline int n_chunks(int kb, int S, bool causal) {
  const int q0 = causal ? kb * BKV2 : 0;
  return (S - q0 + QCH2 - 1) / QCH2;
}

// acc += a.b with the accumulator pinned to AGPRs (two wait states first: the hazard recognizer
// does not look inside inline asm and a VALU op may just have written b)
#ifndef KF2_NOP_N
#define KF2_NOP_N 1
#endif
#define KF2_STR2(x) #x
#define KF2_STR(x) KF2_STR2(x)
#define KF2_NOP "s_nop " KF2_STR(KF2_NOP_N)
__device__ __forceinline__ void mfma_acc(f32x16& acc, bf16x8 a, bf16x8 b) {
  asm volatile(KF2_NOP "\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void drain_mfma() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }
template <int N>
__device__ __forceinline__ void lgkm_t1(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_t3(bf16x8& a, bf16x8& b, bf16x8& c) {
  asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_tf2(float& a, float& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N) : "memory");
}
__device__ __forceinline__ bf16x8 rdv_b128(u32 a) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return as_bf16x8(r);
}
__device__ __forceinline__ float rdv_b32(u32 a) {
  float r;
  asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}
__device__ __forceinline__ bf16x8 rdv_tr2(u32 a0, u32 a1) {
  u32x2 x, y;
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3" : "=&v"(x), "=v"(y) : "v"(a0), "v"(a1) : "memory");
  return as_bf16x8(u32x4{x[0], x[1], y[0], y[1]});
}
}  // namespace f2

template <bool CAUSAL>
__global__ __launch_bounds__(256, 1) void flash_bwd_dkdv2_kernel(
    const bf16_t* __restrict__ qkv, long ld, const bf16_t* __restrict__ dout, long lddo,
    const float* __restrict__ lse, const float* __restrict__ delta, float* __restrict__ dk_acc,
    float* __restrict__ dv_acc, int B, int S, int Hq, int Hkv, float scale, int items_per_head) {
  using namespace f2;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  const int G = Hq / Hkv;
  const int lid = xcd_remap(blockIdx.x, B * Hkv * items_per_head);
  int item = lid % items_per_head;
  const int bh = lid / items_per_head;
  const int hkv = bh % Hkv, b = bh / Hkv;
  const int nkb = S / BKV2;
  int kb = 0;
  for (; kb < nkb; ++kb) {
    const int n = n_chunks(kb, S, CAUSAL);
    if (item < n) break;
    item -= n;
  }
  const int kv0 = kb * BKV2;
  const int qs = (CAUSAL ? kv0 : 0) + item * QCH2;
  const int qe = min(S, qs + QCH2);
  const int ntq = (qe - qs) / QT2;
  const int niter = ntq * G;
  // causally masked iterations: query tiles below kv0 + 256 (first chunk only), all heads
  const int ndiag = (CAUSAL && item == 0) ? min(ntq, BKV2 / QT2) * G : 0;

  const int tid = threadIdx.x, l = tid & 63, lr = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kw0 = kv0 + KPW * w;
  const float c = scale * LOG2E;
  const long rowB = (long)b * S;
  const bf16_t* kp = qkv + rowB * ld + (long)(Hq + hkv) * D;
  const bf16_t* vp = qkv + rowB * ld + (long)(Hq + Hkv + hkv) * D;
  const u32 sbase = lds_addr(smem);

  // ---- K' = c K into LDS (256 rows), V into registers (B operand of dP = dO V^T)
  stage_rows(kp + (long)kv0 * ld, ld, smem + OFF_K, BKV2, w, NW2, l);
  bf16x8 vf[2][8];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      vf[g][ks] = as_bf16x8(ld16(vp + (long)(kw0 + 32 * g + lr) * ld + 16 * ks + 8 * hh));
  wait_dma_barrier();
  {
    u32x4* kimg = reinterpret_cast<u32x4*>(smem + OFF_K);
#pragma unroll 4
    for (int i = tid; i < BKV2 * 16; i += 256) {
      float f[8];
      unpack8(kimg[i], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= c;
      kimg[i] = pack8(f);
    }
  }
  // V must be in registers before the loop (a first use inside it would wait vmcnt(0) on DMA)
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) asm volatile("" : "+v"(vf[g][ks]));
  __syncthreads();

  // ---- per-iteration Q / dO / (lse, delta) staging; iteration it = (query tile it / G, head it % G)
  u32 dma_q, dma_do;
  {
    const int row = 4 * w + (l >> 4), ch = (l & 15) ^ swz_x(row);
    dma_q = (u32)((row * ld + ch * 8) * 2);
    dma_do = (u32)((row * lddo + ch * 8) * 2);
  }
  auto stage = [&](int it) {
    const int qt = it / G, hq = it - qt * G;
    const int h = hkv * G + hq;
    const int q0 = qs + qt * QT2;
    const int buf = it & (NBUF - 1);
    const char* qb_ = reinterpret_cast<const char*>(qkv + (rowB + q0) * ld + (long)h * D);
    const char* db_ = reinterpret_cast<const char*>(dout + (rowB + q0) * lddo + (long)h * D);
    const u32 lq = sbase + OFF_BUF + buf * BUFB + IQ + 1024 * w, ldo_ = sbase + OFF_BUF + buf * BUFB + IDO + 1024 * w;
    dma_sv(qb_, dma_q, lq);
    dma_sv(db_, dma_do, ldo_);
    dma_sv(qb_ + 32 * ld, dma_q, lq + 4096);
    dma_sv(db_ + 32 * lddo, dma_do, ldo_ + 4096);
    if (w == 0) {
      int lo = l;
      asm volatile("" : "+v"(lo));
      const float* src = (lo < 32 ? lse : delta) + ((long)b * Hq + h) * S + q0 + (lo & 31);
      glds4(src, smem + OFF_LD + buf * 256);
    }
  };
  // wait until the stage after `it` landed, leaving the one after that in flight if it exists
  auto wait_next = [&](int it) {
    if (it + 2 < niter) {
      if (w == 0) vm_wait<5>(); else vm_wait<4>();
    } else {
      vm_wait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
  };

  f32x16 dK[2][4], dV[2][4];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int t = 0; t < 4; ++t) { dK[g][t] = f32x16{}; dV[g][t] = f32x16{}; }

  // lane address parts (smem 1024-aligned; k-step / column-block terms are carry-free XORs)
  const u32 a_row0 = sbase + lr * 256 + 16 * (hh ^ swz_x(lr));
  const u32 a_k00 = a_row0 + OFF_K + (KPW * w) * 256;        // group g: + 8192 g
  const u32 a_rowb = a_row0 + OFF_BUF;                        // + buffer offset per iteration
  const int vrow = 4 * hh + ((l & 15) >> 2);
  const int vcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);
  u32 a_tr0[2][2];
#pragma unroll
  for (int ss = 0; ss < 2; ++ss)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int row = 16 * ss + vrow + 8 * hf;
      a_tr0[ss][hf] = sbase + OFF_BUF + row * 256 + 16 * ((vcol >> 3) ^ swz_x(row)) + 8 * (l & 1);
    }
  const bf16x8 ones = fold_ones(hh);

  // pipeline state carried between iterations: group g1 of the previous iteration
  f32x16 s1, dp1;               // its S' / dP' accumulators (softmax pending)
  int q0_prev = 0;              // its query tile
  u32 buf_prev = 0;             // its Q/dO buffer offset

  // S/dP chain of group g (both accumulators start from the folded row constants); the buffer
  // offset is in the lane base, the tile offsets are ds_read immediates.  After each k-step's two
  // MFMAs the caller's VALU chunk fill(ks) is placed (sched_barrier: the emitted order is this
  // order, one chunk per two MFMA issue gaps).
  auto sdp_chain = [&](auto gc, u32 boff, float lse_v, float dl_v, f32x16& s, f32x16& dp, auto&& fill) {
    constexpr int g = decltype(gc)::value;
    u32 a_b = a_rowb + boff, a_k = a_k00;
    asm volatile("" : "+v"(a_b), "+v"(a_k));
    constexpr int PA = KF2_PA;
    bf16x8 fq[PA + 1], fk[PA + 1], fd[PA + 1];
    auto rdA = [&](auto kc) {
      constexpr int ks = decltype(kc)::value, sl = ks % (PA + 1);
      fq[sl] = rd_b128<IQ>(a_b ^ (32 * ks));
      fk[sl] = rd_b128<8192 * g>(a_k ^ (32 * ks));
      fd[sl] = rd_b128<IDO>(a_b ^ (32 * ks));
    };
    static_for<0, PA>([&](auto kc) { rdA(kc); });
    s = mfma32(fold_const(lse_v * LOG2E, hh), ones, f32x16{});
    dp = mfma32(fold_const(dl_v, hh), ones, f32x16{});
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, 8>([&](auto kc) {
      constexpr int ks = decltype(kc)::value, sl = ks % (PA + 1);
      if constexpr (ks + PA < 8) rdA(std::integral_constant<int, ks + PA>());
      lgkm_t3<3 * (ks + PA < 8 ? PA : 7 - ks)>(fq[sl], fk[sl], fd[sl]);
      s = mfma32(fq[sl], fk[sl], s);
      dp = mfma32(fd[sl], vf[g][ks], dp);
      fill(kc);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  // VALU chunks on one group's S'/dP' (element pair i = 2i, 2i+1; packed pair i lands in word i)
  auto p_pair = [&](auto maskc, int key, int q0, f32x16& s, u32 (&pu)[8], auto ic) {
    constexpr bool MASK = decltype(maskc)::value;
    constexpr int i = decltype(ic)::value;
    float p0 = __builtin_amdgcn_exp2f(s[2 * i]), p1 = __builtin_amdgcn_exp2f(s[2 * i + 1]);
    if constexpr (MASK) {
      constexpr int r0 = 2 * i, r1 = 2 * i + 1;
      const int qb = q0 + 4 * hh - key;        // masked iff key > q, i.e. qb + row(r) < 0
      p0 = qb + (r0 & 3) + 8 * (r0 >> 2) < 0 ? 0.f : p0;
      p1 = qb + (r1 & 3) + 8 * (r1 >> 2) < 0 ? 0.f : p1;
    }
    s[2 * i] = p0;
    s[2 * i + 1] = p1;
    pu[i] = pack2(p0, p1);
  };
  auto ds_pair = [&](const f32x16& s, const f32x16& dp, u32 (&su)[8], auto ic) {
    constexpr int i = decltype(ic)::value;
    su[i] = pack2(s[2 * i] * dp[2 * i], s[2 * i + 1] * dp[2 * i + 1]);
  };
  auto as_frag = [](const u32 (&u)[8], int ss) {
    return as_bf16x8(u32x4{u[4 * ss], u[4 * ss + 1], u[4 * ss + 2], u[4 * ss + 3]});
  };
  // dV^T += dO^T P and dK^T += Q^T dS for group g from the buffer at `boff`; transposed fragments
  // (dO^T then Q^T; column block t, row half ss) three ahead; fill(j) after MFMA j
  auto dvdk = [&](auto gc, u32 boff, const u32 (&pu)[8], const u32 (&su)[8], auto&& fill) {
    constexpr int g = decltype(gc)::value;
    u32 t00 = a_tr0[0][0] + boff, t01 = a_tr0[0][1] + boff, t10 = a_tr0[1][0] + boff, t11 = a_tr0[1][1] + boff;
    asm volatile("" : "+v"(t00), "+v"(t01), "+v"(t10), "+v"(t11));
    const u32 a_t[2][2] = {{t00, t01}, {t10, t11}};
    constexpr int PT = KF2_PT;
    bf16x8 ft[PT + 1];
    auto rdT = [&](auto jc) {
      constexpr int j = decltype(jc)::value, t = (j & 7) >> 1, ss = j & 1;
      ft[j % (PT + 1)] = rd_tr2<(j < 8 ? IDO : IQ)>(a_t[ss][0] ^ (64 * t), a_t[ss][1] ^ (64 * t));
    };
    static_for<0, PT>([&](auto jc) { rdT(jc); });
    static_for<0, 16>([&](auto jc) {
      constexpr int j = decltype(jc)::value, t = (j & 7) >> 1, ss = j & 1, sl = j % (PT + 1);
      if constexpr (j + PT < 16) rdT(std::integral_constant<int, j + PT>());
      lgkm_t1<2 * (j + PT < 16 ? PT : 15 - j)>(ft[sl]);
      if constexpr (j < 8) mfma_acc(dV[g][t], ft[sl], as_frag(pu, ss));
      else mfma_acc(dK[g][t], ft[sl], as_frag(su, ss));
      fill(jc);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // A self-contained (not pipelined) iteration: both groups finished here.  Used for the
  // causally masked iterations (the first 256 query rows of a key block, ~5 % of the work):
  // folding the mask into the pipelined body raised its register pressure until hipcc moved
  // accumulators between AGPRs and VGPRs around the inline-asm MFMAs, whose hazards it cannot
  // see (wrong dV measured).
  auto iteration_np = [&](auto maskc, int it) {
    const int q0 = qs + (it / G) * QT2;
    const u32 boff = (u32)(it & (NBUF - 1)) * BUFB;
    u32 a_ls = sbase + OFF_LD + (u32)(it & (NBUF - 1)) * 256 + 4 * lr;
    asm volatile("" : "+v"(a_ls));
    float lse_v = rd_b32<0>(a_ls), dl_v = rd_b32<128>(a_ls);
    lgkm_tf2<0>(lse_v, dl_v);
    const int key0 = kw0 + lr, key1 = kw0 + 32 + lr;
    f32x16 sa, da;
    u32 pa[8], sa8[8];
    sdp_chain(I0(), boff, lse_v, dl_v, sa, da, [&](auto) {});
    static_for<0, 8>([&](auto ic) { p_pair(maskc, key0, q0, sa, pa, ic); ds_pair(sa, da, sa8, ic); });
    dvdk(I0(), boff, pa, sa8, [&](auto) {});
    sdp_chain(I1(), boff, lse_v, dl_v, sa, da, [&](auto) {});
    static_for<0, 8>([&](auto ic) { p_pair(maskc, key1, q0, sa, pa, ic); ds_pair(sa, da, sa8, ic); });
    dvdk(I1(), boff, pa, sa8, [&](auto) {});
    if (it + 1 < niter) wait_next(it);
    if (it + 3 < niter) stage(it + 3);
  };
  // one pipelined iteration (never causally masked); FIRST: there is no previous iteration.
  u32 pu1[8], su1[8];           // g1 of the previous iteration, packed P / dS
  auto iteration = [&](auto firstc, int it) {
    using maskc = std::false_type;
    constexpr bool FIRST = decltype(firstc)::value;
    const int qt = it / G;
    const int q0 = qs + qt * QT2;
    const u32 boff = (u32)(it & (NBUF - 1)) * BUFB;
    u32 a_ls = sbase + OFF_LD + (u32)(it & (NBUF - 1)) * 256 + 4 * lr;
    asm volatile("" : "+v"(a_ls));
    float lse_v = rd_b32<0>(a_ls), dl_v = rd_b32<128>(a_ls);
    lgkm_tf2<0>(lse_v, dl_v);
    // A: S/dP(g0, it) | softmax(g1, it-1): P, dS
    f32x16 s0, dp0;
    const int key1 = kw0 + 32 + lr, key0 = kw0 + lr;
    const int q0p = q0_prev;
    sdp_chain(I0(), boff, lse_v, dl_v, s0, dp0, [&](auto ic) {
      if constexpr (!FIRST) {
        p_pair(maskc(), key1, q0p, s1, pu1, ic);
        ds_pair(s1, dp1, su1, ic);
      }
    });
    // B: dV/dK(g1, it-1) | P(g0, it)
    u32 pu0[8], su0[8];
    if constexpr (!FIRST) {
      dvdk(I1(), buf_prev, pu1, su1, [&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j % 2 == 0) p_pair(maskc(), key0, q0, s0, pu0, std::integral_constant<int, j / 2>());
      });
    } else {
      static_for<0, 8>([&](auto ic) { p_pair(maskc(), key0, q0, s0, pu0, ic); });
    }
    // C: S/dP(g1, it) | dS(g0, it)
    sdp_chain(I1(), boff, lse_v, dl_v, s1, dp1, [&](auto ic) { ds_pair(s0, dp0, su0, ic); });
    // D: dV/dK(g0, it)
    dvdk(I0(), boff, pu0, su0, [&](auto) {});
    q0_prev = q0;
    buf_prev = boff;
    if (it + 1 < niter) wait_next(it);
    if (it + 3 < niter) stage(it + 3);
  };

  // prologue: stages 0..2 in flight, stage 0 published
  if (niter > 0) stage(0);
  if (niter > 1) stage(1);
  if (niter > 2) stage(2);
  {
    const int ahead = min(niter, 3) - 1;   // stages issued after stage 0
    if (ahead >= 2) { if (w == 0) vm_wait<10>(); else vm_wait<8>(); }
    else if (ahead == 1) { if (w == 0) vm_wait<5>(); else vm_wait<4>(); }
    else vm_wait<0>();
    barrier();
  }
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (niter > 0) {
    int it = 0;
#if KF2_NOPIPE
    for (; it < niter; ++it) {
      if (it < ndiag) iteration_np(T_(), it);
      else iteration_np(F_(), it);
    }
#else
    for (; it < ndiag; ++it) iteration_np(T_(), it);
    if (it < niter) {
      // the pipelined loop starts on an empty previous g1: p = exp2(-inf) = 0 and dS = 0 add
      // nothing (one idle dV/dK half-step per work item instead of a separate FIRST body)
#pragma unroll
      for (int r = 0; r < 16; ++r) { s1[r] = -INFINITY; dp1[r] = 0.f; }
      q0_prev = qs;
      buf_prev = (u32)(it & (NBUF - 1)) * BUFB;
      for (; it < niter; ++it) iteration(F_(), it);
      // epilogue: g1 of the last iteration
      const int key1 = kw0 + 32 + lr;
      static_for<0, 8>([&](auto ic) {
        p_pair(F_(), key1, q0_prev, s1, pu1, ic);
        ds_pair(s1, dp1, su1, ic);
      });
      dvdk(I1(), buf_prev, pu1, su1, [&](auto) {});
    }
#endif
  }
  drain_mfma();
  __syncthreads();

  // ---- partial sums: transpose [d][key] accumulators through LDS, row-contiguous fp32 adds
  float* T = reinterpret_cast<float*>(smem);   // [256 keys][128 d] fp32 = 128 KB
  auto flush = [&](const f32x16 (&acc)[2][4], float mul, float* dst_base) {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
          const int key = KPW * w + 32 * g + lr;
          T[key * 128 + (d ^ ((key & 31) << 2))] = acc[g][t][r] * mul;
        }
    __syncthreads();
    float* dst = dst_base + (rowB + kv0) * (long)(Hkv * D) + (long)hkv * D;
    for (int e = tid; e < BKV2 * 128; e += 256) {
      const int key = e >> 7, d = e & 127;
      atomicAdd(dst + (long)key * Hkv * D + d, T[key * 128 + (d ^ ((key & 31) << 2))]);
    }
    __syncthreads();
  };
  flush(dK, scale, dk_acc);
  flush(dV, 1.f, dv_acc);
}

extern "C" int kf_flash_bwd_dkdv2(const void* qkv, long ld, const void* dout, long lddo, const float* lse,
                                  const float* delta, float* dk_acc, float* dv_acc, int B, int S, int Hq, int Hkv,
                                  float scale, int causal, hipStream_t st) {
  using namespace f2;
  if (S % BKV2 || Hq % Hkv) return 1;
  int items = 0;
  for (int kb = 0; kb < S / BKV2; ++kb) items += n_chunks(kb, S, causal);
  const int grid = B * Hkv * items;
  if (causal)
    flash_bwd_dkdv2_kernel<true><<<grid, 256, 0, st>>>((const bf16_t*)qkv, ld, (const bf16_t*)dout, lddo, lse, delta,
                                                       dk_acc, dv_acc, B, S, Hq, Hkv, scale, items);
  else
    flash_bwd_dkdv2_kernel<false><<<grid, 256, 0, st>>>((const bf16_t*)qkv, ld, (const bf16_t*)dout, lddo, lse,
                                                        delta, dk_acc, dv_acc, B, S, Hq, Hkv, scale, items);
  return 0;
}
