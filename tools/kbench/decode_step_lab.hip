// Small-batch decode step (1-4 sequences) as ONE persistent launch (VERDICT r3
// "Next round" #5).
//
// At batch 1-4 a Llama-3-8B token step is a 16 GB weight stream with a dependency chain on top:
// norm -> QKV -> RoPE / KV append -> attention -> O -> norm -> gate/up + SwiGLU -> down, 32 times,
// then the LM head.  As graph-captured kernels (gemv.hip, decode_attn.hip, ...) every one of the
// ~160 launches pays a grid fill / drain and a ~1.2 us boundary, and the short ones (wo: 33 MB)
// never reach the HBM rate.  Here one workgroup per CU (256 x 512 threads) walks the whole step:
//
//  * Weight stream: each WG owns a fixed slice of every projection (QKV 12 RoPE pairs = 24 rows,
//    O 16 rows, gate/up 56 + 56 rows, down 64 rows x a quarter of K, LM head V/256 rows), and each
//    of its 8 waves owns every 8th of those rows, so a wave's weight bytes for the WHOLE step are
//    a sequence of 1 KB pieces known before any activation exists.  The wave streams them by
//    LDS-DMA (global_load_lds_dwordx4 nt) into a private ring of RS slots and consumes exactly the
//    pieces it loaded: no workgroup barrier or handshake in the stream, one counted vmcnt per
//    piece, one wave reduction per row.  The ring runs across phase and layer seams, so while a WG
//    waits at a grid barrier or computes attention its next RS pieces per wave keep arriving.
//  * Activations stay in the caches: every WG tracks the residual stream of the M rows itself in
//    registers (bf16, as the kernel-per-op path rounds it), stages the normalised GEMV operand in LDS
//    once per phase, and the per-layer hand-offs (q/k/v, attention output, O output, SwiGLU
//    output, down partials) go through small global buffers.  The down projection is split over
//    K in quarters (its operand slice fits LDS at 4 rows); the next phase sums the 4 partials.
//  * Hand-offs (MI355X_MICROARCH.md "Valid forms" row 1): producers store `sc1` (agent atomic
//    stores), every storing wave drains (vmcnt 0), a workgroup barrier, then ONE lane adds to its
//    shard of an 8-way sharded barrier counter; consumers poll every shard with `sc1` loads, join
//    a workgroup barrier and read the bytes with `sc1` loads only.  The attention split merge is
//    done by the last arriver of each (row, kv head) (its ticket add's return value), as in
//    decode_attn.hip's fused kernel.  Every spin is bounded: a timeout sets the error word and
//    every WG leaves after draining its DMA (the engine then falls back and recomputes the step).
//  * Numerics follow the kernel-per-op path: bf16 residual, bf16 normalised operands, fp32 dot
//    products (v_dot2c_f32_bf16), bf16 q/k/v with RoPE on the rounded values, fp32 online
//    softmax, bf16 attention / SwiGLU / projection outputs; only the summation order differs.
//
// Shape: Llama-3-8B (hidden 4096, ffn 14336, 32 q / 8 kv heads of 128, vocab % 256 == 0), TP 1,
// 256 CUs.  Anything else keeps the kernel-per-op path (kf_decode_step returns non-zero).
// LAB COPY of ops/csrc/decode_step.hip with ablation knobs (tools/kbench/make_ds_lab.py); never shipped.
#include "common.h"
#ifndef KF_DS_NOBAR
#define KF_DS_NOBAR 0
#endif
#ifndef KF_DS_NOATT
#define KF_DS_NOATT 0
#endif
#ifndef KF_DS_NODMA
#define KF_DS_NODMA 0
#endif

#include <type_traits>

using namespace kf;

namespace ds {

constexpr int H = 4096, F = 14336, HQ = 32, HKV = 8, HD = 128, G = HQ / HKV;
constexpr int NQKV = (HQ + 2 * HKV) * HD;          // 6144 qkv rows
constexpr int NWG = 256, NT = 512, NW = NT / 64;   // one 8-wave workgroup per CU
constexpr int PIECE = 1024;                        // 512 bf16: one wave-instruction of LDS-DMA
constexpr int PPR = H * 2 / PIECE;                 // 8 pieces per K-4096 row
constexpr int PAIRS = NQKV / 2 / NWG;              // 12 RoPE pairs per WG
constexpr int R_QKV = 2 * PAIRS, R_O = H / NWG, R_G = F / NWG;   // 24, 16, 56 (+56 up) rows per WG
constexpr int DKS = 4, KQ = F / DKS;               // down: K quarters of 3584 columns
constexpr int PPD = KQ * 2 / PIECE;                // 7 pieces per down row segment
constexpr int R_D = H / (NWG / DKS);               // 64 down row segments per WG
constexpr int P_QKV = R_QKV / NW * PPR, P_O = R_O / NW * PPR, P_GU = 2 * R_G / NW * PPR, P_D = R_D / NW * PPD;
constexpr int P_LAYER = P_QKV + P_O + P_GU + P_D;  // 208 pieces per wave per layer (1.66 MB per WG)
constexpr int MAXL = 32, MAXM = 4;
constexpr int MAXROWS_LM = 512;                    // V / 256 rows per WG
constexpr int ATT_BYTES = (G * HD + 2 * HD + NW * G * HD + 2 * NW * G + 2 * 32 * G) * 4;
constexpr int SHARD = 32;                          // ints between counters (128-B lines)
constexpr int N_TICKETS = MAXM * HKV;
constexpr int ERR_INT = (8 + N_TICKETS) * SHARD;   // sticky: the engine drops the path when set
constexpr int EXIT_INT = ERR_INT + SHARD;          // workgroups done with every barrier
constexpr int SYNC_INTS = EXIT_INT + SHARD;
constexpr unsigned SPIN_LIMIT = 1u << 23;
static_assert(H == 4096 && F % (DKS * 512) == 0 && (NQKV / 2) % NWG == 0 && PAIRS % 4 == 0, "geometry");
static_assert(R_QKV % NW == 0 && R_O % NW == 0 && (2 * R_G) % NW == 0 && R_D % NW == 0, "rows per wave");

// per M: ring slots per wave (1 KB each; the LDS left after the operand / attention scratch) and
// PF, pieces per wave each workgroup prefetches towards the caches while it waits at a grid
// barrier (the ring is full then; PF = 0: none)
template <int M> struct Cfg;
#ifndef KF_DS_RS1
#define KF_DS_RS1 16
#endif
#ifndef KF_DS_PF1
#define KF_DS_PF1 0
#endif
template <> struct Cfg<1> { static constexpr int RS = KF_DS_RS1, PF = KF_DS_PF1; };
#ifndef KF_DS_RS2
#define KF_DS_RS2 16
#endif
#ifndef KF_DS_PF2
#define KF_DS_PF2 0
#endif
template <> struct Cfg<2> { static constexpr int RS = KF_DS_RS2, PF = KF_DS_PF2; };
#ifndef KF_DS_RS3
#define KF_DS_RS3 16
#endif
#ifndef KF_DS_PF3
#define KF_DS_PF3 0
#endif
template <> struct Cfg<3> { static constexpr int RS = KF_DS_RS3, PF = KF_DS_PF3; };
#ifndef KF_DS_RS4
#define KF_DS_RS4 14
#endif
#ifndef KF_DS_PF4
#define KF_DS_PF4 0
#endif
template <> struct Cfg<4> { static constexpr int RS = KF_DS_RS4, PF = KF_DS_PF4; };

struct Tab {                 // per layer, device memory (built once by the engine)
  const bf16_t *wqkv, *wo, *wgu, *wd, *n1, *n2;
  bf16_t *kc, *vc;           // [n_slots, HKV, lmax, HD]
};

struct Args {
  const Tab* tab;
  int L, V, lmax, ns;        // ns: key splits per (row, kv head)
  const bf16_t* embed;
  const bf16_t* fnorm;
  const bf16_t* lm;
  const float* cos_t;        // [max_seq, 64]
  const float* sin_t;
  const long* token;         // [M] device (graph-static)
  const int* slot;
  const int* pos;
  float eps, scale_log2;
  float* qkvf;               // [M][NQKV] bf16-exact q / k / v after RoPE
  bf16_t* ob;                // [M][H] attention output
  bf16_t* dab;               // [M][H] O projection
  bf16_t* sb;                // [M][F] SwiGLU output
  float* dpart;              // [DKS][M][H] down partial sums
  float* part;               // [M][HKV][32][G][HD + 2] attention split partials
  int* sync;                 // SYNC_INTS: zero at the first launch, left zero by every clean launch
  bf16_t* logits;            // [M][V]
};

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ float dot2(u32 a, u32 b, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), acc, false);
}
__device__ __forceinline__ float dot8(const u32x4& w, const u32x4& x, float acc) {
  acc = dot2(w.x, x.x, acc);
  acc = dot2(w.y, x.y, acc);
  acc = dot2(w.z, x.z, acc);
  return dot2(w.w, x.w, acc);
}
__device__ __forceinline__ u32 lds_u32(const void* p) {
  return (u32)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// the ring slot read: inline asm + an explicit wait tied to the destination (the compiler never
// sees the DMA that fills the slot)
__device__ __forceinline__ u32x4 ring_read(u32 addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ const char* uniform_ptr(const char* p) {
  const uint64_t v = (uint64_t)p;
  return (const char*)(((uint64_t)__builtin_amdgcn_readfirstlane((u32)(v >> 32)) << 32) |
                       (u32)__builtin_amdgcn_readfirstlane((u32)v));
}
#pragma clang diagnostic ignored "-Winline-asm"
// one 1 KB piece: lane l fetches 16 B at src + 16 l into LDS lds + 16 l (non-temporal: read once)
__device__ __forceinline__ void dma_piece(const char* src, u32 lds, u32 voff) {
  if (KF_DS_NODMA) return;
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2 nt" : : "s"(lds), "v"(voff), "s"(src)
               : "memory", "m0");
}
// hand-off accesses: agent-scope relaxed atomics = global_load / global_store ... sc1
__device__ __forceinline__ void st_f(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ld_f(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_u(bf16_t* p, u32 v) {
  __hip_atomic_store(reinterpret_cast<u32*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32 ld_u(const bf16_t* p) {
  return __hip_atomic_load(reinterpret_cast<const u32*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int I, int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    static_for<I + 1, N>(f);
  }
}

template <int M>
__global__ __launch_bounds__(NT) void decode_step_kernel(Args a) {
  constexpr int RS = Cfg<M>::RS;
  constexpr int XS_BYTES = (M * H * 2 > ATT_BYTES ? M * H * 2 : ATT_BYTES);
  constexpr int PF = Cfg<M>::PF;
  __shared__ __attribute__((aligned(16))) char ring[NW * RS * PIECE + (PF > 0 ? PIECE : 0)];   // + prefetch sink
  __shared__ __attribute__((aligned(16))) char xsb[XS_BYTES];   // operand rows / attention scratch
  __shared__ float outr[MAXROWS_LM][M];                          // row results of the current phase
  __shared__ const char* wtab[MAXL][4];
  __shared__ float bsum[NW][M];
  __shared__ int tok_sh[M], slot_sh[M], pos_sh[M];
  __shared__ int flag_sh;
  __shared__ int dead_sh;
  // the arguments live in LDS and are re-read where used (volatile): kept in SGPRs for the whole
  // kernel they overflow the SGPR file (spills) -- only the stream's own values stay in registers
  __shared__ Args sa;
  volatile Args& A = sa;

  int tid = threadIdx.x;    // re-made opaque every layer (below): no hoisted lane masks
  int lane = tid & 63;
  int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int g = blockIdx.x;
  const int L = a.L, rows_lm = a.V / NWG;
  const int nlm = (rows_lm - wave + NW - 1) / NW;               // this wave's LM head rows
  const int T = L * P_LAYER + nlm * PPR;                        // pieces in this wave's stream
  bf16_t* xs = reinterpret_cast<bf16_t*>(xsb);
  // the residual stream: thread t holds elements 8 t .. 8 t + 7 of every row (bf16), the slice
  // its norm and residual-add work on
  u32x4 rr[M];

  if (tid < 4 * L) {
    const Tab& tb = a.tab[tid >> 2];
    const int k = tid & 3;
    wtab[tid >> 2][k] = (const char*)(k == 0 ? tb.wqkv : k == 1 ? tb.wo : k == 2 ? tb.wgu : tb.wd);
  }
  if (tid < M) {
    tok_sh[tid] = (int)a.token[tid];
    slot_sh[tid] = a.slot[tid];
    pos_sh[tid] = a.pos[tid];
  }
  if (tid == 0) {
    dead_sh = 0;
    sa = a;
  }
  __syncthreads();
  {
    bool bad = false;
#pragma unroll
    for (int m = 0; m < M; ++m)
      bad |= tok_sh[m] < 0 || tok_sh[m] >= a.V || slot_sh[m] < 0 || pos_sh[m] < 0 || pos_sh[m] >= a.lmax;
    if (bad) {                                                   // nothing issued yet
      if (tid == 0) __hip_atomic_store(a.sync + ERR_INT, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }

  // ---- the weight stream: this wave's pieces, in consumption order ---------------------------
  const u32 ring0 = lds_u32(ring) + wave * RS * PIECE;
  const u32 voff = 16 * lane;
  const bf16_t* const lm = a.lm;
  const char* const dummy = uniform_ptr((const char*)(lm + (long)(g * rows_lm + wave) * H));
  // base of the row (or down row segment) that starts at piece t of this wave's stream, and its
  // piece count; past the stream's end a dummy row of L2-resident LM-head bytes
  auto row_base = [&](int t, int& ppr) -> const char* {
    ppr = PPR;
    if (t >= T) return dummy;                                   // keeps the count uniform
    const int lt = L * P_LAYER;
    if (t >= lt) return (const char*)(lm + (long)(g * rows_lm + wave + NW * ((t - lt) >> 3)) * H);
    const int l = t / P_LAYER, u = t - l * P_LAYER;
    if (u < P_QKV) {                                            // RoPE pair (p, p + 64) of a head
      const int i = wave + NW * (u >> 3), pr = g * PAIRS + (i >> 1);
      const long row = (long)(pr >> 6) * HD + (pr & 63) + 64 * (i & 1);
      return uniform_ptr(wtab[l][0]) + row * (H * 2);
    }
    if (u < P_QKV + P_O) {
      const long row = (long)g * R_O + wave + NW * ((u - P_QKV) >> 3);
      return uniform_ptr(wtab[l][1]) + row * (H * 2);
    }
    if (u < P_QKV + P_O + P_GU) {
      const int i = wave + NW * ((u - P_QKV - P_O) >> 3);
      const long row = i < R_G ? (long)g * R_G + i : (long)F + g * R_G + (i - R_G);
      return uniform_ptr(wtab[l][2]) + row * (H * 2);
    }
    ppr = PPD;
    const long row = (long)(g / DKS) * R_D + wave + NW * ((u - P_QKV - P_O - P_GU) / PPD);
    return uniform_ptr(wtab[l][3]) + row * (F * 2) + (long)(g % DKS) * (KQ * 2);
  };
  // issue cursor: the next piece to DMA walks the stream in order, one row lookup per row
  int ip_t = 0, ip_j = 0, ip_ppr = PPR;
  const char* ip_row = dummy;
  auto next_src = [&]() -> const char* {
    if (ip_j == 0) ip_row = uniform_ptr(row_base(ip_t, ip_ppr));
    const char* src = ip_row + ip_j * PIECE;
    ++ip_t;
    ip_j = ip_j + 1 == ip_ppr ? 0 : ip_j + 1;
    return src;
  };
  auto issue = [&](int t) { dma_piece(next_src(), ring0 + (t % RS) * PIECE, voff); };
  // piece t of this wave (landed: RS - 1 younger DMAs may still be in flight); its slot is
  // refilled with piece t + RS right after the read
  auto take = [&](int t) -> u32x4 {
    const char* src = next_src();                               // piece t + RS; SALU work ahead of the waits
    vm_wait<RS - 1>();
    const u32 slot = ring0 + (t % RS) * PIECE;
    const u32x4 w = ring_read(slot + voff);
    dma_piece(src, slot, voff);
    return w;
  };
  // pieces t and t + 1 (RS - 2 younger DMAs may be in flight): both slot reads under one wait
  auto take2 = [&](int t, u32x4& w0, u32x4& w1) {
    const char* s0 = next_src();                                // pieces t + RS, t + RS + 1
    const char* s1 = next_src();
    vm_wait<RS - 2>();
    const u32 l0 = ring0 + (t % RS) * PIECE, l1 = ring0 + ((t + 1) % RS) * PIECE;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(w0), "=&v"(w1) : "v"(l0 + voff), "v"(l1 + voff) : "memory");
    dma_piece(s0, l0, voff);
    dma_piece(s1, l1, voff);
  };
  for (int t = 0; t < RS; ++t) issue(t);

  // ---- grid barrier k (1, 2, ...): 8-way sharded monotonic counter ---------------------------
  auto grid_barrier = [&](int k) -> bool {
#if KF_DS_NOBAR == 2
    __syncthreads();
    return true;
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#if KF_DS_NOBAR == 1
    return true;
#endif
    if (PF > 0 && wave != 0) {
      // the ring is full: pull this wave's next PF pieces past it towards the L2 / MALL while the
      // barrier settles (default cache policy; the bytes land in a shared LDS sink nobody reads).
      // Not wave 0: its barrier poll would queue behind them (vector memory returns in order)
      int t = ip_t, j = ip_j, ppr = ip_ppr;
      const char* row = ip_row;
      for (int i = 0; i < PF; ++i) {
        if (j == 0) row = uniform_ptr(row_base(t, ppr));
        asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" : : "s"(lds_u32(ring) + NW * RS * PIECE),
                     "v"(voff), "s"(uniform_ptr(row + j * PIECE)) : "memory", "m0");
        ++t;
        j = j + 1 == ppr ? 0 : j + 1;
      }
    }
    if (wave == 0) {
      if (lane == 0) __hip_atomic_fetch_add(A.sync + (g & 7) * SHARD, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane < 8) {
        const int target = (NWG / 8) * k;
        unsigned spins = 0;
        while (__hip_atomic_load(A.sync + lane * SHARD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          if (++spins > SPIN_LIMIT) {
            __hip_atomic_store(A.sync + ERR_INT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            dead_sh = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    __syncthreads();
    return dead_sh == 0;
  };

  // ---- normalised operands: xs[m] = bf16(r[m] * rstd[m] * w) over the residual rows ----------
  auto norm_into_xs = [&](const bf16_t* w) {
    float hv[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      unpack8(rr[m], hv[m]);
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += hv[m][e] * hv[m][e];
      ss = wave_sum(ss);
      if (lane == 0) bsum[wave][m] = ss;
    }
    __syncthreads();
    float wf[8];
    unpack8(ld16(w + 8 * tid), wf);
#pragma unroll 2
    for (int m = 0; m < M; ++m) {
      float tot = 0.f;
#pragma unroll
      for (int v = 0; v < NW; ++v) tot += bsum[v][m];
      const float rs = rsqrtf(tot / (float)H + A.eps);
#pragma unroll
      for (int e = 0; e < 8; ++e) hv[m][e] = hv[m][e] * rs * wf[e];
      *reinterpret_cast<u32x4*>(xs + m * H + 8 * tid) = pack8(hv[m]);
    }
    __syncthreads();
  };
  // residual update r[m] = bf16(r[m] + delta[m]); delta = bf16 hand-off rows, or (dpart) the
  // bf16-rounded sum of the down projection's 4 K-quarter partials
  auto residual_add = [&](const bf16_t* delta, const float* dpart) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float hv[8], dv[8];
      unpack8(rr[m], hv);
      if (dpart) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float s = 0.f;
#pragma unroll
          for (int q = 0; q < DKS; ++q) s += ld_f(dpart + ((long)q * M + m) * H + 8 * tid + e);
          dv[e] = bf2f(f2bf(s));
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u32 v = ld_u(delta + (long)m * H + 8 * tid + 2 * i);
          dv[2 * i] = bflo(v);
          dv[2 * i + 1] = bfhi(v);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) hv[e] += dv[e];
      rr[m] = pack8(hv);
    }
    __syncthreads();
  };
  // this wave's rows of a projection: nrows rows of P pieces each; piece j of EVERY row meets
  // the same operand columns xs[m * xld + 512 j + 8 lane] (held in registers for the phase);
  // row k's result -> outr[wave + 8 k][m].  Pieces are taken two at a time.
  auto gemv = [&](int t0, int nrows, auto pc, int xld) {
    constexpr int P = decltype(pc)::value;
    u32x4 xr[P][M];
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int m = 0; m < M; ++m) xr[j][m] = *reinterpret_cast<const u32x4*>(xs + m * xld + 512 * j + 8 * lane);
#pragma unroll 1
    for (int k = 0; k < nrows; ++k) {
      asm volatile("" : "+s"(g));     // the cursor's row lookups: recomputed, not hoisted (SGPRs)
      const int tb = t0 + k * P;
      float acc[M];
#pragma unroll
      for (int m = 0; m < M; ++m) acc[m] = 0.f;
      static_for<0, P / 2>([&](auto ic) {
        constexpr int j = 2 * decltype(ic)::value;
        u32x4 w0, w1;
        take2(tb + j, w0, w1);
#pragma unroll
        for (int m = 0; m < M; ++m) acc[m] = dot8(w1, xr[j + 1][m], dot8(w0, xr[j][m], acc[m]));
      });
      if constexpr (P % 2) {
        const u32x4 w = take(tb + P - 1);
#pragma unroll
        for (int m = 0; m < M; ++m) acc[m] = dot8(w, xr[P - 1][m], acc[m]);
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const float s = wave_sum(acc[m]);
        if (lane == 0) outr[wave + NW * k][m] = s;
      }
    }
    __syncthreads();
  };
  using P8 = std::integral_constant<int, PPR>;
  using P7 = std::integral_constant<int, PPD>;

  int bar = 0;
  for (int l = 0; l < L; ++l) {
    // Loop-invariant values (`tid < n` exec masks, offsets from g) hoisted out of the layer loop
    // would pin ~40 SGPRs for the whole kernel and spill; made opaque once per iteration they are
    // recomputed in the phase that uses them (a few SALU ops per layer)
    asm volatile("" : "+v"(tid), "+v"(lane), "+s"(g), "+s"(wave));
    const Tab& tb = A.tab[l];
    const int t0 = l * P_LAYER;
    // ---- residual + norm1 -> xs; QKV rows ---------------------------------------------------
    if (l == 0) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        rr[m] = ld16(A.embed + (long)tok_sh[m] * H + 8 * tid);
      __syncthreads();
    } else {
      residual_add(nullptr, A.dpart);
    }
    norm_into_xs(tb.n1);
    gemv(t0, R_QKV / NW, P8(), H);
    if (tid < (PAIRS / 4) * M) {
      // 4 consecutive RoPE pairs of row m: rows p..p+3 and p+64..p+67 of one head
      const int m = tid / (PAIRS / 4), q = tid % (PAIRS / 4);
      const int pr0 = g * PAIRS + 4 * q, head = pr0 >> 6, p0 = pr0 & 63;
      const int ps = pos_sh[m];
      float lo[4], hi[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 2 * (4 * q + i);
        float v0 = bf2f(f2bf(outr[r][m])), v1 = bf2f(f2bf(outr[r + 1][m]));
        if (head < HQ + HKV) {                                   // q and k heads rotate
          const float c = A.cos_t[(long)ps * 64 + p0 + i], s = A.sin_t[(long)ps * 64 + p0 + i];
          const float r0 = v0 * c - v1 * s, r1 = v1 * c + v0 * s;
          v0 = bf2f(f2bf(r0));
          v1 = bf2f(f2bf(r1));
        }
        lo[i] = v0;
        hi[i] = v1;
      }
      float* q0 = A.qkvf + (long)m * NQKV + head * HD + p0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st_f(q0 + i, lo[i]);
        st_f(q0 + 64 + i, hi[i]);
      }
      if (head >= HQ) {                                          // K / V cache append (next steps read it)
        const bool is_v = head >= HQ + HKV;
        const int kh = is_v ? head - HQ - HKV : head - HQ;
        bf16_t* c = (is_v ? tb.vc : tb.kc) + (((long)slot_sh[m] * HKV + kh) * A.lmax + ps) * HD + p0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          c[i] = f2bf(lo[i]);
          c[64 + i] = f2bf(hi[i]);
        }
      }
    }
    if (!grid_barrier(++bar)) break;

    // ---- attention: WG (row m, kv head hk, key split j); the last split to finish merges ------
    const int ns = A.ns;
    if (!KF_DS_NOATT && g < M * HKV * ns) {
      const int m = g / (HKV * ns), rem = g % (HKV * ns), hk = rem % HKV, j = rem / HKV;
      const int ps = pos_sh[m];
      float* qs = reinterpret_cast<float*>(xsb);                 // [G][HD] scaled q
      float* kcur = qs + G * HD;                                 // [HD] current key / value
      float* vcur = kcur + HD;
      float* so = vcur + HD;                                     // [NW][G][HD]
      float* sm = so + NW * G * HD;                              // [NW][G]
      float* sl = sm + NW * G;
      const float* qrow = A.qkvf + (long)m * NQKV;
      qs[tid] = ld_f(qrow + hk * G * HD + tid) * A.scale_log2;
      if (tid < HD) kcur[tid] = ld_f(qrow + (HQ + hk) * HD + tid);
      else if (tid < 2 * HD) vcur[tid - HD] = ld_f(qrow + (HQ + HKV + hk) * HD + tid - HD);
      __syncthreads();
      const int len = ps + 1;
      const int chunk = ((len + ns - 1) / ns + 15) & ~15;
      const int start = j * chunk, end = min(len, start + chunk);
      const int sub = lane & 15, grp = tid >> 4;                 // 32 key streams x 16 lanes
      float qf[G][8];
#pragma unroll
      for (int h = 0; h < G; ++h)
#pragma unroll
        for (int i = 0; i < 8; ++i) qf[h][i] = qs[h * HD + sub * 8 + i];
      const long kvbase = ((long)slot_sh[m] * HKV + hk) * A.lmax * HD;
      const bf16_t* kp = tb.kc + kvbase;
      const bf16_t* vp = tb.vc + kvbase;
      float mx[G], lsum[G], acc[G][8];
#pragma unroll
      for (int h = 0; h < G; ++h) {
        mx[h] = -INFINITY;
        lsum[h] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[h][i] = 0.f;
      }
      for (int r0 = start; r0 < end; r0 += 32) {
        const int jk = r0 + grp;
        const bool ok = jk < end;
        float kf[8], vf[8];
        if (ok && jk == ps) {
#pragma unroll
          for (int i = 0; i < 8; ++i) { kf[i] = kcur[sub * 8 + i]; vf[i] = vcur[sub * 8 + i]; }
        } else {
          const u32x4 zero = u32x4{0u, 0u, 0u, 0u};
          unpack8(ok ? ld16(kp + (long)jk * HD + sub * 8) : zero, kf);
          unpack8(ok ? ld16(vp + (long)jk * HD + sub * 8) : zero, vf);
        }
#pragma unroll
        for (int h = 0; h < G; ++h) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) s = fmaf(qf[h][i], kf[i], s);
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
          s = ok ? s : -INFINITY;
          const float mn = fmaxf(mx[h], s);
          if (mn == -INFINITY) continue;
          const float al = exp2f(mx[h] - mn), p = exp2f(s - mn);
          mx[h] = mn;
          lsum[h] = fmaf(lsum[h], al, p);
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[h][i] = fmaf(acc[h][i], al, p * vf[i]);
        }
      }
      // the wave's 4 key streams (lanes l, l^16, l^32, l^48 hold the same columns)
#pragma unroll
      for (int h = 0; h < G; ++h) {
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {
          const float mo = __shfl_xor(mx[h], o, 64), lo_ = __shfl_xor(lsum[h], o, 64);
          const float mn = fmaxf(mx[h], mo);
          const float x0 = mn == -INFINITY ? 0.f : exp2f(mx[h] - mn), x1 = mn == -INFINITY ? 0.f : exp2f(mo - mn);
          lsum[h] = lsum[h] * x0 + lo_ * x1;
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[h][i] = acc[h][i] * x0 + __shfl_xor(acc[h][i], o, 64) * x1;
          mx[h] = mn;
        }
      }
      if (lane < 16) {
#pragma unroll
        for (int h = 0; h < G; ++h) {
#pragma unroll
          for (int i = 0; i < 8; ++i) so[(wave * G + h) * HD + sub * 8 + i] = acc[h][i];
          if (sub == 0) { sm[wave * G + h] = mx[h]; sl[wave * G + h] = lsum[h]; }
        }
      }
      __syncthreads();
      // this split's partial (write-through), then the ticket
      float* const pbase = A.part + ((long)m * HKV + hk) * 32 * G * (HD + 2);
      {
        float* pp = pbase + (long)j * G * (HD + 2);
        const int h = tid / HD, d = tid % HD;                   // 512 threads = G x HD
        float Mx = sm[h];
#pragma unroll
        for (int w = 1; w < NW; ++w) Mx = fmaxf(Mx, sm[w * G + h]);
        float o = 0.f;
        if (Mx != -INFINITY) {
#pragma unroll
          for (int w = 0; w < NW; ++w) o = fmaf(exp2f(sm[w * G + h] - Mx), so[(w * G + h) * HD + d], o);
        }
        st_f(pp + h * (HD + 2) + d, o);
        if (d == 0) {
          float Ls = 0.f;
          if (Mx != -INFINITY) {
#pragma unroll
            for (int w = 0; w < NW; ++w) Ls = fmaf(exp2f(sm[w * G + h] - Mx), sl[w * G + h], Ls);
          }
          st_f(pp + h * (HD + 2) + HD, Mx);
          st_f(pp + h * (HD + 2) + HD + 1, Ls);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(A.sync + (8 + m * HKV + hk) * SHARD, 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        flag_sh = old == ns * (l + 1) - 1;
      }
      __syncthreads();
      if (flag_sh) {
        // merge the ns splits of this (row, kv head): every split's (max, sum) in one parallel
        // load, the weights in LDS, then each of the 512 outputs sums its splits with all of
        // its loads in flight at once (a serial chain of dependent loads here costs ~1 us each)
        float* wt = so;                                          // [32][G]  (so is consumed)
        float* lt = wt + 32 * G;                                 // [32][G]
        float* den = lt + 32 * G;                                // [G]
        if (tid < ns * G) {
          wt[tid] = ld_f(pbase + (long)tid * (HD + 2) + HD);
          lt[tid] = ld_f(pbase + (long)tid * (HD + 2) + HD + 1);
        } else if (tid < 32 * G) {
          wt[tid] = -INFINITY;                                   // splits past ns weigh 0
          lt[tid] = 0.f;
        }
        __syncthreads();
        if (tid < G) {
          float Mx = -INFINITY;
          for (int s = 0; s < 32; ++s) Mx = fmaxf(Mx, wt[s * G + tid]);
          float D = 0.f;
          for (int s = 0; s < 32; ++s) {
            const float ms = wt[s * G + tid];
            const float w = (Mx == -INFINITY || ms == -INFINITY) ? 0.f : exp2f(ms - Mx);
            D = fmaf(w, lt[s * G + tid], D);
            wt[s * G + tid] = w;
          }
          den[tid] = D;
        }
        __syncthreads();
        {
          const int h = tid / HD, d = tid % HD;                 // 512 threads = G x HD outputs
          float v[32];
          const float* pv = pbase + (long)h * (HD + 2) + d;
#pragma unroll
          for (int s = 0; s < 32; ++s) v[s] = ld_f(pv + (long)min(s, ns - 1) * G * (HD + 2));   // weight 0 past ns
          float o = 0.f;
#pragma unroll
          for (int s = 0; s < 32; ++s) o = fmaf(wt[s * G + h], v[s], o);
          o *= den[h] > 0.f ? 1.f / den[h] : 0.f;
          const float o1 = __shfl_xor(o, 1, 64);
          if ((d & 1) == 0) st_u(A.ob + (long)m * H + (hk * G + h) * HD + d, pack2(o, o1));
        }
      }
    }
    if (!grid_barrier(++bar)) break;

    // ---- O projection -----------------------------------------------------------------------
    for (int i = tid; i < M * H / 2; i += NT) reinterpret_cast<u32*>(xs)[i] = ld_u(A.ob + 2 * i);
    __syncthreads();
    gemv(t0 + P_QKV, R_O / NW, P8(), H);
    if (tid < (R_O / 2) * M) {
      const int m = tid / (R_O / 2), k = tid % (R_O / 2);
      st_u(A.dab + (long)m * H + g * R_O + 2 * k, pack2(outr[2 * k][m], outr[2 * k + 1][m]));
    }
    if (!grid_barrier(++bar)) break;

    // ---- residual + norm2 -> xs; gate/up rows + SwiGLU --------------------------------------
    residual_add(A.dab, nullptr);
    norm_into_xs(tb.n2);
    gemv(t0 + P_QKV + P_O, 2 * R_G / NW, P8(), H);
    if (tid < (R_G / 2) * M) {
      const int m = tid / (R_G / 2), k = tid % (R_G / 2);
      float o[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float gt = outr[2 * k + i][m], up = outr[R_G + 2 * k + i][m];
        o[i] = gt * sigmoidf_(gt) * up;
      }
      st_u(A.sb + (long)m * F + g * R_G + 2 * k, pack2(o[0], o[1]));
    }
    if (!grid_barrier(++bar)) break;

    // ---- down projection: 64 rows x this WG's K quarter; fp32 partials per quarter ----------
    {
      const int kq = g % DKS;
      for (int i = tid; i < M * KQ / 2; i += NT) {
        const int m = i / (KQ / 2), c = i % (KQ / 2);
        reinterpret_cast<u32*>(xs)[m * (KQ / 2) + c] = ld_u(A.sb + (long)m * F + kq * KQ + 2 * c);
      }
      __syncthreads();
      gemv(t0 + P_QKV + P_O + P_GU, R_D / NW, P7(), KQ);
      if (tid < (R_D / 4) * M) {
        const int m = tid / (R_D / 4), k = tid % (R_D / 4);
        float* dp = A.dpart + ((long)kq * M + m) * H + (g / DKS) * R_D + 4 * k;
#pragma unroll
        for (int i = 0; i < 4; ++i) st_f(dp + i, outr[4 * k + i][m]);
      }
    }
    if (!grid_barrier(++bar)) break;
  }

  if (dead_sh == 0) {
    // ---- final norm + LM head: this WG's V / 256 rows ------------------------------------
    residual_add(nullptr, A.dpart);
    norm_into_xs(A.fnorm);
    gemv(L * P_LAYER, nlm, P8(), H);
    for (int i = tid; i < rows_lm * M; i += NT) {
      const int m = i / rows_lm, r = i % rows_lm;
      A.logits[(long)m * A.V + (long)g * rows_lm + r] = f2bf(outr[r][m]);
    }
    // re-arm the counters for the next launch (no memset node in the graph): every WG counts
    // itself out after its last barrier poll; the last one zeroes the shards, tickets and itself
    if (tid == 0) {
      int* sy = A.sync;
      if (__hip_atomic_fetch_add(sy + EXIT_INT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NWG - 1) {
        for (int i = 0; i < 8 + N_TICKETS; ++i) __hip_atomic_store(sy + i * SHARD, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sy + EXIT_INT, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  vm_wait<0>();                                                  // no DMA may outlive the LDS
}

template <int M>
constexpr long ws_bytes_m() {
  return (long)M * NQKV * 4 + (long)M * H * 2 * 2 + (long)M * F * 2 + (long)DKS * M * H * 4 +
         (long)M * HKV * 32 * G * (HD + 2) * 4;
}

}  // namespace ds

using namespace ds;

// workspace for up to MAXM rows: hand-off buffers, then the sync words (re-armed in-kernel)
extern "C" __attribute__((weak)) long kf_decode_step_ws_bytes() { return ws_bytes_m<MAXM>() + (long)SYNC_INTS * 4 + 1024; }
extern "C" __attribute__((weak)) long kf_decode_step_err_offset() { return ws_bytes_m<MAXM>() + (long)ERR_INT * 4; }

// Rows 1..4 (M): token int64 [M], slot / pos int32 [M], logits bf16 [M, V].  Returns 0 when
// launched; non-zero (nothing launched) when the model / device is not the shape this kernel is
// built for.  ws: kf_decode_step_ws_bytes() bytes, 16-B aligned, ZEROED before the first launch
// (every clean launch leaves its sync words zero again; a non-zero error word is sticky).
extern "C" __attribute__((weak)) int kf_decode_step(const void* tab, int L, int M, int hidden, int ffn, int hq, int hkv, int hd, int V,
                              const void* embed, const void* fnorm, const void* lm, const float* cos_t,
                              const float* sin_t, const long* token, const int* slot, const int* pos, int lmax,
                              float eps, float scale, void* ws, void* logits, hipStream_t st) {
  if (hidden != H || ffn != F || hq != HQ || hkv != HKV || hd != HD) return 1;
  if (M < 1 || M > MAXM || L < 1 || L > MAXL || V % NWG != 0 || V / NWG > MAXROWS_LM) return 2;
  if (((uintptr_t)ws & 15) || ((uintptr_t)embed & 15) || ((uintptr_t)lm & 15)) return 3;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 4;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus != NWG) return 5;
  char* w = static_cast<char*>(ws);
  Args a{};
  a.tab = static_cast<const Tab*>(tab);
  a.L = L;
  a.V = V;
  a.lmax = lmax;
  a.ns = NWG / (M * HKV) > 32 ? 32 : NWG / (M * HKV);
  a.embed = static_cast<const bf16_t*>(embed);
  a.fnorm = static_cast<const bf16_t*>(fnorm);
  a.lm = static_cast<const bf16_t*>(lm);
  a.cos_t = cos_t;
  a.sin_t = sin_t;
  a.token = token;
  a.slot = slot;
  a.pos = pos;
  a.eps = eps;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.qkvf = reinterpret_cast<float*>(w);
  w += (long)MAXM * NQKV * 4;
  a.ob = reinterpret_cast<bf16_t*>(w);
  w += (long)MAXM * H * 2;
  a.dab = reinterpret_cast<bf16_t*>(w);
  w += (long)MAXM * H * 2;
  a.sb = reinterpret_cast<bf16_t*>(w);
  w += (long)MAXM * F * 2;
  a.dpart = reinterpret_cast<float*>(w);
  w += (long)DKS * MAXM * H * 4;
  a.part = reinterpret_cast<float*>(w);
  w += (long)MAXM * HKV * 32 * G * (HD + 2) * 4;
  a.sync = reinterpret_cast<int*>(w);
  a.logits = static_cast<bf16_t*>(logits);
  switch (M) {
    case 1: hipLaunchKernelGGL(decode_step_kernel<1>, dim3(NWG), dim3(NT), 0, st, a); break;
    case 2: hipLaunchKernelGGL(decode_step_kernel<2>, dim3(NWG), dim3(NT), 0, st, a); break;
    case 3: hipLaunchKernelGGL(decode_step_kernel<3>, dim3(NWG), dim3(NT), 0, st, a); break;
    default: hipLaunchKernelGGL(decode_step_kernel<4>, dim3(NWG), dim3(NT), 0, st, a); break;
  }
  KF_CHECK_LAUNCH();
  return 0;
}
