// Batch-1 decode step as ONE persistent launch (VERDICT r3 "Next round" #5).
//
// At batch 1 a Llama-3-8B token is a 16 GB weight stream with a dependency chain on top:
// norm -> QKV -> RoPE / KV append -> attention -> O -> norm -> gate/up + SwiGLU -> down, 32 times,
// then the LM head.  As graph-captured kernels (gemv.hip, decode_attn.hip, ...) every one of the
// ~160 launches pays a grid fill / drain and a ~1.2 us boundary, and the short ones (wo: 33 MB)
// never reach the HBM rate.  Here one workgroup per CU (256 x 512 threads) walks the whole step:
//
//  * Weight stream: each WG owns a fixed slice of every projection (QKV 12 RoPE pairs = 24 rows,
//    O 16 rows, gate/up 56 + 56 rows, down 16 rows, LM head V/256 rows), so its weight bytes for
//    the WHOLE step are a sequence of 8 KB stages known before any activation exists.  Each of
//    the 8 waves streams its own 1 KB piece of every stage by LDS-DMA (global_load_lds_dwordx4
//    nt) into a private ring slot, RS stages ahead, and consumes exactly the piece it loaded: no
//    workgroup barrier or handshake in the stream, one counted vmcnt per stage.  The ring runs
//    across phase and layer seams, so while a WG waits at a grid barrier or computes attention
//    its next RS stages keep arriving (the "prefetch credit" of a run-ahead loader).
//  * Activations never leave the chip's caches: the residual stream is tracked by EVERY WG
//    redundantly in LDS (bf16, as the kernel-per-op path rounds it), the normalised GEMV operand
//    is staged in LDS once per phase, and the five per-layer hand-offs (q/k/v, attention output,
//    O output, SwiGLU output, down output) go through small global buffers.
//  * Hand-offs (MI355X_MICROARCH.md "Valid forms" row 1): producers store `sc1` (agent atomic
//    stores), every storing wave drains (vmcnt 0), a workgroup barrier, then ONE lane adds to its
//    shard of an 8-way sharded barrier counter; consumers poll every shard with `sc1` loads, join
//    a workgroup barrier and read the bytes with `sc1` loads only.  The attention split merge is
//    done by the last arriver of each kv head (its ticket add's return value), as in
//    decode_attn.hip's fused kernel.  Every spin is bounded: a timeout sets the error word and
//    every WG leaves after draining its DMA (the engine raises and falls back).
//  * Numerics follow the kernel-per-op path: bf16 residual, bf16 normalised operands, fp32 dot
//    products (v_dot2c_f32_bf16), bf16 q/k/v with RoPE on the rounded values, fp32 online
//    softmax, bf16 attention / SwiGLU / projection outputs; only the summation order differs.
//
// Shape: Llama-3-8B (hidden 4096, ffn 14336, 32 q / 8 kv heads of 128, vocab % 256 == 0), batch 1,
// TP 1, 256 CUs.  Anything else keeps the kernel-per-op path (kf_decode_step returns non-zero).
#include "common.h"

using namespace kf;

namespace ds {

constexpr int H = 4096, F = 14336, HQ = 32, HKV = 8, HD = 128, G = HQ / HKV;
constexpr int NQKV = (HQ + 2 * HKV) * HD;          // 6144 qkv rows
constexpr int NWG = 256, NT = 512, NW = NT / 64;   // one 8-wave workgroup per CU
constexpr int PIECE = 1024, STAGE = NW * PIECE;    // a stage = 4096 bf16 = one K-4096 row
constexpr int RS = 14;                             // ring stages (112 KB of LDS)
constexpr int PAIRS = NQKV / 2 / NWG;              // 12 RoPE pairs per WG
constexpr int S_QKV = 2 * PAIRS;                   // 24
constexpr int ROWS_O = H / NWG;                    // 16 (also the down rows)
constexpr int ROWS_G = F / NWG;                    // 56 gate (+ 56 up) rows
constexpr int S_O = ROWS_O, S_GU = 2 * ROWS_G, S_D = ROWS_O * F / 4096;
constexpr int S_LAYER = S_QKV + S_O + S_GU + S_D;  // 208 stages = 1.66 MB per WG per layer
constexpr int NS = NWG / HKV;                      // 32 key splits per kv head
constexpr int MAXL = 32;
constexpr int XS_BYTES = 2 * F;                    // staged operand (down: 14336 bf16)
constexpr int SHARD = 32;                          // ints between counters (128-B lines)
constexpr int SYNC_INTS = 8 * SHARD + HKV * SHARD + SHARD;
constexpr unsigned SPIN_LIMIT = 1u << 23;
static_assert(H == 4096 && F % 512 == 0 && (NQKV / 2) % NWG == 0 && PAIRS % 4 == 0, "stage geometry");
static_assert((ROWS_O * F) % 4096 == 0 && ROWS_G % 2 == 0 && ROWS_O % 2 == 0, "row slices");

struct Tab {                 // per layer, device memory (built once by the engine)
  const bf16_t *wqkv, *wo, *wgu, *wd, *n1, *n2;
  bf16_t *kc, *vc;           // [n_slots, HKV, lmax, HD]
};

struct Args {
  const Tab* tab;
  int L, V, lmax;
  const bf16_t* embed;
  const bf16_t* fnorm;
  const bf16_t* lm;
  const float* cos_t;        // [max_seq, 64]
  const float* sin_t;
  const long* token;         // device scalars (graph-static)
  const int* slot;
  const int* pos;
  float eps, scale_log2;
  float* qkvf;               // [NQKV] bf16-exact q / k / v after RoPE
  bf16_t* ob;                // [H] attention output
  bf16_t* dab;               // [H] O projection
  bf16_t* sb;                // [F] SwiGLU output
  bf16_t* db;                // [H] down projection
  float* part;               // [HKV][NS][G][HD + 2]
  int* sync;                 // SYNC_INTS, zero at launch
  bf16_t* logits;            // [V]
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

__global__ __launch_bounds__(NT) void decode_step_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) char ring[RS * STAGE];
  __shared__ __attribute__((aligned(16))) char xsb[XS_BYTES];
  __shared__ __attribute__((aligned(16))) bf16_t rres[H];     // residual stream (bf16)
  __shared__ float red[S_GU][NW];                              // per-row wave partials
  __shared__ const char* wtab[MAXL][4];
  __shared__ float bsum[NW];
  __shared__ int flag_sh;
  __shared__ int dead_sh;
  // the arguments live in LDS and are re-read where used (volatile): kept in SGPRs for the whole
  // kernel they overflow the SGPR file (spills) -- only the stream's own values stay in registers
  __shared__ Args sa;
  volatile Args& A = sa;

  int tid = threadIdx.x;    // re-made opaque every layer (below): no hoisted lane masks
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int g = blockIdx.x;
  const int L = a.L, rows_lm = a.V / NWG;
  const int T = L * S_LAYER + rows_lm;                         // stages in this WG's stream
  bf16_t* xs = reinterpret_cast<bf16_t*>(xsb);

  if (tid < 4 * L) {
    const Tab& tb = a.tab[tid >> 2];
    const int k = tid & 3;
    wtab[tid >> 2][k] = (const char*)(k == 0 ? tb.wqkv : k == 1 ? tb.wo : k == 2 ? tb.wgu : tb.wd);
  }
  if (tid == 0) {
    dead_sh = 0;
    sa = a;
  }
  int token = (int)a.token[0], slot = a.slot[0], pos = a.pos[0];
  __syncthreads();
  if (token < 0 || token >= a.V || slot < 0 || pos < 0 || pos >= a.lmax) {   // nothing issued yet
    if (tid == 0) __hip_atomic_store(a.sync + (8 + HKV) * SHARD, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }

  // ---- the weight stream -------------------------------------------------------------------
  const u32 ring0 = lds_u32(ring) + wave * PIECE;
  const u32 voff = 16 * lane;
  const bf16_t* const lm = a.lm;
  const char* const dummy = uniform_ptr((const char*)(lm + (long)g * rows_lm * H) + wave * PIECE);
  auto piece = [&](int t) -> const char* {
    if (t >= T) return dummy;                                   // keeps the count uniform
    const int lt = L * S_LAYER;
    if (t >= lt) return (const char*)(lm + (long)(g * rows_lm + (t - lt)) * H) + wave * PIECE;
    const int l = t / S_LAYER, u = t - l * S_LAYER;
    long row;
    int k;
    if (u < S_QKV) {                                            // RoPE pair (p, p + 64) of a head
      const int pr = g * PAIRS + (u >> 1);
      row = (long)(pr >> 6) * HD + (pr & 63) + 64 * (u & 1);
      k = 0;
    } else if (u < S_QKV + S_O) {
      row = (long)g * ROWS_O + (u - S_QKV);
      k = 1;
    } else if (u < S_QKV + S_O + S_GU) {
      const int v = u - S_QKV - S_O;
      row = v < ROWS_G ? (long)g * ROWS_G + v : (long)F + g * ROWS_G + (v - ROWS_G);
      k = 2;
    } else {                                                    // down: the WG's 16 rows are contiguous
      const int v = u - S_QKV - S_O - S_GU;
      return uniform_ptr(wtab[l][3]) + (long)g * ROWS_O * F * 2 + (long)v * STAGE + wave * PIECE;
    }
    return uniform_ptr(wtab[l][k]) + row * (H * 2) + wave * PIECE;
  };
  auto issue = [&](int t) { dma_piece(uniform_ptr(piece(t)), ring0 + (t % RS) * STAGE, voff); };
  // stage t's piece of this wave (landed: RS - 1 younger DMAs may still be in flight); its slot
  // is refilled with stage t + RS right after the read
  auto take = [&](int t) -> u32x4 {
    vm_wait<RS - 1>();
    const u32x4 w = ring_read(ring0 + (t % RS) * STAGE + voff);
    issue(t + RS);
    return w;
  };
  for (int t = 0; t < RS; ++t) issue(t);

  // ---- grid barrier k (1, 2, ...): 8-way sharded monotonic counter ---------------------------
  auto grid_barrier = [&](int k) -> bool {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // every wave drains its stores
    __syncthreads();
    if (wave == 0) {
      if (lane == 0) __hip_atomic_fetch_add(A.sync + (g & 7) * SHARD, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane < 8) {
        const int target = (NWG / 8) * k;
        unsigned spins = 0;
        while (__hip_atomic_load(A.sync + lane * SHARD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          if (++spins > SPIN_LIMIT) {
            __hip_atomic_store(A.sync + (8 + HKV) * SHARD, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

  // ---- normalised operand: xs = bf16(r * rstd * w) over the residual in rres ----------------
  auto norm_into_xs = [&](const bf16_t* w) {
    float ss = 0.f;
    {
      float hv[8];
      unpack8(*reinterpret_cast<const u32x4*>(rres + 8 * tid), hv);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += hv[e] * hv[e];
    }
    ss = wave_sum(ss);
    if (lane == 0) bsum[wave] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) tot += bsum[v];
    const float rs = rsqrtf(tot / (float)H + A.eps);
    float hv[8], wf[8];
    unpack8(*reinterpret_cast<const u32x4*>(rres + 8 * tid), hv);
    unpack8(ld16(w + 8 * tid), wf);
#pragma unroll
    for (int e = 0; e < 8; ++e) hv[e] = hv[e] * rs * wf[e];
    *reinterpret_cast<u32x4*>(xs + 8 * tid) = pack8(hv);
    __syncthreads();
  };
  // residual update: rres = bf16(rres + delta), delta a hand-off buffer (bf16)
  auto residual_add = [&](const bf16_t* delta) {
    float hv[8], dv[8];
    unpack8(*reinterpret_cast<const u32x4*>(rres + 8 * tid), hv);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32 v = ld_u(delta + 8 * tid + 2 * i);
      dv[2 * i] = bflo(v);
      dv[2 * i + 1] = bfhi(v);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) hv[e] += dv[e];
    *reinterpret_cast<u32x4*>(rres + 8 * tid) = pack8(hv);
    __syncthreads();
  };
  // K = 4096 projection: one stage per row, the wave's 512 columns of x fixed for the phase
  auto gemv_rows = [&](int t0, int nst, float* redp) {
    const u32x4 xv = *reinterpret_cast<const u32x4*>(xs + 512 * wave + 8 * lane);
    for (int u = 0; u < nst; ++u) {
      const u32x4 w = take(t0 + u);
      const float p = wave_sum(dot8(w, xv, 0.f));
      if (lane == 0) redp[u * NW + wave] = p;
    }
    __syncthreads();
  };
  auto row_total = [&](const float* redp, int r) {
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) s += redp[r * NW + v];
    return s;
  };

  int bar = 0;
  for (int l = 0; l < L; ++l) {
    // Loop-invariant values (`tid < n` exec masks, offsets from g / pos / slot) hoisted out of
    // the layer loop would pin ~40 SGPRs for the whole kernel and spill; made opaque once per
    // iteration they are recomputed in the phase that uses them (a few SALU ops per layer)
    asm volatile("" : "+v"(tid), "+s"(g), "+s"(pos), "+s"(slot));
    const Tab& tb = A.tab[l];
    const int t0 = l * S_LAYER;
    // ---- residual + norm1 -> xs; QKV rows ---------------------------------------------------
    if (l == 0) {
      *reinterpret_cast<u32x4*>(rres + 8 * tid) = ld16(A.embed + (long)token * H + 8 * tid);
      __syncthreads();
    } else {
      residual_add(A.db);
    }
    norm_into_xs(tb.n1);
    gemv_rows(t0, S_QKV, &red[0][0]);
    if (tid < PAIRS / 4) {
      // 4 consecutive RoPE pairs: rows p..p+3 and p+64..p+67 of one head
      const int pr0 = g * PAIRS + 4 * tid, head = pr0 >> 6, p0 = pr0 & 63;
      float lo[4], hi[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = 2 * (4 * tid + i);
        float v0 = bf2f(f2bf(row_total(&red[0][0], u))), v1 = bf2f(f2bf(row_total(&red[0][0], u + 1)));
        if (head < HQ + HKV) {                                   // q and k heads rotate
          const float c = A.cos_t[(long)pos * 64 + p0 + i], s = A.sin_t[(long)pos * 64 + p0 + i];
          const float r0 = v0 * c - v1 * s, r1 = v1 * c + v0 * s;
          v0 = bf2f(f2bf(r0));
          v1 = bf2f(f2bf(r1));
        }
        lo[i] = v0;
        hi[i] = v1;
      }
      float* q0 = A.qkvf + head * HD + p0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st_f(q0 + i, lo[i]);
        st_f(q0 + 64 + i, hi[i]);
      }
      if (head >= HQ) {                                          // K / V cache append (next steps read it)
        const bool is_v = head >= HQ + HKV;
        const int kh = is_v ? head - HQ - HKV : head - HQ;
        bf16_t* c = (is_v ? tb.vc : tb.kc) + (((long)slot * HKV + kh) * A.lmax + pos) * HD + p0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          c[i] = f2bf(lo[i]);
          c[64 + i] = f2bf(hi[i]);
        }
      }
    }
    if (!grid_barrier(++bar)) break;

    // ---- attention: WG (kv head hk, key split j); the last split to finish merges ---------
    {
      const int hk = g & (HKV - 1), j = g / HKV;
      float* qs = reinterpret_cast<float*>(xsb);                 // [G][HD] scaled q
      float* kcur = qs + G * HD;                                 // [HD] current key / value
      float* vcur = kcur + HD;
      float* so = vcur + HD;                                     // [NW][G][HD]
      float* sm = so + NW * G * HD;                              // [NW][G]
      float* sl = sm + NW * G;
      qs[tid] = ld_f(A.qkvf + hk * G * HD + tid) * A.scale_log2;
      if (tid < HD) kcur[tid] = ld_f(A.qkvf + (HQ + hk) * HD + tid);
      else if (tid < 2 * HD) vcur[tid - HD] = ld_f(A.qkvf + (HQ + HKV + hk) * HD + tid - HD);
      __syncthreads();
      const int len = pos + 1;
      const int chunk = ((len + NS - 1) / NS + 15) & ~15;
      const int start = j * chunk, end = min(len, start + chunk);
      const int sub = lane & 15, grp = tid >> 4;                 // 32 key streams x 16 lanes
      float qf[G][8];
#pragma unroll
      for (int h = 0; h < G; ++h)
#pragma unroll
        for (int i = 0; i < 8; ++i) qf[h][i] = qs[h * HD + sub * 8 + i];
      const long kvbase = ((long)slot * HKV + hk) * A.lmax * HD;
      const bf16_t* kp = tb.kc + kvbase;
      const bf16_t* vp = tb.vc + kvbase;
      float m[G], lsum[G], acc[G][8];
#pragma unroll
      for (int h = 0; h < G; ++h) {
        m[h] = -INFINITY;
        lsum[h] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[h][i] = 0.f;
      }
      for (int r0 = start; r0 < end; r0 += 32) {
        const int jk = r0 + grp;
        const bool ok = jk < end;
        float kf[8], vf[8];
        if (ok && jk == pos) {
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
          const float mn = fmaxf(m[h], s);
          if (mn == -INFINITY) continue;
          const float al = exp2f(m[h] - mn), p = exp2f(s - mn);
          m[h] = mn;
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
          const float mo = __shfl_xor(m[h], o, 64), lo_ = __shfl_xor(lsum[h], o, 64);
          const float mn = fmaxf(m[h], mo);
          const float x0 = mn == -INFINITY ? 0.f : exp2f(m[h] - mn), x1 = mn == -INFINITY ? 0.f : exp2f(mo - mn);
          lsum[h] = lsum[h] * x0 + lo_ * x1;
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[h][i] = acc[h][i] * x0 + __shfl_xor(acc[h][i], o, 64) * x1;
          m[h] = mn;
        }
      }
      if (lane < 16) {
#pragma unroll
        for (int h = 0; h < G; ++h) {
#pragma unroll
          for (int i = 0; i < 8; ++i) so[(wave * G + h) * HD + sub * 8 + i] = acc[h][i];
          if (sub == 0) { sm[wave * G + h] = m[h]; sl[wave * G + h] = lsum[h]; }
        }
      }
      __syncthreads();
      // this split's partial (write-through), then the ticket
      float* pp = A.part + ((long)hk * NS + j) * G * (HD + 2);
      {
        const int h = tid / HD, d = tid % HD;                   // 512 threads = G x HD
        float M = sm[h];
#pragma unroll
        for (int w = 1; w < NW; ++w) M = fmaxf(M, sm[w * G + h]);
        float o = 0.f;
        if (M != -INFINITY) {
#pragma unroll
          for (int w = 0; w < NW; ++w) o = fmaf(exp2f(sm[w * G + h] - M), so[(w * G + h) * HD + d], o);
        }
        st_f(pp + h * (HD + 2) + d, o);
        if (d == 0) {
          float Ls = 0.f;
          if (M != -INFINITY) {
#pragma unroll
            for (int w = 0; w < NW; ++w) Ls = fmaf(exp2f(sm[w * G + h] - M), sl[w * G + h], Ls);
          }
          st_f(pp + h * (HD + 2) + HD, M);
          st_f(pp + h * (HD + 2) + HD + 1, Ls);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(A.sync + (8 + hk) * SHARD, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag_sh = old == NS * (l + 1) - 1;
      }
      __syncthreads();
      if (flag_sh) {
        // merge the NS splits of this kv head: weights per (split, head), then every output
        float* wt = sm;                                          // [NS][G] (reuses the scratch)
        float* den = wt + NS * G;
        const float* pk = A.part + (long)hk * NS * G * (HD + 2);
        if (tid < NS * G) wt[tid] = ld_f(pk + (long)tid * (HD + 2) + HD);
        __syncthreads();
        if (tid < G) {
          float M = -INFINITY;
#pragma unroll 1
          for (int s = 0; s < NS; ++s) M = fmaxf(M, wt[s * G + tid]);
          float D = 0.f;
#pragma unroll 1
          for (int s = 0; s < NS; ++s) {
            const float ms = wt[s * G + tid];
            const float w = (M == -INFINITY || ms == -INFINITY) ? 0.f : exp2f(ms - M);
            D = fmaf(w, ld_f(pk + (long)(s * G + tid) * (HD + 2) + HD + 1), D);
            wt[s * G + tid] = w;
          }
          den[tid] = D;
        }
        __syncthreads();
        if (tid < G * HD / 2) {
          const int h = (2 * tid) / HD, d = (2 * tid) % HD;
          float o0 = 0.f, o1 = 0.f;
#pragma unroll 4
          for (int s = 0; s < NS; ++s) {
            const float w = wt[s * G + h];
            const float* ps = pk + (long)(s * G + h) * (HD + 2) + d;
            o0 = fmaf(w, ld_f(ps), o0);
            o1 = fmaf(w, ld_f(ps + 1), o1);
          }
          const float inv = den[h] > 0.f ? 1.f / den[h] : 0.f;
          st_u(A.ob + (hk * G + h) * HD + d, pack2(o0 * inv, o1 * inv));
        }
      }
    }
    if (!grid_barrier(++bar)) break;

    // ---- O projection -----------------------------------------------------------------------
    for (int i = tid; i < H / 2; i += NT) reinterpret_cast<u32*>(xs)[i] = ld_u(A.ob + 2 * i);
    __syncthreads();
    gemv_rows(t0 + S_QKV, S_O, &red[0][0]);
    if (tid < ROWS_O / 2)
      st_u(A.dab + g * ROWS_O + 2 * tid, pack2(row_total(&red[0][0], 2 * tid), row_total(&red[0][0], 2 * tid + 1)));
    if (!grid_barrier(++bar)) break;

    // ---- residual + norm2 -> xs; gate/up rows + SwiGLU --------------------------------------
    residual_add(A.dab);
    norm_into_xs(tb.n2);
    gemv_rows(t0 + S_QKV + S_O, S_GU, &red[0][0]);
    if (tid < ROWS_G / 2) {
      float o[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float gt = row_total(&red[0][0], 2 * tid + i), up = row_total(&red[0][0], ROWS_G + 2 * tid + i);
        o[i] = gt * sigmoidf_(gt) * up;
      }
      st_u(A.sb + g * ROWS_G + 2 * tid, pack2(o[0], o[1]));
    }
    if (!grid_barrier(++bar)) break;

    // ---- down projection: 16 contiguous rows of K = F, 3.5 stages per row ----------------
    for (int i = tid; i < F / 2; i += NT) reinterpret_cast<u32*>(xs)[i] = ld_u(A.sb + 2 * i);
    __syncthreads();
    {
      int cur = -1;
      float acc = 0.f;
      for (int u = 0; u < S_D; ++u) {
        const int e0 = u * 4096 + 512 * wave;                    // wave-uniform: a piece never
        const int row = e0 / F, col = e0 - row * F + 8 * lane;  // straddles rows (F % 512 == 0)
        const u32x4 w = take(t0 + S_QKV + S_O + S_GU + u);
        const u32x4 xv = *reinterpret_cast<const u32x4*>(xs + col);
        if (row != cur) {
          if (cur >= 0) {
            const float p = wave_sum(acc);
            if (lane == 0) red[cur][wave] = p;
          }
          cur = row;
          acc = 0.f;
        }
        acc = dot8(w, xv, acc);
      }
      const float p = wave_sum(acc);
      if (lane == 0) red[cur][wave] = p;
      __syncthreads();
    }
    if (tid < ROWS_O / 2)
      st_u(A.db + g * ROWS_O + 2 * tid, pack2(row_total(&red[0][0], 2 * tid), row_total(&red[0][0], 2 * tid + 1)));
    if (!grid_barrier(++bar)) break;
  }

  if (dead_sh == 0) {
    // ---- final norm + LM head: this WG's V / 256 rows ------------------------------------
    residual_add(A.db);
    norm_into_xs(A.fnorm);
    float* redl = reinterpret_cast<float*>(xsb + 2 * H);        // [rows_lm][NW] after x
    gemv_rows(L * S_LAYER, rows_lm, redl);
    for (int r = tid; r < rows_lm; r += NT) A.logits[(long)g * rows_lm + r] = f2bf(row_total(redl, r));
  }
  vm_wait<0>();                                                  // no DMA may outlive the LDS
}

}  // namespace ds

using namespace ds;

extern "C" long kf_decode_step_ws_bytes() {
  return (long)NQKV * 4 + 2L * H * 2 + (long)F * 2 + (long)H * 2 + (long)HKV * NS * G * (HD + 2) * 4 +
         (long)SYNC_INTS * 4 + 1024;
}

// Returns 0 when launched; non-zero (nothing launched) when the model / device is not the shape
// this kernel is built for.  ws: kf_decode_step_ws_bytes() bytes, 16-B aligned; its sync words
// are zeroed here (a memset node when captured).  err word: kf_decode_step_err_offset().
extern "C" long kf_decode_step_err_offset() {
  const long off = kf_decode_step_ws_bytes() - 1024 - (long)SYNC_INTS * 4;
  return off + (long)(8 + HKV) * SHARD * 4;
}

extern "C" int kf_decode_step(const void* tab, int L, int hidden, int ffn, int hq, int hkv, int hd, int V,
                              const void* embed, const void* fnorm, const void* lm, const float* cos_t,
                              const float* sin_t, const long* token, const int* slot, const int* pos, int lmax,
                              float eps, float scale, void* ws, void* logits, hipStream_t st) {
  if (hidden != H || ffn != F || hq != HQ || hkv != HKV || hd != HD) return 1;
  if (L < 1 || L > MAXL || V % NWG != 0 || V / NWG > (XS_BYTES - 2 * H) / (NW * 4)) return 2;
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
  w += (long)NQKV * 4;
  a.ob = reinterpret_cast<bf16_t*>(w);
  w += (long)H * 2;
  a.dab = reinterpret_cast<bf16_t*>(w);
  w += (long)H * 2;
  a.sb = reinterpret_cast<bf16_t*>(w);
  w += (long)F * 2;
  a.db = reinterpret_cast<bf16_t*>(w);
  w += (long)H * 2;
  a.part = reinterpret_cast<float*>(w);
  w += (long)HKV * NS * G * (HD + 2) * 4;
  a.sync = reinterpret_cast<int*>(w);
  a.logits = static_cast<bf16_t*>(logits);
  if (hipMemsetAsync(a.sync, 0, (size_t)SYNC_INTS * 4, st) != hipSuccess) return 6;
  hipLaunchKernelGGL(decode_step_kernel, dim3(NWG), dim3(NT), 0, st, a);
  KF_CHECK_LAUNCH();
  return 0;
}
