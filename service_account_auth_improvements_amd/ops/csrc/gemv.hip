// Decode GEMV for 1 <= M <= 4 rows: Y[M, N] = X[M, K] . W[N, K]^T (bf16 in/out, fp32 sum).
//
// At batch 1-4 the decode step is a pure weight stream (2-8 flops per weight byte), so the
// kernel is laid out for HBM, not for the matrix cores: one wave owns R whole rows of W and
// its 64 lanes read 64 consecutive 16-byte chunks of a row per instruction (1 KB contiguous
// per row and instruction, full 128-byte lines), U chunks per row in flight per lane.  The
// MFMA skinny kernel (skinny_gemm.hip) has to give each lane (row l%16, k-chunk l/16) and so
// touches 16 rows x 64 B per instruction; it stays the path for 5 <= M <= 64.
//
//  * VALU dot products on the packed bf16 pairs (v_dot2c_f32_bf16, fp32 accumulate): no
//    unpacking of W or X (vs unpack + fp32 FMAs: equal at M = 1, 10-20 % faster at M = 4).
//    R x M partial sums per lane, one wave reduction per (row, x-row) at the end.  X chunks
//    are shared by the R rows of the wave (read once per chunk from L1/L2, or from LDS when
//    the norm prologue staged them).  At M = 8 the MFMA skinny kernel wins again (gate/up
//    52 vs 56 us, wd 30 vs 38 us: X re-reads and VALU work grow with M), hence M <= 4.
//  * Chunks in flight GV_U and rows per wave GV_R: a round-4 sweep of R in {1, 2, 4, 8} x
//    U in {2, 4, 8} (tools/kbench/gemv_bench.hip, then -D knobs) kept R = 4, U = 4.
//  * SWIGLU: the wave's R gate rows n.. and the matching up rows n + up_off.. are streamed
//    together and the wave writes silu(gate) * up.
//  * NORM prologue (decode layer norms fused in, as in skinny_gemm.hip): each workgroup
//    forms h = bf16(x + res) and its sum of squares, stages y = bf16(h * rstd * w_norm) in
//    LDS; workgroup 0 stores h.
//  * Load order: every operand that does not depend on the product (RoPE position / slot, the
//    prologue's x, residual and gain chunks) is requested BEFORE the weights, the RoPE cos/sin
//    right after them, and no load sits under a branch (out-of-range rows / chunks are clamped
//    and never stored).  vmcnt retires in order, so each wait then covers only what it needs
//    while the weights stream: batch 4 decode 4.25 -> 3.68 ms, batch 1 3.05 -> 2.94 ms
//    (profiles/serve_gemv_upfront_loads_r4.txt).
//  * K split inside the workgroup (KS = 4) for narrow, deep projections (wd: N = 4096,
//    K = 14336): with one wave per R rows it launches 256 workgroups, one wave per SIMD, and
//    each wave walks its K/512 chunk slots in a serial chain of 7 load -> wait -> dot rounds.
//    With KS = 4 the four waves of a workgroup share its R rows and take a quarter of K each
//    (4x the waves, a quarter of the chain); the partial sums meet in LDS.  Measured
//    (tools/kbench/gemv_bench, profiles/serve_gemv_ksplit.txt): wd 24.1 -> 19.5 us at M = 1
//    (6.0 TB/s), 29.2 -> 24.9 us at M = 4; at K = 4096 it is null at M = 1 and 10-15 % slower
//    at M = 4, and with the norm prologue (every workgroup normalises X itself) 1.3-1.6x
//    slower.  Hence: no prologue, K >= 8192 (or M <= 2) and < 4 workgroups per CU unsplit.
//    KFAMD_GEMV_KSPLIT=1 / 4 forces it off / on.
#include "common.h"
#include <cstdlib>

using namespace kf;

namespace {

constexpr int GV_WAVES = 4;       // 256-thread workgroups
constexpr int GV_U = 4;           // chunks per row in flight per lane
constexpr int GV_R = 4;           // rows per wave
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
// acc + a.lo * b.lo + a.hi * b.hi for packed bf16 pairs (v_dot2c_f32_bf16)
__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), acc, false);
}

struct GvNorm {
  const bf16_t* res;   // nullable
  const bf16_t* w;
  bf16_t* h_out;
  long ldh;
  float eps;
};

// ROPE epilogue (decode qkv projection): RoPE at pos[m] on the q/k heads and the rotated k
// plus v written into the KV cache at (slot[m], pos[m]) -- rope_append_kernel folded in.
struct GvRope {
  const float* cos_t;   // [max_seq, 64]
  const float* sin_t;
  const int* slots;
  const int* pos;
  bf16_t* kc;           // [n_slots, Hkv, Lmax, 128]
  bf16_t* vc;
  int hq, hkv, lmax;
};

template <int M, int R, bool SWIGLU, bool NORM, bool ROPE = false, int KS = 1, int WV = GV_WAVES, int U = GV_U>
__global__ __launch_bounds__(64 * WV) void gemv_kernel(const bf16_t* __restrict__ x, long ldx,
                                                            const bf16_t* __restrict__ w, int N, int K,
                                                            bf16_t* __restrict__ y, long ldy, int up_off,
                                                            GvNorm na, GvRope ra) {
  static_assert(!ROPE || (R == 4 && !SWIGLU), "rope epilogue: 4 rows = two rotation pairs per wave");
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];   // NORM: M x K normalised rows
  __shared__ float ssq[WV][M];
  constexpr int NR = SWIGLU ? 2 * R : R;
  static_assert(KS == 1 || (KS == GV_WAVES && WV == GV_WAVES), "K split: 1 or all waves of the workgroup");
  __shared__ float red[KS > 1 ? GV_WAVES : 1][NR][M];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int gw = KS > 1 ? (int)blockIdx.x : (int)blockIdx.x * WV + wave;   // owner of R rows
  // ROPE: wave gw owns rotation pairs (p, p + 64) and (p + 1, p + 65) of head gw / 32
  const int r0 = ROPE ? (gw >> 5) * 128 + (gw & 31) * 2 : gw * R;
  const int nch = K >> 3;                       // 16-byte chunks per row
  const int J = (nch + 63) >> 6;                // chunk slots per lane
  const int Jw = (J + KS - 1) / KS;             // this wave's slots: [jb, je)
  const int jb = KS > 1 ? wave * Jw : 0;
  const int je = KS > 1 ? min(J, jb + Jw) : J;

  auto row_of = [&](int i) -> int {
    if constexpr (ROPE) return r0 + (i & 1) + (i >> 1) * 64;
    return i < R ? r0 + i : r0 + (i - R);
  };
  // Every load below is unconditional (rows past N read row N - 1, chunks past the row its last
  // chunk; neither sum is ever stored): with no load under a branch the compiler's vmcnt
  // bookkeeping stays exact, so each wait covers only the loads it needs.
  auto row_ptr = [&](int i) -> const bf16_t* {
    const int rc = min(row_of(i), N - 1);
    return w + (long)((SWIGLU && i >= R) ? rc + up_off : rc) * K;
  };

  // Loads that do not depend on the product go out ahead of the weights, so none of them is a
  // round trip of its own later: the epilogue's (position, slot), the norm prologue's x,
  // residual and gain chunks; the RoPE cos/sin (which need the position) right behind them.
  const int ep_i = lane / M;
  int ep_m = lane % M;
  // a per-lane (VGPR) index keeps these vector loads: as wave-uniform scalar loads (M = 1) the
  // compiler waited for them before issuing anything else
  asm volatile("" : "+v"(ep_m));
  int ep_pos = 0, ep_slot = 0;
  if constexpr (ROPE) {
    ep_pos = ra.pos[ep_m];
    ep_slot = ra.slots[ep_m];
  }
  constexpr int PW = 2;   // prologue passes whose operands are loaded up front (K <= 1024 WV)
  u32x4 wn[PW], xq[PW][M], rq[PW][M];
  const bf16_t* resp = na.res ? na.res : x;   // no residual: a harmless duplicate load of x
  if constexpr (NORM) {
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int c = min(tid + p * 64 * WV, nch - 1);
      wn[p] = ld16(na.w + 8 * c);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        xq[p][m] = ld16(x + (long)m * ldx + 8 * c);
        rq[p][m] = ld16(resp + (long)m * ldx + 8 * c);
      }
    }
  }
  u32x4 wv[NR][U];
  auto load_w = [&](int j0) {
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // slots past this wave's K range repeat its last slot (never another wave's: with a K
        // split that would stream the neighbour's weights a second time)
        const int c = min(lane + 64 * min(j0 + u, je - 1), nch - 1);
        wv[i][u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row_ptr(i) + 8 * c));
      }
  };
  load_w(jb);
  float ep_cos = 1.f, ep_sin = 0.f;
  if constexpr (ROPE) {
    // the position is consumed only here, behind the weight loads (the memory clobber keeps
    // them ahead of this wait)
    asm volatile("" : "+v"(ep_pos) : : "memory");
    const int pr = row_of(ep_i) & 63;
    ep_cos = ra.cos_t[(long)ep_pos * 64 + pr];
    ep_sin = ra.sin_t[(long)ep_pos * 64 + pr];
  }

  if constexpr (NORM) {
    float ss[M];
#pragma unroll
    for (int m = 0; m < M; ++m) ss[m] = 0.f;
    // h = x + res (kept, and normed, in bf16), its sum of squares, h staged in LDS.  The
    // up-front passes compute unconditionally (a pass past the row repeats its last chunk and
    // counts nothing): with the operands' uses under a branch hipcc sank their loads into it,
    // behind a wait for every weight load
    const bool has_res = na.res != nullptr;
    auto absorb = [&](int c_raw, const u32x4* xc, const u32x4* rc) {
      const bool valid = c_raw < nch;
      const int c = min(c_raw, nch - 1);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float hv[8], t[8];
        unpack8(xc[m], hv);
        unpack8(rc[m], t);
        // selects, not a branch on na.res (hipcc sank the residual load into it); without a
        // residual h = x, which the bf16 round trip leaves unchanged
#pragma unroll
        for (int e = 0; e < 8; ++e) hv[e] += has_res ? t[e] : 0.f;
        const u32x4 hb = pack8(hv);
        if (has_res && blockIdx.x == 0 && valid) st16(na.h_out + (long)m * na.ldh + 8 * c, hb);
        unpack8(hb, hv);
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) s += hv[e] * hv[e];
        ss[m] += valid ? s : 0.f;
        if (valid) *reinterpret_cast<u32x4*>(xs + (long)m * K + 8 * c) = pack8(hv);
      }
    };
#pragma unroll
    for (int p = 0; p < PW; ++p) absorb(tid + p * 64 * WV, xq[p], rq[p]);
    for (int c = tid + PW * 64 * WV; c < nch; c += 64 * WV) {
      u32x4 xc[M], rc[M];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        xc[m] = ld16(x + (long)m * ldx + 8 * c);
        rc[m] = ld16(resp + (long)m * ldx + 8 * c);
      }
      absorb(c, xc, rc);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float v = wave_sum(ss[m]);
      if (lane == 0) ssq[wave][m] = v;
    }
    __syncthreads();
    float rs[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float tot = 0.f;
#pragma unroll
      for (int v = 0; v < WV; ++v) tot += ssq[v][m];
      rs[m] = rsqrtf(tot / (float)K + na.eps);
    }
    // (in place, so only the owner of a chunk writes it back)
    auto apply = [&](int c_raw, u32x4 wq) {
      const int c = min(c_raw, nch - 1);
      float wf[8];
      unpack8(wq, wf);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float hv[8];
        unpack8(*reinterpret_cast<const u32x4*>(xs + (long)m * K + 8 * c), hv);
#pragma unroll
        for (int e = 0; e < 8; ++e) hv[e] = hv[e] * rs[m] * wf[e];
        if (c_raw < nch) *reinterpret_cast<u32x4*>(xs + (long)m * K + 8 * c) = pack8(hv);
      }
    };
#pragma unroll
    for (int p = 0; p < PW; ++p) apply(tid + p * 64 * WV, wn[p]);
    for (int c = tid + PW * 64 * WV; c < nch; c += 64 * WV) apply(c, ld16(na.w + 8 * c));
    __syncthreads();
  }

  float acc[NR][M];
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[i][m] = 0.f;

  for (int j0 = jb; j0 < je; j0 += U) {
    if (j0 > jb) load_w(j0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = lane + 64 * (j0 + u);
      if (j0 + u >= je || c >= nch) continue;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const u32x4 xv = NORM ? *reinterpret_cast<const u32x4*>(xs + (long)m * K + 8 * c)
                              : ld16(x + (long)m * ldx + 8 * c);
        // packed bf16 pairs straight into v_dot2c_f32_bf16: no unpacking of W or X
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const u32x4 wq = wv[i][u];
          acc[i][m] = dot2_bf16(wq.x, xv.x, acc[i][m]);
          acc[i][m] = dot2_bf16(wq.y, xv.y, acc[i][m]);
          acc[i][m] = dot2_bf16(wq.z, xv.z, acc[i][m]);
          acc[i][m] = dot2_bf16(wq.w, xv.w, acc[i][m]);
        }
      }
    }
  }

#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[i][m] = wave_sum(acc[i][m]);
  if constexpr (KS > 1) {
    // the workgroup's four K quarters meet in LDS; wave 0 runs the epilogue
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int m = 0; m < M; ++m) red[wave][i][m] = acc[i][m];
    }
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
      for (int m = 0; m < M; ++m) acc[i][m] = red[0][i][m] + red[1][i][m] + red[2][i][m] + red[3][i][m];
  }
  if (lane < R * M) {
    const int i = ep_i, m = ep_m;
    float g = 0.f, u = 0.f;
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
      for (int b = 0; b < M; ++b)
        if (a == i && b == m) {
          g = acc[a][b];
          if constexpr (SWIGLU) u = acc[R + a][b];
          if constexpr (ROPE) u = acc[a ^ 2][b];   // the other half of the rotation pair
        }
    const int row = row_of(i);
    if (row < N) {
      if constexpr (SWIGLU) g = g * sigmoidf_(g) * u;
      if constexpr (ROPE) {
        // same arithmetic as rope_append_kernel on the bf16 GEMM output
        const int head = row >> 7, d = row & 127, ps = ep_pos;
        float v = bf2f(f2bf(g));
        if (head < ra.hq + ra.hkv) {
          const float o = bf2f(f2bf(u)), c = ep_cos, sn = ep_sin;
          v = d < 64 ? __builtin_fmaf(v, c, -(o * sn)) : __builtin_fmaf(v, c, o * sn);   // == rope_lo / rope_hi
        }
        const bf16_t vb = f2bf(v);
        y[(long)m * ldy + row] = vb;
        if (head >= ra.hq) {
          const bool is_v = head >= ra.hq + ra.hkv;
          const int kh = is_v ? head - ra.hq - ra.hkv : head - ra.hq;
          (is_v ? ra.vc : ra.kc)[(((long)ep_slot * ra.hkv + kh) * ra.lmax + ps) * 128 + d] = vb;
        }
      } else {
        y[(long)m * ldy + row] = f2bf(g);
      }
    }
  }
}

// K split for deep K without the norm prologue when the unsplit grid leaves the 256 CUs
// with < 4 workgroups each; KFAMD_GEMV_KSPLIT=1 / 4 forces it off / on (A/B)
bool use_ksplit(int blocks_unsplit, int M, int K, bool norm) {
  static const int force = [] {
    const char* e = getenv("KFAMD_GEMV_KSPLIT");
    return e ? atoi(e) : 0;
  }();
  if (force == 1) return false;
  if (force == GV_WAVES) return true;
  // K = 4096 (wo) gains at 1-2 rows (8.9 -> 8.1-8.3 us, 9.7-10.1 -> 9.2-9.8 us) and loses at 4
  return !norm && (K >= 8192 || M <= 2) && blocks_unsplit < 4 * 256;
}

template <int M, bool SWIGLU, bool NORM>
int gv_launch(const bf16_t* x, long ldx, const bf16_t* w, int N, int K, bf16_t* y, long ldy, int up_off,
              GvNorm na, hipStream_t st) {
  constexpr int R = SWIGLU ? GV_R / 2 : GV_R;
  const int blocks = (N + R * GV_WAVES - 1) / (R * GV_WAVES);
  const size_t dyn = NORM ? (size_t)M * K * 2 : 0;
  const int jw = ((K / 8 + 63) / 64 + GV_WAVES - 1) / GV_WAVES;   // K-split: chunk slots per wave
  if (use_ksplit(blocks, M, K, NORM) && jw <= 2)   // (wo: 2 slots, no round of repeated loads)
    hipLaunchKernelGGL((gemv_kernel<M, R, SWIGLU, NORM, false, GV_WAVES, GV_WAVES, 2>), dim3((N + R - 1) / R),
                       dim3(64 * GV_WAVES), dyn, st, x, ldx, w, N, K, y, ldy, up_off, na, GvRope{});
  else if (use_ksplit(blocks, M, K, NORM))
    hipLaunchKernelGGL((gemv_kernel<M, R, SWIGLU, NORM, false, GV_WAVES>), dim3((N + R - 1) / R),
                       dim3(64 * GV_WAVES), dyn, st, x, ldx, w, N, K, y, ldy, up_off, na, GvRope{});
  else
    hipLaunchKernelGGL((gemv_kernel<M, R, SWIGLU, NORM>), dim3(blocks), dim3(64 * GV_WAVES), dyn, st, x, ldx, w,
                       N, K, y, ldy, up_off, na, GvRope{});
  KF_CHECK_LAUNCH();
  return 0;
}

template <bool SWIGLU, bool NORM>
int gv_dispatch(int M, const bf16_t* x, long ldx, const bf16_t* w, int N, int K, bf16_t* y, long ldy, int up_off,
                GvNorm na, hipStream_t st) {
  switch (M) {
    case 1: return gv_launch<1, SWIGLU, NORM>(x, ldx, w, N, K, y, ldy, up_off, na, st);
    case 2: return gv_launch<2, SWIGLU, NORM>(x, ldx, w, N, K, y, ldy, up_off, na, st);
    case 3: return gv_launch<3, SWIGLU, NORM>(x, ldx, w, N, K, y, ldy, up_off, na, st);
    case 4: return gv_launch<4, SWIGLU, NORM>(x, ldx, w, N, K, y, ldy, up_off, na, st);
    default: return 1;
  }
}

template <int M>
int gv_rope_launch(const bf16_t* x, long ldx, const bf16_t* w, int N, int K, bf16_t* y, long ldy, GvNorm na,
                   GvRope ra, hipStream_t st) {
  const int blocks = N / (4 * GV_WAVES);
  // Llama-3-8B qkv (6144 rows = 1536 four-row waves): 4-wave workgroups make 384, i.e. 1.5 per CU,
  // so half the CUs stream twice the bytes (12.1 us, 4.2 TB/s, gpurun_out/r4u); 6-wave workgroups
  // make exactly one per CU
  if ((N / 4) % (6 * 256) == 0 && !use_ksplit(blocks, M, K, true)) {
    // (the whole row in one round of 8 loads per lane: equal at 1 row, 0.6-0.7 % slower at 2-4,
    // gpurun_out/r4an)
    hipLaunchKernelGGL((gemv_kernel<M, 4, false, true, true, 1, 6>), dim3(N / 24), dim3(64 * 6), (size_t)M * K * 2,
                       st, x, ldx, w, N, K, y, ldy, 0, na, ra);
    KF_CHECK_LAUNCH();
    return 0;
  }
  if (use_ksplit(blocks, M, K, true))
    hipLaunchKernelGGL((gemv_kernel<M, 4, false, true, true, GV_WAVES>), dim3(N / 4), dim3(64 * GV_WAVES),
                       (size_t)M * K * 2, st, x, ldx, w, N, K, y, ldy, 0, na, ra);
  else
    hipLaunchKernelGGL((gemv_kernel<M, 4, false, true, true>), dim3(blocks), dim3(64 * GV_WAVES), (size_t)M * K * 2,
                       st, x, ldx, w, N, K, y, ldy, 0, na, ra);
  KF_CHECK_LAUNCH();
  return 0;
}

}  // namespace

constexpr int GV_MAX_M = 4;
constexpr long GV_NORM_LDS = 64 * 1024;

// y[M, N] = x . W^T (swiglu: W = [gate; up] with up rows at +up_off, y = silu(gate) * up).
// Optional norm prologue when nw != nullptr: x := rmsnorm(x + res) * nw, h_out = x + res.
// Returns 1 (nothing launched) when the shape is outside the kernel's range.
extern "C" int kf_gemv(const void* x, long ldx, int M, const void* res, const void* nw, float eps, void* h_out,
                       long ldh, const void* w, int N, int K, void* y, long ldy, int swiglu, int up_off,
                       hipStream_t st) {
  if (M < 1 || M > GV_MAX_M || K % 8 != 0 || ldx % 8 != 0 || N <= 0) return 1;
  if ((((uintptr_t)x) | ((uintptr_t)w)) & 15) return 1;
  const bool norm = nw != nullptr;
  if (norm && ((long)M * K * 2 > GV_NORM_LDS || (res && !h_out) || (res && (((uintptr_t)res) & 15)))) return 1;
  const GvNorm na{(const bf16_t*)res, (const bf16_t*)nw, (bf16_t*)h_out, ldh, eps};
  auto X = (const bf16_t*)x;
  auto W = (const bf16_t*)w;
  auto Y = (bf16_t*)y;
  if (swiglu) return norm ? gv_dispatch<true, true>(M, X, ldx, W, N, K, Y, ldy, up_off, na, st)
                          : gv_dispatch<true, false>(M, X, ldx, W, N, K, Y, ldy, up_off, na, st);
  return norm ? gv_dispatch<false, true>(M, X, ldx, W, N, K, Y, ldy, 0, na, st)
              : gv_dispatch<false, false>(M, X, ldx, W, N, K, Y, ldy, 0, na, st);
}

// Decode qkv projection with everything around it fused: h = x + res, rmsnorm(h) * nw as the
// X operand, Y = X . Wqkv^T, RoPE at pos[m] on the q/k heads (fp32 cos/sin [max_seq, 64]),
// and the rotated k plus v stored into the KV cache at (slots[m], pos[m]).  Head dim 128.
extern "C" int kf_gemv_norm_rope(const void* x, long ldx, int M, const void* res, const void* nw, float eps,
                                 void* h_out, long ldh, const void* w, int N, int K, void* y, long ldy,
                                 const float* cos_t, const float* sin_t, const int* slots, const int* pos, void* kc,
                                 void* vc, int hq, int hkv, int lmax, hipStream_t st) {
  if (M < 1 || M > GV_MAX_M || K % 8 != 0 || ldx % 8 != 0 || (long)M * K * 2 > GV_NORM_LDS) return 1;
  if (N != (hq + 2 * hkv) * 128 || (res && !h_out)) return 1;
  if ((((uintptr_t)x) | ((uintptr_t)w) | ((uintptr_t)res)) & 15) return 1;
  const GvNorm na{(const bf16_t*)res, (const bf16_t*)nw, (bf16_t*)h_out, ldh, eps};
  const GvRope ra{cos_t, sin_t, slots, pos, (bf16_t*)kc, (bf16_t*)vc, hq, hkv, lmax};
  auto X = (const bf16_t*)x;
  auto W = (const bf16_t*)w;
  auto Y = (bf16_t*)y;
  switch (M) {
    case 1: return gv_rope_launch<1>(X, ldx, W, N, K, Y, ldy, na, ra, st);
    case 2: return gv_rope_launch<2>(X, ldx, W, N, K, Y, ldy, na, ra, st);
    case 3: return gv_rope_launch<3>(X, ldx, W, N, K, Y, ldy, na, ra, st);
    default: return gv_rope_launch<4>(X, ldx, W, N, K, Y, ldy, na, ra, st);
  }
}
