// K8: single-query GQA decode attention over a slot-major KV cache (InferenceService).
//
// Cache layout per layer: k/v [n_slots, Hkv, Lmax, 128] bf16 -- one contiguous 256-byte
// row per (slot, head, position), so a head's keys stream linearly from HBM.  Each decode
// row b reads the slot slots[b] up to lengths[b] keys.  288 GB of HBM holds ~2M tokens of
// Llama-3-8B KV (128 KB/token), so slots are preallocated at full context length and no
// paging indirection sits on the memory-bound path.
//
// Split-K ("flash decoding"): grid (splits, Hkv, B), 256 threads.  One workgroup owns one
// (row, kv head, key chunk) and serves all G = Hq/Hkv query heads of the group, so every
// K/V byte is read exactly once.  A 16-lane quarter-wave owns one key row (16 lanes x 16 B);
// a wave covers 4 keys per load, the block 16.  The chunk is walked in sub-chunks of up to
// SUB keys (the LDS score rows), merged online, so the split count follows the batch
// (kf_decode_splits: ~2 workgroups per CU), never the slot length Lmax:
//   phase 1: s[h][j] = q_h . k_j: v_dot2 on packed bf16 pairs, the 16-lane row sum by DPP
//            (four VALU ops; __shfl_xor compiled to a chain of ds_bpermute LDS round trips),
//            lane h of the row stores head h's score -> LDS
//   phase 2: per head max / exp2 / sum over the sub-chunk (one wave per head), merged with
//            the running (max, sum); the padding past the sub-chunk becomes p = 0
//   phase 3: o[h] += p[h][j] v_j with 16 independent key streams (no masking), reduced
//            into LDS with the previous sub-chunks' rescaled sum
// Partial (o, m, l) per split go to an fp32 workspace and decode_combine merges the splits;
// with one split the workgroup normalises and writes the bf16 output itself (no combine).
// Measured (tools/bench_decode_splits.py, 32-layer graph, ctx 1024): 6.1 TB/s at batch 64,
// 5.7 TB/s at batch 128 (round 4: 4.2-4.3).  Decode is HBM-bound (2 flops/byte), so VALU dot
// products are the right tool: MFMA would pad the G<=8 query rows to 16/32 and buy nothing.
#include "common.h"

using namespace kf;

namespace {

constexpr int D = 128;
constexpr int NT = 256;
constexpr int MAXG = 8;
constexpr int SUB = 1024;       // keys per sub-chunk (LDS score rows)
constexpr float LOG2E = 1.4426950408889634f;

// DPP lane moves within a 16-lane row: one VALU op each (ds_bpermute, which __shfl_xor becomes,
// is an LDS round trip, and the per-key score reductions were a chain of them)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// acc + a.lo * b.lo + a.hi * b.hi for packed bf16 pairs (v_dot2c_f32_bf16)
__device__ __forceinline__ float dot2_bf16(u32 a, u32 b, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), acc, false);
}
// sum over the 16 lanes of a row, identical bits in every lane (each step pairs lanes
// symmetrically): quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror
__device__ __forceinline__ float row16_sum(float a) {
  a += dpp<0xB1>(a);
  a += dpp<0x4E>(a);
  a += dpp<0x141>(a);
  a += dpp<0x140>(a);
  return a;
}

// One workgroup per (split, kv head, row).  4 workgroups per CU at G = 4 (launch bounds:
// <= 128 VGPRs): B * Hkv = 1024 workgroups at batch 128 run in one round.  (A grid capped at 2
// workgroups per CU walking 2 items each, with 6 rows per stream in flight, measured the same
// 93.5 us per layer at batch 128 and spilled SGPRs.)
template <int G>
__global__ __launch_bounds__(NT, G <= 4 ? 4 : 2) void decode_split_kernel(
    const bf16_t* __restrict__ q, long q_ld, int hq_total,
    const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ slots, const int* __restrict__ lengths,
    long slot_stride, long head_stride, int splits, float scale_log2,
    float* __restrict__ part_o, float* __restrict__ part_ml, bf16_t* __restrict__ out, long out_ld) {
  // score rows padded by one round of keys: the last round writes (never read) past the chunk
  __shared__ float sc[G][SUB + 64];
  __shared__ float red[4][G][D];
  __shared__ float hm[G], hl[G], ha[G];

  const int s = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int sub = lane & 15;            // 16-byte column within the key row
  const int grp = tid >> 4;             // 0..15: key stream within the block
  const int len = min(lengths[b], (int)(head_stride / D));   // never read past the slot
  const int chunk = ((len + splits - 1) / splits + 15) & ~15;
  const int start = s * chunk;
  const int end = min(len, start + chunk);
  const long obase = ((long)b * hq_total + (long)hk * G) * splits + s;   // index of (b, h0, s)
  // one split (large batch: B * Hkv workgroups fill the chip on their own): normalise here and
  // write the bf16 output, no combine launch
  const bool direct = splits == 1;

  if (start >= end) {   // empty split: neutral element for the combine
    if (direct) {
      for (int e = tid; e < G * D; e += NT) out[(long)b * out_ld + (long)(hk * G) * D + e] = f2bf(0.f);
      return;
    }
    if (tid < G) {
      part_ml[(obase + (long)tid * splits) * 2 + 0] = -INFINITY;
      part_ml[(obase + (long)tid * splits) * 2 + 1] = 0.f;
    }
    // zero partial o too: the combine weighs it by 0, and 0 x (NaN left in an uninitialised
    // workspace) is NaN
    for (int e = tid; e < G * D; e += NT) part_o[(obase + (long)(e / D) * splits) * D + e % D] = 0.f;
    return;
  }
  const int n = end - start;
  for (int e = tid; e < 4 * G * D; e += NT) (&red[0][0][0])[e] = 0.f;   // ordered by phase 1's barrier

  // Memory-level parallelism is the whole game here: at large batch every CU runs 4 of these
  // workgroups and the chip is HBM-bound only if each keeps enough bytes in flight.  Every
  // 16-lane stream therefore loads R = 3 key rows per round and issues the NEXT round's rows
  // before it computes on the current ones (6 rows = 96 B per lane in flight, 96 KB per CU);
  // the first V round is issued before phase 1 ends.  (R = 4 at 3 workgroups per CU has the
  // same bytes in flight but left B * Hkv = 1024 workgroups a 1.33-round tail: 102 vs 93.5 us
  // per layer at batch 128.)  Row indices are clamped to the sub-chunk (always valid
  // addresses, no load under a branch: hipcc waited for every load in flight at each branch);
  // what lies past it is masked in the arithmetic.  One load in flight per stream measured
  // 4.2-4.3 TB/s at batch 64-128 (profiles/serve_llama3_8b_r4_final.jsonl).
  constexpr int R = 3;
  const long kvbase = (long)slots[b] * slot_stride + (long)hk * head_stride;
  const bf16_t* kbase = kc + kvbase + (long)start * D + sub * 8;
  const bf16_t* vbase = vc + kvbase + (long)start * D + sub * 8;


  // The chunk is walked in sub-chunks of at most SUB keys (the LDS score buffer), merged online
  // (running max / sum per head, the accumulator rescaled between sub-chunks): the split count
  // is chosen for parallelism alone, not bounded below by the slot length Lmax.
  for (int c0 = 0; c0 < n; c0 += SUB) {
    const int nc = min(SUB, n - c0);
    const bf16_t* kp = kbase + (long)c0 * D;
    const bf16_t* vp = vbase + (long)c0 * D;
    auto row = [&](int j) { return (long)min(j, nc - 1) * D; };
    u32x4 kb[R];
#pragma unroll
    for (int u = 0; u < R; ++u) kb[u] = ld16(kp + row(grp + 16 * u));
    // q for the G heads of this kv head: 8 dims per lane, packed bf16 (the dot products are
    // v_dot2 on bf16 pairs, exact products summed in fp32; the log2-domain scale is applied to
    // the reduced score).  Re-read per sub-chunk (an L2 hit) so it is not live in phase 3.
    u32x4 qb[G];
#pragma unroll
    for (int h = 0; h < G; ++h) qb[h] = ld16(q + (long)b * q_ld + (long)(hk * G + h) * D + sub * 8);

    // ---- phase 1: scores, R keys per stream per round, the next round's rows in flight
    for (int j0 = 0; j0 < nc; j0 += 16 * R) {
      u32x4 kn[R];
#pragma unroll
      for (int u = 0; u < R; ++u) kn[u] = ld16(kp + row(j0 + 16 * R + grp + 16 * u));
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int j = j0 + grp + 16 * u;
        // 4 v_dot2 per head on the packed rows (no bf16 -> fp32 unpack of k; decode attention
        // is close to VALU-bound at G = 4), then the 16-lane row sum by DPP
        float a[G];
#pragma unroll
        for (int h = 0; h < G; ++h) {
          float t = dot2_bf16(qb[h][0], kb[u][0], 0.f);
          t = dot2_bf16(qb[h][1], kb[u][1], t);
          t = dot2_bf16(qb[h][2], kb[u][2], t);
          t = dot2_bf16(qb[h][3], kb[u][3], t);
          a[h] = row16_sum(t);
        }
        // lane `sub` of the row stores head `sub`'s score (no per-head branch); j >= nc lands
        // in the padding, which phase 2 overwrites with p = 0
        float v = a[0];
#pragma unroll
        for (int h = 1; h < G; ++h) v = sub == h ? a[h] : v;
        if (sub < G) sc[sub][j] = v * scale_log2;
        kb[u] = kn[u];
      }
    }
    // the first V round goes out before the barrier
    u32x4 vb[R];
#pragma unroll
    for (int u = 0; u < R; ++u) vb[u] = ld16(vp + row(grp + 16 * u));
    __syncthreads();

    // ---- phase 2: softmax statistics per head (wave w handles heads w, w+4), merged with the
    // previous sub-chunks'
    for (int h = wave; h < G; h += 4) {
      float m = -INFINITY;
      for (int j = lane; j < nc; j += 64) m = fmaxf(m, sc[h][j]);
      m = wave_max(m);
      const float m_old = c0 == 0 ? -INFINITY : hm[h];
      const float mn = fmaxf(m, m_old);
      float l = 0.f;
      // through the padding of the last 16R-key round: phase 3 reads p = 0 there, no masking
      for (int j = lane; j < (nc + 16 * R - 1) / (16 * R) * (16 * R); j += 64) {
        const float p = j < nc ? exp2f(sc[h][j] - mn) : 0.f;
        sc[h][j] = p;
        l += p;
      }
      l = wave_sum(l);
      if (lane == 0) {
        const float alpha = c0 == 0 ? 0.f : exp2f(m_old - mn);
        hm[h] = mn;
        hl[h] = c0 == 0 ? l : fmaf(hl[h], alpha, l);
        ha[h] = alpha;
      }
    }
    __syncthreads();

    // ---- phase 3: P.V, R keys per stream per round, the next round's rows in flight.  The
    // sub-chunk's sum is folded into the wave's row of `red` at the end (rescaled by alpha), so
    // no accumulator stays live through phase 1.
    float acc[G][8];
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] = 0.f;
    for (int j0 = 0; j0 < nc; j0 += 16 * R) {
      u32x4 vn[R];
#pragma unroll
      for (int u = 0; u < R; ++u) vn[u] = ld16(vp + row(j0 + 16 * R + grp + 16 * u));
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int j = j0 + grp + 16 * u;       // < nc rounded up to 16R: zero past nc (phase 2)
        float vf[8];
        unpack8(vb[u], vf);
#pragma unroll
        for (int h = 0; h < G; ++h) {
          const float p = sc[h][j];
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[h][i] = fmaf(p, vf[i], acc[h][i]);
        }
        vb[u] = vn[u];
      }
    }
    // reduce the 4 streams of a wave (lanes l, l^16, l^32, l^48 share a column) into red[wave]
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float a = acc[h][i];
        a += __shfl_xor(a, 16, 64);
        a += __shfl_xor(a, 32, 64);
        acc[h][i] = a;
      }
    if (lane < 16) {
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const float al = ha[h];                 // 0 for the first sub-chunk (red starts at 0)
#pragma unroll
        for (int i = 0; i < 8; ++i) red[wave][h][sub * 8 + i] = fmaf(red[wave][h][sub * 8 + i], al, acc[h][i]);
      }
    }
    if (c0 + SUB < n) __syncthreads();     // the next sub-chunk's phase 1 rewrites sc
  }
  __syncthreads();
  for (int e = tid; e < G * D; e += NT) {
    const int h = e / D, d = e % D;
    const float o = red[0][h][d] + red[1][h][d] + red[2][h][d] + red[3][h][d];
    if (direct)
      out[(long)b * out_ld + (long)(hk * G + h) * D + d] = f2bf(hl[h] > 0.f ? o / hl[h] : 0.f);
    else
      part_o[(obase + (long)h * splits) * D + d] = o;
  }
  if (tid < G && !direct) {
    part_ml[(obase + (long)tid * splits) * 2 + 0] = hm[tid];
    part_ml[(obase + (long)tid * splits) * 2 + 1] = hl[tid];
  }
}

// one block per (b, q head), 256 threads: merge the split partials, normalise, write bf16.
// At B = 1 the merge is latency-bound (up to ~128 splits of a few keys each), so the work
// is spread over the block instead of one dependent loop per output element:
//   1. the split maxima / weights w_s = exp2(m_s - M) and den = sum w_s l_s are computed
//      once per block (one split per thread) and w_s is kept in LDS;
//   2. the two 128-thread halves each sum w_s o_s[d] over every other split (independent,
//      coalesced L2 loads, 8 in flight per thread), then add their halves through LDS.
constexpr int CB_NT = 256, CB_MAXS = 1024;
__global__ __launch_bounds__(CB_NT) void decode_combine_kernel(const float* __restrict__ part_o,
                                                               const float* __restrict__ part_ml,
                                                               int splits, bf16_t* __restrict__ out,
                                                               long out_ld, int hq) {
  __shared__ float ws[CB_MAXS];
  __shared__ float red[CB_NT / 64];
  __shared__ float half_num[D];
  const int bh = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = bh / hq, h = bh % hq;
  const float* ml = part_ml + (long)bh * splits * 2;
  const int d = tid & (D - 1), half = tid / D;
  const float* po = part_o + (long)bh * splits * D + d;
  // up to 32 splits (every batch-1 launch): this thread's 16 partial values are loaded up front,
  // together with the (max, sum) pairs, so the merge costs one memory round trip, not three
  // Loads are unconditional (indices clamped; what is past the splits is never used): under
  // per-split branches hipcc waited for every load in flight at each one.  Up to CB_NT splits
  // this thread's (max, sum) pair stays in registers for the weight pass below (no second read).
  constexpr int PRE = 16;
  float pre[PRE];
  const bool preload = splits <= 2 * PRE;
  const bool one = splits <= CB_NT;
  const f32x2_t ml_own = *reinterpret_cast<const f32x2_t*>(ml + 2 * min(tid, splits - 1));
#pragma unroll
  for (int i = 0; i < PRE; ++i) pre[i] = po[(long)min(half + 2 * i, splits - 1) * D];
  float mloc = tid < splits ? ml_own[0] : -INFINITY;
  for (int s = tid + CB_NT; s < splits; s += CB_NT) mloc = fmaxf(mloc, ml[2 * s]);
  mloc = wave_max(mloc);
  if (lane == 0) red[wave] = mloc;
  __syncthreads();
  float M = red[0];
#pragma unroll
  for (int w = 1; w < CB_NT / 64; ++w) M = fmaxf(M, red[w]);
  __syncthreads();
  float dl = 0.f;
  if (one) {
    if (tid < splits) {
      const float w = ml_own[0] == -INFINITY ? 0.f : exp2f(ml_own[0] - M);
      ws[tid] = w;
      dl = w * ml_own[1];
    }
  } else {
    for (int s = tid; s < splits; s += CB_NT) {
      const float m = ml[2 * s];
      const float w = m == -INFINITY ? 0.f : exp2f(m - M);
      ws[s] = w;
      dl = fmaf(w, ml[2 * s + 1], dl);
    }
  }
  dl = wave_sum(dl);
  if (lane == 0) red[wave] = dl;
  __syncthreads();
  float den = 0.f;
#pragma unroll
  for (int w = 0; w < CB_NT / 64; ++w) den += red[w];
  __syncthreads();                                   // ws complete
  float num = 0.f;
  if (preload) {
#pragma unroll
    for (int i = 0; i < PRE; ++i) {
      const int s = half + 2 * i;
      if (s < splits) num = fmaf(ws[s], pre[i], num);
    }
  } else {
#pragma unroll 8
    for (int s = half; s < splits; s += 2) num = fmaf(ws[s], po[(long)s * D], num);
  }
  if (half == 1) half_num[d] = num;
  __syncthreads();
  if (half == 0) {
    num += half_num[d];
    out[(long)b * out_ld + (long)h * D + d] = f2bf(den > 0.f ? num / den : 0.f);
  }
}

// ---- small-batch decode (B <= SMALL_B): split-K and the combine in ONE launch ------------------
// At B = 1 the two-kernel form is latency-bound (ctx 1024: 4 MB of K/V per layer in 8 + 4.7 us,
// ~0.3 TB/s): each split kernel block runs three dependent phases, then a second launch merges.
// Here every block streams its chunk in rounds of 32 keys with all four of a thread's 16-byte
// loads (2 K rows, 2 V rows) in flight together, keeps an online softmax per thread (its own
// keys), merges the 16 key streams of the block at the end, publishes its partial with
// write-through (sc1) stores, and takes a ticket on a per-(row, kv head) counter: the block
// whose ticket comes last merges all splits (sc1 loads) and writes the output, then re-arms the
// counter for the next launch (the hand-off form of MI355X_MICROARCH.md "Valid forms", row 1).
constexpr int SMALL_B = 4, MAX_SPLITS1 = 64, KR = 32;   // keys per round: 2 per 16-lane group
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int G>
__global__ __launch_bounds__(NT) void decode_fused_kernel(
    const bf16_t* __restrict__ q, long q_ld, int hq_total,
    const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ slots, const int* __restrict__ lengths,
    long slot_stride, long head_stride, int splits, float scale_log2,
    float* __restrict__ part_o, float* __restrict__ part_ml, int* __restrict__ tickets,
    bf16_t* __restrict__ out, long out_ld) {
  __shared__ float sm[4][G], sl[4][G];
  __shared__ float so[4][G][D];
  __shared__ int is_last;
  const int s = blockIdx.x, hk = blockIdx.y, b = blockIdx.z, Hkv = gridDim.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int sub = lane & 15, grp = tid >> 4;
  const int len = min(lengths[b], (int)(head_stride / D));
  const int chunk = ((len + splits - 1) / splits + 15) & ~15;     // 16-key granules
  const int start = s * chunk, end = min(len, start + chunk);

  // q packed bf16 (scores are v_dot2 on bf16 pairs, fp32 sums; the log2-domain scale is
  // applied to the reduced score)
  u32x4 qb[G];
#pragma unroll
  for (int h = 0; h < G; ++h) qb[h] = ld16(q + (long)b * q_ld + (long)(hk * G + h) * D + sub * 8);
  const long kvbase = (long)slots[b] * slot_stride + (long)hk * head_stride;
  const bf16_t* kp = kc + kvbase;
  const bf16_t* vp = vc + kvbase;

  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[h][i] = 0.f;
  }
  for (int r0 = start; r0 < end; r0 += KR) {
    const int j0 = r0 + grp, j1 = r0 + 16 + grp;
    const bool ok0 = j0 < end, ok1 = j1 < end;
    // rows clamped into the chunk: every load is unconditional (no load under a branch), what
    // lies past the chunk is masked in the arithmetic
    const long o0 = (long)min(j0, end - 1) * D + sub * 8, o1 = (long)min(j1, end - 1) * D + sub * 8;
    const u32x4 k0 = ld16(kp + o0), k1 = ld16(kp + o1), v0 = ld16(vp + o0), v1 = ld16(vp + o1);
    float vf0[8], vf1[8];
    unpack8(v0, vf0);
    unpack8(v1, vf1);
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float a0 = dot2_bf16(qb[h][0], k0[0], 0.f), a1 = dot2_bf16(qb[h][0], k1[0], 0.f);
#pragma unroll
      for (int c = 1; c < 4; ++c) {
        a0 = dot2_bf16(qb[h][c], k0[c], a0);
        a1 = dot2_bf16(qb[h][c], k1[c], a1);
      }
      a0 = ok0 ? row16_sum(a0) * scale_log2 : -INFINITY;
      a1 = ok1 ? row16_sum(a1) * scale_log2 : -INFINITY;
      const float mn = fmaxf(m[h], fmaxf(a0, a1));
      if (mn == -INFINITY) continue;              // no valid key yet for this stream
      const float al = exp2f(m[h] - mn), p0 = exp2f(a0 - mn), p1 = exp2f(a1 - mn);
      m[h] = mn;
      l[h] = fmaf(l[h], al, p0 + p1);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] = fmaf(acc[h][i], al, fmaf(p0, vf0[i], p1 * vf1[i]));
    }
  }
  // merge the 4 key streams of each wave (lanes l, l^16, l^32, l^48 hold the same columns)
#pragma unroll
  for (int h = 0; h < G; ++h) {
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      const float mo = __shfl_xor(m[h], o, 64), lo_ = __shfl_xor(l[h], o, 64);
      const float mn = fmaxf(m[h], mo);
      const float a = mn == -INFINITY ? 0.f : exp2f(m[h] - mn), c = mn == -INFINITY ? 0.f : exp2f(mo - mn);
      l[h] = l[h] * a + lo_ * c;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] = acc[h][i] * a + __shfl_xor(acc[h][i], o, 64) * c;
      m[h] = mn;
    }
  }
  if (lane < 16) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
#pragma unroll
      for (int i = 0; i < 8; ++i) so[wave][h][sub * 8 + i] = acc[h][i];
      if (sub == 0) { sm[wave][h] = m[h]; sl[wave][h] = l[h]; }
    }
  }
  __syncthreads();
  // the block's partial: merge the 4 waves, publish write-through
  const long pbase = ((long)b * Hkv + hk) * MAX_SPLITS1 + s;          // (row, kv head, split)
  for (int e = tid; e < G * D; e += NT) {
    const int h = e / D, d = e % D;
    float M = sm[0][h];
#pragma unroll
    for (int w = 1; w < 4; ++w) M = fmaxf(M, sm[w][h]);
    float o = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < 4; ++w) o = fmaf(exp2f(sm[w][h] - M), so[w][h][d], o);
    }
    st_sc1(part_o + (pbase * G + h) * D + d, o);
  }
  if (tid < G) {
    float M = sm[0][tid];
#pragma unroll
    for (int w = 1; w < 4; ++w) M = fmaxf(M, sm[w][tid]);
    float L = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < 4; ++w) L = fmaf(exp2f(sm[w][tid] - M), sl[w][tid], L);
    }
    st_sc1(part_ml + (pbase * G + tid) * 2 + 0, M);
    st_sc1(part_ml + (pbase * G + tid) * 2 + 1, L);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // every storing wave drains its stores
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(tickets + (long)b * Hkv + hk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = t == splits - 1;
  }
  __syncthreads();
  if (!is_last) return;
  // last block: merge every split of this (row, kv head) and write the G heads' outputs.
  // (1) all (m, l) pairs at once; (2) per head one wave: global max, split weights, denominator;
  // (3) every output element sums its splits' weighted partials, 8 independent loads in flight.
  const long obase = ((long)b * Hkv + hk) * MAX_SPLITS1;
  __shared__ float wt[MAX_SPLITS1][G], lt[MAX_SPLITS1][G], den[G];
  for (int e = tid; e < splits * G; e += NT) {
    const int t = e / G, h = e % G;
    wt[t][h] = ld_sc1(part_ml + ((obase + t) * G + h) * 2);
    lt[t][h] = ld_sc1(part_ml + ((obase + t) * G + h) * 2 + 1);
  }
  __syncthreads();
  for (int h = wave; h < G; h += NT / 64) {
    const float ms = lane < splits ? wt[lane][h] : -INFINITY;
    const float M = wave_max(ms);
    const float w = (M == -INFINITY || ms == -INFINITY) ? 0.f : exp2f(ms - M);
    const float L = wave_sum(lane < splits ? w * lt[lane][h] : 0.f);
    if (lane < splits) wt[lane][h] = w;
    if (lane == 0) den[h] = L;
  }
  __syncthreads();
  for (int e = tid; e < G * D; e += NT) {
    const int h = e / D, d = e % D;
    float o = 0.f;
#pragma unroll 8
    for (int t = 0; t < splits; ++t) o = fmaf(wt[t][h], ld_sc1(part_o + ((obase + t) * G + h) * D + d), o);
    out[(long)b * out_ld + (long)(hk * G + h) * D + d] = f2bf(den[h] > 0.f ? o / den[h] : 0.f);
  }
  if (tid == 0) __hip_atomic_store(tickets + (long)b * Hkv + hk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int G>
void launch_fused(dim3 grid, hipStream_t st, const bf16_t* q, long q_ld, int hq, const bf16_t* kc,
                  const bf16_t* vc, const int* slots, const int* lengths, long slot_stride, long head_stride,
                  int splits, float sl2, float* po, float* pml, int* tickets, bf16_t* out, long out_ld) {
  hipLaunchKernelGGL(decode_fused_kernel<G>, grid, dim3(NT), 0, st, q, q_ld, hq, kc, vc, slots, lengths,
                     slot_stride, head_stride, splits, sl2, po, pml, tickets, out, out_ld);
}

template <int G>
void launch_split(dim3 grid, hipStream_t st, const bf16_t* q, long q_ld, int hq, const bf16_t* kc,
                  const bf16_t* vc, const int* slots, const int* lengths, long slot_stride,
                  long head_stride, int splits, float sl2, float* po, float* pml, bf16_t* out, long out_ld) {
  hipLaunchKernelGGL(decode_split_kernel<G>, grid, dim3(NT), 0, st, q, q_ld, hq, kc, vc, slots, lengths,
                     slot_stride, head_stride, splits, sl2, po, pml, out, out_ld);
}

}  // namespace

// Number of key splits for a batch: about two workgroups per CU (B * Hkv * splits >= 512) and
// chunks of at least 64 keys.  Any chunk length works (sub-chunks of SUB keys).  Measured in a
// 32-layer graph at context 1024 (tools/bench_decode_splits.py): batch 64 runs 42.5 us per layer
// at 1 split (512 workgroups, no combine) against 53.4 at 2 and 49.7 at 3.
extern "C" int kf_decode_splits(int B, int Hkv, int Lmax) {
  const int want = std::max(1, (512 + B * Hkv - 1) / (B * Hkv));
  const int max_by_len = std::max(1, Lmax / 64);
  return std::min(want, max_by_len);
}

// Small-batch single-launch decode attention (B <= SMALL_B).  splits1: key splits per (row, kv
// head), <= MAX_SPLITS1; workspace part_o fp32 [B*Hkv*MAX_SPLITS1*G*D], part_ml fp32
// [B*Hkv*MAX_SPLITS1*G*2]; tickets int32 [B*Hkv], zero before the first launch (each launch
// leaves them zero).
extern "C" int kf_decode_splits1(int B, int Hkv, int Lmax) {
  // ~one workgroup per CU (B = 1, 8 kv heads: 32 splits), <= MAX_SPLITS1 splits: more splits
  // lengthen the last block's merge (its loads are a serial tail) more than they shorten the rest
  const int want = std::max(1, 256 / std::max(1, B * Hkv));
  return std::max(1, std::min({want, MAX_SPLITS1, (Lmax + 15) / 16}));
}

extern "C" int kf_decode_attn_fused(const void* q, long q_ld, const void* kc, const void* vc, const int* slots,
                                    const int* lengths, void* out, long out_ld, float* part_o, float* part_ml,
                                    int* tickets, int B, int Hq, int Hkv, int Dh, int Lmax, int splits,
                                    float scale, hipStream_t st) {
  if (Dh != D || Hkv <= 0 || Hq % Hkv != 0) return 1;
  const int G = Hq / Hkv;
  if (G > MAXG || splits <= 0 || splits > MAX_SPLITS1 || B > SMALL_B) return 2;
  if (B == 0) return 0;
  const long head_stride = (long)Lmax * D, slot_stride = (long)Hkv * head_stride;
  const float sl2 = scale * LOG2E;
  dim3 grid(splits, Hkv, B);
  auto q16 = (const bf16_t*)q;
  auto k16 = (const bf16_t*)kc;
  auto v16 = (const bf16_t*)vc;
  auto o16 = (bf16_t*)out;
  switch (G) {
    case 1: launch_fused<1>(grid, st, q16, q_ld, Hq, k16, v16, slots, lengths, slot_stride, head_stride, splits, sl2, part_o, part_ml, tickets, o16, out_ld); break;
    case 2: launch_fused<2>(grid, st, q16, q_ld, Hq, k16, v16, slots, lengths, slot_stride, head_stride, splits, sl2, part_o, part_ml, tickets, o16, out_ld); break;
    case 4: launch_fused<4>(grid, st, q16, q_ld, Hq, k16, v16, slots, lengths, slot_stride, head_stride, splits, sl2, part_o, part_ml, tickets, o16, out_ld); break;
    case 8: launch_fused<8>(grid, st, q16, q_ld, Hq, k16, v16, slots, lengths, slot_stride, head_stride, splits, sl2, part_o, part_ml, tickets, o16, out_ld); break;
    default: return 4;
  }
  KF_CHECK_LAUNCH();
  return 0;
}

// q: rows of [Hq*D] bf16 with row stride q_ld (the q columns of a fused qkv row work).
// k/v cache: [n_slots, Hkv, Lmax, D]. workspace: part_o fp32 [B*Hq*splits*D],
// part_ml fp32 [B*Hq*splits*2]. out: rows of [Hq*D] with stride out_ld.
extern "C" int kf_decode_attn(const void* q, long q_ld, const void* kc, const void* vc, const int* slots,
                              const int* lengths, void* out, long out_ld, float* part_o, float* part_ml,
                              int B, int Hq, int Hkv, int Dh, int Lmax, int splits, float scale,
                              hipStream_t st) {
  if (Dh != D || Hkv <= 0 || Hq % Hkv != 0) return 1;
  const int G = Hq / Hkv;
  if (G > MAXG || splits <= 0 || splits > CB_MAXS) return 2;
  if (B == 0) return 0;
  const long head_stride = (long)Lmax * D, slot_stride = (long)Hkv * head_stride;
  const float sl2 = scale * LOG2E;
  dim3 grid(splits, Hkv, B);
  auto q16 = (const bf16_t*)q;
  auto k16 = (const bf16_t*)kc;
  auto v16 = (const bf16_t*)vc;
  switch (G) {
    case 1: launch_split<1>(grid, st, q16, q_ld, Hq, k16, v16, slots, lengths, slot_stride, head_stride, splits, sl2, part_o, part_ml, (bf16_t*)out, out_ld); break;
    case 2: launch_split<2>(grid, st, q16, q_ld, Hq, k16, v16, slots, lengths, slot_stride, head_stride, splits, sl2, part_o, part_ml, (bf16_t*)out, out_ld); break;
    case 4: launch_split<4>(grid, st, q16, q_ld, Hq, k16, v16, slots, lengths, slot_stride, head_stride, splits, sl2, part_o, part_ml, (bf16_t*)out, out_ld); break;
    case 8: launch_split<8>(grid, st, q16, q_ld, Hq, k16, v16, slots, lengths, slot_stride, head_stride, splits, sl2, part_o, part_ml, (bf16_t*)out, out_ld); break;
    default: return 4;
  }
  if (splits > 1)
    hipLaunchKernelGGL(decode_combine_kernel, dim3(B * Hq), dim3(CB_NT), 0, st, part_o, part_ml, splits,
                       (bf16_t*)out, out_ld, Hq);
  KF_CHECK_LAUNCH();
  return 0;
}

// The rotation of one RoPE pair with the rounding pinned down (explicit fma, the other product
// rounded on its own): hipcc contracts `a * c - b * s` differently from kernel to kernel, and the
// decode kernels that rotate (rope_append, rope_append_parts, gemv_norm_rope) must agree bit for bit
__device__ __forceinline__ float rope_lo(float a, float b, float c, float s) { return __builtin_fmaf(a, c, -(b * s)); }
__device__ __forceinline__ float rope_hi(float b, float a, float c, float s) { return __builtin_fmaf(b, c, a * s); }

// Decode step prologue fused into one launch: RoPE (half-split, fp32 tables) in place on the
// q and k heads of each fused qkv row at position pos[b], and the rotated k plus v appended
// to the cache at pos[b] of slot slots[b].  One thread per 8 rotation pairs.
__global__ void rope_append_kernel(bf16_t* __restrict__ qkv, long ld, int Hq, int Hkv,
                                   const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                   const int* __restrict__ slots, const int* __restrict__ pos,
                                   bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, int Lmax, int B) {
  constexpr int HALF = D / 2, CPH = HALF / 8;            // 8 chunks of 8 pairs per head
  const int it = blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = (Hq + 2 * Hkv) * CPH;
  if (it >= B * per_row) return;
  const int b = it / per_row, rem = it % per_row, h = rem / CPH, c = rem % CPH;
  const int p = pos[b];
  bf16_t* px = qkv + (long)b * ld + (long)h * D + c * 8;
  const bool is_v = h >= Hq + Hkv;
  u32x4 lo = ld16(px), hi = ld16(px + HALF);
  if (!is_v) {
    float a[8], bb[8], o1[8], o2[8];
    unpack8(lo, a);
    unpack8(hi, bb);
    const float* pc = cos_t + (long)p * HALF + c * 8;
    const float* ps = sin_t + (long)p * HALF + c * 8;
    const f32x4 c0 = ldf4(pc), c1 = ldf4(pc + 4), s0 = ldf4(ps), s1 = ldf4(ps + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cc = j < 4 ? c0[j] : c1[j - 4], ss = j < 4 ? s0[j] : s1[j - 4];
      o1[j] = rope_lo(a[j], bb[j], cc, ss);
      o2[j] = rope_hi(bb[j], a[j], cc, ss);
    }
    lo = pack8(o1);
    hi = pack8(o2);
    st16(px, lo);
    st16(px + HALF, hi);
  }
  if (h >= Hq) {
    const int kh = is_v ? h - Hq - Hkv : h - Hq;
    bf16_t* dst = (is_v ? vc : kc) + (((long)slots[b] * Hkv + kh) * Lmax + p) * D + c * 8;
    st16(dst, lo);
    st16(dst + HALF, hi);
  }
}

// rope_append_kernel fed by the fp32 K-split partials [S, B, (Hq + 2 Hkv) * D] of the qkv
// batched-decode GEMM (its reduce launch skipped): each thread sums its 8 + 8 elements in slice
// order, rounds them to bf16 exactly as bgemm_reduce_kernel does, writes the qkv row (rotated q
// and k, v as is) and appends k / v to the cache -- the same values as reduce + rope_append.
template <int S>
__global__ void rope_append_parts_kernel(const float* __restrict__ part, bf16_t* __restrict__ qkv, int Hq, int Hkv,
                                         const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                         const int* __restrict__ slots, const int* __restrict__ pos,
                                         bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, int Lmax, int B) {
  constexpr int HALF = D / 2, CPH = HALF / 8;
  const int it = blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = (Hq + 2 * Hkv) * CPH, N = (Hq + 2 * Hkv) * D;
  if (it >= B * per_row) return;
  const int b = it / per_row, rem = it % per_row, h = rem / CPH, c = rem % CPH;
  const long off = (long)b * N + (long)h * D + c * 8;
  const long pstride = (long)B * N;
  f32x4 v[S][4];
#pragma unroll
  for (int t = 0; t < S; ++t) {
    v[t][0] = ldf4(part + t * pstride + off);
    v[t][1] = ldf4(part + t * pstride + off + 4);
    v[t][2] = ldf4(part + t * pstride + off + HALF);
    v[t][3] = ldf4(part + t * pstride + off + HALF + 4);
  }
  f32x4 sl0 = f32x4{0.f, 0.f, 0.f, 0.f}, sl1 = sl0, sh0 = sl0, sh1 = sl0;
#pragma unroll
  for (int t = 0; t < S; ++t) {
    sl0 += v[t][0];
    sl1 += v[t][1];
    sh0 += v[t][2];
    sh1 += v[t][3];
  }
  u32x4 lo = u32x4{pack2(sl0[0], sl0[1]), pack2(sl0[2], sl0[3]), pack2(sl1[0], sl1[1]), pack2(sl1[2], sl1[3])};
  u32x4 hi = u32x4{pack2(sh0[0], sh0[1]), pack2(sh0[2], sh0[3]), pack2(sh1[0], sh1[1]), pack2(sh1[2], sh1[3])};
  const int p = pos[b];
  const bool is_v = h >= Hq + Hkv;
  if (!is_v) {
    float a[8], bb[8], o1[8], o2[8];
    unpack8(lo, a);
    unpack8(hi, bb);
    const float* pc = cos_t + (long)p * HALF + c * 8;
    const float* ps = sin_t + (long)p * HALF + c * 8;
    const f32x4 c0 = ldf4(pc), c1 = ldf4(pc + 4), s0 = ldf4(ps), s1 = ldf4(ps + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cc = j < 4 ? c0[j] : c1[j - 4], ss = j < 4 ? s0[j] : s1[j - 4];
      o1[j] = rope_lo(a[j], bb[j], cc, ss);
      o2[j] = rope_hi(bb[j], a[j], cc, ss);
    }
    lo = pack8(o1);
    hi = pack8(o2);
  }
  bf16_t* px = qkv + off;
  st16(px, lo);
  st16(px + HALF, hi);
  if (h >= Hq) {
    const int kh = is_v ? h - Hq - Hkv : h - Hq;
    bf16_t* dst = (is_v ? vc : kc) + (((long)slots[b] * Hkv + kh) * Lmax + p) * D + c * 8;
    st16(dst, lo);
    st16(dst + HALF, hi);
  }
}

extern "C" int kf_rope_append_parts(const float* part, int S, void* qkv, int B, int Hq, int Hkv, int Dh,
                                    const float* cos_t, const float* sin_t, const int* slots, const int* pos, void* kc,
                                    void* vc, int Lmax, hipStream_t st) {
  if (Dh != D || B < 1) return 1;
  const int threads = B * (Hq + 2 * Hkv) * (D / 16);
  const dim3 grid(cdiv(threads, 256));
#define RA_PARTS(SV)                                                                                            \
  hipLaunchKernelGGL(rope_append_parts_kernel<SV>, grid, dim3(256), 0, st, part, (bf16_t*)qkv, Hq, Hkv, cos_t, sin_t, \
                     slots, pos, (bf16_t*)kc, (bf16_t*)vc, Lmax, B)
  if (S == 2) RA_PARTS(2);
  else if (S == 4) RA_PARTS(4);
  else if (S == 8) RA_PARTS(8);
  else return 1;
#undef RA_PARTS
  KF_CHECK_LAUNCH();
  return 0;
}

extern "C" int kf_rope_append(void* qkv, long ld, int B, int Hq, int Hkv, int Dh, const float* cos_t,
                              const float* sin_t, const int* slots, const int* pos, void* kc, void* vc, int Lmax,
                              hipStream_t st) {
  if (Dh != D) return 1;
  if (B == 0) return 0;
  const int threads = B * (Hq + 2 * Hkv) * (D / 16);
  hipLaunchKernelGGL(rope_append_kernel, dim3(cdiv(threads, 256)), dim3(256), 0, st, (bf16_t*)qkv, ld, Hq, Hkv,
                     cos_t, sin_t, slots, pos, (bf16_t*)kc, (bf16_t*)vc, Lmax, B);
  KF_CHECK_LAUNCH();
  return 0;
}

// Append the current token's K/V (post-RoPE, taken from the fused qkv rows) into the cache at
// position pos[b] of slot slots[b].  One 16-lane group per (row, kv head, k|v).
__global__ void kv_append_kernel(const bf16_t* __restrict__ qkv, long ld, int Hq, int Hkv,
                                 const int* __restrict__ slots, const int* __restrict__ pos,
                                 bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, int Lmax, int B) {
  const int g = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;   // (b, kv, h)
  const int sub = threadIdx.x & 15;
  if (g >= B * 2 * Hkv) return;
  const int b = g / (2 * Hkv), r = g % (2 * Hkv), which = r / Hkv, h = r % Hkv;
  const bf16_t* src = qkv + (long)b * ld + (long)(Hq + which * Hkv + h) * D + sub * 8;
  bf16_t* dst = (which ? vc : kc) + (((long)slots[b] * Hkv + h) * Lmax + pos[b]) * D + sub * 8;
  st16(dst, ld16(src));
}

extern "C" int kf_kv_append(const void* qkv, long ld, int B, int Hq, int Hkv, int Dh, const int* slots,
                            const int* pos, void* kc, void* vc, int Lmax, hipStream_t st) {
  if (Dh != D) return 1;
  if (B == 0) return 0;
  const int threads = B * 2 * Hkv * 16;
  hipLaunchKernelGGL(kv_append_kernel, dim3(cdiv(threads, 256)), dim3(256), 0, st, (const bf16_t*)qkv, ld,
                     Hq, Hkv, slots, pos, (bf16_t*)kc, (bf16_t*)vc, Lmax, B);
  KF_CHECK_LAUNCH();
  return 0;
}

// Prefill: copy rows [0, S) of one sequence's fused qkv into slot `slot` (positions 0..S-1).
__global__ void kv_fill_kernel(const bf16_t* __restrict__ qkv, long ld, int S, int Hq, int Hkv, int slot,
                               bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, int Lmax) {
  const long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 4;   // (t, kv, h)
  const int sub = threadIdx.x & 15;
  if (g >= (long)S * 2 * Hkv) return;
  const int t = g / (2 * Hkv), r = g % (2 * Hkv), which = r / Hkv, h = r % Hkv;
  const bf16_t* src = qkv + (long)t * ld + (long)(Hq + which * Hkv + h) * D + sub * 8;
  bf16_t* dst = (which ? vc : kc) + (((long)slot * Hkv + h) * Lmax + t) * D + sub * 8;
  st16(dst, ld16(src));
}

extern "C" int kf_kv_fill(const void* qkv, long ld, int S, int Hq, int Hkv, int Dh, int slot, void* kc,
                          void* vc, int Lmax, hipStream_t st) {
  if (Dh != D || S > Lmax) return 1;
  if (S == 0) return 0;
  const long threads = (long)S * 2 * Hkv * 16;
  hipLaunchKernelGGL(kv_fill_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                     (const bf16_t*)qkv, ld, S, Hq, Hkv, slot, (bf16_t*)kc, (bf16_t*)vc, Lmax);
  KF_CHECK_LAUNCH();
  return 0;
}
