// K5: fused softmax cross-entropy over bf16 logits, gradient written IN PLACE.
//
// With 288 GB of HBM the full [T, V] logits of Llama-3 (V = 128256, 2.1 GB bf16 per
// 8k tokens) stay resident, so the LM head is one hipBLASLt GEMM and this kernel makes
// exactly two streaming passes over each row (the second one mostly from L2):
//   pass 1: online (max, sum-exp) over the row, 8 x bf16 per 16-byte load
//   pass 2: dlogits = (softmax - onehot(label)) * scale, stored over the logits
// One 256-thread block per row.  Rows whose label == ignore_index get loss 0, grad 0.
//
// Vocab-parallel (TP) use splits the work: mode STATS returns each shard's
// (max, sumexp, target logit) so the caller can all-reduce them over the TP group, then
// mode GRAD writes the gradient with the global log-sum-exp.
#include "common.h"

using namespace kf;

enum { CE_FUSED = 0, CE_STATS = 1, CE_GRAD = 2 };

__device__ __forceinline__ void ms_combine(float& m, float& s, float mo, float so) {
  const float mn = fmaxf(m, mo);
  if (mn == -INFINITY) { m = mn; s = 0.f; return; }
  s = s * __expf(m - mn) + so * __expf(mo - mn);
  m = mn;
}

template <int MODE>
__global__ __launch_bounds__(256) void ce_kernel(bf16_t* __restrict__ logits, long ld, int V,
                                                 const long* __restrict__ labels, long vocab_start,
                                                 long ignore_index, float* __restrict__ loss,
                                                 float* __restrict__ lse_io, float* __restrict__ stat_m,
                                                 float* __restrict__ stat_s, float* __restrict__ stat_xy,
                                                 const float* __restrict__ scale_ptr, float scale_h) {
  __shared__ float red_m[4], red_s[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  bf16_t* x = logits + (long)row * ld;
  const long label = labels[row];
  const bool ignored = (label == ignore_index);
  const long loc = label - vocab_start;            // target column inside this shard
  const int nv = V >> 3;
  float lse;
  if (MODE != CE_GRAD) {
    float m = -INFINITY, s = 0.f;
    for (int v = tid; v < nv; v += 256) {
      float f[8];
      unpack8(ld16(x + v * 8), f);
      float vm = f[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) vm = fmaxf(vm, f[j]);
      if (vm > m) { s *= __expf(m - vm); m = vm; }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(f[j] - m);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
      ms_combine(m, s, mo, so);
    }
    if (lane == 0) { red_m[wv] = m; red_s[wv] = s; }
    __syncthreads();
    m = red_m[0]; s = red_s[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) ms_combine(m, s, red_m[k], red_s[k]);
    const float xy = (loc >= 0 && loc < V) ? bf2f(x[loc]) : 0.f;
    if (MODE == CE_STATS) {
      if (tid == 0) { stat_m[row] = m; stat_s[row] = s; stat_xy[row] = xy; }
      return;
    }
    lse = m + __logf(s);
    if (tid == 0) {
      lse_io[row] = lse;
      loss[row] = ignored ? 0.f : (lse - xy);
    }
    __syncthreads();  // all lanes have read x[loc] before pass 2 overwrites it
  } else {
    lse = lse_io[row];
  }
  // pass 2: gradient in place
  const float scale = ignored ? 0.f : (scale_ptr ? scale_ptr[0] : scale_h);
  for (int v = tid; v < nv; v += 256) {
    float f[8];
    unpack8(ld16(x + v * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(f[j] - lse);
      if ((long)(v * 8 + j) == loc) p -= 1.f;
      f[j] = p * scale;
    }
    st16(x + v * 8, pack8(f));
  }
}

extern "C" int kf_cross_entropy(void* logits, long ld, int rows, int V, const long* labels,
                                long vocab_start, long ignore_index, float* loss, float* lse,
                                float* stat_m, float* stat_s, float* stat_xy,
                                const float* scale_ptr, float scale_h, int mode, hipStream_t s) {
  if (V % 8 || ld % 8) return 1;
  if (rows == 0) return 0;
  switch (mode) {
    case CE_FUSED:
      ce_kernel<CE_FUSED><<<rows, 256, 0, s>>>((bf16_t*)logits, ld, V, labels, vocab_start,
                                               ignore_index, loss, lse, stat_m, stat_s, stat_xy,
                                               scale_ptr, scale_h);
      break;
    case CE_STATS:
      ce_kernel<CE_STATS><<<rows, 256, 0, s>>>((bf16_t*)logits, ld, V, labels, vocab_start,
                                               ignore_index, loss, lse, stat_m, stat_s, stat_xy,
                                               scale_ptr, scale_h);
      break;
    case CE_GRAD:
      ce_kernel<CE_GRAD><<<rows, 256, 0, s>>>((bf16_t*)logits, ld, V, labels, vocab_start,
                                              ignore_index, loss, lse, stat_m, stat_s, stat_xy,
                                              scale_ptr, scale_h);
      break;
    default:
      return 2;
  }
  return 0;
}
