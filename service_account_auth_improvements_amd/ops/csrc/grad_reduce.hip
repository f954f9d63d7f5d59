// fp32 data-parallel gradient reduction and micro-batch accumulation (C1, ZeRO-1).
//
// Why not an fp32 reduce-scatter: it doubles the bytes on xGMI.  A bf16 ring
// reduce-scatter instead rounds every partial sum to bf16 (N-1 roundings per element).
// The ZeRO-1 reducer therefore moves each bucket with an all-to-all of its bf16 shards
// -- the same bytes per GPU as a bf16 reduce-scatter, and on the fully connected 8-GPU
// xGMI mesh every shard travels its own point-to-point link -- and this kernel sums
// the N received shards in fp32 in a fixed rank order (bitwise deterministic), writing
// the fp32 gradient shard that AdamW consumes directly.  Each element is rounded to bf16
// once (by its producer on its own rank) and never again.
//
// Micro-batch accumulation (grad_accum > 1) runs in an fp32 main-gradient buffer instead
// of bf16 beta=1 GEMM accumulation: after each micro-batch main (+)= grads; the last one
// is folded as grads = bf16(main + grads) right before its bucket is sent (one rounding),
// or main += grads when the fp32 buffer itself is the optimizer's operand.
#include "common.h"

using namespace kf;

// out[i] (+)= sum_{r < R} in[r * n + i]   (bf16 in, fp32 out, r ascending)
__global__ __launch_bounds__(256) void shard_sum_kernel(const bf16_t* __restrict__ in, int R, size_t n,
                                                        size_t nvec, float* __restrict__ out, int accumulate) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t e = i * 8;
    float acc[8];
    if (accumulate) {
      f32x4 a = ldf4(out + e), b = ldf4(out + e + 4);
      acc[0] = a[0]; acc[1] = a[1]; acc[2] = a[2]; acc[3] = a[3];
      acc[4] = b[0]; acc[5] = b[1]; acc[6] = b[2]; acc[7] = b[3];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    }
    for (int r = 0; r < R; ++r) {
      float f[8];
      unpack8(ld16(in + (size_t)r * n + e), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    stf4(out + e, f32x4{acc[0], acc[1], acc[2], acc[3]});
    stf4(out + e + 4, f32x4{acc[4], acc[5], acc[6], acc[7]});
  }
}

// mode 0: main = g; 1: main += g; 2: g = bf16(main + g)
__global__ __launch_bounds__(256) void grad_accum_kernel(float* __restrict__ main_, bf16_t* __restrict__ g,
                                                         size_t nvec, int mode) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t e = i * 8;
    float f[8];
    unpack8(ld16(g + e), f);
    if (mode == 0) {
      stf4(main_ + e, f32x4{f[0], f[1], f[2], f[3]});
      stf4(main_ + e + 4, f32x4{f[4], f[5], f[6], f[7]});
      continue;
    }
    f32x4 a = ldf4(main_ + e), b = ldf4(main_ + e + 4);
    float s[8] = {a[0] + f[0], a[1] + f[1], a[2] + f[2], a[3] + f[3],
                  b[0] + f[4], b[1] + f[5], b[2] + f[6], b[3] + f[7]};
    if (mode == 1) {
      stf4(main_ + e, f32x4{s[0], s[1], s[2], s[3]});
      stf4(main_ + e + 4, f32x4{s[4], s[5], s[6], s[7]});
    } else {
      st16(g + e, pack8(s));
    }
  }
}

static int grid_for(size_t nvec) {
  size_t grid = (nvec + 255) / 256;
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  return (int)grid;
}

extern "C" {

int kf_shard_sum(const void* in, int R, size_t n, float* out, int accumulate, hipStream_t s) {
  if (n % 8 || R < 1) return 1;
  const size_t nvec = n / 8;
  shard_sum_kernel<<<grid_for(nvec), 256, 0, s>>>((const bf16_t*)in, R, n, nvec, out, accumulate);
  return 0;
}

int kf_grad_accum(float* main_, void* g, size_t n, int mode, hipStream_t s) {
  if (n % 8 || mode < 0 || mode > 2) return 1;
  const size_t nvec = n / 8;
  grad_accum_kernel<<<grid_for(nvec), 256, 0, s>>>(main_, (bf16_t*)g, nvec, mode);
  return 0;
}
}
