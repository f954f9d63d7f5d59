// K2: rotary position embedding, in place on the fused QKV activation.
//
// The Llama block produces qkv = x @ Wqkv^T as one [T, (Hq + 2*Hkv) * D] bf16 buffer
// (q heads, then k heads, then v heads). This kernel rotates the first
// (Hq + Hkv) heads of every row in place, using the half-split ("rotate_half")
// pairing (i, i + D/2) and a host-precomputed fp32 cos/sin table [max_pos, D/2]
// (no on-device trig: guide App. B "Element-wise").
//
//   fwd: (x1, x2) -> (x1*c - x2*s, x2*c + x1*s)
//   bwd: (g1, g2) -> (g1*c + g2*s, g2*c - g1*s)      (inverse rotation, sign = -1)
//
// One thread handles 8 pairs = two 16-byte bf16 vectors + two 32-byte table reads.
#include "common.h"

using namespace kf;

__global__ __launch_bounds__(256) void rope_kernel(bf16_t* __restrict__ x, long ld, int rows,
                                                   int nheads, int D, const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t,
                                                   const int* __restrict__ pos, int S, float sign) {
  const int half = D >> 1;
  const int cpr = half >> 3;            // 8-pair chunks per head
  const int per_row = nheads * cpr;
  const int total = per_row * rows;  // host guarantees < 2^31
  for (int it = blockIdx.x * blockDim.x + threadIdx.x; it < total; it += gridDim.x * blockDim.x) {
    const int row = it / per_row;
    const int rem = it - row * per_row;
    const int h = rem / cpr, c = rem - h * cpr;
    const int p = pos ? pos[row] : (row % S);
    bf16_t* px = x + (long)row * ld + (long)h * D + c * 8;
    const float* pc = cos_t + (long)p * half + c * 8;
    const float* ps = sin_t + (long)p * half + c * 8;
    float a[8], b[8], cc[8], ss[8];
    unpack8(ld16(px), a);
    unpack8(ld16(px + half), b);
    f32x4 c0 = ldf4(pc), c1 = ldf4(pc + 4), s0 = ldf4(ps), s1 = ldf4(ps + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { cc[j] = c0[j]; cc[j + 4] = c1[j]; ss[j] = sign * s0[j]; ss[j + 4] = sign * s1[j]; }
    float o1[8], o2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = a[j] * cc[j] - b[j] * ss[j];
      o2[j] = b[j] * cc[j] + a[j] * ss[j];
    }
    st16(px, pack8(o1));
    st16(px + half, pack8(o2));
  }
}

extern "C" int kf_rope(void* x, long ld, int rows, int nheads, int D, const float* cos_t,
                       const float* sin_t, const int* pos, int S, int inverse, hipStream_t s) {
  if (D % 16 != 0 || ld % 8 != 0) return 1;
  if ((long)rows * nheads * (D / 16) >= (1L << 31)) return 2;
  long total = (long)rows * nheads * (D / 16);
  int grid = (int)((total + 255) / 256);
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  rope_kernel<<<grid, 256, 0, s>>>((bf16_t*)x, ld, rows, nheads, D, cos_t, sin_t, pos, S,
                                   inverse ? -1.f : 1.f);
  return 0;
}
