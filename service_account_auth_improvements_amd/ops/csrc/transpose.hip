// bf16 matrix transpose out[C, R] = in[R, C]^T through 64 x 64 LDS tiles.
//
// Used to hand hipBLASLt the activation-gradient products dX = dY . W in the same operand
// layout as the forward (x . W^T): with W^T materialised row-major, dX = dY . (W^T)^T runs on
// the faster "A^T B" solutions (1.4-1.5 PF vs 1.1-1.36 PF for dY . W at the Llama-3-8B
// shapes, tools/bench_gemm.py).  The copy streams each weight once per step (~0.14 ms per
// Llama-3-8B layer at HBM rate) and lives only in the caching allocator's scratch.
//
// One workgroup (256 threads) per 64 x 64 tile: every thread loads two 16-byte row pieces
// (coalesced) into a padded LDS tile, then gathers 16 elements of one tile column and writes
// them as two 16-byte pieces of an output row (coalesced).
#include "common.h"

using namespace kf;

namespace {
constexpr int TT = 64, PAD = 2;   // row pitch 66 bf16 = 132 B: column reads spread over banks

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ in, long ldi,
                                                              bf16_t* __restrict__ out, long ldo, int R, int C) {
  __shared__ bf16_t tile[TT][TT + PAD];
  const int r0 = blockIdx.y * TT, c0 = blockIdx.x * TT, t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int piece = t + 256 * k;            // 512 pieces of 8 elements = 64 rows x 8 pieces
    const int rr = piece >> 3, cc = (piece & 7) * 8;
    const u32x4 v = ld16(in + (long)(r0 + rr) * ldi + c0 + cc);
    const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[rr][cc + j] = e[j];
  }
  __syncthreads();
  const int oc = t >> 2, or0 = (t & 3) * 16;   // output row c0 + oc, columns r0 + or0 .. +15
  bf16_t o[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) o[j] = tile[or0 + j][oc];
  bf16_t* dst = out + (long)(c0 + oc) * ldo + r0 + or0;
  st16(dst, *reinterpret_cast<const u32x4*>(o));
  st16(dst + 8, *reinterpret_cast<const u32x4*>(o + 8));
}
}  // namespace

extern "C" int kf_transpose_bf16(const void* in, long ldi, void* out, long ldo, int R, int C, hipStream_t st) {
  if (R % TT || C % TT || ldi % 8 || ldo % 8) return 1;
  if ((((uintptr_t)in) | ((uintptr_t)out)) & 15) return 2;
  if (R == 0 || C == 0) return 0;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3(C / TT, R / TT), dim3(256), 0, st, (const bf16_t*)in, ldi,
                     (bf16_t*)out, ldo, R, C);
  KF_CHECK_LAUNCH();
  return 0;
}
