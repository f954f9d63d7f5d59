// K7: embedding gather (forward) and deterministic scatter-add (backward), vocab-parallel aware.
//
// Forward: one wave per token row; H bf16 = H/8 16-byte chunks, lane-strided (fully coalesced),
// rows whose id falls outside this rank's vocab shard [vstart, vstart + vl) are zero (the TP
// all-reduce then sums the shards).
// Backward: the caller sorts the token ids once (rocprim radix sort via torch.sort), so equal
// ids are adjacent; one wave per sorted position i that STARTS a run sums the run's gradient
// rows in fp32 in a fixed order and writes (or accumulates into) the bf16 gradient row -- no
// atomics, bit-reproducible, and every embedding row is written by exactly one wave.  Rows of
// ids that do not occur are zeroed by the caller only when not accumulating.
#include "common.h"

using namespace kf;

__global__ __launch_bounds__(256) void embed_fwd_kernel(const long* __restrict__ tok, const bf16_t* __restrict__ E,
                                                        bf16_t* __restrict__ out, int T, int H, long vstart,
                                                        long vl) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= T) return;
  const long id = tok[row] - vstart;
  const bool in = id >= 0 && id < vl;
  bf16_t* o = out + (long)row * H;
  const bf16_t* e = E + (in ? id : 0) * (long)H;
  for (int c = lane; c < H / 8; c += 64) st16(o + c * 8, in ? ld16(e + c * 8) : u32x4{0, 0, 0, 0});
}

__global__ __launch_bounds__(256) void embed_bwd_kernel(const long* __restrict__ sorted, const long* __restrict__ perm,
                                                        const bf16_t* __restrict__ g, bf16_t* __restrict__ dE,
                                                        int T, int H, long vstart, long vl, int accumulate) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= T) return;
  const long id = sorted[i];
  if (i > 0 && sorted[i - 1] == id) return;          // not the start of a run
  const long loc = id - vstart;
  if (loc < 0 || loc >= vl) return;                   // another TP rank's vocab shard
  int end = i + 1;
  while (end < T && sorted[end] == id) ++end;
  bf16_t* dst = dE + loc * (long)H;
  for (int c = lane; c < H / 8; c += 64) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = i; j < end; ++j) {
      float v[8];
      unpack8(ld16(g + perm[j] * (long)H + c * 8), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
    if (accumulate) {
      float old[8];
      unpack8(ld16(dst + c * 8), old);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += old[k];
    }
    st16(dst + c * 8, pack8(acc));
  }
}

extern "C" int kf_embed_fwd(const long* tok, const void* E, void* out, int T, int H, long vstart, long vl,
                            hipStream_t s) {
  if (H % 8 != 0) return 1;
  if (T == 0) return 0;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(cdiv(T, 4)), dim3(256), 0, s, tok, (const bf16_t*)E, (bf16_t*)out, T,
                     H, vstart, vl);
  KF_CHECK_LAUNCH();
  return 0;
}

extern "C" int kf_embed_bwd(const long* sorted, const long* perm, const void* g, void* dE, int T, int H, long vstart,
                            long vl, int accumulate, hipStream_t s) {
  if (H % 8 != 0) return 1;
  if (T == 0) return 0;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(cdiv(T, 4)), dim3(256), 0, s, sorted, perm, (const bf16_t*)g,
                     (bf16_t*)dE, T, H, vstart, vl, accumulate);
  KF_CHECK_LAUNCH();
  return 0;
}
