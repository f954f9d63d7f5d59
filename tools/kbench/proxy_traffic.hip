// Stand-in for RCCL's channel kernels during a data-parallel step, on ONE GPU
// (tools/dp8_overlap_proxy.py).
//
// At N = 8 a ZeRO-1 step moves ~28 GB per GPU over xGMI: the bucketed all-to-all of the bf16
// gradients while backward runs, the bf16 parameter all-gather while the next forward runs.
// RCCL does that with one workgroup per channel, resident on the CUs the step's GEMMs and
// attention also need, for as long as the transfer takes at LINK speed.  This kernel holds
// `blocks` workgroups for that long: each copies its share of the bucket through HBM in 64-KB
// pieces (the sender's read and the receiver's write land in HBM on a real node too) and paces
// the pieces to the modelled link rate with s_sleep against the 100-MHz real-time counter, so
// both the CU occupancy and the HBM traffic have the real transfer's shape.  Built as a
// tools-only shared library (never part of the production extension):
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC proxy_traffic.hip -o bin/libproxy_traffic.so
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int NT = 256;          // threads per workgroup (an RCCL channel runs 256-512)
constexpr int PIECE = 65536;     // bytes per paced piece
constexpr int U = 8;             // 16-B loads in flight per thread (32 KB per workgroup), as a channel
                                 // kernel keeps many outstanding: ~15-20 GB/s per workgroup

__global__ __launch_bounds__(NT) void proxy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                    long bytes_per_block, long ticks_per_piece) {
  // the LDS an RCCL channel kernel reserves for its FIFOs; keeps the co-residency realistic
  __shared__ uint4 fifo[2048];   // 32 KB
  const long n16 = bytes_per_block / 16, p16 = PIECE / 16;
  const uint4* s = src + blockIdx.x * n16;
  uint4* d = dst + blockIdx.x * n16;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  long piece = 0;
  for (long base = 0; base < n16; base += p16, ++piece) {
    const long end = base + p16 < n16 ? base + p16 : n16;
    long i0 = base + threadIdx.x;
    for (; i0 + (long)(U - 1) * NT < end; i0 += (long)NT * U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = s[i0 + (long)u * NT];
#pragma unroll
      for (int u = 0; u < U; ++u) d[i0 + (long)u * NT] = v[u];
    }
    for (; i0 < end; i0 += NT) d[i0] = s[i0];
    fifo[threadIdx.x] = s[base];    // the FIFO reservation stays live (read below, never taken)
    if (ticks_per_piece < 0) d[base] = fifo[threadIdx.x ^ 1];
    // pace: piece k may finish no earlier than t0 + (k + 1) * ticks_per_piece
    const uint64_t due = t0 + (uint64_t)(piece + 1) * (uint64_t)ticks_per_piece;
    while (__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(8);
  }
}
}  // namespace

// Move `bytes` (a multiple of 16 x blocks) from src to dst with `blocks` workgroups, paced so the
// whole transfer takes bytes / rate_gbs (GB/s) -- one modelled collective.  Returns 0 on launch.
extern "C" int proxy_traffic(const void* src, void* dst, long bytes, int blocks, double rate_gbs, void* stream) {
  if (blocks < 1 || bytes <= 0 || bytes % (16L * blocks) != 0 || rate_gbs <= 0) return 1;
  const long per_block = bytes / blocks;
  const double seconds_per_piece = (double)PIECE * blocks / (rate_gbs * 1e9);
  const long ticks = (long)(seconds_per_piece * 1e8);   // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(proxy_kernel, dim3(blocks), dim3(NT), 0, (hipStream_t)stream, (const uint4*)src, (uint4*)dst,
                     per_block, ticks > 0 ? ticks : 1);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
