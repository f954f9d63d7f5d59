// HBM read-pattern microbench for the decode GEMM weight stream (round 5): how fast can a
// [N, K] bf16 weight be streamed when each wave-instruction reads
//   rows : 1 KB of ONE row (64 lanes x 16 B contiguous; the GEMV pattern), 4 KB runs per row
//   16x64B: 16 rows x 64 B (lane l: row l & 15, 16-B chunk l >> 4; the MFMA A-operand layout the
//          batched-decode GEMM loads straight into registers), KS instructions back to back
// Every byte is read once per pass; the loads are folded into one word per lane and stored so
// nothing is dead.  Several copies of the weight rotate so every pass streams from HBM.
// run: stream_bench [N K reps]
#include "common.h"

#include <cstdio>
#include <cstdlib>

using namespace kf;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

// work unit = (rows, K segment of SEG 16-B chunks = 4 KB per row); waves stride over units
constexpr int SEG = 256;

// rows: unit = 1 row x SEG chunks, read as 1 KB instructions (64 lanes x 16 B), 4 in flight
__global__ __launch_bounds__(256) void stream_rows(const u32x4* __restrict__ w, int N, int K, u32* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  const int cpr = K / 8, nseg = cpr / SEG;
  u32 acc = 0;
  for (int u = wave; u < N * nseg; u += nw) {
    const u32x4* p = w + (long)(u / nseg) * cpr + (u % nseg) * SEG + lane;
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = p[64 * i];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// 16x64B: unit = 1 KB of each of 16 rows; a wave-instruction reads 16 rows x 64 B (lane: row
// l & 15, chunk l >> 4), KS instructions back to back along the rows (64 KS-byte runs)
template <int KS>
__global__ __launch_bounds__(256) void stream_tiles(const u32x4* __restrict__ w, int N, int K, u32* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  const int cpr = K / 8, nseg = cpr / 64;          // 64 chunks = 1 KB per row per unit
  const int ntile = N / 16;
  u32 acc = 0;
  for (int u = wave; u < ntile * nseg; u += nw) {
    const u32x4* p = w + (long)(16 * (u / nseg) + (lane & 15)) * cpr + (u % nseg) * 64 + (lane >> 4);
#pragma unroll
    for (int c = 0; c < 64; c += 4 * KS) {
      u32x4 v[KS];
#pragma unroll
      for (int i = 0; i < KS; ++i) v[i] = p[c + 4 * i];
#pragma unroll
      for (int i = 0; i < KS; ++i) acc ^= v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3];
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 14336;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const long bytes = (long)N * K * 2;
  // several copies so every rep streams from HBM (MALL is 256 MB)
  const int copies = (int)std::max(2L, (1L << 30) / bytes + 1);
  u32x4* w;
  u32* out;
  CK(hipMalloc(&w, bytes * copies));
  CK(hipMemset(w, 1, bytes * copies));
  CK(hipMalloc(&out, 1 << 24));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("N %d K %d: %.1f MB per pass, %d copies\n", N, K, bytes / 1e6, copies);
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch(w);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch((u32x4*)((char*)w + (i % copies) * bytes));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("%-34s %8.2f us  %6.2f TB/s\n", name, us, bytes / us / 1e6);
  };
  for (int wgs : {256, 512, 1024}) {
    char nm[64];
    snprintf(nm, sizeof nm, "rows 1KB/instr, %d WGs", wgs);
    run(nm, [&](u32x4* p) { hipLaunchKernelGGL(stream_rows, dim3(wgs), dim3(256), 0, 0, p, N, K, out); });
    snprintf(nm, sizeof nm, "16x64B KS=4, %d WGs", wgs);
    run(nm, [&](u32x4* p) { hipLaunchKernelGGL(stream_tiles<4>, dim3(wgs), dim3(256), 0, 0, p, N, K, out); });
    snprintf(nm, sizeof nm, "16x64B KS=8, %d WGs", wgs);
    run(nm, [&](u32x4* p) { hipLaunchKernelGGL(stream_tiles<8>, dim3(wgs), dim3(256), 0, 0, p, N, K, out); });
  }
  return 0;
}
