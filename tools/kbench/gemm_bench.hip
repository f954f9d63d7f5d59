// Standalone microbench for the dW GEMM (ops/csrc/gemm.hip) at the Llama-3-8B training shapes
// (K = 32768 tokens = micro-batch 4 x 8192 by default): C[M,N] = A^T B with A [K, M], B [K, N].  Prints per-shape time, TFLOP/s
// and a checksum so build variants (-D flags) can be compared.  Run: gemm_bench [iters].
#include "gemm_lab.hip"   // production kernel + lab variants (KF_GEMM_IMPL=4: 4-wave tn4)

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

__global__ void init_bf16(bf16_t* p, long n, u32 seed, float amp) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    u32 x = (u32)i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
    p[i] = f2bf(((float)(x & 0xffffff) / 8388608.f - 1.f) * amp);
  }
}

// full-matrix checksum: sum_i C[i] * (i % 7 + 1) in double (per-thread partials, one atomic per block)
__global__ void checksum(const bf16_t* c, long n, double* out) {
  double acc = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += (double)bf2f(c[i]) * (double)(i % 7 + 1);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const int K = argc > 2 ? atoi(argv[2]) : 32768;
  const int impl = getenv("KF_GEMM_IMPL") ? atoi(getenv("KF_GEMM_IMPL")) : 8;
  printf("impl %d\n", impl);
  struct Shape { const char* name; int M, N; };
  const Shape shapes[] = {{"wqkv", 6144, 4096}, {"wo", 4096, 4096}, {"wgu", 28672, 4096},
                          {"wd", 4096, 14336}, {"lm_head", 128256, 4096}};
  bf16_t *A, *B, *C;
  CK(hipMalloc(&A, (size_t)K * 128256 * 2));
  CK(hipMalloc(&B, (size_t)K * 14336 * 2));
  CK(hipMalloc(&C, (size_t)128256 * 4096 * 2));
  init_bf16<<<4096, 256>>>(A, (long)K * 128256, 0x1111u, 1.f);
  init_bf16<<<4096, 256>>>(B, (long)K * 14336, 0x2222u, 1.f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double tot_ms = 0, tot_fl = 0;
  for (const Shape& s : shapes) {
    auto run = [&] {
      const int rc = impl == 4 ? kf_gemm_tn4(A, s.M, B, s.N, C, s.N, s.M, s.N, K, 0, 0)
                               : kf_gemm_tn(A, s.M, B, s.N, C, s.N, s.M, s.N, K, 0, 0);
      if (rc) { fprintf(stderr, "bad shape\n"); exit(1); }
    };
    for (int i = 0; i < 3; ++i) run();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) run();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    const double fl = 2.0 * s.M * s.N * K;
    const double mult = strcmp(s.name, "lm_head") ? 32 : 1;
    tot_ms += mult * ms;
    tot_fl += mult * fl;
    double* dcs;
    CK(hipMalloc(&dcs, 8));
    CK(hipMemset(dcs, 0, 8));
    checksum<<<1024, 256>>>(C, (long)s.M * s.N, dcs);
    double cs = 0;
    CK(hipMemcpy(&cs, dcs, 8, hipMemcpyDeviceToHost));
    CK(hipFree(dcs));
    printf("%-8s M=%6d N=%6d  %8.3f ms  %6.0f TF  chk %.6e\n", s.name, s.M, s.N, ms, fl / (ms * 1e-3) / 1e12, cs);
  }
  printf("dW per step: %.1f ms  %.0f TF\n", tot_ms, tot_fl / (tot_ms * 1e-3) / 1e12);
  return 0;
}
