// Decode weight-streaming microbench: MFMA skinny GEMM (ops/csrc/skinny_gemm.hip) vs the VALU
// GEMV (ops/csrc/gemv.hip) at the Llama-3-8B decode shapes, M = 1..4 rows.  Weights rotate
// over >= 1 GB of copies so every launch streams from HBM (not the 256 MB MALL).  Prints
// time, effective TB/s and the max difference between the two kernels' outputs.
#include "../../service_account_auth_improvements_amd/ops/csrc/skinny_gemm.hip"
#include "../../service_account_auth_improvements_amd/ops/csrc/gemv.hip"

#include <cstdio>
#include <vector>
#include <cstdlib>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

__global__ void init_bf16(bf16_t* p, long n, u32 seed, float amp) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    u32 x = (u32)i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
    p[i] = f2bf(((float)(x & 0xffffff) / 8388608.f - 1.f) * amp);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 50;
  struct Shape { const char* name; int N, K, swiglu; };
  const Shape shapes[] = {{"wqkv", 6144, 4096, 0}, {"wo", 4096, 4096, 0}, {"wgu", 14336, 4096, 1},
                          {"wd", 4096, 14336, 0}, {"lm_head", 128256, 4096, 0}};
  bf16_t *x, *res, *nw, *y0, *y1, *h;
  CK(hipMalloc(&x, 4 * 14336 * 2));
  CK(hipMalloc(&res, 4 * 14336 * 2));
  CK(hipMalloc(&nw, 14336 * 2));
  CK(hipMalloc(&h, 4 * 14336 * 2));
  CK(hipMalloc(&y0, 4 * 128256 * 2));
  CK(hipMalloc(&y1, 4 * 128256 * 2));
  init_bf16<<<64, 256>>>(x, 4 * 14336, 0x77u, 1.f);
  init_bf16<<<64, 256>>>(res, 4 * 14336, 0x78u, 1.f);
  init_bf16<<<64, 256>>>(nw, 14336, 0x79u, 1.f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int bad = 0;
  for (const Shape& s : shapes) {
    const long rows = s.swiglu ? 2L * s.N : s.N;
    const long bytes = rows * s.K * 2;
    // GEMV_HOT=1: one copy, re-read every launch (MALL / Infinity-Cache resident)
    const bool hot = getenv("GEMV_HOT") && atoi(getenv("GEMV_HOT"));
    const int copies = hot ? 1 : (int)std::max<long>(1, ((1L << 30) + bytes - 1) / bytes);
    std::vector<bf16_t*> W(copies);
    for (auto& p : W) {
      CK(hipMalloc(&p, bytes));
      init_bf16<<<2048, 256>>>(p, rows * s.K, 0x1234u, 0.05f);
    }
    CK(hipDeviceSynchronize());
    for (int M : {1, 2, 4}) {
      for (int norm = 0; norm < (s.K == 4096 ? 2 : 1); ++norm) {
        auto sk = [&](int c) {
          int rc = norm ? kf_skinny_gemm_norm(x, s.K, M, res, nw, 1e-5f, h, s.K, W[c], s.N, s.K, y0, s.N, s.swiglu, s.N, 0)
                        : kf_skinny_gemm(x, s.K, M, W[c], s.N, s.K, y0, s.N, s.swiglu, s.N, 0);
          if (rc) { fprintf(stderr, "skinny rc %d\n", rc); exit(1); }
        };
        auto gv = [&](int c) {
          int rc = kf_gemv(x, s.K, M, norm ? res : nullptr, norm ? nw : nullptr, 1e-5f, h, s.K, W[c], s.N, s.K, y1,
                           s.N, s.swiglu, s.N, 0);
          if (rc) { fprintf(stderr, "gemv rc %d\n", rc); exit(1); }
        };
        auto time = [&](auto&& fn) {
          for (int i = 0; i < 3; ++i) fn(i % copies);
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0));
          for (int i = 0; i < iters; ++i) fn(i % copies);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          return ms * 1e3 / iters;
        };
        const float us_sk = time(sk), us_gv = time(gv);
        sk(0);
        gv(0);
        CK(hipDeviceSynchronize());
        std::vector<uint16_t> a((size_t)M * s.N), b((size_t)M * s.N);
        CK(hipMemcpy(a.data(), y0, a.size() * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), y1, b.size() * 2, hipMemcpyDeviceToHost));
        double md = 0, mx = 0;
        for (size_t i = 0; i < a.size(); ++i) {
          const double va = __builtin_bit_cast(float, (u32)a[i] << 16), vb = __builtin_bit_cast(float, (u32)b[i] << 16);
          md = std::max(md, std::fabs(va - vb));
          mx = std::max(mx, std::fabs(va));
        }
        const bool ok = md <= 2e-2 * mx + 1e-3;
        bad += !ok;
        printf("%-8s M=%d norm=%d  skinny %7.1f us %5.2f TB/s | gemv %7.1f us %5.2f TB/s | maxdiff %.2e (max %.2e) %s\n",
               s.name, M, norm, us_sk, bytes / us_sk / 1e6, us_gv, bytes / us_gv / 1e6, md, mx, ok ? "" : "MISMATCH");
      }
    }
    for (auto p : W) CK(hipFree(p));
  }
  printf(bad ? "NUMERICS FAIL\n" : "NUMERICS OK\n");
  return bad ? 3 : 0;
}
