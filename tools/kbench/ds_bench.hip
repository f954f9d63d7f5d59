// Persistent decode-step microbench (tools/kbench/decode_step_lab.hip = ops/csrc/decode_step.hip
// plus ablation knobs): Llama-3-8B shapes, random weights, L layers, M rows, context C.  Times
// the launch alone with HIP events (no graph, no host sync per step) and prints us / step and
// the weight stream rate.  Usage: ds_bench [L=32] [M=1] [ctx=1024] [iters=20]
#include "decode_step_lab.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

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
  const int L = argc > 1 ? atoi(argv[1]) : 32, M = argc > 2 ? atoi(argv[2]) : 1;
  const int ctx = argc > 3 ? atoi(argv[3]) : 1024, iters = argc > 4 ? atoi(argv[4]) : 20;
  const int V = 128256, lmax = 2048, slots = 4;
  auto alloc = [](long n, u32 seed, float amp) {
    bf16_t* p;
    CK(hipMalloc(&p, n * 2));
    init_bf16<<<4096, 256>>>(p, n, seed, amp);
    return p;
  };
  std::vector<ds::Tab> tab(L);
  long wbytes = 0;
  for (int l = 0; l < L; ++l) {
    tab[l].wqkv = alloc((long)ds::NQKV * ds::H, 11 + l, 0.02f);
    tab[l].wo = alloc((long)ds::H * ds::H, 101 + l, 0.02f);
    tab[l].wgu = alloc(2L * ds::F * ds::H, 201 + l, 0.02f);
    tab[l].wd = alloc((long)ds::H * ds::F, 301 + l, 0.02f);
    tab[l].n1 = alloc(ds::H, 401 + l, 1.f);
    tab[l].n2 = alloc(ds::H, 501 + l, 1.f);
    tab[l].kc = alloc((long)slots * ds::HKV * lmax * ds::HD, 601 + l, 1.f);
    tab[l].vc = alloc((long)slots * ds::HKV * lmax * ds::HD, 701 + l, 1.f);
    wbytes += 2L * ((long)ds::NQKV * ds::H + (long)ds::H * ds::H + 2L * ds::F * ds::H + (long)ds::H * ds::F);
  }
  const bf16_t* embed = alloc((long)V * ds::H, 7, 0.02f);
  const bf16_t* fnorm = alloc(ds::H, 8, 1.f);
  const bf16_t* lm = alloc((long)V * ds::H, 9, 0.02f);
  wbytes += 2L * V * ds::H;
  ds::Tab* dtab;
  CK(hipMalloc(&dtab, sizeof(ds::Tab) * L));
  CK(hipMemcpy(dtab, tab.data(), sizeof(ds::Tab) * L, hipMemcpyHostToDevice));
  std::vector<float> cs(lmax * 64, 1.f), sn(lmax * 64, 0.f);
  float *dcos, *dsin;
  CK(hipMalloc(&dcos, cs.size() * 4));
  CK(hipMalloc(&dsin, sn.size() * 4));
  CK(hipMemcpy(dcos, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsin, sn.data(), sn.size() * 4, hipMemcpyHostToDevice));
  std::vector<long> tok(M, 5);
  std::vector<int> sl(M), ps(M, ctx);
  for (int m = 0; m < M; ++m) sl[m] = m;
  long* dtok;
  int *dsl, *dps;
  CK(hipMalloc(&dtok, 8 * M));
  CK(hipMalloc(&dsl, 4 * M));
  CK(hipMalloc(&dps, 4 * M));
  CK(hipMemcpy(dtok, tok.data(), 8 * M, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsl, sl.data(), 4 * M, hipMemcpyHostToDevice));
  CK(hipMemcpy(dps, ps.data(), 4 * M, hipMemcpyHostToDevice));
  const long wsb = kf_decode_step_ws_bytes();
  void* ws;
  CK(hipMalloc(&ws, wsb));
  CK(hipMemset(ws, 0, wsb));
  bf16_t* logits;
  CK(hipMalloc(&logits, (long)M * V * 2));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&]() {
    const int rc = kf_decode_step(dtab, L, M, ds::H, ds::F, ds::HQ, ds::HKV, ds::HD, V, embed, fnorm, lm, dcos, dsin,
                                  dtok, dsl, dps, lmax, 1e-5f, 0.0883883f, ws, logits, 0);
    if (rc) { fprintf(stderr, "rc %d\n", rc); exit(1); }
  };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  int err = 0;
  CK(hipMemcpy(&err, (char*)ws + kf_decode_step_err_offset(), 4, hipMemcpyDeviceToHost));
  const double us = 1e3 * ms / iters;
  printf("ds L=%d M=%d ctx=%d: %.1f us/step  %.2f TB/s weights  err=%d\n", L, M, ctx, us, wbytes / (us * 1e-6) / 1e12, err);
  return err ? 2 : 0;
}
