// Standalone microbench for the K3 flash-attention kernels (no torch): times the forward and
// each backward kernel separately with hipEvents at the Llama-3-8B training shape, and checks
// sampled rows of O, lse, dQ, dK and dV against a float64 CPU reference.  Build variants
// with -D flags on flash_attn_lab.hip, a lab copy of ops/csrc/flash_attn.hip (tools/kbench/build.sh); run: fa_bench [B S Hq Hkv iters].
#include "flash_attn_lab.hip"   // the production kernels plus the measured-and-rejected knobs and stamps
#include "fa_fwd128_lab.hip"    // KFAMD_FA_FWD=128: the 128-key-tile forward
#include "fa_dq128_lab.hip"     // KFAMD_FA_DQ=128: dQ with 128-key stages

#include <cmath>
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

static float hbf(uint16_t v) { return __builtin_bit_cast(float, (u32)v << 16); }

template <typename T>
static std::vector<T> fetch(const void* d, size_t n) {
  std::vector<T> h(n);
  CK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
  return h;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 2, S = argc > 2 ? atoi(argv[2]) : 8192;
  const int Hq = argc > 3 ? atoi(argv[3]) : 32, Hkv = argc > 4 ? atoi(argv[4]) : 8;
  const int iters = argc > 5 ? atoi(argv[5]) : 10;
  const int T = B * S, ldq = (Hq + 2 * Hkv) * D, ldo = Hq * D, G = Hq / Hkv;
  const float scale = 1.f / sqrtf((float)D), sl2 = scale * LOG2E;
  bf16_t *qkv, *o, *dout, *dqkv;
  float *lse, *delta, *dk, *dv;
  CK(hipMalloc(&qkv, (size_t)T * ldq * 2));
  CK(hipMalloc(&dqkv, (size_t)T * ldq * 2));
  CK(hipMalloc(&o, (size_t)T * ldo * 2));
  CK(hipMalloc(&dout, (size_t)T * ldo * 2));
  CK(hipMalloc(&lse, (size_t)B * Hq * S * 4));
  CK(hipMalloc(&delta, (size_t)B * Hq * S * 4));
  CK(hipMalloc(&dk, (size_t)T * Hkv * D * 4));
  CK(hipMalloc(&dv, (size_t)T * Hkv * D * 4));
  init_bf16<<<4096, 256>>>(qkv, (long)T * ldq, 0x1234u, 1.7f);
  init_bf16<<<4096, 256>>>(dout, (long)T * ldo, 0x9876u, 1.0f);
  CK(hipDeviceSynchronize());

  int items = 0, items64 = 0;
  const int g_q = B * Hq * ((S + BQ8 - 1) / BQ8), g_f = B * Hq * ((S + BQ8 - 1) / BQ8);
  for (int kb = 0; kb < S / fb::BKVW; ++kb) items += fb::n_chunks(kb, S, true);
  for (int kb = 0; kb < S / fb2::BKV2; ++kb) items64 += fb2::n_chunks(kb, S, true);
  const int g_kv64 = B * Hkv * items64, g_kv = B * Hkv * items;
  const char* dkv_env = getenv("KFAMD_FA_DKDV");
  const bool use64 = dkv_env && atoi(dkv_env) == 64;
  auto dkdv_run = [&] {
    if (use64)
      flash_bwd_dkdv64_kernel<true><<<g_kv64, 256>>>(qkv, ldq, dout, ldo, lse, delta, dk, dv, B, S, Hq, Hkv, scale, items64);
    else
      flash_bwd_dkdv_kernel<true><<<g_kv, 64 * fb::NWK>>>(qkv, ldq, dout, ldo, lse, delta, dk, dv, B, S, Hq, Hkv, scale, items);
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // flush=1 (argv[6]): overwrite a 1 GB buffer before every timed launch, so the inputs come
  // from HBM as inside a training step (not from the 256 MB MALL / L2 of a hot loop)
  const int flush = argc > 6 ? atoi(argv[6]) : 0;
  char* junk = nullptr;
  if (flush) CK(hipMalloc(&junk, 1L << 30));
  auto timeit = [&](const char* name, double flops, auto&& fn) {
    for (int i = 0; i < 2; ++i) fn();
    CK(hipDeviceSynchronize());
    float ms = 0;
    if (flush) {
      for (int i = 0; i < iters; ++i) {
        CK(hipMemsetAsync(junk, i & 0xff, 1L << 30));
        CK(hipEventRecord(e0));
        fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float one;
        CK(hipEventElapsedTime(&one, e0, e1));
        ms += one;
      }
    } else {
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    ms /= iters;
    printf("%-6s %8.1f us  %6.0f TF\n", name, ms * 1e3, flops / (ms * 1e-3) / 1e12);
    return ms;
  };
  const double mm = 2.0 * B * Hq * (double)S * S / 2 * D;   // FLOPs of one causal [S,S]x[S,D] product
  auto zero = [&] {
    CK(hipMemsetAsync(dk, 0, (size_t)T * Hkv * D * 4));
    CK(hipMemsetAsync(dv, 0, (size_t)T * Hkv * D * 4));
  };
  auto post = [&] {
    const long chunks = (long)T * Hkv * 32;
    flash_bwd_post_kernel<<<(int)std::min<long>((chunks + 255) / 256, 16384), 256>>>(dk, dv, dqkv, ldq, T, Hq, Hkv);
  };
  const char* fwd_env = getenv("KFAMD_FA_FWD");
  const bool fwd128 = fwd_env && atoi(fwd_env) == 128;
  timeit(fwd128 ? "fwd128" : "fwd", 2 * mm, [&] {
    if (fwd128) flash_fwd128_kernel<true><<<g_f, 512>>>(qkv, ldq, o, ldo, lse, B, S, Hq, Hkv, sl2);
    else flash_fwd_kernel<true><<<g_f, 512>>>(qkv, ldq, o, ldo, lse, B, S, Hq, Hkv, sl2);
  });
  CK(hipGetLastError());
  double bwd = 0;
  bwd += timeit("pre", 0, [&] { flash_bwd_pre_kernel<<<(T * Hq + 15) / 16, 256>>>(o, ldo, dout, ldo, delta, B, S, Hq); });
  bwd += timeit(use64 ? "dkdv64" : "dkdv", 4 * mm, dkdv_run);
  const char* dq_env = getenv("KFAMD_FA_DQ");
  const bool dq128 = dq_env && atoi(dq_env) == 128;
  auto dq_run = [&] {
    if (dq128) flash_bwd_dq128_kernel<true><<<g_q, 512>>>(qkv, ldq, dout, ldo, lse, delta, dqkv, ldq, B, S, Hq, Hkv, sl2, scale);
    else flash_bwd_dq_kernel<true><<<g_q, 512>>>(qkv, ldq, dout, ldo, lse, delta, dqkv, ldq, B, S, Hq, Hkv, sl2, scale);
  };
  bwd += timeit(dq128 ? "dq128" : "dq", 3 * mm, dq_run);
  bwd += timeit("post", 0, post);
  // one clean pass for the checks (the timing loops accumulated dK/dV repeatedly)
  zero();
  dkdv_run();
  dq_run();
  post();
  CK(hipDeviceSynchronize());
  printf("bwd_total %8.1f us  %6.0f TF(5-product)\n", bwd * 1e3, 5 * mm / (bwd * 1e-3) / 1e12);
#if KF_FA_STAMPS
  {  // dK/dV phase shares from the diagnostic stamps of the last dK/dV launch (see flash_attn.hip)
    static unsigned long long st[1 << 16][8];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(kf_fa_stamps), sizeof(st)));
    const char* names[5] = {"dma issue", "S/dP chain", "softmax", "dV/dK chain", "barrier"};
    double sum[5] = {0, 0, 0, 0, 0}, tot = 0, its = 0, pro = 0, fl = 0, nw = 0;
    const int waves = std::min(g_kv * fb::NWK, 1 << 16);
    for (int i = 0; i < waves; ++i) {
      if (!st[i][5]) continue;
      its += (double)st[i][5];
      nw += 1;
      pro += (double)st[i][6];
      fl += (double)st[i][7];
      for (int k = 0; k < 5; ++k) { sum[k] += (double)st[i][k]; tot += (double)st[i][k]; }
    }
    printf("dkdv phases (s_memtime, all waves, %.0f iterations):", its);
    for (int k = 0; k < 5; ++k) printf("  %s %.1f%% (%.0f cyc/it)", names[k], 100 * sum[k] / tot, sum[k] / its);
    printf("\ndkdv per work item (wave mean): prologue %.0f cyc, loop %.0f cyc, flush %.0f cyc (%.1f / %.1f %% of the wave's time)\n",
           pro / nw, tot / nw, fl / nw, 100 * pro / (pro + tot + fl), 100 * fl / (pro + tot + fl));
  }
#endif

  // ---- float64 reference on sampled rows
  auto hq = fetch<uint16_t>(qkv, (size_t)T * ldq), hdo = fetch<uint16_t>(dout, (size_t)T * ldo);
  auto ho = fetch<uint16_t>(o, (size_t)T * ldo), hdq = fetch<uint16_t>(dqkv, (size_t)T * ldq);
  auto hl = fetch<float>(lse, (size_t)B * Hq * S);
  auto Q = [&](int b, int t, int h, int d) { return (double)hbf(hq[((size_t)b * S + t) * ldq + h * D + d]); };
  auto K = [&](int b, int t, int hk, int d) { return (double)hbf(hq[((size_t)b * S + t) * ldq + (Hq + hk) * D + d]); };
  auto V = [&](int b, int t, int hk, int d) { return (double)hbf(hq[((size_t)b * S + t) * ldq + (Hq + Hkv + hk) * D + d]); };
  auto dO = [&](int b, int t, int h, int d) { return (double)hbf(hdo[((size_t)b * S + t) * ldo + h * D + d]); };
  // exact softmax row: p[k], lse, o[d], delta
  auto row = [&](int b, int h, int qi, std::vector<double>& p, double& ls, std::vector<double>& orow, double& dl) {
    const int hk = h / G;
    p.assign(qi + 1, 0.0);
    double mx = -1e300;
    for (int k = 0; k <= qi; ++k) {
      double sdot = 0;
      for (int d = 0; d < D; ++d) sdot += Q(b, qi, h, d) * K(b, k, hk, d);
      p[k] = sdot * scale;
      mx = std::max(mx, p[k]);
    }
    double sum = 0;
    for (int k = 0; k <= qi; ++k) { p[k] = exp(p[k] - mx); sum += p[k]; }
    for (int k = 0; k <= qi; ++k) p[k] /= sum;
    ls = mx + log(sum);
    orow.assign(D, 0.0);
    for (int k = 0; k <= qi; ++k)
      for (int d = 0; d < D; ++d) orow[d] += p[k] * V(b, k, hk, d);
    dl = 0;
    for (int d = 0; d < D; ++d) dl += orow[d] * dO(b, qi, h, d);
  };
  double eo = 0, el = 0, edq = 0, mo = 0, mdq = 0;
  u32 rs = 12345;
  auto rnd = [&](int n) { rs = rs * 1664525u + 1013904223u; return (int)((rs >> 8) % (u32)n); };
  std::vector<double> p, orow;
  for (int it = 0; it < 12; ++it) {
    const int b = rnd(B), h = rnd(Hq), qi = it < 2 ? it : rnd(S), hk = h / G;
    double ls, dl;
    row(b, h, qi, p, ls, orow, dl);
    for (int d = 0; d < D; ++d) {
      eo = std::max(eo, fabs(orow[d] - hbf(ho[((size_t)b * S + qi) * ldo + h * D + d])));
      mo = std::max(mo, fabs(orow[d]));
    }
    el = std::max(el, fabs(ls - hl[((size_t)b * Hq + h) * S + qi]));
    std::vector<double> dq(D, 0.0);
    for (int k = 0; k <= qi; ++k) {
      double dp = 0;
      for (int d = 0; d < D; ++d) dp += dO(b, qi, h, d) * V(b, k, hk, d);
      const double ds = p[k] * (dp - dl);
      for (int d = 0; d < D; ++d) dq[d] += ds * K(b, k, hk, d) * scale;
    }
    for (int d = 0; d < D; ++d) {
      edq = std::max(edq, fabs(dq[d] - hbf(hdq[((size_t)b * S + qi) * ldq + h * D + d])));
      mdq = std::max(mdq, fabs(dq[d]));
    }
  }
  // dK / dV rows: sum over the G query heads and every query q >= key
  double edk = 0, edv = 0, mdk = 0, mdv = 0;
  for (int it = 0; it < 3; ++it) {
    const int b = rnd(B), hk = rnd(Hkv), key = it == 0 ? S - 1 : rnd(S);
    std::vector<double> dkr(D, 0.0), dvr(D, 0.0);
    for (int g = 0; g < G; ++g) {
      const int h = hk * G + g;
      for (int qi = key; qi < S; ++qi) {
        double sdot = 0, dp = 0, dl = 0;
        for (int d = 0; d < D; ++d) sdot += Q(b, qi, h, d) * K(b, key, hk, d);
        const double pk = exp(sdot * scale - (double)hl[((size_t)b * Hq + h) * S + qi]);
        for (int d = 0; d < D; ++d) {
          dp += dO(b, qi, h, d) * V(b, key, hk, d);
          dl += hbf(ho[((size_t)b * S + qi) * ldo + h * D + d]) * dO(b, qi, h, d);
        }
        const double ds = pk * (dp - dl);
        for (int d = 0; d < D; ++d) {
          dvr[d] += pk * dO(b, qi, h, d);
          dkr[d] += ds * Q(b, qi, h, d) * scale;
        }
      }
    }
    for (int d = 0; d < D; ++d) {
      edk = std::max(edk, fabs(dkr[d] - hbf(hdq[((size_t)b * S + key) * ldq + (Hq + hk) * D + d])));
      edv = std::max(edv, fabs(dvr[d] - hbf(hdq[((size_t)b * S + key) * ldq + (Hq + Hkv + hk) * D + d])));
      mdk = std::max(mdk, fabs(dkr[d]));
      mdv = std::max(mdv, fabs(dvr[d]));
    }
  }
  printf("err o %.2e (max %.2f)  lse %.2e  dq %.2e (max %.2f)  dk %.2e (max %.2f)  dv %.2e (max %.2f)\n", eo, mo, el,
         edq, mdq, edk, mdk, edv, mdv);
  const bool ok = eo < 0.02 * mo + 1e-3 && el < 3e-3 && edq < 0.02 * mdq + 1e-3 && edk < 0.02 * mdk + 1e-3 &&
                  edv < 0.02 * mdv + 1e-3;
  printf("%s\n", ok ? "NUMERICS OK" : "NUMERICS FAIL");
  return ok ? 0 : 3;
}
