// A/B microbench: the production dK/dV kernel (ops/csrc/flash_attn.hip) against the one-wave-
// per-SIMD pipelined candidate (fa_dkdv2_lab.hip), same inputs, alternating timed rounds, and
// float64 checks of sampled dK / dV rows from BOTH (plus the production forward / dQ for the
// reference inputs).  run: fa2_bench [B S Hq Hkv iters flush rounds]
#include "fa_dkdv2_lab.hip"

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

  int items = 0;
  const int g_q = B * Hq * ((S + BQ8 - 1) / BQ8), g_f = g_q;
  for (int kb = 0; kb < S / fb::BKVW; ++kb) items += fb::n_chunks(kb, S, true);
  const int g_kv = B * Hkv * items;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int flush = argc > 6 ? atoi(argv[6]) : 1;
  const int rounds = argc > 7 ? atoi(argv[7]) : 3;
  char* junk = nullptr;
  if (flush) CK(hipMalloc(&junk, 1L << 30));
  auto timeit = [&](auto&& fn) {
    for (int i = 0; i < 2; ++i) fn();
    CK(hipDeviceSynchronize());
    float ms = 0;
    for (int i = 0; i < iters; ++i) {
      if (flush) CK(hipMemsetAsync(junk, i & 0xff, 1L << 30));
      CK(hipEventRecord(e0));
      fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float one;
      CK(hipEventElapsedTime(&one, e0, e1));
      ms += one;
    }
    return ms / iters;
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
  auto dkdv_prod = [&] {
    flash_bwd_dkdv_kernel<true><<<g_kv, 64 * fb::NWK>>>(qkv, ldq, dout, ldo, lse, delta, dk, dv, B, S, Hq, Hkv, scale, items);
  };
  auto dkdv_new = [&] {
    if (kf_flash_bwd_dkdv2(qkv, ldq, dout, ldo, lse, delta, dk, dv, B, S, Hq, Hkv, scale, 1, 0)) { fprintf(stderr, "dkdv2 rc\n"); exit(1); }
  };
  flash_fwd_kernel<true><<<g_f, 512>>>(qkv, ldq, o, ldo, lse, B, S, Hq, Hkv, sl2);
  flash_bwd_pre_kernel<<<(T * Hq + 15) / 16, 256>>>(o, ldo, dout, ldo, delta, B, S, Hq);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r) {
    const float a = timeit(dkdv_prod), b2 = timeit(dkdv_new);
    printf("round %d  dkdv %8.1f us %6.0f TF   dkdv2 %8.1f us %6.0f TF   ratio %.3f\n", r, a * 1e3, 4 * mm / (a * 1e-3) / 1e12,
           b2 * 1e3, 4 * mm / (b2 * 1e-3) / 1e12, a / b2);
  }
  CK(hipGetLastError());
  // numerics: dK/dV of each kernel (fresh accumulators), dQ from the production kernel
  std::vector<float> dk_ref, dv_ref;
  zero();
  dkdv_prod();
  CK(hipDeviceSynchronize());
  dk_ref = fetch<float>(dk, (size_t)T * Hkv * D);
  dv_ref = fetch<float>(dv, (size_t)T * Hkv * D);
  zero();
  dkdv_new();
  flash_bwd_dq_kernel<true><<<g_q, 512>>>(qkv, ldq, dout, ldo, lse, delta, dqkv, ldq, B, S, Hq, Hkv, sl2, scale);
  post();
  CK(hipDeviceSynchronize());
  {
    auto dk2 = fetch<float>(dk, (size_t)T * Hkv * D), dv2 = fetch<float>(dv, (size_t)T * Hkv * D);
    double mk = 0, mv = 0, ek = 0, ev = 0;
    for (size_t i = 0; i < dk2.size(); ++i) {
      mk = std::max(mk, (double)fabs(dk_ref[i]));
      mv = std::max(mv, (double)fabs(dv_ref[i]));
      ek = std::max(ek, (double)fabs(dk2[i] - dk_ref[i]));
      ev = std::max(ev, (double)fabs(dv2[i] - dv_ref[i]));
    }
    printf("dkdv2 vs production (fp32 accumulators, every element): dk %.2e (max %.2f)  dv %.2e (max %.2f)\n", ek, mk, ev, mv);
    // where the differences sit: by 32-key group of the 256-key block (wave w, group g = 2w+g) and by block
    double byg_k[8] = {0}, byg_v[8] = {0}, byb_v[64] = {0};
    for (size_t i = 0; i < dk2.size(); ++i) {
      const long row = (long)(i / (Hkv * D));
      const int key = (int)(row % S), grp = (key % 256) / 32, kb = key / 256;
      byg_k[grp] = std::max(byg_k[grp], (double)fabs(dk2[i] - dk_ref[i]));
      byg_v[grp] = std::max(byg_v[grp], (double)fabs(dv2[i] - dv_ref[i]));
      if (kb < 64) byb_v[kb] = std::max(byb_v[kb], (double)fabs(dv2[i] - dv_ref[i]));
    }
    printf("by 32-key group  dk:");
    for (int g = 0; g < 8; ++g) printf(" %.1e", byg_k[g]);
    printf("\nby 32-key group  dv:");
    for (int g = 0; g < 8; ++g) printf(" %.1e", byg_v[g]);
    printf("\nby key block     dv:");
    for (int k = 0; k < S / 256 && k < 64; ++k) printf(" %.1e", byb_v[k]);
    printf("\n");
    if (!(ek < 0.01 * mk && ev < 0.01 * mv)) { printf("NUMERICS FAIL (vs production)\n"); return 3; }
  }

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
