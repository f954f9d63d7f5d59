// v_dot2c_f32_bf16 semantics probe: prints dot2(a, b, c) for a few packed bf16 pairs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
__global__ void k(const unsigned* a, const unsigned* b, const float* c, float* o) {
  int i = threadIdx.x;
  o[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a[i]), __builtin_bit_cast(bf16x2, b[i]), c[i], false);
}
static unsigned bf(float f) { unsigned u; memcpy(&u, &f, 4); return u >> 16; }
int main() {
  const int n = 4;
  float av[n][2] = {{1, 2}, {3, -1}, {0.5f, 0.25f}, {1, 0}}, bv[n][2] = {{1, 1}, {2, 2}, {4, 8}, {0, 1}}, cv[n] = {0, 1, 0, 10};
  unsigned ha[n], hb[n];
  for (int i = 0; i < n; ++i) { ha[i] = bf(av[i][0]) | (bf(av[i][1]) << 16); hb[i] = bf(bv[i][0]) | (bf(bv[i][1]) << 16); }
  unsigned *da, *db; float *dc, *dout;
  hipMalloc(&da, 64); hipMalloc(&db, 64); hipMalloc(&dc, 64); hipMalloc(&dout, 64);
  hipMemcpy(da, ha, 16, hipMemcpyHostToDevice); hipMemcpy(db, hb, 16, hipMemcpyHostToDevice); hipMemcpy(dc, cv, 16, hipMemcpyHostToDevice);
  k<<<1, n>>>(da, db, dc, dout);
  float o[n]; hipMemcpy(o, dout, 16, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) printf("a=(%g,%g) b=(%g,%g) c=%g -> %g (expect %g)\n", av[i][0], av[i][1], bv[i][0], bv[i][1], cv[i], o[i], av[i][0]*bv[i][0]+av[i][1]*bv[i][1]+cv[i]);
  return 0;
}
