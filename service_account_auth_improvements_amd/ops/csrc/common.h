// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels of this package.
//
// Conventions (all kernels):
//  * bf16 tensors are moved as raw 16-bit patterns (uint16_t) in 16-byte vectors
//    (8 x bf16 per lane) -- hipcc does not auto-vectorise bf16 loads (guide G13).
//  * math is done in fp32; f32 -> bf16 uses the compiler cast, which lowers to
//    v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-preserving).
//  * wave = 64 lanes; block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <stdlib.h>

namespace kf {

typedef uint16_t bf16_t;
typedef uint32_t u32;

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;   // 8 x bf16
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;   // 4 x bf16
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short s16x8;      // MFMA bf16 fragment (8 elems)

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((u32)v) << 16); }
__device__ __forceinline__ float bflo(u32 v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bfhi(u32 v) { return __uint_as_float(v & 0xffff0000u); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
// two floats -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (RNE); the scalar-cast form
// costs a convert per half plus a shift and an or
__device__ __forceinline__ u32 pack2(float lo, float hi) {
  return __builtin_bit_cast(u32, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

// unpack 8 bf16 held in a u32x4 into 8 floats
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[2 * i] = bflo(v[i]); f[2 * i + 1] = bfhi(v[i]); }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2(f[2 * i], f[2 * i + 1]);
  return r;
}

__device__ __forceinline__ u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ void st16(void* p, const u32x4& v) { *reinterpret_cast<u32x4*>(p) = v; }
__device__ __forceinline__ f32x4 ldf4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void stf4(float* p, const f32x4& v) { *reinterpret_cast<f32x4*>(p) = v; }

// ---- wave64 reductions (DPP/ds_swizzle via __shfl_xor over all 64 lanes) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x == NT (multiple of 64); `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT == 64) return v;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float fast_exp(float x) { return __expf(x); }
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace kf

#define KF_CHECK_LAUNCH() (void)hipGetLastError()
