// Shared device helpers for the gfx950 (CDNA4) StableAvatar hot-path kernels.
// Wave = 64 lanes; MFMA fragments follow cdna_hip_programming.md §3 maps.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

#define SA_OK 0
#define SA_ERR_ARG 1
#define SA_ERR_LAUNCH 2

// error mapping used by every extern "C" entry point: never throw across the ABI
#define SA_LAUNCH_CHECK()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return SA_ERR_LAUNCH * 1000 + (int)_e; \
  } while (0)

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

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

__device__ __forceinline__ float gelu_tanh(float x) {
  // 0.5 x (1 + tanh(u)) = x / (1 + exp(-2u)),  u = sqrt(2/pi) (x + 0.044715 x^3)
  // (nn.GELU(approximate='tanh')); 4 VALU + exp2 + rcp per element
  const float c0 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;  // -2 sqrt(2/pi) log2(e)
  const float c1 = c0 * 0.044715f;
  const float e = __builtin_amdgcn_exp2f(x * fmaf(c1, x * x, c0));
  return x * __builtin_amdgcn_rcpf(1.0f + e);
}
typedef __attribute__((ext_vector_type(2))) float f32x2;
// gelu_tanh on a pair: the polynomial and the final product as packed f32 VALU (v_pk_mul / v_pk_fma: two
// elements per instruction), the exp2 / rcp per element -- the same operations, so the same results
__device__ __forceinline__ f32x2 gelu_tanh2(f32x2 x) {
  const float c0 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
  const float c1 = c0 * 0.044715f;
  const f32x2 z = x * __builtin_elementwise_fma((f32x2){c1, c1}, x * x, (f32x2){c0, c0});
  const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(z[0]), __builtin_amdgcn_exp2f(z[1])} + (f32x2){1.0f, 1.0f};
  return x * (f32x2){__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
}
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

// bijective XCD-aware remap of a flat workgroup id (cdna_hip_programming.md §5 "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nx = 8;
  int q = nwg / nx, r = nwg % nx, x = orig % nx;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / nx;
}
