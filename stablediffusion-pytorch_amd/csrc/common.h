// Shared device helpers for the gfx950 (MI355X, CDNA4) latent-diffusion kernels.
// bf16 is carried as raw uint16 bits; every conversion is explicit round-to-nearest-even.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launch.h"

typedef uint16_t bf16_t;
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define SDMI_LDS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// round-to-nearest-even fp32 -> bf16 on the hardware converter (v_cvt_pk_bf16_f32; NaN stays NaN)
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// two floats -> packed bf16x2 in ONE v_cvt_pk_bf16_f32 (a in the low half)
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// IEEE fp32 operations that the compiler may not fuse into FMAs (HIP compiles with fp-contract=fast; the
// header intrinsics __fmul_rn / __fadd_rn are plain contractible operators). Used where results must be
// bit-identical to the reference's eager fp32 ops (scheduler arithmetic).
__device__ __forceinline__ float mul_ieee(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float add_ieee(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float sub_ieee(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}

// raw v_exp_f32 (2^x): the libm exp2f adds a denormal-range fix-up (compare, 2 selects, add, ldexp) around it,
// 5 extra VALU ops per element that softmax / sigmoid never need (2^x below 2^-126 contributes nothing)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// raw v_rcp_f32 (1 ulp): replaces the ~10-instruction correctly rounded division where results are rounded to bf16
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float silu_f(float x) { return x * fast_rcp(1.0f + fast_exp2(-x * kLog2e)); }

// d/dx silu(x) = s(x) * (1 + x * (1 - s(x)))
__device__ __forceinline__ float silu_grad_f(float x) {
  float s = fast_rcp(1.0f + fast_exp2(-x * kLog2e));
  return s * (1.0f + x * (1.0f - s));
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2bf(f[0], f[1]); r.y = pack2bf(f[2], f[3]);
  r.z = pack2bf(f[4], f[5]); r.w = pack2bf(f[6], f[7]);
  return r;
}

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

// Division of a non-negative int (< 2^31) by a runtime constant d >= 1 with one multiply-high and a shift:
// m = ceil(2^(31+s) / d), s = ceil(log2 d) -> n / d = umulhi(n, m) >> (s - 1) exactly for every n < 2^31
// (m * d - 2^(31+s) < d and 2^-s <= 1/d bound the error below one); d == 1 is m = 0 (identity).
// Conv pixel grids of any size (the reference only requires H, W divisible by the down-sampling,
// utils/config_utils.py:30-31: MNIST's 28x28 -> 7x7 latents) decompose without a hardware divide.
struct FastDiv {
  unsigned m;    // 0: d == 1
  unsigned dsh;  // d | (s - 1) << 24  (d < 2^24)
  __device__ __forceinline__ unsigned div(unsigned n) const { return m ? (__umulhi(n, m) >> (dsh >> 24)) : n; }
  __host__ __device__ __forceinline__ int d() const { return (int)(dsh & 0xFFFFFFu); }
  static FastDiv make(int d) {
    FastDiv f;
    if (d <= 1) {
      f.m = 0;
      f.dsh = 1;
      return f;
    }
    int s = 0;
    while ((1LL << s) < d) ++s;
    f.m = (unsigned)(((1ULL << (31 + s)) + (unsigned long long)d - 1) / (unsigned long long)d);
    f.dsh = (unsigned)d | ((unsigned)(s - 1) << 24);
    return f;
  }
};

#define SDMI_CHECK_LAUNCH()                                  \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return (int)_e;                    \
  } while (0)
