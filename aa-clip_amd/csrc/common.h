// Shared device helpers for the AA-CLIP gfx950 kernels.
// Wave = 64 lanes (CDNA); every reduction below is written for 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/aaclip.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(8))) short short8_t;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(4))) float float4_t;
typedef __attribute__((ext_vector_type(2))) float float2_t;

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

// ---------------------------------------------------------------- bf16 <-> f32
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// round-to-nearest-even; a plain cast lowers to v_cvt_pk_bf16_f32 on gfx950
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
// one v_cvt_pk_bf16_f32 (RNE) for the pair; the scalar form costs 2 cvt + shift + or
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2v_t));
}

// ---------------------------------------------------------------- fp16 <-> f32
// fp16 (IEEE binary16, 11 significant bits) is the parity-grade 16-bit storage:
// same MFMA rate as bf16 (v_mfma_f32_16x16x32_f16), 8x finer rounding. One
// v_cvt_pk_f16_f32 (RNE) per pair on gfx950.
__device__ __forceinline__ float f16_to_f32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f32_to_f16(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
__device__ __forceinline__ uint32_t pack_f16x2(float lo, float hi) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef _Float16 f16x2v_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, f16x2v_t));
}

// 16-bit storage flavour chosen at compile time: H16 = false -> bf16, true -> fp16
template <bool H16>
__device__ __forceinline__ uint32_t pack_h16x2(float lo, float hi) {
  if constexpr (H16) return pack_f16x2(lo, hi);
  else return pack_bf16x2(lo, hi);
}
template <bool H16>
__device__ __forceinline__ float h16_to_f32(uint16_t h) {
  if constexpr (H16) return f16_to_f32(h);
  else return bf16_to_f32(h);
}
template <bool H16>
using h16x8_t = typename std::conditional<H16, f16x8_t, bf16x8_t>::type;
template <bool H16>
using h16_t = typename std::conditional<H16, _Float16, __bf16>::type;

// C^T-tile MFMA on 16-bit operands (bf16 or fp16 by overload; same cycles)
__device__ __forceinline__ float4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const float4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float4_t mfma16(const f16x8_t& a, const f16x8_t& b, const float4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- wave reductions
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

// ---------------------------------------------------------------- launch checking
#define AACLIP_CHECK_LAUNCH()                                 \
  do {                                                        \
    hipError_t _e = hipGetLastError();                        \
    if (_e != hipSuccess) return AACLIP_ERR_LAUNCH + (int)_e; \
  } while (0)

#define AACLIP_REQUIRE(cond) \
  do {                       \
    if (!(cond)) return AACLIP_ERR_ARG; \
  } while (0)

// Dynamic-LDS opt-in for a kernel, once per device: the attribute lives in the
// current device's context, so a process driving several GPUs sets it on each.
// `done` is the call site's bitmask of devices already set (a race between host
// threads only repeats the idempotent attribute write).
inline bool lds_attr_once(const void* fn, int bytes, unsigned& done) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const unsigned bit = (dev >= 0 && dev < 32) ? 1u << dev : 0u;
  if (bit && (done & bit)) return true;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) return false;
  done |= bit;
  return true;
}

__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
