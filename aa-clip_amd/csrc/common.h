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

// ---------------------------------------------------------------- step timeline (diagnostic)
// Built only with -DAACLIP_TRACE (`make trace` -> libaaclip_hip_trace.so; the product
// library compiles none of this): every wave of an instrumented kernel appends one
// record {t0, t1 (s_memrealtime, the chip-wide 100 MHz clock), tag, HW_ID, XCC_ID | the
// wave's shader-clock cycles (s_memtime delta) << 4, workgroup} to a caller-provided
// device buffer (aaclip_trace_buffer), so a tool can rebuild which CU ran what when over
// a whole concurrent step, and at what clock (tools/timeline.py).
// Records go to a per-CU slab (slot = XCC, SE, SH, CU: 2048 slots) through a per-slot
// counter 64 B apart: one counter for the whole chip serialised ~1.7 M same-address
// atomics per step and doubled the step time. Written with vector stores after the
// wave's own last memory op.
enum TraceTag : uint32_t {
  TR_GEMM_8PH = 1, TR_GEMM_TILE = 2, TR_GEMM_FP8MX = 3, TR_ATTN = 4, TR_LAYERNORM = 5, TR_BLOCK_TAIL = 6,
  TR_EMBED_LN = 7, TR_IM2COL = 8, TR_PARTIAL_SCORES = 9, TR_BLUR_SCORE = 10, TR_GEMM_F32 = 11, TR_ATTN_F32 = 12,
  TR_PATCH_SCORES = 13, TR_BLUR = 14, TR_DET = 15
};
constexpr int kTraceSlots = 2048;  // XCC (3 bits) x SE (3) x SH (1) x CU (4)
#ifdef AACLIP_TRACE
struct TraceState {
  uint32_t* rec;   // [kTraceSlots][cap][8] uint32
  uint32_t* count; // [kTraceSlots][16] uint32 (slot counters, one per 64 B)
  uint32_t cap;    // records per slot
};
static __device__ TraceState g_trace;
struct TraceScope {
  uint64_t t0, c0;
  uint32_t tag;
  __device__ __forceinline__ explicit TraceScope(uint32_t tag_) : tag(tag_) {
    t0 = __builtin_amdgcn_s_memrealtime();
    c0 = __builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ ~TraceScope() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t dc = __builtin_amdgcn_s_memtime() - c0;  // shader cycles over the same span
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if ((threadIdx.x & 63) == 0 && g_trace.rec) {
      const uint32_t slot = ((xcc & 7) << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
      const uint32_t i = atomicAdd(g_trace.count + slot * 16, 1u);
      if (i < g_trace.cap) {
        const uint32_t wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        uint4* r = (uint4*)(g_trace.rec + ((size_t)slot * g_trace.cap + i) * 8);
        r[0] = uint4{(uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1, (uint32_t)(t1 >> 32)};
        r[1] = uint4{tag, hw, (xcc & 15) | ((uint32_t)min(dc, (uint64_t)0xFFFFFFF) << 4), wg};
      }
    }
  }
};
#define AACLIP_TRACE_SCOPE(tag) TraceScope _aaclip_trace_scope(tag)
// one per translation unit: points this TU's g_trace at the buffer (host side)
#define AACLIP_TRACE_SETTER(name)                                                          \
  int name(void* rec, void* count, unsigned cap) {                                        \
    TraceState t{(uint32_t*)rec, (uint32_t*)count, cap};                                  \
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &t, sizeof t) == hipSuccess ? 0 : -1;  \
  }
#else
#define AACLIP_TRACE_SCOPE(tag) ((void)0)
#define AACLIP_TRACE_SETTER(name)
#endif
