// Row-wise kernels of the AA-CLIP path: token assembly + LayerNorm, the fused
// post-block tail (adapter blend + next ln_1 + level tap/ln_post), text
// embedding, EOT gather, anchor reduction, L2 normalisation, im2col.
//
// HBM-bound streaming work. One wave (64 lanes) owns one row of width
// 256*VEC (768 -> VEC 3, 1024 -> VEC 4); lane l holds elements 256c + 4l .. +3,
// so every load/store instruction moves one contiguous 1 KiB (fp32) or 512 B
// (bf16) segment of the row. Mean/variance/norms are wave-shuffle reductions.
#include "common.h"

namespace {

constexpr float kLnEps = 1e-5f;  // nn.LayerNorm default (transformer.py:37-43)

template <int VEC>
__device__ __forceinline__ void load_f32(const float* p, float4_t (&v)[VEC], int lane) {
#pragma unroll
  for (int c = 0; c < VEC; ++c) v[c] = *(const float4_t*)(p + 256 * c + 4 * lane);
}

template <int VEC>
__device__ __forceinline__ void load_any(const void* p, int dtype, float4_t (&v)[VEC], int lane) {
  if (dtype == AACLIP_F32) {
    load_f32<VEC>((const float*)p, v, lane);
  } else if (dtype == AACLIP_F16) {
    const uint16_t* q = (const uint16_t*)p;
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      uint2 r = *(const uint2*)(q + 256 * c + 4 * lane);
      v[c][0] = f16_to_f32((uint16_t)(r.x & 0xffff));
      v[c][1] = f16_to_f32((uint16_t)(r.x >> 16));
      v[c][2] = f16_to_f32((uint16_t)(r.y & 0xffff));
      v[c][3] = f16_to_f32((uint16_t)(r.y >> 16));
    }
  } else {
    const uint16_t* q = (const uint16_t*)p;
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      uint2 r = *(const uint2*)(q + 256 * c + 4 * lane);
      v[c][0] = __uint_as_float(r.x << 16);
      v[c][1] = __uint_as_float(r.x & 0xffff0000u);
      v[c][2] = __uint_as_float(r.y << 16);
      v[c][3] = __uint_as_float(r.y & 0xffff0000u);
    }
  }
}

template <int VEC>
__device__ __forceinline__ void store_any(void* p, int dtype, const float4_t (&v)[VEC], int lane) {
  if (dtype == AACLIP_F32) {
#pragma unroll
    for (int c = 0; c < VEC; ++c) *(float4_t*)((float*)p + 256 * c + 4 * lane) = v[c];
  } else {
    const bool h = dtype == AACLIP_F16;
    uint16_t* q = (uint16_t*)p;
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      uint2 r;
      r.x = h ? pack_f16x2(v[c][0], v[c][1]) : pack_bf16x2(v[c][0], v[c][1]);
      r.y = h ? pack_f16x2(v[c][2], v[c][3]) : pack_bf16x2(v[c][2], v[c][3]);
      *(uint2*)(q + 256 * c + 4 * lane) = r;
    }
  }
}

template <int VEC>
__device__ __forceinline__ float row_sumsq(const float4_t (&v)[VEC]) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < VEC; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[c][j] * v[c][j];
  return wave_sum(s);
}

// F.layer_norm: (x - mean) / sqrt(var + eps) * w + b, biased variance.
template <int VEC>
__device__ __forceinline__ void layer_norm(const float4_t (&x)[VEC], const float* w, const float* b,
                                           float4_t (&y)[VEC], int lane) {
  constexpr float inv_d = 1.0f / (256 * VEC);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < VEC; ++c) s += (x[c][0] + x[c][1]) + (x[c][2] + x[c][3]);
  const float mean = wave_sum(s) * inv_d;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < VEC; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float d = x[c][j] - mean;
      q += d * d;
    }
  const float rstd = 1.0f / sqrtf(wave_sum(q) * inv_d + kLnEps);
#pragma unroll
  for (int c = 0; c < VEC; ++c) {
    float4_t wv = *(const float4_t*)(w + 256 * c + 4 * lane);
    float4_t bv = *(const float4_t*)(b + 256 * c + 4 * lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) y[c][j] = (x[c][j] - mean) * rstd * wv[j] + bv[j];
  }
}

__device__ __forceinline__ size_t esize(int dtype) { return dtype == AACLIP_F32 ? 4 : (dtype == AACLIP_FP8 ? 1 : 2); }

// smallest e with amax * 2^-e <= 448 (largest finite e4m3): the e8m0 block scale
__device__ __forceinline__ int mx_exp_row(float amax) {
  if (!(amax > 0.f)) return 0;
  int x;
  (void)frexpf(amax, &x);  // amax = m * 2^x, m in [0.5, 1)
  int e = x - 9;           // amax * 2^-e in [256, 512)
  if (ldexpf(amax, -e) > 448.f) e += 1;
  return max(min(e, 127), -126);
}

// MX fp8 row store (AACLIP_FP8 outputs, config C5): lane l holds elements 256c + 4l..+3,
// so a 64-element block is 16 lanes: max over them (4 xor-shuffles inside the 16-lane
// group), e8m0 scale, RNE to e4m3 after the exact 2^-e scaling; 4 bytes per lane and
// chunk; the block's first lane writes the scale byte to sc[(blk/2)*ld_sc + row][blk%2].
template <int VEC>
__device__ __forceinline__ void store_mx(uint8_t* q, uint8_t* sc, int64_t ld_sc, size_t row,
                                         const float4_t (&v)[VEC], int lane) {
#pragma unroll
  for (int c = 0; c < VEC; ++c) {
    float amax = fmaxf(fmaxf(fabsf(v[c][0]), fabsf(v[c][1])), fmaxf(fabsf(v[c][2]), fabsf(v[c][3])));
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    const int e = mx_exp_row(amax);
    const float inv = __uint_as_float((uint32_t)(127 - e) << 23);
    uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][0] * inv, v[c][1] * inv, 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][2] * inv, v[c][3] * inv, w, true);
    *(uint32_t*)(q + row * (256 * VEC) + 256 * c + 4 * lane) = w;
    if ((lane & 15) == 0) {
      const int blk = 4 * c + (lane >> 4);
      sc[((size_t)(blk >> 1) * ld_sc + row) * 2 + (blk & 1)] = (uint8_t)(e + 127);
    }
  }
}

template <int VEC>
__device__ __forceinline__ void store_out(void* p, int dtype, size_t row, uint8_t* sc, int64_t ld_sc,
                                          const float4_t (&v)[VEC], int lane) {
  if (dtype == AACLIP_FP8)
    store_mx<VEC>((uint8_t*)p, sc, ld_sc, row, v, lane);
  else
    store_any<VEC>((char*)p + row * (256 * VEC) * esize(dtype), dtype, v, lane);
}

// ------------------------------------------------------------------ kernels
template <int VEC>
__global__ __launch_bounds__(256) void embed_ln_kernel(int out_dtype, float* x, const float* cls,
                                                       const float* pos, const float* pw,
                                                       const float* pb, const float* w1,
                                                       const float* b1, void* h, int rows,
                                                       int n_tok, uint8_t* sc, int64_t ld_sc) {
  AACLIP_TRACE_SCOPE(TR_EMBED_LN);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = 256 * VEC;
  const int t = row % n_tok;
  float* xr = x + (size_t)row * D;
  float4_t e[VEC], p[VEC];
  load_f32<VEC>(t == 0 ? cls : xr, e, lane);
  load_f32<VEC>(pos + (size_t)t * D, p, lane);
#pragma unroll
  for (int c = 0; c < VEC; ++c) e[c] += p[c];
  float4_t y[VEC];
  layer_norm<VEC>(e, pw, pb, y, lane);
  store_any<VEC>(xr, AACLIP_F32, y, lane);
  layer_norm<VEC>(y, w1, b1, e, lane);
  store_out<VEC>(h, out_dtype, row, sc, ld_sc, e, lane);
}

template <int VEC>
__global__ __launch_bounds__(256) void block_tail_kernel(int out_dtype, float* x, const float* u,
                                                         float aw, const float* lw,
                                                         const float* lb, void* h,
                                                         const float* pw, const float* pb,
                                                         void* tap, int rows, int n_tok, uint8_t* sc,
                                                         int64_t ld_sc) {
  AACLIP_TRACE_SCOPE(TR_BLOCK_TAIL);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = 256 * VEC;
  float* xr = x + (size_t)row * D;
  float4_t v[VEC];
  load_f32<VEC>(xr, v, lane);
  if (u) {
    // adapter.py:94-99: u * ||x|| / ||u||, then w*u + (1-w)*x
    float4_t a[VEC];
    load_f32<VEC>(u + (size_t)row * D, a, lane);
    const float xn = sqrtf(row_sumsq<VEC>(v));
    const float un = sqrtf(row_sumsq<VEC>(a));
    const float keep = 1.0f - aw;
#pragma unroll
    for (int c = 0; c < VEC; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[c][j] = aw * (a[c][j] * xn / un) + keep * v[c][j];
    store_any<VEC>(xr, AACLIP_F32, v, lane);
  }
  float4_t y[VEC];
  if (h) {
    layer_norm<VEC>(v, lw, lb, y, lane);
    store_out<VEC>(h, out_dtype, row, sc, ld_sc, y, lane);
  }
  if (tap) {  // level taps stay bf16 (seg_proj inputs) when h is fp8
    const int tdt = out_dtype == AACLIP_FP8 ? AACLIP_BF16 : out_dtype;
    const int t = row % n_tok;
    if (t >= 1) {
      const size_t trow = (size_t)(row / n_tok) * (n_tok - 1) + (t - 1);
      layer_norm<VEC>(v, pw, pb, y, lane);
      store_any<VEC>((char*)tap + trow * D * esize(tdt), tdt, y, lane);
    }
  }
}

template <int VEC>
__global__ __launch_bounds__(256) void layernorm_kernel(int out_dtype, const float* x, int64_t ldx,
                                                        const float* w, const float* b, void* y,
                                                        int64_t ldy, int rows, uint8_t* sc, int64_t ld_sc) {
  AACLIP_TRACE_SCOPE(TR_LAYERNORM);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float4_t v[VEC], o[VEC];
  load_f32<VEC>(x + (size_t)row * ldx, v, lane);
  layer_norm<VEC>(v, w, b, o, lane);
  if (out_dtype == AACLIP_FP8)
    store_mx<VEC>((uint8_t*)y, sc, ld_sc, row, o, lane);  // ldy == width (checked on the host)
  else
    store_any<VEC>((char*)y + (size_t)row * ldy * esize(out_dtype), out_dtype, o, lane);
}

template <int VEC>
__global__ __launch_bounds__(256) void text_embed_ln_kernel(int out_dtype, const int32_t* tokens,
                                                            const float* temb, const float* pos,
                                                            const float* w1, const float* b1,
                                                            float* x, void* h, int rows, int ctx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = 256 * VEC;
  const int t = row % ctx;
  const int tok = tokens[row];
  float4_t e[VEC], p[VEC];
  load_f32<VEC>(temb + (size_t)tok * D, e, lane);
  load_f32<VEC>(pos + (size_t)t * D, p, lane);
#pragma unroll
  for (int c = 0; c < VEC; ++c) e[c] += p[c];
  store_any<VEC>(x + (size_t)row * D, AACLIP_F32, e, lane);
  layer_norm<VEC>(e, w1, b1, p, lane);
  store_any<VEC>((char*)h + (size_t)row * D * esize(out_dtype), out_dtype, p, lane);
}

template <int VEC>
__global__ __launch_bounds__(256) void eot_ln_kernel(int out_dtype, const float* x,
                                                     const int32_t* tokens, const float* w,
                                                     const float* b, void* y, int n_seq,
                                                     int ctx) {
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= n_seq) return;
  constexpr int D = 256 * VEC;
  // argmax over the row, first occurrence (EOT = 49407 is the largest id)
  int best_v = -2147483647 - 1, best_i = 0;
  for (int t = lane; t < ctx; t += 64) {
    int v = tokens[(size_t)s * ctx + t];
    if (v > best_v) { best_v = v; best_i = t; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int ov = __shfl_xor(best_v, o, 64);
    int oi = __shfl_xor(best_i, o, 64);
    if (ov > best_v || (ov == best_v && oi < best_i)) { best_v = ov; best_i = oi; }
  }
  float4_t v[VEC], o[VEC];
  load_f32<VEC>(x + ((size_t)s * ctx + best_i) * D, v, lane);
  layer_norm<VEC>(v, w, b, o, lane);
  store_any<VEC>((char*)y + (size_t)s * D * esize(out_dtype), out_dtype, o, lane);
}

template <int VEC>
__global__ __launch_bounds__(256) void l2norm_kernel(int in_dtype, int out_dtype, const void* x,
                                                     int64_t ldx, void* y, int64_t ldy,
                                                     int rows) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float4_t v[VEC];
  load_any<VEC>((const char*)x + (size_t)row * ldx * esize(in_dtype), in_dtype, v, lane);
  const float inv = 1.0f / fmaxf(sqrtf(row_sumsq<VEC>(v)), 1e-12f);
#pragma unroll
  for (int c = 0; c < VEC; ++c) v[c] = v[c] * inv;
  store_any<VEC>((char*)y + (size_t)row * ldy * esize(out_dtype), out_dtype, v, lane);
}

// forward_utils.py:155-159 — one 256-thread block.
__global__ __launch_bounds__(256) void anchor_reduce_kernel(const float* emb, int n, int dim,
                                                            float* T, int col, int ncols) {
  __shared__ float inv_norm[256];
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int s = wid; s < n; s += 4) {
    float q = 0.f;
    for (int j = lane; j < dim; j += 64) {
      float e = emb[(size_t)s * dim + j];
      q += e * e;
    }
    q = wave_sum(q);
    if (lane == 0) inv_norm[s] = 1.0f / sqrtf(q);
  }
  __syncthreads();
  float part = 0.f;
  float m_local[4];  // dim <= 1024
  int cnt = 0;
  for (int j = threadIdx.x; j < dim; j += 256, ++cnt) {
    float acc = 0.f;
    for (int s = 0; s < n; ++s) acc += emb[(size_t)s * dim + j] * inv_norm[s];
    const float m = acc / (float)n;
    m_local[cnt] = m;
    part += m * m;
  }
  part = wave_sum(part);
  if (lane == 0) red[wid] = part;
  __syncthreads();
  const float inv = 1.0f / sqrtf((red[0] + red[1]) + (red[2] + red[3]));
  cnt = 0;
  for (int j = threadIdx.x; j < dim; j += 256, ++cnt) T[(size_t)j * ncols + col] = m_local[cnt] * inv;
}

// One workgroup per (image, patch row, channel): the P image rows a patch row spans
// are P*S contiguous floats, read with full-width loads into LDS; each of the g
// patches then writes this channel's P*P values as one contiguous run of its cols row
// (two k per lane-store), and the last channel's workgroup zero-fills k >= C*P*P.
// Both sides coalesced (the per-thread 8-k form reads 2 scattered 32-B runs per
// thread). Pure copy + the same conversions: the same bits as im2col_kernel.
__global__ __launch_bounds__(256) void im2col_band_kernel(int out_dtype, const float* img, void* cols, int C,
                                                          int S, int P, int g, int kp) {
  AACLIP_TRACE_SCOPE(TR_IM2COL);
  extern __shared__ __attribute__((aligned(16))) float band[];  // [P][S]
  const int c = blockIdx.x % C;
  const int bp = blockIdx.x / C;
  const int py = bp % g, b = bp / g;
  const float* src = img + (((size_t)b * C + c) * S + (size_t)py * P) * S;
  const int n = P * S;
  if ((S & 3) == 0 && ((uintptr_t)img & 15) == 0) {
    for (int i = threadIdx.x; i < n / 4; i += 256) ((float4_t*)band)[i] = ((const float4_t*)src)[i];
  } else {
    for (int i = threadIdx.x; i < n; i += 256) band[i] = src[i];
  }
  __syncthreads();
  const int pp = P * P;
  const int kreal = C * pp;
  const int k0 = c * pp;
  const int kend = c == C - 1 ? kp : k0 + pp;  // the last channel also writes the zero pad
  const int npair = (kend - k0) / 2;          // pp, kreal and kp are even
  const size_t row0 = ((size_t)b * g + py) * g;
  for (int i = threadIdx.x; i < g * npair; i += 256) {
    const int px = i / npair;
    const int k = k0 + 2 * (i % npair);
    float v[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kk = k + j - k0;
      v[j] = k + j < kreal ? band[(kk / P) * S + px * P + kk % P] : 0.f;
    }
    const size_t o = (row0 + px) * kp + k;
    if (out_dtype == AACLIP_F32)
      *(float2_t*)((float*)cols + o) = float2_t{v[0], v[1]};
    else if (out_dtype == AACLIP_F16)
      *(uint32_t*)((uint16_t*)cols + o) = pack_f16x2(v[0], v[1]);
    else
      *(uint32_t*)((uint16_t*)cols + o) = pack_bf16x2(v[0], v[1]);
  }
}

// 8 consecutive k of one patch row per thread.
__global__ __launch_bounds__(256) void im2col_kernel(int out_dtype, const float* img, void* cols,
                                                     int batch, int C, int S, int P, int g,
                                                     int kp) {
  const int kchunks = kp / 8;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)batch * g * g * kchunks;
  if (idx >= total) return;
  const int kc = idx % kchunks;
  const size_t row = idx / kchunks;
  const int b = row / (g * g);
  const int pp = row % (g * g);
  const int py = pp / g, px = pp % g;
  const int kreal = C * P * P;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = kc * 8 + j;
    if (k < kreal) {
      const int c = k / (P * P), r = k % (P * P);
      const int kh = r / P, kw = r % P;
      v[j] = img[(((size_t)b * C + c) * S + (size_t)py * P + kh) * S + (size_t)px * P + kw];
    } else {
      v[j] = 0.f;
    }
  }
  if (out_dtype == AACLIP_F32) {
    float* o = (float*)cols + row * kp + kc * 8;
    *(float4_t*)o = float4_t{v[0], v[1], v[2], v[3]};
    *(float4_t*)(o + 4) = float4_t{v[4], v[5], v[6], v[7]};
  } else if (out_dtype == AACLIP_F16) {
    uint4 r;
    r.x = pack_f16x2(v[0], v[1]);
    r.y = pack_f16x2(v[2], v[3]);
    r.z = pack_f16x2(v[4], v[5]);
    r.w = pack_f16x2(v[6], v[7]);
    *(uint4*)((uint16_t*)cols + row * kp + kc * 8) = r;
  } else {
    uint4 r;
    r.x = pack_bf16x2(v[0], v[1]);
    r.y = pack_bf16x2(v[2], v[3]);
    r.z = pack_bf16x2(v[4], v[5]);
    r.w = pack_bf16x2(v[6], v[7]);
    *(uint4*)((uint16_t*)cols + row * kp + kc * 8) = r;
  }
}

#define DISPATCH_VEC(width, ...)                 \
  switch ((width)) {                             \
    case 768: { constexpr int V = 3; __VA_ARGS__; break; } \
    case 1024: { constexpr int V = 4; __VA_ARGS__; break; } \
    default: return AACLIP_ERR_ARG;              \
  }

inline bool dtype_ok(int d) { return d == AACLIP_F32 || d == AACLIP_BF16 || d == AACLIP_F16; }
// fp8 MX outputs (config C5) need the e8m0 scale buffer [width/128][ld_mx >= rows][2]
inline bool mx_ok(int d, const void* mx, int64_t ld_mx, int rows, int width) {
  return dtype_ok(d) || (d == AACLIP_FP8 && mx && ld_mx >= rows && width % 128 == 0);
}


// ------------------------------------------------------------------ fp8 quantisation
// Per-row symmetric quantisation to OCP e4m3 for the fp8 GEMM (config C5):
// scale[row] = max|x[row]| / 448 (448 = largest finite e4m3), q = RNE(x / scale)
// via v_cvt_pk_fp8_f32. One wave per row; lane l owns elements 8l + 512c .. +7,
// so each pass moves 16-B (bf16) / 32-B (fp32) contiguous pieces.
__device__ __forceinline__ void load8(const void* p, int dtype, size_t off, float (&v)[8]) {
  if (dtype == AACLIP_F32) {
    const float4_t a = *(const float4_t*)((const float*)p + off), b = *(const float4_t*)((const float*)p + off + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = a[j];
      v[4 + j] = b[j];
    }
  } else {
    const uint4 r = *(const uint4*)((const uint16_t*)p + off);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  }
}

__global__ __launch_bounds__(256) void quant_fp8_kernel(int in_dtype, const void* __restrict__ x, int64_t ldx,
                                                        uint8_t* __restrict__ q, int64_t ldq,
                                                        float* __restrict__ scale, int rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float amax = 0.f;
  for (int c0 = 8 * lane; c0 < cols; c0 += 512) {
    float v[8];
    load8(x, in_dtype, (size_t)row * ldx + c0, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
  }
  amax = wave_max(amax);
  const float sc = amax > 0.f ? amax * (1.0f / 448.0f) : 1.0f;
  const float inv = amax > 0.f ? 448.0f / amax : 1.0f;
  if (lane == 0) scale[row] = sc;
  for (int c0 = 8 * lane; c0 < cols; c0 += 512) {
    float v[8];
    load8(x, in_dtype, (size_t)row * ldx + c0, v);
    uint32_t w0 = 0, w1 = 0;
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, w0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, w0, true);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, w1, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, w1, true);
    *(uint2*)(q + (size_t)row * ldq + c0) = uint2{w0, w1};
  }
}


// MX variant: one wave per row, lane l owns elements 8l + 512c .. +7, so a 64-element
// block is 8 consecutive lanes: max over them (3 xor-shuffles), power-of-two e8m0
// scale, RNE to e4m3 after an exact 2^-e scaling.

__global__ __launch_bounds__(256) void quant_mx_kernel(int in_dtype, const void* __restrict__ x, int64_t ldx,
                                                       uint8_t* __restrict__ q, int64_t ldq,
                                                       uint8_t* __restrict__ sc, int64_t ld_sc, int rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  for (int c0 = 8 * lane; c0 < cols; c0 += 512) {
    float v[8];
    load8(x, in_dtype, (size_t)row * ldx + c0, v);
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    const int e = mx_exp_row(amax);
    const float inv = __uint_as_float((uint32_t)(127 - e) << 23);
    uint32_t w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, 0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, w0, true);
    uint32_t w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, 0, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, w1, true);
    *(uint2*)(q + (size_t)row * ldq + c0) = uint2{w0, w1};
    if ((lane & 7) == 0) {
      const int blk = c0 >> 6;
      sc[((size_t)(blk >> 1) * ld_sc + row) * 2 + (blk & 1)] = (uint8_t)(e + 127);
    }
  }
}

}  // namespace

extern "C" int aaclip_embed_ln(int out_dtype, float* x, const float* cls, const float* pos,
                               const float* ln_pre_w, const float* ln_pre_b, const float* ln1_w,
                               const float* ln1_b, void* h, int batch, int n_tok, int width,
                               void* h_mx, int64_t ld_mx, void* stream) {
  AACLIP_REQUIRE(mx_ok(out_dtype, h_mx, ld_mx, batch * n_tok, width));
  AACLIP_REQUIRE(x && cls && pos && ln_pre_w && ln_pre_b && ln1_w && ln1_b && h);
  AACLIP_REQUIRE(batch > 0 && n_tok > 1);
  const int rows = batch * n_tok;
  DISPATCH_VEC(width, embed_ln_kernel<V><<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(
                          out_dtype, x, cls, pos, ln_pre_w, ln_pre_b, ln1_w, ln1_b, h, rows, n_tok,
                          (uint8_t*)h_mx, ld_mx));
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_block_tail(int out_dtype, float* x, const float* u, float adapt_weight,
                                 const float* ln_w, const float* ln_b, void* h,
                                 const float* post_w, const float* post_b, void* tap, int rows,
                                 int n_tok, int width, void* h_mx, int64_t ld_mx, void* stream) {
  AACLIP_REQUIRE(mx_ok(out_dtype, h ? h_mx : (void*)1, h ? ld_mx : rows, rows, width));
  AACLIP_REQUIRE(x && rows > 0 && n_tok > 0);
  AACLIP_REQUIRE(!h || (ln_w && ln_b));
  AACLIP_REQUIRE(!tap || (post_w && post_b && n_tok > 1 && rows % n_tok == 0));
  DISPATCH_VEC(width, block_tail_kernel<V><<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(
                          out_dtype, x, u, adapt_weight, ln_w, ln_b, h, post_w, post_b, tap, rows,
                          n_tok, (uint8_t*)h_mx, ld_mx));
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_layernorm(int out_dtype, const float* x, int64_t ldx, const float* w,
                                const float* b, void* y, int64_t ldy, int rows, int width,
                                void* y_mx, int64_t ld_mx, void* stream) {
  AACLIP_REQUIRE(mx_ok(out_dtype, y_mx, ld_mx, rows, width) && x && w && b && y && rows >= 0);
  AACLIP_REQUIRE(ldx >= width && ldy >= width && ldx % 4 == 0 && ldy % 4 == 0);
  AACLIP_REQUIRE(out_dtype != AACLIP_FP8 || ldy == width);
  if (rows == 0) return AACLIP_OK;
  DISPATCH_VEC(width, layernorm_kernel<V><<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(
                          out_dtype, x, ldx, w, b, y, ldy, rows, (uint8_t*)y_mx, ld_mx));
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_text_embed_ln(int out_dtype, const int32_t* tokens, const float* tok_emb,
                                    const float* pos, const float* ln1_w, const float* ln1_b,
                                    float* x, void* h, int n_seq, int ctx, int width,
                                    void* stream) {
  AACLIP_REQUIRE(dtype_ok(out_dtype) && tokens && tok_emb && pos && ln1_w && ln1_b && x && h);
  AACLIP_REQUIRE(n_seq > 0 && ctx > 0);
  const int rows = n_seq * ctx;
  DISPATCH_VEC(width, text_embed_ln_kernel<V><<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(
                          out_dtype, tokens, tok_emb, pos, ln1_w, ln1_b, x, h, rows, ctx));
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_eot_ln(int out_dtype, const float* x, const int32_t* tokens, const float* w,
                             const float* b, void* y, int n_seq, int ctx, int width,
                             void* stream) {
  AACLIP_REQUIRE(dtype_ok(out_dtype) && x && tokens && w && b && y && n_seq > 0 && ctx > 0);
  DISPATCH_VEC(width, eot_ln_kernel<V><<<ceil_div(n_seq, 4), 256, 0, (hipStream_t)stream>>>(
                          out_dtype, x, tokens, w, b, y, n_seq, ctx));
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_anchor_reduce(const float* emb, int n, int dim, float* T, int col,
                                    int ncols, void* stream) {
  AACLIP_REQUIRE(emb && T && n > 0 && n <= 256 && dim > 0 && dim <= 1024 && col >= 0 && col < ncols);
  anchor_reduce_kernel<<<1, 256, 0, (hipStream_t)stream>>>(emb, n, dim, T, col, ncols);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_l2_normalize(int in_dtype, int out_dtype, const void* x, int64_t ldx,
                                   void* y, int64_t ldy, int rows, int width, void* stream) {
  AACLIP_REQUIRE(dtype_ok(in_dtype) && dtype_ok(out_dtype) && x && y && rows >= 0);
  AACLIP_REQUIRE(ldx >= width && ldy >= width && ldx % 4 == 0 && ldy % 4 == 0);
  if (rows == 0) return AACLIP_OK;
  DISPATCH_VEC(width, l2norm_kernel<V><<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(
                          in_dtype, out_dtype, x, ldx, y, ldy, rows));
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_im2col(int out_dtype, const float* img, void* cols, int batch, int channels,
                             int img_size, int patch, int k_padded, void* stream) {
  AACLIP_REQUIRE(dtype_ok(out_dtype) && img && cols && batch > 0 && channels > 0 && patch > 0);
  AACLIP_REQUIRE(img_size % patch == 0 && k_padded % 8 == 0 && k_padded >= channels * patch * patch);
  const int g = img_size / patch;
  const size_t band_bytes = (size_t)patch * img_size * sizeof(float);
  if (band_bytes <= 65536 && patch % 2 == 0) {  // every ViT-L/14 size (14 x 518 x 4 = 29 KB)
    im2col_band_kernel<<<(unsigned)(batch * g * channels), 256, band_bytes, (hipStream_t)stream>>>(
        out_dtype, img, cols, channels, img_size, patch, g, k_padded);
  } else {
    const size_t total = (size_t)batch * g * g * (k_padded / 8);
    im2col_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        out_dtype, img, cols, batch, channels, img_size, patch, g, k_padded);
  }
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_quant_fp8_rows(int in_dtype, const void* x, int64_t ldx, void* q, int64_t ldq, float* scale,
                                     int rows, int cols, void* stream) {
  AACLIP_REQUIRE((in_dtype == AACLIP_F32 || in_dtype == AACLIP_BF16) && x && q && scale && rows >= 0 && cols > 0 && cols % 8 == 0);
  AACLIP_REQUIRE(ldx >= cols && ldq >= cols && ldx % 8 == 0 && ldq % 8 == 0);
  AACLIP_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)q % 8) == 0);
  if (rows == 0) return AACLIP_OK;
  quant_fp8_kernel<<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(in_dtype, x, ldx, (uint8_t*)q, ldq, scale,
                                                                        rows, cols);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_quant_fp8_mx(int in_dtype, const void* x, int64_t ldx, void* q, int64_t ldq, void* sc,
                                   int64_t ld_sc, int rows, int cols, void* stream) {
  AACLIP_REQUIRE((in_dtype == AACLIP_F32 || in_dtype == AACLIP_BF16) && x && q && sc && rows >= 0 && cols > 0 && cols % 128 == 0);
  AACLIP_REQUIRE(ldx >= cols && ldq >= cols && ldx % 8 == 0 && ldq % 8 == 0 && ld_sc >= rows);
  AACLIP_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)q % 8) == 0);
  if (rows == 0) return AACLIP_OK;
  quant_mx_kernel<<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(in_dtype, x, ldx, (uint8_t*)q, ldq,
                                                                       (uint8_t*)sc, ld_sc, rows, cols);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

AACLIP_TRACE_SETTER(trace_set_rows)
