// Anomaly-map kernels (forward_utils.py:196-216, test.py:83-93).
//
// Stage 1 — patch_scores: HBM-bound stream over the level features. One wave
// per patch position reads that position's row in every level (L x 768 values,
// bf16 or fp32; each load instruction = one contiguous 512 B / 1 KiB segment),
// computes ||f||, f.t0, f.t1 with wave shuffles, and emits the level-summed
// test score  sum_l (100 f^.t1 + 1 - 100 f^.t0) / 2  (the level sum is moved
// ahead of blur+upsample, which are linear), or the two train logits.
// Stage 2 — blur_upsample: one block per (image, band of output rows) stages
// the grid rows the band needs in LDS, applies the separable reflect-border
// Gaussian (kornia 0.6.9 semantics) to them and writes the bilinear
// (align_corners) upsample with coalesced stores (any output size).
#include <math.h>

#include "common.h"

namespace {

constexpr int kMaxLevels = 8;
struct LevelPtrs {
  const void* p[kMaxLevels];
};

__global__ __launch_bounds__(256) void patch_scores_kernel(int in_dtype, LevelPtrs lv, int nl,
                                                           int64_t ld, const float* T, int rows,
                                                           int normalize, int mode, int group,
                                                           float* out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  // anchors at this lane's 12 channels (C = 768 = 3 x 256)
  float4_t t0[3], t1[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* tp = T + 2 * (256 * c + 4 * lane);
    float4_t a = *(const float4_t*)tp, b = *(const float4_t*)(tp + 4);
    t0[c] = float4_t{a[0], a[2], b[0], b[2]};
    t1[c] = float4_t{a[1], a[3], b[1], b[3]};
  }
  // issue every level's loads before reducing (memory-level parallelism)
  float4_t f[kMaxLevels][3];
#pragma unroll
  for (int l = 0; l < kMaxLevels; ++l) {
    if (l < nl) {
      if (in_dtype == AACLIP_F32) {
        const float* p = (const float*)lv.p[l] + (size_t)row * ld;
#pragma unroll
        for (int c = 0; c < 3; ++c) f[l][c] = *(const float4_t*)(p + 256 * c + 4 * lane);
      } else {
        const uint16_t* p = (const uint16_t*)lv.p[l] + (size_t)row * ld;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          uint2 r = *(const uint2*)(p + 256 * c + 4 * lane);
          f[l][c] = float4_t{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                             __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u)};
        }
      }
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int l = 0; l < kMaxLevels; ++l) {
    if (l < nl) {
      float ss = 0.f, a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = f[l][c][j];
          ss += v * v;
          a0 += v * t0[c][j];
          a1 += v * t1[c][j];
        }
      ss = wave_sum(ss);
      a0 = wave_sum(a0);
      a1 = wave_sum(a1);
      const float inv = normalize ? 1.0f / fmaxf(sqrtf(ss), 1e-12f) : 1.0f;
      const float A0 = 100.0f * (a0 * inv), A1 = 100.0f * (a1 * inv);
      if (mode == 0) {
        acc += (A1 + 1.0f - A0) / 2.0f;
      } else if (lane == 0) {
        const size_t base = (size_t)(row / group) * 2 * group + row % group;
        out[base] = A0;
        out[base + group] = A1;
      }
    }
  }
  if (mode == 0 && lane == 0) out[row] = acc;
}

// Train-branch logits for any number of anchors (forward_utils.py:199-202 with
// C anchors): out[b, a, p] = 100 * f[b*group + p] . T[:, a], channel-major so it
// feeds blur_upsample directly. One wave per patch row, anchors in sequence.
__global__ __launch_bounds__(256) void patch_logits_kernel(int in_dtype, const void* f, int64_t ld,
                                                           const float* T, int n_anchor, int rows,
                                                           int group, float* out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float4_t v[3];
  if (in_dtype == AACLIP_F32) {
    const float* p = (const float*)f + (size_t)row * ld;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = *(const float4_t*)(p + 256 * c + 4 * lane);
  } else {
    const uint16_t* p = (const uint16_t*)f + (size_t)row * ld;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      uint2 r = *(const uint2*)(p + 256 * c + 4 * lane);
      v[c] = float4_t{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                      __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u)};
    }
  }
  const size_t base = (size_t)(row / group) * n_anchor * group + row % group;
  for (int a = 0; a < n_anchor; ++a) {
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) d += v[c][j] * T[(size_t)(256 * c + 4 * lane + j) * n_anchor + a];
    d = wave_sum(d);
    if (lane == 0) out[base + (size_t)a * group] = 100.0f * d;
  }
}

// Reflect index for F.pad(mode='reflect') (no edge repeat).
__device__ __forceinline__ int reflect(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}

struct Gauss {
  float w[16];
};

constexpr int kBand = 8;  // output rows per block
constexpr int kMaxC = 8;  // channels of the train branch (anchors), softmax over them

// grid: [B, C, g, g]; out: [B, C, S, S]. One block (4 waves) per (b, band of kBand
// output rows). A band's bilinear taps read at most a few source rows, so only the
// grid rows those need are staged and blurred: rows r_lo..r_hi for the y pass, their
// reflect-padded neighbourhood r_lo-r..r_hi+r for the x pass (a reflected index of
// that range stays inside it). One wave per grid row (lane = column, g <= 64): no
// integer division anywhere. Same arithmetic, same order as the whole-grid blur, so
// the output is bit-identical to it. The upsample runs one wave per output row:
// 16-B stores of 4 consecutive pixels when S % 4 == 0, dword stores otherwise
// (518 px, the reference's default size).
__global__ __launch_bounds__(256) void blur_upsample_kernel(const float* grid, float* out, int C,
                                                            int g, int S, int ksize, Gauss gw,
                                                            int softmax, float scale) {
  // no FMA contraction: ATen rounds src = scale * dst before taking the lambdas
  // (a fused scale * dst - i0 shifts them by up to an ulp of src, ~1e-5 in the map)
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int gg = g * g;
  float* src = smem;           // C * gg (raw, then blurred rows r_lo..r_hi)
  float* tmp = smem + C * gg;  // C * gg (x-blurred rows)
  const int y0 = blockIdx.x * kBand;
  const int y1 = min(y0 + kBand, S);
  const int r_lo = (int)(scale * (float)y0);
  const int r_hi = min((int)(scale * (float)(y1 - 1)) + 1, g - 1);
  const int r = ksize / 2;  // (k-1)//2 left pad == k//2 for odd k
  const int x_lo = ksize > 0 ? max(0, r_lo - r) : r_lo;
  const int x_hi = ksize > 0 ? min(g - 1, r_hi + r) : r_hi;
  for (int c = 0; c < C; ++c)
    for (int h = x_lo + wid; h <= x_hi; h += 4)
      if (lane < g) src[c * gg + h * g + lane] = grid[((size_t)b * C + c) * gg + h * g + lane];
  __syncthreads();
  if (ksize > 0) {
    for (int c = 0; c < C; ++c)  // x pass
      for (int h = x_lo + wid; h <= x_hi; h += 4)
        if (lane < g) {
          const float* row = src + c * gg + h * g;
          float acc = 0.f;
          for (int t = 0; t < ksize; ++t) acc += gw.w[t] * row[reflect(lane + t - r, g)];
          tmp[c * gg + h * g + lane] = acc;
        }
    __syncthreads();
    for (int c = 0; c < C; ++c)  // y pass
      for (int h = r_lo + wid; h <= r_hi; h += 4)
        if (lane < g) {
          const float* col = tmp + c * gg + lane;
          float acc = 0.f;
          for (int t = 0; t < ksize; ++t) acc += gw.w[t] * col[reflect(h + t - r, g) * g];
          src[c * gg + h * g + lane] = acc;
        }
    __syncthreads();
  }
  const bool vec4 = (S & 3) == 0;
  for (int y = y0 + wid; y < y1; y += 4) {
    // ATen upsample_bilinear2d, align_corners=True: src = scale * dst (fp32)
    const float sy = scale * (float)y;
    const int iy0 = (int)sy;
    const int iy1 = iy0 + (iy0 < g - 1 ? 1 : 0);
    const float hy1 = fminf(fmaxf(sy - (float)iy0, 0.f), 1.f), hy0 = 1.0f - hy1;
    const int step = vec4 ? 256 : 64;
    for (int x0 = (vec4 ? 4 : 1) * lane; x0 < S; x0 += step) {
      float v[kMaxC][4];
      const int nx = vec4 ? 4 : 1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= nx) break;
        const float sx = scale * (float)(x0 + j);
        const int ix0 = (int)sx;
        const int ix1 = ix0 + (ix0 < g - 1 ? 1 : 0);
        const float wx1 = fminf(fmaxf(sx - (float)ix0, 0.f), 1.f), wx0 = 1.0f - wx1;
        for (int c = 0; c < C; ++c) {
          const float* s = src + c * gg;
          v[c][j] = hy0 * (wx0 * s[iy0 * g + ix0] + wx1 * s[iy0 * g + ix1]) +
                    hy1 * (wx0 * s[iy1 * g + ix0] + wx1 * s[iy1 * g + ix1]);
        }
      }
      if (softmax && C > 1) {  // torch.softmax over the channel dim (forward_utils.py:214-215)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j >= nx) break;
          float m = v[0][j];
          for (int c = 1; c < C; ++c) m = fmaxf(m, v[c][j]);
          float sum = 0.f;
          for (int c = 0; c < C; ++c) {
            v[c][j] = expf(v[c][j] - m);
            sum += v[c][j];
          }
          const float inv = 1.0f / sum;
          for (int c = 0; c < C; ++c) v[c][j] *= inv;
        }
      }
      for (int c = 0; c < C; ++c) {
        float* o = out + (((size_t)b * C + c) * S + y) * S + x0;
        if (vec4)
          *(float4_t*)o = float4_t{v[c][0], v[c][1], v[c][2], v[c][3]};
        else
          *o = v[c][0];
      }
    }
  }
}

// Image score, stage 1: per (image, chunk of 64 patches) the sum of
// normalised det rows -> partial[b][chunk][768]. 4 waves x 16 rows.
__global__ __launch_bounds__(256) void det_partial_kernel(int in_dtype, const void* det, int64_t ld,
                                                          int n_patch, int normalize,
                                                          float* partial, int nchunk) {
  __shared__ float red[4][768];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = blockIdx.y, ch = blockIdx.x;
  float4_t acc[3] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int k = 0; k < 16; ++k) {
    const int p = ch * 64 + wid * 16 + k;
    if (p >= n_patch) break;
    const size_t row = (size_t)b * n_patch + p;
    float4_t v[3];
    if (in_dtype == AACLIP_F32) {
      const float* q = (const float*)det + row * ld;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = *(const float4_t*)(q + 256 * c + 4 * lane);
    } else {
      const uint16_t* q = (const uint16_t*)det + row * ld;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        uint2 r = *(const uint2*)(q + 256 * c + 4 * lane);
        v[c] = float4_t{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                        __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u)};
      }
    }
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) ss += v[c][j] * v[c][j];
    ss = wave_sum(ss);
    const float inv = normalize ? 1.0f / fmaxf(sqrtf(ss), 1e-12f) : 1.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += v[c] * inv;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) *(float4_t*)&red[wid][256 * c + 4 * lane] = acc[c];
  __syncthreads();
  for (int j = threadIdx.x; j < 768; j += 256) {
    partial[((size_t)b * nchunk + ch) * 768 + j] = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
  }
}

// Image score, stage 2: det[b] = sum(partials) / n_patch; score = (det.T1 + 1)/2.
__global__ __launch_bounds__(256) void det_finalize_kernel(const float* partial, int nchunk,
                                                           int n_patch, const float* T,
                                                           float* det, float* score) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  float dot = 0.f;
  for (int j = threadIdx.x; j < 768; j += 256) {
    float s = 0.f;
    for (int c = 0; c < nchunk; ++c) s += partial[((size_t)b * nchunk + c) * 768 + j];
    const float m = s / (float)n_patch;
    if (det) det[(size_t)b * 768 + j] = m;
    if (T) dot += m * T[2 * j + 1];
  }
  if (!score) return;  // block-uniform
  dot = wave_sum(dot);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dot;
  __syncthreads();
  if (threadIdx.x == 0) score[b] = (((red[0] + red[1]) + (red[2] + red[3])) + 1.0f) / 2.0f;
}

// kornia 0.6.9 get_gaussian_kernel1d in fp32.
Gauss gaussian_weights(int k, float sigma) {
  Gauss g{};
  float sum = 0.f;
  for (int i = 0; i < k; ++i) {
    float x = (float)i - (float)(k / 2);
    if (k % 2 == 0) x += 0.5f;
    g.w[i] = expf(-(x * x) / (2.0f * sigma * sigma));
    sum += g.w[i];
  }
  for (int i = 0; i < k; ++i) g.w[i] /= sum;
  return g;
}

}  // namespace

extern "C" int aaclip_patch_scores(int in_dtype, const void* const* levels, int n_levels,
                                   int64_t ld, const float* T, int rows, int channels,
                                   int normalize, int mode, int group, float* out,
                                   void* stream) {
  AACLIP_REQUIRE(in_dtype == AACLIP_F32 || in_dtype == AACLIP_BF16);
  AACLIP_REQUIRE(levels && T && out && rows >= 0 && channels == 768 && ld >= channels && ld % 4 == 0);
  AACLIP_REQUIRE(n_levels >= 1 && n_levels <= kMaxLevels && (mode == 0 || (mode == 1 && n_levels == 1)));
  AACLIP_REQUIRE(mode == 0 || (group > 0 && rows % group == 0));
  LevelPtrs lv{};
  for (int i = 0; i < n_levels; ++i) {
    AACLIP_REQUIRE(levels[i] != nullptr);
    lv.p[i] = levels[i];
  }
  if (rows == 0) return AACLIP_OK;
  patch_scores_kernel<<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(
      in_dtype, lv, n_levels, ld, T, rows, normalize, mode, mode == 1 ? group : 1, out);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_patch_logits(int in_dtype, const void* f, int64_t ld, const float* T, int n_anchor,
                                   int rows, int channels, int group, float* out, void* stream) {
  AACLIP_REQUIRE(in_dtype == AACLIP_F32 || in_dtype == AACLIP_BF16);
  AACLIP_REQUIRE(f && T && out && rows >= 0 && channels == 768 && ld >= channels && ld % 4 == 0);
  AACLIP_REQUIRE(n_anchor >= 1 && n_anchor <= 64 && group > 0 && rows % group == 0);
  if (rows == 0) return AACLIP_OK;
  patch_logits_kernel<<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(in_dtype, f, ld, T, n_anchor, rows,
                                                                          group, out);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_blur_upsample(const float* grid, float* out, int batch, int channels, int g,
                                    int out_size, int ksize, float sigma, int softmax,
                                    void* stream) {
  AACLIP_REQUIRE(grid && out && batch > 0 && channels >= 1 && channels <= kMaxC);
  AACLIP_REQUIRE(g >= 2 && g <= 64 && out_size >= 2);
  AACLIP_REQUIRE(ksize >= 0 && ksize <= 15 && (ksize == 0 || (ksize % 2 == 1 && ksize / 2 < g)));
  const Gauss gw = ksize > 0 ? gaussian_weights(ksize, sigma) : Gauss{};
  const float scale = (float)(g - 1) / (float)(out_size - 1);
  const size_t lds = (size_t)(ksize > 0 ? 2 : 1) * channels * g * g * sizeof(float);
  AACLIP_REQUIRE(lds <= 160 * 1024);
  static unsigned attr_dev = 0;
  if (lds > 64 * 1024 && !lds_attr_once((const void*)blur_upsample_kernel, 160 * 1024, attr_dev))
    return AACLIP_ERR_LAUNCH;
  dim3 grd(ceil_div(out_size, kBand), batch);
  blur_upsample_kernel<<<grd, 256, lds, (hipStream_t)stream>>>(grid, out, channels, g, out_size,
                                                               ksize, gw, softmax, scale);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_anomaly_map(int in_dtype, const void* const* levels, int n_levels, int64_t ld,
                                  const float* T, int batch, int g, int channels, int normalize,
                                  int out_size, int ksize, float sigma, float* grid_ws,
                                  float* out, void* stream) {
  AACLIP_REQUIRE(grid_ws && batch > 0);
  int rc = aaclip_patch_scores(in_dtype, levels, n_levels, ld, T, batch * g * g, channels,
                               normalize, 0, 0, grid_ws, stream);
  if (rc) return rc;
  return aaclip_blur_upsample(grid_ws, out, batch, 1, g, out_size, ksize, sigma, 0, stream);
}

extern "C" int aaclip_image_score(int in_dtype, const void* det_raw, int64_t ld, const float* T,
                                  int batch, int n_patch, int channels, int normalize,
                                  float* partial, float* det, float* score, void* stream) {
  AACLIP_REQUIRE(in_dtype == AACLIP_F32 || in_dtype == AACLIP_BF16);
  AACLIP_REQUIRE(det_raw && partial && batch > 0 && n_patch > 0);
  AACLIP_REQUIRE((T && score) || (!T && !score && det));
  AACLIP_REQUIRE(channels == 768 && ld >= channels && ld % 4 == 0);
  const int nchunk = ceil_div(n_patch, 64);
  det_partial_kernel<<<dim3(nchunk, batch), 256, 0, (hipStream_t)stream>>>(
      in_dtype, det_raw, ld, n_patch, normalize, partial, nchunk);
  AACLIP_CHECK_LAUNCH();
  det_finalize_kernel<<<batch, 256, 0, (hipStream_t)stream>>>(partial, nchunk, n_patch, T, det,
                                                              score);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}
