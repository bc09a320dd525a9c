// Anomaly-map kernels (forward_utils.py:196-216, test.py:83-93).
//
// Stage 1 — patch_scores: HBM-bound stream over the level features. One wave
// per patch position reads that position's row in every level (L x 768 values,
// bf16 or fp32; each load instruction = one contiguous 512 B / 1 KiB segment),
// computes ||f||, f.t0, f.t1 with wave shuffles, and emits the level-summed
// test score  sum_l (100 f^.t1 + 1 - 100 f^.t0) / 2  (the level sum is moved
// ahead of blur+upsample, which are linear), or the two train logits.
// Stage 2 — blur_upsample: one wave per (image, band of output rows) stages
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

// The lane's 12 anchor channels (C = 768 = 3 x 256): t0 / t1 = normal / abnormal.
__device__ __forceinline__ void load_anchors(const float* T, float4_t (&t0)[3], float4_t (&t1)[3], int lane) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* tp = T + 2 * (256 * c + 4 * lane);
    float4_t a = *(const float4_t*)tp, b = *(const float4_t*)(tp + 4);
    t0[c] = float4_t{a[0], a[2], b[0], b[2]};
    t1[c] = float4_t{a[1], a[3], b[1], b[3]};
  }
}

// One patch row through every level (one wave): loads of all levels issued before
// the reductions (memory-level parallelism), then ||f||, f.t0, f.t1 per level.
// mode 0 returns sum_l (A1 + 1 - A0) / 2 (every lane); mode 1 (one level) writes
// the two logits [b, 2, group] from lane 0.
// F32IN: fp32 features (compile time, so every level's loads issue back to back
// with no per-level dtype branch and its vmcnt(0) join), else bf16.
template <bool F32IN, int NLMAX = kMaxLevels>
__device__ __forceinline__ float patch_row_score(LevelPtrs lv, int nl, int64_t ld, size_t row,
                                                 const float4_t (&t0)[3], const float4_t (&t1)[3], int normalize,
                                                 int mode, int group, float* out, int lane) {
  // explicit FMAs and no other contraction: the same bits in every kernel that
  // inlines this (patch_scores_kernel, anomaly_map_kernel), whatever the compiler
  // would fuse in each context
#pragma clang fp contract(off)
  float4_t f[NLMAX][3];
#pragma unroll
  for (int l = 0; l < NLMAX; ++l) {
    if (l < nl) {
      if constexpr (F32IN) {
        const float* p = (const float*)lv.p[l] + row * ld;
#pragma unroll
        for (int c = 0; c < 3; ++c) f[l][c] = *(const float4_t*)(p + 256 * c + 4 * lane);
      } else {
        const uint16_t* p = (const uint16_t*)lv.p[l] + row * ld;
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
  for (int l = 0; l < NLMAX; ++l) {
    if (l < nl) {
      float ss = 0.f, a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = f[l][c][j];
          ss = fmaf(v, v, ss);
          a0 = fmaf(v, t0[c][j], a0);
          a1 = fmaf(v, t1[c][j], a1);
        }
      ss = wave_sum(ss);
      a0 = wave_sum(a0);
      a1 = wave_sum(a1);
      const float inv = normalize ? 1.0f / fmaxf(sqrtf(ss), 1e-12f) : 1.0f;
      const float A0 = 100.0f * (a0 * inv), A1 = 100.0f * (a1 * inv);
      if (mode == 0) {
        acc += (A1 + 1.0f - A0) / 2.0f;
      } else if (lane == 0) {
        const size_t base = (row / group) * 2 * group + row % group;
        out[base] = A0;
        out[base + group] = A1;
      }
    }
  }
  return acc;
}

// NLMAX: registers for that many levels (the level count at compile time where it is
// known: 4 levels of fp32 rows take 48 registers instead of kMaxLevels' 96, which
// lets 5 instead of 4 waves per SIMD keep their loads in flight).
template <bool F32IN, int NLMAX = kMaxLevels>
__global__ __launch_bounds__(256) void patch_scores_kernel(LevelPtrs lv, int nl,
                                                           int64_t ld, const float* T, int rows,
                                                           int normalize, int mode, int group,
                                                           float* out) {
  AACLIP_TRACE_SCOPE(TR_PATCH_SCORES);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float4_t t0[3], t1[3];
  load_anchors(T, t0, t1, lane);
  const float acc = patch_row_score<F32IN, NLMAX>(lv, nl, ld, (size_t)row, t0, t1, normalize, mode, group, out,
                                                  lane);
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

constexpr int kBand = 8;  // output rows per wave (= per workgroup); 4 and 8 measured equal, 2 / 16 slower
constexpr int kMaxC = 8;  // channels of the train branch (anchors), softmax over them

// Stage 2: one WAVE per (image, band of kBand output rows) — no workgroup barriers
// (a wave's LDS operations execute in order). The band's bilinear taps read source
// rows r_lo..r_hi only, so the wave stages the raw rows those need (their reflect
// neighbourhood x_lo..x_hi; a reflected index of that range stays inside it), x-blurs
// them, y-blurs rows r_lo..r_hi, and writes the band: 16-B stores of 4 consecutive
// pixels when S % 4 == 0, dwords otherwise (518 px, the reference's default).
// kornia 0.6.9 gaussian_blur2d semantics (separable, reflect border, x then y) and
// ATen's align_corners bilinear arithmetic (src = scale * dst rounded before the
// lambdas: no FMA contraction). K = ksize at compile time for the domains' 7 and 9
// (tap loads issued together), -1 = any ksize at run time, 0 = no blur.
// LDS: C * (2 * xrows + brows) * g floats, sized by the host for the band.
// The band body is a device function: blur_upsample_kernel and blur_upsample_score_kernel
// run it for one (image, band) per workgroup.
template <int C, int K>
__device__ __forceinline__ void blur_band(const float* grid, float* out, int b, int band, int g, int S,
                                          int ksize_rt, const Gauss& gw, int softmax, float scale, int xrows,
                                          int brows, float* smem, int lane) {
#pragma clang fp contract(off)
  const int ksize = K >= 0 ? K : ksize_rt;
  const int y0 = band * kBand;
  const int y1 = min(y0 + kBand, S);
  const int r_lo = (int)(scale * (float)y0);
  const int r_hi = min((int)(scale * (float)(y1 - 1)) + 1, g - 1);
  const int r = ksize / 2;  // (k-1)//2 left pad == k//2 for odd k
  const int x_lo = ksize > 0 ? max(0, r_lo - r) : r_lo;
  const int x_hi = ksize > 0 ? min(g - 1, r_hi + r) : r_hi;
  const int nx = x_hi - x_lo + 1, nb = r_hi - r_lo + 1;
  float* raw = smem;                  // [C][xrows][g]: rows x_lo..
  float* xbl = raw + C * xrows * g;   // [C][xrows][g]: x-blurred rows x_lo..
  float* bl = xbl + C * xrows * g;    // [C][brows][g]: blurred rows r_lo..
  if (lane < g) {
#pragma unroll
    for (int c = 0; c < C; ++c)
      for (int h = 0; h < nx; ++h) raw[(c * xrows + h) * g + lane] = grid[(((size_t)b * C + c) * g + x_lo + h) * g + lane];
  }
  __builtin_amdgcn_wave_barrier();
  const float* src = raw;  // rows relative to x_lo (== r_lo without blur)
  int sld = xrows;
  if (ksize > 0) {
    if (lane < g) {
      int xi[16];  // reflected column of each tap (shared by every row)
      const int kk = K > 0 ? K : ksize;
#pragma unroll
      for (int t = 0; t < (K > 0 ? K : 15); ++t)
        if (t < kk) xi[t] = reflect(lane + t - r, g);
#pragma unroll
      for (int c = 0; c < C; ++c)
        for (int h = 0; h < nx; ++h) {
          const float* row = raw + (c * xrows + h) * g;
          float acc = 0.f;
#pragma unroll
          for (int t = 0; t < (K > 0 ? K : 15); ++t)
            if (t < kk) acc += gw.w[t] * row[xi[t]];
          xbl[(c * xrows + h) * g + lane] = acc;
        }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int c = 0; c < C; ++c)
        for (int j = 0; j < nb; ++j) {
          const int h = r_lo + j;
          const float* col = xbl + c * xrows * g + lane;
          float acc = 0.f;
#pragma unroll
          for (int t = 0; t < (K > 0 ? K : 15); ++t)
            if (t < kk) acc += gw.w[t] * col[(reflect(h + t - r, g) - x_lo) * g];
          bl[(c * brows + j) * g + lane] = acc;
        }
    }
    __builtin_amdgcn_wave_barrier();
    src = bl;
    sld = brows;
  }
  // Upsample. Per lane 8 columns of a 512-column chunk (16-B path: 4 consecutive
  // pixels at 4*lane + 256*it; dword path: lane + 64*it). The column taps (ix0, ix1,
  // wx0, wx1) are computed once per chunk, and the horizontal blends
  // H_j(x) = wx0 * s[j][ix0] + wx1 * s[j][ix1] once per source row j: every output row
  // with iy0 = j reuses them (~15 rows per source row at 336 / 518 px), leaving
  // hy0 * H_iy0 + hy1 * H_iy1 per pixel -- ATen's expression, same order, same bits.
  const bool vec4 = (S & 3) == 0;
  for (int cx = 0; cx < S; cx += 512) {
    int o0[8], o1[8];
    float w0[8], w1[8];
    bool ok[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int x = cx + (vec4 ? 4 * lane + 256 * (p >> 2) + (p & 3) : lane + 64 * p);
      ok[p] = x < S;
      const float sx = scale * (float)x;
      const int ix0 = (int)sx;
      const int ix1 = ix0 + (ix0 < g - 1 ? 1 : 0);
      w1[p] = fminf(fmaxf(sx - (float)ix0, 0.f), 1.f);
      w0[p] = 1.0f - w1[p];
      o0[p] = ok[p] ? ix0 : 0;
      o1[p] = ok[p] ? ix1 : 0;
    }
    float H0[C][8], H1[C][8];
    auto hblend = [&](int jrow, float (&H)[C][8]) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float* sr = src + (c * sld + jrow) * g;
#pragma unroll
        for (int p = 0; p < 8; ++p) H[c][p] = w0[p] * sr[o0[p]] + w1[p] * sr[o1[p]];
      }
    };
    int cur0 = -1, cur1 = -1;
    for (int y = y0; y < y1; ++y) {
      // ATen upsample_bilinear2d, align_corners=True: src = scale * dst (fp32)
      const float sy = scale * (float)y;
      const int iy0 = (int)sy;
      const int iy1 = iy0 + (iy0 < g - 1 ? 1 : 0);
      const float hy1 = fminf(fmaxf(sy - (float)iy0, 0.f), 1.f), hy0 = 1.0f - hy1;
      if (iy0 != cur0) {
        if (iy0 == cur1) {
#pragma unroll
          for (int c = 0; c < C; ++c)
#pragma unroll
            for (int p = 0; p < 8; ++p) H0[c][p] = H1[c][p];
        } else {
          hblend(iy0 - r_lo, H0);
        }
        cur0 = iy0;
      }
      if (iy1 != cur1) {
        hblend(iy1 - r_lo, H1);
        cur1 = iy1;
      }
      float v[C][8];
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int p = 0; p < 8; ++p) v[c][p] = hy0 * H0[c][p] + hy1 * H1[c][p];
      if (C > 1 && softmax) {  // torch.softmax over the channel dim (forward_utils.py:214-215)
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          float m = v[0][p];
#pragma unroll
          for (int c = 1; c < C; ++c) m = fmaxf(m, v[c][p]);
          float sum = 0.f;
#pragma unroll
          for (int c = 0; c < C; ++c) {
            v[c][p] = expf(v[c][p] - m);
            sum += v[c][p];
          }
          const float inv = 1.0f / sum;
#pragma unroll
          for (int c = 0; c < C; ++c) v[c][p] *= inv;
        }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float* orow = out + (((size_t)b * C + c) * S + y) * S + cx;
        if (vec4) {
#pragma unroll
          for (int it = 0; it < 2; ++it)
            if (ok[4 * it])
              *(float4_t*)(orow + 4 * lane + 256 * it) =
                  float4_t{v[c][4 * it], v[c][4 * it + 1], v[c][4 * it + 2], v[c][4 * it + 3]};
        } else {
#pragma unroll
          for (int p = 0; p < 8; ++p)
            if (ok[p]) orow[lane + 64 * p] = v[c][p];
        }
      }
    }
  }
}

template <int C, int K>
__global__ __launch_bounds__(64) void blur_upsample_kernel(const float* grid, float* out, int g, int S,
                                                           int ksize_rt, Gauss gw, int softmax, float scale,
                                                           int xrows, int brows) {
  AACLIP_TRACE_SCOPE(TR_BLUR);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  blur_band<C, K>(grid, out, blockIdx.y, blockIdx.x, g, S, ksize_rt, gw, softmax, scale, xrows, brows, smem,
                  threadIdx.x);
}

// Stage 1 from GEMM partials (aaclip_gemm_scores wrote, per patch row and 32-column group
// q of each level, {||v||^2, v.t0, v.t1}): 8 lanes per patch row, 8 rows per wave. Lane j
// loads groups j, j+8, j+16 of every level (three float4 per level: each load instruction
// covers 128 contiguous bytes of 8 rows) and sums them, (g_j + g_j+8) + g_j+16; the 8 lane
// sums meet in three DPP butterfly steps inside the 8-lane group (quad swaps 1 and 2, then
// the half-row mirror i <-> 7 - i), a + b on one lane and b + a on its partner, so every lane
// ends with the same bits. Then patch_row_score's normalise + anchor arithmetic
// (normalize = 1). The det level (with_det) leaves d.t1 / ||d|| per row for the image
// score. 1.9 KB read per C2 patch row instead of 15 KB of projected rows. (Round 4 used one
// half-wave per row and five-step shuffle sums: 24 of 32 lanes loading, 75 LDS swizzles per
// 2 rows; 18.4 us at B = 32 in the bench's rocprofv3 trace.)
constexpr int kGroups = 768 / 32;  // 32-column groups per level
constexpr int kRowLanes = 8;       // lanes per patch row in partial_scores_kernel

template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  const float o = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF,
                                                                           true));
  return v + o;
}
__device__ __forceinline__ float sum8(float v) {
  v = dpp_add<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v = dpp_add<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  return dpp_add<0x141>(v);  // row_half_mirror
}

template <int NLMAX>
__global__ __launch_bounds__(256) void partial_scores_kernel(const float* __restrict__ part, int64_t ld, int nl,
                                                             int with_det, int rows, float* __restrict__ grid,
                                                             float* __restrict__ det_rows) {
#pragma clang fp contract(off)
  AACLIP_TRACE_SCOPE(TR_PARTIAL_SCORES);
  const int j = threadIdx.x & (kRowLanes - 1);
  const int row = blockIdx.x * (256 / kRowLanes) + (threadIdx.x / kRowLanes);
  if (row >= rows) return;  // all 8 lanes of a row leave together: the DPP steps stay inside a row's lanes
  const float* pr = part + (size_t)row * ld + 4 * j;
  const int nt = nl + with_det;
  float4_t v[NLMAX + 1][3];
#pragma unroll
  for (int l = 0; l <= NLMAX; ++l)
    if (l < nt) {
#pragma unroll
      for (int k = 0; k < 3; ++k) v[l][k] = *(const float4_t*)(pr + l * 4 * kGroups + 4 * kRowLanes * k);
    }
  float acc = 0.f;
#pragma unroll
  for (int l = 0; l <= NLMAX; ++l) {
    if (l < nt) {
      const float4_t t = (v[l][0] + v[l][1]) + v[l][2];
      const float ss = sum8(t[0]), a0 = sum8(t[1]), a1 = sum8(t[2]);
      const float inv = 1.0f / fmaxf(sqrtf(ss), 1e-12f);
      if (l < nl) {
        const float A0 = 100.0f * (a0 * inv), A1 = 100.0f * (a1 * inv);
        acc += (A1 + 1.0f - A0) / 2.0f;
      } else if (j == 0) {
        det_rows[row] = a1 * inv;  // normalize(d) . t1
      }
    }
  }
  if (j == 0) grid[row] = acc;
}

// Stage 2 + the image score: blur_upsample_kernel's bands, and the band-0 wave of each
// image also reduces its n_patch det rows (fixed order: lane-strided sums, then the wave
// butterfly) to score[b] = (mean_p normalize(d_p).t1 + 1) / 2 (test.py:83-84).
template <int K>
__global__ __launch_bounds__(64) void blur_upsample_score_kernel(const float* grid, float* out, int g, int S,
                                                                 int ksize_rt, Gauss gw, float scale, int xrows,
                                                                 int brows, const float* det_rows, int n_patch,
                                                                 float* score) {
#pragma clang fp contract(off)
  AACLIP_TRACE_SCOPE(TR_BLUR_SCORE);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (blockIdx.x == 0 && det_rows) {
    const float* d = det_rows + (size_t)blockIdx.y * n_patch;
    float t = 0.f;
    for (int p = threadIdx.x; p < n_patch; p += 64) t += d[p];
    t = wave_sum(t);
    if (threadIdx.x == 0) score[blockIdx.y] = (t / (float)n_patch + 1.0f) / 2.0f;
  }
  blur_band<1, K>(grid, out, blockIdx.y, blockIdx.x, g, S, ksize_rt, gw, 0, scale, xrows, brows, smem, threadIdx.x);
}

// Image score, stage 1: one workgroup per (image, chunk of kDetRows = 16 patch rows),
// 16 waves, one row each. Per row the wave reads the det_proj row, normalises it into
// its LDS slot; the 16 slots meet in a fixed tree per column,
// partial[b][chunk][j] = ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7)) + (same for s8..s15).
// (A one-pass form that also scored the level rows -- aaclip_anomaly_map_score --
// measured slower than two passes and was removed in round 5.)
constexpr int kDetRows = 16;

template <bool F32IN>
__global__ __launch_bounds__(64 * kDetRows) void map_det_kernel(int64_t ld, const void* det, int n_patch,
                                                                int normalize, float* partial, int nchunk) {
  AACLIP_TRACE_SCOPE(TR_DET);
  __shared__ float red[kDetRows][768];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = blockIdx.y, ch = blockIdx.x;
  {
    const int slot = wid;
    const int p = ch * kDetRows + slot;
    float4_t v[3] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    if (p < n_patch) {
      const size_t row = (size_t)b * n_patch + p;
      if constexpr (F32IN) {
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
      for (int c = 0; c < 3; ++c) v[c] = v[c] * inv;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) *(float4_t*)&red[slot][256 * c + 4 * lane] = v[c];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 768; j += 64 * kDetRows) {
    float h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = red[2 * i][j] + red[2 * i + 1][j];
    partial[((size_t)b * nchunk + ch) * 768 + j] =
        ((h[0] + h[1]) + (h[2] + h[3])) + ((h[4] + h[5]) + (h[6] + h[7]));
  }
}

// Image score, stage 2: det[b] = sum(partials) / n_patch; score = (det.T1 + 1)/2.
// One thread per column (768 = 12 waves per image); the partials are summed in chunk
// order, their loads issued 8 at a time (a chain of 36 dependent loads was latency-bound).
__global__ __launch_bounds__(768) void det_finalize_kernel(const float* partial, int nchunk,
                                                           int n_patch, const float* T,
                                                           float* det, float* score) {
  AACLIP_TRACE_SCOPE(TR_DET);
  __shared__ float red[12];
  const int b = blockIdx.x, j = threadIdx.x;
  const float* pp = partial + (size_t)b * nchunk * 768 + j;
  float s = 0.f;
  for (int c0 = 0; c0 < nchunk; c0 += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = c0 + i < nchunk ? pp[(size_t)(c0 + i) * 768] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (c0 + i < nchunk) s += v[i];
  }
  const float m = s / (float)n_patch;
  if (det) det[(size_t)b * 768 + j] = m;
  if (!score) return;  // block-uniform
  float dot = wave_sum(m * T[2 * j + 1]);
  if ((j & 63) == 0) red[j >> 6] = dot;
  __syncthreads();
  if (j == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 12; i += 4) t += (red[i] + red[i + 1]) + (red[i + 2] + red[i + 3]);
    score[b] = (t + 1.0f) / 2.0f;
  }
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
  const int grp = mode == 1 ? group : 1;
  hipStream_t s = (hipStream_t)stream;
  if (in_dtype == AACLIP_F32) {
    if (n_levels <= 4)  // C2's 4 levels (and the single-level calls)
      patch_scores_kernel<true, 4><<<ceil_div(rows, 4), 256, 0, s>>>(lv, n_levels, ld, T, rows, normalize, mode,
                                                                    grp, out);
    else
      patch_scores_kernel<true><<<ceil_div(rows, 4), 256, 0, s>>>(lv, n_levels, ld, T, rows, normalize, mode, grp,
                                                                 out);
  } else {
    if (n_levels <= 4)
      patch_scores_kernel<false, 4><<<ceil_div(rows, 4), 256, 0, s>>>(lv, n_levels, ld, T, rows, normalize, mode,
                                                                     grp, out);
    else
      patch_scores_kernel<false><<<ceil_div(rows, 4), 256, 0, s>>>(lv, n_levels, ld, T, rows, normalize, mode, grp,
                                                                  out);
  }
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

// LDS bytes stage 2 needs for C channels: the source rows a band's taps can reach.
static size_t blur_upsample_lds(int C, int g, int S, int ksize) {
  const float scale = (float)(g - 1) / (float)(S - 1);
  const int span = (int)(scale * (float)(kBand - 1)) + 4;  // source rows a band's taps can reach (+1 margin)
  const int brows = min(g, span);
  const int xrows = min(g, brows + 2 * (ksize / 2));
  return (size_t)C * (2 * xrows + brows) * g * sizeof(float);
}

// Every argument check of aaclip_blur_upsample, so the multi-launch entry points can
// reject a bad call before their first launch (no half-written map on an error).
static bool blur_upsample_args_ok(int channels, int g, int out_size, int ksize) {
  return channels >= 1 && channels <= kMaxC && g >= 2 && g <= 64 && out_size >= 2 && ksize >= 0 && ksize <= 15 &&
         (ksize == 0 || (ksize % 2 == 1 && ksize / 2 < g)) && blur_upsample_lds(channels, g, out_size, ksize) <= 64 * 1024;
}

// Launch stage 2 for (C, ksize): rows of LDS the band needs, sized on the host.
template <int C>
int launch_blur_upsample(const float* grid, float* out, int batch, int g, int S, int ksize, const Gauss& gw,
                         int softmax, float scale, hipStream_t s) {
  const int span = (int)(scale * (float)(kBand - 1)) + 4;  // source rows a band's taps can reach (+1 margin)
  const int brows = min(g, span);
  const int xrows = min(g, brows + 2 * (ksize / 2));
  const size_t lds = blur_upsample_lds(C, g, S, ksize);
  if (lds > 64 * 1024) return AACLIP_ERR_ARG;
  const dim3 grd(ceil_div(S, kBand), batch);
#define BU_LAUNCH(K) \
  blur_upsample_kernel<C, K><<<grd, 64, lds, s>>>(grid, out, g, S, ksize, gw, softmax, scale, xrows, brows)
  if (ksize == 0) BU_LAUNCH(0);
  else if (ksize == 7) BU_LAUNCH(7);
  else if (ksize == 9) BU_LAUNCH(9);
  else BU_LAUNCH(-1);
#undef BU_LAUNCH
  return AACLIP_OK;
}

extern "C" int aaclip_blur_upsample(const float* grid, float* out, int batch, int channels, int g,
                                    int out_size, int ksize, float sigma, int softmax,
                                    void* stream) {
  AACLIP_REQUIRE(grid && out && batch > 0);
  AACLIP_REQUIRE(blur_upsample_args_ok(channels, g, out_size, ksize));
  const Gauss gw = ksize > 0 ? gaussian_weights(ksize, sigma) : Gauss{};
  const float scale = (float)(g - 1) / (float)(out_size - 1);
  hipStream_t s = (hipStream_t)stream;
  int rc = AACLIP_ERR_ARG;
  switch (channels) {
    case 1: rc = launch_blur_upsample<1>(grid, out, batch, g, out_size, ksize, gw, softmax, scale, s); break;
    case 2: rc = launch_blur_upsample<2>(grid, out, batch, g, out_size, ksize, gw, softmax, scale, s); break;
    case 3: rc = launch_blur_upsample<3>(grid, out, batch, g, out_size, ksize, gw, softmax, scale, s); break;
    case 4: rc = launch_blur_upsample<4>(grid, out, batch, g, out_size, ksize, gw, softmax, scale, s); break;
    case 5: rc = launch_blur_upsample<5>(grid, out, batch, g, out_size, ksize, gw, softmax, scale, s); break;
    case 6: rc = launch_blur_upsample<6>(grid, out, batch, g, out_size, ksize, gw, softmax, scale, s); break;
    case 7: rc = launch_blur_upsample<7>(grid, out, batch, g, out_size, ksize, gw, softmax, scale, s); break;
    default: rc = launch_blur_upsample<8>(grid, out, batch, g, out_size, ksize, gw, softmax, scale, s); break;
  }
  if (rc) return rc;
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_anomaly_map(int in_dtype, const void* const* levels, int n_levels, int64_t ld,
                                  const float* T, int batch, int g, int channels, int normalize,
                                  int out_size, int ksize, float sigma, float* grid_ws,
                                  float* out, void* stream) {
  AACLIP_REQUIRE(grid_ws && out && batch > 0);
  AACLIP_REQUIRE(blur_upsample_args_ok(1, g, out_size, ksize));  // before the first launch
  int rc = aaclip_patch_scores(in_dtype, levels, n_levels, ld, T, batch * g * g, channels,
                               normalize, 0, 0, grid_ws, stream);
  if (rc) return rc;
  return aaclip_blur_upsample(grid_ws, out, batch, 1, g, out_size, ksize, sigma, 0, stream);
}

extern "C" int aaclip_anomaly_map_partials(const float* part, int64_t ld_part, int n_levels, int with_det,
                                           int batch, int g, int out_size, int ksize, float sigma, float* grid_ws,
                                           float* det_ws, float* out, float* score, void* stream) {
  AACLIP_REQUIRE(part && grid_ws && out && batch > 0 && n_levels >= 1 && n_levels <= kMaxLevels);
  AACLIP_REQUIRE(with_det == 0 || (with_det == 1 && det_ws && score));
  AACLIP_REQUIRE(ld_part >= (int64_t)(n_levels + with_det) * 4 * kGroups && ld_part % 4 == 0);
  AACLIP_REQUIRE(((uintptr_t)part % 16) == 0);
  AACLIP_REQUIRE(blur_upsample_args_ok(1, g, out_size, ksize));  // before the first launch
  const int rows = batch * g * g;
  hipStream_t s = (hipStream_t)stream;
  if (n_levels <= 4)
    partial_scores_kernel<4><<<ceil_div(rows, 256 / kRowLanes), 256, 0, s>>>(part, ld_part, n_levels, with_det, rows, grid_ws,
                                                                det_ws);
  else
    partial_scores_kernel<kMaxLevels><<<ceil_div(rows, 256 / kRowLanes), 256, 0, s>>>(part, ld_part, n_levels, with_det, rows,
                                                                         grid_ws, det_ws);
  AACLIP_CHECK_LAUNCH();
  const Gauss gw = ksize > 0 ? gaussian_weights(ksize, sigma) : Gauss{};
  const float scale = (float)(g - 1) / (float)(out_size - 1);
  const int span = (int)(scale * (float)(kBand - 1)) + 4;  // as launch_blur_upsample
  const int brows = min(g, span);
  const int xrows = min(g, brows + 2 * (ksize / 2));
  const size_t lds = blur_upsample_lds(1, g, out_size, ksize);
  const dim3 grd(ceil_div(out_size, kBand), batch);
  const float* dr = with_det ? det_ws : nullptr;
#define BS_LAUNCH(K)                                                                                      \
  blur_upsample_score_kernel<K><<<grd, 64, lds, s>>>(grid_ws, out, g, out_size, ksize, gw, scale, xrows, brows, \
                                                     dr, g * g, score)
  if (ksize == 0) BS_LAUNCH(0);
  else if (ksize == 7) BS_LAUNCH(7);
  else if (ksize == 9) BS_LAUNCH(9);
  else BS_LAUNCH(-1);
#undef BS_LAUNCH
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_image_score(int in_dtype, const void* det_raw, int64_t ld, const float* T,
                                  int batch, int n_patch, int channels, int normalize,
                                  float* partial, float* det, float* score, void* stream) {
  AACLIP_REQUIRE(in_dtype == AACLIP_F32 || in_dtype == AACLIP_BF16);
  AACLIP_REQUIRE(det_raw && partial && batch > 0 && n_patch > 0);
  AACLIP_REQUIRE((T && score) || (!T && !score && det));
  AACLIP_REQUIRE(channels == 768 && ld >= channels && ld % 4 == 0);
  const int nchunk = ceil_div(n_patch, kDetRows);
  const dim3 grd(nchunk, batch);
  if (in_dtype == AACLIP_F32)
    map_det_kernel<true><<<grd, 1024, 0, (hipStream_t)stream>>>(ld, det_raw, n_patch, normalize, partial, nchunk);
  else
    map_det_kernel<false><<<grd, 1024, 0, (hipStream_t)stream>>>(ld, det_raw, n_patch, normalize, partial, nchunk);
  AACLIP_CHECK_LAUNCH();
  det_finalize_kernel<<<batch, 768, 0, (hipStream_t)stream>>>(partial, nchunk, n_patch, T, det,
                                                              score);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

AACLIP_TRACE_SETTER(trace_set_anomaly_map)
