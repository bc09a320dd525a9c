// Test-time preprocessing on device: the reference's
// transform_x = Resize((S,S), BICUBIC) -> ToTensor -> Normalize(CLIP) and
// transform_mask = Resize((S,S), NEAREST) -> ToTensor -> != 0
// (dataset/__init__.py:127-143, applied at :152-162). torchvision hands PIL
// images to Pillow, so the arithmetic restated here is Pillow's, bit for bit:
//
//   * plan (host, double precision, same expression order as Pillow's
//     precompute_coeffs / normalize_coeffs_8bpc): per output coordinate the
//     first source tap and the tap count, and int32 weights with 22 fraction
//     bits (a = -0.5 cubic, support 2 * max(in/out, 1), normalised to sum 1);
//   * kernels: two 8-bit passes, horizontal first, each value of the
//     intermediate clipped exactly like Pillow's intermediate image; the
//     vertical pass writes float32 (v / 255 - mean) / std (IEEE division, as
//     torch's div_) into the CHW plane layout the visual embed reads. Default
//     (caller workspace): resample_h_kernel over every source row into a uint8
//     intermediate, then resample_v_kernel. Without a workspace: one tiled
//     kernel per (TY x TX output tile) that resamples the source rows its
//     vertical taps touch into an LDS strip and runs the vertical taps there.
//   * masks: nearest index tables (Pillow's accumulated xo += in/out) and a
//     one-pass gather writing (v != 0) as float32.
//
// HBM bytes per image: H*W*3 read + 3*S*S*4 written (+ the tiny plans).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"

namespace {

constexpr int PREC = 22;  // Pillow PRECISION_BITS for 8-bit images
constexpr int NT = 256;   // threads per workgroup

__device__ __forceinline__ uint32_t clip8(int v) {
  v >>= PREC;  // arithmetic shift, as Pillow's lookup index
  return (uint32_t)min(max(v, 0), 255);
}

struct PrepArgs {
  const uint8_t* src;
  int64_t img_stride, pitch;
  int in_h, in_w, S, ty, tx;
  const int32_t *xb, *xk, *yb, *yk;
  int kx, ky;
  float mean[3], stdv[3];
  float* out;
  int tiles_x, tiles_y, max_rows, max_cols, srow;
};

// One workgroup = ty output rows x tx output columns of one image.
// STAGED: the source patch the tile touches (rows r0..r1, columns c0..c1) is
// first copied into LDS with aligned dword loads (every load of the tile in
// flight at once, coalesced along the row), so the tap loops below read LDS
// instead of waiting on one scattered byte load per tap. Direct: taps read the
// source through L1/L2 (only for extreme downscales whose patch exceeds LDS).
template <bool STAGED>
__global__ __launch_bounds__(NT) void bicubic_normalize_kernel(PrepArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  // STAGED layout: tap weights of the tile's columns [tx][kx] and rows [ty][ky] (int32),
  // then the horizontal-pass strip [max_rows][tx][3], then the source patch [max_rows][srow]
  int32_t* kxs = (int32_t*)lds;
  int32_t* kys = kxs + (STAGED ? a.tx * a.kx : 0);
  uint8_t* strip = (uint8_t*)(kys + (STAGED ? a.ty * a.ky : 0));
  uint8_t* patch = strip + ((a.max_rows * a.tx * 3 + 15) & ~15);
  const int tile = blockIdx.x;
  const int b = blockIdx.y;
  const int txi = tile % a.tiles_x, tyi = tile / a.tiles_x;
  const int x0 = txi * a.tx, y0 = tyi * a.ty;
  const int y1 = min(y0 + a.ty, a.S), x1 = min(x0 + a.tx, a.S);
  const int r0 = a.yb[2 * y0];
  // r1 - r0 <= (ty-1)*in/S + 2*support + 1 <= max_rows (strip_bound); the min only guards LDS
  const int nrows = min(a.yb[2 * (y1 - 1)] + a.yb[2 * (y1 - 1) + 1] - r0, a.max_rows);
  const uint8_t* img = a.src + (size_t)b * a.img_stride;
  const int c0 = a.xb[2 * x0];

  if constexpr (STAGED) {
    const int ncols = min(a.xb[2 * (x1 - 1)] + a.xb[2 * (x1 - 1) + 1] - c0, a.max_cols);
    const int ndw = (ncols * 3 + 3 + 3) >> 2;  // dwords per row incl. the <= 3-byte alignment shift
    // 8 independent loads in flight per thread before the first LDS write (a
    // one-load-per-iteration loop serialises on HBM latency: measured 4x slower)
    constexpr int U = 8;
    const int total = nrows * ndw;
    for (int i0 = threadIdx.x; i0 < total; i0 += NT * U) {
      uint32_t v[U];
      int dst[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * NT;
        dst[u] = -1;
        if (i < total) {
          const int r = i / ndw, d = i - r * ndw;
          const uintptr_t row = (uintptr_t)(img + (size_t)(r0 + r) * a.pitch + (size_t)c0 * 3);
          const uintptr_t base = row & ~(uintptr_t)3;  // aligned dwords never cross a page: no fault past the end
          if ((int)(row - base) + ncols * 3 > d * 4) {
            v[u] = *(const uint32_t*)(base + 4 * (uintptr_t)d);
            dst[u] = r * a.srow + 4 * d;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (dst[u] >= 0) *(uint32_t*)(patch + dst[u]) = v[u];
    }
    for (int i = threadIdx.x; i < (x1 - x0) * a.kx; i += NT) kxs[i] = a.xk[(size_t)x0 * a.kx + i];
    for (int i = threadIdx.x; i < (y1 - y0) * a.ky; i += NT) kys[i] = a.yk[(size_t)y0 * a.ky + i];
    __syncthreads();
  }

  // pass 1: horizontal taps for source rows r0..r1 of this tile's columns
  for (int i = threadIdx.x; i < nrows * a.tx; i += NT) {
    const int r = i / a.tx, xo = i - r * a.tx, x = x0 + xo;
    if (x >= x1) continue;
    const int xmin = a.xb[2 * x], n = a.xb[2 * x + 1];
    const int32_t* k = STAGED ? kxs + xo * a.kx : a.xk + (size_t)x * a.kx;
    const uint8_t* p;
    if constexpr (STAGED) {
      const uintptr_t row = (uintptr_t)(img + (size_t)(r0 + r) * a.pitch + (size_t)c0 * 3);
      p = patch + r * a.srow + (int)(row & 3) + (xmin - c0) * 3;
    } else {
      p = img + (size_t)(r0 + r) * a.pitch + (size_t)xmin * 3;
    }
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
#pragma unroll 4
    for (int t = 0; t < n; ++t) {
      const int w = k[t];
      s0 += (int)p[3 * t + 0] * w;
      s1 += (int)p[3 * t + 1] * w;
      s2 += (int)p[3 * t + 2] * w;
    }
    uint8_t* d = strip + (r * a.tx + xo) * 3;
    d[0] = (uint8_t)clip8(s0);
    d[1] = (uint8_t)clip8(s1);
    d[2] = (uint8_t)clip8(s2);
  }
  __syncthreads();

  // pass 2: vertical taps out of LDS, normalise, CHW fp32 stores (consecutive x per wave)
  const size_t plane = (size_t)a.S * a.S;
  float* ob = a.out + (size_t)b * 3 * plane;
  for (int i = threadIdx.x; i < (y1 - y0) * a.tx; i += NT) {
    const int yo = i / a.tx, xo = i - yo * a.tx, x = x0 + xo, y = y0 + yo;
    if (x >= x1) continue;
    const int ymin = a.yb[2 * y] - r0, n = a.yb[2 * y + 1];
    const int32_t* k = STAGED ? kys + yo * a.ky : a.yk + (size_t)y * a.ky;
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
#pragma unroll 4
    for (int t = 0; t < n; ++t) {
      const int w = k[t];
      const uint8_t* q = strip + ((ymin + t) * a.tx + xo) * 3;
      s0 += (int)q[0] * w;
      s1 += (int)q[1] * w;
      s2 += (int)q[2] * w;
    }
    const size_t o = (size_t)y * a.S + x;
    ob[o] = ((float)clip8(s0) / 255.0f - a.mean[0]) / a.stdv[0];
    ob[plane + o] = ((float)clip8(s1) / 255.0f - a.mean[1]) / a.stdv[1];
    ob[2 * plane + o] = ((float)clip8(s2) / 255.0f - a.mean[2]) / a.stdv[2];
  }
}

// ---- two-pass path (default when the caller passes a workspace): full-occupancy
// passes with no per-tile row overlap. B=32 1024^2 -> 336 (profiles/r02/preprocess.txt):
// H 51 us + V 18 us (round 1: 91 + 33; single tiled kernel: 152 us). H is VALU-bound
// (14 tap slots x 3 channels of byte * weight MACs per output, as SDWA byte-select
// v_mul_i32_i24 + v_add3). Pass H resamples every source row into the uint8
// intermediate image tmp [B][in_h][S][3] (Pillow's clipped intermediate); pass V
// runs the vertical taps out of tmp (L2-resident rows, each read by ~ky/scale
// output rows) and writes the normalised CHW fp32 output.
struct HArgs {
  const uint8_t* src;
  int64_t img_stride, pitch;
  int in_h, in_w, S, rows;  // rows: source rows per workgroup
  const int32_t *xb, *xk;
  int kx, srow, tstride;    // tstride: bytes per intermediate row (S*3 rounded up to 16)
  uint8_t* tmp;
};

constexpr int HK = 16;  // max taps held in registers by the horizontal pass (kx <= HK)

// blockDim = 64 * ceil(S / 64): thread x owns output column x, its taps live in
// registers for all the workgroup's rows; the rows are staged in LDS by aligned
// 16-byte loads (all of a thread's loads in flight) and read back as aligned dwords.
// K tap slots per column (tap_slots), unpredicated: the plan zero-fills taps past
// each column's count (and srow carries 3*HK spare bytes), so the short columns add
// 0 * byte instead of branching per tap (a per-lane `t < n` test serialised the LDS reads).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 24-bit signed view of a tap weight. Pillow's 8-bit weights are round(v * 2^22)
// with |v| < 2 (normalised cubic taps), so the value is unchanged, and the
// compiler can then use the full-rate v_mad_i32_i24 for byte * weight instead of
// the quarter-rate 32-bit v_mul_lo_u32 (the product fits 31 bits either way).
__device__ __forceinline__ int tap24(int w) { return (w << 8) >> 8; }

template <int K>
__global__ __launch_bounds__(1024) void resample_h_kernel(HArgs a) {
  const int nt = blockDim.x;
  extern __shared__ __attribute__((aligned(16))) uint8_t rows[];  // [rows][srow]
  const int b = blockIdx.y;
  const int r0 = blockIdx.x * a.rows, nr = min(a.rows, a.in_h - r0);
  const uint8_t* img = a.src + (size_t)b * a.img_stride;
  // staging: 16-byte aligned quads (an aligned quad holding a byte of the row never
  // crosses a page: no fault past the end), all of a thread's loads in flight
  // before its LDS writes. (row, quad) advances by nt without a per-load division.
  const int nq = (a.in_w * 3 + 15 + 15) >> 4;  // quads per row incl. the <= 15-byte alignment shift
  constexpr int U = 4;
  int r = threadIdx.x / nq, q = threadIdx.x - r * nq;
  const int rstep = nt / nq, qstep = nt - rstep * nq;
  while (r < nr) {
    u32x4 v[U];
    int dst[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // unconditional load (a past-the-end slot re-reads the row's first quad) so the
      // compiler issues all U loads back to back; only the LDS store is predicated
      const int rr = min(r, nr - 1);
      const uint8_t* row = img + (size_t)(r0 + rr) * a.pitch;
      const int mis = (int)((uintptr_t)row & 15);
      const bool ok = r < nr && 16 * q < mis + a.in_w * 3;
      v[u] = *(const u32x4*)(row - mis + (ok ? 16 * q : 0));
      dst[u] = ok ? rr * a.srow + 16 * q : -1;
      r += rstep;
      q += qstep;
      if (q >= nq) {
        q -= nq;
        ++r;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) asm volatile("" : "+v"(v[u]));  // keep every load ahead of the stores
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (dst[u] >= 0) *(u32x4*)(rows + dst[u]) = v[u];
  }
  __syncthreads();
  const int x = threadIdx.x;
  if (x < a.S) {
    const int xmin = a.xb[2 * x];
    int w[K];
#pragma unroll
    for (int t = 0; t < K; ++t) {  // clamped unconditional loads (all in flight), zero past kx (uniform)
      const int wt = tap24(a.xk[(size_t)x * a.kx + min(t, a.kx - 1)]);
      w[t] = t < a.kx ? wt : 0;
    }
    // the column's 3K-byte tap window starts at an arbitrary byte: read the dwords
    // covering it at dword-aligned addresses and realign with v_alignbyte (byte-
    // misaligned wide LDS reads measured ~33 LDS cycles per instruction: the pass
    // was LDS-bound), then the byte picks below are compile-time (SDWA operands)
    constexpr int NW = (3 * K + 3) / 4;  // window dwords
    for (int r = 0; r < nr; ++r) {
      const uintptr_t row = (uintptr_t)(img + (size_t)(r0 + r) * a.pitch);
      const int off = r * a.srow + (int)(row & 15) + xmin * 3;
      const uint32_t* pd = (const uint32_t*)(rows + (off & ~3));
      const uint32_t sh = (uint32_t)(off & 3);
      uint32_t dw[NW + 1], win[NW];
#pragma unroll
      for (int j = 0; j <= NW; ++j) dw[j] = pd[j];
#pragma unroll
      for (int j = 0; j < NW; ++j) win[j] = __builtin_amdgcn_alignbyte(dw[j + 1], dw[j], sh);
      auto byte = [&](int i) { return (int)((win[i >> 2] >> (8 * (i & 3))) & 255); };
      int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
#pragma unroll
      for (int t = 0; t < K; ++t) {
        s0 += byte(3 * t + 0) * w[t];
        s1 += byte(3 * t + 1) * w[t];
        s2 += byte(3 * t + 2) * w[t];
      }
      uint8_t* d = a.tmp + ((size_t)b * a.in_h + r0 + r) * a.tstride + x * 3;
      d[0] = (uint8_t)clip8(s0);
      d[1] = (uint8_t)clip8(s1);
      d[2] = (uint8_t)clip8(s2);
    }
  }
}

// one thread = 4 consecutive output pixels (12 intermediate bytes = 3 aligned
// dwords per tap) of one output row; the (row, pixel-quad) pairs of an image are
// numbered consecutively over 256-thread blocks, so every lane has work (a block
// per output row left a third of the lanes idle at S = 336).
// K > 0: K unpredicated taps, every tap row's loads in flight at once (the plan
// zero-fills taps past each row's count; rows past the image are clamped, their
// weight is 0). K == 0: the row's own tap count, a loop (ky > 16 downscales).
struct VArgs {
  const uint8_t* tmp;
  int in_h, S, tstride;
  const int32_t *yb, *yk;
  int ky;
  float mean[3], stdv[3];
  float* out;
};

template <int K>
__global__ __launch_bounds__(256) void resample_v_kernel(VArgs a) {
  const uint8_t* __restrict__ tmp = a.tmp;
  const int in_h = a.in_h, S = a.S, tstride = a.tstride, ky = a.ky;
  const int32_t* __restrict__ yb = a.yb;
  const int32_t* __restrict__ yk = a.yk;
  float* __restrict__ out = a.out;
  const int q4 = (S + 3) >> 2;
  const int i = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  const int y = i / q4, x0 = (i - y * q4) * 4;
  // normalisation table: lut[c][v] = (v / 255 - mean[c]) / std[c], the same IEEE
  // expression per entry, so a lookup equals computing it per pixel (3 x 256 entries
  // per block instead of 2 divisions for each of a thread's 12 outputs)
  __shared__ float lut[3][256];
#pragma unroll
  for (int c = 0; c < 3; ++c) lut[c][threadIdx.x] = ((float)threadIdx.x / 255.0f - a.mean[c]) / a.stdv[c];
  __syncthreads();
  if (y >= S) return;
  const int ymin = yb[2 * y];
  const int32_t* k = yk + (size_t)y * ky;
  const uint8_t* col = tmp + (size_t)b * in_h * tstride + x0 * 3;  // x0*3 % 12 == 0, tstride % 16 == 0
  int acc[12];
#pragma unroll
  for (int e = 0; e < 12; ++e) acc[e] = 1 << (PREC - 1);
  auto tap = [&](uint32_t d0, uint32_t d1, uint32_t d2, int w) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[e] += (int)((d0 >> (8 * e)) & 255) * w;
      acc[4 + e] += (int)((d1 >> (8 * e)) & 255) * w;
      acc[8 + e] += (int)((d2 >> (8 * e)) & 255) * w;
    }
  };
  if constexpr (K > 0) {
    int w[K];
    uint32_t d[K][3];
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const int wt = tap24(k[min(t, ky - 1)]);
      w[t] = t < ky ? wt : 0;
      const uint32_t* q = (const uint32_t*)(col + (size_t)min(ymin + t, in_h - 1) * tstride);
      d[t][0] = q[0];
      d[t][1] = q[1];
      d[t][2] = q[2];
    }
#pragma unroll
    for (int t = 0; t < K; ++t) tap(d[t][0], d[t][1], d[t][2], w[t]);
  } else {
    const int n = yb[2 * y + 1];
#pragma unroll 2
    for (int t = 0; t < n; ++t) {
      const uint32_t* q = (const uint32_t*)(col + (size_t)(ymin + t) * tstride);
      tap(q[0], q[1], q[2], tap24(k[t]));
    }
  }
  const size_t plane = (size_t)S * S, o = (size_t)b * 3 * plane + (size_t)y * S + x0;
  float v[3][4];
#pragma unroll
  for (int px = 0; px < 4; ++px)
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c][px] = lut[c][clip8(acc[3 * px + c])];
  if ((S & 3) == 0) {  // 16-byte aligned quads: one dwordx4 store per plane
#pragma unroll
    for (int c = 0; c < 3; ++c)
      *(float4*)(out + o + c * plane) = make_float4(v[c][0], v[c][1], v[c][2], v[c][3]);
  } else {
#pragma unroll
    for (int px = 0; px < 4; ++px)
      if (x0 + px < S)
#pragma unroll
        for (int c = 0; c < 3; ++c) out[o + c * plane + px] = v[c][px];
  }
}

__global__ __launch_bounds__(NT) void nearest_mask_kernel(const uint8_t* __restrict__ src, int64_t img_stride,
                                                          int64_t pitch, const int32_t* __restrict__ xi,
                                                          const int32_t* __restrict__ yi, int S,
                                                          float* __restrict__ out) {
  const int b = blockIdx.y;
  const size_t plane = (size_t)S * S;
  for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < plane; i += (size_t)gridDim.x * NT) {
    const int y = (int)(i / S), x = (int)(i - (size_t)y * S);
    const uint8_t v = src[(size_t)b * img_stride + (size_t)yi[y] * pitch + xi[x]];
    out[(size_t)b * plane + i] = v != 0 ? 1.0f : 0.0f;
  }
}

double bicubic_filter(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

int bicubic_ksize(int in_size, int out_size) {
  double filterscale = (double)in_size / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  return (int)ceil(2.0 * filterscale) * 2 + 1;
}

// source rows (or columns) the taps of `t` consecutive output coordinates can touch:
// (t-1)*in/S + 2*support + 1 <= ceil((t-1)*in/S) + ksize + 2
int strip_bound(int in_size, int S, int t, int ksize) {
  const double scale = (double)in_size / S;
  return min(in_size, (int)ceil((t - 1) * scale) + ksize + 2);
}

constexpr int STAGED_LDS = 64 * 1024;   // staged tiles: patch + strip
constexpr int DIRECT_LDS = 128 * 1024;  // direct tiles: strip only

}  // namespace

extern "C" int aaclip_bicubic_taps(int in_size, int out_size, int* ksize) {
  AACLIP_REQUIRE(in_size > 0 && out_size > 0 && ksize);
  *ksize = bicubic_ksize(in_size, out_size);
  return AACLIP_OK;
}

extern "C" int aaclip_bicubic_plan(int in_size, int out_size, int32_t* bounds, int32_t* coeffs, int ksize) {
#pragma clang fp contract(off)
  AACLIP_REQUIRE(in_size > 0 && out_size > 0);
  const int need = bicubic_ksize(in_size, out_size);
  AACLIP_REQUIRE(bounds && coeffs && ksize >= need);
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  std::vector<double> w(need);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      w[x] = bicubic_filter((x + xmin - center + 0.5) * ss);
      ww += w[x];
    }
    int32_t* k = coeffs + (size_t)xx * ksize;
    for (int x = 0; x < ksize; ++x) {
      if (x >= xmax) {
        k[x] = 0;
        continue;
      }
      const double v = ww != 0.0 ? w[x] / ww : w[x];
      k[x] = v < 0 ? (int32_t)(-0.5 + v * (1 << PREC)) : (int32_t)(0.5 + v * (1 << PREC));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return AACLIP_OK;
}

extern "C" int aaclip_nearest_plan(int in_size, int out_size, int32_t* index) {
#pragma clang fp contract(off)
  AACLIP_REQUIRE(in_size > 0 && out_size > 0 && index);
  const double a = (double)in_size / out_size;
  double xo = a * 0.5;
  for (int x = 0; x < out_size; ++x) {
    index[x] = xo < 0.0 ? -1 : (int32_t)xo;
    xo += a;
  }
  for (int x = 0; x < out_size; ++x) AACLIP_REQUIRE(index[x] >= 0 && index[x] < in_size);
  return AACLIP_OK;
}

namespace {
int tmp_stride(int S) { return (S * 3 + 12 + 15) & ~15; }  // + 12: the last 4-pixel group's dwords
constexpr int H_LDS = 64 * 1024;
// bytes of LDS the horizontal pass needs for `rows` source rows (0 = does not fit)
int h_lds_bytes(int in_w, int rows, int* srow) {
  *srow = (in_w * 3 + 15 + 15 + 3 * HK + 8 + 15) & ~15;  // + 3*HK + 8: zero-weight taps / read tail
  const int64_t bytes = (int64_t)rows * *srow;
  return bytes <= H_LDS ? (int)bytes : 0;
}

// register tap slots for one axis: an upper bound on every output coordinate's tap
// count (xmax - xmin <= floor(2 * support) + 1; + 1 more against rounding in the
// plan's double arithmetic), at most the plan's ksize, rounded up to even; 0 when it
// exceeds HK (the fixed-slot kernels do not apply). Slots past a coordinate's count
// carry weight 0 in the plan, so fewer slots than ksize lose nothing.
int tap_slots(int in_size, int out_size, int ksize) {
  const double scale = (double)in_size / out_size;
  const double support = 2.0 * (scale < 1.0 ? 1.0 : scale);
  const int n = std::min(ksize, (int)floor(2.0 * support) + 2);
  const int k = std::max(4, (n + 1) & ~1);
  return k <= HK ? k : 0;
}

template <int K>
int launch_h(const HArgs& h, dim3 grid, int block, int lds, hipStream_t st) {
  static unsigned done = 0;
  if (!lds_attr_once((const void*)resample_h_kernel<K>, H_LDS, done)) return AACLIP_ERR_LAUNCH;
  resample_h_kernel<K><<<grid, block, lds, st>>>(h);
  return AACLIP_OK;
}
}  // namespace

extern "C" int aaclip_preprocess_workspace(int batch, int in_h, int in_w, int out_size, size_t* bytes) {
  AACLIP_REQUIRE(batch >= 0 && in_h > 0 && in_w > 0 && out_size > 0 && bytes);
  *bytes = (size_t)batch * in_h * tmp_stride(out_size);  // the uint8 intermediate image of the two-pass path
  return AACLIP_OK;
}

extern "C" int aaclip_preprocess_images(const uint8_t* src, int64_t img_stride, int64_t row_pitch, int batch,
                                        int in_h, int in_w, const int32_t* x_bounds, const int32_t* x_coeffs,
                                        int kx, const int32_t* y_bounds, const int32_t* y_coeffs, int ky,
                                        int out_size, const float* mean_std, float* out, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  AACLIP_REQUIRE(src && x_bounds && x_coeffs && y_bounds && y_coeffs && out && batch >= 0);
  AACLIP_REQUIRE(in_h > 0 && in_w > 0 && out_size > 0 && row_pitch >= (int64_t)in_w * 3);
  AACLIP_REQUIRE(img_stride >= row_pitch * in_h || batch <= 1);
  AACLIP_REQUIRE(kx >= bicubic_ksize(in_w, out_size) && ky >= bicubic_ksize(in_h, out_size));
  if (batch == 0) return AACLIP_OK;
  PrepArgs a{};
  a.src = src;
  a.img_stride = img_stride;
  a.pitch = row_pitch;
  a.in_h = in_h;
  a.in_w = in_w;
  a.S = out_size;
  a.xb = x_bounds;
  a.xk = x_coeffs;
  a.yb = y_bounds;
  a.yk = y_coeffs;
  a.kx = kx;
  a.ky = ky;
  static const float clip_mean_std[6] = {0.48145466f, 0.4578275f, 0.40821073f,
                                         0.26862954f, 0.26130258f, 0.27577711f};
  const float* ms = mean_std ? mean_std : clip_mean_std;
  for (int c = 0; c < 3; ++c) {
    a.mean[c] = ms[c];
    a.stdv[c] = ms[3 + c];
  }
  a.out = out;
  // two-pass path: needs the caller's workspace and the source rows + tap table in LDS
  int srow = 0, hrows = 8, hlds = 0;
  if (const char* e = getenv("AACLIP_PREP_HROWS")) hrows = std::max(1, atoi(e));  // tuning
  while (hrows > 0 && !(hlds = h_lds_bytes(in_w, hrows, &srow))) hrows >>= 1;
  const int tstride = tmp_stride(out_size);
  if (workspace && workspace_bytes >= (size_t)batch * in_h * tstride && hlds && tap_slots(in_w, out_size, kx) &&
      out_size <= 1024 && batch <= 65535 &&
      !getenv("AACLIP_PREP_TILE")) {
    HArgs h{src, img_stride, row_pitch, in_h, in_w, out_size, hrows, x_bounds, x_coeffs, kx, srow, tstride,
            (uint8_t*)workspace};
    const dim3 hgrid(ceil_div(in_h, hrows), batch);
    const hipStream_t st = (hipStream_t)stream;
    int rc = AACLIP_ERR_ARG;
    switch (tap_slots(in_w, out_size, kx)) {
#define AACLIP_H_CASE(K) \
  case K:                \
    rc = launch_h<K>(h, hgrid, 64 * ceil_div(out_size, 64), hlds, st); \
    break;
      AACLIP_H_CASE(4) AACLIP_H_CASE(6) AACLIP_H_CASE(8) AACLIP_H_CASE(10) AACLIP_H_CASE(12) AACLIP_H_CASE(14)
      AACLIP_H_CASE(16)
#undef AACLIP_H_CASE
    }
    if (rc != AACLIP_OK) return rc;
    AACLIP_CHECK_LAUNCH();
    const dim3 vgrid(ceil_div(out_size * ceil_div(out_size, 4), 256), batch);
    const VArgs v{(const uint8_t*)workspace, in_h, out_size, tstride, y_bounds, y_coeffs, ky,
                  {a.mean[0], a.mean[1], a.mean[2]}, {a.stdv[0], a.stdv[1], a.stdv[2]}, out};
    switch (tap_slots(in_h, out_size, ky)) {
#define AACLIP_V_CASE(K) \
  case K:                \
    resample_v_kernel<K><<<vgrid, 256, 0, st>>>(v); \
    break;
      AACLIP_V_CASE(4) AACLIP_V_CASE(6) AACLIP_V_CASE(8) AACLIP_V_CASE(10) AACLIP_V_CASE(12) AACLIP_V_CASE(14)
      AACLIP_V_CASE(16)
#undef AACLIP_V_CASE
      default:
        resample_v_kernel<0><<<vgrid, 256, 0, st>>>(v);
    }
    AACLIP_CHECK_LAUNCH();
    return AACLIP_OK;
  }
  // single-kernel path (no workspace, or rows too wide for LDS): tile choice: the tallest/widest staged tile (from 16 x 32) whose weights + strip + patch
  // fit STAGED_LDS, else direct taps. 1024 -> 336: 16 x 32 tiles, 62 x 111-pixel patches,
  // 32 KB -> 4 workgroups per CU. Measured at B=32 1024^2 (AACLIP_PREP_TILE + kbench --only prep):
  // 16x64 257 us, 8x64 195, 16x32 152, 16x16 144, direct 257 -- occupancy-bound.
  bool staged = false;
  int lds = 0;
  int ty_max = 16, tx_max = 32, force_direct = 0;
  if (const char* e = getenv("AACLIP_PREP_TILE")) sscanf(e, "%d,%d,%d", &ty_max, &tx_max, &force_direct);  // tuning
  for (int tx = tx_max; tx >= 16 && !staged && !force_direct; tx >>= 1)
    for (int ty = ty_max; ty >= 1 && !staged; ty >>= 1) {
      const int rows = strip_bound(in_h, out_size, ty, ky), cols = strip_bound(in_w, out_size, tx, kx);
      const int srow = (cols * 3 + 3 + 3 + 15) & ~15;
      const int bytes = (tx * kx + ty * ky) * 4 + ((rows * tx * 3 + 15) & ~15) + rows * srow;
      if (bytes <= STAGED_LDS) {
        staged = true;
        a.ty = ty;
        a.tx = tx;
        a.max_rows = rows;
        a.max_cols = cols;
        a.srow = srow;
        lds = bytes;
      }
    }
  if (!staged) {
    a.tx = 64;
    a.ty = 16;
    while (a.ty > 1 && strip_bound(in_h, out_size, a.ty, ky) * a.tx * 3 > DIRECT_LDS) a.ty >>= 1;
    a.max_rows = strip_bound(in_h, out_size, a.ty, ky);
    lds = a.max_rows * a.tx * 3;
    AACLIP_REQUIRE(lds <= DIRECT_LDS);
  }
  a.tiles_x = ceil_div(out_size, a.tx);
  a.tiles_y = ceil_div(out_size, a.ty);
  AACLIP_REQUIRE(batch <= 65535 && (int64_t)a.tiles_x * a.tiles_y < (1ll << 31));
  static unsigned staged_dev = 0, direct_dev = 0;
  if (!lds_attr_once((const void*)bicubic_normalize_kernel<true>, STAGED_LDS, staged_dev) ||
      !lds_attr_once((const void*)bicubic_normalize_kernel<false>, DIRECT_LDS, direct_dev))
    return AACLIP_ERR_LAUNCH;
  const dim3 grid(a.tiles_x * a.tiles_y, batch);
  if (staged)
    bicubic_normalize_kernel<true><<<grid, NT, lds, (hipStream_t)stream>>>(a);
  else
    bicubic_normalize_kernel<false><<<grid, NT, lds, (hipStream_t)stream>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

extern "C" int aaclip_resize_masks_nearest(const uint8_t* src, int64_t img_stride, int64_t row_pitch, int batch,
                                           int in_h, int in_w, const int32_t* x_index, const int32_t* y_index,
                                           int out_size, float* out, void* stream) {
  AACLIP_REQUIRE(src && x_index && y_index && out && batch >= 0 && in_h > 0 && in_w > 0 && out_size > 0);
  AACLIP_REQUIRE(row_pitch >= in_w && (img_stride >= row_pitch * in_h || batch <= 1) && batch <= 65535);
  if (batch == 0) return AACLIP_OK;
  const size_t plane = (size_t)out_size * out_size;
  const int blocks = (int)std::min<size_t>((plane + NT - 1) / NT, 1024);
  nearest_mask_kernel<<<dim3(blocks, batch), NT, 0, (hipStream_t)stream>>>(src, img_stride, row_pitch, x_index,
                                                                           y_index, out_size, out);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}
