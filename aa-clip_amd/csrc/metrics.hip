// Device metrics_eval (reference forward_utils.py:233-280): the
// class-global min-max normalisation of the pixel maps and image scores, the
// pixel-max fusion of the image score, and EXACT sklearn roc_auc_score /
// average_precision_score (tie-aware) for pixels and images.
//
// Pixels (up to ~19 M per class at C4) are ranked by one radix sort of 33-bit
// keys: (order-preserving bits of the normalised fp32 score << 1) | label, so
// equal scores form contiguous groups with their negatives first. Then
//   * AUROC = U / (P*N), U the Mann-Whitney count (pairs pos > neg, ties 1/2),
//     equal to sklearn's trapezoid over the tie-grouped ROC curve; 2U is summed
//     exactly in 64-bit integers;
//   * AP = (1/P) * sum over positives of TP(>= s) / N(>= s), i.e. sklearn's
//     sum_n (R_n - R_{n-1}) P_n over distinct thresholds, in fp64.
// Per sorted position i both need only P_excl[i] (positives before i: a scan of
// the label bits) and a_g (start of i's score group: a max-scan of flagged
// indices). Reductions are two-level and fixed-order, so results are
// deterministic run to run. Images (hundreds) use direct O(n^2) pair counts.
// Sort and scans are rocPRIM device primitives; the caller owns all memory
// (workspace size from aaclip_metrics_workspace).
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.h"

namespace {

constexpr int MT = 256;  // threads per block for the element-wise passes

__device__ __forceinline__ float block_min(float v, float* sh) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  v = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) v = fminf(v, sh[i]);
  return v;
}
__device__ __forceinline__ float block_max(float v, float* sh) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  v = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) v = fmaxf(v, sh[i]);
  return v;
}

// per-image min / max of the raw maps (one block per image)
__global__ __launch_bounds__(MT) void row_minmax_kernel(const float* __restrict__ p, int64_t pix,
                                                        float* __restrict__ rmin, float* __restrict__ rmax) {
  __shared__ float sh[MT / 64];
  const float* row = p + (size_t)blockIdx.x * pix;
  float lo = INFINITY, hi = -INFINITY;
  for (int64_t i = threadIdx.x; i < pix; i += MT) {
    const float v = row[i];
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
  lo = block_min(lo, sh);
  hi = block_max(hi, sh);
  if (threadIdx.x == 0) {
    rmin[blockIdx.x] = lo;
    rmax[blockIdx.x] = hi;
  }
}

struct Norm {  // numpy float32 semantics of forward_utils.py:241-248
  float pmin, pmax, imin, imax;
  int pnorm, inorm;
};

// One block: global min/max, normalisation flags, fused image scores.
__global__ __launch_bounds__(MT) void image_scores_kernel(const float* __restrict__ rmin,
                                                          const float* __restrict__ rmax,
                                                          const float* __restrict__ img, int n_img, int medical,
                                                          Norm* __restrict__ nrm, float* __restrict__ fused) {
  __shared__ float sh[MT / 64];
  float lo = INFINITY, hi = -INFINITY, ilo = INFINITY, ihi = -INFINITY;
  for (int i = threadIdx.x; i < n_img; i += MT) {
    lo = fminf(lo, rmin[i]);
    hi = fmaxf(hi, rmax[i]);
    ilo = fminf(ilo, img[i]);
    ihi = fmaxf(ihi, img[i]);
  }
  lo = block_min(lo, sh);
  hi = block_max(hi, sh);
  ilo = block_min(ilo, sh);
  ihi = block_max(ihi, sh);
  const bool pn = hi != 1.0f, in = ihi != 1.0f;
  if (threadIdx.x == 0) *nrm = Norm{lo, hi, ilo, ihi, pn, in};
  for (int i = threadIdx.x; i < n_img; i += MT) {
    // max over pixels of the normalised map == normalised row max: fl((x-a)/b) is monotone
    const float pm = pn ? (rmax[i] - lo) / (hi - lo) : rmax[i];
    const float is = in ? (img[i] - ilo) / (ihi - ilo) : img[i];
    fused[i] = medical ? pm : pm * 0.5f + is * 0.5f;
  }
}

// order-preserving uint32 image of a float (+0 and -0 map to the same key)
__device__ __forceinline__ uint32_t ord_bits(float v) {
  if (v == 0.0f) v = 0.0f;
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(MT) void make_keys_kernel(const float* __restrict__ p, const uint8_t* __restrict__ lab,
                                                       int64_t n, const Norm* __restrict__ nrm,
                                                       uint64_t* __restrict__ keys) {
  const Norm z = *nrm;
  for (int64_t i = (int64_t)blockIdx.x * MT + threadIdx.x; i < n; i += (int64_t)gridDim.x * MT) {
    float v = p[i];
    if (z.pnorm) v = (v - z.pmin) / (z.pmax - z.pmin);
    keys[i] = ((uint64_t)ord_bits(v) << 1) | (lab[i] != 0 ? 1u : 0u);
  }
}

// label bit and flagged group-start index of every sorted position
__global__ __launch_bounds__(MT) void split_keys_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                        uint32_t* __restrict__ lbl, uint32_t* __restrict__ gstart) {
  for (int64_t i = (int64_t)blockIdx.x * MT + threadIdx.x; i < n; i += (int64_t)gridDim.x * MT) {
    const uint64_t k = keys[i];
    lbl[i] = (uint32_t)(k & 1);
    gstart[i] = (i == 0 || (keys[i - 1] >> 1) != (k >> 1)) ? (uint32_t)i : 0u;
  }
}

struct Partial {
  unsigned long long u2;  // 2U contribution
  double ap;              // sum of TP(>=s)/N(>=s) over positives
};

__device__ __forceinline__ Partial block_sum(Partial v, Partial* sh) {
  for (int o = 32; o > 0; o >>= 1) {
    v.u2 += __shfl_xor(v.u2, o, 64);
    v.ap += __shfl_xor(v.ap, o, 64);
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  Partial r = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
    r.u2 += sh[i].u2;
    r.ap += sh[i].ap;
  }
  return r;
}

// pixel pass over sorted positions: P = exclusive label scan (P[n] = total),
// A = inclusive max-scan of group starts. Deterministic per-block partials.
__global__ __launch_bounds__(MT) void pixel_partial_kernel(const uint32_t* __restrict__ lbl,
                                                           const uint32_t* __restrict__ P,
                                                           const uint32_t* __restrict__ A, int64_t n,
                                                           int64_t per_block, Partial* __restrict__ part) {
  __shared__ Partial sh[MT / 64];
  const uint64_t ptot = (uint64_t)P[n - 1] + lbl[n - 1];
  const int64_t lo = (int64_t)blockIdx.x * per_block, hi = min(n, lo + per_block);
  Partial acc{0ull, 0.0};
  for (int64_t i = lo + threadIdx.x; i < hi; i += MT) {
    if (!lbl[i]) continue;
    const uint64_t a = A[i];
    const uint64_t pa = P[a];
    const uint64_t nb_i = (uint64_t)i - P[i];  // negatives at positions < i (incl. this group's)
    const uint64_t nb_a = a - pa;              // negatives strictly below the group
    acc.u2 += nb_i + nb_a;
    acc.ap += (double)(ptot - pa) / (double)((uint64_t)n - a);
  }
  acc = block_sum(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// image pass: O(n^2) pair counts, one thread per image
__global__ __launch_bounds__(MT) void image_partial_kernel(const float* __restrict__ s,
                                                           const uint8_t* __restrict__ lab, int n,
                                                           Partial* __restrict__ part) {
  __shared__ Partial sh[MT / 64];
  Partial acc{0ull, 0.0};
  const int i = blockIdx.x * MT + threadIdx.x;
  if (i < n && lab[i]) {
    const float si = s[i];
    uint64_t below = 0, eq_neg = 0, ge = 0, ge_pos = 0;
    for (int j = 0; j < n; ++j) {
      const float sj = s[j];
      const bool pj = lab[j] != 0;
      if (sj >= si) {
        ++ge;
        ge_pos += pj;
      }
      if (!pj) {
        below += sj < si;
        eq_neg += sj == si;
      }
    }
    acc.u2 = 2 * below + eq_neg;
    acc.ap = (double)ge_pos / (double)ge;
  }
  acc = block_sum(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// out[0..1] = pixel AUROC, AP; out[2..3] = image AUROC, AP (0, 0 when the image
// labels are all equal, forward_utils.py:264-271; NaN when the pixel labels are,
// where sklearn raises).
__global__ __launch_bounds__(64) void finalize_kernel(const Partial* __restrict__ pp, int npp,
                                                     const uint32_t* __restrict__ P,
                                                     const uint32_t* __restrict__ lbl, int64_t n,
                                                     const Partial* __restrict__ ip, int nip,
                                                     const uint8_t* __restrict__ ilab, int n_img,
                                                     double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  Partial a{0ull, 0.0};
  for (int i = 0; i < npp; ++i) {
    a.u2 += pp[i].u2;
    a.ap += pp[i].ap;
  }
  const uint64_t pos = (uint64_t)P[n - 1] + lbl[n - 1], neg = (uint64_t)n - pos;
  if (pos == 0 || neg == 0) {
    out[0] = out[1] = NAN;
  } else {
    out[0] = (double)a.u2 / (2.0 * (double)pos * (double)neg);
    out[1] = a.ap / (double)pos;
  }
  Partial b{0ull, 0.0};
  for (int i = 0; i < nip; ++i) {
    b.u2 += ip[i].u2;
    b.ap += ip[i].ap;
  }
  uint64_t ipos = 0;
  for (int i = 0; i < n_img; ++i) ipos += ilab[i] != 0;
  const uint64_t ineg = (uint64_t)n_img - ipos;
  if (ipos == 0 || ineg == 0) {
    out[2] = out[3] = 0.0;
  } else {
    out[2] = (double)b.u2 / (2.0 * (double)ipos * (double)ineg);
    out[3] = b.ap / (double)ipos;
  }
}

struct Layout {  // workspace carve-up (256-B aligned pieces)
  size_t keys_a, keys_b, lbl, gst, P, A, rmin, rmax, fused, norm, ppart, ipart, temp, temp_bytes, total;
  int npp, nip;
  int64_t per_block;
};

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

int plan(int64_t n, int n_img, Layout& L) {
  size_t sort_b = 0, scan_b = 0, max_b = 0;
  if (rocprim::radix_sort_keys((void*)nullptr, sort_b, (uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)n, 0, 33) !=
      hipSuccess)
    return AACLIP_ERR_LAUNCH;
  if (rocprim::exclusive_scan((void*)nullptr, scan_b, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n,
                              rocprim::plus<uint32_t>()) != hipSuccess)
    return AACLIP_ERR_LAUNCH;
  if (rocprim::inclusive_scan((void*)nullptr, max_b, (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n,
                              rocprim::maximum<uint32_t>()) != hipSuccess)
    return AACLIP_ERR_LAUNCH;
  L.per_block = 64 * MT;
  L.npp = (int)((n + L.per_block - 1) / L.per_block);
  L.nip = (n_img + MT - 1) / MT;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += align_up(bytes);
    return at;
  };
  // keys_a (8 B per pixel) is reused, once sorted into keys_b, for two 4-B arrays
  // (labels, group starts) at 256-B aligned offsets: size it for both aligned halves
  // (8n alone is too small when 4n is not a multiple of 256, e.g. 4 maps of 518^2)
  L.keys_a = take(2 * align_up(4 * (size_t)n));
  L.keys_b = take(8 * (size_t)n);
  L.lbl = L.keys_a;
  L.gst = L.keys_a + align_up(4 * (size_t)n);
  L.P = take(4 * (size_t)n);
  L.A = take(4 * (size_t)n);
  L.rmin = take(4 * (size_t)n_img);
  L.rmax = take(4 * (size_t)n_img);
  L.fused = take(4 * (size_t)n_img);
  L.norm = take(sizeof(Norm));
  L.ppart = take(sizeof(Partial) * (size_t)L.npp);
  L.ipart = take(sizeof(Partial) * (size_t)L.nip);
  L.temp_bytes = std::max(sort_b, std::max(scan_b, max_b));
  L.temp = take(L.temp_bytes);
  L.total = o;
  return AACLIP_OK;
}

}  // namespace

extern "C" int aaclip_metrics_workspace(int64_t n_pixels, int n_images, size_t* bytes) {
  AACLIP_REQUIRE(bytes && n_pixels > 0 && n_images > 0 && n_pixels < (1LL << 32) - 1);
  Layout L;
  const int rc = plan(n_pixels, n_images, L);
  if (rc) return rc;
  *bytes = L.total;
  return AACLIP_OK;
}

extern "C" int aaclip_metrics_eval(const float* pixel_preds, const uint8_t* pixel_label, const float* image_preds,
                                   const uint8_t* image_label, int n_images, int64_t pix_per_image, int medical,
                                   void* workspace, size_t workspace_bytes, double* out, void* stream) {
  AACLIP_REQUIRE(pixel_preds && pixel_label && image_preds && image_label && workspace && out);
  AACLIP_REQUIRE(n_images > 0 && pix_per_image > 0);
  const int64_t n = (int64_t)n_images * pix_per_image;
  AACLIP_REQUIRE(n < (1LL << 32) - 1);
  Layout L;
  int rc = plan(n, n_images, L);
  if (rc) return rc;
  AACLIP_REQUIRE(workspace_bytes >= L.total && ((uintptr_t)workspace % 256) == 0);
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  uint64_t* keys_a = (uint64_t*)(ws + L.keys_a);
  uint64_t* keys_b = (uint64_t*)(ws + L.keys_b);
  uint32_t* lbl = (uint32_t*)(ws + L.lbl);
  uint32_t* gst = (uint32_t*)(ws + L.gst);
  uint32_t* P = (uint32_t*)(ws + L.P);
  uint32_t* A = (uint32_t*)(ws + L.A);
  float* rmin = (float*)(ws + L.rmin);
  float* rmax = (float*)(ws + L.rmax);
  float* fused = (float*)(ws + L.fused);
  Norm* nrm = (Norm*)(ws + L.norm);
  Partial* ppart = (Partial*)(ws + L.ppart);
  Partial* ipart = (Partial*)(ws + L.ipart);
  void* temp = ws + L.temp;
  size_t tb = L.temp_bytes;

  const int grid = (int)std::min<int64_t>((n + MT - 1) / MT, 4096);
  row_minmax_kernel<<<n_images, MT, 0, s>>>(pixel_preds, pix_per_image, rmin, rmax);
  image_scores_kernel<<<1, MT, 0, s>>>(rmin, rmax, image_preds, n_images, medical, nrm, fused);
  make_keys_kernel<<<grid, MT, 0, s>>>(pixel_preds, pixel_label, n, nrm, keys_a);
  AACLIP_CHECK_LAUNCH();
  if (rocprim::radix_sort_keys(temp, tb, keys_a, keys_b, (size_t)n, 0, 33, s) != hipSuccess) return AACLIP_ERR_LAUNCH;
  split_keys_kernel<<<grid, MT, 0, s>>>(keys_b, n, lbl, gst);
  tb = L.temp_bytes;
  if (rocprim::exclusive_scan(temp, tb, lbl, P, 0u, (size_t)n, rocprim::plus<uint32_t>(), s) != hipSuccess)
    return AACLIP_ERR_LAUNCH;
  tb = L.temp_bytes;
  if (rocprim::inclusive_scan(temp, tb, gst, A, (size_t)n, rocprim::maximum<uint32_t>(), s) != hipSuccess)
    return AACLIP_ERR_LAUNCH;
  pixel_partial_kernel<<<L.npp, MT, 0, s>>>(lbl, P, A, n, L.per_block, ppart);
  image_partial_kernel<<<L.nip, MT, 0, s>>>(fused, image_label, n_images, ipart);
  finalize_kernel<<<1, 64, 0, s>>>(ppart, L.npp, P, lbl, n, ipart, L.nip, image_label, n_images, out);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}
