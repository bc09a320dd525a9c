// GEMM family for the AA-CLIP path: C[M,N] = epilogue(A[M,K] . W[N,K]^T).
//
// Both operands are K-contiguous (activations [M,K], nn.Linear weights [N,K]),
// which is the natural MFMA "NT" form: every A and B fragment of
// v_mfma_f32_16x16x32_bf16 is 8 consecutive K values = one 16-byte ds_read_b128.
//
// bf16 kernel (perf path):
//   * block tile BM x BN x 64, 8 waves (512 threads), wave tile (BM/WM) x (BN/WN);
//     default 320x256 (wave tile 160x64 = 10x4 MFMA tiles, 144 KiB LDS double buffer)
//   * global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
//     instruction = 8 rows of 128 B). The LDS image is lane-linear, so the bank
//     swizzle (16-B chunk c of row r stored at chunk c ^ (r & 7)) is applied on
//     the per-lane SOURCE address and undone on the ds_read (rule: swizzle both
//     sides through the same involution) -> conflict-free fragment reads.
//   * 2-stage double buffer, one barrier per K-step: the DMA of tile k+1 is
//     issued before the MFMAs of tile k.
//   * XCD-aware, bijective block remap + grouped tile order for L2 reuse.
//   * fused epilogue: bias, erf-GELU, LeakyReLU, fp32 residual, bf16 aux copy,
//     output row remap (patch rows -> token rows after the CLS slot).
// fp32 kernel (parity mode): v_mfma_f32_16x16x4_f32 (exact fp32 FMA chain),
//   64x64x16 register-staged tiles. Same epilogue.
#include <math.h>

#include <atomic>
#include <mutex>

#include "common.h"

namespace {

struct GemmArgs {
  const void* A;
  const void* W;
  void* C;
  const float* bias;
  const float* res;
  void* aux;
  int64_t lda, ldw, ldc, ldr, ldaux;
  int M, N, K;
  int epi, out_dtype;
  int row_group, row_group_out, row_offset;
  int tiles_m, tiles_n;
  int group_m;   // tile-order group height (L2 reuse), default 8
  int setprio;   // raise wave priority around the MFMA cluster
  int dbg;       // diagnostic: 1 = skip the epilogue (accumulators kept live)
  const float* a_scale;  // fp8 only: per-row scale of A (dequant = q * a_scale[m])
  const float* w_scale;  // fp8 only: per-output-channel scale of W
  const uint8_t* a_mx;   // fp8 MX A operand: e8m0 scale per (row, 64-K block), [K/128][ld_amx][2]
  int64_t ld_amx;
  uint8_t* c_mx;         // fp8 MX output: e8m0 scale per (row, 64-column block), [N/128][ld_cmx][2]
  int64_t ld_cmx;
  const float* anchors;  // score-partials output (OUTM 3): text anchors T [t_period][2] (normal, abnormal)
  int t_period;          // column c uses anchor row c % t_period (the level width, 768)
  // fixed split-K (aaclip_gemm_ksplit): every output tile is computed by `ksplit` workgroups,
  // part h over K-steps [h nk / S, (h + 1) nk / S); each stores its fp32 partial tile to
  // kpart, and the last to arrive (kcount[tile]) sums the S partials in index order and runs
  // the epilogue. The split depends only on K, so the bits do not depend on M or the family.
  int ksplit = 1;
  float* kpart = nullptr;
  unsigned* kcount = nullptr;
};

// out_dtype tag of the score-partials output (aaclip_gemm_scores; never a public dtype)
constexpr int kOutScores = 100;

// trace-build tag of a GEMM launch: N/64 in bits 4-11, K/64 in bits 12-19 (each capped at
// 255, so N or K >= 16384 saturates its field instead of spilling into the next), epilogue
// flags from bit 20 (diagnostic builds only; tools/timeline.py decodes it)
__host__ __device__ inline uint32_t gemm_trace_tag(const GemmArgs& a) {
  return (uint32_t)min(a.N / 64, 255) << 4 | (uint32_t)min(a.K / 64, 255) << 12 | (uint32_t)a.epi << 20;
}

// smallest e with amax * 2^-e <= 448 (largest finite e4m3): the e8m0 block scale
__device__ __forceinline__ int mx_exp(float amax) {
  if (!(amax > 0.f)) return 0;
  int x;
  (void)frexpf(amax, &x);  // amax = m * 2^x, m in [0.5, 1)
  int e = x - 9;           // amax * 2^-e in [256, 512)
  if (ldexpf(amax, -e) > 448.f) e += 1;
  return max(min(e, 127), -126);
}
__device__ __forceinline__ float pow2i(int e) { return __uint_as_float((uint32_t)(e + 127) << 23); }

// cross-lane max over the 4 lanes {c, c+16, c+32, c+48} (one row of the C^T tile)
__device__ __forceinline__ float max_over_fq(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// sum over the 4 lanes {c, c+16, c+32, c+48} in a fixed association, (fq0 + fq1) + (fq2 + fq3)
// with the pairs' operands swapped on the partner lanes -- fp32 addition commutes, so all
// four lanes end with the same bits
__device__ __forceinline__ float sum_over_fq(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// 4x4 dword transpose across the lane groups fq = lane/16: on entry lane fq holds
// d[j] = its 4 fp8 columns of column tile j; on exit it holds tile j = fq's 16
// consecutive bytes (d[q] = the 4 columns of lane group q).
__device__ __forceinline__ void transpose_fq(uint32_t (&d)[4]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    auto r = __builtin_amdgcn_permlane32_swap(d[j], d[j + 2], false, false);
    d[j] = r[0];
    d[j + 2] = r[1];
  }
#pragma unroll
  for (int k = 0; k < 4; k += 2) {
    auto r = __builtin_amdgcn_permlane16_swap(d[k], d[k + 1], false, false);
    d[k] = r[0];
    d[k + 1] = r[1];
  }
}

__device__ __forceinline__ int remap_row(const GemmArgs& a, int m) {
  return a.row_group > 0 ? (m / a.row_group) * a.row_group_out + a.row_offset + (m % a.row_group) : m;
}

__device__ __forceinline__ float gelu_erf(float v) {
  return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
}

// GELU for the bf16-input kernel: v * sigmoid(v * P(v^2)), P quadratic, fitted
// (minimax on [-12, 12]) to the erf form: |error| <= 2.6e-5 absolute, an order
// below the bf16 rounding of the output for |y| >= 0.01. The clamp keeps the
// quintic in its monotone range (|v| > 8: sigmoid is 0/1 to 1e-12). 7 VALU + one
// v_exp + one v_rcp per element, vs 16 + 2 for an erfc-polynomial form; the c_fc
// epilogue is VALU-bound (all waves of the chip run it at once, no MFMA to hide
// behind). -log2(e) is folded into the coefficients so v_exp_f32 (2^x) applies
// directly. The fp32 parity kernel keeps the exact erff form (gelu_erf).
__device__ __forceinline__ float gelu_fast(float v) {
  const float vc = __builtin_amdgcn_fmed3f(v, -8.0f, 8.0f);
  const float s = vc * vc;
  const float w = vc * fmaf(s, fmaf(s, 0.0010142630f, -0.10677572f), -2.3011212f);
  return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(w));
}

// gelu_fast on a column pair in packed f32 arithmetic (v_pk_mul/v_pk_fma/v_pk_add: two
// elements per VALU issue; the epilogue runs with no MFMA beside it, so the packed
// forms are pure savings here): 2 v_med3 + 5 packed + 2 v_exp + 2 v_rcp per pair,
// the same roundings as gelu_fast element by element.
__device__ __forceinline__ float2_t gelu_fast2(float2_t v) {
  const float2_t vc = {__builtin_amdgcn_fmed3f(v[0], -8.0f, 8.0f), __builtin_amdgcn_fmed3f(v[1], -8.0f, 8.0f)};
  const float2_t s = vc * vc;
  const float2_t c2 = {0.0010142630f, 0.0010142630f}, c1 = {-0.10677572f, -0.10677572f},
                 c0 = {-2.3011212f, -2.3011212f}, one = {1.0f, 1.0f};
  const float2_t w = vc * __builtin_elementwise_fma(s, __builtin_elementwise_fma(s, c2, c1), c0);
  const float2_t d = float2_t{__builtin_amdgcn_exp2f(w[0]), __builtin_amdgcn_exp2f(w[1])} + one;
  return v * float2_t{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
}

// QuickGELU (reference transformer.py:46-49: x * sigmoid(1.702 x)). Exact form for the
// fp32 parity kernel: the same expf/division as torch.sigmoid's fp32 CPU path.
__device__ __forceinline__ float qgelu_exact(float v) { return v * (1.0f / (1.0f + expf(-1.702f * v))); }

// 16-bit kernels, a column pair in packed f32: v * rcp(1 + 2^(-1.702 log2(e) v)); the
// argument is clamped to |.| <= 64 (exp2 stays finite, sigmoid is 0/1 to 1e-19 there).
// |error| vs qgelu_exact <= 2 ulp, far below the 16-bit rounding of the output.
__device__ __forceinline__ float2_t qgelu_fast2(float2_t v) {
  constexpr float c = -1.702f * 1.44269504088896340736f;
  const float2_t w = float2_t{__builtin_amdgcn_fmed3f(v[0] * c, -64.0f, 64.0f),
                              __builtin_amdgcn_fmed3f(v[1] * c, -64.0f, 64.0f)};
  const float2_t d = float2_t{__builtin_amdgcn_exp2f(w[0]), __builtin_amdgcn_exp2f(w[1])} + float2_t{1.0f, 1.0f};
  return v * float2_t{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
}

// Epilogue on one element C[m, n] (m < M checked by the caller).
__device__ __forceinline__ void epilogue_store1(const GemmArgs& a, int m, int n, float v) {
  const int orow = remap_row(a, m);
  if (a.epi & AACLIP_EPI_BIAS) v += a.bias[n];
  if (a.epi & AACLIP_EPI_GELU) v = gelu_erf(v);
  if (a.epi & AACLIP_EPI_QGELU) v = qgelu_exact(v);
  if (a.epi & AACLIP_EPI_LEAKY) v = v >= 0.f ? v : 0.01f * v;
  if (a.epi & AACLIP_EPI_RESID) v += a.res[(size_t)orow * a.ldr + n];
  if (a.out_dtype == AACLIP_F32)
    ((float*)a.C)[(size_t)orow * a.ldc + n] = v;
  else
    ((uint16_t*)a.C)[(size_t)orow * a.ldc + n] = f32_to_bf16(v);
  if (a.epi & AACLIP_EPI_AUX_BF16) ((uint16_t*)a.aux)[(size_t)orow * a.ldaux + n] = f32_to_bf16(v);
}

// Bijective XCD remap (blocks b, b+8, ... share an XCD) + grouped tile order.
__device__ __forceinline__ void tile_coords(int bid, int tiles_m, int tiles_n, int& tm, int& tn,
                                            int GROUP_M = 4) {
  const int nwg = tiles_m * tiles_n;
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid % per_group;
  tm = first_m + in_group % gsize;
  tn = in_group / gsize;
}

// ---------------------------------------------------------------- fixed split-K
// Workgroup -> (tile, part) for a split launch: the grid is 8 x ksplit x ceil(T/8) slots
// (T = tiles). XCD x (= bid % 8, the hardware's round-robin) owns a contiguous run of tiles
// (the bijective split of tile_coords) and its slots s = bid / 8 take part h = s % S of tile
// s / S of that run: the S parts of a tile always share an XCD, so the L2 they meet in is
// one cache (no agent-scope write-back / invalidate), and run back to back. Slots past the
// XCD's run return false (nothing to do). Then the grouped tile order as in tile_coords.
__device__ __forceinline__ bool split_coords(const GemmArgs& a, int bid, int& tm, int& tn, int& h) {
  const int S = a.ksplit, T = a.tiles_m * a.tiles_n;
  const int xcd = bid & 7, slot = bid >> 3;
  const int q = T >> 3, r = T & 7;
  const int run = q + (xcd < r ? 1 : 0);
  const int lt = slot / S;
  h = slot - lt * S;
  if (lt >= run) return false;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + lt;
  const int per_group = a.group_m * a.tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * a.group_m;
  const int gsize = min(a.tiles_m - first_m, a.group_m);
  const int in_group = wgid % per_group;
  tm = first_m + in_group % gsize;
  tn = in_group / gsize;
  return true;
}

// K-steps [k0, k1) of part h of a fixed S-way split of nk steps
__device__ __forceinline__ void split_range(int nk, int S, int h, int& k0, int& k1) {
  k0 = (int)(((int64_t)h * nk) / S);
  k1 = (int)(((int64_t)(h + 1) * nk) / S);
}

// After the main loop of a split launch (KS parts, a compile-time instantiation of its own,
// so the unsplit kernels keep their registers): store this part's fp32 accumulators
// (wave-linear, 1 KiB per wave instruction), count the arrival; every part but the last
// returns false (no epilogue). The last one reloads the KS partials -- its own included,
// so its accumulators are dead across the sum and their registers hold the loads -- and
// sums them IN INDEX ORDER, ((P0 + P1) + P2) + ..., the same bits whichever part came
// last; one accumulator row block's loads are in flight together (the memory clobber
// between blocks keeps the compiler from hoisting every block's loads: scratch spills).
// It resets the counter for the next launch and runs the epilogue. Arrival words carry
// the XCC id (count in bits 0-7, sum of the parts' XCC ids from bit 8): parts that met
// across XCDs (whose L2s are not coherent) would read stale partials, so that case
// poisons the tile with NaN instead.
template <int KS, int RM, int RN>
__device__ __forceinline__ bool ksplit_combine(const GemmArgs& a, float4_t (&acc)[RM][RN], int tile, int h,
                                               int nwaves, int wid, int lane, int* lds_flag) {
  constexpr int PER_WAVE = RM * RN * 64;  // float4 per wave
  const size_t part_f4 = (size_t)nwaves * PER_WAVE;
  const float4_t* const base = (const float4_t*)a.kpart + (size_t)tile * KS * part_f4 + (size_t)wid * PER_WAVE + lane;
  float4_t* const mine = (float4_t*)base + (size_t)h * part_f4;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) mine[(i * RN + j) * 64] = acc[i][j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial has reached the L2
  __syncthreads();                                   // ... and every wave's
  if (threadIdx.x == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const unsigned old = atomicAdd(a.kcount + tile, 1u + (xcc << 8));
    const bool last = (int)(old & 0xff) == KS - 1;
    if (last) a.kcount[tile] = 0u;  // ready for the next launch (kernel boundaries order it)
    *lds_flag = last ? ((old >> 8) == (unsigned)(KS - 1) * xcc ? 1 : 2) : 0;
  }
  __syncthreads();
  const int f = *lds_flag;
  if (f == 0) return false;
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    asm volatile("" ::: "memory");
    float4_t p[KS][RN];
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int j = 0; j < RN; ++j) p[q][j] = base[(size_t)q * part_f4 + (i * RN + j) * 64];
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      float4_t sum = p[0][j];
#pragma unroll
      for (int q = 1; q < KS; ++q) sum += p[q][j];
      acc[i][j] = f == 1 ? sum : float4_t{NAN, NAN, NAN, NAN};
    }
  }
  return true;
}

// Epilogue of one wave's (16*RM) x 64 output tile straight from the accumulators.
// The main loop issues the MFMA with the W fragment as the first operand, so it
// computes the tile transposed: lane (fr, fq) holds C[16i + fr][16j + 4fq + e],
// e = 0..3 -- one row, 4 consecutive columns. fp32 rows leave as one 16-B store per
// (i, j); bf16 rows are packed to 8 B and paired across column tiles j, j+1 with
// v_permlane16_swap (lanes fq even/odd exchange halves) into 16-B stores. No LDS
// round trip (round 1 measured an LDS-staged form slower on the 320-row kernel); the
// 8-phase kernel does go through LDS (wave_epilogue_lds) to coalesce its accesses.
// The residual rows of tile-row i+1 are loaded before tile-row i's stores (vmcnt
// retires in issue order).
constexpr int EPI_REMAP = 64;

template <bool H16>
__device__ __forceinline__ uint4 pair_h16(const float4_t& lo, const float4_t& hi, int fq) {
  // lo = this lane's 4 columns of tile j0, hi = of tile j1 (both row fr, cols 4fq..4fq+3)
  uint32_t a0 = pack_h16x2<H16>(lo[0], lo[1]), a1 = pack_h16x2<H16>(lo[2], lo[3]);
  uint32_t b0 = pack_h16x2<H16>(hi[0], hi[1]), b1 = pack_h16x2<H16>(hi[2], hi[3]);
  auto x = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
  auto y = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
  // fq even: tile j0 cols 8(fq/2)..+7; fq odd: tile j1 cols 8(fq/2)..+7
  (void)fq;
  return uint4{x[0], y[0], x[1], y[1]};
}

// EPI >= 0: compile-time epilogue flags (AACLIP_EPI_* | EPI_REMAP) so each used
// combination is straight-line code; EPI = -1: flags read at run time (any combination).
// OUTM: 0 = fp32 C, 1 = bf16 C, 2 = fp8 e4m3 C with an e8m0 scale per (row, 64
// columns) -- the wave's 64-column tile is one block: row max over the 4 lane
// groups, power-of-two scale, RNE to e4m3, 4x4 lane-group transpose -> 16-B stores.
// SCALED: 0 = none, 1 = a_scale[row] * w_scale[col] (fp8 per-row), 2 = w_scale[col]
// only (fp8 MX: the activation block scales were applied by the MFMA).
// H16: the 16-bit storage of OUTM 1 and of the aux copy is fp16 (else bf16).
template <int RM, int RN, int OUTM, int EPI, int SCALED, bool H16 = false, int PD = 2>
__device__ __forceinline__ void wave_epilogue(const GemmArgs& a, float4_t (&acc)[RM][RN], int mw, int nw,
                                              int lane, const float* lbias = nullptr) {
  static_assert(RN % 2 == 0, "column tiles are paired");
  static_assert(OUTM != 2 || RN == 4, "fp8 MX output: one 64-column block per wave");
  static_assert(OUTM != 3 || RN == 2 || RN == 4, "score partials: one or two 32-column groups per wave");
  constexpr bool BF16OUT = OUTM == 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int epi = EPI >= 0 ? EPI : a.epi | (a.row_group > 0 ? EPI_REMAP : 0);
  auto out_row = [&](int m) { return (epi & EPI_REMAP) ? remap_row(a, m) : m; };
  const int ncol = nw + 4 * fq;               // fp32 layout: this lane's first column in tile j = 0
  const int pcol = nw + 16 * (fq & 1) + 8 * (fq >> 1);  // paired bf16 layout
  float4_t bias[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j)  // lbias: the tile's bias staged in LDS by the kernel (indexed by column)
    bias[j] = (epi & AACLIP_EPI_BIAS) ? *(const float4_t*)((lbias ? lbias : a.bias) + ncol + 16 * j)
                                      : float4_t{0.f, 0.f, 0.f, 0.f};
  // OUTM 3 (score partials): this lane's anchor values, t0 / t1 of columns ncol + 16 j + e
  float4_t ta0[RN], ta1[RN];
  if constexpr (OUTM == 3) {
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int c = (ncol + 16 * j) % a.t_period;
      const float4_t lo = *(const float4_t*)(a.anchors + 2 * c), hi = *(const float4_t*)(a.anchors + 2 * c + 4);
      ta0[j] = float4_t{lo[0], lo[2], hi[0], hi[2]};
      ta1[j] = float4_t{lo[1], lo[3], hi[1], hi[3]};
    }
  }
  float4_t wsc[RN];  // fp8: per-column weight scales of this lane's 4 columns in tile j
  if constexpr (SCALED) {
#pragma unroll
    for (int j = 0; j < RN; ++j) wsc[j] = *(const float4_t*)(a.w_scale + ncol + 16 * j);
  }
  // residual rows in a PD-deep register ring: tile-row i + PD - 1 is requested before
  // tile-row i is used. PD = 4 on the 8-phase kernel (244 VGPRs, no spill) measured
  // 0.4 % SLOWER in the two-stream step than PD = 2 (224 VGPRs): above 224 the 8-wave
  // workgroup leaves no room on a SIMD for a 64-VGPR row-kernel wave of the other chunk.
  static_assert(PD >= 2 && PD <= RM, "residual ring depth");
  float4_t res[PD][RN];
  auto load_res = [&](int i, float4_t (&dst)[RN]) {
    const float* src = a.res + (size_t)out_row(min(mw + 16 * i + fr, a.M - 1)) * a.ldr + ncol;
#pragma unroll
    for (int j = 0; j < RN; ++j) dst[j] = *(const float4_t*)(src + 16 * j);
  };
  if (epi & AACLIP_EPI_RESID) {
#pragma unroll
    for (int i = 0; i < PD - 1 && i < RM; ++i) load_res(i, res[i]);
  }
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    if ((epi & AACLIP_EPI_RESID) && i + PD - 1 < RM) load_res(i + PD - 1, res[(i + PD - 1) % PD]);
    float4_t v[RN];
    float asc = 1.f;
    if constexpr (SCALED == 1) asc = a.a_scale[min(mw + 16 * i + fr, a.M - 1)];
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      if constexpr (SCALED == 1)
        v[j] = acc[i][j] * (wsc[j] * asc) + bias[j];
      else if constexpr (SCALED == 2)
        v[j] = acc[i][j] * wsc[j] + bias[j];
      else
        v[j] = acc[i][j] + bias[j];
      if (epi & AACLIP_EPI_GELU) {
        const float2_t lo = gelu_fast2(float2_t{v[j][0], v[j][1]}), hi = gelu_fast2(float2_t{v[j][2], v[j][3]});
        v[j] = float4_t{lo[0], lo[1], hi[0], hi[1]};
      }
      if (epi & AACLIP_EPI_QGELU) {
        const float2_t lo = qgelu_fast2(float2_t{v[j][0], v[j][1]}), hi = qgelu_fast2(float2_t{v[j][2], v[j][3]});
        v[j] = float4_t{lo[0], lo[1], hi[0], hi[1]};
      }
      if (epi & AACLIP_EPI_LEAKY)
#pragma unroll
        for (int t = 0; t < 4; ++t) v[j][t] = v[j][t] >= 0.f ? v[j][t] : 0.01f * v[j][t];
      if (epi & AACLIP_EPI_RESID) v[j] += res[i % PD][j];
    }
    if (a.dbg & 2) {  // diagnostic: everything but the global stores
#pragma unroll
      for (int j = 0; j < RN; ++j) asm volatile("" ::"v"(v[j]));
      continue;
    }
    const int m = mw + 16 * i + fr;
    const size_t orow = (size_t)out_row(min(m, a.M - 1));
    if constexpr (OUTM == 3) {
      // anomaly-map partials of row m over each 32-column group (column tiles 2q, 2q+1):
      // ||v||^2, v.t0, v.t1 -- lane-local fixed-order FMA chains over its 8 values, then
      // the fixed-order sum over the 4 lane groups. Every tile family holds the same
      // lane layout and 32-column-aligned groups, so the partials (and the map) do not
      // depend on which family ran. Lane group q < RN/2 stores group q as one float4.
      float4_t pr[RN / 2];
#pragma unroll
      for (int q = 0; q < RN / 2; ++q) {
        float ss = 0.f, x0 = 0.f, x1 = 0.f;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float u = v[2 * q + jj][e];
            ss = fmaf(u, u, ss);
            x0 = fmaf(u, ta0[2 * q + jj][e], x0);
            x1 = fmaf(u, ta1[2 * q + jj][e], x1);
          }
        pr[q] = float4_t{sum_over_fq(ss), sum_over_fq(x0), sum_over_fq(x1), 0.f};
      }
      if (m < a.M && fq < RN / 2)
        *(float4_t*)((float*)a.C + orow * a.ldc + (nw >> 3) + 4 * fq) = (fq == 0) ? pr[0] : pr[RN / 2 - 1];
      continue;
    }
    if constexpr (OUTM == 2) {
      float amax = 0.f;
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) amax = fmaxf(amax, fabsf(v[j][t]));
      const int e = mx_exp(max_over_fq(amax));
      const float inv = pow2i(-e);
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(v[j][0] * inv, v[j][1] * inv, 0, false);
        d[j] = __builtin_amdgcn_cvt_pk_fp8_f32(v[j][2] * inv, v[j][3] * inv, w, true);
      }
      transpose_fq(d);
      if (m < a.M) {
        *(uint4*)((uint8_t*)a.C + orow * a.ldc + nw + 16 * fq) = uint4{d[0], d[1], d[2], d[3]};
        const int blk = nw >> 6;
        if (fq == 0) a.c_mx[((size_t)(blk >> 1) * a.ld_cmx + orow) * 2 + (blk & 1)] = (uint8_t)(e + 127);
      }
      continue;
    }
    uint4 pk[RN / 2];
    if (BF16OUT || (epi & AACLIP_EPI_AUX_BF16)) {
#pragma unroll
      for (int q = 0; q < RN / 2; ++q) pk[q] = pair_h16<H16>(v[2 * q], v[2 * q + 1], fq);
    }
    if (m < a.M) {
      if constexpr (BF16OUT) {
#pragma unroll
        for (int q = 0; q < RN / 2; ++q) *(uint4*)((uint16_t*)a.C + orow * a.ldc + pcol + 32 * q) = pk[q];
      } else {
#pragma unroll
        for (int j = 0; j < RN; ++j) *(float4_t*)((float*)a.C + orow * a.ldc + ncol + 16 * j) = v[j];
      }
      if (epi & AACLIP_EPI_AUX_BF16) {
#pragma unroll
        for (int q = 0; q < RN / 2; ++q) *(uint4*)((uint16_t*)a.aux + orow * a.ldaux + pcol + 32 * q) = pk[q];
      }
    }
  }
}

// The 8-phase kernel's epilogue (OUTM 0 / 1, one wave's 128 x 64 tile): the same
// arithmetic as wave_epilogue, but every global access is quad-coalesced. In the
// accumulator layout consecutive lanes hold consecutive ROWS, so each 4-lane quad of a
// 16-B store or load touches 4 rows; the per-CU address path handles such an
// instruction at a third of the rate of one whose quads each cover 64 contiguous bytes
// (tools/atomic_bench.hip: 16-B stores 6.0k vs 2.0k cycles per 128 KiB, load + store
// 13.1k vs 5.6k, with 32 CUs busy). Each 16-row group goes through a per-wave LDS slot
// (written in the accumulator layout, read back with lane L on row L/4, 16-B chunk
// L%4 + 4k), XOR-swizzled so both sides are bank-conflict free; the residual is loaded,
// added and stored in the read-back layout (same fp32 adds, so the same bits). A
// wave's LDS operations execute in order, so the slot is reused without waits between
// groups.
// fp32 rows: 16 chunks of 16 B, chunk c of row r at c ^ f(r), f(r) = (r & 3) << 2 | r >> 2;
// 16-bit rows: 8 chunks, slot 8r + (c ^ g(r)), g(r) = ((r >> 1) & 1) << 2 | (r >> 2) & 3
// (16-bit rows with a residual take the fp32 form and store 8 B per lane).
// fp8 MX rows (OUTM 2, the fp8 kernel's c_fc): the 64-B row of e4m3 bytes after
// transpose_fq, 4 chunks, slot 4r + (c ^ (r >> 2)); SCALED 2 as in wave_epilogue.
template <int RM, int RN, int OUTM, int EPI, bool H16, int SCALED = 0, int PD = 2>
__device__ __forceinline__ void wave_epilogue_lds(const GemmArgs& a, float4_t (&acc)[RM][RN], int mw, int nw,
                                                  int lane, const float* lbias, char* slot) {
  static_assert(RN == 4 && OUTM >= 0 && OUTM <= 2, "one wave's 64 columns: fp32, 16-bit or fp8 MX rows");
  static_assert(SCALED == 0 || SCALED == 2, "no per-row A scales");
  static_assert(PD >= 2 && PD <= RM, "residual ring depth");
  constexpr bool BF16OUT = OUTM == 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int qr = lane >> 2, qc = lane & 3;  // read-back layout: row, first 16-B chunk
  const int epi = EPI >= 0 ? EPI : a.epi | (a.row_group > 0 ? EPI_REMAP : 0);
  auto out_row = [&](int m) { return (epi & EPI_REMAP) ? remap_row(a, m) : m; };
  const int ncol = nw + 4 * fq;
  float4_t bias[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j)
    bias[j] = (epi & AACLIP_EPI_BIAS) ? *(const float4_t*)((lbias ? lbias : a.bias) + ncol + 16 * j)
                                      : float4_t{0.f, 0.f, 0.f, 0.f};
  float4_t wsc[RN];  // fp8: per-column weight scales of this lane's 4 columns in tile j
  if constexpr (SCALED) {
#pragma unroll
    for (int j = 0; j < RN; ++j) wsc[j] = *(const float4_t*)(a.w_scale + ncol + 16 * j);
  }
  const int fw = ((fr & 3) << 2) | (fr >> 2), fqr = ((qr & 3) << 2) | (qr >> 2);
  const int gw = (((fr >> 1) & 1) << 2) | ((fr >> 2) & 3), gqr = (((qr >> 1) & 1) << 2) | ((qr >> 2) & 3);
  // residual of group i (read-back layout: row mw + 16 i + qr, columns nw + 4 qc + 16 k)
  float4_t res[PD][4];
  auto load_res = [&](int i, float4_t (&dst)[4]) {
    const float* src = a.res + (size_t)out_row(min(mw + 16 * i + qr, a.M - 1)) * a.ldr + nw + 4 * qc;
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = *(const float4_t*)(src + 16 * k);
  };
  if (epi & AACLIP_EPI_RESID) {
#pragma unroll
    for (int i = 0; i < PD - 1; ++i) load_res(i, res[i]);
  }
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    if ((epi & AACLIP_EPI_RESID) && i + PD - 1 < RM) load_res(i + PD - 1, res[(i + PD - 1) % PD]);
    // bias + activation of all four column tiles first (independent chains: the VALU
    // interleaves them; computing each tile at its LDS write measured 0.5 % slower)
    float4_t v[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      if constexpr (SCALED == 2)
        v[j] = acc[i][j] * wsc[j] + bias[j];
      else
        v[j] = acc[i][j] + bias[j];
      if (epi & AACLIP_EPI_GELU) {
        const float2_t lo = gelu_fast2(float2_t{v[j][0], v[j][1]}), hi = gelu_fast2(float2_t{v[j][2], v[j][3]});
        v[j] = float4_t{lo[0], lo[1], hi[0], hi[1]};
      }
      if (epi & AACLIP_EPI_QGELU) {
        const float2_t lo = qgelu_fast2(float2_t{v[j][0], v[j][1]}), hi = qgelu_fast2(float2_t{v[j][2], v[j][3]});
        v[j] = float4_t{lo[0], lo[1], hi[0], hi[1]};
      }
      if (epi & AACLIP_EPI_LEAKY)
#pragma unroll
        for (int t = 0; t < 4; ++t) v[j][t] = v[j][t] >= 0.f ? v[j][t] : 0.01f * v[j][t];
    }
    const int m = mw + 16 * i + qr;
    const size_t orow = (size_t)out_row(min(m, a.M - 1));
    if constexpr (OUTM == 2) {
      float amax = 0.f;
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) amax = fmaxf(amax, fabsf(v[j][t]));
      const int e = mx_exp(max_over_fq(amax));
      const float inv = pow2i(-e);
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(v[j][0] * inv, v[j][1] * inv, 0, false);
        d[j] = __builtin_amdgcn_cvt_pk_fp8_f32(v[j][2] * inv, v[j][3] * inv, w, true);
      }
      transpose_fq(d);  // lane (fr, fq): row fr, bytes 16 fq .. 16 fq + 15
      *(uint4*)(slot + (4 * fr + (fq ^ (fr >> 2))) * 16) = uint4{d[0], d[1], d[2], d[3]};
      const uint4 w = *(const uint4*)(slot + (4 * qr + (qc ^ (qr >> 2))) * 16);
      if (a.dbg & 2) {
        asm volatile("" ::"v"(w.x), "v"(w.y), "v"(w.z), "v"(w.w));
        continue;
      }
      if (m < a.M) *(uint4*)((uint8_t*)a.C + orow * a.ldc + nw + 16 * qc) = w;
      const int mr = mw + 16 * i + fr;  // the block scale: one byte per row, lanes fq = 0
      if (mr < a.M && fq == 0) {
        const int blk = nw >> 6;
        a.c_mx[((size_t)(blk >> 1) * a.ld_cmx + out_row(mr)) * 2 + (blk & 1)] = (uint8_t)(e + 127);
      }
      continue;
    }
    if (BF16OUT && !(epi & AACLIP_EPI_RESID)) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = 4 * q + 2 * (fq & 1) + (fq >> 1);
        *(uint4*)(slot + (fr * 8 + (c ^ gw)) * 16) = pair_h16<H16>(v[2 * q], v[2 * q + 1], fq);
      }
      uint4 w[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) w[k] = *(const uint4*)(slot + (qr * 8 + ((qc + 4 * k) ^ gqr)) * 16);
      if (a.dbg & 2) {  // diagnostic: everything but the global stores
#pragma unroll
        for (int k = 0; k < 2; ++k) asm volatile("" ::"v"(w[k].x), "v"(w[k].y), "v"(w[k].z), "v"(w[k].w));
        continue;
      }
      if (m < a.M) {
#pragma unroll
        for (int k = 0; k < 2; ++k) *(uint4*)((uint16_t*)a.C + orow * a.ldc + nw + 8 * qc + 32 * k) = w[k];
      }
    } else {
#pragma unroll
      for (int j = 0; j < RN; ++j) *(float4_t*)(slot + (fr * 16 + ((4 * j + fq) ^ fw)) * 16) = v[j];
      float4_t u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        u[k] = *(const float4_t*)(slot + (qr * 16 + ((qc + 4 * k) ^ fqr)) * 16);
        if (epi & AACLIP_EPI_RESID) u[k] += res[i % PD][k];
      }
      if (a.dbg & 2) {
#pragma unroll
        for (int k = 0; k < 4; ++k) asm volatile("" ::"v"(u[k]));
        continue;
      }
      if (m < a.M && BF16OUT) {  // 16-bit rows with a residual: 8 B per lane
#pragma unroll
        for (int k = 0; k < 4; ++k)
          *(uint2*)((uint16_t*)a.C + orow * a.ldc + nw + 4 * qc + 16 * k) =
              uint2{pack_h16x2<H16>(u[k][0], u[k][1]), pack_h16x2<H16>(u[k][2], u[k][3])};
      } else if (m < a.M) {
#pragma unroll
        for (int k = 0; k < 4; ++k) *(float4_t*)((float*)a.C + orow * a.ldc + nw + 4 * qc + 16 * k) = u[k];
        if (epi & AACLIP_EPI_AUX_BF16) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            *(uint2*)((uint16_t*)a.aux + orow * a.ldaux + nw + 4 * qc + 16 * k) =
                uint2{pack_h16x2<H16>(u[k][0], u[k][1]), pack_h16x2<H16>(u[k][2], u[k][3])};
        }
      }
    }
  }
}

// ==================================================== bf16 / fp8 MFMA kernel
// FP8: A and W are OCP e4m3 bytes with a per-row (A) and per-output-channel (W)
// fp32 scale folded into the epilogue; the main loop runs the block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit (e8m0 127) block scales -- the
// K=128 form runs at 2x the bf16 MFMA rate. The LDS image is the same 128-byte
// row per K-step (64 bf16 or 128 fp8 elements), so staging is shared; a lane's
// fp8 fragment is 32 consecutive K bytes = two swizzled 16-B chunks.
typedef __attribute__((ext_vector_type(8))) int i32x8_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;

// Q: 0 = bf16, 1 = fp8 with per-row A scales (epilogue), 2 = fp8 MX: A carries an
// e8m0 scale per (row, 64-K block) staged through LDS next to the tiles and applied
// by the MFMA's B-operand scale (the A tile is the MFMA's second operand).
// H16 (Q == 0 only): fp16 operands on v_mfma_f32_16x16x32_f16 (same tiles and cycles).
template <int BM, int BN, int WM, int WN, int Q = 0, bool H16 = false, int KS = 0>
__global__ __launch_bounds__(WM * WN * 64) void gemm_bf16_kernel(GemmArgs a) {
  AACLIP_TRACE_SCOPE(TR_GEMM_TILE | gemm_trace_tag(a));
  static_assert(!H16 || Q == 0, "fp16 operands: 16-bit path only");
  constexpr bool FP8 = Q != 0, MX = Q == 2;
  constexpr int NWAVES = WM * WN;
  constexpr int ES = FP8 ? 1 : 2;  // element bytes
  constexpr int BK = 128 / ES;     // K elements per stage (128 bytes per row)
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int RM = TM / 16, RN = TN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_LOADS = A_BYTES / (NWAVES * 1024);  // glds per wave per tile
  constexpr int B_LOADS = B_BYTES / (NWAVES * 1024);
  static_assert(A_LOADS * NWAVES * 1024 == A_BYTES && B_LOADS * NWAVES * 1024 == B_BYTES, "tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  static_assert(KS == 0 || !FP8, "split-K: 16-bit operands only");
  int tm, tn, kh = 0;
  if constexpr (KS > 1) {
    if (!split_coords(a, blockIdx.x, tm, tn, kh)) return;  // a slot past this XCD's run of tiles
  } else {
    tile_coords(blockIdx.x, a.tiles_m, a.tiles_n, tm, tn, a.group_m);
  }
  const int m0 = tm * BM, n0 = tn * BN;
  int kb0 = 0, nk = a.K / BK;  // this part's K-steps [kb0, kb0 + nk)
  if constexpr (KS > 1) {
    int kb1;
    split_range(nk, KS, kh, kb0, kb1);
    nk = kb1 - kb0;
  }

  const char* __restrict__ Ag = (const char*)a.A;
  const char* __restrict__ Wg = (const char*)a.W;

  // Per-lane source pointers for the DMA pieces (row r = piece*8 + lane/8,
  // physical 16-B chunk p = lane%8 holds logical chunk p ^ (r&7)).
  const char* a_src[A_LOADS];
  const char* b_src[B_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i) {
    const int r = (i * NWAVES + wid) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const int gr = min(m0 + r, a.M - 1);
    a_src[i] = Ag + ((size_t)gr * a.lda) * ES + c * 16 + kb0 * 128;
  }
#pragma unroll
  for (int i = 0; i < B_LOADS; ++i) {
    const int r = (i * NWAVES + wid) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    b_src[i] = Wg + ((size_t)(n0 + r) * a.ldw) * ES + c * 16 + kb0 * 128;
  }

  // MX: the A tile's scales for K-step kt = BM rows x 2 bytes, contiguous in the
  // [K/128][ld_amx][2] layout; BM/128 waves DMA one dword per lane
  constexpr int SC_BYTES = BM * 2;
  const auto srs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.a_mx, 0, MX ? (int)((a.K / 128) * a.ld_amx * 2) : 0, 0x00020000);
  auto stage_scales = [&](int kt, int buf) {
    if constexpr (MX) {
      if (wid < SC_BYTES / 256)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(srs, LDS_PTR(smem + 2 * STAGE_BYTES + buf * SC_BYTES + wid * 256), 4,
                                                 (m0 * 2 + wid * 256 + lane * 4), (int)(kt * a.ld_amx * 2), 0, 0);
    }
  };

#define GEMM_STAGE(kt, buf)                                                                  \
  do {                                                                                       \
    stage_scales(kt, buf);                                                                   \
    char* base_ = smem + (buf) * STAGE_BYTES;                                                \
    const int koff_ = (kt) * 128;                                                            \
    _Pragma("unroll") for (int i = 0; i < A_LOADS; ++i)                                      \
      __builtin_amdgcn_global_load_lds((const void*)(a_src[i] + koff_),                      \
                                       LDS_PTR(base_ + (i * NWAVES + wid) * 1024), 16, 0, 0); \
    _Pragma("unroll") for (int i = 0; i < B_LOADS; ++i)                                      \
      __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + koff_),                      \
                                       LDS_PTR(base_ + A_BYTES + (i * NWAVES + wid) * 1024), \
                                       16, 0, 0);                                            \
  } while (0)


  float4_t acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes within a stage): 16-B chunk kk*4 + fq of the row.
  // bf16: kk = 0/1 half of the 64-element K-step. fp8: the lane's 32-byte fragment
  // of the 128-element K-step is chunks fq and 4 + fq -- the K=128 MFMA takes a
  // lane's bytes 0-15 as K 16fq.. and bytes 16-31 as K 64+16fq.. (probed with
  // tools/mxprobe.py), so hardware 32-K block b is logical K 32b..32b+31 and the
  // lane supplying its e8m0 scale (lane group b) owns exactly that range.
  const int fr = lane & 15, fq = lane >> 4;
  auto chunk = [&](int kk) { return kk * 4 + fq; };
  int a_off[RM][2], b_off[RN][2];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int r = wm * TM + i * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) a_off[i][kk] = r * 128 + ((chunk(kk) ^ (r & 7)) << 4);
  }
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int r = wn * TN + j * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) b_off[j][kk] = A_BYTES + r * 128 + ((chunk(kk) ^ (r & 7)) << 4);
  }

  GEMM_STAGE(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) GEMM_STAGE(kt + 1, cur ^ 1);
    const char* base = smem + cur * STAGE_BYTES;
    if (a.setprio) __builtin_amdgcn_s_setprio(1);
    if constexpr (FP8) {
      i32x8_t bf[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int4 lo = *(const int4*)(base + b_off[j][0]), hi = *(const int4*)(base + b_off[j][1]);
        bf[j] = i32x8_t{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      }
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int4 lo = *(const int4*)(base + a_off[i][0]), hi = *(const int4*)(base + a_off[i][1]);
        const i32x8_t af = i32x8_t{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        int sb = 127;  // e8m0 2^0
        if constexpr (MX)  // this lane's A block: row wm*TM + 16i + fr, 64-block fq/2 of the K-step
          sb = *(const uint8_t*)(smem + 2 * STAGE_BYTES + cur * SC_BYTES + (wm * TM + 16 * i + fr) * 2 + (fq >> 1));
#pragma unroll
        for (int j = 0; j < RN; ++j)  // formats 0/0 = e4m3/e4m3; W block scale 2^0, A block scale sb
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af, acc[i][j], 0, 0, 0, 127, 0, sb);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        using V8 = h16x8_t<H16>;
        V8 bf[RN];
#pragma unroll
        for (int j = 0; j < RN; ++j) bf[j] = *(const V8*)(base + b_off[j][kk]);
#pragma unroll
        for (int i = 0; i < RM; ++i) {
          const V8 af = *(const V8*)(base + a_off[i][kk]);
#pragma unroll
          for (int j = 0; j < RN; ++j) acc[i][j] = mfma16(bf[j], af, acc[i][j]);  // C^T tile
        }
      }
    }
    if (a.setprio) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
  }

  if (a.dbg & 1) {  // diagnostic timing path: keep the MFMA results live, store nothing
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  if constexpr (KS > 1) {
    if (!ksplit_combine<KS, RM, RN>(a, acc, tm * a.tiles_n + tn, kh, NWAVES, wid, lane, (int*)smem))
      return;  // not the last part of this tile: its partial is stored
  }
  const int mw = m0 + wm * TM, nw = n0 + wn * TN;
  const int key = a.epi | (a.row_group > 0 ? EPI_REMAP : 0);
  constexpr int SC = Q == 1 ? 1 : (Q == 2 ? 2 : 0);
  const int outm =
      a.out_dtype == AACLIP_F32 ? 0 : (a.out_dtype == AACLIP_FP8 ? 2 : (a.out_dtype == kOutScores ? 3 : 1));
#define EPI_CASE(OM, E)                                                \
  if (outm == (OM) && key == (E)) {                                    \
    wave_epilogue<RM, RN, OM, E, SC, H16>(a, acc, mw, nw, lane);       \
    return;                                                            \
  }
  // the combinations the visual/text engines issue (engine.py)
  EPI_CASE(1, AACLIP_EPI_BIAS)                                        // qkv
  EPI_CASE(1, AACLIP_EPI_BIAS | AACLIP_EPI_GELU)                      // c_fc
  EPI_CASE(1, AACLIP_EPI_BIAS | AACLIP_EPI_QGELU)                     // c_fc, quick_gelu towers
  EPI_CASE(0, AACLIP_EPI_BIAS | AACLIP_EPI_RESID)                     // out-proj, c_proj
  EPI_CASE(0, AACLIP_EPI_BIAS | AACLIP_EPI_RESID | AACLIP_EPI_AUX_BF16)  // c_proj + bf16 copy
  EPI_CASE(0, AACLIP_EPI_BIAS)                                        // out-proj, deferred residual
  EPI_CASE(0, AACLIP_EPI_LEAKY)                                       // adapters, seg/det proj
  EPI_CASE(0, 0)                                                      // seg/det proj (no relu)
  EPI_CASE(0, EPI_REMAP)                                              // patch embedding
  if constexpr (!FP8 && (BN / WN == 64 || BN / WN == 32)) {
    EPI_CASE(3, AACLIP_EPI_LEAKY)                                     // seg/det proj -> map partials
    EPI_CASE(3, 0)
  }
  if constexpr (BN / WN == 64) {
    EPI_CASE(2, AACLIP_EPI_BIAS | AACLIP_EPI_GELU)                    // c_fc -> fp8 MX c_proj input
    EPI_CASE(2, AACLIP_EPI_BIAS | AACLIP_EPI_QGELU)
  }
#undef EPI_CASE
  if (outm == 1)
    wave_epilogue<RM, RN, 1, -1, SC, H16>(a, acc, mw, nw, lane);
  else if (outm == 0)
    wave_epilogue<RM, RN, 0, -1, SC, H16>(a, acc, mw, nw, lane);
}

// ============================================================== fp32 MFMA kernel
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs a) {
  AACLIP_TRACE_SCOPE(TR_GEMM_F32 | gemm_trace_tag(a));
  constexpr int BM = 64, BN = 64, BK = 16, LDK = BK + 1;
  __shared__ float As[BM][LDK];
  __shared__ float Bs[BN][LDK];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int tm, tn;
  tile_coords(blockIdx.x, a.tiles_m, a.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const float* Ag = (const float*)a.A;
  const float* Wg = (const float*)a.W;
  const int lr = threadIdx.x >> 2, lc = (threadIdx.x & 3) * 4;
  const float* a_src = Ag + (size_t)min(m0 + lr, a.M - 1) * a.lda + lc;
  const float* b_src = Wg + (size_t)(n0 + lr) * a.ldw + lc;
  float4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = lane >> 4;
  for (int k0 = 0; k0 < a.K; k0 += BK) {
    const float4_t av = *(const float4_t*)(a_src + k0);
    const float4_t bv = *(const float4_t*)(b_src + k0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      As[lr][lc + j] = av[j];
      Bs[lr][lc + j] = bv[j];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      float af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = As[wm * 32 + i * 16 + fr][ks * 4 + fk];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = Bs[wn * 32 + j * 16 + fr][ks * 4 + fk];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + wm * 32 + i * 16 + fk * 4 + e;
      if (m < a.M) {
#pragma unroll
        for (int j = 0; j < 2; ++j) epilogue_store1(a, m, n0 + wn * 32 + j * 16 + fr, acc[i][j][e]);
      }
    }
}

// ================================ 8-phase ping-pong bf16 kernel (256x256x64)
// The K-step is cut into 4 phases, one per C quadrant of the wave tile (64x32 =
// 4x2 MFMA tiles x 2 k-halves = 16 MFMAs). Each phase: ds_read the quadrant's
// register subtile, issue ONE 16-KiB LDS region of a later K-step (2 LDS-DMA per
// thread), counted vmcnt, barrier, MFMA cluster, barrier. The two wave rows are
// staggered by one barrier, so on every SIMD one wave runs its MFMA cluster while
// the other issues its LDS reads and DMA (ping-pong). LDS per stage = 4 regions of
// 128 rows x 128 B grouped by the phase that first reads them:
//   A0 = rows {0..63, 128..191} (A sub-block 0 of both wave rows), A1 = the other
//   rows, B0 / B1 = the first / second 32 W-rows of every wave column.
// Phase reads: P1 A0+B0, P2 B1, P3 A1, P4 -- and issues (K-step k): P1 B1(k+1),
// P2 A1(k+1), P3 A0(k+2), P4 B0(k+2): every region is rewritten >= 2 phases after
// its last read (WAR) and lands 5-6 phases before it is read; each phase's
// vmcnt(8) (4 regions of 2 DMAs in flight) retires the region the next phase
// reads (RAW: read one phase after the wait, past both groups' barriers).
// The last two K-steps issue nothing past the end and count their waits down (below).
// Operands via buffer descriptors (rows >= M read as zero; outputs dropped by the
// epilogue's bound check).
// (A persistent form -- one workgroup per CU walking tiles, the next tile's first
// K-steps fetched by the phantom loads under the epilogue -- measured -1.0 % in the C2
// step and was removed in round 5; it is in the round-4 history, family 5.)
// SCORES: the instantiation for aaclip_gemm_scores (OUTM 3 epilogue only), so the
// anomaly-map partials path adds no registers to the block-GEMM instantiations.
#ifdef AACLIP_PHASE_STAMPS
constexpr int kKsplitFlag = 2 * 4 * 128 * 128 + 1024 + 8 * 8 * 4 * 2 * 8;  // LDS byte offset of the split-K flag
#else
constexpr int kKsplitFlag = 2 * 4 * 128 * 128 + 1024;
#endif

template <bool H16, bool SCORES = false, int KS = 0>
__global__ __launch_bounds__(512) void gemm_bf16_8ph_kernel(GemmArgs a) {
  AACLIP_TRACE_SCOPE(TR_GEMM_8PH | gemm_trace_tag(a));
  using V8 = h16x8_t<H16>;
  constexpr int BM = 256, BN = 256, TM = 128, TN = 64, RM = 8, RN = 4;
  constexpr int REGION = 128 * 128;                 // bytes per LDS region
  constexpr int STAGE = 4 * REGION;                 // A0, A1, B0, B1
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const auto ars = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (int)((uint32_t)a.M * (uint32_t)a.lda * 2u),
                                                     0x00020000);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, (int)((uint32_t)a.N * (uint32_t)a.ldw * 2u),
                                                     0x00020000);
  // DMA: thread t fills row t/8 of a 64-row piece, physical 16-B chunk t%8 holds
  // logical chunk (t%8) ^ (row%8) (row%8 = (t/8)%8 in every piece)
  const int prow = t >> 3;
  const int pchunk = ((t & 7) ^ (prow & 7)) * 8;
  auto a_vo_of = [&](int m0) { return ((m0 + prow) * (int)a.lda + pchunk) * 2; };
  auto w_vo_of = [&](int n0) { return ((n0 + ((prow >> 5) & 1) * 64 + (prow & 31)) * (int)a.ldw + pchunk) * 2; };
  const int a_row = (int)a.lda * 2, w_row = (int)a.ldw * 2;  // bytes per row
  int nk = a.K / 64;
  static_assert(KS == 0 || !SCORES, "split-K: block GEMMs only");
  int tm, tn, kh = 0, kb0 = 0;
  if constexpr (KS > 1) {
    if (!split_coords(a, blockIdx.x, tm, tn, kh)) return;  // a slot past this XCD's run of tiles
    int kb1;
    split_range(nk, KS, kh, kb0, kb1);
    nk = kb1 - kb0;  // this part's K-steps [kb0, kb1): the operands' voffsets start at kb0
  } else {
    tile_coords(blockIdx.x, a.tiles_m, a.tiles_n, tm, tn, a.group_m);
  }
  const int avo = a_vo_of(tm * BM) + kb0 * 128, wvo = w_vo_of(tn * BN) + kb0 * 128;
  // region r of K-step kt into stage kt&1 (r: 0 = A0, 1 = A1, 2 = B0, 3 = B1)
  auto issue = [&](int r, int kt) {
    const int kc = kt * 128;
    char* dst = smem + (kt & 1) * STAGE + r * REGION;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (r < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, LDS_PTR(dst + g * 8192 + wid * 1024), 16, avo,
                                                 (g * 128 + r * 64) * a_row + kc, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, LDS_PTR(dst + g * 8192 + wid * 1024), 16, wvo,
                                                 (g * 128 + (r - 2) * 32) * w_row + kc, 0, 0);
    }
  };
  // fragment offsets inside a region: local row (A: wr*64 + 16i + fr, B: wc*32 + 16j + fr),
  // 16-B chunk (kk*4 + fq) ^ (fr & 7)
  int a_rd[2], b_rd[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int sw = ((kk * 4 + fq) ^ (fr & 7)) << 4;
    a_rd[kk] = (wr * 64 + fr) * 128 + sw;
    b_rd[kk] = 2 * REGION + (wc * 32 + fr) * 128 + sw;
  }
  float4_t acc[RM][RN];
  V8 af[4][2], bfr[2][2][2];  // A sub-block (4 tiles x kk), B sub-blocks [q][j][kk]

  // the tile's 256 bias values into LDS behind the ring (one 1-KiB DMA by wave 0, retired by
  // the prologue's vmcnt(8) as the oldest op): the epilogue reads them from LDS instead of
  // waiting out a global-load round trip at its start
  const bool lds_bias = !SCORES && (a.epi & AACLIP_EPI_BIAS);
  if (lds_bias && wid == 0) {
    const auto brs = __builtin_amdgcn_make_buffer_rsrc((void*)a.bias, 0, (int)((uint32_t)a.N * 4u), 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, LDS_PTR(smem + 2 * STAGE), 16, (tn * BN + 4 * lane) * 4, 0, 0, 0);
  }
  // prologue: all of K-step 0, then A0 / B0 of K-step 1 (the steady state's P3/P4 of K-step -1)
  issue(0, 0);
  issue(2, 0);
  issue(3, 0);
  issue(1, 0);
  if (nk > 1) {
    issue(0, 1);
    issue(2, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A0(0), B0(0) landed
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // one K-step: B1(0), A1(0) may fly
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: wave row 1 runs one barrier behind
  // No s_setprio flips around the MFMA clusters (the sched_barrier fences already pin each
  // cluster between its barriers): C2 step +0.8 % over setprio 1/0 around every cluster;
  // a static prio 1 for the younger wave row measured the same as none, keeping the flips
  // for the older row -2.5 % (profiles/r04/gemm_8ph_priority_ab.txt)

  auto mfma_q = [&](int qa, int qb) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qa * 4 + i][qb * 2 + j] = mfma16(bfr[qb][j][kk], af[i][kk], acc[qa * 4 + i][qb * 2 + j]);
  };
  auto read_a = [&](const char* st, int q) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = *(const V8*)(st + q * REGION + a_rd[kk] + i * 2048);
  };
  auto read_b = [&](const char* st, int q) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        bfr[q][j][kk] = *(const V8*)(st + q * REGION + b_rd[kk] + j * 2048);
  };
#define PH_SYNC_MFMA(QA, QB, W)                              \
  asm volatile("s_waitcnt vmcnt(" #W ")" ::: "memory");      \
  __builtin_amdgcn_s_barrier();                              \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");         \
  PHASE_STAMP_A                                              \
  __builtin_amdgcn_sched_barrier(0);                         \
  mfma_q(QA, QB);                                            \
  __builtin_amdgcn_sched_barrier(0);                         \
  PHASE_STAMP_B                                              \
  __builtin_amdgcn_s_barrier();                              \
  PHASE_STAMP_STORE

  const bool bf16_out = a.out_dtype != AACLIP_F32;
  const int key = a.epi | (a.row_group > 0 ? EPI_REMAP : 0);
  // diagnostic stamps (variant bit 11): shader-clock s_memtime at kernel start, main-loop
  // end, epilogue issued, epilogue stores complete -> a.aux
  const bool stamp = (a.dbg & 4) && a.aux && !(a.epi & AACLIP_EPI_AUX_BF16);
#ifdef AACLIP_PHASE_STAMPS
  // diagnostic build (tools/ab_build.sh ... -DAACLIP_PHASE_STAMPS, tools/gemm_phase_stamps.py): every
  // wave stamps s_memtime at the start and the end of each MFMA cluster of K-steps 4..11 (taken right
  // after the pre-cluster lgkmcnt(0) and after the cluster), kept in LDS and copied to a.aux at the end
  // in place of the 4 stamps of variant bit 11 (needs K >= 768)
  constexpr int kPS0 = 4, kPSN = 8;  // K-steps stamped
  uint64_t* const ps_lds = (uint64_t*)(smem + 2 * STAGE + 1024) + wid * kPSN * 4 * 2;
  int ps_i = 0;  // phase index since kernel start
  uint64_t ps_a = 0, ps_b = 0;
  // the previous phase's pair is stored at the next cluster start, right after that phase's
  // lgkmcnt(0) has retired both s_memtime reads: the stamps add no wait of their own
#define PHASE_STAMP_A                                                                       \
  {                                                                                         \
    const int q_ = ps_i - 1 - 4 * kPS0;                                                     \
    if (q_ >= 0 && q_ < 4 * kPSN && lane == 0) {                                            \
      ps_lds[2 * q_] = ps_a;                                                                \
      ps_lds[2 * q_ + 1] = ps_b;                                                            \
    }                                                                                       \
    ps_a = __builtin_amdgcn_s_memtime();                                                    \
  }
#define PHASE_STAMP_B ps_b = __builtin_amdgcn_s_memtime();
#define PHASE_STAMP_STORE ++ps_i;
#else
#define PHASE_STAMP_A
#define PHASE_STAMP_B
#define PHASE_STAMP_STORE
#endif
  uint64_t ts[4] = {0, 0, 0, 0};
  if (stamp) ts[0] = __builtin_amdgcn_s_memtime();
  const int m0 = tm * BM, n0 = tn * BN;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
  // One K-step: P1 A0 x B0, P2 A0 x B1, P3 A1 x B1, P4 A1 x B0, each phase's counted wait
  // W1..W4; I1 / I2: the K-step issues its regions of K-steps kt+1 / kt+2.
#define PH_KSTEP(KT, W1, W2, W3, W4, I1, I2)        \
  {                                                 \
    const char* st = smem + ((KT) & 1) * STAGE;     \
    read_b(st, 0);                                  \
    read_a(st, 0);                                  \
    if (I1) issue(3, (KT) + 1);                     \
    PH_SYNC_MFMA(0, 0, W1)                          \
    read_b(st, 1);                                  \
    if (I1) issue(1, (KT) + 1);                     \
    PH_SYNC_MFMA(0, 1, W2)                          \
    read_a(st, 1);                                  \
    if (I2) issue(0, (KT) + 2);                     \
    PH_SYNC_MFMA(1, 1, W3)                          \
    if (I2) issue(2, (KT) + 2);                     \
    PH_SYNC_MFMA(1, 0, W4)                          \
  }
  int kt = 0;
  for (; kt < nk - 2; ++kt) PH_KSTEP(kt, 8, 8, 8, 8, true, true)
  // The last two K-steps issue nothing past the last K-step: in K-step nk-2 P3 / P4 issue
  // nothing, so P4 waits for A0 / B0 of nk-1 with only B1 / A1 of nk-1 left in flight
  // (vmcnt 4); in K-step nk-1 P1 leaves A1 (vmcnt 2) and P2 drains. (Until round 5 the
  // steady-state body ran to the end with phantom re-reads of the last K-step -- 1.5 K-steps
  // of DMA per tile nobody read, still in flight ahead of the epilogue's own loads.)
  if (nk >= 2) {
    PH_KSTEP(kt, 8, 8, 8, 4, true, false)
    ++kt;
  }
  PH_KSTEP(kt, 2, 0, 0, 0, false, false)
#undef PH_KSTEP
  // both wave rows run the epilogue together (row 0 waits out row 1's last phase)
  if (wr == 0) __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // the epilogue's LDS slot writes stay behind that barrier
  // split-K: the flag word sits past the ring and the staged bias (+16 B in launch_bf16_8ph)
  if constexpr (KS > 1) {
    if (!ksplit_combine<KS, RM, RN>(a, acc, tm * a.tiles_n + tn, kh, 8, wid, lane, (int*)(smem + kKsplitFlag)))
      return;  // not the last part of this tile: its partial is stored
  }
  const int mw = m0 + wr * TM, nw = n0 + wc * TN;
  const float* lbp = (const float*)(smem + 2 * STAGE) - n0;  // staged bias, by column
  // the epilogue's per-wave 4-KiB LDS slot: regions A1 / B1 of the last K-step's stage,
  // whose last reads (P3 / P2) every wave finished before the barrier above (no DMA is
  // issued after the last K-step's regions)
  char* slot = smem + ((nk - 1) & 1) * STAGE + (wr ? 3 : 1) * REGION + wc * 4096;
  if (stamp) ts[1] = __builtin_amdgcn_s_memtime();
  if (a.dbg & 1) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) asm volatile("" ::"v"(acc[i][j]));
  } else if constexpr (SCORES) {  // seg/det proj -> map partials
    if (key == AACLIP_EPI_LEAKY)
      wave_epilogue<RM, RN, 3, AACLIP_EPI_LEAKY, 0, H16>(a, acc, mw, nw, lane);
    else
      wave_epilogue<RM, RN, 3, 0, 0, H16>(a, acc, mw, nw, lane);
  } else {
#define EPI_CASE(BF, E)                                                                          \
  if (bf16_out == (BF) && key == (E)) {                                                          \
    wave_epilogue_lds<RM, RN, BF ? 1 : 0, E, H16>(a, acc, mw, nw, lane,                          \
                                                  ((E) & AACLIP_EPI_BIAS) ? lbp : nullptr, slot); \
  } else
    EPI_CASE(true, AACLIP_EPI_BIAS)
    EPI_CASE(true, AACLIP_EPI_BIAS | AACLIP_EPI_GELU)
    EPI_CASE(true, AACLIP_EPI_BIAS | AACLIP_EPI_QGELU)
    EPI_CASE(false, AACLIP_EPI_BIAS | AACLIP_EPI_RESID)
    EPI_CASE(false, AACLIP_EPI_BIAS | AACLIP_EPI_RESID | AACLIP_EPI_AUX_BF16)
    EPI_CASE(false, AACLIP_EPI_LEAKY)
#undef EPI_CASE
    // any other flag combination (row remap, 16-bit rows + residual, ...): run-time flags
    if (bf16_out)
      wave_epilogue_lds<RM, RN, 1, -1, H16>(a, acc, mw, nw, lane, lds_bias ? lbp : nullptr, slot);
    else
      wave_epilogue_lds<RM, RN, 0, -1, H16>(a, acc, mw, nw, lane, lds_bias ? lbp : nullptr, slot);
  }
#undef PH_SYNC_MFMA
#undef PHASE_STAMP_A
#undef PHASE_STAMP_B
#undef PHASE_STAMP_STORE
  if (stamp) ts[2] = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every load / store retired before exit
  if (stamp) {
    ts[3] = __builtin_amdgcn_s_memtime();
#ifdef AACLIP_PHASE_STAMPS
    if (lane < 2 * 4 * kPSN) ((uint64_t*)a.aux)[((size_t)blockIdx.x * 8 + wid) * 2 * 4 * kPSN + lane] = ps_lds[lane];
#else
    if (lane < 4) ((uint64_t*)a.aux)[((size_t)blockIdx.x * 8 + wid) * 4 + lane] = ts[lane];
#endif
  }
}

// ============================ 8-phase ping-pong fp8 MX kernel (256x256, K-step 128)
// The bf16 8-phase schedule above on e4m3 operands: a 128-byte LDS row is one
// 128-K step, each phase is 4x2 K=128 MFMAs (256 cycles, as 16 bf16 MFMAs), and the
// A tile's e8m0 block scales (512 B per K-step) ride in a 3-slot LDS ring issued in
// P3 with region A0: every wave issues one dword LDS-DMA there (waves 0-1 carry the
// 512 B, waves 2-7 write a scratch area nobody reads) so the per-phase DMA counts
// (2, 2, 3, 2) are uniform and any 4 consecutive phases hold 9 -> vmcnt(9). Slot
// (k+2)%3 is rewritten at P3(k), 4 phases after K-step k-1's last scale read.
__global__ __launch_bounds__(512) void gemm_fp8mx_8ph_kernel(GemmArgs a) {
  AACLIP_TRACE_SCOPE(TR_GEMM_FP8MX | gemm_trace_tag(a));
  constexpr int BM = 256, BN = 256, TM = 128, TN = 64, RM = 8, RN = 4;
  constexpr int REGION = 128 * 128;
  constexpr int STAGE = 4 * REGION;
  constexpr int SCB = 2 * STAGE, SC_SLOT = 512;  // 3 scale slots, then 6 x 256 B scratch
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  int tm, tn;
  tile_coords(blockIdx.x, a.tiles_m, a.tiles_n, tm, tn, a.group_m);
  const int m0 = tm * BM, n0 = tn * BN;
  const auto ars = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (int)((uint32_t)a.M * (uint32_t)a.lda),
                                                     0x00020000);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, (int)((uint32_t)a.N * (uint32_t)a.ldw),
                                                     0x00020000);
  const auto srs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.a_mx, 0, (int)((a.K / 128) * a.ld_amx * 2), 0x00020000);
  const int prow = t >> 3;
  const int pchunk = ((t & 7) ^ (prow & 7)) * 16;
  const int a_vo = (m0 + prow) * (int)a.lda + pchunk;
  const int w_vo = (n0 + ((prow >> 5) & 1) * 64 + (prow & 31)) * (int)a.ldw + pchunk;
  const int a_row = (int)a.lda, w_row = (int)a.ldw;
  const int nk = a.K / 128;
  auto issue = [&](int r, int kt) {
    const int kc = kt * 128;
    char* dst = smem + (kt & 1) * STAGE + r * REGION;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (r < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, LDS_PTR(dst + g * 8192 + wid * 1024), 16, a_vo,
                                                 (g * 128 + r * 64) * a_row + kc, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, LDS_PTR(dst + g * 8192 + wid * 1024), 16, w_vo,
                                                 (g * 128 + (r - 2) * 32) * w_row + kc, 0, 0);
    }
  };
  // scale slot of K-step kt is kt % 3; waves 2..7 park their (unused) DMA lanes in
  // scratch. Branch-free on purpose: a branch here splits the loop body into two
  // blocks and the (memory-free) MFMAs then get sunk across the phase barriers.
  auto issue_sc = [&](int kt, int slot) {
    const int kc = kt;
    const int lo = (int)(wid < 2);
    const int off = lo * (slot * SC_SLOT + wid * 256) + (1 - lo) * (3 * SC_SLOT + (wid - 2) * 256);
    char* dst = smem + SCB + off;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(srs, LDS_PTR(dst), 4, m0 * 2 + (wid & 1) * 256 + lane * 4,
                                             (int)(kc * a.ld_amx * 2), 0, 0);
  };
  int a_rd[2], b_rd[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int sw = ((kk * 4 + fq) ^ (fr & 7)) << 4;
    a_rd[kk] = (wr * 64 + fr) * 128 + sw;
    b_rd[kk] = 2 * REGION + (wc * 32 + fr) * 128 + sw;
  }
  float4_t acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
  i32x8_t af[4], bfr[2][2];
  int sa[4];

  // prologue = the steady state's P3(-2), P4(-2), P1(-1), P2(-1), P3(-1), P4(-1) issues
  issue(0, 0);
  issue_sc(0, 0);
  issue(2, 0);
  issue(3, 0);
  issue(1, 0);
  if (nk > 1) {
    issue(0, 1);
    issue_sc(1, 1);
    issue(2, 1);
    asm volatile("s_waitcnt vmcnt(9)" ::: "memory");  // A0(0), SC(0), B0(0) landed
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // one K-step: B1(0), A1(0) may fly
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();

  auto frag = [&](const char* p0, const char* p1) {
    const i32x4_t lo = *(const i32x4_t*)p0, hi = *(const i32x4_t*)p1;
    return i32x8_t{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  };
  auto read_a = [&](const char* st, int q, int slot) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i] = frag(st + q * REGION + a_rd[0] + i * 2048, st + q * REGION + a_rd[1] + i * 2048);
      sa[i] = *(const uint8_t*)(smem + SCB + slot * SC_SLOT + (wr * 128 + q * 64 + 16 * i + fr) * 2 + (fq >> 1));
    }
  };
  auto read_b = [&](const char* st, int q) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bfr[q][j] = frag(st + q * REGION + b_rd[0] + j * 2048, st + q * REGION + b_rd[1] + j * 2048);
  };
  auto mfma_q = [&](int qa, int qb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[qa * 4 + i][qb * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            bfr[qb][j], af[i], acc[qa * 4 + i][qb * 2 + j], 0, 0, 0, 127, 0, sa[i]);
    __builtin_amdgcn_s_setprio(0);
  };
#define PH_SYNC_MFMA(QA, QB, W)                              \
  asm volatile("s_waitcnt vmcnt(" #W ")" ::: "memory");      \
  __builtin_amdgcn_s_barrier();                              \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");         \
  __builtin_amdgcn_sched_barrier(0);                         \
  mfma_q(QA, QB);                                            \
  __builtin_amdgcn_sched_barrier(0);                         \
  __builtin_amdgcn_s_barrier();

  int slot = 0, slot2 = 2;  // kt % 3, (kt + 2) % 3
  // one K-step with its four counted waits; I1 / I2: it issues K-step kt+1's / kt+2's
  // regions (compile-time constants at every use: no branch splits the body)
#define MX_KSTEP(KT, W1, W2, W3, W4, I1, I2)        \
  {                                                 \
    const char* st = smem + ((KT) & 1) * STAGE;     \
    read_b(st, 0); /* P1: A0 x B0 */                \
    read_a(st, 0, slot);                            \
    if (I1) issue(3, (KT) + 1);                     \
    PH_SYNC_MFMA(0, 0, W1)                          \
    read_b(st, 1); /* P2: A0 x B1 */                \
    if (I1) issue(1, (KT) + 1);                     \
    PH_SYNC_MFMA(0, 1, W2)                          \
    read_a(st, 1, slot); /* P3: A1 x B1 */          \
    if (I2) {                                       \
      issue(0, (KT) + 2);                           \
      issue_sc((KT) + 2, slot2);                    \
    }                                               \
    PH_SYNC_MFMA(1, 1, W3)                          \
    if (I2) issue(2, (KT) + 2); /* P4: A1 x B0 */   \
    PH_SYNC_MFMA(1, 0, W4)                          \
    slot = slot == 2 ? 0 : slot + 1;                \
    slot2 = slot2 == 2 ? 0 : slot2 + 1;             \
  }
  int kt = 0;
  for (; kt < nk - 2; ++kt) MX_KSTEP(kt, 9, 9, 9, 9, true, true)
  // the last two K-steps issue nothing past the end (as the bf16 kernel): P4 of K-step nk-2
  // leaves B1 / A1 of nk-1 in flight (vmcnt 4), P1 of nk-1 only A1 (2), P2 drains
  if (nk >= 2) {
    MX_KSTEP(kt, 9, 9, 9, 4, true, false)
    ++kt;
  }
  MX_KSTEP(kt, 2, 0, 0, 0, false, false)
#undef MX_KSTEP
#undef PH_SYNC_MFMA
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wr == 0) __builtin_amdgcn_s_barrier();
  if (a.dbg & 1) {  // diagnostic timing path (variant bit 9): keep the MFMA results live, store nothing
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  asm volatile("" ::: "memory");  // the epilogue's LDS slot writes stay behind that barrier
  const int mw = m0 + wr * TM, nw = n0 + wc * TN;
  const int key = a.epi;
  const int outm = a.out_dtype == AACLIP_F32 ? 0 : (a.out_dtype == AACLIP_BF16 ? 1 : 2);
  // quad-coalesced epilogue through the same per-wave LDS slot as the bf16 8-phase
  // kernel (A1 / B1 of the last K-step's stage: no DMA lands there after their last reads)
  char* eslot = smem + ((nk - 1) & 1) * STAGE + (wr ? 3 : 1) * REGION + wc * 4096;
#define EPI_CASE(OM, E)                                                         \
  if (outm == (OM) && key == (E)) {                                             \
    wave_epilogue_lds<RM, RN, OM, E, false, 2>(a, acc, mw, nw, lane, nullptr, eslot); \
    return;                                                                     \
  }
  EPI_CASE(1, AACLIP_EPI_BIAS)                                          // qkv
  EPI_CASE(0, AACLIP_EPI_BIAS | AACLIP_EPI_RESID)                       // out-proj, c_proj
  EPI_CASE(0, AACLIP_EPI_BIAS | AACLIP_EPI_RESID | AACLIP_EPI_AUX_BF16)  // c_proj + bf16 copy
  EPI_CASE(2, AACLIP_EPI_BIAS | AACLIP_EPI_GELU)                        // c_fc -> fp8 MX
  EPI_CASE(2, AACLIP_EPI_BIAS | AACLIP_EPI_QGELU)
#undef EPI_CASE
  if (outm == 1)
    wave_epilogue<RM, RN, 1, -1, 2>(a, acc, mw, nw, lane);
  else if (outm == 0)
    wave_epilogue<RM, RN, 0, -1, 2>(a, acc, mw, nw, lane);
}

int launch_fp8mx_8ph(GemmArgs a, hipStream_t s) {
  a.tiles_m = ceil_div(a.M, 256);
  a.tiles_n = a.N / 256;
  const size_t lds = 2 * 4 * 128 * 128 + 3 * 512 + 6 * 256;
  static unsigned attr_dev = 0;
  if (!lds_attr_once((const void*)gemm_fp8mx_8ph_kernel, (int)lds, attr_dev)) return AACLIP_ERR_LAUNCH;
  gemm_fp8mx_8ph_kernel<<<a.tiles_m * a.tiles_n, 512, lds, s>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

int cu_count();

// workgroups of a launch: one per tile, or 8 x ksplit x ceil(tiles / 8) slots for a split
// launch (split_coords: each XCD's run of tiles, ksplit parts each; slots past a run idle)
unsigned grid_of(const GemmArgs& a) {
  const int64_t T = (int64_t)a.tiles_m * a.tiles_n;
  return (unsigned)(a.ksplit > 1 ? 8 * a.ksplit * ((T + 7) / 8) : T);
}

template <bool H16, bool SCORES = false, int KS = 0>
int launch_bf16_8ph_ks(GemmArgs a, hipStream_t s) {
  // the ring + the tile's bias (+ the phase stamps in the diagnostic build) + the split-K flag
  const size_t lds = kKsplitFlag + 16;
  static unsigned attr_dev = 0;
  if (!lds_attr_once((const void*)gemm_bf16_8ph_kernel<H16, SCORES, KS>, (int)lds, attr_dev))
    return AACLIP_ERR_LAUNCH;
  gemm_bf16_8ph_kernel<H16, SCORES, KS><<<grid_of(a), 512, lds, s>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

template <bool H16, bool SCORES = false>
int launch_bf16_8ph(GemmArgs a, hipStream_t s) {
  if (a.N % 256 || a.K % 64) return AACLIP_ERR_ARG;
  a.tiles_m = ceil_div(a.M, 256);
  a.tiles_n = a.N / 256;
  if constexpr (!SCORES) {
    if (a.ksplit == 2) return launch_bf16_8ph_ks<H16, false, 2>(a, s);
    if (a.ksplit == 3) return launch_bf16_8ph_ks<H16, false, 3>(a, s);
    if (a.ksplit == 4) return launch_bf16_8ph_ks<H16, false, 4>(a, s);
  }
  return launch_bf16_8ph_ks<H16, SCORES, 0>(a, s);
}

template <int BM, int BN, int WM, int WN, int Q, bool H16, int KS>
int launch_bf16_ks(GemmArgs a, hipStream_t s) {
  const size_t lds = 2 * (size_t)(BM + BN) * 128 + (Q == 2 ? 2 * BM * 2 : 0);
  static unsigned attr_dev = 0;
  if (!lds_attr_once((const void*)gemm_bf16_kernel<BM, BN, WM, WN, Q, H16, KS>, (int)lds, attr_dev))
    return AACLIP_ERR_LAUNCH;
  gemm_bf16_kernel<BM, BN, WM, WN, Q, H16, KS><<<grid_of(a), WM * WN * 64, lds, s>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

template <int BM, int BN, int WM, int WN, int Q = 0, bool H16 = false>
int launch_bf16(GemmArgs a, hipStream_t s) {
  if (a.N % BN) return AACLIP_ERR_ARG;
  a.tiles_m = ceil_div(a.M, BM);
  a.tiles_n = a.N / BN;
  if constexpr (Q == 0) {
    if (a.ksplit == 2) return launch_bf16_ks<BM, BN, WM, WN, Q, H16, 2>(a, s);
    if (a.ksplit == 3) return launch_bf16_ks<BM, BN, WM, WN, Q, H16, 3>(a, s);
    if (a.ksplit == 4) return launch_bf16_ks<BM, BN, WM, WN, Q, H16, 4>(a, s);
  }
  return launch_bf16_ks<BM, BN, WM, WN, Q, H16, 0>(a, s);
}


int g_gemm_variant = 0;  // tuning hook (aaclip_set_gemm_variant); 0 = default dispatch

int cu_count() {
  static int n[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 256;
  if (!n[dev] && hipDeviceGetAttribute(&n[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    n[dev] = 256;  // benign race: idempotent
  return n[dev] > 0 ? n[dev] : 256;
}

// Small M (a few images): when the big-tile choice would fill less than half of the
// CUs, 128x128 tiles (4 waves, 2 workgroups per CU) win -- measured 1.4-2x at 1-2
// images on every block GEMM, on out-proj / c_proj / adapters up to 8 images, and
// never worse within 10 % where the rule picks them (tools/kbench.py --batch 1..16).
bool prefer_small(int M, int N, bool ph8) {
  const int64_t tiles = (int64_t)ceil_div(M, ph8 ? 256 : 320) * (N / 256);
  return 2 * tiles < cu_count();
}

// Single images (M = 577): when even 128x128 tiles number fewer than half the CUs
// (batch-1 QKV 120, out-proj / c_proj / adapters 40), 64x64 tiles (4 waves of 32x32)
// give 4x the workgroups; same K order, same bits.
bool prefer_tiny(int M, int N) {
  return N % 64 == 0 && 2 * (int64_t)ceil_div(M, 128) * (N / 128) < cu_count();
}

// tile rounds x tile rows, 8-phase 256-row tiles weighted 10/11 for their faster main loop
bool prefer_8ph(int M, int N) {
  const int cus = cu_count();
  const int64_t t320 = (int64_t)ceil_div(M, 320) * (N / 256), t256 = (int64_t)ceil_div(M, 256) * (N / 256);
  const int64_t c320 = ((t320 + cus - 1) / cus) * 320 * 11, c256 = ((t256 + cus - 1) / cus) * 256 * 10;
  return c256 < c320;
}
// Tile-order group height: 4 M-tiles per group, so an XCD's 32 co-resident tiles are 4 M x 8 N
// -- each activation panel (streamed from HBM) feeds 8 tiles, each weight panel (shared by the
// concurrent chunks, MALL-resident) 4. Two-stream C2 step +0.3-0.5 % over 8 (8 M x 4 N) in
// 5 interleaved rounds (profiles/r03/gemm_group_height_ab.txt); 12 lost 1.2 %. Same bits.
int g_group_m = 4;
int g_setprio = 0;
int g_dbg = 0;

// Per-shape pinned tile family (aaclip_gemm_pin): a measured choice for one
// (dtype, M, N, K) that overrides the heuristic. Written by a tuner (host), read by
// every launch; guarded by a mutex (two engines may launch from two threads --
// ctypes releases the GIL). Unpinning removes the entry, so the table holds only
// live pins and cannot fill up with dead ones.
struct Pin {
  int dtype, M, N, K, fam;
};
constexpr int kPins = 256;
Pin g_pins[kPins];
std::atomic<int> g_npins{0};
std::mutex g_pin_mu;

int pinned_family(int dtype, int M, int N, int K) {
  if (g_npins.load(std::memory_order_acquire) == 0) return 0;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  const int n = g_npins.load(std::memory_order_relaxed);
  for (int i = 0; i < n; ++i)
    if (g_pins[i].dtype == dtype && g_pins[i].M == M && g_pins[i].N == N && g_pins[i].K == K) return g_pins[i].fam;
  return 0;
}

// Concurrent-chunk mode (aaclip_gemm_concurrent), per HOST THREAD: while a thread
// enqueues image chunks on concurrent streams, every block-GEMM shape whose 256x256
// tiles fill at least one round of the CUs takes the 8-phase kernel. The other
// chunk's work fills the partial last round, and the 8-phase tile is faster per
// FLOP (two-stream C2 step 2240 -> 2295 images/s bf16). The choice is made at
// launch (captured graphs keep it); thread-local, so it needs no global pin state.
thread_local int t_concurrent = 0;

enum Kern { KERN_256x256 = 1, KERN_256x128 = 2, KERN_8PH = 3, KERN_320x256 = 8, KERN_128x128 = 9, KERN_64x64 = 11 };

// The kernel a 16-bit GEMM of this shape launches: the A/B variant hook, else a pin,
// else the concurrent-chunk rule, else the per-shape heuristic (fewer tile rounds
// over the CUs, weighted by per-tile cost). M = B*577 tiles unevenly: 320-row tiles
// of the LDS-DMA kernel vs 256-row tiles of the 8-phase kernel (~10 % faster per
// FLOP). E.g. at 16 images per stream (M = 9232) the 8-phase kernel wins on QKV,
// out-proj, c_proj and adapters (148-444 tiles) and the 320-row one on c_fc (464 vs
// 592 tiles = 2 vs 3 rounds); measured per shape with tools/kbench.py.
int choose16(int dtype, int M, int N, int K, bool fits) {
  int fam = g_gemm_variant ? g_gemm_variant : pinned_family(dtype, M, N, K);
  if (!fam && t_concurrent && N % 256 == 0 && fits && (int64_t)ceil_div(M, 256) * (N / 256) >= cu_count())
    fam = KERN_8PH;
  switch (fam) {
    case 1: return KERN_256x256;
    case 2: return KERN_256x128;
    case 3:
    case 4:  // 8-phase for the wide GEMMs only (N >= 2048), 320x256 below
      if (N % 256 == 0 && (fam == 3 || N >= 2048) && fits) return KERN_8PH;
      break;
    case 9: return KERN_128x128;  // 128x128 everywhere (A/B)
    case 11:  // 64x64 everywhere (A/B)
      if (N % 64 == 0) return KERN_64x64;
      break;
    case 8:  // A/B: the 320x256 LDS-DMA kernel wherever N % 256 == 0 (the pre-heuristic default)
      if (N % 256 == 0) return KERN_320x256;
      break;
    default: break;
  }
  if (N % 256 == 0 && fam == 0) {
    const bool ph8 = fits && prefer_8ph(M, N);
    if (prefer_small(M, N, ph8)) return prefer_tiny(M, N) ? KERN_64x64 : KERN_128x128;
    if (ph8) return KERN_8PH;
  }
  return N % 256 == 0 ? KERN_320x256 : KERN_256x128;
}

// 16-bit dispatch (bf16 or fp16 operands; same tiles, same per-shape choice)
template <bool H16>
int dispatch16(GemmArgs a, hipStream_t s) {
  const int M = a.M, N = a.N;
  if (a.K % 64 || N % 128) return AACLIP_ERR_ARG;
  const bool fits = (int64_t)M * a.lda * 2 < (1ll << 31) && (int64_t)N * a.ldw * 2 < (1ll << 31);
  switch (choose16(H16 ? AACLIP_F16 : AACLIP_BF16, M, N, a.K, fits)) {
    case KERN_256x256: return launch_bf16<256, 256, 2, 4, 0, H16>(a, s);
    case KERN_8PH: return launch_bf16_8ph<H16>(a, s);
    case KERN_320x256: return launch_bf16<320, 256, 2, 4, 0, H16>(a, s);
    case KERN_128x128: return launch_bf16<128, 128, 2, 2, 0, H16>(a, s);
    case KERN_64x64: return launch_bf16<64, 64, 2, 2, 0, H16>(a, s);
    default: return launch_bf16<256, 128, 4, 2, 0, H16>(a, s);
  }
}

}  // namespace

// Which kernel aaclip_gemm launches for this shape (same decision as the dispatch,
// for operands with lda = ldw = K, on the calling thread). Host only, for reports.
extern "C" const char* aaclip_gemm_plan(int in_dtype, int M, int N, int K) {
  if (in_dtype != AACLIP_BF16 && in_dtype != AACLIP_F16) return "gemm_f32_kernel";
  if (M <= 0 || N % 128 || K % 64) return "invalid";
  const bool fits = (int64_t)M * K * 2 < (1ll << 31) && (int64_t)N * K * 2 < (1ll << 31);
  switch (choose16(in_dtype, M, N, K, fits)) {
    case KERN_256x256: return "gemm_bf16_kernel<256,256,2,4>";
    case KERN_8PH: return "gemm_bf16_8ph_kernel<256,256>";
    case KERN_320x256: return "gemm_bf16_kernel<320,256,2,4>";
    case KERN_128x128: return "gemm_bf16_kernel<128,128,2,2>";
    case KERN_64x64: return "gemm_bf16_kernel<64,64,2,2>";
    default: return "gemm_bf16_kernel<256,128,4,2>";
  }
}

extern "C" int aaclip_gemm_pin(int in_dtype, int M, int N, int K, int family) {
  AACLIP_REQUIRE((in_dtype == AACLIP_BF16 || in_dtype == AACLIP_F16) && M > 0 && N > 0 && K > 0);
  AACLIP_REQUIRE(family == 0 || family == 1 || family == 2 || family == 3 || family == 8 || family == 9 ||
                 family == 11);
  AACLIP_REQUIRE(family == 0 || family == 2 || family == 11 || N % 256 == 0);
  std::lock_guard<std::mutex> lk(g_pin_mu);
  const int n = g_npins.load(std::memory_order_relaxed);
  for (int i = 0; i < n; ++i)
    if (g_pins[i].dtype == in_dtype && g_pins[i].M == M && g_pins[i].N == N && g_pins[i].K == K) {
      if (family) {
        g_pins[i].fam = family;
      } else {  // unpin: move the last entry into the hole
        g_pins[i] = g_pins[n - 1];
        g_npins.store(n - 1, std::memory_order_release);
      }
      return AACLIP_OK;
    }
  if (family == 0) return AACLIP_OK;
  AACLIP_REQUIRE(n < kPins);
  g_pins[n] = Pin{in_dtype, M, N, K, family};
  g_npins.store(n + 1, std::memory_order_release);
  return AACLIP_OK;
}

extern "C" int aaclip_gemm_concurrent(int on, int* previous) {
  AACLIP_REQUIRE(on == 0 || on == 1);
  if (previous) *previous = t_concurrent;
  t_concurrent = on;
  return AACLIP_OK;
}

extern "C" int aaclip_set_gemm_variant(int variant) {
  // bits 0-3: tile family (0 default = per-shape choice, 1 = 256x256, 2 = 256x128, 3/4 = 256x256
  // 8-phase ping-pong everywhere / for N >= 2048, 6 = MX fp8 on the 256x256 LDS-DMA kernel
  // instead of its 8-phase default, 8 = 320x256 everywhere, 9 = 128x128, 11 = 64x64; the
  // persistent 8-phase family 5 and the two-workgroup family 10 measured slower and were
  // removed in round 5); bits 4-7: tile-order
  // group height (0 = 4); bit 8: setprio around the MFMA cluster; bits 9-11: diagnostics
  const int fam = variant & 15, grp = (variant >> 4) & 15;
  if (variant < 0 || variant >= 4096 || fam > 11 || fam == 5 || fam == 7 || fam == 10) return AACLIP_ERR_ARG;
  g_gemm_variant = fam;
  g_group_m = grp ? grp : 4;
  g_setprio = (variant >> 8) & 1;
  // bit 9 skip epilogue, bit 10 skip the global stores, bit 11 the 8-phase kernel's
  // per-wave s_memtime stamps into the aux pointer (bf16 / fp32 epilogues without aux only)
  g_dbg = (variant >> 9) & 7;
  return AACLIP_OK;
}

extern "C" int aaclip_gemm(int in_dtype, int out_dtype, int M, int N, int K, const void* A,
                           int64_t lda, const void* W, int64_t ldw, void* C, int64_t ldc,
                           int epilogue, const float* bias, const float* residual, int64_t ldr,
                           void* aux, int64_t ldaux, int row_group, int row_group_out,
                           int row_offset, void* stream) {
  AACLIP_REQUIRE(in_dtype == AACLIP_F32 || in_dtype == AACLIP_BF16 || in_dtype == AACLIP_F16);
  AACLIP_REQUIRE(out_dtype == AACLIP_F32 || (in_dtype != AACLIP_F32 && out_dtype == in_dtype) ||
                 (in_dtype == AACLIP_F32 && out_dtype == AACLIP_BF16));
  AACLIP_REQUIRE(A && W && C && M >= 0 && N > 0 && K > 0);
  AACLIP_REQUIRE(lda >= K && ldw >= K && ldc >= N && lda % 8 == 0 && ldw % 8 == 0 && ldc % 4 == 0);
  AACLIP_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0 && ((uintptr_t)C % 16) == 0);
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_BIAS) || bias);
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_BIAS) || ((uintptr_t)bias % 16) == 0);
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_RESID) || (residual && ldr >= N && ldr % 4 == 0));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_AUX_BF16) || (aux && ldaux >= N && ldaux % 4 == 0));
  AACLIP_REQUIRE((epilogue & ~63) == 0 && (epilogue & (AACLIP_EPI_GELU | AACLIP_EPI_QGELU)) !=
                                               (AACLIP_EPI_GELU | AACLIP_EPI_QGELU));
  AACLIP_REQUIRE(row_group >= 0 && (row_group == 0 || row_group_out >= row_group));
  if (M == 0) return AACLIP_OK;
  GemmArgs a{A, W, C, bias, residual, aux, lda, ldw, ldc, ldr, ldaux, M, N, K, epilogue,
             out_dtype, row_group, row_group_out, row_offset, 0, 0, g_group_m, g_setprio, g_dbg,
             nullptr, nullptr, nullptr, 0, nullptr, 0};
  hipStream_t s = (hipStream_t)stream;
  if (in_dtype == AACLIP_BF16) return dispatch16<false>(a, s);
  if (in_dtype == AACLIP_F16) return dispatch16<true>(a, s);
  AACLIP_REQUIRE(K % 16 == 0 && N % 64 == 0);
  a.tiles_m = ceil_div(M, 64);
  a.tiles_n = N / 64;
  gemm_f32_kernel<<<a.tiles_m * a.tiles_n, 256, 0, s>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

// Split-K workspace bound over every tile family the dispatch may pick for (M, N): S fp32
// partial tiles per output tile (<= S (M + 319) N floats: 320-row tiles pad M the most) and
// one arrival counter per tile (most tiles: 64x64).
extern "C" int aaclip_gemm_ksplit_workspace(int M, int N, int K, int ksplit, size_t* part_bytes,
                                            int64_t* counters) {
  AACLIP_REQUIRE(M > 0 && N > 0 && K > 0 && K % 64 == 0 && N % 64 == 0 && ksplit >= 2 && ksplit <= 4 &&
                 ksplit <= K / 64 && part_bytes && counters);
  *part_bytes = (size_t)ksplit * ((size_t)M + 319) * (size_t)N * 4;
  *counters = (int64_t)ceil_div(M, 64) * (N / 64);
  return AACLIP_OK;
}

extern "C" int aaclip_gemm_ksplit(int in_dtype, int out_dtype, int M, int N, int K, const void* A, int64_t lda,
                                  const void* W, int64_t ldw, void* C, int64_t ldc, int epilogue, const float* bias,
                                  const float* residual, int64_t ldr, void* aux, int64_t ldaux, int ksplit,
                                  void* part, size_t part_bytes, void* counters, int64_t n_counters, void* stream) {
  AACLIP_REQUIRE(in_dtype == AACLIP_BF16 || in_dtype == AACLIP_F16);
  AACLIP_REQUIRE(out_dtype == AACLIP_F32 || out_dtype == in_dtype);
  AACLIP_REQUIRE(A && W && C && M >= 0 && N > 0 && K > 0 && K % 64 == 0);
  AACLIP_REQUIRE(lda >= K && ldw >= K && ldc >= N && lda % 8 == 0 && ldw % 8 == 0 && ldc % 4 == 0);
  AACLIP_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0 && ((uintptr_t)C % 16) == 0);
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_BIAS) || (bias && ((uintptr_t)bias % 16) == 0));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_RESID) || (residual && ldr >= N && ldr % 4 == 0));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_AUX_BF16) || (aux && ldaux >= N && ldaux % 4 == 0));
  AACLIP_REQUIRE((epilogue & ~63) == 0 && (epilogue & (AACLIP_EPI_GELU | AACLIP_EPI_QGELU)) !=
                                               (AACLIP_EPI_GELU | AACLIP_EPI_QGELU));
  AACLIP_REQUIRE(ksplit >= 2 && ksplit <= 4 && ksplit <= K / 64);
  AACLIP_REQUIRE(part && counters && ((uintptr_t)part % 16) == 0 && ((uintptr_t)counters % 4) == 0);
  if (M == 0) return AACLIP_OK;
  size_t need_bytes = 0;
  int64_t need_counters = 0;
  if (aaclip_gemm_ksplit_workspace(M, N, K, ksplit, &need_bytes, &need_counters) != AACLIP_OK)
    return AACLIP_ERR_ARG;
  AACLIP_REQUIRE(part_bytes >= need_bytes && n_counters >= need_counters);
  GemmArgs a{A, W, C, bias, residual, aux, lda, ldw, ldc, ldr, ldaux, M, N, K, epilogue,
             out_dtype, 0, 0, 0, 0, 0, g_group_m, g_setprio, g_dbg & 2,
             nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr, 0, ksplit, (float*)part, (unsigned*)counters};
  hipStream_t s = (hipStream_t)stream;
  if (in_dtype == AACLIP_BF16) return dispatch16<false>(a, s);
  return dispatch16<true>(a, s);
}

extern "C" int aaclip_gemm_scores(int in_dtype, int M, int N, int K, const void* A, int64_t lda, const void* W,
                                  int64_t ldw, int epilogue, const float* T, int t_period, float* part,
                                  int64_t ld_part, void* stream) {
  AACLIP_REQUIRE(in_dtype == AACLIP_BF16 || in_dtype == AACLIP_F16);
  AACLIP_REQUIRE(A && W && T && part && M >= 0 && N > 0 && K > 0 && K % 64 == 0 && N % 256 == 0);
  AACLIP_REQUIRE(t_period > 0 && t_period % 64 == 0 && ld_part >= N / 8 && ld_part % 4 == 0);
  AACLIP_REQUIRE(lda >= K && ldw >= K && lda % 8 == 0 && ldw % 8 == 0);
  AACLIP_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0 && ((uintptr_t)part % 16) == 0 &&
                 ((uintptr_t)T % 16) == 0);
  AACLIP_REQUIRE(epilogue == 0 || epilogue == AACLIP_EPI_LEAKY);
  if (M == 0) return AACLIP_OK;
  GemmArgs a{A, W, part, nullptr, nullptr, nullptr, lda, ldw, ld_part, 0, 0, M, N, K, epilogue,
             kOutScores, 0, 0, 0, 0, 0, g_group_m, g_setprio, g_dbg & 1,
             nullptr, nullptr, nullptr, 0, nullptr, 0, T, t_period};
  hipStream_t s = (hipStream_t)stream;
  const bool h16 = in_dtype == AACLIP_F16;
  const bool fits = (int64_t)M * lda * 2 < (1ll << 31) && (int64_t)N * ldw * 2 < (1ll << 31);
  // the same per-shape choice as aaclip_gemm (same K order, same bits)
  switch (choose16(in_dtype, M, N, K, fits)) {
    case KERN_256x256:
      return h16 ? launch_bf16<256, 256, 2, 4, 0, true>(a, s) : launch_bf16<256, 256, 2, 4, 0, false>(a, s);
    case KERN_320x256:
      return h16 ? launch_bf16<320, 256, 2, 4, 0, true>(a, s) : launch_bf16<320, 256, 2, 4, 0, false>(a, s);
    case KERN_128x128:
      return h16 ? launch_bf16<128, 128, 2, 2, 0, true>(a, s) : launch_bf16<128, 128, 2, 2, 0, false>(a, s);
    case KERN_64x64:
      return h16 ? launch_bf16<64, 64, 2, 2, 0, true>(a, s) : launch_bf16<64, 64, 2, 2, 0, false>(a, s);
    case KERN_256x128:
      return h16 ? launch_bf16<256, 128, 4, 2, 0, true>(a, s) : launch_bf16<256, 128, 4, 2, 0, false>(a, s);
    default:
      if (!fits) return h16 ? launch_bf16<320, 256, 2, 4, 0, true>(a, s) : launch_bf16<320, 256, 2, 4, 0, false>(a, s);
      return h16 ? launch_bf16_8ph<true, true>(a, s) : launch_bf16_8ph<false, true>(a, s);
  }
}

extern "C" int aaclip_gemm_fp8(int out_dtype, int M, int N, int K, const void* A, int64_t lda,
                               const float* a_scale, const void* W, int64_t ldw, const float* w_scale,
                               void* C, int64_t ldc, int epilogue, const float* bias, const float* residual,
                               int64_t ldr, void* aux, int64_t ldaux, int row_group, int row_group_out,
                               int row_offset, void* stream) {
  AACLIP_REQUIRE(out_dtype == AACLIP_F32 || out_dtype == AACLIP_BF16);
  AACLIP_REQUIRE(A && W && C && a_scale && w_scale && M >= 0 && N > 0 && K > 0);
  AACLIP_REQUIRE(K % 128 == 0 && N % 128 == 0);
  AACLIP_REQUIRE(lda >= K && ldw >= K && ldc >= N && lda % 16 == 0 && ldw % 16 == 0 && ldc % 4 == 0);
  AACLIP_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0 && ((uintptr_t)C % 16) == 0);
  AACLIP_REQUIRE(((uintptr_t)w_scale % 16) == 0);
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_BIAS) || (bias && ((uintptr_t)bias % 16) == 0));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_RESID) || (residual && ldr >= N && ldr % 4 == 0));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_AUX_BF16) || (aux && ldaux >= N && ldaux % 4 == 0));
  AACLIP_REQUIRE((epilogue & ~63) == 0 && (epilogue & (AACLIP_EPI_GELU | AACLIP_EPI_QGELU)) !=
                                               (AACLIP_EPI_GELU | AACLIP_EPI_QGELU));
  AACLIP_REQUIRE(row_group >= 0 && (row_group == 0 || row_group_out >= row_group));
  if (M == 0) return AACLIP_OK;
  GemmArgs a{A, W, C, bias, residual, aux, lda, ldw, ldc, ldr, ldaux, M, N, K, epilogue,
             out_dtype, row_group, row_group_out, row_offset, 0, 0, g_group_m, g_setprio, 0,
             a_scale, w_scale, nullptr, 0, nullptr, 0};
  hipStream_t s = (hipStream_t)stream;
  if (N % 256 == 0) return launch_bf16<256, 256, 2, 4, 1>(a, s);  // 320x256 spills with 8-VGPR fp8 fragments
  return launch_bf16<256, 128, 4, 2, 1>(a, s);
}

extern "C" int aaclip_gemm_fp8mx(int out_dtype, int M, int N, int K, const void* A, int64_t lda, const void* a_mx,
                                 int64_t ld_amx, const void* W, int64_t ldw, const float* w_scale, void* C,
                                 int64_t ldc, int epilogue, const float* bias, const float* residual, int64_t ldr,
                                 void* aux, int64_t ldaux, void* c_mx, int64_t ld_cmx, void* stream) {
  AACLIP_REQUIRE(out_dtype == AACLIP_F32 || out_dtype == AACLIP_BF16 || out_dtype == AACLIP_FP8);
  AACLIP_REQUIRE(A && W && C && a_mx && w_scale && M >= 0 && N > 0 && K > 0);
  // ld_amx even: the scale DMA moves dwords, and with an odd ld the K-step bases sit at
  // 2 mod 4 bytes, so the last row's dword in the last K-step straddles the buffer
  // end and the range check drops it (scale 0 -> that row wrong; found by the
  // batch-composition invariance test at odd image counts)
  AACLIP_REQUIRE(K % 128 == 0 && N % 256 == 0 && ld_amx >= M && ld_amx % 2 == 0);
  AACLIP_REQUIRE(lda >= K && ldw >= K && ldc >= N && lda % 16 == 0 && ldw % 16 == 0 && ldc % 16 == 0);
  AACLIP_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0 && ((uintptr_t)C % 16) == 0);
  AACLIP_REQUIRE(((uintptr_t)w_scale % 16) == 0 && ((uintptr_t)a_mx % 4) == 0);
  AACLIP_REQUIRE((int64_t)(K / 128) * ld_amx * 2 < (1ll << 31) && (int64_t)M * lda < (1ll << 31));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_BIAS) || (bias && ((uintptr_t)bias % 16) == 0));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_RESID) || (residual && ldr >= N && ldr % 4 == 0));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_AUX_BF16) || (aux && ldaux >= N && ldaux % 4 == 0));
  AACLIP_REQUIRE((epilogue & ~63) == 0 && (epilogue & (AACLIP_EPI_GELU | AACLIP_EPI_QGELU)) !=
                                               (AACLIP_EPI_GELU | AACLIP_EPI_QGELU));
  AACLIP_REQUIRE(out_dtype != AACLIP_FP8 || (c_mx && ld_cmx >= M && (epilogue == (AACLIP_EPI_BIAS | AACLIP_EPI_GELU) ||
                                                         epilogue == (AACLIP_EPI_BIAS | AACLIP_EPI_QGELU))));
  if (M == 0) return AACLIP_OK;
  GemmArgs a{A, W, C, bias, residual, aux, lda, ldw, ldc, ldr, ldaux, M, N, K, epilogue,
             out_dtype, 0, 0, 0, 0, 0, g_group_m, g_setprio, g_dbg,
             nullptr, w_scale, (const uint8_t*)a_mx, ld_amx, (uint8_t*)c_mx, ld_cmx};
  // 8-phase ping-pong by default (C5 at B=32: qkv/fc/out +6-8%, c_proj +28% vs the
  // 256x256 LDS-DMA kernel; whole C5 step 1400 -> 1511 img/s); variant 6 = A/B hook
  if (g_gemm_variant == 6) return launch_bf16<256, 256, 2, 4, 2>(a, (hipStream_t)stream);
  return launch_fp8mx_8ph(a, (hipStream_t)stream);
}

AACLIP_TRACE_SETTER(trace_set_gemm)
