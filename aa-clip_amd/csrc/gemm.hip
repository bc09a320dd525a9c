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
};

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

// Epilogue on one element C[m, n] (m < M checked by the caller).
__device__ __forceinline__ void epilogue_store1(const GemmArgs& a, int m, int n, float v) {
  const int orow = remap_row(a, m);
  if (a.epi & AACLIP_EPI_BIAS) v += a.bias[n];
  if (a.epi & AACLIP_EPI_GELU) v = gelu_erf(v);
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
                                            int GROUP_M = 8) {
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

// Epilogue of one wave's (16*RM) x 64 output tile, staged through a wave-private
// LDS slot ep[16][EP_LD] one 16-row block at a time (accumulator layout: lane
// holds C[16i + 4*fq + e][16j + fr]; re-read row-major so every lane owns CPL
// consecutive columns and issues 16-B stores: 8 bf16 or 4 fp32).
// Latency, not bandwidth, bounds this phase (all waves of the chip reach it
// together), and vmcnt retires in issue order, so a load issued after a store
// cannot be waited on without also waiting for that store. Hence: the bias is
// loaded once per tile before any store, and the residual rows of block i+1 are
// loaded before block i's stores are issued (one block of prefetch).
constexpr int EP_LD = 64 + 4;  // floats per staged row (pad: conflict-free writes)

// EPI >= 0: compile-time epilogue flags (AACLIP_EPI_* | EPI_REMAP) so each used
// combination is straight-line code; EPI = -1: flags read at run time (any combination).
constexpr int EPI_REMAP = 64;

template <int RM, int RN, bool BF16OUT, int EPI>
__device__ __forceinline__ void wave_epilogue(const GemmArgs& a, float4_t (&acc)[RM][RN], float* ep,
                                              int mw, int nw, int lane) {
  static_assert(RN == 4, "wave tile is 64 columns wide");
  constexpr int CPL = BF16OUT ? 8 : 4;  // consecutive columns per lane
  constexpr int LPR = 64 / CPL;         // lanes per staged row
  constexpr int RPP = 64 / LPR;         // rows per pass
  constexpr int NP = 16 / RPP;          // passes per 16-row block
  constexpr int NV = CPL / 4;           // float4 per lane per pass
  const int fr = lane & 15, fq = lane >> 4;
  const int col = (lane % LPR) * CPL, rsub = lane / LPR;
  const int n = nw + col;
  const int epi = EPI >= 0 ? EPI : a.epi | (a.row_group > 0 ? EPI_REMAP : 0);
  const bool full = mw + 16 * RM <= a.M;
  auto out_row = [&](int m) { return (epi & EPI_REMAP) ? remap_row(a, m) : m; };
  float4_t bias[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v)
    bias[v] = (epi & AACLIP_EPI_BIAS) ? *(const float4_t*)(a.bias + n + 4 * v) : float4_t{0.f, 0.f, 0.f, 0.f};
  float4_t res[2][NP][NV];
  auto load_res = [&](int i, float4_t (&dst)[NP][NV]) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int m = mw + i * 16 + p * RPP + rsub;
      const float* src = a.res + (size_t)out_row(min(m, a.M - 1)) * a.ldr + n;
#pragma unroll
      for (int v = 0; v < NV; ++v) dst[p][v] = *(const float4_t*)(src + 4 * v);
    }
  };
  if (epi & AACLIP_EPI_RESID) load_res(0, res[0]);
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) ep[(fq * 4 + e) * EP_LD + j * 16 + fr] = acc[i][j][e];
    if ((epi & AACLIP_EPI_RESID) && i + 1 < RM) load_res(i + 1, res[(i + 1) & 1]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int r = p * RPP + rsub;
      const int m = mw + i * 16 + r;
      float4_t v[NV];
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        v[q] = *(const float4_t*)(ep + r * EP_LD + col + 4 * q) + bias[q];
        if (epi & AACLIP_EPI_GELU)
#pragma unroll
          for (int t = 0; t < 4; ++t) v[q][t] = gelu_fast(v[q][t]);
        if (epi & AACLIP_EPI_LEAKY)
#pragma unroll
          for (int t = 0; t < 4; ++t) v[q][t] = v[q][t] >= 0.f ? v[q][t] : 0.01f * v[q][t];
        if (epi & AACLIP_EPI_RESID) v[q] += res[i & 1][p][q];
      }
      if (full || m < a.M) {
        const size_t orow = (size_t)out_row(m);
        if constexpr (BF16OUT) {
          *(uint4*)((uint16_t*)a.C + orow * a.ldc + n) =
              uint4{pack_bf16x2(v[0][0], v[0][1]), pack_bf16x2(v[0][2], v[0][3]),
                    pack_bf16x2(v[1][0], v[1][1]), pack_bf16x2(v[1][2], v[1][3])};
        } else {
#pragma unroll
          for (int q = 0; q < NV; ++q) *(float4_t*)((float*)a.C + orow * a.ldc + n + 4 * q) = v[q];
        }
        if (epi & AACLIP_EPI_AUX_BF16) {
#pragma unroll
          for (int q = 0; q < NV; ++q)
            *(uint2*)((uint16_t*)a.aux + orow * a.ldaux + n + 4 * q) =
                uint2{pack_bf16x2(v[q][0], v[q][1]), pack_bf16x2(v[q][2], v[q][3])};
        }
      }
    }
  }
}

// ============================================================== bf16 MFMA kernel
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void gemm_bf16_kernel(GemmArgs a) {
  constexpr int NWAVES = WM * WN;
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int RM = TM / 16, RN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_LOADS = A_BYTES / (NWAVES * 1024);  // glds per wave per tile
  constexpr int B_LOADS = B_BYTES / (NWAVES * 1024);
  static_assert(A_LOADS * NWAVES * 1024 == A_BYTES && B_LOADS * NWAVES * 1024 == B_BYTES, "tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  int tm, tn;
  tile_coords(blockIdx.x, a.tiles_m, a.tiles_n, tm, tn, a.group_m);
  const int m0 = tm * BM, n0 = tn * BN;

  const uint16_t* __restrict__ Ag = (const uint16_t*)a.A;
  const uint16_t* __restrict__ Wg = (const uint16_t*)a.W;

  // Per-lane source pointers for the DMA pieces (row r = piece*8 + lane/8,
  // physical chunk p = lane%8 holds logical chunk p ^ (r&7)).
  const uint16_t* a_src[A_LOADS];
  const uint16_t* b_src[B_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i) {
    const int r = (i * NWAVES + wid) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const int gr = min(m0 + r, a.M - 1);
    a_src[i] = Ag + (size_t)gr * a.lda + c * 8;
  }
#pragma unroll
  for (int i = 0; i < B_LOADS; ++i) {
    const int r = (i * NWAVES + wid) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    b_src[i] = Wg + (size_t)(n0 + r) * a.ldw + c * 8;
  }

#define GEMM_STAGE(kt, buf)                                                                  \
  do {                                                                                       \
    char* base_ = smem + (buf) * STAGE_BYTES;                                                \
    const int koff_ = (kt) * BK;                                                             \
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

  // fragment read offsets (bytes within a stage), kk = 0/1 half of BK
  const int fr = lane & 15, fq = lane >> 4;
  int a_off[RM][2], b_off[RN][2];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int r = wm * TM + i * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) a_off[i][kk] = r * 128 + (((kk * 4 + fq) ^ (r & 7)) << 4);
  }
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int r = wn * TN + j * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) b_off[j][kk] = A_BYTES + r * 128 + (((kk * 4 + fq) ^ (r & 7)) << 4);
  }

  const int nk = a.K / BK;
  GEMM_STAGE(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) GEMM_STAGE(kt + 1, cur ^ 1);
    const char* base = smem + cur * STAGE_BYTES;
    if (a.setprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t bf[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) bf[j] = *(const bf16x8_t*)(base + b_off[j][kk]);
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const bf16x8_t af = *(const bf16x8_t*)(base + a_off[i][kk]);
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[j], acc[i][j], 0, 0, 0);
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
  // The main loop's last barrier freed the LDS tiles: each wave stages through
  // its own slot, no workgroup barrier needed.
  float* ep = (float*)smem + wid * 16 * EP_LD;
  const int mw = m0 + wm * TM, nw = n0 + wn * TN;
  const int key = a.epi | (a.row_group > 0 ? EPI_REMAP : 0);
#define EPI_CASE(BF, E)                                                \
  if (bf16_out == (BF) && key == (E)) {                                \
    wave_epilogue<RM, RN, BF, E>(a, acc, ep, mw, nw, lane);            \
    return;                                                            \
  }
  // the combinations the visual/text engines issue (engine.py)
  const bool bf16_out = a.out_dtype != AACLIP_F32;
  EPI_CASE(true, AACLIP_EPI_BIAS)                                        // qkv
  EPI_CASE(true, AACLIP_EPI_BIAS | AACLIP_EPI_GELU)                      // c_fc
  EPI_CASE(false, AACLIP_EPI_BIAS | AACLIP_EPI_RESID)                    // out-proj, c_proj
  EPI_CASE(false, AACLIP_EPI_BIAS | AACLIP_EPI_RESID | AACLIP_EPI_AUX_BF16)  // c_proj + bf16 copy
  EPI_CASE(false, AACLIP_EPI_LEAKY)                                      // adapters, seg/det proj
  EPI_CASE(false, 0)                                                     // seg/det proj (no relu)
  EPI_CASE(false, EPI_REMAP)                                             // patch embedding
#undef EPI_CASE
  if (bf16_out)
    wave_epilogue<RM, RN, true, -1>(a, acc, ep, mw, nw, lane);
  else
    wave_epilogue<RM, RN, false, -1>(a, acc, ep, mw, nw, lane);
}

// ============================================================== fp32 MFMA kernel
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs a) {
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

template <int BM, int BN, int WM, int WN>
int launch_bf16(GemmArgs a, hipStream_t s) {
  if (a.N % BN) return AACLIP_ERR_ARG;
  a.tiles_m = ceil_div(a.M, BM);
  a.tiles_n = a.N / BN;
  const size_t lds = 2 * (size_t)(BM + BN) * 64 * 2;
  static bool attr_set = false;  // benign race: idempotent attribute write
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)gemm_bf16_kernel<BM, BN, WM, WN>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return AACLIP_ERR_LAUNCH;
    attr_set = true;
  }
  gemm_bf16_kernel<BM, BN, WM, WN><<<a.tiles_m * a.tiles_n, WM * WN * 64, lds, s>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}


int g_gemm_variant = 0;  // tuning hook (aaclip_set_gemm_variant); 0 = default dispatch
int g_group_m = 8;
int g_setprio = 0;
int g_dbg = 0;

}  // namespace

extern "C" int aaclip_set_gemm_variant(int variant) {
  // bits 0-3: tile family (0 default, 1 = 256x256, 2 = 256x128); bits 4-7: tile-order
  // group height (0 = 8); bit 8: setprio around the MFMA cluster; bit 9: skip epilogue
  const int fam = variant & 15, grp = (variant >> 4) & 15;
  if (variant < 0 || variant >= 1024 || fam > 2) return AACLIP_ERR_ARG;
  g_gemm_variant = fam;
  g_group_m = grp ? grp : 8;
  g_setprio = (variant >> 8) & 1;
  g_dbg = (variant >> 9) & 1;
  return AACLIP_OK;
}

extern "C" int aaclip_gemm(int in_dtype, int out_dtype, int M, int N, int K, const void* A,
                           int64_t lda, const void* W, int64_t ldw, void* C, int64_t ldc,
                           int epilogue, const float* bias, const float* residual, int64_t ldr,
                           void* aux, int64_t ldaux, int row_group, int row_group_out,
                           int row_offset, void* stream) {
  AACLIP_REQUIRE(in_dtype == AACLIP_F32 || in_dtype == AACLIP_BF16);
  AACLIP_REQUIRE(out_dtype == AACLIP_F32 || out_dtype == AACLIP_BF16);
  AACLIP_REQUIRE(A && W && C && M >= 0 && N > 0 && K > 0);
  AACLIP_REQUIRE(lda >= K && ldw >= K && ldc >= N && lda % 8 == 0 && ldw % 8 == 0 && ldc % 4 == 0);
  AACLIP_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0 && ((uintptr_t)C % 16) == 0);
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_BIAS) || bias);
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_BIAS) || ((uintptr_t)bias % 16) == 0);
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_RESID) || (residual && ldr >= N && ldr % 4 == 0));
  AACLIP_REQUIRE(!(epilogue & AACLIP_EPI_AUX_BF16) || (aux && ldaux >= N && ldaux % 4 == 0));
  AACLIP_REQUIRE(row_group >= 0 && (row_group == 0 || row_group_out >= row_group));
  if (M == 0) return AACLIP_OK;
  GemmArgs a{A, W, C, bias, residual, aux, lda, ldw, ldc, ldr, ldaux, M, N, K, epilogue,
             out_dtype, row_group, row_group_out, row_offset, 0, 0, g_group_m, g_setprio, g_dbg};
  hipStream_t s = (hipStream_t)stream;
  if (in_dtype == AACLIP_BF16) {
    AACLIP_REQUIRE(K % 64 == 0 && N % 128 == 0);
    switch (g_gemm_variant) {
      case 1: return launch_bf16<256, 256, 2, 4>(a, s);
      case 2: return launch_bf16<256, 128, 4, 2>(a, s);
      default: break;
    }
    // M = B*577 tiles badly by 256 (18464 = 72.1 x 256 at B=32: 3.42 waves of 256x256
    // tiles for N=3072, 1.14 for N=1024); 320-row tiles give 58 M-tiles -> 0.91 / 2.72 /
    // 3.63 waves for N = 1024 / 3072 / 4096 (measured 1.1-1.4x faster on every block GEMM).
    if (N % 256 == 0) return launch_bf16<320, 256, 2, 4>(a, s);
    return launch_bf16<256, 128, 4, 2>(a, s);
  }
  AACLIP_REQUIRE(K % 16 == 0 && N % 64 == 0);
  a.tiles_m = ceil_div(M, 64);
  a.tiles_n = N / 64;
  gemm_f32_kernel<<<a.tiles_m * a.tiles_n, 256, 0, s>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}
