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

// GELU for the bf16 path: 1 + erf(z) through erfc(|z|) from Abramowitz-Stegun
// 7.1.26 (|error| <= 1.5e-7, far below bf16's 2^-9 output rounding): one rcp,
// one exp and a degree-5 polynomial instead of OCML's branchy erff, which
// dominated the c_fc epilogue. For z < 0 the erfc form keeps GELU's small
// negative tail accurate (no 1 - (1 - e) cancellation).
__device__ __forceinline__ float gelu_fast(float v) {
  const float z = v * 0.70710678118654752440f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float erfc_az = t * p * __expf(-az * az);
  return 0.5f * v * (z >= 0.f ? 2.0f - erfc_az : erfc_az);
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

// Epilogue on 4 consecutive columns C[m, n..n+3] (n % 4 == 0).
__device__ __forceinline__ void epilogue_store4(const GemmArgs& a, int m, int n, float4_t v) {
  const int orow = remap_row(a, m);
  if (a.epi & AACLIP_EPI_BIAS) v += *(const float4_t*)(a.bias + n);
  if (a.epi & AACLIP_EPI_GELU)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gelu_fast(v[j]);
  if (a.epi & AACLIP_EPI_LEAKY)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = v[j] >= 0.f ? v[j] : 0.01f * v[j];
  if (a.epi & AACLIP_EPI_RESID) v += *(const float4_t*)(a.res + (size_t)orow * a.ldr + n);
  if (a.out_dtype == AACLIP_F32) {
    *(float4_t*)((float*)a.C + (size_t)orow * a.ldc + n) = v;
  } else {
    *(uint2*)((uint16_t*)a.C + (size_t)orow * a.ldc + n) =
        uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
  }
  if (a.epi & AACLIP_EPI_AUX_BF16)
    *(uint2*)((uint16_t*)a.aux + (size_t)orow * a.ldaux + n) =
        uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
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

  // ---- epilogue, staged through LDS one 16-row block at a time so that each lane
  // finishes 4 consecutive columns (16-B fp32 / 8-B bf16 stores, coalesced rows).
  // Accumulator layout: lane holds C[16i + 4*fq + e][16j + fr]. Each wave stages
  // through its own LDS slot (the main loop's last barrier freed the tiles), so
  // no workgroup barrier is needed: LDS ops of one wave execute in order, and the
  // asm memory fences keep the compiler from reordering the write/read phases.
  constexpr int EP_LD = TN + 4;  // floats per staged row (pad: conflict-free writes)
  float* ep = (float*)smem + wid * 16 * EP_LD;
  constexpr int F4_PER_ROW = TN / 4;
  if (a.dbg & 1) {  // diagnostic timing build path: keep the MFMA results live, store nothing
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) ep[(fq * 4 + e) * EP_LD + j * 16 + fr] = acc[i][j][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int f = lane; f < 16 * F4_PER_ROW; f += 64) {
      const int r = f / F4_PER_ROW, c4 = f % F4_PER_ROW;
      const int m = m0 + wm * TM + i * 16 + r;
      if (m < a.M) {
        const float4_t v = *(const float4_t*)(ep + r * EP_LD + c4 * 4);
        epilogue_store4(a, m, n0 + wn * TN + c4 * 4, v);
      }
    }
  }
}

// ============================================================== bf16 MFMA, persistent
// Same tile / main loop as gemm_bf16_kernel, but each workgroup loops over the
// tiles L = blockIdx.x, blockIdx.x + gridDim.x, ... (gridDim.x = #CUs; the
// linear id keeps the XCD-aware order of tile_coords). Tile seams are
// pipelined: during the last K-step of tile i the DMA of tile i+1's first
// K-stage is issued into the free buffer; tile i's epilogue stages through the
// buffer just consumed; tile i+1's first barrier waits with vmcnt(NSTORE), not 0.
// vmcnt retires in issue order and the prefetch is older than the epilogue's
// stores, so the wait guarantees the prefetch landed while up to NSTORE of the
// previous tile's output stores keep draining behind the next main loop.
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void gemm_bf16_persistent_kernel(GemmArgs a) {
  constexpr int NWAVES = WM * WN;
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int RM = TM / 16, RN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_LOADS = A_BYTES / (NWAVES * 1024);
  constexpr int B_LOADS = B_BYTES / (NWAVES * 1024);
  constexpr int EP_LD = TN + 4, F4_PER_ROW = TN / 4;
  constexpr int STORES_PER_WAVE = RM * (16 * F4_PER_ROW / 64);  // C stores per wave per tile
  static_assert(A_LOADS * NWAVES * 1024 == A_BYTES && B_LOADS * NWAVES * 1024 == B_BYTES, "tile");
  static_assert((16 * F4_PER_ROW) % 64 == 0, "epilogue store count must be lane-uniform");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = a.tiles_m * a.tiles_n;
  const int nk = a.K / BK;
  const uint16_t* __restrict__ Ag = (const uint16_t*)a.A;
  const uint16_t* __restrict__ Wg = (const uint16_t*)a.W;

  const uint16_t* a_src[A_LOADS];
  const uint16_t* b_src[B_LOADS];
  auto set_sources = [&](int m0_, int n0_) {
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const int r = (i * NWAVES + wid) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      a_src[i] = Ag + (size_t)min(m0_ + r, a.M - 1) * a.lda + c * 8;
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      const int r = (i * NWAVES + wid) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      b_src[i] = Wg + (size_t)(n0_ + r) * a.ldw + c * 8;
    }
  };
#define PGEMM_STAGE(kt, buf)                                                                   \
  do {                                                                                         \
    char* base_ = smem + (buf) * STAGE_BYTES;                                                  \
    const int koff_ = (kt) * BK;                                                               \
    _Pragma("unroll") for (int i = 0; i < A_LOADS; ++i)                                        \
      __builtin_amdgcn_global_load_lds((const void*)(a_src[i] + koff_),                        \
                                       LDS_PTR(base_ + (i * NWAVES + wid) * 1024), 16, 0, 0);   \
    _Pragma("unroll") for (int i = 0; i < B_LOADS; ++i)                                        \
      __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + koff_),                        \
                                       LDS_PTR(base_ + A_BYTES + (i * NWAVES + wid) * 1024),   \
                                       16, 0, 0);                                              \
  } while (0)

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

  int L = blockIdx.x;
  if (L >= ntiles) return;
  int tm, tn;
  tile_coords(L, a.tiles_m, a.tiles_n, tm, tn);
  set_sources(tm * BM, tn * BN);
  int it = 0;  // running K-step counter: buffer parity continues across tiles
  PGEMM_STAGE(0, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  bool pending_stores = false;

  while (true) {
    const int m0 = tm * BM, n0 = tn * BN;
    const int Ln = L + gridDim.x;
    const bool has_next = Ln < ntiles;
    int tm_n = 0, tn_n = 0;
    if (has_next) tile_coords(Ln, a.tiles_m, a.tiles_n, tm_n, tn_n);
    if (pending_stores) {
      // the previous tile's prefetch (older) must have landed; its stores may drain
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(STORES_PER_WAVE < 63 ? STORES_PER_WAVE : 63)
                   : "memory");
    }
    float4_t acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt, ++it) {
      const int cur = it & 1;
      if (kt + 1 < nk) {
        PGEMM_STAGE(kt + 1, cur ^ 1);
      } else if (has_next) {
        set_sources(tm_n * BM, tn_n * BN);  // current tile's DMA all issued: retarget
        PGEMM_STAGE(0, cur ^ 1);
      }
      const char* base = smem + cur * STAGE_BYTES;
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
      if (kt + 1 < nk)
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      else  // all reads of `cur` done before it becomes the epilogue staging area
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // ---- epilogue through the just-consumed buffer (the other one is loading)
    float* ep = (float*)(smem + ((it - 1) & 1) * STAGE_BYTES) + wid * 16 * EP_LD;
    const bool full_tile = m0 + BM <= a.M;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) ep[(fq * 4 + e) * EP_LD + j * 16 + fr] = acc[i][j][e];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (int f = lane; f < 16 * F4_PER_ROW; f += 64) {
        const int r = f / F4_PER_ROW, c4 = f % F4_PER_ROW;
        const int m = m0 + wm * TM + i * 16 + r;
        if (full_tile || m < a.M) {
          const float4_t v = *(const float4_t*)(ep + r * EP_LD + c4 * 4);
          epilogue_store4(a, m, n0 + wn * TN + c4 * 4, v);
        }
      }
    }
    if (!has_next) break;
    // a partial tile issued fewer stores than the counted wait assumes: drain fully
    if (!full_tile) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // epilogue LDS reads done before the barrier
    pending_stores = true;
    L = Ln;
    tm = tm_n;
    tn = tn_n;
  }
#undef PGEMM_STAGE
}

// ============================================================== bf16 MFMA, 4-phase pipeline
// 256x256x64 tile, 8 waves (2 along M x 4 along N, wave tile 128x64 = 8x4
// MFMA tiles). Each K-tile is computed in 4 phases, one 64x32 quadrant of the
// wave tile (16 MFMAs) per phase:
//   P1 (A lo, B lo)   P2 (A lo, B hi)   P3 (A hi, B hi)   P4 (A hi, B lo)
// The LDS image of one K-tile is cut into 4 regions of 128 rows x 128 B by the
// phase that first reads them, across waves:
//   R1 = A lo rows of both M-halves, R2 = B lo rows of all 4 N-quarters,
//   R3 = B hi rows, R4 = A hi rows.
// Phase p of K-tile t issues region R_p of K-tile t+1 (2 LDS-DMA instructions
// per wave) into the other buffer, then runs its MFMAs, then waits with a
// COUNTED vmcnt(4) — two regions stay in flight across the barrier — before the
// one raw s_barrier of the phase. Every region therefore has >= 3 phases between
// issue and first read (P1->P1, P2->P1, P3->P2, P4->P3), and its buffer slot was
// last read >= 1 barrier earlier (R1: P2, R2: P4, R3: P2, R4: P3 of tile t-1).
// The last K-tile drains with vmcnt(0).
__device__ __forceinline__ int reg_a_row(int q, int hi) {  // region row -> tile row (A)
  return (q >> 6) * 128 + hi * 64 + (q & 63);
}
__device__ __forceinline__ int reg_b_row(int q, int hi) {  // region row -> tile row (B / n)
  return (q >> 5) * 64 + hi * 32 + (q & 31);
}

#define VM_WAIT_BARRIER(N) asm volatile("s_waitcnt vmcnt(" #N ")\n\ts_barrier" ::: "memory")

__global__ __launch_bounds__(512) void gemm_bf16_4ph_kernel(GemmArgs a) {
  constexpr int REG = 128 * 128;      // bytes per region
  constexpr int STAGE = 4 * REG;      // R1 R2 R3 R4
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  int tm, tn;
  tile_coords(blockIdx.x, a.tiles_m, a.tiles_n, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const uint16_t* __restrict__ Ag = (const uint16_t*)a.A;
  const uint16_t* __restrict__ Wg = (const uint16_t*)a.W;

  // DMA sources: region rows q = (piece)*8 + lane/8 for pieces wid and wid+8;
  // physical chunk lane%8 holds logical chunk (lane%8) ^ (q&7).
  const uint16_t* src[4][2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = (wid + 8 * k) * 8 + (lane >> 3);
    const int c = ((lane & 7) ^ (q & 7)) * 8;
    src[0][k] = Ag + (size_t)min(m0 + reg_a_row(q, 0), a.M - 1) * a.lda + c;  // R1
    src[1][k] = Wg + (size_t)(n0 + reg_b_row(q, 0)) * a.ldw + c;              // R2
    src[2][k] = Wg + (size_t)(n0 + reg_b_row(q, 1)) * a.ldw + c;              // R3
    src[3][k] = Ag + (size_t)min(m0 + reg_a_row(q, 1), a.M - 1) * a.lda + c;  // R4
  }
#define ISSUE_REGION(r, kt, buf)                                                             \
  do {                                                                                       \
    char* dst_ = smem + (buf) * STAGE + (r) * REG;                                           \
    const int ko_ = (kt) * 64;                                                               \
    __builtin_amdgcn_global_load_lds((const void*)(src[r][0] + ko_), LDS_PTR(dst_ + wid * 1024), 16, 0, 0); \
    __builtin_amdgcn_global_load_lds((const void*)(src[r][1] + ko_), LDS_PTR(dst_ + (wid + 8) * 1024), 16, 0, 0); \
  } while (0)

  const int fr = lane & 15, fq = lane >> 4;
  // fragment byte offsets inside a region (row q, logical chunk kk*4+fq)
  auto roff = [&](int q, int kk) { return q * 128 + (((kk * 4 + fq) ^ (q & 7)) << 4); };
  int aoff[4][2], boff[2][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) aoff[i][kk] = roff(wm * 64 + i * 16 + fr, kk);
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) boff[j][kk] = roff(wn * 32 + j * 16 + fr, kk);

  float4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / 64;
  ISSUE_REGION(0, 0, 0);
  ISSUE_REGION(1, 0, 0);
  ISSUE_REGION(2, 0, 0);
  ISSUE_REGION(3, 0, 0);
  VM_WAIT_BARRIER(0);

  bf16x8_t af[4][2], bf[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* st = smem + (kt & 1) * STAGE;
    const bool more = kt + 1 < nk;
    const int nb = (kt + 1) & 1;
    // ---- P1: A lo (R1) x B lo (R2)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bf[j][kk] = *(const bf16x8_t*)(st + REG + boff[j][kk]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = *(const bf16x8_t*)(st + aoff[i][kk]);
    if (more) ISSUE_REGION(0, kt + 1, nb);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], acc[i][j], 0, 0, 0);
    if (more) VM_WAIT_BARRIER(4); else VM_WAIT_BARRIER(0);
    // ---- P2: A lo (regs) x B hi (R3)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bf[j][kk] = *(const bf16x8_t*)(st + 2 * REG + boff[j][kk]);
    if (more) ISSUE_REGION(1, kt + 1, nb);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], acc[i][2 + j], 0, 0, 0);
    if (more) VM_WAIT_BARRIER(4); else VM_WAIT_BARRIER(0);
    // ---- P3: A hi (R4) x B hi (regs)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = *(const bf16x8_t*)(st + 3 * REG + aoff[i][kk]);
    if (more) ISSUE_REGION(2, kt + 1, nb);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], acc[4 + i][2 + j], 0, 0, 0);
    if (more) VM_WAIT_BARRIER(6); else VM_WAIT_BARRIER(0);
    // ---- P4: A hi (regs) x B lo (R2 re-read)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bf[j][kk] = *(const bf16x8_t*)(st + REG + boff[j][kk]);
    if (more) ISSUE_REGION(3, kt + 1, nb);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], acc[4 + i][j], 0, 0, 0);
    if (more) VM_WAIT_BARRIER(4); else VM_WAIT_BARRIER(0);
  }
#undef ISSUE_REGION

  // ---- epilogue (LDS free: every DMA retired by the final vmcnt(0) + barrier)
  constexpr int TN = 64, EP_LD = TN + 4, F4_PER_ROW = TN / 4;
  float* ep = (float*)smem + wid * 16 * EP_LD;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) ep[(fq * 4 + e) * EP_LD + j * 16 + fr] = acc[i][j][e];
    __syncthreads();
    for (int f = lane; f < 16 * F4_PER_ROW; f += 64) {
      const int r = f / F4_PER_ROW, c4 = f % F4_PER_ROW;
      const int m = m0 + wm * 128 + i * 16 + r;
      if (m < a.M) {
        const float4_t v = *(const float4_t*)(ep + r * EP_LD + c4 * 4);
        epilogue_store4(a, m, n0 + wn * TN + c4 * 4, v);
      }
    }
  }
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

int launch_bf16_4ph(GemmArgs a, hipStream_t s) {
  if (a.N % 256) return AACLIP_ERR_ARG;
  a.tiles_m = ceil_div(a.M, 256);
  a.tiles_n = a.N / 256;
  const size_t lds = 2 * 4 * 128 * 128;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)gemm_bf16_4ph_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return AACLIP_ERR_LAUNCH;
    attr_set = true;
  }
  gemm_bf16_4ph_kernel<<<a.tiles_m * a.tiles_n, 512, lds, s>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int BM, int BN, int WM, int WN>
int launch_bf16_persistent(GemmArgs a, hipStream_t s) {
  if (a.N % BN) return AACLIP_ERR_ARG;
  a.tiles_m = ceil_div(a.M, BM);
  a.tiles_n = a.N / BN;
  const int ntiles = a.tiles_m * a.tiles_n;
  const size_t lds = 2 * (size_t)(BM + BN) * 64 * 2;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)gemm_bf16_persistent_kernel<BM, BN, WM, WN>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return AACLIP_ERR_LAUNCH;
    attr_set = true;
  }
  const int grid = min(ntiles, num_cus());
  gemm_bf16_persistent_kernel<BM, BN, WM, WN><<<grid, WM * WN * 64, lds, s>>>(a);
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

int g_gemm_variant = 0;  // tuning hook (aaclip_set_gemm_variant); 0 = default dispatch
int g_group_m = 8;
int g_setprio = 0;
int g_dbg = 0;

}  // namespace

extern "C" int aaclip_set_gemm_variant(int variant) {
  // bits 0-3: kernel family; bits 4-7: tile-order group height (0 = 8); bit 8: setprio
  const int fam = variant & 15, grp = (variant >> 4) & 15;
  if (variant < 0 || fam > 5) return AACLIP_ERR_ARG;
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
    // 256x256 tiles when they fill the chip; 256x128 otherwise (N = 768/1024 GEMMs)
    const long t256 = (long)ceil_div(M, 256) * (N / 256);
    const bool big = N % 256 == 0 && t256 >= 2 * 256;
    switch (g_gemm_variant) {
      case 1: return launch_bf16<256, 256, 2, 4>(a, s);                                  // 2-stage only
      case 2: return N % 256 == 0 ? launch_bf16_4ph(a, s) : launch_bf16<256, 128, 4, 2>(a, s);  // 4-phase always
      case 3: return launch_bf16<256, 128, 4, 2>(a, s);
      case 4: return N % 256 == 0 ? launch_bf16<320, 256, 2, 4>(a, s) : launch_bf16<256, 128, 4, 2>(a, s);
      case 5: return N % 256 == 0 ? launch_bf16_persistent<320, 256, 2, 4>(a, s) : launch_bf16<256, 128, 4, 2>(a, s);
      default: break;
    }
    (void)big;
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
