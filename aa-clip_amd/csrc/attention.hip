// Fused multi-head attention (flash-style, scores never leave the CU) for the
// ViT-L/14 visual tower (seq 577 @336 px, 16 heads x 64) and the causal text
// tower (seq 77, 12 heads x 64). Replaces torch F.multi_head_attention_forward
// as called from nn.MultiheadAttention (reference model/transformer.py:200).
//
// bf16 kernel layout choices (gfx950, v_mfma_f32_16x16x32_bf16):
//   * workgroup = 4 waves = 128 queries of one (image, head); wave = 2 x 16 queries
//   * S^T = K . Q^T (keys on accumulator rows, the query on the lane): each lane
//     owns one query's scores, so the softmax row reductions are in-register plus
//     two cross-lane steps, and P^T leaves the accumulator already in the B-operand
//     layout of the next MFMA — no LDS round trip for P.
//   * O^T = V^T . P^T: the V^T operand comes from the row-major V tile through the
//     gfx950 transposing LDS read ds_read_b64_tr_b16; the key order inside each
//     32-key MFMA step is permuted consistently on both operands.
//   * K/V tiles (64 keys) arrive by LDS-DMA (global_load_lds_dwordx4) into a
//     double-buffered, XOR-swizzled LDS image; Q stays in registers.
//   * online softmax in the log2 domain (v_exp_f32), fp32 statistics.
#include <math.h>

#include "common.h"

namespace {

constexpr int HD_ = 64;      // head dim
constexpr int KT = 64;       // keys per tile

__device__ __forceinline__ short4_t tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(p));
}

// byte offset of (row, 16-B chunk) in a swizzled [64][128 B] tile
__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// Cross-lane max over the 4 lanes {c, c+16, c+32, c+48} that hold one query's
// scores: v_permlane16_swap / v_permlane32_swap (VALU, no LDS round trip). The two
// combines are single v_max_f32 in asm: fmaxf's IEEE semantics make hipcc
// canonicalise both permlane outputs first (2 extra v_max per combine); the inputs
// here are finite scores or -inf. The s_nop covers the VALU-write -> permlane-read
// hazard the compiler does not see through the asm.
__device__ __forceinline__ float max_over_groups(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  float m;
  asm("v_max_f32 %0, %1, %2\n\ts_nop 1" : "=v"(m) : "v"(a[0]), "v"(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  asm("v_max_f32 %0, %1, %2" : "=v"(m) : "v"(b[0]), "v"(b[1]));
  return m;
}

// Max of a lane's 4 x NKB scores as a tree of v_max3 (depth 3 for 16 values instead
// of a 16-long dependent chain; max is exact, so the order does not change the bits).
template <int NKB>
__device__ __forceinline__ float tile_lane_max(const float4_t (&st)[NKB]) {
  if constexpr (NKB == 4) {
    const float a = fmaxf(fmaxf(st[0][0], st[0][1]), st[0][2]);
    const float b = fmaxf(fmaxf(st[0][3], st[1][0]), st[1][1]);
    const float c = fmaxf(fmaxf(st[1][2], st[1][3]), st[2][0]);
    const float d = fmaxf(fmaxf(st[2][1], st[2][2]), st[2][3]);
    const float e = fmaxf(fmaxf(st[3][0], st[3][1]), st[3][2]);
    return fmaxf(fmaxf(fmaxf(a, b), c), fmaxf(fmaxf(d, e), st[3][3]));
  } else {
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) mx = fmaxf(mx, st[kb][i]);
    return mx;
  }
}

// One 64-key tile for one wave: NKB live 16-key blocks (1, 2 or 4), NQB live
// 16-query blocks (1 or 2), MASK = tile needs the key-tail / causal mask.
// Dead blocks and the mask are resolved at compile time, so the 577 = 9*64 + 1
// key tail costs 1/4 of a tile and full tiles carry no masking code.
// Q arrives pre-scaled by log2(e)/sqrt(64) (folded into the Q projection by the
// caller, or applied to the Q fragments at load), so S' = K.Q^T is already in
// the log2 domain, and the QK^T accumulator is initialised to -m (m = this
// query's running max): the MFMA delivers S' - m and p = exp2(S' - m) is one
// v_exp_f32 per score, no FMA. The running max is DEFERRED: it only moves when
// a tile's max exceeds it by more than 2^8 (kRescaleLog2), so p <= 256 and the
// O/l rescale (and the shift of this tile's scores) runs on the first tile and
// then almost never. The result is the same softmax: O and l carry the same
// factor 2^-m.
// The softmax denominator is one more MFMA per 32 keys: an all-ones A operand
// against the same bf16 P^T fragment gives sum_k p[k][q] in every accumulator
// row (lane-local, already reduced over keys), replacing 16 v_add per 16 queries
// per tile on an issue-bound loop; numerator and denominator then use the same
// bf16-rounded p.
constexpr float kRescaleLog2 = 8.0f;

template <int NKB, int NQB, bool MASK, bool H16>
__device__ __forceinline__ void attn_tile(const char* kt_lds, const h16x8_t<H16> (&qf)[NQB][2],
                                          float4_t (&ot)[NQB][4], float (&m_run)[NQB], float4_t (&l_acc)[NQB],
                                          int key0, int q0, int N, int causal, int g, int c, bool first) {
  using V8 = h16x8_t<H16>;
  using E = h16_t<H16>;
  const char* vt_lds = kt_lds + KT * 128;
  float4_t st[NQB][NKB];
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    const float nm = -m_run[qb];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) st[qb][kb] = float4_t{nm, nm, nm, nm};
  }
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const V8 kf = *(const V8*)(kt_lds + swz(kb * 16 + c, ks * 4 + g));
#pragma unroll
      for (int qb = 0; qb < NQB; ++qb) st[qb][kb] = mfma16(kf, qf[qb][ks], st[qb][kb]);
    }
  }
  constexpr int NKS = (NKB + 1) / 2;  // 32-key MFMA steps for P.V
  V8 pf[NQB][NKS];
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    float mx = -INFINITY;
    if constexpr (MASK) {
      // keys valid for this lane's query: key < lim
      const int q = q0 + qb * 16 + c;
      const int lim = (causal ? min(N, q + 1) : N) - key0 - 4 * g;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sv = (kb * 16 + i < lim) ? st[qb][kb][i] : -INFINITY;
          st[qb][kb][i] = sv;
          mx = fmaxf(mx, sv);
        }
    } else {
      mx = tile_lane_max<NKB>(st[qb]);
    }
    // The deferred max only moves when some query's tile max beats it by 2^8. A query's
    // max is the max of its 4 lanes' maxes, so "no lane's own max exceeds the bound"
    // (one ballot) means no query moves: the cross-lane reduction runs only on the
    // rare rescale path (and on tile 0).
    if (__builtin_amdgcn_ballot_w64(first || mx > kRescaleLog2) != 0) {  // wave-uniform, rare after tile 0
      mx = max_over_groups(mx);  // max over the tile of S' - m for this lane's query
      const bool move = first || mx > kRescaleLog2;
      const float d = move ? mx : 0.f;  // tile 0 always has a valid key: mx is finite
      m_run[qb] += d;
      const float alpha = __builtin_amdgcn_exp2f(-d);
      l_acc[qb][0] *= alpha;  // only element 0 is read at the end
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int e = 0; e < 4; ++e) ot[qb][db][e] *= alpha;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) st[qb][kb][i] -= d;
    }
    float p[2 * NKS][4];
#pragma unroll
    for (int kb = 0; kb < 2 * NKS; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) p[kb][i] = kb < NKB ? __builtin_amdgcn_exp2f(st[qb][kb < NKB ? kb : 0][i]) : 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      V8 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = (E)p[2 * ks][i];
        v[4 + i] = (E)p[2 * ks + 1][i];
      }
      pf[qb][ks] = v;
    }
  }
  // l += 1 . P^T
  const V8 ones = {(E)1.f, (E)1.f, (E)1.f, (E)1.f, (E)1.f, (E)1.f, (E)1.f, (E)1.f};
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) l_acc[qb] = mfma16(ones, pf[qb][ks], l_acc[qb]);
  // O^T += V^T . P^T ; V^T fragment via transposing LDS reads
#pragma unroll
  for (int db = 0; db < 4; ++db) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int qq = c >> 2, pp = c & 3;
      const int chunk = db * 2 + (pp >> 1);
      const int r0 = ks * 32 + 4 * g + qq;
      const short4_t lo = tr_read(vt_lds + swz(r0, chunk) + (pp & 1) * 8);
      const short4_t hi = tr_read(vt_lds + swz(r0 + 16, chunk) + (pp & 1) * 8);
      const short8_t vv = short8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const V8 vf = __builtin_bit_cast(V8, vv);
#pragma unroll
      for (int qb = 0; qb < NQB; ++qb) ot[qb][db] = mfma16(vf, pf[qb][ks], ot[qb][db]);
    }
  }
}

// Full 64-key tile for two 16-query blocks, phase-split: the same arithmetic as
// attn_tile<4, 2, false>, ordered so each straight-line block pairs one block's
// softmax VALU with the other block's MFMAs (Kᵀ·Q of block 1 beside the
// exponentials of block 0, then P·V of block 0 beside the exponentials of block
// 1). Each block's max-move branch sits between the two, before any of its p is
// formed (the deferred-max rule of attn_tile).
template <bool H16>
__device__ __forceinline__ void attn_tile_split(const char* kt_lds, const h16x8_t<H16> (&qf)[2][2],
                                                float4_t (&ot)[2][4], float (&m_run)[2], float4_t (&l_acc)[2],
                                                int g, int c, bool first) {
  using V8 = h16x8_t<H16>;
  using E = h16_t<H16>;
  const char* vt_lds = kt_lds + KT * 128;
  auto qk = [&](int qb, float4_t (&st)[4]) {
    const float nm = -m_run[qb];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) st[kb] = float4_t{nm, nm, nm, nm};
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const V8 kf = *(const V8*)(kt_lds + swz(kb * 16 + c, ks * 4 + g));
        st[kb] = mfma16(kf, qf[qb][ks], st[kb]);
      }
  };
  auto max_decide = [&](int qb, float4_t (&st)[4]) {
    float mx = tile_lane_max<4>(st);
    if (__builtin_amdgcn_ballot_w64(first || mx > kRescaleLog2) != 0) {  // lane-local check, as attn_tile
      mx = max_over_groups(mx);
      const bool move = first || mx > kRescaleLog2;
      const float d = move ? mx : 0.f;
      m_run[qb] += d;
      const float alpha = __builtin_amdgcn_exp2f(-d);
      l_acc[qb][0] *= alpha;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int e = 0; e < 4; ++e) ot[qb][db][e] *= alpha;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) st[kb][i] -= d;
    }
  };
  auto expo = [&](const float4_t (&st)[4], V8 (&pf)[2]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      V8 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = (E)__builtin_amdgcn_exp2f(st[2 * ks][i]);
        v[4 + i] = (E)__builtin_amdgcn_exp2f(st[2 * ks + 1][i]);
      }
      pf[ks] = v;
    }
  };
  float4_t s0[4], s1[4];
  V8 p0[2], p1[2];
  qk(0, s0);
  max_decide(0, s0);
  expo(s0, p0);
  qk(1, s1);
  // keep block 0's exponentials in this block: hipcc otherwise sinks them past the
  // next branch (their first use is P.V), and the two VALU runs end up together
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) asm volatile("" : "+v"(p0[ks]));
  max_decide(1, s1);
  expo(s1, p1);
  const V8 ones = {(E)1.f, (E)1.f, (E)1.f, (E)1.f, (E)1.f, (E)1.f, (E)1.f, (E)1.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) l_acc[0] = mfma16(ones, p0[ks], l_acc[0]);
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int qq = c >> 2, pp = c & 3;
      const int chunk = db * 2 + (pp >> 1);
      const int r0 = ks * 32 + 4 * g + qq;
      const short4_t lo = tr_read(vt_lds + swz(r0, chunk) + (pp & 1) * 8);
      const short4_t hi = tr_read(vt_lds + swz(r0 + 16, chunk) + (pp & 1) * 8);
      const V8 vf = __builtin_bit_cast(V8, short8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      ot[0][db] = mfma16(vf, p0[ks], ot[0][db]);
      ot[1][db] = mfma16(vf, p1[ks], ot[1][db]);
    }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) l_acc[1] = mfma16(ones, p1[ks], l_acc[1]);
}

#ifndef ATTN_STAGES
#define ATTN_STAGES 3  // K/V ring depth (LDS: ATTN_STAGES x 16 KiB per workgroup)
#endif
#ifndef ATTN_OCC
#define ATTN_OCC 3  // workgroups per CU the register budget is sized for
#endif

// Counted wait for the K/V ring + workgroup barrier: PIECES = LDS-DMA pieces one
// wave issues per stage (K and V), i.e. how many may stay in flight (the newest stage).
template <int PIECES>
__device__ __forceinline__ void wait_barrier(bool deep) {
  if (!deep)
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (PIECES == 4)
    asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  else if constexpr (PIECES == 8)
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else
    static_assert(PIECES == 4 || PIECES == 8, "pieces per wave per stage");
}

// H16: fp16 q/k/v/p on v_mfma_f32_16x16x32_f16 (the parity-grade mode), else bf16.
// QB 16-query blocks per wave, NW waves per workgroup (QT = 16 * QB * NW queries),
// NS-stage K/V ring. Every wave reads the whole K and V tile from LDS, so queries
// per wave set the LDS bytes per FLOP: QB = 4 halves them against QB = 2.
template <bool H16, int QB, int NW, int NS, int SPLIT>
__global__ __launch_bounds__(64 * NW, NW == 4 ? ATTN_OCC : 4) void attn_bf16_kernel(
    const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out, int batch, int N, int H, int flags,
    uint8_t* __restrict__ out_mx, int64_t ld_mx) {
  AACLIP_TRACE_SCOPE(TR_ATTN);
  const int causal = flags & AACLIP_ATTN_CAUSAL;
  constexpr int QW = 16 * QB;     // queries per wave
  constexpr int QT = QW * NW;     // queries per workgroup
  constexpr int PR = 64 / (8 * NW);  // 8-row DMA pieces per wave per K (and per V) tile
  // the prologue fills NS-1 <= 2 stages and the counted waits assume <= 2 tiles in
  // flight: a 4-stage ring would read a never-filled slot (measured: checksums
  // differ run to run), so only 2 and 3 are valid
  static_assert(NS == 2 || NS == 3, "ATTN_STAGES must be 2 or 3");
  using V8 = h16x8_t<H16>;
  using E = h16_t<H16>;
  // [stage][K|V][64][128B], then the key tail's K and V rows ([K|V][8][128B])
  __shared__ __attribute__((aligned(16))) char smem[NS * 2 * KT * 128 + 2048];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, c = lane & 15;
  // XCD-aware remap of the 1-D grid: blocks b, b+8, ... share an XCD (its L2), so
  // give each XCD a contiguous run of work ids and order work ids query-tile
  // fastest: all query tiles of one (image, head) then read that head's K/V from
  // the same L2 instead of from 5 different XCDs (PMC: L2 hit rate 20% before).
  const int nq = (N + QT - 1) / QT;
  const int nwg = gridDim.x;
  const int xcd = blockIdx.x & 7, qd = nwg >> 3, rd = nwg & 7;
  const int wgid = (xcd < rd ? xcd * (qd + 1) : rd * (qd + 1) + (xcd - rd) * qd) + (blockIdx.x >> 3);
  const int qtile = wgid % nq;
  const int bh = wgid / nq;
  const int b = bh / H, h = bh % H;
  const int HDt = H * HD_;
  const int64_t ld = 3 * (int64_t)HDt;
  const uint16_t* base = qkv + (size_t)b * N * ld + h * HD_;
  const int q0 = qtile * QT + wid * QW;

  // ---- Q fragments (B operand of K.Q^T): lane holds Q[q][ks*32 + 8g .. +7]
  V8 qf[QB][2];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const int q = min(q0 + qb * 16 + c, N - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[qb][ks] = *(const V8*)(base + (size_t)q * ld + ks * 32 + 8 * g);
  }
  if (!(flags & AACLIP_ATTN_Q_PRESCALED)) {  // log2(e)/sqrt(64) not folded by the caller: apply it here
    constexpr float sl2 = 0.125f * 1.4426950408889634f;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[qb][ks][e] = (E)((float)qf[qb][ks][e] * sl2);
  }

  // ---- DMA sources: wave w loads pieces i*4+w (8 rows each) of the K and V tiles
  // through a buffer descriptor spanning this head's rows to the end of the batch:
  // lane offsets are tile-invariant (VGPR), the tile step is a scalar offset, and
  // keys past the last image read as zeros (keys past N inside the batch are the
  // next image's finite rows; both are masked to p = 0 in the tail tile).
  const int64_t head0 = (int64_t)b * N * ld + h * HD_;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(qkv + head0), 0, (int)(((int64_t)batch * N * ld - head0) * 2), 0x00020000);
  int voff[4];  // PR <= 4 used (fixed size: a template-dependent array captured by the staging
               // lambda makes clang's host pass drop the kernel's instantiation)
  static_assert(PR <= 4, "DMA pieces per wave");
#pragma unroll
  for (int i = 0; i < PR; ++i) {
    const int r = (i * NW + wid) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ (r & 7);
    voff[i] = (int)(r * ld + HDt + chunk * 8) * 2;
  }
  const int row_bytes = (int)ld * 2, v_off = HDt * 2;
  auto stage = [&](int t, int buf) {
    char* kb = smem + buf * (2 * KT * 128);
    char* vb = kb + KT * 128;
    const int so = t * KT * row_bytes;
#pragma unroll
    for (int i = 0; i < 64 / (8 * NW); ++i) {  // PR pieces (template expression: no capture in the lambda)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(kb + (i * NW + wid) * 1024), 16, voff[i], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(vb + (i * NW + wid) * 1024), 16, voff[i], so + v_off,
                                               0, 0);
    }
  };

  float4_t ot[QB][4];
  float m_run[QB];     // set from the first tile (attn_tile first = true)
  float4_t l_acc[QB];  // row sums (MFMA)
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
#pragma unroll
    for (int db = 0; db < 4; ++db) ot[qb][db] = float4_t{0.f, 0.f, 0.f, 0.f};
    m_run[qb] = 0.f;
    l_acc[qb] = float4_t{0.f, 0.f, 0.f, 0.f};
  }

  int ntiles = (N + KT - 1) / KT;
  if (causal) {
    const int last_q = min(qtile * QT + QT - 1, N - 1);
    ntiles = min(ntiles, last_q / KT + 1);
  }
  // A short key tail (non-causal, N % 64 <= 8: 577 = 9*64 + 1, 1025 = 16*64 + 1) is
  // folded in after the tile loop as exact per-key online-softmax updates from the
  // K/V rows in global memory, instead of a whole masked tile iteration (DMA, QK^T,
  // softmax, P.V and a barrier for one key: 9 % of the C2 attention time).
  const int tail_keys = causal ? 0 : N % KT;
  const bool tail_inline = tail_keys > 0 && tail_keys <= 8;
  if (tail_inline) ntiles = N / KT;

  // Ring of NS K/V stages: tile t+NS-1 is issued while tile t is computed; the
  // end-of-tile wait is COUNTED (vmcnt retires in order, 4 DMAs per wave per
  // stage) so tiles t+2.. stay in flight across the barrier.
  // the key tail's K / V rows (<= 8) into LDS behind the ring, by wave 0 ahead of the
  // first stage (the oldest ops: the prologue's counted wait retires them), so the fold
  // after the tile loop reads LDS instead of waiting out a global-load round trip
  char* const tail_lds = smem + NS * 2 * KT * 128;
  if (tail_inline && wid == 0) {
    const int tvo = ((N - tail_keys + (lane >> 3)) * (int)ld + HDt + (lane & 7) * 8) * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(tail_lds), 16, tvo, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(tail_lds + 1024), 16, tvo, v_off, 0, 0);
  }
  stage(0, 0);
  if (NS > 2 && ntiles > 1) stage(1, 1);
  wait_barrier<2 * PR>(NS > 2 && ntiles > 1);
  // Waves always compute both 16-query blocks (rows past N are clamped copies,
  // discarded at the store); a wave with no valid query skips the math but keeps
  // staging and barriers. Full tiles (no key tail, no causal cut for any wave of
  // the workgroup) run one tile instance in a loop of their own: a per-tile
  // dispatch over several instances costs ~40 accumulator register copies per tile
  // on this issue-bound loop. The masked tail (key tail; causal diagonal) follows.
  const bool active = q0 < N;
  const int nfull = causal ? min(N / KT, (qtile * QT + 1) / KT) : N / KT;
  int t = 0, cur = 0;
  auto advance = [&]() {  // issue tile t+NS-1, then wait for tile t+1 and sync
    const int nxt = t + NS - 1;
    int nb = cur + NS - 1;
    if (nb >= NS) nb -= NS;
    if (nxt < ntiles) stage(nxt, nb);
    return nxt < ntiles && NS > 2;
  };
  for (; t < nfull; ++t) {
    const bool deep = advance();
    if (active) {
      if constexpr (SPLIT == 1 && QB == 2)
        attn_tile_split<H16>(smem + cur * (2 * KT * 128), qf, ot, m_run, l_acc, g, c, t == 0);
      else
        attn_tile<4, QB, false, H16>(smem + cur * (2 * KT * 128), qf, ot, m_run, l_acc, t * KT, q0, N, causal, g,
                                     c, t == 0);
    }
    wait_barrier<2 * PR>(deep);
    cur = cur + 1 == NS ? 0 : cur + 1;
  }
  for (; t < ntiles; ++t) {
    const bool deep = advance();
    const char* kt_lds = smem + cur * (2 * KT * 128);
    const int key0 = t * KT;
    const int live = min(KT, N - key0);  // valid keys in this tile
    if (active) {
      const bool first = t == 0;
      if (live > 32) attn_tile<4, QB, true, H16>(kt_lds, qf, ot, m_run, l_acc, key0, q0, N, causal, g, c, first);
      else if (live > 16) attn_tile<2, QB, true, H16>(kt_lds, qf, ot, m_run, l_acc, key0, q0, N, causal, g, c, first);
      else attn_tile<1, QB, true, H16>(kt_lds, qf, ot, m_run, l_acc, key0, q0, N, causal, g, c, first);
    }
    wait_barrier<2 * PR>(deep);
    cur = cur + 1 == NS ? 0 : cur + 1;
  }
  if (ntiles == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the prologue's tile-0 DMA

  if (tail_inline && active) {
    for (int j = N - tail_keys; j < N; ++j) {
      const char* kr = tail_lds + (j - (N - tail_keys)) * 128;  // K row j (LDS), V row j at +1024
      const V8 k0 = *(const V8*)(kr + 16 * g), k1 = *(const V8*)(kr + 64 + 16 * g);
      float vv[4][4];  // V[j][d = db*16 + 4g + i], the lane's O columns
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const uint2 w = *(const uint2*)(kr + 1024 + db * 32 + 8 * g);
        vv[db][0] = h16_to_f32<H16>((uint16_t)(w.x & 0xffff));
        vv[db][1] = h16_to_f32<H16>((uint16_t)(w.x >> 16));
        vv[db][2] = h16_to_f32<H16>((uint16_t)(w.y & 0xffff));
        vv[db][3] = h16_to_f32<H16>((uint16_t)(w.y >> 16));
      }
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        float sp = 0.f;  // this lane's 16 of the 64 dims (Q prescaled: log2 domain)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          sp = fmaf((float)qf[qb][0][e], (float)k0[e], fmaf((float)qf[qb][1][e], (float)k1[e], sp));
        auto a2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(sp), __float_as_uint(sp), false, false);
        sp = __uint_as_float(a2[0]) + __uint_as_float(a2[1]);
        auto b2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(sp), __float_as_uint(sp), false, false);
        sp = __uint_as_float(b2[0]) + __uint_as_float(b2[1]);
        const float mn = fmaxf(m_run[qb], sp);
        const float alpha = __builtin_amdgcn_exp2f(m_run[qb] - mn), p = __builtin_amdgcn_exp2f(sp - mn);
        m_run[qb] = mn;
        l_acc[qb][0] = fmaf(l_acc[qb][0], alpha, p);
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
          for (int i = 0; i < 4; ++i) ot[qb][db][i] = fmaf(ot[qb][db][i], alpha, p * vv[db][i]);
      }
    }
  }

  // ---- epilogue: O[q][d = db*16 + 4g + i] = ot / l
  if (!H16 && out_mx) {
    // MX fp8 output (config C5, the out-proj input): one head = one 64-column block,
    // held by the 4 lanes {c, c+16, c+32, c+48}: block max over them, e8m0 scale,
    // RNE e4m3, 4x4 dword transpose so lane g owns columns 16g..16g+15 -> 16-B stores
    uint8_t* o8 = (uint8_t*)out;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const float inv = 1.0f / l_acc[qb][0];
      const int q = q0 + qb * 16 + c;
      float amax = 0.f;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int i = 0; i < 4; ++i) amax = fmaxf(amax, fabsf(ot[qb][db][i] * inv));
      amax = max_over_groups(amax);
      int e = 0;
      if (amax > 0.f) {
        int x;
        (void)frexpf(amax, &x);
        e = x - 9;
        if (ldexpf(amax, -e) > 448.f) e += 1;
        e = max(min(e, 127), -126);
      }
      const float s = inv * __uint_as_float((uint32_t)(127 - e) << 23);
      uint32_t d[4];
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(ot[qb][db][0] * s, ot[qb][db][1] * s, 0, false);
        d[db] = __builtin_amdgcn_cvt_pk_fp8_f32(ot[qb][db][2] * s, ot[qb][db][3] * s, w, true);
      }
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
      if (q < N) {
        const size_t row = (size_t)b * N + q;
        *(uint4*)(o8 + row * HDt + h * HD_ + 16 * g) = uint4{d[0], d[1], d[2], d[3]};
        if (g == 0) out_mx[((size_t)(h >> 1) * ld_mx + row) * 2 + (h & 1)] = (uint8_t)(e + 127);
      }
    }
    return;
  }
  // 16-B stores: lane group g holds columns 4g..4g+3 of each 16-column block db; a
  // v_permlane16_swap per packed dword pairs blocks (2p, 2p+1) across groups g, g^1, so
  // group g ends with 8 consecutive columns: block 2p + (g & 1), columns 8 (g >> 1) .. +7
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const float inv = 1.0f / l_acc[qb][0];
    const int q = q0 + qb * 16 + c;
    uint4 w[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const uint32_t a0 = pack_h16x2<H16>(ot[qb][2 * pr][0] * inv, ot[qb][2 * pr][1] * inv);
      const uint32_t a1 = pack_h16x2<H16>(ot[qb][2 * pr][2] * inv, ot[qb][2 * pr][3] * inv);
      const uint32_t b0 = pack_h16x2<H16>(ot[qb][2 * pr + 1][0] * inv, ot[qb][2 * pr + 1][1] * inv);
      const uint32_t b1 = pack_h16x2<H16>(ot[qb][2 * pr + 1][2] * inv, ot[qb][2 * pr + 1][3] * inv);
      const auto x = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
      const auto y = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
      w[pr] = uint4{x[0], y[0], x[1], y[1]};
    }
    if (q < N) {
      uint16_t* o = out + ((size_t)b * N + q) * HDt + h * HD_ + 16 * (g & 1) + 8 * (g >> 1);
      *(uint4*)(o) = w[0];
      *(uint4*)(o + 32) = w[1];
    }
  }
}

// ---------------------------------------------------------------- fp32 (parity mode)
// Flash attention on v_mfma_f32_16x16x4f32 (exact fp32 products, fp32 accumulation; the
// fp32 matrix rate is the fp32 vector peak, and the softmax VALU is small beside it).
// Workgroup = 4 waves x 32 queries of one (image, head); K/V tiles of 64 keys staged
// through registers into row-padded LDS (68 floats per row: the strided fragment reads
// below are bank-conflict-free); the next tile's global loads are in flight while the
// current one is computed. Same swapped layout as the 16-bit kernel: S^T = K . Q^T puts
// one query's scores on the 4 lanes {fr, fr+16, fr+32, fr+48}, and each lane's own P
// registers are the B operand of O^T = V^T . P^T (the key order inside a 4-key MFMA step
// is the lane group's). Online softmax in the log2 domain (log2(e)/8 folded into Q).
constexpr int F32_LDK = 68;

__global__ __launch_bounds__(256, 2) void attn_f32_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                          int N, int H, int causal) {
  AACLIP_TRACE_SCOPE(TR_ATTN_F32);
  constexpr int QB = 2;  // 16-query blocks per wave
  __shared__ __attribute__((aligned(16))) float Ks[KT][F32_LDK];
  __shared__ __attribute__((aligned(16))) float Vs[KT][F32_LDK];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int bh = blockIdx.y;
  const int b = bh / H, h = bh % H;
  const int HDt = H * HD_;
  const int64_t ld = 3 * (int64_t)HDt;
  const float* base = qkv + (size_t)b * N * ld + h * HD_;
  const int q0 = blockIdx.x * 128 + wid * 32;
  const bool active = q0 < N;

  constexpr float qscale = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
  float qv[QB][16];  // Q[q][4s + fq] for this lane's query q = q0 + 16 qb + fr
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const float* qr = base + (size_t)min(q0 + qb * 16 + fr, N - 1) * ld;
#pragma unroll
    for (int s4 = 0; s4 < 16; ++s4) qv[qb][s4] = qr[4 * s4 + fq] * qscale;
  }

  int ntiles = (N + KT - 1) / KT;
  if (causal) ntiles = min(ntiles, min((int)blockIdx.x * 128 + 127, N - 1) / KT + 1);

  // staging: thread t moves float4 number t + 256 j (j < 4) of the K and of the V tile
  float4_t kreg[4], vreg[4];
  auto load_tile = [&](int tile) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = t + 256 * j, r = f >> 4, c4 = f & 15;
      const float* src = base + (size_t)min(tile * KT + r, N - 1) * ld + HDt + 4 * c4;
      kreg[j] = *(const float4_t*)src;
      vreg[j] = *(const float4_t*)(src + HDt);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = t + 256 * j, r = f >> 4, c4 = f & 15;
      *(float4_t*)&Ks[r][4 * c4] = kreg[j];
      *(float4_t*)&Vs[r][4 * c4] = vreg[j];
    }
  };

  float4_t o[QB][4];
  float m[QB], l[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
#pragma unroll
    for (int db = 0; db < 4; ++db) o[qb][db] = float4_t{0.f, 0.f, 0.f, 0.f};
    m[qb] = -INFINITY;
    l[qb] = 0.f;
  }

  load_tile(0);
  store_tile();
  __syncthreads();
  for (int tile = 0; tile < ntiles; ++tile) {
    if (tile + 1 < ntiles) load_tile(tile + 1);  // lands while this tile is computed
    if (active) {
      const int key0 = tile * KT;
      float4_t st[QB][4];
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) st[qb][kb] = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int s4 = 0; s4 < 16; ++s4) {
          const float kf = Ks[kb * 16 + fr][4 * s4 + fq];
#pragma unroll
          for (int qb = 0; qb < QB; ++qb)
            st[qb][kb] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf, qv[qb][s4], st[qb][kb], 0, 0, 0);
        }
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        // st[qb][kb][e] = score of key key0 + 16 kb + 4 fq + e for query q
        const int q = q0 + qb * 16 + fr;
        const int lim = (causal ? min(N, q + 1) : N) - key0 - 4 * fq;  // valid: 16 kb + e < lim
        float mx = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = (16 * kb + e < lim) ? st[qb][kb][e] : -INFINITY;
            st[qb][kb][e] = v;
            mx = fmaxf(mx, v);
          }
        mx = max_over_groups(mx);
        const float mn = fmaxf(m[qb], mx);
        const float mu = mn == -INFINITY ? 0.f : mn;  // no valid key yet: keep p = 0, alpha = 1
        const float alpha = __builtin_amdgcn_exp2f(m[qb] - mu);
        m[qb] = mn;
        float ls = 0.f;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float p = __builtin_amdgcn_exp2f(st[qb][kb][e] - mu);
            st[qb][kb][e] = p;
            ls += p;
          }
        l[qb] = l[qb] * alpha + ls;
#pragma unroll
        for (int db = 0; db < 4; ++db) o[qb][db] *= alpha;
      }
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float vf = Vs[kb * 16 + 4 * fq + i][db * 16 + fr];
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
              o[qb][db] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf, st[qb][kb][i], o[qb][db], 0, 0, 0);
          }
    }
    __syncthreads();
    if (tile + 1 < ntiles) {
      store_tile();
      __syncthreads();
    }
  }
  if (!active) return;
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    // the query's row sum is split over its 4 lane groups
    auto a2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(l[qb]), __float_as_uint(l[qb]), false, false);
    float lt = __uint_as_float(a2[0]) + __uint_as_float(a2[1]);
    auto b2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
    lt = __uint_as_float(b2[0]) + __uint_as_float(b2[1]);
    const int q = q0 + qb * 16 + fr;
    if (q < N) {
      float* op = out + ((size_t)b * N + q) * HDt + h * HD_ + 4 * fq;
#pragma unroll
      for (int db = 0; db < 4; ++db) *(float4_t*)(op + 16 * db) = o[qb][db] / lt;
    }
  }
}

// 1 = 4 waves x 32 queries (3-stage ring, 3 workgroups per CU), 2 = 2 waves x 64
// queries (2-stage ring, 4 workgroups per CU: half the LDS bytes per FLOP), 3 = 1
// with the phase-split full tile (attn_tile_split: 3-6 % faster, the default). Removed
// after measuring slower or equal: 4 = speculative exponentials (same bits, equal), 5-7 =
// the 32x32x16 cross-tile pipelined kernel (10 % slower at 2 workgroups per CU, spills at
// 3) in round 5 (round-4 history); in round 6, 4 / 5 = 4 / 8 of every 16 exponentials as
// a Cody-Waite cubic on the VALU (-1.4 / -2.9 % in the step: profiles/r06/attn_exp_emulation_ab.txt).
constexpr int kAttnDefault = 3;
int g_attn_variant = 0;

template <bool H16, int QB, int NW, int NS, int SPLIT = 0>
void launch_attn(const uint16_t* q, uint16_t* o, int batch, int seq, int heads, int flags, uint8_t* mx, int64_t ld_mx,
                 hipStream_t s) {
  const long nwg = (long)ceil_div(seq, 16 * QB * NW) * batch * heads;
  attn_bf16_kernel<H16, QB, NW, NS, SPLIT>
      <<<(unsigned)nwg, 64 * NW, 0, s>>>(q, o, batch, seq, heads, flags, mx, ld_mx);
}

}  // namespace

extern "C" int aaclip_set_attn_variant(int variant) {
  AACLIP_REQUIRE(variant >= 0 && variant <= 3);
  g_attn_variant = variant;
  return AACLIP_OK;
}

extern "C" int aaclip_attention(int dtype, const void* qkv, void* out, int batch, int seq,
                                int heads, int head_dim, int flags, void* out_mx, int64_t ld_mx,
                                void* stream) {
  AACLIP_REQUIRE(dtype == AACLIP_F32 || dtype == AACLIP_BF16 || dtype == AACLIP_FP8 || dtype == AACLIP_F16);
  AACLIP_REQUIRE(qkv && out && batch > 0 && seq > 0 && heads > 0 && head_dim == HD_);
  AACLIP_REQUIRE((flags & ~(AACLIP_ATTN_CAUSAL | AACLIP_ATTN_Q_PRESCALED)) == 0);
  AACLIP_REQUIRE(dtype != AACLIP_F32 || !(flags & AACLIP_ATTN_Q_PRESCALED));
  AACLIP_REQUIRE((int64_t)batch * seq * 3 * heads * HD_ * 2 < (1ll << 31));  // buffer-descriptor range
  AACLIP_REQUIRE(dtype != AACLIP_FP8 || (out_mx && ld_mx >= (int64_t)batch * seq && heads % 2 == 0));
  hipStream_t s = (hipStream_t)stream;
  if (dtype != AACLIP_F32) {  // bf16 / fp16 compute; fp8 = bf16 inputs with an MX e4m3 output
    const int v = g_attn_variant ? g_attn_variant : kAttnDefault;
    const long nwg = (long)ceil_div(seq, 128) * batch * heads;  // every variant: 128 queries per workgroup
    AACLIP_REQUIRE(nwg < (1L << 31));
    const uint16_t* q = (const uint16_t*)qkv;
    uint16_t* o = (uint16_t*)out;
    uint8_t* mx = dtype == AACLIP_FP8 ? (uint8_t*)out_mx : nullptr;
    if (dtype == AACLIP_F16) {
      if (v == 2) launch_attn<true, 4, 2, 2>(q, o, batch, seq, heads, flags, nullptr, 0, s);
      else if (v == 3) launch_attn<true, 2, 4, ATTN_STAGES, 1>(q, o, batch, seq, heads, flags, nullptr, 0, s);
      else launch_attn<true, 2, 4, ATTN_STAGES>(q, o, batch, seq, heads, flags, nullptr, 0, s);
    } else {
      if (v == 2) launch_attn<false, 4, 2, 2>(q, o, batch, seq, heads, flags, mx, ld_mx, s);
      else if (v == 3) launch_attn<false, 2, 4, ATTN_STAGES, 1>(q, o, batch, seq, heads, flags, mx, ld_mx, s);
      else launch_attn<false, 2, 4, ATTN_STAGES>(q, o, batch, seq, heads, flags, mx, ld_mx, s);
    }
  } else {
    dim3 grid(ceil_div(seq, 128), batch * heads);
    attn_f32_kernel<<<grid, 256, 0, s>>>((const float*)qkv, (float*)out, seq, heads, flags & AACLIP_ATTN_CAUSAL);
  }
  AACLIP_CHECK_LAUNCH();
  return AACLIP_OK;
}

AACLIP_TRACE_SETTER(trace_set_attention)
