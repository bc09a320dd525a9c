/*
 * aaclip.h — C ABI of libaaclip_hip.so, the MI355X (gfx950) kernels behind
 * AA-CLIP's anomaly-map inference path.
 *
 * Conventions (every entry point):
 *   - extern "C", stateless, re-entrant; returns 0 (AACLIP_OK) or an error
 *     code (AACLIP_ERR_ARG for a rejected argument, AACLIP_ERR_LAUNCH + hipError_t
 *     when the launch itself failed).
 *   - All tensor arguments are caller-owned DEVICE pointers (the caller's
 *     allocator owns them; nothing here allocates, frees or synchronises, so every
 *     call can be captured into a hipGraph). Row-major, leading dimensions in
 *     ELEMENTS. `stream` is a hipStream_t passed as void*.
 *   - dtype enums: AACLIP_F32 = 0, AACLIP_BF16 = 1, AACLIP_FP8 = 2, AACLIP_F16 = 3.
 *     bf16 / fp16 are stored as uint16.
 *
 * The reference (wei-paul/AA-CLIP) has no native code: each entry point below
 * replaces the PyTorch/kornia call sites cited next to it
 * (paths relative to the reference root). The binding a maintainer adds on the
 * reference side is the ctypes stub shown in INTEGRATION.md.
 */
#ifndef AACLIP_H_
#define AACLIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AACLIP_OK 0
#define AACLIP_ERR_ARG 1
#define AACLIP_ERR_LAUNCH 1000

#define AACLIP_F32 0
#define AACLIP_BF16 1
#define AACLIP_FP8 2   /* OCP e4m3 + e8m0 block scales (fp8 MX activations, config C5) */
#define AACLIP_F16 3   /* IEEE fp16: the parity-grade 16-bit mode (fp16 MFMA, same rate as bf16) */

/* GEMM epilogue flags (applied in this order) */
#define AACLIP_EPI_BIAS 1      /* + bias[n] (fp32)                          */
#define AACLIP_EPI_GELU 2      /* exact erf GELU (nn.GELU)                  */
#define AACLIP_EPI_LEAKY 4     /* LeakyReLU(0.01) (nn.LeakyReLU)            */
#define AACLIP_EPI_RESID 8     /* + residual[row, n] (fp32; may alias C)    */
#define AACLIP_EPI_AUX_BF16 16 /* also store a 16-bit copy of the result: fp16 when
                                  in_dtype is AACLIP_F16, bf16 otherwise      */
#define AACLIP_EPI_QGELU 32    /* QuickGELU v * sigmoid(1.702 v), applied where GELU
                                  is (reference model/transformer.py:46-49; the
                                  towers built with quick_gelu=True, model.py:84,129);
                                  exclusive with AACLIP_EPI_GELU               */

/* ABI version (bumped on any signature change; 2 = MX fp8 LayerNorm outputs, 3 = fp16 dtype,
 * aaclip_patch_logits, any-size blur_upsample; 6 = round 5: the rejected A/B entry points
 * removed, aaclip_trace_buffer added) and the target. */
int aaclip_abi_version(void);
const char* aaclip_arch(void);

/*
 * Diagnostic step timeline (trace builds only: `make trace` -> libaaclip_hip_trace.so;
 * the product library returns AACLIP_ERR_ARG). Every wave of an instrumented kernel
 * appends one record of 8 uint32 {t0 lo, t0 hi, t1 lo, t1 hi, tag, HW_ID, word 6 = XCC_ID
 * (bits 0-3) | the wave's s_memtime shader-cycle delta capped at 2^28-1 (bits 4-31),
 * workgroup} to the slab of its CU: slot = XCC << 8 | SE << 5 | SH << 4 | CU (2048
 * slots), records [2048][capacity][8], counter [2048][16] uint32 (slot s counts at
 * counter[16 s]; zero it before a traced run); a slot's records past capacity are
 * dropped (its counter still counts them). t0 / t1 are s_memrealtime (100 MHz,
 * chip-wide). records = counter = NULL, capacity = 0 turns it off. Not a reference
 * interface: tools/timeline.py reads it to measure the gap share of a step.
 */
int aaclip_trace_buffer(void* records, void* counter, unsigned capacity);

/*
 * C[M,N] = epilogue(A[M,K] . W[N,K]^T)        (nn.Linear / conv-as-GEMM)
 * Replaces: every addmm/mm of the path — MHA in_proj / out_proj
 * (model/transformer.py:200 via torch F.multi_head_attention_forward), MLP
 * c_fc + GELU and c_proj (transformer.py:211-219, :256-257), conv1 as GEMM
 * (transformer.py:359-365), adapter Linear+LeakyReLU (model/adapter_modules.py:6-26,
 * model/adapter.py:93), seg_proj/det_proj (adapter.py:107-110), text projection
 * (adapter.py:140, model/model.py:200).
 * in_dtype: A and W (bf16 -> bf16 MFMA, f16 -> f16 MFMA, f32 -> f32 MFMA).
 * out_dtype: C, either f32 or the 16-bit in_dtype.
 * K % 64 == 0 (bf16/f16) / K % 16 == 0 (f32); lda, ldw multiples of 8.
 * Output row remap when row_group > 0:
 *   out_row = (m / row_group) * row_group_out + row_offset + (m % row_group)
 * (used to write patch embeddings after each image's CLS slot). The same
 * remapped row indexes `residual` and `aux`.
 */
int aaclip_gemm(int in_dtype, int out_dtype, int M, int N, int K,
                const void* A, int64_t lda, const void* W, int64_t ldw,
                void* C, int64_t ldc, int epilogue, const float* bias,
                const float* residual, int64_t ldr, void* aux, int64_t ldaux,
                int row_group, int row_group_out, int row_offset, void* stream);

/*
 * aaclip_gemm with a FIXED ksplit-way split of K (the MLP c_proj, K = 4096:
 * model/transformer.py:216 / :257): every output tile is computed by `ksplit`
 * workgroups, part h over K-steps [h*nk/ksplit, (h+1)*nk/ksplit) (nk = K/64), each
 * storing its fp32 partial tile to `part`; the last part to arrive sums the partials
 * in index order ((P0 + P1) + P2 ...) and runs the epilogue. The split depends only on
 * K, so the bits do not depend on M, the batch composition or the tile family (every
 * family splits alike) -- but they differ from the unsplit aaclip_gemm's. Fills the
 * CUs that a launch with few K-long tiles leaves idle. 16-bit in_dtype only, no row
 * remap; 2 <= ksplit <= min(4, K/64). Workspace: `part` >= part_bytes and `counters`
 * (uint32, ZERO before first use; every launch leaves them zero) >= n_counters from
 * aaclip_gemm_ksplit_workspace. Concurrent launches need separate workspaces.
 */
int aaclip_gemm_ksplit_workspace(int M, int N, int K, int ksplit, size_t* part_bytes, int64_t* n_counters);
int aaclip_gemm_ksplit(int in_dtype, int out_dtype, int M, int N, int K, const void* A, int64_t lda,
                       const void* W, int64_t ldw, void* C, int64_t ldc, int epilogue, const float* bias,
                       const float* residual, int64_t ldr, void* aux, int64_t ldaux, int ksplit,
                       void* part, size_t part_bytes, void* counters, int64_t n_counters, void* stream);

/*
 * Level projection straight into anomaly-map partials (the predict path: the full
 * projected rows are never written):
 *   v = epilogue(A[M,K] . W[N,K]^T)   (epilogue 0 or AACLIP_EPI_LEAKY)
 *   part[m][g] = { sum ||v||^2, sum v.t0, sum v.t1, 0 } over columns 32g .. 32g+31
 * with t0/t1 = T[c % t_period][0/1] (T [t_period][2] fp32: normal, abnormal anchor),
 * as fp32 float4 per (row, 32-column group): part [M][ld_part >= N/8] floats.
 * Each group is summed in a fixed order that does not depend on the tile family, so
 * the partials of a row are the same whatever the batch. 16-bit in_dtype only;
 * K % 64 == 0, N % 256 == 0, t_period % 64 == 0.
 * Replaces: seg_proj / det_proj (adapter.py:107-110) + the row norms and anchor dots
 * of calculate_similarity_map (forward_utils.py:197-202) and of the image score
 * (test.py:83-84).
 */
int aaclip_gemm_scores(int in_dtype, int M, int N, int K, const void* A, int64_t lda,
                       const void* W, int64_t ldw, int epilogue, const float* T, int t_period,
                       float* part, int64_t ld_part, void* stream);

/*
 * fp8 GEMM (config C5: fp8 MFMA weights):
 *   C[M,N] = epilogue( a_scale[m] * w_scale[n] * (A8[M,K] . W8[N,K]^T) )
 * A8, W8: OCP e4m3 bytes (gfx950 FP8), per-row / per-output-channel fp32 scales
 * (dequantised value = byte * scale). The main loop runs the block-scaled
 * K=128 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4, unit block scales) at twice the
 * bf16 rate; the scales fold into the epilogue ahead of bias/activation/residual.
 * Same epilogue flags and row remap as aaclip_gemm. K % 128 == 0, N % 128 == 0,
 * lda/ldw multiples of 16 bytes, w_scale 16-B aligned.
 * Replaces: the same nn.Linear call sites as aaclip_gemm, at reduced precision.
 */
int aaclip_gemm_fp8(int out_dtype, int M, int N, int K, const void* A, int64_t lda,
                    const float* a_scale, const void* W, int64_t ldw, const float* w_scale,
                    void* C, int64_t ldc, int epilogue, const float* bias,
                    const float* residual, int64_t ldr, void* aux, int64_t ldaux,
                    int row_group, int row_group_out, int row_offset, void* stream);

/*
 * fp8 MX GEMM (config C5): C[M,N] = epilogue( w_scale[n] * sum_k A[m,k] 2^(a_mx[m,k/64]-127) W8[n,k] )
 * A: e4m3 with an e8m0 scale per (row, 64-K block), stored [K/128][ld_amx][2] bytes
 * (the two 64-blocks of one 128-K step adjacent); W8: e4m3 with fp32 per-output-
 * channel scales. The block scales are applied by the MFMA itself
 * (v_mfma_scale_f32_16x16x128_f8f6f4's per-lane B scale), staged through LDS.
 * out_dtype AACLIP_FP8 (only with bias+GELU, the c_fc -> c_proj hand-off): C is
 * written as e4m3 with its own e8m0 scale per (row, 64 columns) in c_mx
 * [N/128][ld_cmx][2], ready to be the A operand of the next MX GEMM.
 * K % 128 == 0, N % 256 == 0, ld_amx >= M and even (the scales move as dwords).
 */
int aaclip_gemm_fp8mx(int out_dtype, int M, int N, int K, const void* A, int64_t lda,
                      const void* a_mx, int64_t ld_amx, const void* W, int64_t ldw,
                      const float* w_scale, void* C, int64_t ldc, int epilogue,
                      const float* bias, const float* residual, int64_t ldr, void* aux,
                      int64_t ldaux, void* c_mx, int64_t ld_cmx, void* stream);

/*
 * MX fp8 quantisation: q[r,c] = e4m3(x[r,c] * 2^-e), e = the smallest exponent with
 * max|x[r, 64-block]| * 2^-e <= 448; sc[(c/128)*ld_sc + r][(c/64)%2] = e + 127.
 * x: fp32 or bf16 [rows, cols], cols % 128 == 0.
 */
int aaclip_quant_fp8_mx(int in_dtype, const void* x, int64_t ldx, void* q, int64_t ldq, void* sc,
                        int64_t ld_sc, int rows, int cols, void* stream);

/*
 * Per-row fp8 quantisation for aaclip_gemm_fp8's A operand:
 *   scale[r] = max_c |x[r,c]| / 448 (1 for an all-zero row); q[r,c] = e4m3(x[r,c] / scale[r])
 * (round-to-nearest-even, v_cvt_pk_fp8_f32). x: fp32 or bf16 [rows, cols], cols % 8 == 0.
 */
int aaclip_quant_fp8_rows(int in_dtype, const void* x, int64_t ldx, void* q, int64_t ldq,
                          float* scale, int rows, int cols, void* stream);

/*
 * Tuning hook: select the bf16 GEMM tile family for benchmarking. Bits 0-3:
 * 0 = default dispatch (N % 256 == 0: per shape, 256x256 8-phase ping-pong or
 * 320x256 LDS-DMA, whichever needs fewer tile rounds weighted by per-tile cost,
 * and 128x128 when that choice would fill under half the CUs; else 256x128),
 * 1 = 256x256 (N % 256 == 0), 2 = 256x128, 3 = 8-phase everywhere, 4 = 8-phase
 * for N >= 2048 only, 8 = 320x256 everywhere, 9 = 128x128 everywhere, 11 = 64x64
 * everywhere (N % 64 == 0; the default for single-image shapes); for the
 * fp8 MX GEMM: 0 = 8-phase ping-pong (default), 6 = the 256x256 LDS-DMA kernel; bits 4-7:
 * tile-order group height (0 = 4); bit 8: s_setprio around the MFMA cluster;
 * bit 9: diagnostic timing mode that skips the epilogue (outputs NOT written);
 * bit 10: diagnostic mode that runs the epilogue but skips its global stores;
 * bit 11: the 8-phase kernel writes 4 s_memtime stamps per wave (start, main loop
 * done, epilogue issued, stores complete) as uint64 to aaclip_gemm's aux pointer,
 * [tile][wave][4] (only for epilogues without AACLIP_EPI_AUX_BF16).
 * Process-global; not for production use.
 */
int aaclip_set_gemm_variant(int variant);

/*
 * Pin the tile family aaclip_gemm uses for one (in_dtype, M, N, K) (bf16 / f16):
 * 1 = 256x256, 2 = 256x128, 3 = 256x256 8-phase ping-pong, 8 = 320x256,
 * 9 = 128x128, 11 = 64x64, 0 = unpin (back to the
 * heuristic). Set by a measuring tuner at
 * engine setup (aaclip/ops.py tune_gemm); every family accumulates K in the same
 * order, so a pin changes speed, never bits. Process-global (mutex-guarded), host
 * only; unpinning removes the entry, so at most 256 shapes are pinned at once.
 */
int aaclip_gemm_pin(int in_dtype, int M, int N, int K, int family);

/*
 * Concurrent-chunk mode for the CALLING HOST THREAD (on = 1 / 0; *previous, if
 * non-null, receives the old state): while set, 16-bit GEMMs whose 256x256 tiles fill
 * at least one round of the CUs launch the 8-phase kernel (the other stream's chunk
 * fills the partial last round). Set by VisualEngine.predict around the enqueue of
 * concurrent image chunks (graph capture included: the choice is made at launch).
 * Pins and the variant hook take precedence. Same K order, so bits are unchanged.
 */
int aaclip_gemm_concurrent(int on, int* previous);

/* Name of the kernel aaclip_gemm launches for (in_dtype, M, N, K) with lda = ldw = K,
 * on the calling thread, under the current variant / pins / concurrent mode (the
 * dispatch's own decision). Host only, for reports. */
const char* aaclip_gemm_plan(int in_dtype, int M, int N, int K);

/*
 * Multi-head attention core, softmax(q k^T / sqrt(d)) v per head, flash-style
 * (scores never materialised). qkv: [batch*seq, 3*heads*head_dim] packed
 * [q|k|v] exactly as nn.MultiheadAttention's in_proj output; out:
 * [batch*seq, heads*head_dim] (heads merged, ready for out_proj).
 * flags: AACLIP_ATTN_CAUSAL adds the text tower's -inf upper triangle
 * (transformer.py:629-635); AACLIP_ATTN_Q_PRESCALED (bf16/fp8 only) says the q
 * columns already carry log2(e)/sqrt(head_dim) (folded into the Q projection
 * weights and bias, so the kernel's softmax runs in the log2 domain with no
 * per-score scaling); without it the kernel scales its Q fragments itself.
 * head_dim must be 64.
 * Replaces: torch F.multi_head_attention_forward's q-scale/bmm/softmax/bmm
 * (transformer.py:200, need_weights=True branch; the averaged weights are
 * discarded by the caller, model/adapter.py:91 — never computed here).
 */
#define AACLIP_ATTN_CAUSAL 1
#define AACLIP_ATTN_Q_PRESCALED 2
int aaclip_attention(int dtype, const void* qkv, void* out, int batch, int seq,
                     int heads, int head_dim, int flags, void* out_mx, int64_t ld_mx,
                     void* stream);
/* dtype AACLIP_FP8: bf16 qkv in, out written as MX e4m3 [batch*seq, heads*64] with one
 * e8m0 scale per (row, head) in out_mx [heads/2][ld_mx >= batch*seq][2] (the out-proj
 * A operand of aaclip_gemm_fp8mx, config C5); out_mx ignored otherwise. */

/* Tuning hook for the 16-bit attention kernel: 0 = default (3), 1 = 4 waves x 32 queries per
 * workgroup, 2 = 2 waves x 64 queries, 3 = 1 with each full key tile phase-split so one
 * query block's softmax runs beside the other's MFMAs. Process-global; for benchmarking. */
int aaclip_set_attn_variant(int variant);

/*
 * Patchify for conv1-as-GEMM: img [batch, channels, S, S] fp32 ->
 * cols [batch*(S/patch)^2, k_padded], column k = c*patch*patch + kh*patch + kw
 * (conv weight flattening order), zero for k >= channels*patch^2.
 * Replaces: the im2col inside conv1 (model/adapter.py:68).
 */
int aaclip_im2col(int out_dtype, const float* img, void* cols, int batch, int channels,
                  int img_size, int patch, int k_padded, void* stream);

/*
 * Visual token assembly + ln_pre + block-0 ln_1, one row per token:
 *   e = (t == 0 ? cls : x[row]) + pos[t];  x[row] = LN_pre(e);  h[row] = LN_1(x[row])
 * x: [batch*n_tok, width] fp32, rows t>=1 already hold conv1 patch embeddings.
 * Replaces: model/adapter.py:72-85 + the first ln_1 (transformer.py:254).
 */
int aaclip_embed_ln(int out_dtype, float* x, const float* cls, const float* pos,
                    const float* ln_pre_w, const float* ln_pre_b, const float* ln1_w,
                    const float* ln1_b, void* h, int batch, int n_tok, int width,
                    void* h_mx, int64_t ld_mx, void* stream);

/*
 * Row epilogue after a residual block (all optional stages, one pass):
 *   if u:   x = w*(u*||x||/||u||) + (1-w)*x              (adapter blend)
 *   if h:   h = LN(x; ln_w, ln_b)                         (next block's ln_1)
 *   if tap: tap[b*(n_tok-1)+t-1] = LN(x; post_w, post_b)  for t >= 1 (level tap + ln_post)
 * x: [rows, width] fp32, rows = batch*n_tok.
 * Replaces: model/adapter.py:92-101 (image) / :129-136 (text), the ln_1 of
 * transformer.py:254, and ln_post of level taps (adapter.py:100-105).
 */
int aaclip_block_tail(int out_dtype, float* x, const float* u, float adapt_weight,
                      const float* ln_w, const float* ln_b, void* h, const float* post_w,
                      const float* post_b, void* tap, int rows, int n_tok, int width,
                      void* h_mx, int64_t ld_mx, void* stream);

/* y = LN(x) rows (F.layer_norm, eps 1e-5, biased variance; transformer.py:37-43). */
int aaclip_layernorm(int out_dtype, const float* x, int64_t ldx, const float* w,
                     const float* b, void* y, int64_t ldy, int rows, int width,
                     void* y_mx, int64_t ld_mx, void* stream);

/*
 * (embed_ln, block_tail, layernorm) out_dtype AACLIP_FP8: the LayerNorm row (h / y)
 * is written as MX fp8 — e4m3 bytes [rows, width] plus an e8m0 scale per (row, 64
 * columns) in h_mx / y_mx [width/128][ld_mx >= rows][2], the A-operand format of
 * aaclip_gemm_fp8mx (config C5); level taps stay bf16. h_mx / ld_mx are ignored for
 * the other dtypes (pass NULL, 0).
 */

/*
 * Text embedding: x[s*ctx+t] = tok_emb[tokens[s,t]] + pos[t]; h = LN_1(x).
 * Replaces: model/adapter.py:118-123 / model/model.py:192-194 + first ln_1.
 */
int aaclip_text_embed_ln(int out_dtype, const int32_t* tokens, const float* tok_emb,
                         const float* pos, const float* ln1_w, const float* ln1_b, float* x,
                         void* h, int n_seq, int ctx, int width, void* stream);

/*
 * EOT gather + ln_final: y[s] = LN(x[s*ctx + argmax_t tokens[s,t]]).
 * Replaces: model/adapter.py:138-140 / model/model.py:199-200.
 */
int aaclip_eot_ln(int out_dtype, const float* x, const int32_t* tokens, const float* w,
                  const float* b, void* y, int n_seq, int ctx, int width, void* stream);

/*
 * Prompt-ensemble anchor: T[:, col] = normalize(mean_s normalize(emb[s])).
 * T: [dim, ncols] fp32. Replaces: forward_utils.py:155-159.
 */
int aaclip_anchor_reduce(const float* emb, int n, int dim, float* T, int col, int ncols,
                         void* stream);

/* y = x / max(||x||, 1e-12) per row (F.normalize, model/adapter.py:109). */
int aaclip_l2_normalize(int in_dtype, int out_dtype, const void* x, int64_t ldx, void* y,
                        int64_t ldy, int rows, int width, void* stream);

/*
 * Patch x anchor similarity for n_levels feature tensors (levels: HOST array
 * of n_levels device pointers, each [rows, channels], row stride ld):
 *   f_hat = normalize ? f/max(||f||,1e-12) : f;  A_c = 100 * f_hat . T[:, c]
 *   mode 0 (test): out[row] = sum_l (A_1 + 1 - A_0) / 2
 *   mode 1 (train, n_levels == 1): out[b, c, p] = A_c with b = row / group,
 *          p = row % group (channel-major [B, 2, group], ready for blur_upsample)
 * T: [channels, 2] fp32. group = patches per image (mode 1 only). Replaces: forward_utils.py:199-207 (+ the level sum of
 * test.py:93, moved before the blur/upsample: both are linear).
 */
int aaclip_patch_scores(int in_dtype, const void* const* levels, int n_levels, int64_t ld,
                        const float* T, int rows, int channels, int normalize, int mode,
                        int group, float* out, void* stream);

/*
 * Train-branch logits for any number of anchors: out[b, a, p] = 100 * f[b*group+p] . T[:, a]
 * (no normalisation; channel-major [B, n_anchor, group], the grid blur_upsample takes).
 * f: [rows, channels] fp32/bf16 (channels == 768), T: [channels, n_anchor] fp32,
 * 1 <= n_anchor <= 64. Replaces: forward_utils.py:199-202 for C != 2.
 */
int aaclip_patch_logits(int in_dtype, const void* f, int64_t ld, const float* T, int n_anchor,
                        int rows, int channels, int group, float* out, void* stream);

/*
 * Gaussian blur (kornia 0.6.9 gaussian_blur2d, reflect border, separable;
 * skipped when ksize == 0) then bilinear upsample with align_corners=True
 * (F.interpolate) to any out_size, optional softmax over the channel dim
 * (train branch, any 1 <= channels <= 8; channels == 1 leaves the logits as they are).
 * grid: [batch, channels, g, g] fp32 (g <= 64) -> out [batch, channels, S, S] fp32.
 * Replaces: forward_utils.py:208-215.
 */
int aaclip_blur_upsample(const float* grid, float* out, int batch, int channels, int g,
                         int out_size, int ksize, float sigma, int softmax, void* stream);

/*
 * Full test-branch anomaly map for one batch: patch_scores (mode 0) into the
 * caller's workspace grid_ws (>= batch*g*g fp32), then blur + upsample into
 * out [batch, S, S]. Replaces: test.py:86-93 + forward_utils.py:196-213.
 */
int aaclip_anomaly_map(int in_dtype, const void* const* levels, int n_levels, int64_t ld,
                       const float* T, int batch, int g, int channels, int normalize,
                       int out_size, int ksize, float sigma, float* grid_ws, float* out,
                       void* stream);

/*
 * The predict path's map + image score from aaclip_gemm_scores partials (the level
 * projections are never written as rows): part [batch*g*g][ld_part] fp32 holds, per
 * patch row, n_levels levels (+ the det projection when with_det) of 24 float4
 * partials {||v||^2, v.t0, v.t1, 0} (one per 32 columns of the 768). Stage 1 sums each
 * level's 24 partials in a fixed order, normalises and forms the level-summed test
 * score grid (as aaclip_patch_scores, normalize = 1) into grid_ws (>= batch*g*g) and,
 * with_det, normalize(d).t1 per row into det_ws (>= batch*g*g); stage 2 is
 * aaclip_blur_upsample (out [batch, S, S]) plus score[b] = (mean_p det_ws + 1) / 2.
 * Every argument is checked before the first launch.
 * Replaces: test.py:83-93 + forward_utils.py:196-213 after the projections.
 */
int aaclip_anomaly_map_partials(const float* part, int64_t ld_part, int n_levels, int with_det,
                                int batch, int g, int out_size, int ksize, float sigma,
                                float* grid_ws, float* det_ws, float* out, float* score,
                                void* stream);

/*
 * Image-level score: det[b] = mean_p normalize(det_raw[b*n_patch+p]) and
 * score[b] = (det[b] . T[:,1] + 1) / 2. partial: workspace
 * [batch, ceil(n_patch/16), channels] fp32 (fixed-order reduction, deterministic).
 * Replaces: model/adapter.py:110-111 + test.py:83-84.
 */
int aaclip_image_score(int in_dtype, const void* det_raw, int64_t ld, const float* T,
                       int batch, int n_patch, int channels, int normalize, float* partial,
                       float* det, float* score, void* stream);

/*
 * Device metrics_eval for one class (replaces forward_utils.py:233-280 + the
 * sklearn roc_auc_score / average_precision_score it calls): class-global
 * min-max normalisation of the maps (skipped when max == 1) and of the image
 * scores, image score fusion (0.5 * pixel max + 0.5 * score, or pixel max when
 * medical != 0), then exact tie-aware AUROC and AP for pixels and images.
 * pixel_preds [n_images, pix_per_image] fp32, pixel_label [same] uint8 (nonzero =
 * anomalous), image_preds [n_images] fp32, image_label [n_images] uint8.
 * out: device double[4] = pixel AUROC, pixel AP, image AUROC, image AP (unrounded;
 * the image pair is 0, 0 when all image labels are equal, as in the reference;
 * the pixel pair is NaN when all pixel labels are equal, where sklearn raises).
 * workspace: caller-owned device memory, 256-B aligned, of the size
 * aaclip_metrics_workspace reports (about 24 bytes per pixel). Deterministic.
 */
int aaclip_metrics_workspace(int64_t n_pixels, int n_images, size_t* bytes);
int aaclip_metrics_eval(const float* pixel_preds, const uint8_t* pixel_label, const float* image_preds,
                        const uint8_t* image_label, int n_images, int64_t pix_per_image, int medical,
                        void* workspace, size_t workspace_bytes, double* out, void* stream);

/*
 * Test-time preprocessing (replaces dataset/__init__.py:127-143
 * transform_x / transform_mask, i.e. Pillow's Image.resize as torchvision calls it,
 * then ToTensor + Normalize). Bit-exact with Pillow 8-bit resampling.
 *
 * Host-only plan builders (no device work): Pillow BICUBIC per-axis tables --
 * bounds [out_size, 2] int32 = (first source tap, tap count), coeffs
 * [out_size, ksize] int32 with 22 fraction bits; aaclip_bicubic_taps gives the
 * ksize to allocate. Nearest: index [out_size] int32 (Pillow's accumulated
 * in/out stepping).
 */
int aaclip_bicubic_taps(int in_size, int out_size, int* ksize);
int aaclip_bicubic_plan(int in_size, int out_size, int32_t* bounds, int32_t* coeffs, int ksize);
int aaclip_nearest_plan(int in_size, int out_size, int32_t* index);

/*
 * src: batch uint8 RGB images [in_h, in_w, 3] (row pitch / image stride in
 * bytes); plans (device copies) from aaclip_bicubic_plan(in_w, S) and (in_h, S).
 * out: fp32 [batch, 3, S, S] = (bicubic(src) / 255 - mean) / std; mean_std:
 * host float[6] (mean rgb, std rgb) or NULL for the CLIP constants.
 */
int aaclip_preprocess_images(const uint8_t* src, int64_t img_stride, int64_t row_pitch, int batch,
                             int in_h, int in_w, const int32_t* x_bounds, const int32_t* x_coeffs,
                             int kx, const int32_t* y_bounds, const int32_t* y_coeffs, int ky,
                             int out_size, const float* mean_std, float* out, void* workspace,
                             size_t workspace_bytes, void* stream);
/* workspace (optional, caller-owned device memory of aaclip_preprocess_workspace
 * bytes): enables the two-pass path (horizontal pass into a uint8 intermediate,
 * then the vertical pass); NULL = one tiled kernel with no intermediate. Same
 * output bits either way. */
int aaclip_preprocess_workspace(int batch, int in_h, int in_w, int out_size, size_t* bytes);

/*
 * src: batch uint8 L masks [in_h, in_w]; out fp32 [batch, 1, S, S] =
 * (nearest-resized mask != 0). Index tables from aaclip_nearest_plan (device copies).
 */
int aaclip_resize_masks_nearest(const uint8_t* src, int64_t img_stride, int64_t row_pitch, int batch,
                                int in_h, int in_w, const int32_t* x_index, const int32_t* y_index,
                                int out_size, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AACLIP_H_ */
