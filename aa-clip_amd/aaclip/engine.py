"""Device-side execution of AA-CLIP's inference path on libaaclip_hip.so.

VisualEngine = AdaptedCLIP.forward (reference model/adapter.py:67-112) +
the anomaly map / image score of test.py:80-93; TextEngine =
AdaptedCLIP.encode_text / CLIP.encode_text (adapter.py:114-145,
model/model.py:190-201) + the prompt-ensemble anchors (forward_utils.py:138-162).

Data layout in HBM (token-major "NLD", one row per token):
  x      fp32 [B*(P+1), 1024]   residual stream (kept fp32 across all 24 blocks)
  h      cdt  [B*(P+1), 1024]   LayerNorm output feeding the next GEMM
  qkv    cdt  [B*(P+1), 3072]   packed [q|k|v] (nn.MultiheadAttention in_proj order)
  attn   cdt  [B*(P+1), 1024]   merged heads
  fc     cdt  [B*(P+1), 4096]   GELU(c_fc)
  xb     bf16 [B*(P+1), 1024]   bf16 copy of x written by the c_proj epilogue (adapter input)
  u      fp32 [B*(P+1), 1024]   LeakyReLU(adapter(x))
  tap_l  cdt  [B*P, 1024]       ln_post(x[:, 1:]) at each level
  seg    fp32 [B*P, (L+1)*768]  seg_proj of level l in cols l*768.., det_proj in cols L*768.. (forward())
  spart  fp32 [B*P, (L+1)*96]   predict(), 16-bit modes: per (row, level, 32 columns) {|v|^2, v.t0, v.t1, 0}
cdt = compute dtype: bf16 (MFMA bf16, perf path) or fp32 (fp32 MFMA, parity mode).
Weights are packed once: nn.Linear [N,K] layout kept (the GEMM is A.W^T);
conv1 flattened to [1024, 640] (K padded 588 -> 640 with zeros).
"""
from __future__ import annotations

import os

import torch

from . import ops

WIDTH = 1024
HEADS = 16
Q_LOG2_SCALE = 0.125 * 1.4426950408889634  # 1/sqrt(64) * log2(e)
WS_KEEP = 16  # resident per-chunk workspaces (per image size)
MAX_STREAMS = 8  # concurrent image chunks per predict (<= WS_KEEP / 2: two chunk sizes per stream)
LAYERS = 24
PATCH = 14
EMBED = 768
KPATCH = 640  # 3*14*14 = 588 padded to a multiple of 64
DOMAIN_BLUR = {"Industrial": (7, 1.0), "Medical": (9, 1.5)}
# measure + pin the GEMM tile family per block-GEMM shape at workspace creation
# (ops.tune_gemm) when AACLIP_GEMM_TUNE=1. Off by default: in the two-stream C2 pipeline the
# isolated ranking does not carry over (tools/pin_search.py: the heuristic ~= the best pins)
TUNE = os.environ.get("AACLIP_GEMM_TUNE", "0") == "1"
CPROJ_KSPLIT = int(os.environ.get("AACLIP_CPROJ_KSPLIT", "0"))


def _on_device(fn):
    """Run an engine entry point with its device current (ops launch on the current
    device's stream; an engine on cuda:1 must not launch on cuda:0's)."""
    import functools

    @functools.wraps(fn)
    def wrap(self, *a, **k):
        with torch.cuda.device(self.device):
            return fn(self, *a, **k)
    return wrap


def _blur_for(domain: str):
    # forward_utils.py:205-206: Industrial k=7 sigma=1, anything else k=9 sigma=1.5
    return DOMAIN_BLUR["Industrial"] if domain == "Industrial" else DOMAIN_BLUR["Medical"]


def _proj_weight(ad: dict, prefix: str):
    if prefix + ".fc.0.weight" in ad:
        return ad[prefix + ".fc.0.weight"], True
    return ad[prefix + ".fc.weight"], False


FP8 = ops.FP8


def _quant_weight_fp8(w: torch.Tensor):
    """Per-output-channel e4m3 weights: scale[n] = max|W[n]|/448, W8 = RNE(W/scale)."""
    w = w.detach().float()
    s = (w.abs().amax(dim=1) / 448.0).clamp_min(1e-30)
    return (w / s[:, None]).to(FP8).contiguous(), s.contiguous()


class VisualEngine:
    def __init__(self, vparams: dict, adapter: dict, *, levels=(6, 12, 18, 24), image_adapt_until=6,
                 image_adapt_weight=0.1, dtype=torch.bfloat16, fold_q_scale=True, fp8_scope="mlp",
                 quick_gelu=False):
        """dtype: bfloat16 (perf path), float16 (parity-grade 16-bit path: fp16 MFMA at the
        bf16 rate with 8x finer operand rounding; the weights the OpenAI loader produces
        are fp16-exact, reference model/model.py:366), float32 (fp32-MFMA parity mode) or
        float8_e4m3fn (config C5:
        block GEMMs on e4m3 weights (per-output-channel scales) and MX e4m3 activations
        (e8m0 scale per 64 values, applied by the K=128 block-scaled MFMA), every input
        written in that format by its producer (LayerNorm / attention / c_fc epilogues).
        fp8_scope: "mlp" (default) = c_fc and c_proj in fp8, QKV / attention / out-proj in
        bf16 -- measured at C5: map rel-L2 0.9 % vs the fp32 mode at +24 % images/s over
        bf16; "all" = the four block GEMMs in fp8: +38 % but 8 % map rel-L2 (e4m3 q/k
        logits amplified by the softmax).
        quick_gelu: the MLP activation is QuickGELU (a tower built with quick_gelu=True,
        reference model/model.py:84) instead of nn.GELU; fused into the c_fc epilogue."""
        self.act = "quick" if quick_gelu else True
        if dtype not in (torch.bfloat16, torch.float16, torch.float32, FP8):
            raise ValueError("dtype must be bfloat16, float16, float32 or float8_e4m3fn")
        self.fp8 = dtype == FP8
        if fp8_scope not in ("all", "mlp"):
            raise ValueError("fp8_scope must be 'all' (QKV, out-proj, c_fc, c_proj) or 'mlp' (c_fc, c_proj)")
        self.fp8_mlp_only = self.fp8 and fp8_scope == "mlp"
        if self.fp8:
            dtype = torch.bfloat16
        self.dtype = dtype
        self.levels = list(levels)
        self.adapt_until = int(image_adapt_until)
        self.i_w = float(image_adapt_weight)
        if len(self.levels) > 8 or sorted(self.levels) != self.levels or self.levels[-1] > LAYERS:
            raise ValueError("levels must be sorted block indices in 1..24 (at most 8)")
        dev = vparams["visual.conv1.weight"].device
        if dev.type != "cuda":
            raise RuntimeError("VisualEngine needs device tensors (no CPU path)")
        self.device = dev
        f32 = lambda t: t.detach().to(dev, torch.float32).contiguous()  # noqa: E731
        cdt = lambda t: t.detach().to(dev, dtype).contiguous()  # noqa: E731
        w = vparams["visual.conv1.weight"].detach().reshape(WIDTH, -1)
        conv = torch.zeros(WIDTH, KPATCH, device=dev, dtype=torch.float32)
        conv[:, : w.shape[1]] = w
        self.conv = conv.to(dtype).contiguous()
        self.cls = f32(vparams["visual.class_embedding"])
        self.pos = f32(vparams["visual.positional_embedding"])
        self.ln_pre = (f32(vparams["visual.ln_pre.weight"]), f32(vparams["visual.ln_pre.bias"]))
        self.ln_post = (f32(vparams["visual.ln_post.weight"]), f32(vparams["visual.ln_post.bias"]))
        # bf16/fp8: the attention softmax runs in the log2 domain on q' = q * log2(e)/8;
        # the factor is folded into the Q rows of in_proj (weights and bias, in fp32
        # before the bf16/e4m3 rounding), so no per-score scaling remains in the kernel
        self.q_prescaled = dtype != torch.float32 and fold_q_scale  # False: the kernel scales Q at load (A/B)

        def qkv_param(t):
            t = t.detach().to(dev, torch.float32).clone()
            if self.q_prescaled:
                t[:WIDTH] *= Q_LOG2_SCALE
            return t.contiguous()

        self.blocks = []
        for i in range(LAYERS):
            p = f"visual.transformer.resblocks.{i}."
            self.blocks.append(dict(
                ln1=(f32(vparams[p + "ln_1.weight"]), f32(vparams[p + "ln_1.bias"])),
                ln2=(f32(vparams[p + "ln_2.weight"]), f32(vparams[p + "ln_2.bias"])),
                w_qkv=cdt(qkv_param(vparams[p + "attn.in_proj_weight"])),
                b_qkv=qkv_param(vparams[p + "attn.in_proj_bias"]),
                w_o=cdt(vparams[p + "attn.out_proj.weight"]), b_o=f32(vparams[p + "attn.out_proj.bias"]),
                w_fc=cdt(vparams[p + "mlp.c_fc.weight"]), b_fc=f32(vparams[p + "mlp.c_fc.bias"]),
                w_pr=cdt(vparams[p + "mlp.c_proj.weight"]), b_pr=f32(vparams[p + "mlp.c_proj.bias"]),
            ))
        if self.fp8:  # e4m3 copies of the block GEMM weights (the bf16 copies are dropped)
            for blk in self.blocks:
                for k in (("w_fc", "w_pr") if self.fp8_mlp_only else ("w_qkv", "w_o", "w_fc", "w_pr")):
                    blk[k] = _quant_weight_fp8(blk[k])
        self.w_adapt = [cdt(adapter[f"layer_adapters.{i}.fc.0.weight"]) for i in range(self.adapt_until)]
        self.w_seg, relus = [], []
        for i in range(len(self.levels)):
            wt, r = _proj_weight(adapter, f"seg_proj.{i}")
            self.w_seg.append(wt)
            relus.append(r)
        w_det, r_det = _proj_weight(adapter, "det_proj")
        if len(set(relus + [r_det])) != 1:
            raise ValueError("seg_proj/det_proj relu variants must agree")
        self.relu = r_det
        self.w_seg = [cdt(t) for t in self.w_seg[:-1]] + [cdt(torch.cat([self.w_seg[-1], w_det], 0))]
        self._ws = {}
        self.poison = False  # tests: fill new workspaces with NaN (read-before-write screen)
        # predict(): projections straight into map partials (aaclip_gemm_scores +
        # aaclip_anomaly_map_partials) instead of segbuf rows + a stream over them;
        # AACLIP_MAP_PARTIALS=0 restores the row path (A/B). Captured graphs are keyed on it
        # (predict_cached).
        self.map_partials = os.environ.get("AACLIP_MAP_PARTIALS", "1") == "1"
        # c_proj (K = 4096) as a fixed CPROJ_KSPLIT-way split-K GEMM in the 16-bit modes
        # (aaclip_gemm_ksplit): the same split at every batch size, so per-image bits stay
        # independent of the batch composition. 0 / 1 = unsplit.
        self.cproj_ksplit = CPROJ_KSPLIT if (self.dtype != torch.float32 and not self.fp8) else 0

    # ------------------------------------------------------------------ workspace
    def _workspace(self, B: int, S: int, slot: int = 0):
        key = (B, S, slot)
        if key in self._ws:
            self._ws[key] = self._ws.pop(key)  # most recently used last
            return self._ws[key]
        g = S // PATCH
        P = g * g
        n_tok = P + 1
        if self.pos.shape[0] != n_tok:
            raise ValueError(f"positional embedding has {self.pos.shape[0]} rows, image needs {n_tok} "
                             "(resize it at load time, reference model/model.py:395-426)")
        R = B * n_tok
        dev, cdt = self.device, self.dtype
        e = lambda *s, dt=cdt: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
        L = len(self.levels)
        ws = dict(
            g=g, P=P, n_tok=n_tok,
            cols=e(B * P, KPATCH), x=e(R, WIDTH, dt=torch.float32), h=e(R, WIDTH), qkv=e(R, 3 * WIDTH),
            attn=e(R, WIDTH), fc=e(R, 4 * WIDTH), u=e(R, WIDTH, dt=torch.float32),
            xb=e(R, WIDTH) if cdt != torch.float32 else None,  # 16-bit adapter input (bf16 / fp16)
            taps=[e(B * P, WIDTH) for _ in range(L)],
            # all level projections + det in one [B*P, (L+1)*768] fp32 buffer: level l at
            # columns l*768, det_proj at L*768 (one row stride for the map kernel).
            # fp32 even in bf16 mode: bf16 rounding of these final features moves a
            # patch cosine by ~1e-4 (x100 in the map) — the largest single bf16
            # term in the anomaly-map error budget, for ~15 us per batch of 32.
            segbuf=e(B * P, (L + 1) * EMBED, dt=torch.float32),
            # predict() in the 16-bit modes: the level / det projections leave as anomaly-map
            # partials (aaclip_gemm_scores: per row and 32 columns {||v||^2, v.t0, v.t1}),
            # 384 B per (row, level) instead of 3 KB rows; segbuf is then only forward()'s
            spart=e(B * P, (L + 1) * 4 * ops.SCORE_GROUPS, dt=torch.float32) if cdt != torch.float32 else None,
            detrow=e(B * P, dt=torch.float32),
            # fp8 mode (MX): e4m3 GEMM inputs with e8m0 scales per (row, 64 columns):
            # a8/asc for the 1024-wide inputs (quantised from bf16), f8/fsc for the
            # 4096-wide GELU output (written in fp8 by the c_fc epilogue itself)
            a8=e(R, WIDTH, dt=FP8) if self.fp8 else None,
            asc=ops.mx_scales(R, WIDTH, dev) if self.fp8 else None,
            f8=e(R, 4 * WIDTH, dt=FP8) if self.fp8 else None,
            fsc=ops.mx_scales(R, 4 * WIDTH, dev) if self.fp8 else None,
            # split-K c_proj: fp32 partial tiles + arrival counters (zeroed once; launches leave them zero)
            kws=(ops.ksplit_workspace(R, WIDTH, 4 * WIDTH, self.cproj_ksplit, dev) if self.cproj_ksplit > 1
                 else None),
            grid=e(B * P, dt=torch.float32), partial=e(B * ((P + 15) // 16) * EMBED, dt=torch.float32),
            det=e(B, EMBED, dt=torch.float32), score=e(B, dt=torch.float32),
            map=e(B, S, S, dt=torch.float32),
        )
        # keep the workspaces of the current image size, at most WS_KEEP of them (least
        # recently used dropped first): uneven chunks (e.g. 16 + 17 images) use one per
        # chunk and must not evict each other. A captured graph keeps its own references
        # (graphed_predict), so dropping an entry here never frees memory a graph replays.
        def size_of(k):  # (B, S, slot) workspaces, ("out", B, S) chunked-output buffers
            return k[2] if k[0] == "out" else k[1]

        drop = [k for k in self._ws if size_of(k) != S]
        chunk_keys = [k for k in self._ws if k[0] != "out" and size_of(k) == S]
        drop += chunk_keys[:max(0, len(chunk_keys) - (WS_KEEP - 1))]
        if drop and not torch.cuda.is_current_stream_capturing():
            # a dropped workspace may have been written by another stream than the one it
            # was allocated on; let that work finish before its memory returns to the pool
            torch.cuda.synchronize(self.device)
        for k in drop:
            del self._ws[k]
        self._ws[key] = ws
        if self.poison:  # test hook: every buffer starts as NaN / 0xFF, so a read-before-write shows
            for t in list(ws.values()) + ws["taps"]:
                if isinstance(t, torch.Tensor):
                    if t.is_floating_point() and t.dtype != FP8:
                        t.fill_(float("nan"))
                    else:
                        t.view(torch.uint8).fill_(0xFF)
        if TUNE and cdt != torch.float32:
            self._tune(ws)
        return ws

    def _tune(self, ws):
        """Pin the fastest tile family for each 16-bit block-GEMM shape of this
        workspace (ops.tune_gemm: measured once per shape and process, on the
        workspace's own buffers and epilogues; bit-neutral). Runs when a workspace
        is first created, i.e. outside any graph capture (graphed_predict warms up
        eagerly first)."""
        blk, X, H = self.blocks[0], ws["x"], ws["h"]
        scratch = torch.empty_like(X)
        if not (self.fp8 and not self.fp8_mlp_only):
            ops.tune_gemm(H, blk["w_qkv"], ws["qkv"], bias=blk["b_qkv"])
            ops.tune_gemm(ws["attn"], blk["w_o"], scratch, bias=blk["b_o"], residual=scratch)
        if not self.fp8:
            ops.tune_gemm(H, blk["w_fc"], ws["fc"], bias=blk["b_fc"], gelu=self.act)
            ops.tune_gemm(ws["fc"], blk["w_pr"], scratch, bias=blk["b_pr"], residual=scratch, aux=ws["xb"])
        if self.adapt_until > 0:
            ops.tune_gemm(ws["xb"], self.w_adapt[0], ws["u"], leaky=True)
        del scratch

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    @_on_device
    def forward_raw(self, x: torch.Tensor, slot: int = 0, T: torch.Tensor | None = None):
        """Run the visual tower; returns (seg_raw list of [B*P, 768] views,
        det_raw [B*P, 768] view, workspace). Rows are unnormalised projections.
        With T (predict, 16-bit modes) the projections are written as anomaly-map
        partials against T into ws["spart"] instead, and (None, None, ws) is returned."""
        if x.dim() != 4 or x.shape[1] != 3 or x.shape[2] != x.shape[3] or x.shape[2] % PATCH:
            raise ValueError("input must be [B, 3, S, S] with S a multiple of 14")
        x = x.to(self.device, torch.float32).contiguous()
        B, _, S, _ = x.shape
        ws = self._workspace(B, S, slot)
        P, n_tok = ws["P"], ws["n_tok"]
        X, H = ws["x"], ws["h"]
        ops.im2col(x, ws["cols"], PATCH)
        ops.gemm(ws["cols"], self.conv, X, row_group=P, row_group_out=n_tok, row_offset=1)
        lvl = {lv: j for j, lv in enumerate(self.levels)}
        last = self.levels[-1]
        if self.fp8 and not self.fp8_mlp_only:
            # every GEMM input is MX e4m3, written directly by its producer: the LayerNorm
            # kernels, the attention epilogue and the c_fc epilogue (no quantisation pass)
            a8, asc, f8, fsc = ws["a8"], ws["asc"], ws["f8"], ws["fsc"]
            Hq, Hsc = a8, asc
            ops.embed_ln(X, self.cls, self.pos, self.ln_pre, self.blocks[0]["ln1"], a8, B, n_tok, h_sc=asc)

            def qkv(blk):
                ops.gemm_fp8mx(a8, asc, blk["w_qkv"][0], blk["w_qkv"][1], ws["qkv"], bias=blk["b_qkv"])

            def attend():  # attention epilogue writes the out-proj input as MX e4m3
                ops.attention(ws["qkv"], a8, B, n_tok, HEADS, out_sc=asc, q_prescaled=self.q_prescaled)

            def out_proj(blk):
                ops.gemm_fp8mx(a8, asc, blk["w_o"][0], blk["w_o"][1], X, bias=blk["b_o"], residual=X)

            def mlp(blk, aux):  # c_fc writes e4m3 + block scales that c_proj consumes directly
                ops.layernorm(X, blk["ln2"][0], blk["ln2"][1], a8, y_sc=asc)
                ops.gemm_fp8mx(a8, asc, blk["w_fc"][0], blk["w_fc"][1], f8, out_sc=fsc, bias=blk["b_fc"], gelu=self.act)
                ops.gemm_fp8mx(f8, fsc, blk["w_pr"][0], blk["w_pr"][1], X, bias=blk["b_pr"], residual=X, aux=aux)
        else:
            Hq, Hsc = H, None
            ops.embed_ln(X, self.cls, self.pos, self.ln_pre, self.blocks[0]["ln1"], H, B, n_tok)

            def qkv(blk):
                ops.gemm(H, blk["w_qkv"], ws["qkv"], bias=blk["b_qkv"])

            def attend():
                ops.attention(ws["qkv"], ws["attn"], B, n_tok, HEADS, q_prescaled=self.q_prescaled)

            def out_proj(blk):
                ops.gemm(ws["attn"], blk["w_o"], X, bias=blk["b_o"], residual=X)

            def ln2(blk, y, y_sc=None):
                ops.layernorm(X, blk["ln2"][0], blk["ln2"][1], y, y_sc=y_sc)

            def mlp(blk, aux):
                if self.fp8_mlp_only:  # ln_2 -> MX e4m3 -> c_fc (fp8, GELU, MX out) -> c_proj (fp8)
                    a8, asc, f8, fsc = ws["a8"], ws["asc"], ws["f8"], ws["fsc"]
                    ln2(blk, a8, y_sc=asc)
                    ops.gemm_fp8mx(a8, asc, blk["w_fc"][0], blk["w_fc"][1], f8, out_sc=fsc, bias=blk["b_fc"],
                                   gelu=self.act)
                    ops.gemm_fp8mx(f8, fsc, blk["w_pr"][0], blk["w_pr"][1], X, bias=blk["b_pr"], residual=X,
                                   aux=aux)
                    return
                ln2(blk, H)
                ops.gemm(H, blk["w_fc"], ws["fc"], bias=blk["b_fc"], gelu=self.act)
                ops.gemm(ws["fc"], blk["w_pr"], X, bias=blk["b_pr"], residual=X, aux=aux, ksplit=self.cproj_ksplit,
                         ksplit_ws=ws["kws"])
        for i in range(last):
            blk = self.blocks[i]
            qkv(blk)
            attend()
            out_proj(blk)
            adapt = i < self.adapt_until
            mlp(blk, ws["xb"] if (adapt and ws["xb"] is not None) else None)
            tap = ws["taps"][lvl[i + 1]] if (i + 1) in lvl else None
            nxt = self.blocks[i + 1]["ln1"] if i + 1 < last else None
            u = None
            if adapt:
                ops.gemm(ws["xb"] if ws["xb"] is not None else X, self.w_adapt[i], ws["u"], leaky=True)
                u = ws["u"]
            if u is not None or nxt is not None or tap is not None:
                ops.block_tail(X, n_tok, u=u, adapt_weight=self.i_w, ln=nxt, h=Hq if nxt else None,
                               post=self.ln_post, tap=tap, h_sc=Hsc)
        L = len(self.levels)
        if T is not None and ws["spart"] is not None:
            sp = ws["spart"]
            G = 4 * ops.SCORE_GROUPS
            for j in range(L):
                ncol = self.w_seg[j].shape[0]
                ops.gemm_scores(ws["taps"][j], self.w_seg[j], T, sp[:, j * G:j * G + ncol // 8], leaky=self.relu)
            return None, None, ws
        sb = ws["segbuf"]
        for j in range(L):
            ncol = self.w_seg[j].shape[0]
            ops.gemm(ws["taps"][j], self.w_seg[j], sb[:, j * EMBED:j * EMBED + ncol], leaky=self.relu)
        seg = [sb[:, j * EMBED:(j + 1) * EMBED] for j in range(L)]
        det = sb[:, L * EMBED:]
        return seg, det, ws

    @staticmethod
    def max_chunk(img_size: int) -> int:
        """Most images one forward_raw may take: the attention kernel addresses a
        chunk's packed qkv through one buffer descriptor (< 2^31 bytes), i.e.
        B * n_tok * 3 * 1024 * 2 B (606 images at 336 px, 254 at 518). Larger
        batches are split into chunks of at most this many images."""
        n_tok = (img_size // PATCH) ** 2 + 1
        return max(1, ((1 << 31) - 1) // (n_tok * 3 * WIDTH * 2))

    @torch.no_grad()
    @_on_device
    def forward(self, x: torch.Tensor):
        """AdaptedCLIP.forward contract: (list[L] of [B,P,768] unit rows, det [B,768]) fp32
        (fresh tensors; batches above max_chunk run as consecutive chunks)."""
        B, S = x.shape[0], x.shape[-1]
        mc = self.max_chunk(S)
        out, det = None, None
        for b0 in range(0, B, mc):
            b1 = min(B, b0 + mc)
            seg_raw, det_raw, ws = self.forward_raw(x[b0:b1])
            P = ws["P"]
            if out is None:
                out = [torch.empty(B * P, EMBED, device=self.device, dtype=torch.float32) for _ in seg_raw]
                det = torch.empty(B, EMBED, device=self.device, dtype=torch.float32)
            for s_, y in zip(seg_raw, out):
                ops.l2_normalize(s_, y[b0 * P:b1 * P])
            ops.image_score(det_raw, b1 - b0, P, ws["partial"], det=det[b0:b1])
        P = out[0].shape[0] // B
        return [y.view(B, P, EMBED) for y in out], det

    def _tail(self, seg_raw, det_raw, ws, T, out_map, out_score, k, s):
        """Anomaly map + image score of one chunk from its projections: from the GEMM-emitted
        partials (predict, 16-bit modes), else two passes over segbuf (the level features,
        then the det rows). One-pass and one-launch forms measured slower (round 3) and were
        removed in round 5."""
        if seg_raw is None:  # projections as partials (forward_raw with T)
            ops.anomaly_map_partials(ws["spart"], len(self.levels), out_map, ws["grid"], g=ws["g"], ksize=k, sigma=s,
                                     det_ws=ws["detrow"], score=out_score)
            return
        ops.anomaly_map(seg_raw, T, out_map, ws["grid"], g=ws["g"], ksize=k, sigma=s)
        ops.image_score(det_raw, out_map.shape[0], ws["P"], ws["partial"], det=ws["det"], T=T, score=out_score)

    def _chunk_streams(self, n: int):
        if len(getattr(self, "_streams", [])) < n:
            self._streams = [torch.cuda.Stream(device=self.device) for _ in range(n)]
        return self._streams[:n]

    @torch.no_grad()
    @_on_device
    def predict(self, x: torch.Tensor, T: torch.Tensor, domain: str = "Industrial", streams: int = 1,
                _slot0: int = 0):
        """Fused test path: (anomaly map [B,S,S] fp32, image score [B] fp32),
        = test.py:80-93 with the level sum ahead of blur+upsample.

        streams > 1 splits the batch into that many image chunks, each run on its
        own HIP stream with its own workspace: the GEMM tails of one chunk
        (tile counts that leave CUs idle in the last wave) are filled by another
        chunk's tiles. A tuple gives the chunk sizes explicitly (summing to B).
        Batches above max_chunk(S) are cut into more chunks, round-robin over the
        streams (chunks sharing a stream share its workspace, in stream order).
        The outputs are ENGINE-OWNED buffers, overwritten by the next predict of the
        same (B, S): clone them to keep them (test.py does)."""
        B, S = x.shape[0], x.shape[-1]
        T = T.to(self.device, torch.float32).contiguous()
        k, s = _blur_for(domain)
        mc = self.max_chunk(S)
        if isinstance(streams, (tuple, list)):
            sizes = [int(v) for v in streams if int(v) > 0]
            if sum(sizes) != B:
                raise ValueError(f"chunk sizes {tuple(streams)} do not sum to the batch {B}")
            if max(sizes) > mc:
                raise ValueError(f"chunk of {max(sizes)} images exceeds max_chunk({S}) = {mc}")
            if len(sizes) > MAX_STREAMS:
                raise ValueError(f"at most {MAX_STREAMS} explicit chunks")
            nstreams = len(sizes)
        else:
            nstreams = max(1, min(int(streams), B, MAX_STREAMS))
            nchunks = max(nstreams, -(-B // mc))
            sizes = [(B * (i + 1)) // nchunks - (B * i) // nchunks for i in range(nchunks)]
        bounds = [0]
        for v in sizes:
            bounds.append(bounds[-1] + v)
        if len(sizes) == 1:
            seg_raw, det_raw, ws = self.forward_raw(x, slot=_slot0, T=T if self.map_partials else None)
            self._tail(seg_raw, det_raw, ws, T, ws["map"], ws["score"], k, s)
            return ws["map"], ws["score"]
        key = ("out", B, S, _slot0)
        if key not in self._ws:
            self._ws[key] = (torch.empty(B, S, S, device=self.device), torch.empty(B, device=self.device))
        out_map, out_score = self._ws[key]
        x = x.to(self.device, torch.float32).contiguous()
        main = torch.cuda.current_stream(self.device)
        if len(getattr(self, "_events", [])) < nstreams + 1:
            self._events = [torch.cuda.Event() for _ in range(nstreams + 1)]
        ready, done = self._events[0], self._events[1:nstreams + 1]
        ready.record(main)
        sts = self._chunk_streams(nstreams)
        for st in sts:
            st.wait_event(ready)
        # every chunk's workspace exists (and, with AACLIP_GEMM_TUNE, is tuned) before any
        # chunk is enqueued: tuning never runs beside the other streams' kernels. Each is
        # allocated on the stream that uses it: the caching allocator orders a block's
        # reuse only on its allocation stream (allocated on the main stream and written
        # by a chunk stream, a workspace came back NaN after a long GPU test session:
        # tests/test_fp16_gpu.py::test_concurrent_chunk_pins in the full suite)
        for i in range(len(sizes)):
            with torch.cuda.stream(sts[i % nstreams]):
                self._workspace(sizes[i], S, _slot0 + i % nstreams)
        # concurrent chunks share the CUs: one chunk's partial last round of GEMM tiles is
        # filled by the other's work, so the 8-phase 256x256 tile (faster per FLOP) wins
        # even where its tile count rounds up worse than the 320-row tile's (c_fc at 16
        # images per chunk): whole two-stream C2 step 2240 -> 2295 images/s bf16 (2164 ->
        # 2220 fp16); a single stream keeps the heuristic (1895 vs 2050). Thread-local
        # (aaclip_gemm_concurrent), chosen at launch, so graph capture keeps it.
        # (holding chunk 1 back by a few block sub-ops, or its stream at a lower priority,
        # measured 0.3-3.5 % slower: the free-running chunks drift into a good pairing,
        # profiles/r04/chunk_stagger_ab.txt, stream_priority_ab.txt)
        with ops.concurrent_gemms(nstreams > 1 and self.dtype in (torch.bfloat16, torch.float16)):
            for i in range(len(sizes)):
                b0, b1 = bounds[i], bounds[i + 1]
                st = sts[i % nstreams]
                with torch.cuda.stream(st):
                    seg_raw, det_raw, ws = self.forward_raw(x[b0:b1], slot=_slot0 + i % nstreams,
                                                            T=T if self.map_partials else None)
                    self._tail(seg_raw, det_raw, ws, T, out_map[b0:b1], out_score[b0:b1], k, s)
        for st, ev in zip(sts, done):
            ev.record(st)
            main.wait_event(ev)
        return out_map, out_score

    GRAPH_CACHE = 4  # captured steps kept per engine (predict_cached), least recently used dropped

    def predict_cached(self, x: torch.Tensor, T: torch.Tensor, domain: str = "Industrial", streams=1):
        """predict() through a captured hipGraph once a (batch, size, domain, streams) shape
        repeats BACK TO BACK (the harness's full batches within a class, or one-batch
        classes of equal size): a shape runs eagerly until it follows a call of the same
        shape, then that call captures and later ones replay (inputs copied into the
        graph's static buffers). A class's tail batch is followed by another shape, so it
        never triggers a capture (no warm-up + capture + device sync for a shape that is
        not coming back) and never evicts a full-batch graph; eviction is least recently
        used. Same kernels, same bits (tests/test_e2e_gpu.py); the outputs are
        graph-owned buffers, overwritten by the next replay of that shape."""
        # every engine setting that changes what a capture records is part of the key
        key = (x.shape[0], x.shape[-1], domain, tuple(streams) if isinstance(streams, (tuple, list)) else streams,
               bool(self.map_partials))
        if not hasattr(self, "_graph_cache"):
            self._graph_cache, self._last_key = {}, None
        run = self._graph_cache.get(key)
        repeat, self._last_key = key == self._last_key, key
        if run is None:
            if not repeat or not x.is_cuda:
                return self.predict(x, T, domain, streams=streams)
            if len(self._graph_cache) >= self.GRAPH_CACHE:
                self._graph_cache.pop(next(iter(self._graph_cache)))  # the least recently used
            run = self.graphed_predict(x.shape[0], x.shape[-1], domain, streams=streams)
        self._graph_cache.pop(key, None)
        self._graph_cache[key] = run  # most recently used last
        return run(x, T.to(self.device, torch.float32))

    @torch.no_grad()
    @_on_device
    def graphed_predict(self, batch: int, img_size: int, domain: str = "Industrial", streams: int = 1):
        """Capture predict() for a fixed (batch, size, domain, streams) into one hipGraph
        (torch.cuda.CUDAGraph records the C-ABI launches on the capturing stream and the
        chunk streams' fork/join). Returns fn(x, T) -> (map, score) that copies the
        inputs into static device buffers and replays the graph: no per-kernel host
        launch cost (matters at small batch, e.g. config C1's bs=1). The graph runs in
        workspaces of its own (a private slot range), so eager predict() calls of the
        same shape never write into the buffers it replays into or returns."""
        self._graphs = getattr(self, "_graphs", 0) + 1
        slot0 = 1000 * self._graphs
        x_s = torch.zeros(batch, 3, img_size, img_size, device=self.device)
        T_s = torch.zeros(EMBED, 2, device=self.device)
        T_s[0, 0] = 1.0
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        before = set(self._ws)
        with torch.cuda.stream(side):  # warm-up: allocate workspaces, set kernel attributes
            self.predict(x_s, T_s, domain, streams=streams, _slot0=slot0)
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        mine = {k: v for k, v in self._ws.items() if k not in before}  # the graph's own workspaces
        graph = torch.cuda.CUDAGraph()
        # thread_local: only this thread's calls are checked against the capture. The harness
        # captures while its DataLoader's pin-memory thread keeps allocating pinned host
        # buffers and querying events; "global" mode would fail the capture (or that
        # thread) for calls that never touch the captured streams
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            out_map, out_score = self.predict(x_s, T_s, domain, streams=streams, _slot0=slot0)
        held = list(mine.values())  # kept alive by the graph even if the LRU drops their keys
        dev = self.device

        def run(x: torch.Tensor, T: torch.Tensor):
            with torch.cuda.device(dev):
                x_s.copy_(x, non_blocking=True)
                T_s.copy_(T, non_blocking=True)
                graph.replay()
            return out_map, out_score

        run.graph = graph
        run.workspaces = held
        run.slot0 = slot0  # the private workspace slots (tools / bench diagnostics re-capture on them)
        return run


class TextEngine:
    """12-block causal text tower; adapted (text_adapter) or plain CLIP projection."""

    def __init__(self, params: dict, text_adapter: dict | None, *, text_adapt_until=3, text_adapt_weight=0.1,
                 dtype=torch.float32, quick_gelu=False):
        self.act = "quick" if quick_gelu else True  # MLP activation (reference model.py:129)
        dev = params["token_embedding.weight"].device
        if dev.type != "cuda":
            raise RuntimeError("TextEngine needs device tensors (no CPU path)")
        self.device, self.dtype = dev, dtype
        f32 = lambda t: t.detach().to(dev, torch.float32).contiguous()  # noqa: E731
        cdt = lambda t: t.detach().to(dev, dtype).contiguous()  # noqa: E731
        self.width = params["ln_final.weight"].shape[0]
        self.heads = self.width // 64
        self.tok_emb = f32(params["token_embedding.weight"])
        self.pos = f32(params["positional_embedding"])
        self.ln_final = (f32(params["ln_final.weight"]), f32(params["ln_final.bias"]))
        nl = len({k.split(".")[2] for k in params if k.startswith("transformer.resblocks.")})
        self.blocks = []
        for i in range(nl):
            p = f"transformer.resblocks.{i}."
            self.blocks.append(dict(
                ln1=(f32(params[p + "ln_1.weight"]), f32(params[p + "ln_1.bias"])),
                ln2=(f32(params[p + "ln_2.weight"]), f32(params[p + "ln_2.bias"])),
                w_qkv=cdt(params[p + "attn.in_proj_weight"]), b_qkv=f32(params[p + "attn.in_proj_bias"]),
                w_o=cdt(params[p + "attn.out_proj.weight"]), b_o=f32(params[p + "attn.out_proj.bias"]),
                w_fc=cdt(params[p + "mlp.c_fc.weight"]), b_fc=f32(params[p + "mlp.c_fc.bias"]),
                w_pr=cdt(params[p + "mlp.c_proj.weight"]), b_pr=f32(params[p + "mlp.c_proj.bias"]),
            ))
        self.adapted = text_adapter is not None
        self.t_w = float(text_adapt_weight)
        if self.adapted:
            self.adapt_until = int(text_adapt_until)
            self.w_adapt = [cdt(text_adapter[f"{i}.fc.0.weight"]) for i in range(self.adapt_until)]
            self.w_out = cdt(text_adapter[f"{self.adapt_until}.fc.0.weight"])  # Linear + LeakyReLU
        else:
            self.adapt_until = 0
            self.w_out = cdt(params["text_projection"].t())  # x @ P == x . (P^T)^T

    @torch.no_grad()
    @_on_device
    def encode(self, tokens: torch.Tensor, truncate: bool = True) -> torch.Tensor:
        """[n, 77] token ids -> [n, embed] (adapted: LeakyReLU(x_eot W^T), else x_eot @ proj).
        truncate: the tower is causal, so the EOT row (argmax token id, model.py:198)
        depends only on the tokens up to it; the columns after the longest prompt's EOT
        are dropped (prompts here are <= 39 of 77 tokens: ~half the text FLOPs). Rows are
        independent in every kernel, so the result is bit-identical to the full 77."""
        n, ctx = tokens.shape
        if ctx != self.pos.shape[0]:
            raise ValueError("token context length mismatch")
        if truncate and n > 0:
            ctx = int(tokens.argmax(-1).max()) + 1
            tokens = tokens[:, :ctx]
        tokens = tokens.to(self.device, torch.int32).contiguous()
        R, W = n * ctx, self.width
        dev, cdt = self.device, self.dtype
        e = lambda *s, dt=cdt: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
        X, H = e(R, W, dt=torch.float32), e(R, W)
        qkv, att, fc, u = e(R, 3 * W), e(R, W), e(R, 4 * W), e(R, W, dt=torch.float32)
        xb = e(R, W) if cdt != torch.float32 else None
        ops.text_embed_ln(tokens, self.tok_emb, self.pos, self.blocks[0]["ln1"], X, H)
        nb = len(self.blocks)
        for i, blk in enumerate(self.blocks):
            ops.gemm(H, blk["w_qkv"], qkv, bias=blk["b_qkv"])
            ops.attention(qkv, att, n, ctx, self.heads, causal=True)
            ops.gemm(att, blk["w_o"], X, bias=blk["b_o"], residual=X)
            ops.layernorm(X, blk["ln2"][0], blk["ln2"][1], H)
            ops.gemm(H, blk["w_fc"], fc, bias=blk["b_fc"], gelu=self.act)
            adapt = i < self.adapt_until
            ops.gemm(fc, blk["w_pr"], X, bias=blk["b_pr"], residual=X, aux=xb if (adapt and xb is not None) else None)
            nxt = self.blocks[i + 1]["ln1"] if i + 1 < nb else None
            if adapt:
                ops.gemm(xb if xb is not None else X, self.w_adapt[i], u, leaky=True)
                ops.block_tail(X, ctx, u=u, adapt_weight=self.t_w, ln=nxt, h=H if nxt else None)
            elif nxt is not None:
                ops.layernorm(X, nxt[0], nxt[1], H)
        eot = e(n, W)
        ops.eot_ln(X, tokens, self.ln_final, eot)
        out = torch.empty(n, self.w_out.shape[0], device=dev, dtype=torch.float32)
        ops.gemm(eot, self.w_out, out, leaky=self.adapted)
        return out

    @torch.no_grad()
    @_on_device
    def class_anchor(self, tok_normal: torch.Tensor, tok_abnormal: torch.Tensor) -> torch.Tensor:
        """forward_utils.py:146-161 -> T [768, 2] (normal, abnormal)."""
        T = torch.empty(self.w_out.shape[0], 2, device=self.device, dtype=torch.float32)
        for col, tok in enumerate((tok_normal, tok_abnormal)):
            ops.anchor_reduce(self.encode(tok), T, col)
        return T
