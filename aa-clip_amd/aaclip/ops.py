"""Tensor-level wrappers over the C ABI (include/aaclip.h).

torch is plumbing here: device memory, the current HIP stream, dtype tags.
Every function validates shapes/dtypes on the host (a kernel is never launched
on operands whose shapes disagree with what its grid assumes) and launches one
HIP kernel on torch's current stream. There is no eager-PyTorch fallback.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import BF16, F16, F32, call

_DT = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16}


def dtag(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}; expected float32, bfloat16 or float16") from None


def torch_dtype(tag: int) -> torch.dtype:
    return {F32: torch.float32, BF16: torch.bfloat16, F16: torch.float16}[tag]


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _dev(*ts):
    """Every operand must be a device tensor on the CURRENT device: kernels launch on
    the current device's stream (and the C side keys its per-device caches on
    hipGetDevice), so a tensor on another GPU would be a wrong-device pointer. The
    engines enter `torch.cuda.device(their device)` around every launch sequence."""
    cur = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("aaclip ops need device (HIP) tensors; there is no CPU path")
        if cur is None:
            cur = torch.cuda.current_device()
        if t.device.index != cur:
            raise RuntimeError(f"aaclip op operand on {t.device} but the current device is cuda:{cur}; "
                               "wrap the call in torch.cuda.device(...)")


# In-step launch probe (measurement only; None in production): an object with
# begin(kind, name, flops, nbytes) -> token and end(token), called around every
# launch of the ops below so a caller (bench.py) can put HIP timing events around
# each kernel inside a captured step. It never changes what is launched.
_probe = None


def set_probe(probe) -> None:
    global _probe
    _probe = probe


def _launch(kind: str, name, flops: float, nbytes: float, fn, *args) -> None:
    """call(fn, *args), bracketed by the probe when one is set."""
    if _probe is None:
        call(fn, *args)
        return
    tok = _probe.begin(kind, name() if callable(name) else name, flops, nbytes)
    call(fn, *args)
    _probe.end(tok)


def _rowmajor(t: torch.Tensor, name: str):
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name} must be a 2-D tensor with unit column stride")


# ------------------------------------------------------------------------ GEMM
def ksplit_workspace(M: int, N: int, K: int, ksplit: int, device) -> tuple:
    """(partials uint8 buffer, zeroed uint32 arrival counters) for aaclip_gemm_ksplit on
    (M, N, K) split `ksplit` ways. One workspace per concurrently running launch."""
    nbytes, ncnt = ctypes.c_size_t(0), ctypes.c_int64(0)
    call("aaclip_gemm_ksplit_workspace", M, N, K, ksplit, ctypes.byref(nbytes), ctypes.byref(ncnt))
    part = torch.empty(int(nbytes.value), device=device, dtype=torch.uint8)
    cnt = torch.zeros(int(ncnt.value), device=device, dtype=torch.int32)
    return part, cnt


def gemm(a: torch.Tensor, w: torch.Tensor, out: torch.Tensor, *, bias=None, gelu=False, leaky=False,
         residual=None, aux=None, row_group=0, row_group_out=0, row_offset=0, ksplit=0,
         ksplit_ws=None) -> torch.Tensor:
    """out = epilogue(a @ w.T) — a [M,K], w [N,K] (same dtype), out [M', N].
    gelu: True = exact erf GELU (nn.GELU), "quick" = QuickGELU x*sigmoid(1.702x)
    (reference model/transformer.py:46-49).
    ksplit >= 2 (16-bit operands, no row remap): aaclip_gemm_ksplit, K cut into that many
    fixed parts summed in index order, on ksplit_ws = ksplit_workspace(M, N, K, ksplit)."""
    _dev(a, w, out, bias, residual, aux)
    if ksplit and ksplit > 1:
        return _gemm_ksplit(a, w, out, bias, gelu, leaky, residual, aux, row_group, ksplit, ksplit_ws)
    for t, n in ((a, "a"), (w, "w"), (out, "out")):
        _rowmajor(t, n)
    if a.dtype != w.dtype:
        raise TypeError("gemm operands must share a dtype")
    if out.dtype not in (torch.float32, a.dtype) and not (a.dtype == torch.float32 and out.dtype == torch.bfloat16):
        raise TypeError("gemm output must be float32 or the operands' 16-bit dtype")
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K or out.shape[1] != N:
        raise ValueError(f"gemm shape mismatch a{tuple(a.shape)} w{tuple(w.shape)} out{tuple(out.shape)}")
    rows_out = M if row_group == 0 else ((M - 1) // row_group) * row_group_out + row_offset + (M - 1) % row_group + 1
    if out.shape[0] < rows_out or (row_group and M % row_group):
        raise ValueError("gemm output rows too small for the row remap")
    epi, ldr, ldaux = _epilogue_flags(N, rows_out, bias, gelu, leaky, residual, aux,
                                      aux_dtype=torch.float16 if a.dtype == torch.float16 else torch.bfloat16)
    kind = f"gemm N{N} K{K}" + (" leaky" if leaky else "") + (" qgelu" if gelu == "quick" else " gelu" if gelu else "") + (" resid" if residual is not None else "")
    nbytes = (M * K + N * K) * a.element_size() + rows_out * N * out.element_size() * (2 if residual is not None else 1)
    _launch(kind, lambda: gemm_plan(dtag(a), M, N, K) if a.dtype != torch.float32 else "gemm_f32_kernel",
            2.0 * M * N * K, nbytes, "aaclip_gemm", dtag(a), dtag(out), M, N, K, _ptr(a), a.stride(0), _ptr(w),
            w.stride(0), _ptr(out), out.stride(0), epi, _ptr(bias), _ptr(residual), ldr, _ptr(aux), ldaux,
            row_group, row_group_out, row_offset, _stream())
    return out


def _gemm_ksplit(a, w, out, bias, gelu, leaky, residual, aux, row_group, ksplit, ws):
    for t, n in ((a, "a"), (w, "w"), (out, "out")):
        _rowmajor(t, n)
    if a.dtype not in (torch.bfloat16, torch.float16) or w.dtype != a.dtype:
        raise TypeError("split-K gemm takes 16-bit operands of one dtype")
    if out.dtype not in (torch.float32, a.dtype):
        raise TypeError("gemm output must be float32 or the operands' 16-bit dtype")
    if row_group:
        raise ValueError("split-K gemm has no row remap")
    if ws is None:
        raise ValueError("split-K gemm needs its workspace (ops.ksplit_workspace)")
    part, cnt = ws
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K or out.shape[1] != N or out.shape[0] < M:
        raise ValueError(f"gemm shape mismatch a{tuple(a.shape)} w{tuple(w.shape)} out{tuple(out.shape)}")
    _dev(part, cnt)
    if part.dtype != torch.uint8 or cnt.dtype != torch.int32 or not (part.is_contiguous() and cnt.is_contiguous()):
        raise TypeError("split-K workspace: (uint8 partials, int32 counters), contiguous")
    epi, ldr, ldaux = _epilogue_flags(N, M, bias, gelu, leaky, residual, aux,
                                      aux_dtype=torch.float16 if a.dtype == torch.float16 else torch.bfloat16)
    kind = f"gemm N{N} K{K}" + (" leaky" if leaky else "") + (" qgelu" if gelu == "quick" else " gelu" if gelu else "") + (" resid" if residual is not None else "")
    nbytes = (M * K + N * K) * a.element_size() + M * N * out.element_size() * (2 if residual is not None else 1)
    _launch(kind, lambda: gemm_plan(dtag(a), M, N, K) + f" ksplit{ksplit}", 2.0 * M * N * K, nbytes,
            "aaclip_gemm_ksplit", dtag(a), dtag(out), M, N, K, _ptr(a), a.stride(0), _ptr(w), w.stride(0),
            _ptr(out), out.stride(0), epi, _ptr(bias), _ptr(residual), ldr, _ptr(aux), ldaux, ksplit,
            _ptr(part), part.numel(), _ptr(cnt), cnt.numel(), _stream())
    return out


# tile families aaclip_gemm_pin accepts (include/aaclip.h): 8-phase 256x256, 320x256,
# 256x256, 128x128, 256x128, 64x64 (the two-workgroup family 10 was removed in round 5)
GEMM_FAMILIES = (3, 8, 1, 9, 2, 11)
_tuned = {}


def _family_applies(fam: int, N: int, K: int) -> bool:
    """The shapes aaclip_gemm_pin / choose16 honour a family on (else it falls back)."""
    if fam in (1, 3, 8, 9):
        return N % 256 == 0
    if fam == 11:
        return N % 64 == 0
    return True  # 0 (the unpinned per-shape heuristic) and 2


def pin_gemm(dtype: int, M: int, N: int, K: int, family: int) -> None:
    """aaclip_gemm_pin: launch tile family `family` (GEMM_FAMILIES; 0 = back to the
    per-shape heuristic) for every 16-bit GEMM of this (dtype tag, M, N, K)."""
    call("aaclip_gemm_pin", dtype, M, N, K, family)


class concurrent_gemms:
    """Context manager: aaclip_gemm_concurrent for the calling thread while image chunks
    are enqueued on concurrent streams (block-GEMM shapes that fill a round of the CUs
    take the 8-phase kernel; bit-identical). Restores the previous state on exit."""

    def __init__(self, on: bool = True):
        self.on = int(bool(on))
        self.prev = ctypes.c_int(0)

    def __enter__(self):
        call("aaclip_gemm_concurrent", self.on, ctypes.byref(self.prev))
        return self

    def __exit__(self, *exc):
        call("aaclip_gemm_concurrent", self.prev.value, None)
        return False


def gemm_plan(tag: int, M: int, N: int, K: int) -> str:
    """Kernel name aaclip_gemm launches for this shape on this thread (reports)."""
    return _lib.lib().aaclip_gemm_plan(tag, M, N, K).decode()


def tune_gemm(a: torch.Tensor, w: torch.Tensor, out: torch.Tensor, reps: int = 3, **epilogue) -> int:
    """Measure every tile family on these operands with this epilogue (HIP events on the
    current stream) and pin the fastest for the shape (aaclip_gemm_pin). The families
    accumulate K in the same order, so the pin changes speed, never bits. Host-side
    setup only (it synchronises): never call it while a hipGraph is being captured.
    Returns the pinned family; shapes already tuned in this process are skipped."""
    if a.dtype not in (torch.bfloat16, torch.float16):
        return 0
    M, K = a.shape
    N = w.shape[0]
    key = (dtag(a), M, N, K)
    if key in _tuned:
        return _tuned[key]
    st = torch.cuda.current_stream()
    best, best_t = 0, float("inf")
    try:
        # family 0 = unpinned: the heuristic's own choice (e.g. the 64x64 tiles it takes for
        # single-image shapes) is a candidate, so a pin is never slower than no pin
        for fam in (0,) + GEMM_FAMILIES:
            if not _family_applies(fam, N, K):
                continue
            call("aaclip_gemm_pin", key[0], M, N, K, fam)
            gemm(a, w, out, **epilogue)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                gemm(a, w, out, **epilogue)
            e1.record(st)
            e1.synchronize()
            t = e0.elapsed_time(e1)
            if t < best_t:
                best, best_t = fam, t
    finally:
        call("aaclip_gemm_pin", key[0], M, N, K, best)
    _tuned[key] = best
    return best


FP8 = torch.float8_e4m3fn  # OCP e4m3 (gfx950), one byte per element


def quant_fp8_rows(x: torch.Tensor, q: torch.Tensor, scale: torch.Tensor) -> None:
    """Per-row e4m3 quantisation: scale[r] = max|x[r]|/448, q = RNE(x/scale)."""
    _dev(x, q, scale)
    _rowmajor(x, "x")
    _rowmajor(q, "q")
    if q.dtype != FP8 or scale.dtype != torch.float32 or not scale.is_contiguous():
        raise TypeError("q must be float8_e4m3fn and scale contiguous fp32")
    rows, cols = x.shape
    if tuple(q.shape) != (rows, cols) or scale.numel() < rows:
        raise ValueError("quant_fp8_rows shape mismatch")
    call("aaclip_quant_fp8_rows", dtag(x), _ptr(x), x.stride(0), _ptr(q), q.stride(0), _ptr(scale), rows, cols,
         _stream())


def gemm_fp8(a: torch.Tensor, a_scale: torch.Tensor, w: torch.Tensor, w_scale: torch.Tensor, out: torch.Tensor, *,
             bias=None, gelu=False, leaky=False, residual=None, aux=None, row_group=0, row_group_out=0,
             row_offset=0) -> torch.Tensor:
    """out = epilogue(a_scale[:,None] * w_scale[None,:] * (a @ w.T)) with e4m3 a [M,K], w [N,K]."""
    _dev(a, a_scale, w, w_scale, out, bias, residual, aux)
    for t, n in ((a, "a"), (w, "w"), (out, "out")):
        _rowmajor(t, n)
    if a.dtype != FP8 or w.dtype != FP8:
        raise TypeError("gemm_fp8 operands must be float8_e4m3fn")
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K or out.shape[1] != N or a_scale.numel() < M or w_scale.numel() != N:
        raise ValueError(f"gemm_fp8 shape mismatch a{tuple(a.shape)} w{tuple(w.shape)} out{tuple(out.shape)}")
    if a_scale.dtype != torch.float32 or w_scale.dtype != torch.float32:
        raise TypeError("fp8 scales must be fp32")
    rows_out = M if row_group == 0 else ((M - 1) // row_group) * row_group_out + row_offset + (M - 1) % row_group + 1
    if out.shape[0] < rows_out or (row_group and M % row_group):
        raise ValueError("gemm output rows too small for the row remap")
    epi, ldr, ldaux = _epilogue_flags(N, rows_out, bias, gelu, leaky, residual, aux)
    call("aaclip_gemm_fp8", dtag(out), M, N, K, _ptr(a), a.stride(0), _ptr(a_scale), _ptr(w), w.stride(0),
         _ptr(w_scale), _ptr(out), out.stride(0), epi, _ptr(bias), _ptr(residual), ldr, _ptr(aux), ldaux,
         row_group, row_group_out, row_offset, _stream())
    return out


def mx_scales(rows: int, cols: int, device, ld: int = None) -> torch.Tensor:
    """e8m0 scale buffer of an MX fp8 tensor [rows, cols]: [cols/128, ld, 2] uint8
    (one byte per (row, 64-column block); the two blocks of a 128-K step adjacent).
    ld defaults to rows rounded up to even (the MX GEMM moves scales as dwords)."""
    return torch.empty(cols // 128, ld or (rows + 1) // 2 * 2, 2, device=device, dtype=torch.uint8)


def quant_fp8_mx(x: torch.Tensor, q: torch.Tensor, sc: torch.Tensor) -> None:
    """MX fp8: q = e4m3(x * 2^-e), e8m0 e per (row, 64-column block) into sc [cols/128, ld, 2]."""
    _dev(x, q, sc)
    _rowmajor(x, "x")
    _rowmajor(q, "q")
    rows, cols = x.shape
    if q.dtype != FP8 or sc.dtype != torch.uint8 or tuple(q.shape) != (rows, cols):
        raise TypeError("q must be float8_e4m3fn [rows, cols], sc uint8")
    if sc.dim() != 3 or sc.shape[0] != cols // 128 or sc.shape[1] < rows or sc.shape[2] != 2 or not sc.is_contiguous():
        raise ValueError("sc must be contiguous uint8 [cols/128, ld >= rows, 2]")
    call("aaclip_quant_fp8_mx", dtag(x), _ptr(x), x.stride(0), _ptr(q), q.stride(0), _ptr(sc), sc.shape[1],
         rows, cols, _stream())


def gemm_fp8mx(a: torch.Tensor, a_sc: torch.Tensor, w: torch.Tensor, w_scale: torch.Tensor, out: torch.Tensor, *,
               out_sc=None, bias=None, gelu=False, leaky=False, residual=None, aux=None) -> torch.Tensor:
    """out = epilogue(w_scale[None,:] * (MX-dequant(a) @ w.T)); a: e4m3 [M,K] with e8m0 block scales
    a_sc [K/128, ld, 2]; out fp32 / bf16, or e4m3 (then out_sc receives its MX scales)."""
    _dev(a, a_sc, w, w_scale, out, out_sc, bias, residual, aux)
    for t, n in ((a, "a"), (w, "w"), (out, "out")):
        _rowmajor(t, n)
    if a.dtype != FP8 or w.dtype != FP8:
        raise TypeError("gemm_fp8mx operands must be float8_e4m3fn")
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K or out.shape[1] != N or out.shape[0] < M or w_scale.numel() != N:
        raise ValueError(f"gemm_fp8mx shape mismatch a{tuple(a.shape)} w{tuple(w.shape)} out{tuple(out.shape)}")
    if a_sc.dtype != torch.uint8 or a_sc.dim() != 3 or a_sc.shape[0] != K // 128 or a_sc.shape[1] < M or \
            a_sc.shape[1] % 2:
        raise ValueError("a_sc must be uint8 [K/128, ld >= M (even), 2]")
    if out.dtype == FP8:
        if out_sc is None or out_sc.shape[0] != N // 128 or out_sc.shape[1] < M:
            raise ValueError("fp8 output needs out_sc uint8 [N/128, ld >= M, 2]")
        odt = _lib.FP8
    else:
        odt = dtag(out)
    epi, ldr, ldaux = _epilogue_flags(N, M, bias, gelu, leaky, residual, aux)
    kind = f"gemm8 N{N} K{K}" + (" gelu" if gelu else "") + (" resid" if residual is not None else "")
    nbytes = M * K + N * K + M * N * out.element_size() * (2 if residual is not None else 1)
    _launch(kind, "gemm_fp8mx_8ph_kernel", 2.0 * M * N * K, nbytes, "aaclip_gemm_fp8mx", odt, M, N, K, _ptr(a),
            a.stride(0), _ptr(a_sc), a_sc.shape[1], _ptr(w), w.stride(0), _ptr(w_scale), _ptr(out), out.stride(0),
            epi, _ptr(bias), _ptr(residual), ldr, _ptr(aux), ldaux, _ptr(out_sc),
            0 if out_sc is None else out_sc.shape[1], _stream())
    return out


def _epilogue_flags(N, rows_out, bias, gelu, leaky, residual, aux, aux_dtype=torch.bfloat16):
    epi = 0
    if bias is not None:
        if bias.dtype != torch.float32 or bias.numel() != N:
            raise ValueError("bias must be fp32 [N]")
        epi |= _lib.EPI_BIAS
    if gelu not in (False, True, "quick"):
        raise ValueError("gelu must be False, True (erf GELU, nn.GELU) or 'quick' (QuickGELU)")
    if gelu:
        epi |= _lib.EPI_QGELU if gelu == "quick" else _lib.EPI_GELU
    if leaky:
        epi |= _lib.EPI_LEAKY
    ldr = 0
    if residual is not None:
        _rowmajor(residual, "residual")
        if residual.dtype != torch.float32 or residual.shape[1] != N or residual.shape[0] < rows_out:
            raise ValueError("residual must be fp32 [rows, N]")
        epi |= _lib.EPI_RESID
        ldr = residual.stride(0)
    ldaux = 0
    if aux is not None:
        _rowmajor(aux, "aux")
        if aux.dtype != aux_dtype or aux.shape[1] != N or aux.shape[0] < rows_out:
            raise ValueError(f"aux must be {aux_dtype} [rows, N] (fp16 for fp16 operands, else bf16)")
        epi |= _lib.EPI_AUX_BF16
        ldaux = aux.stride(0)
    return epi, ldr, ldaux


# ------------------------------------------------------------------------ attention
def attention(qkv: torch.Tensor, out: torch.Tensor, batch: int, seq: int, heads: int,
              causal: bool = False, out_sc=None, q_prescaled: bool = False) -> torch.Tensor:
    """out = MHA core of packed qkv; out fp8 (e4m3) + out_sc = MX output (bf16 qkv only).
    q_prescaled: the q columns already carry log2(e)/sqrt(64) (bf16 / fp16 qkv only)."""
    _dev(qkv, out, out_sc)
    flags = (_lib.ATTN_CAUSAL if causal else 0) | (_lib.ATTN_Q_PRESCALED if q_prescaled else 0)
    if q_prescaled and qkv.dtype not in (torch.bfloat16, torch.float16):
        raise ValueError("q_prescaled needs bf16 or fp16 qkv")
    hd = 64
    if qkv.shape != (batch * seq, 3 * heads * hd) or out.shape != (batch * seq, heads * hd):
        raise ValueError("attention shape mismatch")
    if not (qkv.is_contiguous() and out.is_contiguous()):
        raise ValueError("attention tensors must be contiguous")
    if out.dtype == FP8:
        if qkv.dtype != torch.bfloat16 or out_sc is None or out_sc.dtype != torch.uint8 or \
                out_sc.shape[0] != heads // 2 or out_sc.shape[1] < batch * seq:
            raise ValueError("fp8 attention output needs bf16 qkv and MX scales [heads/2, ld, 2]")
        call("aaclip_attention", _lib.FP8, _ptr(qkv), _ptr(out), batch, seq, heads, hd, flags,
             _ptr(out_sc), out_sc.shape[1], _stream())
        return out
    if qkv.dtype != out.dtype:
        raise ValueError("attention tensors must share a dtype")
    flops = 4.0 * batch * heads * seq * seq * hd / (2 if causal else 1)
    _launch("attention", {torch.float32: "attn_f32_kernel"}.get(qkv.dtype, "attn_bf16_kernel"), flops,
            qkv.numel() * qkv.element_size() + out.numel() * out.element_size(), "aaclip_attention", dtag(qkv),
            _ptr(qkv), _ptr(out), batch, seq, heads, hd, flags, None, 0, _stream())
    return out


# ------------------------------------------------------------------------ rows
def im2col(img: torch.Tensor, cols: torch.Tensor, patch: int) -> torch.Tensor:
    _dev(img, cols)
    B, C, S, S2 = img.shape
    g = S // patch
    if S != S2 or img.dtype != torch.float32 or not img.is_contiguous():
        raise ValueError("image must be contiguous fp32 [B,C,S,S]")
    if cols.shape[0] != B * g * g or not cols.is_contiguous():
        raise ValueError("cols shape mismatch")
    _launch("im2col", "im2col_band_kernel", 0.0, img.numel() * 4 + cols.numel() * cols.element_size(), "aaclip_im2col",
            dtag(cols), _ptr(img), _ptr(cols), B, C, S, patch, cols.shape[1], _stream())
    return cols


def _mx_out(t, sc, rows):
    """(dtype tag, scale ptr, ld) for an LN output: fp8 MX (t e4m3 + sc e8m0) or plain."""
    if t is not None and t.dtype == FP8:
        if sc is None or sc.dtype != torch.uint8 or sc.dim() != 3 or sc.shape[1] < rows or not t.is_contiguous():
            raise ValueError("fp8 LayerNorm output needs a contiguous e4m3 tensor and MX scales [w/128, ld, 2]")
        return _lib.FP8, _ptr(sc), sc.shape[1]
    return (dtag(t) if t is not None else None), None, 0


def embed_ln(x, cls, pos, ln_pre, ln1, h, batch, n_tok, h_sc=None):
    _dev(x, h)
    width = x.shape[1]
    if x.shape[0] != batch * n_tok or h.shape != x.shape or pos.shape != (n_tok, width):
        raise ValueError("embed_ln shape mismatch")
    od, scp, ld = _mx_out(h, h_sc, x.shape[0])
    _launch("embed_ln", "embed_ln_kernel", 0.0, x.numel() * 4 * 2 + h.numel() * h.element_size(), "aaclip_embed_ln",
            od, _ptr(x), _ptr(cls), _ptr(pos), _ptr(ln_pre[0]), _ptr(ln_pre[1]), _ptr(ln1[0]), _ptr(ln1[1]),
            _ptr(h), batch, n_tok, width, scp, ld, _stream())


def block_tail(x, n_tok, *, u=None, adapt_weight=0.0, ln=None, h=None, post=None, tap=None, out_dtype=None,
               h_sc=None):
    _dev(x, u, h, tap)
    rows, width = x.shape
    if u is not None and u.shape != x.shape:
        raise ValueError("adapter output shape mismatch")
    if h is not None and h.shape != x.shape:
        raise ValueError("h shape mismatch")
    if tap is not None and tap.shape != (rows // n_tok * (n_tok - 1), width):
        raise ValueError("tap shape mismatch")
    od, scp, ld = _mx_out(h, h_sc, rows)
    if od is None:
        od = dtag(tap) if tap is not None else F32
    if h is not None and tap is not None and h.dtype != tap.dtype and not (h.dtype == FP8 and tap.dtype == torch.bfloat16):
        raise ValueError("h and tap must share a dtype (or h fp8 MX with bf16 taps)")
    nb = rows * width * 4 * (3 if u is not None else 2) + (rows * width * h.element_size() if h is not None else 0) \
        + (tap.numel() * tap.element_size() if tap is not None else 0)
    _launch("block_tail", "block_tail_kernel", 0.0, nb, "aaclip_block_tail", od, _ptr(x), _ptr(u), float(adapt_weight),
         _ptr(ln[0]) if ln else None, _ptr(ln[1]) if ln else None, _ptr(h),
         _ptr(post[0]) if post else None, _ptr(post[1]) if post else None, _ptr(tap),
         rows, n_tok, width, scp, ld, _stream())


def layernorm(x, w, b, y, y_sc=None):
    _dev(x, y)
    _rowmajor(x, "x")
    _rowmajor(y, "y")
    if x.shape != y.shape or x.dtype != torch.float32:
        raise ValueError("layernorm shape/dtype mismatch")
    od, scp, ld = _mx_out(y, y_sc, x.shape[0])
    _launch("layernorm", "layernorm_kernel", 0.0, x.numel() * 4 + y.numel() * y.element_size(), "aaclip_layernorm",
            od, _ptr(x), x.stride(0), _ptr(w), _ptr(b), _ptr(y), y.stride(0), x.shape[0], x.shape[1], scp, ld,
            _stream())
    return y


def text_embed_ln(tokens, tok_emb, pos, ln1, x, h):
    _dev(tokens, x, h)
    n, ctx = tokens.shape
    if tokens.dtype != torch.int32 or not tokens.is_contiguous() or x.shape != (n * ctx, tok_emb.shape[1]):
        raise ValueError("text_embed_ln shape mismatch")
    call("aaclip_text_embed_ln", dtag(h), _ptr(tokens), _ptr(tok_emb), _ptr(pos), _ptr(ln1[0]), _ptr(ln1[1]),
         _ptr(x), _ptr(h), n, ctx, x.shape[1], _stream())


def eot_ln(x, tokens, ln, y):
    _dev(x, tokens, y)
    n, ctx = tokens.shape
    if y.shape != (n, x.shape[1]) or x.shape[0] != n * ctx:
        raise ValueError("eot_ln shape mismatch")
    call("aaclip_eot_ln", dtag(y), _ptr(x), _ptr(tokens), _ptr(ln[0]), _ptr(ln[1]), _ptr(y), n, ctx,
         x.shape[1], _stream())
    return y


def anchor_reduce(emb: torch.Tensor, T: torch.Tensor, col: int):
    _dev(emb, T)
    n, dim = emb.shape
    if T.shape[0] != dim or emb.dtype != torch.float32 or not emb.is_contiguous():
        raise ValueError("anchor_reduce shape mismatch")
    call("aaclip_anchor_reduce", _ptr(emb), n, dim, _ptr(T), col, T.shape[1], _stream())


def l2_normalize(x, y):
    _dev(x, y)
    _rowmajor(x, "x")
    _rowmajor(y, "y")
    if x.shape != y.shape:
        raise ValueError("l2_normalize shape mismatch")
    call("aaclip_l2_normalize", dtag(x), dtag(y), _ptr(x), x.stride(0), _ptr(y), y.stride(0),
         x.shape[0], x.shape[1], _stream())
    return y


# ------------------------------------------------------------------------ anomaly map
def _level_array(levels):
    arr = (ctypes.c_void_p * len(levels))(*[t.data_ptr() for t in levels])
    return arr


def patch_scores(levels, T, out, *, normalize=True, mode=0, group=0):
    """mode 0: out[row] = sum_l (A1 + 1 - A0)/2; mode 1 (one level): out [B, 2, group] logits."""
    _dev(*levels, T, out)
    rows, C = levels[0].shape
    for t in levels:
        _rowmajor(t, "level")
        if t.shape != (rows, C) or t.dtype != levels[0].dtype or t.stride(0) != levels[0].stride(0):
            raise ValueError("levels must share shape, dtype and stride")
    if T.shape != (C, 2) or T.dtype != torch.float32 or not T.is_contiguous():
        raise ValueError("T must be contiguous fp32 [C, 2]")
    need = rows if mode == 0 else 2 * rows
    if out.numel() < need or out.dtype != torch.float32:
        raise ValueError("patch_scores output too small")
    if mode == 1 and (group <= 0 or rows % group):
        raise ValueError("mode 1 needs group = patches per image dividing the rows")
    arr = _level_array(levels)
    call("aaclip_patch_scores", dtag(levels[0]), arr, len(levels), levels[0].stride(0), _ptr(T), rows, C,
         int(normalize), mode, group, _ptr(out), _stream())
    return out


def patch_logits(f, T, out, *, group):
    """Train-branch logits for any anchor count: out [B, n_anchor, group] = 100 * f . T."""
    _dev(f, T, out)
    _rowmajor(f, "f")
    rows, C = f.shape
    n = T.shape[1] if T.dim() == 2 else 0
    if T.dim() != 2 or T.shape[0] != C or T.dtype != torch.float32 or not T.is_contiguous():
        raise ValueError("T must be contiguous fp32 [C, n_anchor]")
    if out.numel() < rows * n or out.dtype != torch.float32 or not out.is_contiguous() or group <= 0 or rows % group:
        raise ValueError("patch_logits output / group mismatch")
    call("aaclip_patch_logits", dtag(f), _ptr(f), f.stride(0), _ptr(T), n, rows, C, group, _ptr(out), _stream())
    return out


def blur_upsample(grid, out, *, ksize, sigma, softmax=False):
    _dev(grid, out)
    B, C, g, g2 = grid.shape
    S = out.shape[-1]
    if g != g2 or out.shape != (B, C, S, S) or not grid.is_contiguous() or not out.is_contiguous():
        raise ValueError("blur_upsample shape mismatch")
    call("aaclip_blur_upsample", _ptr(grid), _ptr(out), B, C, g, S, ksize, float(sigma), int(softmax), _stream())
    return out


def anomaly_map(levels, T, out, grid_ws, *, g, ksize, sigma, normalize=True):
    """Test-branch map of all levels: patch_scores into grid_ws (>= B*g*g fp32), then blur_upsample."""
    _dev(*levels, T, out, grid_ws)
    B, S, S2 = out.shape
    rows, C = levels[0].shape
    if rows != B * g * g or S != S2 or grid_ws.numel() < rows or grid_ws.dtype != torch.float32:
        raise ValueError("anomaly_map shape mismatch (grid_ws: fp32 >= [B*g*g])")
    if not out.is_contiguous():
        raise ValueError("anomaly_map output must be contiguous")
    for t in levels:
        if t.shape != (rows, C) or t.stride(0) != levels[0].stride(0) or t.dtype != levels[0].dtype:
            raise ValueError("levels must share shape, dtype and stride")
    arr = _level_array(levels)
    nb = len(levels) * rows * C * levels[0].element_size() + C * 2 * 4 + B * S * S * 4 + 2 * rows * 4
    _launch("anomaly_map", "anomaly_map (patch_scores + blur_upsample)", 0.0, nb, "aaclip_anomaly_map",
            dtag(levels[0]), arr, len(levels), levels[0].stride(0), _ptr(T), B, g, C, int(normalize), S, ksize,
            float(sigma), _ptr(grid_ws), _ptr(out), _stream())
    return out


SCORE_GROUPS = 768 // 32  # float4 partials per (row, level) written by gemm_scores


def gemm_scores(a: torch.Tensor, w: torch.Tensor, T: torch.Tensor, part: torch.Tensor, *, leaky=False):
    """Level projection straight into anomaly-map partials (aaclip_gemm_scores): for
    v = LeakyReLU?(a @ w.T), part[m, 4g:4g+4] = {||v||^2, v.t0, v.t1, 0} over columns
    32g..32g+31, t = T[c % 768]. part: fp32 view [M, >= N/8] (unit column stride)."""
    _dev(a, w, T, part)
    _rowmajor(a, "a")
    _rowmajor(w, "w")
    _rowmajor(part, "part")
    if a.dtype not in (torch.bfloat16, torch.float16) or w.dtype != a.dtype:
        raise TypeError("gemm_scores: 16-bit operands of one dtype")
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K or part.shape[0] != M or part.shape[1] < N // 8 or part.dtype != torch.float32:
        raise ValueError("gemm_scores shape mismatch")
    if T.dtype != torch.float32 or not T.is_contiguous() or T.shape != (768, 2):
        raise ValueError("gemm_scores: T must be contiguous fp32 [768, 2]")
    _launch(f"gemm N{N} K{K} scores" + (" leaky" if leaky else ""), lambda: gemm_plan(dtag(a), M, N, K),
            2.0 * M * N * K, (M * K + N * K) * a.element_size() + M * N // 8 * 4, "aaclip_gemm_scores", dtag(a), M,
            N, K, _ptr(a), a.stride(0), _ptr(w), w.stride(0), 4 if leaky else 0, _ptr(T), 768, _ptr(part),
            part.stride(0), _stream())


def anomaly_map_partials(part, n_levels, out, grid_ws, *, g, ksize, sigma, det_ws=None, score=None):
    """Map (+ image score when det_ws / score are given) from gemm_scores partials
    (aaclip_anomaly_map_partials): part [B*g*g, >= (n_levels + det) * 96] fp32."""
    _dev(part, out, grid_ws, det_ws, score)
    _rowmajor(part, "part")
    B, S, S2 = out.shape
    rows = B * g * g
    det = det_ws is not None
    if part.shape[0] != rows or part.shape[1] < (n_levels + det) * 4 * SCORE_GROUPS or S != S2:
        raise ValueError("anomaly_map_partials shape mismatch")
    if grid_ws.numel() < rows or (det and (det_ws.numel() < rows or score is None or score.numel() < B)):
        raise ValueError("anomaly_map_partials workspace too small")
    if not out.is_contiguous():
        raise ValueError("anomaly_map_partials output must be contiguous")
    nb = rows * (n_levels + det) * 4 * SCORE_GROUPS * 4 + B * S * S * 4 + 2 * rows * 4
    _launch("anomaly_map", "anomaly_map (partial_scores + blur_upsample)", 0.0, nb, "aaclip_anomaly_map_partials",
            _ptr(part), part.stride(0), n_levels, int(det), B, g, S, ksize, float(sigma), _ptr(grid_ws),
            _ptr(det_ws), _ptr(out), _ptr(score), _stream())
    return out


def image_score(det_raw, batch, n_patch, partial, det=None, T=None, score=None, normalize=True):
    _dev(det_raw, partial, det, T, score)
    _rowmajor(det_raw, "det_raw")
    rows, C = det_raw.shape
    if rows != batch * n_patch or partial.numel() < batch * ((n_patch + 15) // 16) * C:
        raise ValueError("image_score shape mismatch")
    _launch("image_score", "image_score (det_partial + det_finalize)", 0.0, rows * C * det_raw.element_size(),
            "aaclip_image_score", dtag(det_raw), _ptr(det_raw), det_raw.stride(0), _ptr(T), batch, n_patch, C,
            int(normalize), _ptr(partial), _ptr(det), _ptr(score), _stream())


def metrics_eval(pixel_preds: torch.Tensor, pixel_label: torch.Tensor, image_preds: torch.Tensor,
                 image_label: torch.Tensor, *, medical: bool) -> list[float]:
    """Device metrics_eval of one class (aaclip_metrics_eval): returns the unrounded
    [pixel AUROC, pixel AP, image AUROC, image AP]. pixel_preds [N, ...] fp32 maps,
    pixel_label same element count (nonzero = anomalous), image_* [N]."""
    N = pixel_preds.shape[0]
    preds = pixel_preds.reshape(N, -1).to(torch.float32).contiguous()
    pix = preds.shape[1]
    lab = pixel_label.reshape(N, -1)
    if lab.shape[1] != pix:
        raise ValueError("pixel_label and pixel_preds must have the same number of elements per image")
    lab = (lab != 0).to(torch.uint8).contiguous()
    ip = image_preds.reshape(-1).to(torch.float32).contiguous()
    il = (image_label.reshape(-1) != 0).to(torch.uint8).contiguous()
    if ip.numel() != N or il.numel() != N:
        raise ValueError("image_preds / image_label must have one entry per image")
    with torch.cuda.device(preds.device):
        return _metrics_eval_dev(preds, lab, ip, il, N, pix, medical).tolist()


def metrics_eval_device(pixel_preds, pixel_label, image_preds, image_label, *, medical: bool) -> torch.Tensor:
    """metrics_eval without the host sync: the device float64[4] result, read later (the
    harness reads every class's at the end, so classes are enqueued back to back)."""
    N = pixel_preds.shape[0]
    preds = pixel_preds.reshape(N, -1).to(torch.float32).contiguous()
    lab = (pixel_label.reshape(N, -1) != 0).to(torch.uint8).contiguous()
    if lab.shape[1] != preds.shape[1]:
        raise ValueError("pixel_label and pixel_preds must have the same number of elements per image")
    ip = image_preds.reshape(-1).to(torch.float32).contiguous()
    il = (image_label.reshape(-1) != 0).to(torch.uint8).contiguous()
    if ip.numel() != N or il.numel() != N:
        raise ValueError("image_preds / image_label must have one entry per image")
    with torch.cuda.device(preds.device):
        return _metrics_eval_dev(preds, lab, ip, il, N, preds.shape[1], medical)


def _metrics_eval_dev(preds, lab, ip, il, N, pix, medical):
    _dev(preds, lab, ip, il)
    need = ctypes.c_size_t(0)
    call("aaclip_metrics_workspace", N * pix, N, ctypes.byref(need))
    ws = torch.empty(int(need.value) + 256, device=preds.device, dtype=torch.uint8)
    off = (-ws.data_ptr()) % 256
    out = torch.empty(4, device=preds.device, dtype=torch.float64)
    call("aaclip_metrics_eval", _ptr(preds), _ptr(lab), _ptr(ip), _ptr(il), N, pix, int(medical),
         ws.data_ptr() + off, need.value, _ptr(out), _stream())
    return out
