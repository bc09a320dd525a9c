"""ctypes binding of libaaclip_hip.so (C ABI: include/aaclip.h).

The product path has NO CPU fallback: if the library is missing or a call
fails, this raises. Build it with `python __graft_entry__.py` (build()) or
`make -C aa-clip_amd/csrc`.
"""
from __future__ import annotations

import ctypes
import os

LIB_PATH = os.environ.get("AACLIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libaaclip_hip.so")
ABI_VERSION = 7

F32 = 0
BF16 = 1
FP8 = 2
F16 = 3
EPI_BIAS = 1
EPI_GELU = 2
EPI_LEAKY = 4
EPI_RESID = 8
EPI_AUX_BF16 = 16
EPI_QGELU = 32
ATTN_CAUSAL = 1
ATTN_Q_PRESCALED = 2

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float

# name -> argtypes (restype int unless noted); mirrors include/aaclip.h
SIGNATURES = {
    "aaclip_abi_version": [],
    "aaclip_arch": [],
    "aaclip_trace_buffer": [_P, _P, ctypes.c_uint],
    "aaclip_gemm": [_I, _I, _I, _I, _I, _P, _L, _P, _L, _P, _L, _I, _P, _P, _L, _P, _L, _I, _I, _I, _P],
    "aaclip_gemm_ksplit_workspace": [_I, _I, _I, _I, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(_L)],
    "aaclip_gemm_ksplit": [_I, _I, _I, _I, _I, _P, _L, _P, _L, _P, _L, _I, _P, _P, _L, _P, _L, _I, _P,
                           ctypes.c_size_t, _P, _L, _P],
    "aaclip_gemm_fp8": [_I, _I, _I, _I, _P, _L, _P, _P, _L, _P, _P, _L, _I, _P, _P, _L, _P, _L, _I, _I, _I, _P],
    "aaclip_quant_fp8_rows": [_I, _P, _L, _P, _L, _P, _I, _I, _P],
    "aaclip_gemm_fp8mx": [_I, _I, _I, _I, _P, _L, _P, _L, _P, _L, _P, _P, _L, _I, _P, _P, _L, _P, _L, _P, _L, _P],
    "aaclip_quant_fp8_mx": [_I, _P, _L, _P, _L, _P, _L, _I, _I, _P],
    "aaclip_set_gemm_variant": [_I],
    "aaclip_gemm_pin": [_I, _I, _I, _I, _I],
    "aaclip_gemm_concurrent": [_I, ctypes.POINTER(_I)],
    "aaclip_gemm_plan": [_I, _I, _I, _I],
    "aaclip_attention": [_I, _P, _P, _I, _I, _I, _I, _I, _P, _L, _P],
    "aaclip_set_attn_variant": [_I],
    "aaclip_im2col": [_I, _P, _P, _I, _I, _I, _I, _I, _P],
    "aaclip_embed_ln": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _L, _P],
    "aaclip_block_tail": [_I, _P, _P, _F, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _L, _P],
    "aaclip_gemm_scores": [_I, _I, _I, _I, _P, _L, _P, _L, _I, _P, _I, _P, _L, _P],
    "aaclip_anomaly_map_partials": [_P, _L, _I, _I, _I, _I, _I, _I, _F, _P, _P, _P, _P, _P],
    "aaclip_layernorm": [_I, _P, _L, _P, _P, _P, _L, _I, _I, _P, _L, _P],
    "aaclip_text_embed_ln": [_I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P],
    "aaclip_eot_ln": [_I, _P, _P, _P, _P, _P, _I, _I, _I, _P],
    "aaclip_anchor_reduce": [_P, _I, _I, _P, _I, _I, _P],
    "aaclip_l2_normalize": [_I, _I, _P, _L, _P, _L, _I, _I, _P],
    "aaclip_patch_scores": [_I, _P, _I, _L, _P, _I, _I, _I, _I, _I, _P, _P],
    "aaclip_patch_logits": [_I, _P, _L, _P, _I, _I, _I, _I, _P, _P],
    "aaclip_blur_upsample": [_P, _P, _I, _I, _I, _I, _I, _F, _I, _P],
    "aaclip_anomaly_map": [_I, _P, _I, _L, _P, _I, _I, _I, _I, _I, _I, _F, _P, _P, _P],
    "aaclip_image_score": [_I, _P, _L, _P, _I, _I, _I, _I, _P, _P, _P, _P],
    "aaclip_metrics_workspace": [_L, _I, ctypes.POINTER(ctypes.c_size_t)],
    "aaclip_metrics_eval": [_P, _P, _P, _P, _I, _L, _I, _P, ctypes.c_size_t, _P, _P],
    "aaclip_bicubic_taps": [_I, _I, ctypes.POINTER(_I)],
    "aaclip_bicubic_plan": [_I, _I, _P, _P, _I],
    "aaclip_nearest_plan": [_I, _I, _P],
    "aaclip_preprocess_images": [_P, _L, _L, _I, _I, _I, _P, _P, _I, _P, _P, _I, _I, _P, _P, _P, ctypes.c_size_t,
                                 _P],
    "aaclip_preprocess_workspace": [_I, _I, _I, _I, ctypes.POINTER(ctypes.c_size_t)],
    "aaclip_resize_masks_nearest": [_P, _L, _L, _I, _I, _I, _P, _P, _I, _P, _P],
}

_lib = None


def load(path: str) -> ctypes.CDLL:
    """Open an aaclip library and bind every SIGNATURES entry. The version check comes
    BEFORE any other symbol is bound: a stale library (built from older sources, missing
    newer entry points) is refused with one clear RuntimeError instead of an
    AttributeError at the first call of a symbol it lacks."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: the HIP kernels are not built "
            "(run `python __graft_entry__.py` or `make -C aa-clip_amd/csrc`). "
            "There is no CPU fallback.")
    handle = ctypes.CDLL(path)
    try:
        ver = handle.aaclip_abi_version
    except AttributeError:
        raise RuntimeError(f"{path} exports no aaclip_abi_version: not an aaclip library; rebuild it "
                           "(`make -C aa-clip_amd/csrc`)") from None
    ver.argtypes, ver.restype = [], ctypes.c_int
    found = ver()
    if found != ABI_VERSION:
        raise RuntimeError(f"{path} has ABI version {found}, this package needs {ABI_VERSION}: the library "
                           "is stale; rebuild it (`make -C aa-clip_amd/csrc`)")
    missing = [name for name in SIGNATURES if not hasattr(handle, name)]
    if missing:
        raise RuntimeError(f"{path} (ABI {found}) lacks {', '.join(missing)}: the library is stale; "
                           "rebuild it (`make -C aa-clip_amd/csrc`)")
    for name, argtypes in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_char_p if name in ("aaclip_arch", "aaclip_gemm_plan") else ctypes.c_int
    return handle


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = load(LIB_PATH)
    return _lib


def check(rc: int, name: str) -> None:
    if rc != 0:
        kind = "bad argument" if rc == 1 else f"launch failed (hipError {rc - 1000})"
        raise RuntimeError(f"{name}: {kind} (rc={rc})")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
