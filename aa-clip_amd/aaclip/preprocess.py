"""Device test-time preprocessing — drop-in for the reference's per-item
transforms (dataset/__init__.py:127-143: transform_x = Resize((S,S), BICUBIC)
-> ToTensor -> Normalize(CLIP mean/std); transform_mask = Resize((S,S),
NEAREST) -> ToTensor, then `(mask != 0).float()` at :158).

Decoded uint8 images go to HBM as they are (HWC RGB / L) and one kernel per
batch resamples + normalises them (aaclip_preprocess_images), bit-exact with
Pillow's 8-bit resampling, so the maps downstream are identical to the
reference's CPU-worker path. Plans (per-axis tap tables) are built on the host
by the C ABI in Pillow's double-precision arithmetic and cached per source size.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import call
from .ops import _dev, _ptr, _stream

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def bicubic_plan(in_size: int, out_size: int):
    """Pillow BICUBIC tables for one axis: bounds int32 [out, 2] = (first tap, taps),
    coeffs int32 [out, ksize] (22 fraction bits). Host only."""
    k = ctypes.c_int()
    call("aaclip_bicubic_taps", in_size, out_size, ctypes.byref(k))
    bounds = np.zeros((out_size, 2), np.int32)
    coeffs = np.zeros((out_size, k.value), np.int32)
    call("aaclip_bicubic_plan", in_size, out_size, bounds.ctypes.data_as(ctypes.c_void_p),
         coeffs.ctypes.data_as(ctypes.c_void_p), k.value)
    return bounds, coeffs


def nearest_plan(in_size: int, out_size: int) -> np.ndarray:
    idx = np.zeros(out_size, np.int32)
    call("aaclip_nearest_plan", in_size, out_size, idx.ctypes.data_as(ctypes.c_void_p))
    return idx


class Preprocessor:
    """`images(u8 [B,H,W,3]) -> fp32 [B,3,S,S]`, `masks(u8 [B,H,W]) -> fp32 [B,1,S,S]`
    on the device of the inputs, on torch's current stream."""

    def __init__(self, img_size: int, mean=CLIP_MEAN, std=CLIP_STD):
        self.S = int(img_size)
        self._ms = (ctypes.c_float * 6)(*mean, *std)
        self._plans: dict = {}

    def _bicubic(self, n: int, dev):
        key = ("b", n, dev)
        if key not in self._plans:
            b, k = bicubic_plan(n, self.S)
            self._plans[key] = (torch.from_numpy(b).to(dev), torch.from_numpy(k).to(dev), k.shape[1])
        return self._plans[key]

    def _nearest(self, n: int, dev):
        key = ("n", n, dev)
        if key not in self._plans:
            self._plans[key] = torch.from_numpy(nearest_plan(n, self.S)).to(dev)
        return self._plans[key]

    @staticmethod
    def _check_u8(x: torch.Tensor, channels: int):
        _dev(x)
        if x.dtype != torch.uint8:
            raise TypeError("preprocess inputs are decoded uint8 images")
        if channels == 3:
            if x.dim() != 4 or x.shape[-1] != 3:
                raise ValueError(f"expected uint8 [B,H,W,3], got {tuple(x.shape)}")
            dense = x.stride(3) == 1 and x.stride(2) == 3
        else:
            if x.dim() != 3:
                raise ValueError(f"expected uint8 [B,H,W], got {tuple(x.shape)}")
            dense = x.stride(2) == 1
        if not dense or x.shape[0] > 65535:
            raise ValueError("pixel rows must be contiguous (row pitch may be padded); batch <= 65535")

    def _workspace(self, B, H, W, dev):
        n = ctypes.c_size_t()
        call("aaclip_preprocess_workspace", B, H, W, self.S, ctypes.byref(n))
        ws = self._plans.get(("ws", dev))
        if ws is None or ws.numel() < n.value:
            ws = torch.empty(max(n.value, 1), device=dev, dtype=torch.uint8)
            self._plans[("ws", dev)] = ws
        return ws, n.value

    def images(self, u8: torch.Tensor, out: torch.Tensor | None = None, two_pass: bool = True) -> torch.Tensor:
        """two_pass: horizontal pass into a uint8 intermediate (a cached workspace), then
        the vertical pass (default, faster); False = one tiled kernel, no workspace."""
        self._check_u8(u8, 3)
        B, H, W, _ = u8.shape
        dev = u8.device
        xb, xk, kx = self._bicubic(W, dev)
        yb, yk, ky = self._bicubic(H, dev)
        if out is None:
            out = torch.empty(B, 3, self.S, self.S, device=dev, dtype=torch.float32)
        if out.shape != (B, 3, self.S, self.S) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("out must be contiguous fp32 [B,3,S,S]")
        ws, nbytes = self._workspace(B, H, W, dev) if two_pass else (None, 0)
        call("aaclip_preprocess_images", _ptr(u8), u8.stride(0), u8.stride(1), B, H, W, _ptr(xb), _ptr(xk), kx,
             _ptr(yb), _ptr(yk), ky, self.S, ctypes.cast(self._ms, ctypes.c_void_p), _ptr(out), _ptr(ws), nbytes,
             _stream())
        return out

    def masks(self, u8: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        self._check_u8(u8, 1)
        B, H, W = u8.shape
        dev = u8.device
        if out is None:
            out = torch.empty(B, 1, self.S, self.S, device=dev, dtype=torch.float32)
        if out.shape != (B, 1, self.S, self.S) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("out must be contiguous fp32 [B,1,S,S]")
        call("aaclip_resize_masks_nearest", _ptr(u8), u8.stride(0), u8.stride(1), B, H, W,
             _ptr(self._nearest(W, dev)), _ptr(self._nearest(H, dev)), self.S, _ptr(out), _stream())
        return out
