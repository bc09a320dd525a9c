"""CPU restatement (numpy, integer arithmetic) of the reference's test-time
image / mask preprocessing.

TEST INFRASTRUCTURE — this is the ORACLE for aaclip_preprocess_images /
aaclip_resize_masks_nearest. Only tests/ may import it.

Reference call sites: dataset/__init__.py:127-143 (transform_x: Resize((S,S),
BICUBIC) -> ToTensor -> Normalize(CLIP mean/std); transform_mask:
Resize((S,S), NEAREST) -> ToTensor -> (mask != 0)), applied per item at
dataset/__init__.py:152-162. torchvision (absent here) hands PIL images to
Pillow's Image.resize, so the arithmetic is Pillow's (12.2.0 in this image;
the reference's requirements.txt leaves it unpinned):

  * BICUBIC (libImaging/Resample.c): separable two-pass, horizontal first over
    the source rows the vertical pass needs; per output coordinate the filter
    support is 2*max(scale, 1), taps are a = -0.5 cubic weights normalised to
    sum 1 in float64, then rounded to int32 with 22 fraction bits; each pass
    accumulates uint8 * int32 from 1 << 21 and clips (>> 22) to uint8.
  * NEAREST (libImaging/Geometry.c ImagingScaleAffine): source index
    int(xo) with xo = 0.5 * in/out, then xo += in/out per output pixel
    (accumulated in float64 — matters at exact .5 boundaries).
  * ToTensor + Normalize: float32 (v / 255 - mean) / std, IEEE division.

Pinned: tests/test_preprocess.py checks every function here against Pillow
itself (present in this image and on the GPU box) over randomised sizes, bit
for bit.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 22
MEAN = np.array((0.48145466, 0.4578275, 0.40821073), np.float32)
STD = np.array((0.26862954, 0.26130258, 0.27577711), np.float32)


def _bicubic(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def bicubic_coeffs(in_size: int, out_size: int):
    """(bounds int32 [out, 2] = (first tap, n taps), coeffs int32 [out, ksize])."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _pass(src: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One 8-bit resampling pass along `axis` of an int array [..., n, ...]."""
    src = np.moveaxis(src.astype(np.int64), axis, 0)
    acc = np.full((bounds.shape[0],) + src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
    for t in range(kk.shape[1]):
        live = t < bounds[:, 1]
        idx = np.where(live, bounds[:, 0] + t, 0)
        w = np.where(live, kk[:, t], 0).astype(np.int64)
        acc += src[idx] * w.reshape((-1,) + (1,) * (src.ndim - 1))
    out = np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)
    return np.moveaxis(out, 0, axis)


def resize_bicubic_u8(img: np.ndarray, size: int) -> np.ndarray:
    """uint8 [H, W, C] -> uint8 [size, size, C], Pillow BICUBIC semantics."""
    H, W = img.shape[:2]
    bx, kx = bicubic_coeffs(W, size)
    by, ky = bicubic_coeffs(H, size)
    first, last = by[0, 0], by[-1, 0] + by[-1, 1]
    tmp = img[first:last]
    if W != size:
        tmp = _pass(tmp, bx, kx, axis=1)
    if H != size:
        by = by.copy()
        by[:, 0] -= first
        tmp = _pass(tmp, by, ky, axis=0)
    return tmp


def nearest_index(in_size: int, out_size: int) -> np.ndarray:
    a = in_size / out_size
    xo = a * 0.5
    idx = np.empty(out_size, np.int32)
    for x in range(out_size):
        idx[x] = int(xo) if xo >= 0 else -1
        xo += a
    return idx


def transform_image(img: np.ndarray, size: int) -> np.ndarray:
    """uint8 RGB [H, W, 3] -> float32 [3, size, size] (resize -> ToTensor -> Normalize)."""
    r = resize_bicubic_u8(img, size).astype(np.float32).transpose(2, 0, 1) / np.float32(255.0)
    return (r - MEAN[:, None, None]) / STD[:, None, None]


def transform_mask(mask: np.ndarray, size: int) -> np.ndarray:
    """uint8 L [H, W] -> float32 [1, size, size] of (nearest-resized mask != 0)."""
    H, W = mask.shape
    m = mask[nearest_index(H, size)][:, nearest_index(W, size)]
    return (m != 0).astype(np.float32)[None]
