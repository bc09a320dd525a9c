"""Test-time preprocessing (reference dataset/__init__.py:127-162).

CPU part: the oracle restatement (oracle/preprocess_np.py) is pinned bit for bit
against Pillow itself — the library the reference's torchvision transforms call —
and the C ABI's host-side plan builders must reproduce the oracle's tables exactly.
GPU part: aaclip_preprocess_images / aaclip_resize_masks_nearest equal the oracle
(and therefore Pillow + ToTensor + Normalize) exactly, fp32 bit for bit.
"""
import math

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import preprocess_np as P

# (H, W, S): MVTec-like sizes, VisA-like non-square, upscales, odd tiny/huge ratios
CASES = [(900, 900, 336), (1024, 1024, 336), (1024, 1024, 448), (1000, 1500, 518), (1217, 1421, 336),
         (224, 224, 336), (336, 336, 336), (240, 512, 336), (5, 7, 336), (3000, 41, 336), (700, 701, 13),
         (2400, 2000, 40)]  # the last one exceeds the staged LDS patch: direct-tap kernel


def _pil_image(img, S):
    r = np.asarray(Image.fromarray(img).resize((S, S), Image.BICUBIC)).astype(np.float32)
    r = r.transpose(2, 0, 1) / np.float32(255.0)  # ToTensor: float32 x / 255
    return (r - P.MEAN[:, None, None]) / P.STD[:, None, None]  # Normalize: sub_, div_


def _img(H, W, seed):
    rng = np.random.default_rng(seed)
    if seed % 2:
        return rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:H, 0:W]  # smooth content + saturating edges (exercises the clip)
    base = 127 + 140 * np.sin(xx / 9.0 + yy / 13.0)
    return np.clip(np.stack([base, base[::-1], 255 - base], -1), 0, 255).astype(np.uint8)


def _mask(H, W, seed):
    rng = np.random.default_rng(seed)
    m = np.zeros((H, W), np.uint8)
    m[rng.integers(0, H):, rng.integers(0, W):] = rng.integers(1, 256)
    return m | (rng.random((H, W)) < 0.02).astype(np.uint8)


@pytest.mark.parametrize("H,W,S", CASES)
def test_oracle_matches_pillow(H, W, S):
    img = _img(H, W, H + W)
    assert np.array_equal(P.resize_bicubic_u8(img, S), np.asarray(Image.fromarray(img).resize((S, S), Image.BICUBIC)))
    assert np.array_equal(P.transform_image(img, S), _pil_image(img, S))
    m = _mask(H, W, S)
    ref = (np.asarray(Image.fromarray(m).resize((S, S), Image.NEAREST)) != 0).astype(np.float32)[None]
    assert np.array_equal(P.transform_mask(m, S), ref)


def test_oracle_matches_pillow_random_sizes():
    rng = np.random.default_rng(7)
    for t in range(40):
        H, W, S = (int(v) for v in rng.integers(1, 1300, 3))
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        assert np.array_equal(P.resize_bicubic_u8(img, S),
                              np.asarray(Image.fromarray(img).resize((S, S), Image.BICUBIC))), (H, W, S)
        m = (rng.random((H, W)) < 0.5).astype(np.uint8)
        ref = np.asarray(Image.fromarray(m).resize((S, S), Image.NEAREST)) != 0
        assert np.array_equal(P.transform_mask(m, S)[0] != 0, ref), (H, W, S)


def test_abi_plans_equal_oracle_tables():
    from aaclip.preprocess import bicubic_plan, nearest_plan
    rng = np.random.default_rng(3)
    sizes = [(n, S) for n, S in ((900, 336), (1024, 448), (1500, 518), (224, 336), (336, 336), (5, 336),
                                 (3000, 336), (701, 13), (33600, 336))]
    sizes += [tuple(int(v) for v in rng.integers(1, 4000, 2)) for _ in range(40)]
    for n, S in sizes:
        b, k = bicubic_plan(n, S)
        ob, ok = P.bicubic_coeffs(n, S)
        assert np.array_equal(b, ob) and np.array_equal(k, ok), (n, S)
        assert np.array_equal(nearest_plan(n, S), P.nearest_index(n, S)), (n, S)


def test_strip_bound_covers_every_tile():
    """The kernel sizes its LDS strip / patch by strip_bound(); every tile's taps
    must fall inside it (restated bound: ceil((t-1)*in/S) + ksize + 2), for the
    row extent (t = ty) and the column extent (t = tx) alike."""
    for n, S in ((900, 336), (1024, 448), (3000, 336), (5, 336), (33600, 336), (1217, 13)):
        b, k = P.bicubic_coeffs(n, S)
        for ty in (64, 32, 16, 8, 4, 2, 1):
            bound = min(n, math.ceil((ty - 1) * n / S) + k.shape[1] + 2)
            for y0 in range(0, S, ty):
                y1 = min(y0 + ty, S)
                assert b[y1 - 1, 0] + b[y1 - 1, 1] - b[y0, 0] <= bound, (n, S, ty, y0)


def test_preprocess_rejects_bad_calls():
    import ctypes

    from aaclip import _lib
    lib = _lib.lib()
    k = ctypes.c_int()
    assert lib.aaclip_bicubic_taps(0, 336, ctypes.byref(k)) == 1
    assert lib.aaclip_bicubic_taps(900, 336, ctypes.byref(k)) == 0 and k.value == 2 * math.ceil(2 * 900 / 336) + 1
    buf = (ctypes.c_int32 * 4096)()
    assert lib.aaclip_bicubic_plan(900, 336, buf, buf, k.value - 1) == 1  # ksize too small
    assert lib.aaclip_nearest_plan(900, 0, buf) == 1
    f16 = ctypes.c_void_p(16)
    # row pitch smaller than a row of RGB pixels
    assert lib.aaclip_preprocess_images(f16, 900 * 900 * 3, 899 * 3, 1, 900, 900, f16, f16, 13, f16, f16, 13, 336,
                                        None, f16, None, 0, None) == 1
    # plan narrower than the resampling support
    assert lib.aaclip_preprocess_images(f16, 900 * 900 * 3, 900 * 3, 1, 900, 900, f16, f16, 5, f16, f16, 13, 336,
                                        None, f16, None, 0, None) == 1
    n = ctypes.c_size_t()
    assert lib.aaclip_preprocess_workspace(4, 900, 700, 336, ctypes.byref(n)) == 0 and n.value >= 4 * 900 * 336 * 3
    assert lib.aaclip_resize_masks_nearest(None, 0, 900, 1, 900, 900, f16, f16, 336, f16, None) == 1


# ---------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("H,W,S", CASES)
def test_device_preprocess_bit_exact(dev, H, W, S):
    from aaclip.preprocess import Preprocessor
    B = 3
    imgs = np.stack([_img(H, W, H + W + i) for i in range(B)])
    masks = np.stack([_mask(H, W, S + i) for i in range(B)])
    pp = Preprocessor(S)
    out = pp.images(torch.from_numpy(imgs).to(dev))
    one = pp.images(torch.from_numpy(imgs).to(dev), two_pass=False)
    mo = pp.masks(torch.from_numpy(masks).to(dev))
    torch.cuda.synchronize()
    assert torch.equal(out, one)  # two-pass and single-kernel paths: same bits
    for i in range(B):
        assert np.array_equal(out[i].cpu().numpy(), P.transform_image(imgs[i], S)), i
        assert np.array_equal(mo[i].cpu().numpy(), P.transform_mask(masks[i], S)), i


@pytest.mark.gpu
def test_device_preprocess_padded_pitch_and_batch_stride(dev):
    """Padded row pitch, an arbitrary image stride and byte-misaligned rows (the
    staged kernel realigns every row to dwords) give the same result."""
    from aaclip.preprocess import Preprocessor
    H, W, S, B = 517, 611, 336, 4
    imgs = np.stack([_img(H, W, i) for i in range(B)])
    ref = Preprocessor(S).images(torch.from_numpy(imgs).to(dev))
    for pitch, off in (((W * 3 + 63) // 64 * 64, 0), (W * 3 + 5, 1), (W * 3 + 2, 3)):
        stage = torch.zeros(B, H + 3, pitch + off, dtype=torch.uint8)
        stage[:, :H, off:off + W * 3] = torch.from_numpy(imgs.reshape(B, H, W * 3))
        stage = stage.to(dev)
        view = stage[:, :H, off:off + W * 3].unflatten(2, (W, 3))
        assert view.stride(1) == pitch + off and view.stride(0) == (H + 3) * (pitch + off)
        for two in (True, False):
            out = Preprocessor(S).images(view, two_pass=two)
            assert torch.equal(out, ref), (pitch, off, two)
    assert np.array_equal(ref[2].cpu().numpy(), P.transform_image(imgs[2], S))


@pytest.mark.gpu
def test_device_preprocess_feeds_the_engine_like_host_transform(dev):
    """Device transform -> the same fp32 tensor the reference's dataset yields
    (the host path in dataset/ uses Pillow directly)."""
    from aaclip.preprocess import Preprocessor
    img = _img(900, 900, 5)
    host = _pil_image(img, 336)
    d = Preprocessor(336).images(torch.from_numpy(img[None]).to(dev))[0].cpu().numpy()
    assert np.array_equal(d, host)


def _disk_dataset(tmp_path, sizes):
    """A reference-layout test set on disk: PNG images + masks and a jsonl index."""
    import json
    rows = []
    for i, (H, W) in enumerate(sizes):
        Image.fromarray(_img(H, W, i)).save(tmp_path / f"img{i}.png")
        row = {"image_path": f"img{i}.png", "label": i % 2, "class_name": "bottle"}
        if i % 2:
            Image.fromarray(_mask(H, W, i) * 255).save(tmp_path / f"mask{i}.png")
            row["mask_path"] = f"mask{i}.png"
        rows.append(row)
    meta = tmp_path / "meta.jsonl"
    meta.write_text("".join(json.dumps(r) + "\n" for r in rows))
    return str(tmp_path), str(meta)


def test_raw_dataset_items_and_collate(tmp_path):
    from dataset import BaseSingleClassDataset, collate_raw
    root, meta = _disk_dataset(tmp_path, [(300, 400), (300, 400), (250, 260)])
    ds = BaseSingleClassDataset(root, meta, 336, "bottle", raw=True)
    it = ds[1]
    assert it["image_u8"].dtype == torch.uint8 and tuple(it["image_u8"].shape) == (300, 400, 3)
    assert np.array_equal(it["image_u8"].numpy(), np.asarray(Image.open(tmp_path / "img1.png").convert("RGB")))
    assert it["mask_u8"].shape == (300, 400) and ds[0]["mask_u8"].sum() == 0
    b = collate_raw([ds[0], ds[1]])
    assert tuple(b["image_u8"].shape) == (2, 300, 400, 3) and b["label"] == [0, 1]
    assert isinstance(collate_raw([ds[0], ds[2]])["image_u8"], list)  # mixed sizes stay a list


@pytest.mark.gpu
def test_raw_dataset_device_transform_equals_host_dataset(dev, tmp_path):
    """The harness's --gpu_preprocess path (raw items -> device transform) yields
    exactly the tensors of the host (Pillow) dataset, mixed sizes included."""
    import importlib.util
    import pathlib
    from dataset import BaseSingleClassDataset, collate_raw
    harness = pathlib.Path(__file__).resolve().parents[1] / "aa-clip_amd" / "test.py"
    spec = importlib.util.spec_from_file_location("aaclip_test_harness", harness)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    _device_batch = mod._device_batch

    from aaclip.preprocess import Preprocessor
    root, meta = _disk_dataset(tmp_path, [(300, 400), (300, 400), (250, 260), (337, 335)])
    host = BaseSingleClassDataset(root, meta, 336, "bottle")
    raw = BaseSingleClassDataset(root, meta, 336, "bottle", raw=True)
    for idx in ([0, 1], [1, 2, 3]):
        img, mask = _device_batch(collate_raw([raw[i] for i in idx]), Preprocessor(336), dev)
        assert torch.equal(img.cpu(), torch.stack([host[i]["image"] for i in idx]))
        assert torch.equal(mask.cpu(), torch.stack([host[i]["mask"] for i in idx]))
