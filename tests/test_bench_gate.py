"""bench.py's parity gate (CPU, no GPU): every bench line is held to the bounds the tests
hold (bf16 sure flips <= 2x measured in total and 2x + 2 per level, >= 99.9 % of pixels in
the 1e-3 + 1e-2 |ref| envelope, image labels equal; fp16 / fp32 the full contract), and to
the TIMED step's own outputs against the CPU oracle. A corrupted map must turn the line's
"parity_gate" false and the exit status non-zero: round 5 showed a kernel that corrupted
activations can run faster and still pass a same-library self-comparison.
Reference contract: test.py:80-93."""
import io
import json
from contextlib import redirect_stdout

import numpy as np
import pytest
import torch

import bench


def _mode(rng, n=8, L=4, P=576, S=64, noise=1e-5, flips_per_level=(0, 0, 0, 0)):
    ref_grid = rng.standard_normal((n, L, P, 2)).astype(np.float32)
    ref_maps = rng.random((n, S, S)).astype(np.float32) * 4.0
    ref_scores = rng.random(n).astype(np.float32)
    lab = (rng.random(n * S * S) < 0.1)
    grid = ref_grid.copy()
    for lv, k in enumerate(flips_per_level):  # swap the two anchors on k sure patches of level lv
        grid[0, lv, :k] = ref_grid[0, lv, :k, ::-1]
    maps = ref_maps + noise * rng.standard_normal(ref_maps.shape).astype(np.float32)
    return (grid, maps, ref_scores.copy(), ref_grid, ref_maps, ref_scores, lab)


def _parity(rng, corrupt=None):
    par = {"sizes": [336, 518]}
    for size in (336, 518):
        par[str(size)] = {}
        lv = bench.BF16_PARITY_FLIPS[str(size)][1]
        for tag in ("bf16", "fp16", "fp32"):
            args = list(_mode(rng, flips_per_level=lv if tag == "bf16" else (0, 0, 0, 0)))
            if corrupt is not None and corrupt[0] == (size, tag):
                corrupt[1](args)
            par[str(size)][tag] = bench.parity_stats(*args)
    return par


def _timed_ok():
    return {"finite": True, "map_max_abs_err": 1e-3, "map_rel_l2": 1e-2, "frac_pixels_within_tol": 0.3,
            "image_score_max_abs_err": 1e-4, "image_labels_equal": True}


def _emit(line):
    buf = io.StringIO()
    with redirect_stdout(buf):
        rc = bench.emit(line)
    printed = json.loads(buf.getvalue().strip().splitlines()[-1])
    return rc, printed


def test_gate_passes_measured_counts():
    rng = np.random.default_rng(0)
    line = {"parity": _parity(rng), "timed_step_vs_oracle": _timed_ok()}
    rc, printed = _emit(line)
    assert rc == 0 and printed["parity_gate"] is True, printed.get("parity_gate_failed")
    assert "timed_step_vs_oracle" in printed["parity_gate_checked"]
    assert printed["parity"]["336"]["bf16"]["patch_label_flips_sure_per_level"] == [4, 0, 29, 0]


def _corrupt_block(args):  # a stale / racing kernel: one image's map zeroed over a block
    args[1][3, 10:40, 10:40] = 0.0


def _corrupt_nan(args):
    args[1][0, 0, 0] = np.nan


def _corrupt_labels(args):  # every level of image 1 flipped
    args[0][1] = args[3][1, :, :, ::-1]


@pytest.mark.parametrize("where,fn", [((336, "bf16"), _corrupt_block), ((518, "fp16"), _corrupt_block),
                                      ((336, "fp32"), _corrupt_nan), ((518, "bf16"), _corrupt_labels)])
def test_gate_fails_corrupted_parity_leg(where, fn):
    rng = np.random.default_rng(1)
    line = {"parity": _parity(rng, corrupt=(where, fn)), "timed_step_vs_oracle": _timed_ok()}
    rc, printed = _emit(line)
    assert rc == 1 and printed["parity_gate"] is False
    assert any(f"{where[0]}px {where[1]}" in f for f in printed["parity_gate_failed"]), printed["parity_gate_failed"]


def test_gate_fails_without_any_parity_leg():
    rc, printed = _emit({"value": 1.0})
    assert rc == 1 and printed["parity_gate"] is False


def test_timed_step_vs_oracle_catches_a_corrupted_map():
    """The timed-step check end to end on the CPU: bench's own synthetic ViT-L/14 weights at a
    112 px image (8 x 8 patches), the CPU oracle's outputs standing in for the timed replay's; the
    same outputs with one image's map corrupted must fail the gate (rc 1)."""
    from oracle import aaclip_torch as RT
    dev = torch.device("cpu")
    vp, ad = bench.synthetic_visual_weights(dev, n_tok=65)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(3, 3, 112, 112, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, generator=g), dim=0)
    w = RT.prepare(vp, ad)
    with torch.no_grad():
        seg, det = RT.visual_forward(w, x)
        maps = RT.anomaly_map(seg, T, 112, "Industrial")
        scores = RT.image_score(det, T)
    ok = bench.timed_step_vs_oracle(vp, ad, x, maps, scores, T)
    assert ok["images"] == [0, 2] and ok["frac_pixels_within_tol"] == 1.0 and ok["map_rel_l2"] < 1e-6
    rc, printed = _emit({"timed_step_vs_oracle": ok})
    assert rc == 0 and printed["parity_gate"]
    bad = maps.clone()
    bad[2, :40] += 5.0
    rc, printed = _emit({"timed_step_vs_oracle": bench.timed_step_vs_oracle(vp, ad, x, bad, scores, T)})
    assert rc == 1 and not printed["parity_gate"]
    assert any("timed step" in f for f in printed["parity_gate_failed"])
