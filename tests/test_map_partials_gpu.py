"""The predict path's projections-as-partials form of the anomaly map (aaclip_gemm_scores
+ aaclip_anomaly_map_partials): the level / det projections (reference adapter.py:107-110)
leave the GEMM as per-(row, 32-column) partials {||v||^2, v.t0, v.t1} against the text
anchors, and the map + image score (forward_utils.py:196-213, test.py:83-93) are formed
from those -- checked against float64 references of the same operands, against the
row path (segbuf + aaclip_anomaly_map + aaclip_image_score), across every tile family
(bit for bit) and end to end against the reference's goldens."""
import numpy as np
import pytest
import torch

from aaclip import _lib, ops
from aaclip.engine import VisualEngine
from oracle import synth

pytestmark = pytest.mark.gpu


def _partials64(a, w, T, leaky):
    v = a.double() @ w.double().T
    if leaky:
        v = torch.where(v >= 0, v, 0.01 * v)
    M, N = v.shape
    t = T.double()[torch.arange(N, device=v.device) % 768]  # [N, 2]
    vg = v.view(M, N // 32, 32)
    tg = t.view(N // 32, 32, 2)
    return torch.stack([(vg * vg).sum(-1), (vg * tg[..., 0]).sum(-1), (vg * tg[..., 1]).sum(-1)], -1)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,leaky", [(576, 768, False), (1152, 1536, True), (9216, 768, True), (300, 768, False)])
def test_gemm_scores_vs_float64(dev, dt, M, N, leaky):
    g = torch.Generator(device=dev).manual_seed(M + N)
    a = torch.randn(M, 1024, device=dev, generator=g).to(dt)
    w = (torch.randn(N, 1024, device=dev, generator=g) * 0.03).to(dt)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    part = torch.full((M, N // 8 + 8), float("nan"), device=dev)  # padded row stride; pad stays NaN
    ops.gemm_scores(a, w, T, part[:, : N // 8], leaky=leaky)
    got = part[:, : N // 8].view(M, N // 32, 4)
    ref = _partials64(a, w, T, leaky)
    torch.testing.assert_close(got[..., :3].double(), ref, rtol=2e-5, atol=2e-5)
    assert torch.equal(got[..., 3], torch.zeros_like(got[..., 3]))
    assert torch.isnan(part[:, N // 8:]).all()


@pytest.mark.parametrize("M,N", [(9232, 768), (577, 1536), (18464, 1536)])
def test_gemm_scores_families_bit_identical(dev, M, N):
    """Every tile family (wave tiles 32 or 64 columns wide) forms the same 32-column
    groups in the same order: the partials, hence an image's map, do not depend on the
    family the per-shape dispatch takes for a batch size."""
    g = torch.Generator(device=dev).manual_seed(N)
    a = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, 1024, device=dev, generator=g) * 0.03).bfloat16()
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    outs = []
    for f in (0, 1, 2, 3, 8, 9, 11):
        _lib.call("aaclip_set_gemm_variant", f)
        try:
            p = torch.empty(M, N // 8, device=dev)
            ops.gemm_scores(a, w, T, p, leaky=True)
        finally:
            _lib.call("aaclip_set_gemm_variant", 0)
        outs.append((f, p))
    for f, p in outs[1:]:
        assert torch.equal(p, outs[0][1]), f


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,S,dom", [(2, 336, "Industrial"), (3, 336, "Medical"), (2, 518, "Industrial")])
def test_predict_partials_vs_row_path(dev, dt, B, S, dom):
    """predict() with the partials form against the row path on the same engine: maps
    within 2e-5 abs (|map| ~ 4 x 100 x cos: the fixed-order sums differ only in
    association), image scores within 1e-6."""
    sd = synth.clip_state_dict(111, img_size=S)
    ia, _ = synth.adapter_state_dicts(111)
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    eng = VisualEngine(vp, {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}, dtype=dt)
    g = torch.Generator(device=dev).manual_seed(S + B)
    x = torch.randn(B, 3, S, S, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    res = []
    for on in (True, False):
        eng.map_partials = on
        m, s = eng.predict(x, T, dom)
        res.append((m.clone(), s.clone()))
    (m1, s1), (m0, s0) = res
    assert torch.isfinite(m1).all()
    err = (m1 - m0).abs().max().item()
    print(dt, B, S, dom, "partials vs rows: map max abs", err, "score", (s1 - s0).abs().max().item())
    assert err < 2e-5 * max(1.0, m0.abs().max().item())
    torch.testing.assert_close(s1, s0, atol=1e-6, rtol=0)


def test_partials_args_rejected_before_launch(dev):
    part = torch.zeros(2 * 24 * 24, 5 * 96, device=dev)
    out = torch.full((2, 336, 336), 7.0, device=dev)
    grid = torch.full((2 * 576,), 7.0, device=dev)
    with pytest.raises(RuntimeError):  # ksize even: rejected before the stage-1 launch writes grid
        _lib.call("aaclip_anomaly_map_partials", ops._ptr(part), part.stride(0), 4, 0, 2, 24, 336, 8, 1.0,
                  ops._ptr(grid), None, ops._ptr(out), None, ops._stream())
    torch.cuda.synchronize()
    assert (grid == 7.0).all() and (out == 7.0).all()


@pytest.mark.parametrize("B,g,S,nl,det", [(2, 24, 336, 4, True), (1, 37, 518, 4, True), (3, 32, 448, 6, True),
                                          (1, 37, 518, 6, False), (5, 24, 336, 3, False)])
def test_partial_scores_stage_vs_float64(dev, B, g, S, nl, det):
    """Stage 1 of aaclip_anomaly_map_partials on its own inputs: per patch row the level
    sums of the 24 group partials, the normalised anchor dots and the level sum (and the
    det dot for the image score) against float64 of the same partials. Ragged row counts
    (1369 rows at 518 px: the last workgroup's 8-lane row groups run past the end), 3 / 4 /
    6 levels, with and without the det level, a padded partials row stride; the map is
    stage 2 (blur + upsample, the row path's band code) on the float64 grid."""
    rows = B * g * g
    nt = nl + int(det)
    G = ops.SCORE_GROUPS
    gen = torch.Generator(device=dev).manual_seed(rows + nt)
    part = torch.full((rows, nt * 4 * G + 12), float("nan"), device=dev)  # padded stride, pad NaN
    p = part[:, : nt * 4 * G].view(rows, nt, G, 4)
    p[..., 0] = torch.rand(rows, nt, G, device=dev, generator=gen) * 2.0 + 0.05   # ||v||^2 group sums > 0
    p[..., 1:3] = torch.randn(rows, nt, G, 2, device=dev, generator=gen) * 0.3
    p[..., 3] = 0.0
    out = torch.empty(B, S, S, device=dev)
    grid = torch.empty(rows, device=dev)
    dws = torch.empty(rows, device=dev) if det else None
    score = torch.empty(B, device=dev) if det else None
    ops.anomaly_map_partials(part, nl, out, grid, g=g, ksize=7, sigma=4.0, det_ws=dws, score=score)
    q = p.double().sum(2)  # [rows, nt, 4]
    inv = 1.0 / q[..., 0].sqrt().clamp_min(1e-12)
    a0, a1 = q[..., 1] * inv, q[..., 2] * inv
    ref_grid = ((100.0 * a1[:, :nl] + 1.0 - 100.0 * a0[:, :nl]) / 2.0).sum(1)
    torch.testing.assert_close(grid.double(), ref_grid, rtol=1e-5, atol=1e-4)
    ref_map = torch.empty_like(out)
    ops.blur_upsample(ref_grid.float().view(B, 1, g, g), ref_map.view(B, 1, S, S), ksize=7, sigma=4.0)
    torch.testing.assert_close(out, ref_map, rtol=1e-5, atol=1e-4)
    if det:
        torch.testing.assert_close(dws.double(), a1[:, nl], rtol=1e-5, atol=1e-6)
        ref_score = (a1[:, nl].view(B, g * g).mean(1) + 1.0) / 2.0
        torch.testing.assert_close(score.double(), ref_score, rtol=0, atol=1e-6)
    # run to run: the same bits
    grid2 = torch.empty_like(grid)
    out2 = torch.empty_like(out)
    ops.anomaly_map_partials(part, nl, out2, grid2, g=g, ksize=7, sigma=4.0, det_ws=dws, score=score)
    assert torch.equal(grid, grid2) and torch.equal(out, out2)
