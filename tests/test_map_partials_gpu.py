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
