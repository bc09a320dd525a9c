"""fp16 mode on the MI355X: the same 16-bit kernels on v_mfma_f32_16x16x32_f16.

fp16 operands carry 11 significant bits (bf16: 8), at the same MFMA rate, so
this is the mode that meets the north_star map contract (1e-3 abs + 1e-2 rel,
argmax labels bit-exact beyond rounding ties) without leaving the 16-bit MFMA
path. Kernel checks are against float64 on the same fp16-rounded operands; the
end-to-end checks are against the REAL reference's golden outputs
(tests/golden/golden_e2e.npz, golden_c5.npz from tests/golden/make_golden.py).
"""
import os

import numpy as np
import pytest
import torch

from aaclip import _lib, ops
from aaclip.engine import VisualEngine
from oracle import synth

pytestmark = pytest.mark.gpu
H16 = torch.float16


# ----------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 8, 9, 11])
@pytest.mark.parametrize("M,N,K", [(1154, 3072, 1024), (37, 1024, 4096), (577 * 3, 768, 1024), (18464, 4096, 1024)])
def test_gemm_f16_variants(dev, variant, M, N, K):
    """Every 16-bit tile family (default per-shape choice, 256x256, 256x128, 8-phase,
    320x256, 128x128) on fp16 operands, fp32 out, float64 reference."""
    if variant in (1, 3, 8) and N % 256:
        pytest.skip("256-wide tile needs N % 256 == 0")
    torch.manual_seed(M * 5 + N)
    a = torch.randn(M, K, device=dev).to(H16)
    w = (torch.randn(N, K, device=dev) * K ** -0.5).to(H16)
    bias = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev)
    _lib.call("aaclip_set_gemm_variant", variant)
    try:
        ops.gemm(a, w, out, bias=bias)
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)
    ref = a.double() @ w.double().T + bias.double()
    assert (out.double() - ref).abs().max().item() < 1e-4 * ref.abs().max().item() + 1e-5


@pytest.mark.parametrize("variant", [0, 3, 8, 9, 11])
def test_gemm_f16_epilogues(dev, variant):
    """fp16 output (bias, bias + GELU), fp32 residual in place + fp16 aux copy, LeakyReLU."""
    torch.manual_seed(11)
    M, N, K = 20 * 577, 1024, 1024
    a = torch.randn(M, K, device=dev).to(H16)
    w = (torch.randn(N, K, device=dev) * 0.03).to(H16)
    bias = torch.randn(N, device=dev)
    base = a.double() @ w.double().T + bias.double()
    _lib.call("aaclip_set_gemm_variant", variant)
    try:
        out = torch.full((M, N), float("nan"), device=dev, dtype=H16)
        ops.gemm(a, w, out, bias=bias)
        assert ((out.double() - base).abs() <= 1e-3 * base.abs() + 1e-4).all()
        ops.gemm(a, w, out, bias=bias, gelu=True)
        ref = torch.nn.functional.gelu(base)
        assert ((out.double() - ref).abs() <= 1e-3 * ref.abs() + 1e-4).all()  # fp16 rounding + 2.6e-5 GELU fit
        x = torch.randn(M, N, device=dev)
        x0 = x.clone()
        aux = torch.empty(M, N, device=dev, dtype=H16)
        ops.gemm(a, w, x, bias=bias, residual=x, aux=aux)
        assert (x.double() - (base + x0.double())).abs().max().item() < 1e-4
        assert torch.equal(aux, x.to(H16))
        out32 = torch.empty(M, N, device=dev)
        ops.gemm(a, w, out32, leaky=True)
        ref = torch.nn.functional.leaky_relu(a.double() @ w.double().T, 0.01)
        assert (out32.double() - ref).abs().max().item() < 1e-4
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)


def test_gemm_f16_identity_and_remap(dev):
    """A = I with an asymmetric B (a transposed write would show), 16-bit output
    columns in place, and the patch-row remap with its fp16 aux copy."""
    M = N = K = 256
    a = torch.eye(M, K, device=dev, dtype=H16)
    w = (torch.arange(N * K, device=dev, dtype=torch.float32).reshape(N, K) % 97).to(H16)
    out = torch.empty(M, N, device=dev, dtype=H16)
    ops.gemm(a, w, out)
    torch.testing.assert_close(out, w.T.contiguous(), atol=0, rtol=0)
    B, P, K, N = 3, 576, 640, 1024
    a = torch.randn(B * P, K, device=dev).to(H16)
    w = (torch.randn(N, K, device=dev) * 0.04).to(H16)
    x = torch.randn(B * (P + 1), N, device=dev)
    x0 = x.clone()
    aux = torch.zeros(B * (P + 1), N, device=dev, dtype=H16)
    ops.gemm(a, w, x, residual=x, aux=aux, row_group=P, row_group_out=P + 1, row_offset=1)
    ref = (a.double() @ w.double().T).view(B, P, N) + x0.view(B, P + 1, N)[:, 1:].double()
    xv = x.view(B, P + 1, N)
    assert torch.equal(xv[:, 0], x0.view(B, P + 1, N)[:, 0])
    assert (xv[:, 1:].double() - ref).abs().max().item() < 1e-4
    assert torch.equal(aux.view(B, P + 1, N)[:, 1:], xv[:, 1:].to(H16))


def test_gemm_rejects_mixed_16bit(dev):
    a = torch.randn(64, 64, device=dev).to(H16)
    w = torch.randn(128, 64, device=dev).to(H16)
    with pytest.raises(TypeError):
        ops.gemm(a, w, torch.empty(64, 128, device=dev, dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        ops.gemm(a, w, torch.empty(64, 128, device=dev), residual=torch.zeros(64, 128, device=dev),
                 aux=torch.empty(64, 128, device=dev, dtype=torch.bfloat16))


# ----------------------------------------------------------------------------- attention
def _attn_ref(qkv, B, N, H, causal):
    q, k, v = qkv.double().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q * 0.125) @ k.transpose(-1, -2)
    if causal:
        s = s + torch.triu(torch.full((N, N), float("-inf"), device=s.device, dtype=s.dtype), 1)
    return (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(B * N, H * 64)


SL2 = 0.125 * 1.4426950408889634


@pytest.mark.parametrize("pre", [False, True])
@pytest.mark.parametrize("B,N,H,causal", [(2, 577, 16, False), (3, 77, 12, True), (1, 1025, 16, False),
                                          (1, 1370, 16, False), (2, 5, 2, False), (2, 73, 4, False),
                                          (4, 130, 4, True)])
def test_attention_f16(dev, B, N, H, causal, pre):
    torch.manual_seed(B * N + H)
    qkv = (torch.randn(B * N, 3 * H * 64, device=dev) * 1.5).to(H16)
    ref_in = qkv.double()
    if pre:  # q in the log2 domain, as the engine folds it into the Q projection
        qkv[:, :H * 64] = (qkv[:, :H * 64].float() * SL2).to(H16)
        ref_in = qkv.double()
        ref_in[:, :H * 64] /= SL2
    out = torch.empty(B * N, H * 64, device=dev, dtype=H16)
    ops.attention(qkv, out, B, N, H, causal=causal, q_prescaled=pre)
    ref = _attn_ref(ref_in, B, N, H, causal)
    err = (out.double() - ref).abs().max().item()
    assert err < 4e-3, err  # bf16 bound is 3e-2: P and the output round to fp16 (2^-11)


# ----------------------------------------------------------------------------- end to end
@pytest.fixture(scope="module")
def weights(dev):
    sd = synth.clip_state_dict(111)
    ia, _ = synth.adapter_state_dicts(111)
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    return vp, {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}


def test_visual_f16_contract(dev, golden, weights):
    """fp16 mode vs the reference's golden B=2 forward: every map pixel inside the
    north_star envelope (1e-3 abs + 1e-2 rel), patch labels identical wherever the
    reference's own margin exceeds 1e-3 on the x100 scale (cos margin 1e-5), image
    labels identical, Medical map too."""
    eng = VisualEngine(*weights, dtype=H16)
    e = golden["e2e"]
    x = torch.from_numpy(synth.images(111, 2, 336)).to(dev)
    T = torch.from_numpy(e["T"]).to(dev)
    seg, det = eng.forward(x)
    grid = np.stack([(100.0 * (f @ T)).cpu().numpy() for f in seg], axis=1)
    ref_grid = e["grid_A"]
    sure = np.abs(ref_grid[..., 1] - ref_grid[..., 0]) > 1e-3
    flips_sure = int((grid.argmax(-1) != ref_grid.argmax(-1))[sure].sum())
    maps, score = eng.predict(x, T, "Industrial")
    maps, score = maps.cpu().numpy(), score.cpu().numpy()
    err = np.abs(maps[0] - e["map_ind0"])
    print(f"fp16: map max abs {err.max():.3e}, grid max abs {np.abs(grid - ref_grid).max():.3e}, "
          f"flips (sure) {flips_sure}/{int(sure.sum())}")
    assert (err <= 1e-3 + 1e-2 * np.abs(e["map_ind0"])).all(), err.max()
    assert flips_sure == 0
    np.testing.assert_allclose(score, e["score"], atol=2e-4)
    assert np.array_equal(score > 0.5, e["score"] > 0.5)
    np.testing.assert_allclose(det.cpu().numpy(), e["det"], atol=5e-4, rtol=5e-3)
    med, _ = eng.predict(x, T, "Medical")
    np.testing.assert_allclose(med.cpu().numpy()[:, ::7, ::7], e["map_med_sub"], atol=1e-3, rtol=1e-2)


def test_visual_f16_c5_golden(dev, golden):
    """448 px (1025 tokens), 6 levels, relu projections in fp16 vs the reference's C5 golden."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_c5.npz"))
    lv = tuple(int(v) for v in g["levels"])
    sd = synth.clip_state_dict(111, img_size=448)
    ia, _ = synth.adapter_state_dicts(111, relu=True, n_levels=len(lv))
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    eng = VisualEngine(vp, {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}, levels=lv, dtype=H16)
    T = torch.from_numpy(golden["text"]["bottle_T_adapted"]).to(dev)
    x = torch.from_numpy(synth.images(111, 1, 448)).to(dev)
    maps, score = eng.predict(x, T, "Medical")
    ref = g["map_med_sub"]
    err = np.abs(maps.cpu().numpy()[:, ::8, ::8] - ref)
    print("fp16 c5 map max abs err", err.max())
    assert (err <= 1e-3 + 1e-2 * np.abs(ref)).all()
    np.testing.assert_allclose(score.cpu().numpy(), g["score"], atol=2e-4)
    # patch labels over all 6 levels x 1024 patches: exact where the reference's margin > 1e-3
    seg, _ = eng.forward(x)
    grid = np.stack([(100.0 * (f @ T)).cpu().numpy() for f in seg], axis=1)
    sure = np.abs(g["grid_A"][..., 1] - g["grid_A"][..., 0]) > 1e-3
    flips = int((grid.argmax(-1) != g["grid_A"].argmax(-1))[sure].sum())
    print(f"fp16 c5 patch-label flips (sure) {flips}/{int(sure.sum())}")
    assert flips == 0


def test_f16_batch_composition_invariance(dev, weights):
    """Per-image bits do not depend on batch size, position or stream chunking (fp16)."""
    eng = VisualEngine(*weights, dtype=H16)
    g = torch.Generator(device=dev).manual_seed(9)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    x = torch.randn(5, 3, 336, 336, device=dev, generator=g)
    ref = [eng.predict(x[i:i + 1], T, "Industrial")[0].clone() for i in range(5)]
    ref = torch.cat(ref)
    for streams in (1, 2, (1, 4)):
        m, _ = eng.predict(x, T, "Industrial", streams=streams)
        assert torch.equal(m, ref), streams


def test_concurrent_chunk_pins(dev, weights):
    """Two 16-image chunks on two streams pin the 8-phase GEMM for their wide block
    shapes while they are enqueued (aaclip_gemm_concurrent, thread-local): the maps and scores
    are bit-identical to one stream (same K order), and the heuristic is back afterwards."""
    from aaclip import _lib
    eng = VisualEngine(*weights, dtype=H16)
    g = torch.Generator(device=dev).manual_seed(5)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    x = torch.randn(32, 3, 336, 336, device=dev, generator=g)
    M = 16 * 577
    plan = lambda: _lib.lib().aaclip_gemm_plan(_lib.F16, M, 4096, 1024).decode()  # noqa: E731
    before = plan()
    m1, s1 = (t.clone() for t in eng.predict(x, T, "Industrial", streams=1))
    m2, s2 = eng.predict(x, T, "Industrial", streams=2)
    bad = [i for i in range(32) if not torch.equal(m1[i], m2[i])]
    nan = [i for i in range(32) if torch.isnan(m2[i]).any()]
    assert not bad and torch.equal(s1, s2), (bad, nan)
    assert plan() == before
