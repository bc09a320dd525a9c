"""Seeded shape fuzz on the MI355X: random (M, N, K) x tile family x epilogue x 16-bit
dtype for aaclip_gemm, and random (batch, sequence, heads, causal, dtype) for
aaclip_attention (16-bit and the fp32 parity kernel), each against a float64 reference of the same rounded operands.
The fixed-shape tests pin the C2/C5 shapes and the known edges; this sweep covers the
shapes between them (ragged M tiles, K of a single K-step, N = 128, odd batches,
sequences that end anywhere in a 64-key tile or a 128-query workgroup). Seeds are fixed,
so a failure names a reproducible case."""
import numpy as np
import pytest
import torch

from aaclip import _lib, ops

pytestmark = pytest.mark.gpu

FAMILIES = (0, 1, 2, 3, 8, 9, 11)  # default dispatch + every forced tile family


def _gemm_case(seed):
    rng = np.random.default_rng(1000 + seed)
    fam = int(FAMILIES[seed % len(FAMILIES)])
    n256 = fam in (1, 3, 5, 8)
    M = int(rng.integers(1, 2600))
    N = int(rng.integers(1, 13)) * (256 if n256 else 128)
    K = int(rng.integers(1, 33)) * 64
    dt = torch.float16 if rng.random() < 0.4 else torch.bfloat16
    epi = rng.choice(["none", "bias", "bias_gelu", "leaky", "bias_resid", "bias_resid_aux", "leaky_resid"])
    return fam, M, N, K, dt, str(epi)


@pytest.mark.parametrize("seed", range(28))
def test_gemm_fuzz(dev, seed):
    fam, M, N, K, dt, epi = _gemm_case(seed)
    g = torch.Generator(device=dev).manual_seed(seed)
    a = torch.randn(M, K, device=dev, generator=g).to(dt)
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
    bias = torch.randn(N, device=dev, generator=g) if "bias" in epi else None
    base = a.double() @ w.double().T + (bias.double() if bias is not None else 0.0)
    kw = {"bias": bias}
    if epi == "bias_gelu":
        out = torch.empty(M, N, device=dev, dtype=dt)
        kw["gelu"] = True
        ref = torch.nn.functional.gelu(base)
    elif epi in ("bias_resid", "bias_resid_aux"):
        out = torch.randn(M, N, device=dev, generator=g)
        ref = base + out.double()
        kw["residual"] = out
        if epi == "bias_resid_aux":
            kw["aux"] = torch.empty(M, N, device=dev, dtype=dt)
    elif epi == "leaky_resid":
        r = torch.randn(M, N, device=dev, generator=g)
        out = torch.empty(M, N, device=dev, dtype=dt)
        kw.update(leaky=True, residual=r)
        ref = torch.nn.functional.leaky_relu(base, 0.01) + r.double()
    elif epi == "leaky":
        out = torch.empty(M, N, device=dev)
        kw["leaky"] = True
        ref = torch.nn.functional.leaky_relu(base, 0.01)
    else:
        out = torch.empty(M, N, device=dev, dtype=dt if seed % 2 else torch.float32)
        ref = base
    _lib.call("aaclip_set_gemm_variant", fam)
    try:
        ops.gemm(a, w, out, **kw)
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)
    torch.cuda.synchronize()
    # fp32 accumulation of rounded operands: 1e-3 of the output scale; a 16-bit output
    # adds its own rounding (bf16 2^-8, fp16 2^-11 relative) on top
    rel = 1e-3 if out.dtype == torch.float32 else (8e-3 if dt == torch.bfloat16 else 2e-3)
    err = (out.double() - ref).abs()
    assert torch.isfinite(out).all(), (fam, M, N, K, dt, epi)
    assert (err <= rel * ref.abs() + 2e-3 * max(1.0, ref.abs().max().item())).all(), \
        (fam, M, N, K, dt, epi, err.max().item())
    if epi == "bias_resid_aux":
        assert torch.equal(kw["aux"], out.to(dt)), (fam, M, N, K, dt)


def _attn_ref(qkv, B, N, H, causal):
    q, k, v = qkv.double().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q * 0.125) @ k.transpose(-1, -2)
    if causal:
        s = s.masked_fill(torch.ones(N, N, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(B * N, H * 64)


@pytest.mark.parametrize("seed", range(16))
def test_attention_fuzz(dev, seed):
    rng = np.random.default_rng(2000 + seed)
    B = int(rng.integers(1, 5))
    N = int(rng.integers(1, 1400))
    H = int(rng.choice([1, 2, 12, 16]))
    causal = bool(rng.random() < 0.3)
    dt = torch.float32 if seed % 4 == 1 else (torch.float16 if seed % 3 == 0 else torch.bfloat16)
    variant = int(rng.choice([0, 1, 2, 3]))
    g = torch.Generator(device=dev).manual_seed(seed)
    qkv = (torch.randn(B * N, 3 * H * 64, device=dev, generator=g) * 1.5).to(dt)
    out = torch.empty(B * N, H * 64, device=dev, dtype=dt)
    _lib.call("aaclip_set_attn_variant", variant)
    try:
        ops.attention(qkv, out, B, N, H, causal=causal)
    finally:
        _lib.call("aaclip_set_attn_variant", 0)
    torch.cuda.synchronize()
    ref = _attn_ref(qkv, B, N, H, causal)
    err = (out.double() - ref).abs().max().item()
    # bf16 / fp16: P and O rounded to the 16-bit type (as test_attention_bf16); fp32: the
    # parity-mode kernel (fp32 MFMA products and sums, exp2 in the log2 domain)
    tol = {torch.bfloat16: 3e-2, torch.float16: 4e-3, torch.float32: 2e-5}[dt]
    assert err < tol, (B, N, H, causal, dt, variant, err)
