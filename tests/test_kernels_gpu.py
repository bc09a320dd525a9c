"""Per-kernel parity on the MI355X: each HIP kernel vs a plain fp32 reference
(torch fp32 / float64 on the host for the floating-point kernels, the numpy
oracle for the row ops, the reference's own golden vectors where they exist).
All calls go through the C ABI (libaaclip_hip.so via aaclip.ops)."""
import numpy as np
import pytest
import torch

from aaclip import _lib, ops
from oracle import aaclip_np as R

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


# ----------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(1154, 3072, 1024), (1154, 1024, 4096), (37, 768, 1024), (513, 1536, 1024),
                                   (600, 4096, 1024), (256 * 9, 2304, 768)])
def test_gemm_bf16_plain(dev, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(dev)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev)
    ab, wb = a.bfloat16(), w.bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.float32)
    ops.gemm(ab, wb, out)
    ref = ab.double() @ wb.double().T
    err = (out.double() - ref).abs().max().item()
    assert err < 1e-3 * ref.abs().max().item() + 1e-4, err


@pytest.mark.parametrize("variant", [1, 2, 3, 8, 9, 11])
@pytest.mark.parametrize("M,N,K", [(1154, 3072, 1024), (37, 1024, 4096), (577 * 3, 768, 1024), (2000, 256, 64),
                                   (18464, 3072, 1024), (577 * 40, 1024, 512), (300, 512, 128)])
def test_gemm_bf16_variants(dev, variant, M, N, K):
    """Forced bf16 tile families (256x256, 256x128, 256x256 8-phase ping-pong, 320x256,
    128x128, 64x64); the default picks among them per shape and is covered by every other
    GEMM test."""
    from aaclip import _lib
    if variant in (1, 3, 8) and N % 256:
        pytest.skip("256x256 tile needs N % 256 == 0")
    torch.manual_seed(M * 7 + N)
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev)
    _lib.call("aaclip_set_gemm_variant", variant)
    try:
        ops.gemm(a, w, out, bias=bias)
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)
    ref = a.double() @ w.double().T + bias.double()
    assert (out.double() - ref).abs().max().item() < 1e-3 * ref.abs().max().item() + 1e-4


@pytest.mark.parametrize("gelu", [False, True])
@pytest.mark.parametrize("M,N", [(18464, 3072), (18464, 4096), (577 * 3, 512), (100, 256)])
def test_gemm_bf16_out_epilogue(dev, gelu, M, N):
    """bf16-output epilogue (QKV: bias; c_fc: bias + GELU) at the C2 shapes and ragged
    small ones: rows leave straight from the accumulators (C^T tile, lane = one row x 4
    columns, permlane16-paired into 16-B stores); float64 reference."""
    K = 1024
    torch.manual_seed(M + N + gelu)
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev) * 0.5
    out = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, out, bias=bias, gelu=gelu)
    ref = a.double() @ w.double().T + bias.double()
    if gelu:
        ref = torch.nn.functional.gelu(ref)
    err = (out.double() - ref).abs()
    assert not torch.isnan(out).any()
    assert (err <= 8e-3 * ref.abs() + 2e-3).all(), err.max().item()


def _qgelu(x):
    return x * torch.sigmoid(1.702 * x)  # reference model/transformer.py:46-49


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 8, 9, 11])
def test_gemm_quick_gelu_epilogue(dev, dtype, variant):
    """AACLIP_EPI_QGELU (towers built with quick_gelu=True) on every tile family, 16-bit
    and fp32 outputs, a ragged last M-tile; float64 reference. The fp32 kernel keeps
    the exact expf form: 1e-5 relative."""
    if dtype == torch.float32 and variant:
        pytest.skip("the fp32 kernel has one tile family")
    M, N, K = 3 * 577, 4096, 1024
    torch.manual_seed(variant)
    a = torch.randn(M, K, device=dev).to(dtype)
    w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dtype)
    bias = torch.randn(N, device=dev) * 0.5
    ref = _qgelu(a.double() @ w.double().T + bias.double())
    _lib.call("aaclip_set_gemm_variant", variant)
    try:
        for odt in ((torch.float32,) if dtype == torch.float32 else (dtype, torch.float32)):
            out = torch.full((M, N), float("nan"), device=dev, dtype=odt)
            ops.gemm(a, w, out, bias=bias, gelu="quick")
            err = (out.double() - ref).abs()
            tol = 1e-5 * ref.abs() + 1e-5 if odt == torch.float32 and dtype == torch.float32 else \
                (8e-3 * ref.abs() + 2e-3 if odt != torch.float32 else 1e-3 * ref.abs() + 1e-3)
            assert not torch.isnan(out).any()
            assert (err <= tol).all(), (odt, err.max().item())
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)
    with pytest.raises(ValueError):
        ops.gemm(a, w, out, bias=bias, gelu="tanh")


def test_gemm_gelu_flags_exclusive(dev):
    """GELU and QuickGELU together, or an unknown epilogue bit, are rejected by the C ABI."""
    a = torch.randn(64, 64, device=dev).bfloat16()
    w = torch.randn(256, 64, device=dev).bfloat16()
    out = torch.empty(64, 256, device=dev)
    bias = torch.zeros(256, device=dev)
    for epi in (_lib.EPI_BIAS | _lib.EPI_GELU | _lib.EPI_QGELU, 128):
        with pytest.raises(RuntimeError):
            _lib.call("aaclip_gemm", _lib.BF16, _lib.F32, 64, 256, 64, a.data_ptr(), 64, w.data_ptr(), 64,
                      out.data_ptr(), 256, epi, bias.data_ptr(), None, 0, None, 0, 0, 0, 0,
                      torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("variant", [3])
@pytest.mark.parametrize("M,N,K", [(18464, 4096, 1024), (4100, 3072, 4096), (513, 256, 192), (9232, 1024, 4096)])
def test_gemm_8phase_race_screen(dev, variant, M, N, K):
    """The 8-phase kernel's LDS hand-offs are placed by vmcnt/barrier counting: a read
    placed too early passes whenever the DMA happens to land first, so screen many
    launches for run-to-run differences (bit-identical expected) and check one
    against float64."""
    from aaclip import _lib
    torch.manual_seed(M + N)
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
    outs = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    _lib.call("aaclip_set_gemm_variant", variant)
    try:
        ops.gemm(a, w, outs[0])
        ref = a.double() @ w.double().T
        assert ((outs[0].double() - ref).abs() <= 8e-3 * ref.abs() + 2e-3).all()
        for _ in range(12):
            ops.gemm(a, w, outs[1])
            assert torch.equal(outs[0], outs[1])
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(18464, 3072, 1024), (9232, 1024, 4096), (577 * 3, 1536, 1024), (300, 256, 192),
                                   (577, 1024, 4096), (577, 768, 1024)])
def test_gemm_families_bit_identical(dev, dt, M, N, K):
    """Every 16-bit tile family accumulates the K dimension in the same order (32-element
    MFMA k-slices, ascending, one fp32 accumulator per output), so their outputs are
    bit-identical -- the engine may pick any family per shape, stream count and batch
    without changing an image's bits. Covers the 8-phase, 320x256, 128x128 and 64x64 kernels
    on every epilogue the engine uses: bf16 out with bias; bias + GELU and bias + QuickGELU
    (16-bit out); fp32 out with residual; fp32 out with residual + 16-bit aux copy; LeakyReLU
    (fp32 out, no bias: the adapters); and the run-time-flag epilogue with the output row
    remap (patch rows -> token rows after the CLS slot: the patch-embedding GEMM)."""
    g = torch.Generator(device=dev).manual_seed(M + K)
    a = torch.randn(M, K, device=dev, generator=g).to(dt)
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
    bias = torch.randn(N, device=dev, generator=g)
    res = torch.randn(M, N, device=dev, generator=g)
    fams = [f for f in (0, 3, 8, 9, 11) if N % 256 == 0 or f in (0, 9, 11)]
    rg = 577 if M % 577 == 0 else 0  # row remap: groups of 577 rows -> 578 with row 0 left out
    outs, extra = [], []
    for f in fams:
        _lib.call("aaclip_set_gemm_variant", f)
        try:
            o16 = torch.empty(M, N, device=dev, dtype=dt)
            ops.gemm(a, w, o16, bias=bias)
            o32 = res.clone()
            ops.gemm(a, w, o32, bias=bias, residual=o32)
            x32 = res.clone()
            xaux = torch.empty(M, N, device=dev, dtype=dt)
            ops.gemm(a, w, x32, bias=bias, residual=x32, aux=xaux)
            ge = torch.empty(M, N, device=dev, dtype=dt)
            ops.gemm(a, w, ge, bias=bias, gelu=True)
            qg = torch.empty(M, N, device=dev, dtype=dt)
            ops.gemm(a, w, qg, bias=bias, gelu="quick")
            lk = torch.empty(M, N, device=dev)
            ops.gemm(a, w, lk, leaky=True)
            rm = None
            if rg:
                rm = torch.zeros(M // rg * (rg + 1), N, device=dev)
                ops.gemm(a, w, rm, row_group=rg, row_group_out=rg + 1, row_offset=1)
        finally:
            _lib.call("aaclip_set_gemm_variant", 0)
        outs.append((o16, o32, x32, xaux))
        extra.append((ge, qg, lk, rm))
    ref = (a.double() @ w.double().T + bias.double()) + res.double()
    assert ((outs[0][1].double() - ref).abs() <= 2e-2 * ref.abs() + 2e-2).all()
    assert torch.equal(outs[0][2], outs[0][1])
    assert torch.equal(outs[0][3], outs[0][1].to(dt))
    for f, (o16, o32, x32, xaux) in zip(fams[1:], outs[1:]):
        assert torch.equal(o16.view(torch.int16), outs[0][0].view(torch.int16)), f
        assert torch.equal(o32, outs[0][1]), f
        assert torch.equal(x32, outs[0][2]), f
        assert torch.equal(xaux.view(torch.int16), outs[0][3].view(torch.int16)), f
    for f, (ge, qg, lk, rm) in zip(fams[1:], extra[1:]):
        assert torch.equal(ge.view(torch.int16), extra[0][0].view(torch.int16)), (f, "gelu")
        assert torch.equal(qg.view(torch.int16), extra[0][1].view(torch.int16)), (f, "quick_gelu")
        assert torch.equal(lk, extra[0][2]), (f, "leaky")
        if rg:
            assert torch.equal(rm, extra[0][3]), (f, "row remap")
    if rg:  # the remap itself: token row 0 of each group untouched, the rest = the plain product
        rm = extra[0][3].view(M // rg, rg + 1, N)
        assert (rm[:, 0] == 0).all()
        lk_ref = torch.empty(M, N, device=dev)
        ops.gemm(a, w, lk_ref)
        assert torch.equal(rm[:, 1:].reshape(M, N), lk_ref)


def test_gemm_bf16_asymmetric_identity(dev):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    M = N = K = 256
    a = torch.eye(M, K, device=dev, dtype=torch.bfloat16)
    w = (torch.arange(N * K, device=dev, dtype=torch.float32).reshape(N, K) % 97).bfloat16()
    out = torch.empty(M, N, device=dev)
    ops.gemm(a, w, out)
    torch.testing.assert_close(out, w.float().T, atol=0, rtol=0)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 8, 9, 11])
def test_gemm_epilogues_bf16(dev, variant):
    from aaclip import _lib
    _lib.call("aaclip_set_gemm_variant", variant)
    try:
        _epilogues(dev)
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)


def _epilogues(dev):
    torch.manual_seed(0)
    M, N, K = 20 * 577, 1024, 1024  # ragged last M-tile
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.03).bfloat16()
    bias = torch.randn(N, device=dev)
    base = a.double() @ w.double().T + bias.double()
    # bias + gelu -> bf16
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, out, bias=bias, gelu=True)
    ref = torch.nn.functional.gelu(base)
    assert (out.double() - ref).abs().max().item() < 2e-2
    # leaky -> fp32
    out32 = torch.empty(M, N, device=dev)
    ops.gemm(a, w, out32, leaky=True)
    ref = torch.nn.functional.leaky_relu(a.double() @ w.double().T, 0.01)
    assert (out32.double() - ref).abs().max().item() < 1e-3
    # bias + residual in place + aux bf16 copy
    x = torch.randn(M, N, device=dev)
    x0 = x.clone()
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, x, bias=bias, residual=x, aux=aux)
    ref = base + x0.double()
    assert (x.double() - ref).abs().max().item() < 1e-3
    assert torch.equal(aux, x.bfloat16())
    # leaky + residual -> bf16 (8-column bf16 store path with the residual prefetch)
    r = torch.randn(M, N, device=dev)
    outb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, outb, bias=bias, leaky=True, residual=r)
    ref = torch.nn.functional.leaky_relu(base, 0.01) + r.double()
    assert (outb.double() - ref).abs().max().item() < 3e-2


def test_gemm_bf16_out_identity(dev):
    """A = I, bf16 output: every output column lands where it belongs (8-wide stores)."""
    M, N, K = 640, 512, 640
    a = torch.eye(M, K, device=dev, dtype=torch.bfloat16)
    w = (torch.arange(N * K, device=dev, dtype=torch.float32).reshape(N, K) % 89).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, out)
    torch.testing.assert_close(out, w.T.contiguous(), atol=0, rtol=0)


def test_gemm_row_remap_residual(dev):
    """Row remap applies to the residual read and to the aux copy as well."""
    B, P, K, N = 3, 576, 640, 1024
    a = torch.randn(B * P, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.04).bfloat16()
    x = torch.randn(B * (P + 1), N, device=dev)
    x0 = x.clone()
    aux = torch.zeros(B * (P + 1), N, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, x, residual=x, aux=aux, row_group=P, row_group_out=P + 1, row_offset=1)
    ref = (a.double() @ w.double().T).view(B, P, N) + x0.view(B, P + 1, N)[:, 1:].double()
    xv = x.view(B, P + 1, N)
    assert torch.equal(xv[:, 0], x0.view(B, P + 1, N)[:, 0])
    assert (xv[:, 1:].double() - ref).abs().max().item() < 1e-3
    assert torch.equal(aux.view(B, P + 1, N)[:, 1:], xv[:, 1:].bfloat16())
    assert torch.all(aux.view(B, P + 1, N)[:, 0] == 0)


def test_gemm_row_remap(dev):
    """Patch-embedding rows land after each image's CLS slot (row_group)."""
    B, P, K, N = 3, 576, 640, 1024
    a = torch.randn(B * P, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.04).bfloat16()
    x = torch.full((B * (P + 1), N), 7.0, device=dev)
    ops.gemm(a, w, x, row_group=P, row_group_out=P + 1, row_offset=1)
    ref = (a.double() @ w.double().T).view(B, P, N)
    xv = x.view(B, P + 1, N)
    assert torch.all(xv[:, 0] == 7.0)
    assert (xv[:, 1:].double() - ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("M,N,K", [(577 * 2, 3072, 1024), (77 * 6, 768, 3072), (33, 64, 16)])
def test_gemm_f32(dev, M, N, K):
    a = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) * K ** -0.5
    b = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev)
    ops.gemm(a, w, out, bias=b)
    ref = a.double() @ w.double().T + b.double()
    assert (out.double() - ref).abs().max().item() < 2e-5 * (K ** 0.5)


# ----------------------------------------------------------------------------- attention
def _attn_ref(qkv, B, N, H, causal):
    D = H * 64
    q, k, v = qkv.double().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q * 0.125) @ k.transpose(-1, -2)
    if causal:
        s = s + torch.triu(torch.full((N, N), float("-inf"), device=s.device, dtype=s.dtype), 1)
    o = torch.softmax(s, -1) @ v
    return o.permute(0, 2, 1, 3).reshape(B * N, D)


@pytest.mark.parametrize("B,N,H,causal", [(2, 577, 16, False), (3, 77, 12, True), (1, 1025, 16, False),
                                          (2, 5, 2, False), (4, 130, 4, True),
                                          # key tails of 8 (inline per-key updates), 9 (masked tile), 0
                                          (2, 72, 4, False), (2, 73, 4, False), (1, 64, 2, False), (3, 136, 2, False)])
def test_attention_bf16(dev, B, N, H, causal):
    torch.manual_seed(B * N + H)
    qkv = (torch.randn(B * N, 3 * H * 64, device=dev) * 1.5).bfloat16()
    out = torch.empty(B * N, H * 64, device=dev, dtype=torch.bfloat16)
    ops.attention(qkv, out, B, N, H, causal=causal)
    ref = _attn_ref(qkv, B, N, H, causal)
    err = (out.double() - ref).abs().max().item()
    assert err < 3e-2, err


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,N,H,causal", [(2, 577, 16, False), (3, 77, 12, True), (2, 73, 4, False),
                                          (1, 200, 2, False)])
def test_attention_variants(dev, variant, dt, B, N, H, causal):
    """aaclip_set_attn_variant: 1 = the un-split full tile, 2 = 2 waves x 64 queries with a
    2-stage ring (the benchmarked alternatives to the default) against the same float64
    reference."""
    torch.manual_seed(B * N + 7)
    qkv = (torch.randn(B * N, 3 * H * 64, device=dev) * 1.5).to(dt)
    out = torch.empty(B * N, H * 64, device=dev, dtype=dt)
    _lib.call("aaclip_set_attn_variant", variant)
    try:
        ops.attention(qkv, out, B, N, H, causal=causal)
    finally:
        _lib.call("aaclip_set_attn_variant", 0)
    err = (out.double() - _attn_ref(qkv, B, N, H, causal)).abs().max().item()
    assert err < (3e-2 if dt == torch.bfloat16 else 4e-3), err


@pytest.mark.parametrize("B,N,H,causal", [(2, 577, 16, False), (3, 77, 12, True)])
def test_attention_f32(dev, B, N, H, causal):
    torch.manual_seed(1)
    qkv = torch.randn(B * N, 3 * H * 64, device=dev)
    out = torch.empty(B * N, H * 64, device=dev)
    ops.attention(qkv, out, B, N, H, causal=causal)
    ref = _attn_ref(qkv, B, N, H, causal)
    assert (out.double() - ref).abs().max().item() < 1e-5


def test_attention_spiky_rows(dev):
    """Force the online-softmax rescale: one key spikes late in the sequence."""
    B, N, H = 1, 577, 2
    qkv = torch.randn(B * N, 3 * H * 64, device=dev) * 0.1
    qkv[:, :64] = 1.0
    qkv[500, H * 64:H * 64 + 64] = 3.0  # key 500, head 0: huge logit for every query
    for dt in (torch.bfloat16, torch.float32):
        x = qkv.to(dt)
        out = torch.empty(B * N, H * 64, device=dev, dtype=dt)
        ops.attention(x, out, B, N, H)
        ref = _attn_ref(x, B, N, H, False)
        assert (out.double() - ref).abs().max().item() < (2e-2 if dt == torch.bfloat16 else 1e-5)


SL2 = 0.125 * 1.4426950408889634  # log2(e)/sqrt(64), what the engine folds into the Q projection


def _prescale_q(qkv, H):
    """q columns * log2(e)/8 rounded to bf16 (the engine's folded weights give the same rounding
    point); returns the prescaled tensor and the unscaled (double) q it represents."""
    x = qkv.clone()
    x[:, :H * 64] = (qkv[:, :H * 64].float() * SL2).bfloat16()
    ref_in = x.double()
    ref_in[:, :H * 64] /= SL2
    return x, ref_in


@pytest.mark.parametrize("B,N,H,causal", [(2, 577, 16, False), (3, 77, 12, True), (1, 1025, 16, False),
                                          (2, 5, 2, False), (4, 130, 4, True)])
def test_attention_bf16_q_prescaled(dev, B, N, H, causal):
    """AACLIP_ATTN_Q_PRESCALED: q already in the log2 domain (engine default for bf16/fp8)."""
    torch.manual_seed(B * N + H + 1)
    qkv = (torch.randn(B * N, 3 * H * 64, device=dev) * 1.5).bfloat16()
    x, ref_in = _prescale_q(qkv, H)
    out = torch.empty(B * N, H * 64, device=dev, dtype=torch.bfloat16)
    ops.attention(x, out, B, N, H, causal=causal, q_prescaled=True)
    ref = _attn_ref(ref_in, B, N, H, causal)
    err = (out.double() - ref).abs().max().item()
    assert err < 3e-2, err


def test_attention_deferred_max_paths(dev):
    """The running max moves only when a tile beats it by > 2^8: a slowly rising key
    norm (max creeps up ~2 log2-units per tile: deferred, p grows up to 256) and a
    late spike (+35 log2-units: the rescale branch) both match the float64 softmax."""
    B, N, H = 2, 577, 2
    torch.manual_seed(3)
    qkv = torch.randn(B * N, 3 * H * 64, device=dev) * 0.1
    qkv[:, :64] = 1.0  # head 0: every query = ones
    ramp = torch.arange(N, device=dev, dtype=torch.float32).repeat(B) / N * 2.0
    qkv[:, H * 64:H * 64 + 64] = ramp[:, None]  # head 0 keys: logits rise with the key index
    qkv[500, H * 64 + 64:H * 64 + 128] = 3.0  # head 1, key 500: a late spike (head-1 queries are small)
    qkv[:, 64:128] = 1.0
    for pre in (False, True):
        x = qkv.bfloat16()
        ref_in = x.double()
        if pre:
            x, ref_in = _prescale_q(x, H)
        out = torch.empty(B * N, H * 64, device=dev, dtype=torch.bfloat16)
        ops.attention(x, out, B, N, H, q_prescaled=pre)
        ref = _attn_ref(ref_in, B, N, H, False)
        assert (out.double() - ref).abs().max().item() < 2e-2, pre


# ----------------------------------------------------------------------------- rows
def test_layernorm_vs_reference(dev, golden):
    o = golden["ops"]
    x = torch.from_numpy(o["ln_x"]).to(dev)
    from oracle import synth
    sd = synth.clip_state_dict(111)
    w = torch.from_numpy(sd["visual.ln_pre.weight"]).to(dev)
    b = torch.from_numpy(sd["visual.ln_pre.bias"]).to(dev)
    y = torch.empty_like(x)
    ops.layernorm(x, w, b, y)
    np.testing.assert_allclose(y.cpu().numpy(), o["ln_y"], atol=2e-5, rtol=1e-5)


def test_block_tail_and_embed(dev):
    rng = np.random.default_rng(0)
    B, n_tok, D = 2, 577, 1024
    x = rng.standard_normal((B * n_tok, D), dtype=np.float32)
    u = rng.standard_normal((B * n_tok, D), dtype=np.float32)
    lw, lb = (1 + 0.1 * rng.standard_normal(D)).astype(np.float32), (0.1 * rng.standard_normal(D)).astype(np.float32)
    pw, pb = (1 + 0.1 * rng.standard_normal(D)).astype(np.float32), (0.1 * rng.standard_normal(D)).astype(np.float32)
    X = torch.from_numpy(x).to(dev)
    H = torch.empty(B * n_tok, D, device=dev)
    tap = torch.empty(B * (n_tok - 1), D, device=dev)
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    ops.block_tail(X, n_tok, u=t(u), adapt_weight=0.1, ln=(t(lw), t(lb)), h=H, post=(t(pw), t(pb)), tap=tap)
    xn = np.linalg.norm(x, axis=-1, keepdims=True)
    un = np.linalg.norm(u, axis=-1, keepdims=True)
    xr = 0.1 * (u * xn / un) + 0.9 * x
    np.testing.assert_allclose(X.cpu().numpy(), xr, atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(H.cpu().numpy(), R.layer_norm(xr, lw, lb), atol=1e-4, rtol=1e-4)
    tr = R.layer_norm(xr.reshape(B, n_tok, D)[:, 1:], pw, pb).reshape(-1, D)
    np.testing.assert_allclose(tap.cpu().numpy(), tr, atol=1e-4, rtol=1e-4)


# ----------------------------------------------------------------------------- im2col
@pytest.mark.parametrize("S", [336, 448, 518, 28])
@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16])
def test_im2col_exact(dev, S, dt):
    """aaclip_im2col (conv1 as a GEMM, model/adapter.py:68): cols[b*g*g + p, c*196 + kh*14 + kw]
    = img[b, c, 14*py + kh, 14*px + kw] cast to the cols dtype, zero for k >= 588 -- bit-exact
    against torch's unfold, including a misaligned (offset) image view."""
    torch.manual_seed(S)
    B, C, P, kp = 3, 3, 14, 640
    base = torch.randn(B * C * S * S + 1, device=dev)
    for img in (base[:-1].view(B, C, S, S), base[1:].view(B, C, S, S)):
        g = S // P
        cols = torch.full((B * g * g, kp), float("nan"), device=dev, dtype=dt)
        ops.im2col(img, cols, P)
        ref = torch.nn.functional.unfold(img, P, stride=P).transpose(1, 2).reshape(B * g * g, C * P * P)
        torch.cuda.synchronize()
        assert torch.equal(cols[:, :C * P * P], ref.to(dt))
        assert torch.equal(cols[:, C * P * P:], torch.zeros_like(cols[:, C * P * P:]))


# ----------------------------------------------------------------------------- anomaly map
@pytest.mark.parametrize("dom", ["Industrial", "Medical"])
def test_similarity_map_golden(dev, golden, dom):
    """Reference calculate_similarity_map (test branch) on a 8x8 grid -> 40x40."""
    o = golden["ops"]
    f = torch.from_numpy(o["sim_f"]).to(dev)  # [2, 64, 32] unit rows, C=32
    T = torch.from_numpy(o["sim_T"]).to(dev)
    # the kernel needs C = 768: embed the 32 channels in 768 zero-padded ones (exact)
    fp = torch.zeros(2 * 64, 768, device=dev)
    fp[:, :32] = f.reshape(-1, 32)
    Tp = torch.zeros(768, 2, device=dev)
    Tp[:32] = T
    grid = torch.empty(2 * 64, device=dev)
    ops.patch_scores([fp], Tp, grid)
    out = torch.empty(2, 1, 40, 40, device=dev)
    k, s = (7, 1.0) if dom == "Industrial" else (9, 1.5)
    ops.blur_upsample(grid.view(2, 1, 8, 8), out, ksize=k, sigma=s)
    np.testing.assert_allclose(out.cpu().numpy(), o[f"sim_test_{dom}"], atol=1e-5, rtol=1e-5)


def test_similarity_map_train_golden(dev, golden):
    o = golden["ops"]
    f = torch.from_numpy(o["sim_f"]).to(dev)
    T = torch.from_numpy(o["sim_T"]).to(dev)
    fp = torch.zeros(2 * 64, 768, device=dev)
    fp[:, :32] = f.reshape(-1, 32)
    Tp = torch.zeros(768, 2, device=dev)
    Tp[:32] = T
    grid = torch.empty(2, 2, 8, 8, device=dev)
    ops.patch_scores([fp], Tp, grid, mode=1, group=64)
    out = torch.empty(2, 2, 40, 40, device=dev)
    ops.blur_upsample(grid, out, ksize=0, sigma=0.0, softmax=True)
    np.testing.assert_allclose(out.cpu().numpy(), o["sim_train"], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_anomaly_map_multi_level(dev, dt):
    rng = np.random.default_rng(3)
    B, g, C, S, L = 3, 24, 768, 336, 4
    feats = [rng.standard_normal((B, g * g, C), dtype=np.float32) for _ in range(L)]
    T = rng.standard_normal((C, 2)).astype(np.float32)
    T /= np.linalg.norm(T, axis=0, keepdims=True)
    lv = [torch.from_numpy(f.reshape(-1, C)).to(dev).to(dt) for f in feats]
    feats = [t.float().cpu().numpy().reshape(B, g * g, C) for t in lv]  # oracle sees the same inputs
    out = torch.empty(B, S, S, device=dev)
    grid = torch.empty(B * g * g, device=dev)
    ops.anomaly_map(lv, torch.from_numpy(T).to(dev), out, grid, g=g, ksize=7, sigma=1.0)
    ref = R.anomaly_map([R.l2_normalize(f) for f in feats], T, S, "Industrial")
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=1e-4, rtol=1e-5)


def test_image_score(dev):
    rng = np.random.default_rng(5)
    B, P, C = 3, 576, 768
    d = rng.standard_normal((B, P, C), dtype=np.float32)
    T = rng.standard_normal((C, 2)).astype(np.float32)
    D = torch.from_numpy(d.reshape(-1, C)).to(dev)
    partial = torch.empty(B * 36 * C, device=dev)
    det = torch.empty(B, C, device=dev)
    score = torch.empty(B, device=dev)
    ops.image_score(D, B, P, partial, det=det, T=torch.from_numpy(T).to(dev), score=score)
    ref_det = R.l2_normalize(d).mean(1)
    np.testing.assert_allclose(det.cpu().numpy(), ref_det, atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(score.cpu().numpy(), R.image_score(ref_det, T), atol=1e-6)


@pytest.mark.parametrize("g,S", [(37, 518), (37, 517), (24, 336), (24, 41), (8, 130), (32, 448), (5, 2), (64, 900)])
@pytest.mark.parametrize("ksize,sigma", [(7, 1.0), (9, 1.5), (0, 0.0)])
def test_blur_upsample_any_size(dev, g, S, ksize, sigma):
    """Band-local blur + bilinear upsample at any output size (518 = the reference's
    default, 518 % 4 = 2: dword-store path) vs the numpy restatement of kornia's
    gaussian_blur2d + ATen's align_corners upsample."""
    if ksize // 2 >= g:
        pytest.skip("kernel wider than the grid")
    rng = np.random.default_rng(g * 1000 + S + ksize)
    B = 3
    grid = rng.standard_normal((B, 1, g, g)).astype(np.float32)
    out = torch.full((B, 1, S, S), float("nan"), device=dev)
    ops.blur_upsample(torch.from_numpy(grid).to(dev), out, ksize=ksize, sigma=sigma)
    ref = R.gaussian_blur2d(grid, ksize, sigma) if ksize else grid
    ref = R.upsample_bilinear_ac(ref, S)
    got = out.cpu().numpy()
    assert not np.isnan(got).any()
    np.testing.assert_allclose(got, ref, atol=2e-6, rtol=1e-5)


@pytest.mark.parametrize("S", [518, 40, 337])
def test_blur_upsample_train_softmax_any_size(dev, S):
    """Train branch (2 channels, no blur, softmax over channels) at odd output sizes."""
    rng = np.random.default_rng(S)
    g = 37 if S == 518 else 8
    grid = (rng.standard_normal((2, 2, g, g)) * 3).astype(np.float32)
    out = torch.empty(2, 2, S, S, device=dev)
    ops.blur_upsample(torch.from_numpy(grid).to(dev), out, ksize=0, sigma=0.0, softmax=True)
    ref = R.softmax(R.upsample_bilinear_ac(grid, S), axis=1)
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,g,S,L,dom", [(3, 24, 336, 4, "Industrial"), (2, 37, 518, 4, "Medical"),
                                         (2, 32, 448, 6, "Medical"), (5, 8, 41, 1, "Industrial")])
def test_anomaly_map_equals_stages(dev, dt, B, g, S, L, dom):
    """aaclip_anomaly_map is bit-identical to patch_scores + blur_upsample, launch after
    launch, at the C2 / 518 / C5 shapes and a ragged small one."""
    torch.manual_seed(B * g + S)
    lv = [torch.randn(B * g * g, 768, device=dev).to(dt) for _ in range(L)]
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev), dim=0).contiguous()
    k, s = (7, 1.0) if dom == "Industrial" else (9, 1.5)
    grid2 = torch.empty(B * g * g, device=dev)
    ops.patch_scores(lv, T, grid2)
    ref = torch.empty(B, 1, S, S, device=dev)
    ops.blur_upsample(grid2.view(B, 1, g, g), ref, ksize=k, sigma=s)
    ws = torch.empty(B * g * g, device=dev)
    for _ in range(3):
        out = torch.full((B, S, S), float("nan"), device=dev)
        ops.anomaly_map(lv, T, out, ws, g=g, ksize=k, sigma=s)
        assert torch.equal(out, ref[:, 0])


# ----------------------------------------------------------------------------- NaN propagation
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("where", ["q", "k", "v"])
def test_attention_nan_propagates_like_reference(dev, dt, where):
    """A NaN in the packed qkv (e.g. an upstream fp16 overflow) reaches exactly the
    outputs it reaches in the reference's softmax(q k^T) v: a NaN in one query row ->
    that row of that head; in one key or value row -> every query of that head (N = 577
    with its key tail, 16 heads). The attention TU is built with -fno-honor-nans for its
    score max: this screens that the flag never turns a NaN into a finite output, and
    that the other heads and rows are unaffected."""
    B, N, H = 2, 577, 16
    torch.manual_seed(5)
    qkv = (torch.randn(B * N, 3 * H * 64, device=dev) * 1.5).to(dt)
    col = {"q": 0, "k": H * 64, "v": 2 * H * 64}[where] + 3 * 64 + 7  # head 3, dim 7
    row = 1 * N + 200  # image 1, token 200
    qkv[row, col] = float("nan")
    out = torch.empty(B * N, H * 64, device=dev, dtype=dt)
    ops.attention(qkv, out, B, N, H)
    ref = _attn_ref(qkv, B, N, H, False)
    assert torch.equal(torch.isnan(out), torch.isnan(ref)), (where, int(torch.isnan(out).sum()),
                                                             int(torch.isnan(ref).sum()))
    fin = ~torch.isnan(ref)
    assert (out.double()[fin] - ref[fin]).abs().max().item() < (3e-2 if dt == torch.bfloat16 else 4e-3)


# ----------------------------------------------------------------------------- train-branch map, any anchor count
@pytest.mark.parametrize("Cn", [1, 3, 8])
def test_similarity_map_train_any_anchor_count(dev, Cn):
    """forward_utils.calculate_similarity_map(test=False) for 1, 3 and 8 anchors at 518 px
    (37x37 grid): 100 f.T -> [B, Cn, g, g] -> bilinear align_corners=True to S x S ->
    softmax over the anchors when Cn > 1 (reference forward_utils.py:199-215), against
    the same formula in fp64 torch."""
    from forward_utils import calculate_similarity_map
    B, g, S = 2, 37, 518
    torch.manual_seed(Cn)
    f = torch.nn.functional.normalize(torch.randn(B, g * g, 768, device=dev), dim=-1)
    T = torch.nn.functional.normalize(torch.randn(768, Cn, device=dev), dim=0)
    got = calculate_similarity_map(f, T, S, test=False)
    A = (100.0 * (f.double() @ T.double())).permute(0, 2, 1).reshape(B, Cn, g, g)
    ref = torch.nn.functional.interpolate(A, size=(S, S), mode="bilinear", align_corners=True)
    if Cn > 1:
        ref = torch.softmax(ref, dim=1)
    assert got.shape == (B, Cn, S, S)
    assert (got.double() - ref).abs().max().item() < (2e-5 if Cn > 1 else 2e-4)


def test_similarity_map_train_rejects_too_many_anchors_before_launch(dev):
    from forward_utils import calculate_similarity_map
    f = torch.randn(1, 24 * 24, 768, device=dev)
    with pytest.raises(ValueError):
        calculate_similarity_map(f, torch.randn(768, 9, device=dev), 336, test=False)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,g,L", [(3, 24, 4), (2, 37, 4), (2, 32, 6), (1, 5, 1), (1, 9, 8)])
def test_image_score_strided_rows(dev, dt, B, g, L):
    """aaclip_image_score on det rows inside a [rows, (L+1)*768] projection buffer (the
    engine's segbuf layout, levels then det; P not a multiple of the 16-row det chunk
    included) against float64: det = mean_p normalize(det_raw), score = (det.t1 + 1) / 2."""
    torch.manual_seed(B * g + L)
    rows = B * g * g
    buf = torch.randn(rows, (L + 1) * 768, device=dev).to(dt)
    det_raw = buf[:, L * 768:]
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev), dim=0).contiguous()
    part = torch.full((B * ((g * g + 15) // 16) * 768,), float("nan"), device=dev)
    s1, d1 = torch.empty(B, device=dev), torch.empty(B, 768, device=dev)
    ops.image_score(det_raw, B, g * g, part, det=d1, T=T, score=s1)
    f = buf.float().view(B, g * g, L + 1, 768)
    ref_det = torch.nn.functional.normalize(f[:, :, L].double(), dim=-1).mean(1)
    assert (d1.double() - ref_det).abs().max().item() < 1e-6
    ref_score = (ref_det @ T[:, 1].double() + 1) / 2
    assert (s1.double() - ref_score).abs().max().item() < 1e-6


def test_tune_gemm_pins_an_accepted_family(dev):
    """ops.tune_gemm (AACLIP_GEMM_TUNE=1 at workspace creation) measures every family in
    GEMM_FAMILIES on one shape and pins the fastest; every family it tries must be one
    aaclip_gemm_pin accepts (round 5 removed family 10 from the library but not from the
    tuner, so the tuner raised on every block-GEMM shape). Pinning is bit-neutral."""
    from aaclip import _lib
    g = torch.Generator(device=dev).manual_seed(3)
    M, N, K = 577 * 2, 1024, 1024
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    res = torch.randn(M, N, device=dev, generator=g)
    ref = res.clone()
    ops.gemm(a, w, ref, residual=ref)
    out = res.clone()
    try:
        fam = ops.tune_gemm(a, w, torch.empty_like(res), residual=torch.zeros_like(res))
        assert fam in (0,) + ops.GEMM_FAMILIES
        for f in ops.GEMM_FAMILIES:  # the tuner's whole list is pinnable
            assert _lib.lib().aaclip_gemm_pin(_lib.BF16, 7, 1024, 1024, f) == 0
            assert _lib.lib().aaclip_gemm_pin(_lib.BF16, 7, 1024, 1024, 0) == 0
        ops.gemm(a, w, out, residual=out)
        assert torch.equal(out, ref)
    finally:
        _lib.call("aaclip_gemm_pin", _lib.BF16, M, N, K, 0)
        ops._tuned.pop((_lib.BF16, M, N, K), None)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("S", [2, 3, 4])
def test_gemm_ksplit_bits_independent_of_family_and_batch(dev, dt, S):
    """aaclip_gemm_ksplit (the c_proj, K = 4096): every tile family splits K the same way
    (K-steps [h nk / S, (h+1) nk / S)) and the last part sums the partials in index order,
    so the bits of a row depend on neither the family nor M (the rows of 1 image inside a
    batch of 5 = the 1-image launch) -- the batch-composition invariance the engine needs.
    Against float64 within bf16 / fp16 accuracy; every counter back at zero afterwards."""
    K, N = 4096, 1024
    g = torch.Generator(device=dev).manual_seed(S)
    M = 577 * 5
    a = torch.randn(M, K, device=dev, generator=g).to(dt)
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
    bias = torch.randn(N, device=dev, generator=g)
    res = torch.randn(M, N, device=dev, generator=g)
    outs = []
    for f in (0, 3, 8, 9, 11):
        _lib.call("aaclip_set_gemm_variant", f)
        try:
            ws = ops.ksplit_workspace(M, N, K, S, dev)
            x = res.clone()
            xaux = torch.empty(M, N, device=dev, dtype=dt)
            ops.gemm(a, w, x, bias=bias, residual=x, aux=xaux, ksplit=S, ksplit_ws=ws)
            o16 = torch.empty(M, N, device=dev, dtype=dt)
            ops.gemm(a, w, o16, bias=bias, ksplit=S, ksplit_ws=ws)
            ws1 = ops.ksplit_workspace(577, N, K, S, dev)
            x1 = res[:577].clone()
            ops.gemm(a[:577], w, x1, bias=bias, residual=x1, ksplit=S, ksplit_ws=ws1)
            torch.cuda.synchronize()
            assert int(ws[1].abs().sum()) == 0 and int(ws1[1].abs().sum()) == 0, f
        finally:
            _lib.call("aaclip_set_gemm_variant", 0)
        assert torch.isfinite(x).all(), f
        assert torch.equal(x1, x[:577]), f  # one image alone = that image inside a batch
        assert torch.equal(xaux.view(torch.int16), x.to(dt).view(torch.int16)), f
        outs.append((x, o16))
    ref = (a.double() @ w.double().T + bias.double()) + res.double()
    assert ((outs[0][0].double() - ref).abs() <= 2e-2 * ref.abs() + 2e-2).all()
    for x, o16 in outs[1:]:
        assert torch.equal(x, outs[0][0])
        assert torch.equal(o16.view(torch.int16), outs[0][1].view(torch.int16))
    # the split is a different fp32 association than the unsplit GEMM: close, not equal
    x0 = res.clone()
    ops.gemm(a, w, x0, bias=bias, residual=x0)
    assert ((x0 - outs[0][0]).abs() <= 1e-4 * x0.abs() + 1e-4).all()


@pytest.mark.parametrize("S", [2, 3, 4])
def test_gemm_ksplit_race_screen(dev, S):
    """The split parts meet through stored partials and an arrival counter: the last part
    must see every other part's partial. Many launches of a many-tile shape (C2's 16-image
    chunk on the 8-phase kernel) must give the same bits every time and leave the counters
    at zero."""
    K, N, M = 4096, 1024, 9232
    g = torch.Generator(device=dev).manual_seed(7 + S)
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    res = torch.randn(M, N, device=dev, generator=g)
    ws = ops.ksplit_workspace(M, N, K, S, dev)
    first = res.clone()
    ops.gemm(a, w, first, bias=bias, residual=first, ksplit=S, ksplit_ws=ws)
    for _ in range(12):
        x = res.clone()
        ops.gemm(a, w, x, bias=bias, residual=x, ksplit=S, ksplit_ws=ws)
        assert torch.equal(x, first)
    torch.cuda.synchronize()
    assert int(ws[1].abs().sum()) == 0
    ref = (a.double() @ w.double().T + bias.double()) + res.double()
    assert ((first.double() - ref).abs() <= 2e-2 * ref.abs() + 2e-2).all()
