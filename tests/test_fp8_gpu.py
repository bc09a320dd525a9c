"""fp8 path of config C5 ("fp8 MFMA weights", BASELINE.json configs[4]) on the MI355X:
per-row e4m3 quantisation (aaclip_quant_fp8_rows) and the K=128 block-scaled MFMA
GEMM (aaclip_gemm_fp8) against float64 references on the dequantised operands.
The fp8 GEMM is exact products + fp32 accumulation of e4m3 values, so it is
checked tightly against float64 on the SAME quantised operands; the end-to-end fp8
error against the fp32 reference path is reported by tests/test_e2e_gpu.py."""
import pytest
import torch

from aaclip import _lib, ops

pytestmark = pytest.mark.gpu
FP8 = torch.float8_e4m3fn


@pytest.fixture(params=[0, 6], ids=["mx8ph", "mx256"])
def mx_variant(request):
    """MX GEMM kernel family: 0 = the default 8-phase ping-pong kernel with the
    3-slot scale ring, 6 = the 256x256 LDS-DMA kernel."""
    _lib.call("aaclip_set_gemm_variant", request.param)
    yield request.param
    _lib.call("aaclip_set_gemm_variant", 0)


def _quant_ref(x):
    xf = x.float()
    amax = xf.abs().amax(dim=1)
    scale = torch.where(amax > 0, amax * (1.0 / 448.0), torch.ones_like(amax))
    inv = torch.where(amax > 0, 448.0 / amax, torch.ones_like(amax))
    return (xf * inv[:, None]).to(FP8), scale


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,cols", [(1, 8), (37, 1024), (577, 4096), (1000, 768)])
def test_quant_fp8_rows(dev, dtype, rows, cols):
    torch.manual_seed(rows + cols)
    x = (torch.randn(rows, cols, device=dev) * torch.logspace(-3, 3, rows, device=dev)[:, None]).to(dtype)
    x[0, :] = 0 if rows > 1 else x[0, :]
    q = torch.empty(rows, cols, device=dev, dtype=FP8)
    s = torch.empty(rows, device=dev)
    ops.quant_fp8_rows(x, q, s)
    q_ref, s_ref = _quant_ref(x)
    assert torch.equal(s, s_ref)
    # v_cvt_pk_fp8_f32 vs torch's cast: identical except rare one-code differences
    # (measured <= 0.1 % of elements, normal-range rounding ties): allow adjacent codes only
    qi, ri = q.view(torch.uint8).int(), q_ref.view(torch.uint8).int()
    diff = qi != ri
    assert diff.float().mean().item() < 5e-3
    assert ((qi - ri).abs()[diff] <= 1).all()
    deq = q.float() * s[:, None]
    err = (deq - x.float()).abs()
    assert (err <= 2.0 ** -4 * x.float().abs() + s[:, None] * 2.0 ** -9).all()


def _wq(w):
    """Per-output-channel weight quantisation (what the engine does at load time)."""
    amax = w.abs().amax(dim=1).clamp_min(1e-30)
    s = amax / 448.0
    return (w / s[:, None]).to(FP8), s.float().contiguous()


@pytest.mark.parametrize("M,N,K", [(1154, 3072, 1024), (37, 1024, 4096), (577 * 3, 768, 1024), (4100, 4096, 1024),
                                   (300, 256, 128)])
def test_gemm_fp8_plain(dev, M, N, K):
    torch.manual_seed(M * 3 + N + K)
    a = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) * K ** -0.5
    a8 = torch.empty(M, K, device=dev, dtype=FP8)
    sa = torch.empty(M, device=dev)
    ops.quant_fp8_rows(a, a8, sa)
    w8, sw = _wq(w)
    out = torch.empty(M, N, device=dev)
    ops.gemm_fp8(a8, sa, w8, sw, out)
    ref = (a8.double() * sa.double()[:, None]) @ (w8.double() * sw.double()[:, None]).T
    scale = (a8.double().abs() * sa.double()[:, None]) @ (w8.double().abs() * sw.double()[:, None]).T
    err = (out.double() - ref).abs()
    # MFMA fp8 products are exact; its internal K=128 reduction is not a strict fp32
    # fmaf chain (measured <= 1.4e-5 of sum|a*b|)
    assert (err <= 3e-5 * scale + 1e-6).all(), (err / scale).max().item()
    # and the fp8 product approximates the unquantised one at e4m3 precision
    full = a.double() @ w.double().T
    rel = ((out.double() - full).norm() / full.norm()).item()
    assert rel < 0.05, rel


def test_gemm_fp8_identity_asymmetric(dev):
    """A = I with an asymmetric B (small integers, exact in e4m3) pins the operand/accumulator layout."""
    M = N = K = 256
    a8 = torch.eye(M, K, device=dev).to(FP8)
    w = (torch.arange(N * K, device=dev, dtype=torch.float32).reshape(N, K) % 13) - 6
    w8 = w.to(FP8)
    ones_m = torch.ones(M, device=dev)
    ones_n = torch.ones(N, device=dev)
    out = torch.empty(M, N, device=dev)
    ops.gemm_fp8(a8, ones_m, w8, ones_n, out)
    torch.testing.assert_close(out, w.T.contiguous(), atol=0, rtol=0)


@pytest.mark.parametrize("case", ["bias_gelu_bf16", "bias_resid_aux", "leaky", "remap"])
def test_gemm_fp8_epilogues(dev, case):
    torch.manual_seed(7)
    M, N, K = 20 * 577, 1024, 1024
    a = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) * K ** -0.5
    a8 = torch.empty(M, K, device=dev, dtype=FP8)
    sa = torch.empty(M, device=dev)
    ops.quant_fp8_rows(a, a8, sa)
    w8, sw = _wq(w)
    bias = torch.randn(N, device=dev) * 0.1
    y = (a8.double() * sa.double()[:, None]) @ (w8.double() * sw.double()[:, None]).T
    tol = 3e-5 * ((a8.double().abs() * sa.double()[:, None]) @ (w8.double().abs() * sw.double()[:, None]).T) + 1e-6
    if case == "bias_gelu_bf16":
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.gemm_fp8(a8, sa, w8, sw, out, bias=bias, gelu=True)
        ref = torch.nn.functional.gelu(y + bias.double())
        assert ((out.double() - ref).abs() <= 8e-3 * ref.abs() + 2e-3).all()
    elif case == "bias_resid_aux":
        x = torch.randn(M, N, device=dev)
        x0 = x.clone()
        aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.gemm_fp8(a8, sa, w8, sw, x, bias=bias, residual=x, aux=aux)
        ref = y + bias.double() + x0.double()
        assert ((x.double() - ref).abs() <= tol + 1e-6 * ref.abs()).all()
        assert ((aux.double() - ref).abs() <= 8e-3 * ref.abs() + 1e-3).all()
    elif case == "leaky":
        out = torch.empty(M, N, device=dev)
        ops.gemm_fp8(a8, sa, w8, sw, out, leaky=True)
        ref = torch.nn.functional.leaky_relu(y, 0.01)
        assert ((out.double() - ref).abs() <= tol).all()
    else:  # patch rows -> token rows after a CLS slot (patch embedding)
        P = 577 - 1
        Mp = 20 * P
        out = torch.zeros(20 * 577, N, device=dev)
        ops.gemm_fp8(a8[:Mp], sa[:Mp], w8, sw, out, row_group=P, row_group_out=577, row_offset=1)
        ref = y[:Mp].view(20, P, N)
        got = out.view(20, 577, N)
        assert (got[:, 0] == 0).all()
        assert ((got[:, 1:].double() - ref).abs() <= tol[:Mp].view(20, P, N)).all()


# ------------------------------------------------------------------ MX (block-scaled) fp8
def _mx_dequant(q, sc):
    """e4m3 [M,K] + e8m0 [K/128, ld, 2] -> float64 [M,K]."""
    M, K = q.shape
    e = sc[:, :M, :].permute(1, 0, 2).reshape(M, K // 64).double() - 127.0  # [M, K/64]
    return q.double() * torch.pow(2.0, e).repeat_interleave(64, dim=1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,cols", [(1, 128), (37, 1024), (577, 4096), (1000, 768)])
def test_quant_fp8_mx(dev, dtype, rows, cols):
    torch.manual_seed(rows * 7 + cols)
    x = torch.randn(rows, cols, device=dev) * torch.logspace(-4, 4, cols // 64, device=dev).repeat_interleave(64)
    x = x.to(dtype)
    if rows > 1:
        x[1, :64] = 0  # an all-zero block
    q = torch.empty(rows, cols, device=dev, dtype=FP8)
    sc = ops.mx_scales(rows, cols, dev, ld=rows + 3)
    ops.quant_fp8_mx(x, q, sc)
    deq = _mx_dequant(q, sc)
    xf = x.double()
    blk_max = xf.abs().view(rows, cols // 64, 64).amax(-1)
    e = sc[:, :rows, :].permute(1, 0, 2).reshape(rows, cols // 64).double() - 127.0
    # the scale is the smallest power of two keeping the block max <= 448
    nz = blk_max > 0
    assert (blk_max[nz] * torch.pow(2.0, -e[nz]) <= 448).all()
    assert (blk_max[nz] * torch.pow(2.0, -e[nz]) > 224).all()
    step = torch.pow(2.0, e).repeat_interleave(64, dim=1)
    assert ((deq - xf).abs() <= 2.0 ** -4 * xf.abs() + step * 2.0 ** -9).all()


# K = 128 / 256 / 384: nk = 1, 2 (the steady-state loop runs zero times: the prologue hands
# straight to the counted nk-2 tail) and 3 (odd) K-steps of 128
@pytest.mark.parametrize("M,N,K", [(1154, 3072, 1024), (37, 1024, 4096), (577 * 3, 768 + 256, 1024), (300, 256, 128),
                                   (4616, 4096, 256), (4616, 1024, 384), (300, 256, 256)])
def test_gemm_fp8mx(dev, mx_variant, M, N, K):
    torch.manual_seed(M + N * 3 + K)
    a = torch.randn(M, K, device=dev) * torch.logspace(-2, 2, K // 64, device=dev).repeat_interleave(64)
    w = torch.randn(N, K, device=dev) * K ** -0.5
    a8 = torch.empty(M, K, device=dev, dtype=FP8)
    asc = ops.mx_scales(M, K, dev, ld=(M + 7) // 2 * 2)  # padded, even
    ops.quant_fp8_mx(a, a8, asc)
    w8, sw = _wq(w)
    bias = torch.randn(N, device=dev) * 0.1
    out = torch.empty(M, N, device=dev)
    ops.gemm_fp8mx(a8, asc, w8, sw, out, bias=bias)
    A = _mx_dequant(a8, asc)
    Wd = w8.double() * sw.double()[:, None]
    ref = A @ Wd.T + bias.double()
    scale = A.abs() @ Wd.abs().T
    err = (out.double() - ref).abs()
    # relative to sum |a||w|: 3e-5 at K >= 1024; the short-K cases with 1e-2..1e2 K-blocks
    # reach 4.3e-5 (the same bits on both MX kernels: the block-scaled MFMA's own rounding)
    assert (err <= (3e-5 if K >= 1024 else 6e-5) * scale + 1e-6).all(), (err / scale).max().item()


@pytest.mark.parametrize("M", [1025, 7175, 1, 255])
def test_gemm_fp8mx_odd_rows_last_row(dev, mx_variant, M):
    """Odd row counts (one image = 1025 tokens): the last row's scales sit at the very
    end of the scale buffer; with the (even-padded) default ld every row is exact,
    and an odd ld is rejected (the dword scale DMA would drop the last row's scale)."""
    torch.manual_seed(M)
    K, N = 1024, 1024
    a = torch.randn(M, K, device=dev)
    a8 = torch.empty(M, K, device=dev, dtype=FP8)
    asc = ops.mx_scales(M, K, dev)
    ops.quant_fp8_mx(a, a8, asc)
    w8, sw = _wq(torch.randn(N, K, device=dev) * K ** -0.5)
    out = torch.empty(M, N, device=dev)
    ops.gemm_fp8mx(a8, asc, w8, sw, out)
    ref = _mx_dequant(a8, asc) @ (w8.double() * sw.double()[:, None]).T
    err = (out.double() - ref).abs().amax(1)
    assert (err <= 1e-3).all(), err.argmax().item()
    if M % 2:
        odd = ops.mx_scales(M, K, dev, ld=M)
        ops.quant_fp8_mx(a, a8, odd)
        with pytest.raises(ValueError):
            ops.gemm_fp8mx(a8, odd, w8, sw, out)


@pytest.mark.parametrize("act", [True, "quick"])
def test_gemm_fp8mx_gelu_fp8_output_chain(dev, mx_variant, act):
    """c_fc -> c_proj hand-off in fp8: the GELU epilogue writes e4m3 + its own e8m0 block
    scales, which feed the next MX GEMM directly (no quantisation pass)."""
    torch.manual_seed(11)
    M, D, F = 577 * 4, 1024, 4096
    h = torch.randn(M, D, device=dev)
    wfc, wpr = torch.randn(F, D, device=dev) * D ** -0.5, torch.randn(D, F, device=dev) * F ** -0.5
    bfc = torch.randn(F, device=dev) * 0.1
    h8 = torch.empty(M, D, device=dev, dtype=FP8)
    hsc = ops.mx_scales(M, D, dev)
    ops.quant_fp8_mx(h, h8, hsc)
    wfc8, sfc = _wq(wfc)
    wpr8, spr = _wq(wpr)
    f8 = torch.empty(M, F, device=dev, dtype=FP8)
    fsc = ops.mx_scales(M, F, dev)
    ops.gemm_fp8mx(h8, hsc, wfc8, sfc, f8, out_sc=fsc, bias=bfc, gelu=act)
    # the fp8 GELU output vs GELU of the exact product of the quantised operands
    pre = _mx_dequant(h8, hsc) @ (wfc8.double() * sfc.double()[:, None]).T + bfc.double()
    g_ref = pre * torch.sigmoid(1.702 * pre) if act == "quick" else torch.nn.functional.gelu(pre)
    g = _mx_dequant(f8, fsc)
    blk = g_ref.abs().view(M, F // 64, 64).amax(-1).repeat_interleave(64, dim=1)
    assert ((g - g_ref).abs() <= 2.0 ** -4 * g_ref.abs() + blk * 2.0 ** -8 + 1e-4).all()
    y = torch.empty(M, D, device=dev)
    ops.gemm_fp8mx(f8, fsc, wpr8, spr, y)
    y_ref = g @ (wpr8.double() * spr.double()[:, None]).T
    scale = g.abs() @ (wpr8.double().abs() * spr.double()[:, None]).T
    assert ((y.double() - y_ref).abs() <= 3e-5 * scale + 1e-6).all()


@pytest.mark.parametrize("K", [1024, 256, 384])
def test_gemm_fp8mx_8ph_race_screen(dev, K):
    """The 8-phase MX kernel places its LDS hand-offs (tiles and the scale ring) by
    vmcnt/barrier counting; repeated launches must be bit-identical. K = 256 / 384 screen
    the counted tail (waits 9/9/9/4 then 2/0/0/0) where the steady-state loop runs zero
    times or once."""
    torch.manual_seed(5 + K)
    M, N = 577 * 8, 4096
    a = torch.randn(M, K, device=dev) * torch.logspace(-1, 1, K // 64, device=dev).repeat_interleave(64)
    a8 = torch.empty(M, K, device=dev, dtype=FP8)
    asc = ops.mx_scales(M, K, dev)
    ops.quant_fp8_mx(a, a8, asc)
    w8, sw = _wq(torch.randn(N, K, device=dev) * K ** -0.5)
    outs = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    try:
        ops.gemm_fp8mx(a8, asc, w8, sw, outs[0])
        _lib.call("aaclip_set_gemm_variant", 6)
        ref = torch.empty_like(outs[0])
        ops.gemm_fp8mx(a8, asc, w8, sw, ref)
        assert torch.equal(outs[0], ref)  # same fp32 sums in the same K order
        _lib.call("aaclip_set_gemm_variant", 0)
        for _ in range(12):
            ops.gemm_fp8mx(a8, asc, w8, sw, outs[1])
            assert torch.equal(outs[0], outs[1])
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)


def test_layernorm_kernels_mx_output(dev):
    """LayerNorm / block-tail / embed rows written straight to MX fp8 equal the MX
    quantisation of the same kernels' fp32 rows, bit for bit (same fp32 values, same
    scaling and rounding); block-tail taps stay bf16."""
    torch.manual_seed(5)
    R, W, n_tok = 577 * 3, 1024, 577
    x = torch.randn(R, W, device=dev) * 3
    w, b = torch.randn(W, device=dev), torch.randn(W, device=dev)
    y32 = torch.empty(R, W, device=dev)
    ops.layernorm(x, w, b, y32)
    q_ref = torch.empty(R, W, device=dev, dtype=FP8)
    s_ref = ops.mx_scales(R, W, dev)
    ops.quant_fp8_mx(y32, q_ref, s_ref)
    q = torch.empty(R, W, device=dev, dtype=FP8)
    s = ops.mx_scales(R, W, dev)
    ops.layernorm(x, w, b, q, y_sc=s)
    assert torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8)) and torch.equal(s[:, :R], s_ref[:, :R])
    # block tail: adapter blend + next ln_1 (MX) + bf16 tap
    u = torch.randn(R, W, device=dev)
    post = (torch.randn(W, device=dev), torch.randn(W, device=dev))
    x1, x2 = x.clone(), x.clone()
    tap1 = torch.empty(R // n_tok * (n_tok - 1), W, device=dev, dtype=torch.bfloat16)
    tap2 = torch.empty_like(tap1)
    h32 = torch.empty(R, W, device=dev)
    ops.block_tail(x1, n_tok, u=u, adapt_weight=0.1, ln=(w, b), h=h32, post=post, tap=None)
    ops.block_tail(x2, n_tok, u=u, adapt_weight=0.1, ln=(w, b), h=q, post=post, tap=tap2, h_sc=s)
    ops.quant_fp8_mx(h32, q_ref, s_ref)
    assert torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8)) and torch.equal(s[:, :R], s_ref[:, :R])
    ops.block_tail(x.clone(), n_tok, u=u, adapt_weight=0.1, ln=None, h=None, post=post, tap=tap1)
    assert torch.equal(tap1, tap2)


@pytest.mark.parametrize("B,N", [(2, 577), (1, 1025), (3, 130)])
def test_attention_mx_output(dev, B, N):
    """The attention epilogue's MX e4m3 output (one e8m0 scale per (row, head)) equals the MX
    quantisation of its fp32-accurate output up to one e4m3 code, and dequantises to the
    bf16 kernel's output within e4m3 precision."""
    torch.manual_seed(B * N)
    H = 16
    qkv = torch.randn(B * N, 3 * H * 64, device=dev).bfloat16()
    o_bf = torch.empty(B * N, H * 64, device=dev, dtype=torch.bfloat16)
    ops.attention(qkv, o_bf, B, N, H)
    o8 = torch.empty(B * N, H * 64, device=dev, dtype=FP8)
    sc = ops.mx_scales(B * N, H * 64, dev)
    ops.attention(qkv, o8, B, N, H, out_sc=sc)
    deq = _mx_dequant(o8, sc)
    ref = o_bf.double()
    blk = ref.abs().view(B * N, H, 64).amax(-1).repeat_interleave(64, dim=1)
    assert ((deq - ref).abs() <= 2.0 ** -4 * ref.abs() + 2.0 ** -8 * blk + 1e-3).all()


def test_attention_mx_output_not_worse_than_requantised_bf16(dev):
    """Quantising in the attention epilogue (from fp32) must be at least as accurate as
    quantising the bf16 output afterwards (double rounding): mean |error| vs the fp32
    attention kernel, and codes differ from the requantised bf16 ones by at most one."""
    torch.manual_seed(3)
    B, N, H = 2, 577, 16
    qkv = torch.randn(B * N, 3 * H * 64, device=dev).bfloat16()
    o32 = torch.empty(B * N, H * 64, device=dev)
    ops.attention(qkv.float(), o32, B, N, H)
    o_bf = torch.empty(B * N, H * 64, device=dev, dtype=torch.bfloat16)
    ops.attention(qkv, o_bf, B, N, H)
    o8 = torch.empty(B * N, H * 64, device=dev, dtype=FP8)
    sc = ops.mx_scales(B * N, H * 64, dev)
    ops.attention(qkv, o8, B, N, H, out_sc=sc)
    r8 = torch.empty_like(o8)
    rsc = ops.mx_scales(B * N, H * 64, dev)
    ops.quant_fp8_mx(o_bf, r8, rsc)
    e_new = (_mx_dequant(o8, sc) - o32.double()).abs().mean().item()
    e_old = (_mx_dequant(r8, rsc) - o32.double()).abs().mean().item()
    assert e_new <= e_old * 1.01, (e_new, e_old)
    sc, rsc = sc[:, :B * N], rsc[:, :B * N]  # the even-ld pad row is never written
    assert torch.equal(sc, rsc) or (sc.int() - rsc.int()).abs().max().item() <= 1
