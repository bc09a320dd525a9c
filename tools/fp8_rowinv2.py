"""MX GEMM row-invariance debug: big (7175 rows) vs small (1025 rows) vs float64
reference on the dequantised operands, per kernel variant and output type."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
FP8 = torch.float8_e4m3fn
torch.manual_seed(0)
K, N = 1024, 3072


def mx(a):
    a8 = torch.empty(a.shape[0], a.shape[1], device=dev, dtype=FP8)
    sc = ops.mx_scales(a.shape[0], a.shape[1], dev)
    ops.quant_fp8_mx(a, a8, sc)
    return a8, sc


def deq(a8, sc):
    M, K = a8.shape
    s = sc[:, :M, :].permute(1, 0, 2).reshape(M, K // 64).double() - 127.0
    return a8.double() * torch.pow(2.0, s).repeat_interleave(64, dim=1)


big = torch.randn(7175, K, device=dev)
b8, bsc = mx(big)
s8, ssc = mx(big[:1025].clone())
w = torch.randn(N, K, device=dev) * K ** -0.5
sw = (w.abs().amax(1) / 448).contiguous()
w8 = (w / sw[:, None]).to(FP8)
bias = torch.randn(N, device=dev) * 0.1
ref = deq(s8, ssc) @ (w8.double() * sw.double()[:, None]).T + bias.double()
for v in (0, 6):
    _lib.call("aaclip_set_gemm_variant", v)
    for dt in (torch.bfloat16, torch.float32):
        ob = torch.empty(7175, N, device=dev, dtype=dt)
        os_ = torch.empty(1025, N, device=dev, dtype=dt)
        ops.gemm_fp8mx(b8, bsc, w8, sw, ob, bias=bias)
        ops.gemm_fp8mx(s8, ssc, w8, sw, os_, bias=bias)
        eb = (ob[:1025].double() - ref).abs()
        es = (os_.double() - ref).abs()
        bad_b = (eb > 0.05).nonzero()
        print(f"variant {v} {dt}: big err {eb.max().item():.3g} small err {es.max().item():.3g} "
              f"bad rows big {bad_b[:, 0].unique()[:8].tolist()} cols {bad_b[:, 1].unique()[:8].tolist()} n={len(bad_b)}")
_lib.call("aaclip_set_gemm_variant", 0)
