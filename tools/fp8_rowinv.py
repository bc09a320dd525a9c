"""fp8 MX ops: are rows of a 1025-row call bit-identical to the same rows inside a
7175-row call? (debug aid for batch-composition invariance)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import ops  # noqa: E402

dev = torch.device("cuda:0")
FP8 = torch.float8_e4m3fn
torch.manual_seed(0)
K, N = 1024, 3072
big = torch.randn(7175, K, device=dev)
small = big[:1025].clone()


def mx(a):
    a8 = torch.empty(a.shape[0], a.shape[1], device=dev, dtype=FP8)
    sc = ops.mx_scales(a.shape[0], a.shape[1], dev)
    ops.quant_fp8_mx(a, a8, sc)
    return a8, sc


b8, bsc = mx(big)
s8, ssc = mx(small)
print("quant rows equal:", torch.equal(b8[:1025].view(torch.uint8), s8.view(torch.uint8)),
      "scales equal:", torch.equal(bsc[:, :1025], ssc[:, :1025]))
w = (torch.randn(N, K, device=dev) * K ** -0.5)
sw = (w.abs().amax(1) / 448).contiguous()
w8 = (w / sw[:, None]).to(FP8)
bias = torch.randn(N, device=dev) * 0.1
ob = torch.empty(7175, N, device=dev, dtype=torch.bfloat16)
os_ = torch.empty(1025, N, device=dev, dtype=torch.bfloat16)
ops.gemm_fp8mx(b8, bsc, w8, sw, ob, bias=bias)
ops.gemm_fp8mx(s8, ssc, w8, sw, os_, bias=bias)
print("gemm bf16-out rows equal:", torch.equal(ob[:1025], os_), (ob[:1025].float() - os_.float()).abs().max().item())
# GELU fp8 MX output (c_fc)
N2 = 4096
w2 = (torch.randn(N2, K, device=dev) * K ** -0.5)
sw2 = (w2.abs().amax(1) / 448).contiguous()
w28 = (w2 / sw2[:, None]).to(FP8)
b2 = torch.randn(N2, device=dev) * 0.1
fb = torch.empty(7175, N2, device=dev, dtype=FP8)
fbs = ops.mx_scales(7175, N2, dev)
fs = torch.empty(1025, N2, device=dev, dtype=FP8)
fss = ops.mx_scales(1025, N2, dev)
ops.gemm_fp8mx(b8, bsc, w28, sw2, fb, out_sc=fbs, bias=b2, gelu=True)
ops.gemm_fp8mx(s8, ssc, w28, sw2, fs, out_sc=fss, bias=b2, gelu=True)
print("gelu fp8 rows equal:", torch.equal(fb[:1025].view(torch.uint8), fs.view(torch.uint8)),
      "scales:", torch.equal(fbs[:, :1025], fss[:, :1025]))
# attention MX output
H = 16
qkv = (torch.randn(7 * 1025, 3 * H * 64, device=dev)).bfloat16()
ab = torch.empty(7 * 1025, H * 64, device=dev, dtype=FP8)
abs_ = ops.mx_scales(7 * 1025, H * 64, dev)
as_ = torch.empty(1025, H * 64, device=dev, dtype=FP8)
ass = ops.mx_scales(1025, H * 64, dev)
ops.attention(qkv, ab, 7, 1025, H, out_sc=abs_, q_prescaled=True)
ops.attention(qkv[:1025].contiguous(), as_, 1, 1025, H, out_sc=ass, q_prescaled=True)
print("attn fp8 rows equal:", torch.equal(ab[:1025].view(torch.uint8), as_.view(torch.uint8)),
      "scales:", torch.equal(abs_[:, :1025], ass[:, :1025]))
x = torch.randn(7175, K, device=dev)
lw, lb = torch.randn(K, device=dev), torch.randn(K, device=dev)
hb = torch.empty(7175, K, device=dev, dtype=FP8)
hbs = ops.mx_scales(7175, K, dev)
hs = torch.empty(1025, K, device=dev, dtype=FP8)
hss = ops.mx_scales(1025, K, dev)
ops.layernorm(x, lw, lb, hb, y_sc=hbs)
ops.layernorm(x[:1025].contiguous(), lw, lb, hs, y_sc=hss)
print("layernorm fp8 rows equal:", torch.equal(hb[:1025].view(torch.uint8), hs.view(torch.uint8)),
      "scales:", torch.equal(hbs[:, :1025], hss[:, :1025]))
