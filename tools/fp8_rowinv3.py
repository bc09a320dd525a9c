"""MX GEMM: which M / scale-ld combinations go wrong (debug aid)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import ops  # noqa: E402

dev = torch.device("cuda:0")
FP8 = torch.float8_e4m3fn
torch.manual_seed(0)
K, N = 1024, 1024
w = torch.randn(N, K, device=dev) * K ** -0.5
sw = (w.abs().amax(1) / 448).contiguous()
w8 = (w / sw[:, None]).to(FP8)
Wd = w8.double() * sw.double()[:, None]
for M in (1025, 1026, 1027, 1028, 1029, 1153, 1154, 7175, 1031, 1024 + 255):
    for ld in (M, M + 1, (M + 3) // 4 * 4):
        a = torch.randn(M, K, device=dev)
        a8 = torch.empty(M, K, device=dev, dtype=FP8)
        sc = ops.mx_scales(M, K, dev, ld=ld)
        ops.quant_fp8_mx(a, a8, sc)
        s = sc[:, :M, :].permute(1, 0, 2).reshape(M, K // 64).double() - 127.0
        A = a8.double() * torch.pow(2.0, s).repeat_interleave(64, dim=1)
        out = torch.empty(M, N, device=dev)
        ops.gemm_fp8mx(a8, sc, w8, sw, out)
        e = (out.double() - A @ Wd.T).abs().amax(1)
        bad = (e > 1e-3).nonzero().flatten()
        print(f"M={M} ld={ld}: max err {e.max().item():.3g} bad rows {len(bad)} "
              f"{bad[:4].tolist()}..{bad[-2:].tolist() if len(bad) else ''}")
