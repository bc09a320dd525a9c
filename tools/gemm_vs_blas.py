"""Headroom check for the block GEMMs: our kernels (default per-shape dispatch and
forced tile families) against the vendor library on the same operands
(torch.nn.functional.linear on ROCm -> hipBLASLt, bf16 in / bf16 out with bias),
graph-timed, interleaved in one process. The library is a yardstick only: the
product GEMMs carry fused epilogues (GELU, residual + aux copy, row remap).
usage: python tools/gemm_vs_blas.py [--variants 0,3,8] [--M 18464,9232]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import _lib, ops  # noqa: E402
from tools.map_bench import graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,3,8")
    ap.add_argument("--M", default="18464,9232")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for M in [int(x) for x in a.M.split(",")]:
        for (N, K, name) in ((3072, 1024, "qkv"), (1024, 1024, "out"), (4096, 1024, "fc"), (1024, 4096, "proj")):
            x = torch.randn(M, K, device=dev, generator=g).bfloat16()
            w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
            bias = torch.randn(N, device=dev, generator=g)
            bias16 = bias.bfloat16()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * M * N * K
            res = []
            for rnd in range(2):
                for v in [int(t) for t in a.variants.split(",")]:
                    if v in (1, 3, 8) and N % 256:
                        continue
                    _lib.call("aaclip_set_gemm_variant", v)
                    t = graph_time(lambda: ops.gemm(x, w, out, bias=bias), reps=20)
                    if rnd:
                        res.append(f"v{v} {t:7.1f} us {fl / t / 1e6:6.0f} TF")
                _lib.call("aaclip_set_gemm_variant", 0)
                t = graph_time(lambda: torch.nn.functional.linear(x, w, bias16), reps=20)
                if rnd:
                    res.append(f"hipBLASLt {t:7.1f} us {fl / t / 1e6:6.0f} TF")
            print(f"M={M} {name:4s} N={N} K={K}: " + " | ".join(res), flush=True)
            del x, w, out


if __name__ == "__main__":
    main()
