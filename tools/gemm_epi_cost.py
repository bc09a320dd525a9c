"""Epilogue share of the block GEMMs: each C2 block GEMM with its real epilogue
(qkv: bias -> 16-bit; out/proj: bias + fp32 residual in place; fc: bias + GELU ->
16-bit) against the same launch with the global stores skipped (variant bit 10)
and with the whole epilogue skipped (bit 9, accumulators kept live), graph-timed.
usage: python tools/gemm_epi_cost.py [--M 18464,9232]"""
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
    ap.add_argument("--M", default="18464,9232")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for M in [int(x) for x in a.M.split(",")]:
        for (N, K, name, fam) in ((3072, 1024, "qkv", 3), (1024, 1024, "out", 8), (4096, 1024, "fc", 3),
                                  (1024, 4096, "proj", 8)):
            x = torch.randn(M, K, device=dev, generator=g).bfloat16()
            w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
            bias = torch.randn(N, device=dev, generator=g)
            if name in ("out", "proj"):
                out = torch.randn(M, N, device=dev, generator=g)
                call = lambda: ops.gemm(x, w, out, bias=bias, residual=out)  # noqa: E731
            else:
                out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                call = lambda: ops.gemm(x, w, out, bias=bias, gelu=name == "fc")  # noqa: E731
            fl = 2.0 * M * N * K
            res = []
            for rnd in range(2):
                for tag, v in (("default", 0), (f"fam{fam}", fam), ("fam3", 3), ("persist", 5), ("no-stores", fam | 1024),
                               ("no-epilogue", fam | 512)):
                    _lib.call("aaclip_set_gemm_variant", v)
                    t = graph_time(call, reps=20)
                    if rnd:
                        res.append(f"{tag} {t:7.1f} us {fl / t / 1e6:5.0f} TF")
                _lib.call("aaclip_set_gemm_variant", 0)
            print(f"M={M} {name:4s} N={N} K={K}: " + " | ".join(res), flush=True)
            del x, w, out


if __name__ == "__main__":
    main()
