"""Isolated c_proj launches (N 1024, K 4096, bias + fp32 residual + bf16 aux: the engine's
epilogue), unsplit vs aaclip_gemm_ksplit with S parts, graph-replayed, HIP events.
usage: python tools/ksplit_bench.py [--rows 9232,18464] [--splits 0,2,3,4]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import ops  # noqa: E402
from bench import time_launches  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="9232,18464")
    ap.add_argument("--splits", default="0,2,3,4")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    K, N = 4096, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    for M in (int(v) for v in a.rows.split(",")):
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        res = torch.randn(M, N, device=dev, generator=g)
        aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for S in (int(v) for v in a.splits.split(",")):
            ws = ops.ksplit_workspace(M, N, K, S, dev) if S > 1 else None
            t = time_launches(lambda: ops.gemm(x, w, res, bias=bias, residual=res, aux=aux, ksplit=S, ksplit_ws=ws),
                              a.reps, torch.cuda.current_stream())
            tf = 2.0 * M * N * K / (t * 1e-3) / 1e12
            print(f"M {M} ksplit {S}: {t * 1e3:.1f} us  {tf:.0f} TF  plan {ops.gemm_plan(1, M, N, K)}", flush=True)


if __name__ == "__main__":
    main()
