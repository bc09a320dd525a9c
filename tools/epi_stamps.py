"""Where a GEMM epilogue's time goes, per wave, from inside the 8-phase kernel: the
s_memtime stamps of variant bit 11 (kernel start, main loop done, epilogue issued,
epilogue stores complete). QKV-like (N 3072, K 1024, bias -> bf16) and out-proj-like
(N 1024, K 1024, bias + fp32 residual) launches at tile counts from a partial round to
several; per launch round: main loop, epilogue ISSUE (compute + store instructions
accepted) and DRAIN (issued -> complete) in shader cycles, median / p90 over waves.
usage: python tools/epi_stamps.py [--M 1024,5376,9232,18464]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import _lib, ops  # noqa: E402


def run(M, N, K, resid, dev, g):
    x = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    out = torch.randn(M, N, device=dev, generator=g) if resid else torch.empty(M, N, device=dev,
                                                                                  dtype=torch.bfloat16)
    tiles = -(-M // 256) * (N // 256)
    stamps = torch.zeros(tiles * 8 * 4, device=dev, dtype=torch.int64)
    epi = _lib.EPI_BIAS | (_lib.EPI_RESID if resid else 0)

    def call():
        _lib.call("aaclip_gemm", ops.dtag(x), ops.dtag(out), M, N, K, ops._ptr(x), K, ops._ptr(w), K,
                  ops._ptr(out), N, epi, ops._ptr(bias), ops._ptr(out) if resid else None, N if resid else 0,
                  ops._ptr(stamps), 0, 0, 0, 0, ops._stream())

    _lib.call("aaclip_set_gemm_variant", 3 | 2048)
    try:
        for _ in range(3):
            call()
        torch.cuda.synchronize()
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)
    t = stamps.view(tiles, 8, 4).cpu().numpy().astype(np.int64)
    return t, tiles


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="1024,5376,9232,18464")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    for (N, K, name, resid) in ((3072, 1024, "qkv", False), (1024, 1024, "out", True)):
        for M in [int(v) for v in a.M.split(",")]:
            t, tiles = run(M, N, K, resid, dev, g)
            t0 = t[:, :, 0].min()
            start = t[:, :, 0] - t0
            main_loop = t[:, :, 1] - t[:, :, 0]
            issue = t[:, :, 2] - t[:, :, 1]
            drain = t[:, :, 3] - t[:, :, 2]
            end = (t[:, :, 3] - t0).max()
            # launch rounds by workgroup start time
            order = np.argsort(start[:, 0])
            rnd = np.zeros(tiles, dtype=int)
            rnd[order] = np.arange(tiles) // cus
            print(f"{name} M={M:6d} tiles={tiles:4d}: launch span {end:8d} cyc", flush=True)
            for r in range(rnd.max() + 1):
                sel = rnd == r
                q = lambda v: f"{int(np.median(v[sel])):6d}/{int(np.percentile(v[sel], 90)):6d}"  # noqa: E731
                print(f"   round {r} ({sel.sum():3d} tiles) start {q(start)}  main {q(main_loop)}  "
                      f"epi-issue {q(issue)}  drain {q(drain)}  (median/p90 cyc)", flush=True)


if __name__ == "__main__":
    main()
