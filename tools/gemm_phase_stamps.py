"""Where the 8-phase GEMM main loop's time goes, per phase, from inside the kernel: the
diagnostic build `bash tools/ab_build.sh phase_stamps -DAACLIP_PHASE_STAMPS` stamps
s_memtime at the start and the end of each wave's MFMA cluster for K-steps 4..11
(32 phases); run with AACLIP_LIB=ab/phase_stamps.so. Per phase and wave:
  cluster = end - start of its 16-MFMA cluster (ideal 16 x 16 = 256 cycles when the
            MFMA pipe is the wave's alone; the other wave row's reads / DMA issue on the
            same SIMD share its issue port),
  period  = start(p+1) - start(p) (ideal: both rows' clusters back to back = 512),
  outside = period - cluster (trailing barrier, fragment reads, DMA issue, counted wait,
            pre-cluster barrier and lgkmcnt wait).
C2 shapes at 16 images per chunk (M = 9232) and 32 (18464): QKV, c_fc (bias -> bf16,
+GELU), c_proj (K 4096, fp32 residual). Medians / p90 over waves and phases, by wave row.
usage: AACLIP_LIB=ab/phase_stamps.so python tools/gemm_phase_stamps.py [--M 9232,18464]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import _lib, ops  # noqa: E402

NPH = 32  # stamped phases per wave (K-steps 4..11)


def run(M, N, K, epi, dev, g):
    x = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    resid = bool(epi & _lib.EPI_RESID)
    out = torch.randn(M, N, device=dev, generator=g) if resid else torch.empty(M, N, device=dev,
                                                                                  dtype=torch.bfloat16)
    tiles = -(-M // 256) * (N // 256)
    stamps = torch.zeros(tiles * 8 * NPH * 2, device=dev, dtype=torch.int64)

    def call():
        _lib.call("aaclip_gemm", ops.dtag(x), ops.dtag(out), M, N, K, ops._ptr(x), K, ops._ptr(w), K,
                  ops._ptr(out), N, epi, ops._ptr(bias), ops._ptr(out) if resid else None, N if resid else 0,
                  ops._ptr(stamps), 0, 0, 0, 0, ops._stream())

    _lib.call("aaclip_set_gemm_variant", 3 | 2048)  # 8-phase kernel, stamps into the aux pointer
    try:
        for _ in range(5):
            call()
        torch.cuda.synchronize()
    finally:
        _lib.call("aaclip_set_gemm_variant", 0)
    return stamps.view(tiles, 8, NPH, 2).cpu().numpy().astype(np.int64), tiles


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="9232,18464")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    shapes = (("qkv", 3072, 1024, _lib.EPI_BIAS), ("c_fc", 4096, 1024, _lib.EPI_BIAS | _lib.EPI_GELU),
              ("c_proj", 1024, 4096, _lib.EPI_BIAS | _lib.EPI_RESID))
    for name, N, K, epi in shapes:
        for M in [int(v) for v in a.M.split(",")]:
            t, tiles = run(M, N, K, epi, dev, g)
            start, end = t[..., 0], t[..., 1]
            cluster = end - start
            period = start[:, :, 1:] - start[:, :, :-1]
            outside = period - cluster[:, :, :-1]
            row = {}
            for wr in (0, 1):
                sl = slice(4 * wr, 4 * wr + 4)
                q = lambda v: [int(np.median(v)), int(np.percentile(v, 90))]  # noqa: E731
                row[f"row{wr}"] = {"cluster": q(cluster[:, sl]), "period": q(period[:, sl]),
                                   "outside": q(outside[:, sl])}
            k = f"{name} M={M}"
            res[k] = {"tiles": tiles, **row,
                      "mfma_frac_of_period": round(float(np.median(cluster[:, :, :-1]) * 2 / np.median(period)), 3),
                      "ideal_period": 512}
            print(k, json.dumps(res[k]), flush=True)
    if a.out:
        open(a.out, "w").write(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
