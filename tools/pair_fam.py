"""The two-stream pair of one block GEMM (two 16-image chunks, same weight, fork/join in
one graph) under each tile family, against the merged single launch at 2x the rows:
which family to pin per shape when the chunks run in lockstep.
usage: python tools/pair_fam.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import _lib, ops  # noqa: E402
from tools.map_bench import graph_time  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M = 9232
    for N, K, name in ((1024, 4096, "c_proj"), (1024, 1024, "out-proj"), (4096, 1024, "c_fc"), (3072, 1024, "qkv")):
        w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
        bias = torch.randn(N, device=dev, generator=g)
        xs = [torch.randn(M, K, device=dev, generator=g).bfloat16() for _ in range(2)]
        resid = N == 1024
        outs = [torch.randn(M, N, device=dev, generator=g) if resid else
                torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        xm = torch.cat(xs)
        om = torch.cat(outs)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

        def one(x, o):
            if resid:
                ops.gemm(x, w, o, bias=bias, residual=o)
            else:
                ops.gemm(x, w, o, bias=bias, gelu=name == "c_fc")

        def pair():
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            with torch.cuda.stream(s1):
                one(xs[0], outs[0])
            with torch.cuda.stream(s2):
                one(xs[1], outs[1])
            cur.wait_stream(s1)
            cur.wait_stream(s2)

        res = {}
        for rnd in range(3):
            for fam in (0, 3, 5, 8, 9):
                if fam in (3, 5, 8) and N % 256:
                    continue
                _lib.call("aaclip_set_gemm_variant", fam)
                res[("pair", fam)] = min(res.get(("pair", fam), 1e9), graph_time(pair))
                res[("merged", fam)] = min(res.get(("merged", fam), 1e9), graph_time(lambda: one(xm, om)))
            _lib.call("aaclip_set_gemm_variant", 0)
        fl = 2.0 * 2 * M * N * K
        print(f"{name:8s} " + " | ".join(f"{k[0]} f{k[1]} {v:6.1f} us {fl / v / 1e6:4.0f} TF" for k, v in sorted(res.items())),
              flush=True)
        del w, xs, outs, xm, om


if __name__ == "__main__":
    main()
