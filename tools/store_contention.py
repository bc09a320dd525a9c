"""Is the GEMM epilogue's store time set by the CU or by the chip? Times the 8-phase
kernel (family 3) on QKV-like (N 3072, K 1024, bias -> bf16) and out-proj-like
(N 1024, K 1024, bias + fp32 residual) launches at M values whose tile counts span
less than one round to several, with and without the global stores (variant bit 10),
graph-timed. Per-CU-bound stores cost the same per round at any tile count;
HBM-bound ones cost in proportion to the tiles storing together.
usage: python tools/store_contention.py [--M 1024,2048,4096,5376,9232,18464]"""
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
    ap.add_argument("--M", default="1024,2048,4096,5376,9232,18464")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    for (N, K, name) in ((3072, 1024, "qkv"), (1024, 1024, "out")):
        for M in [int(x) for x in a.M.split(",")]:
            x = torch.randn(M, K, device=dev, generator=g).bfloat16()
            w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
            bias = torch.randn(N, device=dev, generator=g)
            if name == "out":
                out = torch.randn(M, N, device=dev, generator=g)
                call = lambda: ops.gemm(x, w, out, bias=bias, residual=out)  # noqa: E731
                sb = M * N * 4
            else:
                out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                call = lambda: ops.gemm(x, w, out, bias=bias)  # noqa: E731
                sb = M * N * 2
            tiles = -(-M // 256) * (N // 256)
            rounds = -(-tiles // cus)
            best = {}
            for _ in range(a.rounds):
                for tag, v in (("stores", 3), ("no-stores", 3 | 1024), ("no-epi", 3 | 512)):
                    _lib.call("aaclip_set_gemm_variant", v)
                    try:
                        t = graph_time(call, reps=20)
                    finally:
                        _lib.call("aaclip_set_gemm_variant", 0)
                    best[tag] = min(best.get(tag, 1e9), t)
            d = best["stores"] - best["no-stores"]
            print(f"{name} M={M:6d} tiles={tiles:4d} rounds={rounds}  stores {best['stores']:7.1f} us  "
                  f"no-stores {best['no-stores']:7.1f}  no-epi {best['no-epi']:7.1f}  store cost {d:6.1f} us "
                  f"= {d / rounds:5.2f} us/round, {sb / max(d, 1e-3) / 1e3:6.0f} GB/s over the store time, "
                  f"{sb / tiles / max(d / rounds, 1e-3) / 1e3 / 2.2:5.1f} B/clk/CU @2.2GHz", flush=True)


if __name__ == "__main__":
    main()
