"""Time the 16-bit attention kernel's workgroup shapes (aaclip_set_attn_variant) at the
C2 / C5 / 518 sequence lengths, GPU time (graph-captured launches), plus a max-error
check of each variant against float64 on a small batch.
usage: python tools/attn_variants.py [--variants 1,2] [--batch 32]
       python tools/attn_variants.py --eager 20 --seqs 577 --variants 1   (plain launches, for rocprofv3 --pmc)"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import _lib, ops  # noqa: E402
from tools.map_bench import graph_time  # noqa: E402


def ref_attn(qkv, B, N, H):
    q, k, v = qkv.double().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    p = torch.softmax((q * 0.125) @ k.transpose(-1, -2), -1)
    return (p @ v).permute(0, 2, 1, 3).reshape(B * N, H * 64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--seqs", default="577,1025,1370")
    ap.add_argument("--eager", type=int, default=0, help="launch each variant this many times, no timing")
    ap.add_argument("--rounds", type=int, default=1, help="interleaved timing rounds (all variants per round)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[a.dtype]
    H = 16
    for N in [int(x) for x in a.seqs.split(",")]:
        qkv = (torch.randn(a.batch * N, 3 * H * 64, device=dev)).to(dt)
        out = torch.empty(a.batch * N, H * 64, device=dev, dtype=dt)
        if a.eager:
            for v in [int(x) for x in a.variants.split(",")]:
                _lib.call("aaclip_set_attn_variant", v)
                for _ in range(a.eager):
                    ops.attention(qkv, out, a.batch, N, H)
            torch.cuda.synchronize()
            continue
        small = qkv[: 2 * N]
        osmall = torch.empty(2 * N, H * 64, device=dev, dtype=dt)
        ref = ref_attn(small, 2, N, H)
        for v in [int(x) for x in a.variants.split(",")]:  # warm-up: the first timed launches read high
            _lib.call("aaclip_set_attn_variant", v)
            graph_time(lambda: ops.attention(qkv, out, a.batch, N, H), reps=5)
        first = None
        for r in range(a.rounds):
            for v in [int(x) for x in a.variants.split(",")]:
                _lib.call("aaclip_set_attn_variant", v)
                t = graph_time(lambda: ops.attention(qkv, out, a.batch, N, H), reps=20)
                ops.attention(small, osmall, 2, N, H)
                err = (osmall.double() - ref).abs().max().item()
                ops.attention(qkv, out, a.batch, N, H)
                if first is None:
                    first = out.clone()
                same = torch.equal(first.view(torch.int16), out.view(torch.int16))
                tf = 4.0 * a.batch * N * N * H * 64 / (t * 1e-6) / 1e12
                print(f"N={N} round={r} variant={v} {t:8.2f} us {tf:7.1f} TFLOP/s  max err {err:.2e}"
                      f"  bits={'same' if same else 'DIFF'}", flush=True)
    _lib.call("aaclip_set_attn_variant", 0)


if __name__ == "__main__":
    main()
