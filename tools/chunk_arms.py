"""Whole hipGraph steps of one engine under different image chunkings (predict(streams=...)
with an explicit chunk-size tuple, or an int = equal chunks), captured in ONE process and
timed in interleaved rounds (HIP events on the replay stream). Per-image bits do not depend
on the chunking (checked against the first arm).
usage: python tools/chunk_arms.py [--img-size 448 --levels 4,8,12,16,20,24 --dtype fp8|bf16]
                                  16,16 15,17 14,18 15,15,2"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import ops  # noqa: E402
from aaclip.engine import VisualEngine  # noqa: E402
from bench import synthetic_visual_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("arms", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--img-size", type=int, default=448)
    ap.add_argument("--levels", default="4,8,12,16,20,24")
    ap.add_argument("--dtype", choices=("bf16", "fp8", "fp16"), default="fp8")
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, S = a.batch, a.img_size
    lv = tuple(int(v) for v in a.levels.split(","))
    vp, ad = synthetic_visual_weights(dev, seed=S, n_levels=len(lv), n_tok=(S // 14) ** 2 + 1)
    kw = {"bf16": dict(dtype=torch.bfloat16), "fp16": dict(dtype=torch.float16),
          "fp8": dict(dtype=ops.FP8, fp8_scope="mlp")}[a.dtype]
    eng = VisualEngine(vp, ad, levels=lv, **kw)
    g = torch.Generator(device=dev).manual_seed(111)
    x = torch.randn(B, 3, S, S, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    dom = "Industrial" if S == 336 else "Medical"
    runs = {}
    for arm in a.arms:
        st = tuple(int(v) for v in arm.split(",")) if "," in arm else int(arm)
        runs[arm] = eng.graphed_predict(B, S, dom, streams=st)
    ref = None
    for name, run in runs.items():
        m, s = run(x, T)
        torch.cuda.synchronize()
        if ref is None:
            ref = (m.clone(), s.clone())
        print(f"{name}: bits {'same' if torch.equal(m, ref[0]) and torch.equal(s, ref[1]) else 'DIFF'}", flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for name, run in runs.items():
            for _ in range(2):
                run(x, T)
            e0.record()
            for _ in range(a.steps):
                run(x, T)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            print(f"round {r} {a.dtype} [{name}]: {ms:.3f} ms/step  {B / ms * 1e3:.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
