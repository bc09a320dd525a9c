"""Whole C2 steps (B = 32, bf16, hipGraph) under VisualEngine attribute arms, captured in
ONE process and timed in interleaved rounds (the same-box, same-clock A/B the step
numbers need). An arm is `name=attr:value,attr:value` (value parsed as int, else kept as
a string), set on the engine before its graph is captured; every arm's map and score are
compared bit for bit with arm 0's.
usage: python tools/engine_ab.py base= rows=map_partials:0 [--streams 1] [--dtype fp16]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip.engine import VisualEngine  # noqa: E402
from bench import synthetic_visual_weights  # noqa: E402


def _val(v):
    try:
        return int(v)
    except ValueError:
        return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("arms", nargs="+")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", choices=("bf16", "fp16"), default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    vp, ad = synthetic_visual_weights(dev)
    B, S = a.batch, 336
    g = torch.Generator(device=dev).manual_seed(111)
    x = torch.randn(B, 3, S, S, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    runs = {}
    for arm in a.arms:
        name, _, spec = arm.partition("=")
        eng = VisualEngine(vp, ad, dtype=torch.bfloat16 if a.dtype == "bf16" else torch.float16)
        for kv in filter(None, spec.split(",")):
            k, _, v = kv.partition(":")
            if not hasattr(eng, k):
                sys.exit(f"unknown engine attribute {k}")
            setattr(eng, k, _val(v))
        runs[name] = (eng, eng.graphed_predict(B, S, "Industrial", streams=a.streams))
    ref = None
    for name, (_, run) in runs.items():
        m, s = run(x, T)
        torch.cuda.synchronize()
        if ref is None:
            ref = (m.clone(), s.clone())
        print(f"{name}: bits {'same' if torch.equal(m, ref[0]) and torch.equal(s, ref[1]) else 'DIFF'}", flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {n: [] for n in runs}
    for r in range(a.rounds):
        for name, (_, run) in runs.items():
            for _ in range(3):
                run(x, T)
            e0.record()
            for _ in range(a.steps):
                run(x, T)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            res[name].append(ms)
            print(f"round {r} {name}: {ms:.3f} ms/step = {B / ms * 1e3:.1f} images/s", flush=True)
    for name, v in res.items():
        v = sorted(v)
        print(f"{name}: median {v[len(v) // 2]:.3f} ms, best {v[0]:.3f} ms ({B / v[0] * 1e3:.1f} images/s)")


if __name__ == "__main__":
    main()
