"""Search the GEMM tile-family pins in the REAL pipeline (two-stream C2 step as one
hipGraph) by coordinate descent over the block-GEMM shapes, starting from the
isolated-kernel tuner's choice. Prints each trial and the best assignment.
usage: python tools/pin_search.py [--streams 2] [--batch 32] [--steps 20] [--dtype bf16]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
import bench  # noqa: E402
from aaclip import _lib, ops  # noqa: E402
from aaclip.engine import VisualEngine, WIDTH  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--passes", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[a.dtype]
    tag = ops.dtag(torch.empty(0, dtype=dt))
    vp, ad = bench.synthetic_visual_weights(dev)
    eng = VisualEngine(vp, ad, dtype=dt)
    g = torch.Generator(device=dev).manual_seed(111)
    x = torch.randn(a.batch, 3, 336, 336, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    chunk = a.batch // a.streams
    M = chunk * 577
    shapes = {"qkv": (M, 3 * WIDTH, WIDTH), "out": (M, WIDTH, WIDTH), "fc": (M, 4 * WIDTH, WIDTH),
              "proj": (M, WIDTH, 4 * WIDTH), "adapter": (M, WIDTH, WIDTH)}
    eng.predict(x, T, "Industrial", streams=a.streams)  # workspaces + isolated tuning
    torch.cuda.synchronize()
    cur = {k: ops._tuned.get((tag,) + v, 0) for k, v in shapes.items()}
    # out and adapter share (M, N, K): one pin
    cur.pop("adapter")

    def trial(assign):
        for k, (m, n, kk) in shapes.items():
            if k == "adapter":
                continue
            _lib.call("aaclip_gemm_pin", tag, m, n, kk, assign[k])
        run = eng.graphed_predict(a.batch, 336, "Industrial", streams=a.streams)
        for _ in range(3):
            run(x, T)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            run(x, T)
        torch.cuda.synchronize()
        dt_ = (time.perf_counter() - t0) / a.steps * 1e3
        del run
        return dt_

    best_t = trial(cur)
    print("start", json.dumps(cur), round(best_t, 3), flush=True)
    fams = {"qkv": (3, 8, 1, 9), "out": (3, 8, 1, 9, 2), "fc": (3, 8, 1, 9), "proj": (3, 8, 1, 9, 2)}
    for _ in range(a.passes):
        for k, opts in fams.items():
            for f in opts:
                if f == cur[k]:
                    continue
                cand = dict(cur, **{k: f})
                t = trial(cand)
                print(k, f, round(t, 3), flush=True)
                if t < best_t * 0.995:
                    best_t, cur = t, cand
    print("best", json.dumps(cur), round(best_t, 3), "images/s", round(a.batch / best_t * 1e3, 1), flush=True)


if __name__ == "__main__":
    main()
