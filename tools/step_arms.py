"""Whole two-stream C2 steps (B = 32, bf16, hipGraph) under GEMM tile-family arms, captured
in ONE process and timed in interleaved rounds. An arm is `name=N:K:fam,N:K:fam,...`: the
chunk's block-GEMM shape (rows = the chunk's B*577, N, K) pinned to tile family `fam`
(aaclip_gemm_pin; pins are read at launch, so each capture keeps its own). Same bits in
every arm (every family accumulates K in the same order) -- checked against arm 0. An item
`ksS` sets the engine's c_proj split-K (aaclip_gemm_ksplit, S parts; 0 = unsplit) for that arm
(different bits from the unsplit arms: a different fp32 association); `avN` the attention
variant (aaclip_set_attn_variant), `gvN` the GEMM variant word (aaclip_set_gemm_variant: bits 4-7 =
tile-order group height) captured into that arm.
usage: python tools/step_arms.py base= outproj=1024:1024:8 nk1024=1024:1024:8,1024:4096:8
       [--img-size 448 --levels 4,8,12,16,20,24 --dtype bf16|fp8]  (config C5; fp8 pins only the bf16 GEMMs)"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import _lib  # noqa: E402
from aaclip.engine import VisualEngine  # noqa: E402
from bench import synthetic_visual_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("arms", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--img-size", type=int, default=336)
    ap.add_argument("--levels", default="6,12,18,24")
    ap.add_argument("--dtype", choices=("bf16", "fp8"), default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, S = 32, a.img_size
    lv = tuple(int(v) for v in a.levels.split(","))
    vp, ad = synthetic_visual_weights(dev, seed=S, n_levels=len(lv), n_tok=(S // 14) ** 2 + 1)
    eng = VisualEngine(vp, ad, levels=lv, dtype=torch.bfloat16 if a.dtype == "bf16" else torch.float8_e4m3fn)
    rows = (B // a.streams) * ((S // 14) ** 2 + 1)
    g = torch.Generator(device=dev).manual_seed(111)
    x = torch.randn(B, 3, S, S, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    runs = {}
    for arm in a.arms:
        name, _, spec = arm.partition("=")
        items = [p for p in spec.split(",") if p]
        eng.cproj_ksplit = next((int(p[2:]) for p in items if p.startswith("ks")), 0)
        _lib.call("aaclip_set_attn_variant", next((int(p[2:]) for p in items if p.startswith("av")), 0))
        _lib.call("aaclip_set_gemm_variant", next((int(p[2:]) for p in items if p.startswith("gv")), 0))
        pins = [tuple(int(v) for v in p.split(":")) for p in items if not p[:2] in ("ks", "av", "gv")]
        for n, k, fam in pins:
            _lib.call("aaclip_gemm_pin", _lib.BF16, rows, n, k, fam)
        runs[name] = eng.graphed_predict(B, S, "Industrial", streams=a.streams)  # dispatch baked in
        for n, k, _ in pins:
            _lib.call("aaclip_gemm_pin", _lib.BF16, rows, n, k, 0)
        _lib.call("aaclip_set_attn_variant", 0)
        _lib.call("aaclip_set_gemm_variant", 0)
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
            for _ in range(3):
                run(x, T)
            e0.record()
            for _ in range(a.steps):
                run(x, T)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            print(f"round {r} {name}: {ms:.3f} ms/step  {B / ms * 1e3:.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
