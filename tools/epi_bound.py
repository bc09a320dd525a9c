"""How much of the timed two-stream C2 step the GEMM epilogues cost: the same captured step
with the GEMM epilogue skipped (aaclip_set_gemm_variant bit 9) or only its global stores
skipped (bit 10), on workspaces that a normal replay has filled with real activations first
(so every kernel still multiplies data-like operands: zero-filled operands raise the clock,
which would flatter the skipped arms). Diagnostic only -- the skipped arms compute garbage.
usage: python tools/epi_bound.py [--rounds 3] [--variants 0,512,1024]"""
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,512,1024")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--streams", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    vp, ad = synthetic_visual_weights(dev)
    eng = VisualEngine(vp, ad, dtype=torch.bfloat16)
    B, S = 32, 336
    g = torch.Generator(device=dev).manual_seed(111)
    x = torch.randn(B, 3, S, S, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    run = eng.graphed_predict(B, S, "Industrial", streams=a.streams)
    for _ in range(3):
        run(x, T)  # the graph's workspaces now hold this batch's activations
    torch.cuda.synchronize()
    slot0 = run.slot0  # graphed_predict's private workspace slots
    graphs = {}
    for v in [int(s) for s in a.variants.split(",")]:
        _lib.call("aaclip_set_gemm_variant", v)  # read at launch: baked into this capture
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            eng.predict(x, T, "Industrial", streams=a.streams, _slot0=slot0)
        graphs[v] = gr
    _lib.call("aaclip_set_gemm_variant", 0)
    run(x, T)  # refill with real activations
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for v, gr in graphs.items():
            for _ in range(3):
                gr.replay()
            e0.record()
            for _ in range(a.steps):
                gr.replay()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            print(f"round {r} gemm_variant {v}: {ms:.3f} ms/step  {B / ms * 1e3:.1f} img/s", flush=True)
            run(x, T)  # back to real activations before the next arm
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
