"""Cross-step chunk pipelining, measured: the shipped step (one captured graph that forks the
two 16-image chunks onto two streams and joins them at the end of every step) vs two
independent per-chunk graphs replayed on their own streams with no per-step join (each
stream runs its chunk of step k+1 as soon as its chunk of step k is done, so the chunks
never restart in lockstep and never drain one at a time), and the same two graphs joined
every step. Same images, same kernels (the concurrent-chunk GEMM choice is kept for the
per-chunk captures); bits compared against the shipped step.
usage: python tools/pipe_ab.py [--rounds 3] [--steps 20]"""
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    vp, ad = synthetic_visual_weights(dev)
    eng = VisualEngine(vp, ad, dtype=torch.bfloat16)
    B, S, H = 32, 336, 16
    g = torch.Generator(device=dev).manual_seed(111)
    x = torch.randn(B, 3, S, S, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    xa, xb = x[:H].contiguous(), x[H:].contiguous()
    shipped = eng.graphed_predict(B, S, "Industrial", streams=2)
    with ops.concurrent_gemms(True):
        ga = eng.graphed_predict(H, S, "Industrial", streams=1)
        gb = eng.graphed_predict(H, S, "Industrial", streams=1)
    sa, sb = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    main_s = torch.cuda.current_stream(dev)

    m0, s0 = (t.clone() for t in shipped(x, T))
    for st in (sa, sb):
        st.wait_stream(main_s)
    with torch.cuda.stream(sa):
        ma, sca = ga(xa, T)
    with torch.cuda.stream(sb):
        mb, scb = gb(xb, T)
    torch.cuda.synchronize()
    same = torch.equal(torch.cat([ma, mb]), m0) and torch.equal(torch.cat([sca, scb]), s0)
    print(f"per-chunk graphs bits vs shipped step: {'same' if same else 'DIFF'}", flush=True)

    def run_shipped(k):
        for _ in range(k):
            shipped(x, T)

    def run_pipe(k, join):
        for st in (sa, sb):
            st.wait_stream(main_s)
        for _ in range(k):
            with torch.cuda.stream(sa):
                ga(xa, T)
            with torch.cuda.stream(sb):
                gb(xb, T)
            if join:
                main_s.wait_stream(sa)
                main_s.wait_stream(sb)
                sa.wait_stream(main_s)
                sb.wait_stream(main_s)
        main_s.wait_stream(sa)
        main_s.wait_stream(sb)

    arms = {"shipped (fork/join graph)": run_shipped, "two graphs, no join": lambda k: run_pipe(k, False),
            "two graphs, join per step": lambda k: run_pipe(k, True)}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for name, fn in arms.items():
            fn(3)
            torch.cuda.synchronize()
            e0.record()
            fn(a.steps)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            print(f"round {r} {name}: {ms:.3f} ms/step  {B / ms * 1e3:.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
