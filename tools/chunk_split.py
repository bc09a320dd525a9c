"""Images/s of the C2 / C5 paths vs the per-stream chunk split of a B=32 batch
(tile-count quantisation of the per-chunk GEMMs: DESIGN.md §5).
usage: python tools/chunk_split.py [c2|c5]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
import bench  # noqa: E402
from aaclip.engine import VisualEngine  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    dev = torch.device("cuda:0")
    if cfg == "c5":
        S, lv, dts = 448, (4, 8, 12, 16, 20, 24), (torch.float8_e4m3fn, torch.bfloat16)
    else:
        S, lv, dts = 336, (6, 12, 18, 24), (torch.bfloat16,)
    vp, ad = bench.synthetic_visual_weights(dev, seed=S, n_levels=len(lv), n_tok=(S // 14) ** 2 + 1)
    x = torch.randn(32, 3, S, S, device=dev)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev), dim=0).contiguous()
    splits = [(16, 16), (15, 17), (14, 18), (11, 11, 10), (12, 10, 10), (8, 8, 8, 8), (15, 15, 2)]
    for dt in dts:
        eng = VisualEngine(vp, ad, levels=lv, dtype=dt)
        for sp in splits:
            run = eng.graphed_predict(32, S, "Industrial", streams=sp)
            for _ in range(3):
                run(x, T)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                run(x, T)
            torch.cuda.synchronize()
            dt_s = (time.perf_counter() - t0) / 10
            print(f"{cfg} {str(dt).split('.')[-1]:14s} split {str(sp):16s} {32 / dt_s:8.1f} img/s", flush=True)
            del run
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
