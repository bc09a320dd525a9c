"""Config C5 (448 px, 1025 tokens, 6 levels, B = 32) per-op in-step profile: the eager step with
HIP events around every launch (bench.in_step_profile), one stream and the timed two streams, in
the bf16 and fp8 ("mlp" scope) modes. usage: python tools/c5_profile.py [--modes bf16,fp8]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
import bench  # noqa: E402
from aaclip import ops  # noqa: E402
from aaclip.engine import VisualEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="bf16,fp8")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    S, lv, B = 448, (4, 8, 12, 16, 20, 24), 32
    vp, ad = bench.synthetic_visual_weights(dev, seed=448, n_levels=len(lv), n_tok=(S // 14) ** 2 + 1)
    g = torch.Generator(device=dev).manual_seed(448)
    x = torch.randn(B, 3, S, S, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    out = {}
    for mode in a.modes.split(","):
        kw = dict(dtype=ops.FP8, fp8_scope="mlp") if mode == "fp8" else dict(dtype=torch.bfloat16)
        eng = VisualEngine(vp, ad, levels=lv, **kw)
        prof = {}
        for st in (1, 2):
            p = bench.in_step_profile(eng, x, T, st, replays=4)
            prof[f"streams_{st}"] = {"step_ms_probed": p["step_ms_probed"], "sum_of_launch_ms": p["sum_of_launch_ms"],
                                     "by_op": {k: {kk: v[kk] for kk in ("launches", "ms", "avg_launch_us") if kk in v}
                                               | ({"tflops": v["tflops"]} if "tflops" in v else {})
                                               for k, v in p["by_op"].items()}}
        out[mode] = prof
        for st, p in prof.items():
            print(mode, st, p["step_ms_probed"], p["sum_of_launch_ms"], flush=True)
            for k, v in sorted(p["by_op"].items(), key=lambda kv: -kv[1]["ms"]):
                print(f"   {k:12s} {v['launches']:4d} {v['ms']:8.3f} ms {v['avg_launch_us']:8.2f} us {v.get('tflops', '')}",
                      flush=True)
        del eng
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
