"""A/B the per-GPU batch split over concurrent HIP streams (engine.predict
streams=1..4), interleaved rounds in one process; also checks that every split
gives bit-identical maps/scores (images are independent)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aa-clip_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from aaclip.engine import VisualEngine  # noqa: E402
from bench import synthetic_visual_weights  # noqa: E402

dev = torch.device("cuda:0")
vp, ad = synthetic_visual_weights(dev)
eng = VisualEngine(vp, ad, dtype=torch.bfloat16)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
settings = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3,4").split(",")]
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(B, 3, 336, 336, device=dev, generator=g)
T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
ref_m, ref_s = [t.clone() for t in eng.predict(x, T, streams=1)]
best = {}
for rnd in range(3):
    for s in settings:
        m, sc = eng.predict(x, T, streams=s)
        torch.cuda.synchronize()
        assert torch.equal(m, ref_m) and torch.equal(sc, ref_s), f"streams={s} changed the result"
        t0 = time.perf_counter()
        for _ in range(10):
            eng.predict(x, T, streams=s)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        best[s] = min(best.get(s, 1e9), dt)
for s in settings:
    print(f"B={B} streams={s}: {best[s]*1e3:7.2f} ms/step  {B/best[s]:8.1f} img/s")
