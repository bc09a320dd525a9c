"""Config C5 (448 px, 6 levels): throughput and map error vs the fp32 parity mode for
bf16, fp8 on all four block GEMMs, and fp8 on the MLP only (fp8_scope='mlp')."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
import bench  # noqa: E402
from aaclip.engine import VisualEngine  # noqa: E402

dev = torch.device("cuda:0")
S, lv = 448, (4, 8, 12, 16, 20, 24)
vp, ad = bench.synthetic_visual_weights(dev, seed=448, n_levels=len(lv), n_tok=(S // 14) ** 2 + 1)
g = torch.Generator(device=dev).manual_seed(448)
x = torch.randn(32, 3, S, S, device=dev, generator=g)
T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
ref = VisualEngine(vp, ad, levels=lv, dtype=torch.float32).predict(x[:4], T, "Medical")[0].clone()
for name, kw in (("bf16", dict(dtype=torch.bfloat16)), ("fp8 all", dict(dtype=torch.float8_e4m3fn)),
                 ("fp8 mlp", dict(dtype=torch.float8_e4m3fn, fp8_scope="mlp"))):
    eng = VisualEngine(vp, ad, levels=lv, **kw)
    m = eng.predict(x[:4], T, "Medical")[0]
    d = m - ref
    run = eng.graphed_predict(32, S, "Medical", streams=2)
    for _ in range(3):
        run(x, T)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        run(x, T)
    torch.cuda.synchronize()
    ips = 32 * 8 / (time.perf_counter() - t0)
    within = float((d.abs() <= 1e-3 + 1e-2 * ref.abs()).float().mean())
    print(f"{name:8s} {ips:8.1f} img/s  map rel-L2 {float(d.norm() / ref.norm()):.4f}  max {float(d.abs().max()):.3f}"
          f"  within fp32 contract {within:.4f}", flush=True)
    del eng, run
    torch.cuda.empty_cache()
