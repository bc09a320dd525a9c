"""Which GEMM kernel names does rocprofv3 report for the fp8 (C5) engine, eager vs
hipGraph replay? Checks the profiler's attribution of graph-launched dispatches
(run under rocprofv3 --kernel-trace; the eager and graphed phases are separated
by a marker copy)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
import bench  # noqa: E402
from aaclip.engine import VisualEngine  # noqa: E402

dev = torch.device("cuda:0")
lv = (4, 8, 12, 16, 20, 24)
vp, ad = bench.synthetic_visual_weights(dev, seed=448, n_levels=len(lv), n_tok=1025)
eng = VisualEngine(vp, ad, levels=lv, dtype=torch.float8_e4m3fn)
x = torch.randn(4, 3, 448, 448, device=dev)
T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev), dim=0).contiguous()
eng.predict(x, T, "Industrial")
torch.cuda.synchronize()
run = eng.graphed_predict(4, 448, "Industrial", streams=1)
run(x, T)
torch.cuda.synchronize()
print("ok")
