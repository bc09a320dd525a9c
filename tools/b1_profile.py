"""bs=1 whole-path replay (config C1's shape on the GPU), for rocprofv3 kernel stats."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
import bench  # noqa: E402
from aaclip.engine import VisualEngine  # noqa: E402

dev = torch.device("cuda:0")
vp, ad = bench.synthetic_visual_weights(dev)
eng = VisualEngine(vp, ad, dtype=torch.bfloat16)
T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev), dim=0).contiguous()
x = torch.randn(1, 3, 336, 336, device=dev)
run = eng.graphed_predict(1, 336, "Industrial", streams=1)
for _ in range(20):
    run(x, T)
torch.cuda.synchronize()
print("ok")
