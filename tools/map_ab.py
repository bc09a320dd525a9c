"""A/B of the per-batch tail: the anomaly map and the image score as separate passes over
the projections (aaclip_anomaly_map + aaclip_image_score) vs one pass
(aaclip_anomaly_map_score), graph-timed in one process on the same segbuf-shaped buffer
(fp32, [B*576, 5*768] at 336 px). usage: python tools/map_ab.py [--batch 32 16]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
import torch  # noqa: E402

from aaclip import ops  # noqa: E402
from bench import time_launches  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, nargs="+", default=[32, 16])
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
res = {}
for B in a.batch:
    g, S, L = 24, 336, 4
    rows = B * g * g
    buf = torch.randn(rows, (L + 1) * 768, device=dev)
    lv = [buf[:, j * 768:(j + 1) * 768] for j in range(L)]
    det_raw = buf[:, L * 768:]
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev), dim=0).contiguous()
    grid = torch.empty(rows, device=dev)
    part = torch.empty(B * 36 * 768, device=dev)
    m, sc, d = torch.empty(B, S, S, device=dev), torch.empty(B, device=dev), torch.empty(B, 768, device=dev)
    st = torch.cuda.current_stream()

    def two():
        ops.anomaly_map(lv, T, m, grid, g=g, ksize=7, sigma=1.0)
        ops.image_score(det_raw, B, g * g, part, det=d, T=T, score=sc)

    def one():
        ops.anomaly_map_score(lv, det_raw, T, m, grid, part, sc, g=g, ksize=7, sigma=1.0, det=d)

    def parts():
        return {"patch_scores": time_launches(lambda: ops.patch_scores(lv, T, grid), 20, st),
                "blur_upsample": time_launches(lambda: ops.blur_upsample(grid.view(B, 1, g, g), m.view(B, 1, S, S),
                                                                          ksize=7, sigma=1.0), 20, st),
                "image_score": time_launches(lambda: ops.image_score(det_raw, B, g * g, part, det=d, T=T, score=sc),
                                             20, st)}
    t2, t1 = [], []
    for _ in range(a.rounds):  # interleaved rounds (MI355X_MICROARCH rule 24)
        t2.append(time_launches(two, 20, st) * 1e3)
        t1.append(time_launches(one, 20, st) * 1e3)
    nbytes = (L + 1) * rows * 768 * 4 + B * S * S * 4
    res[B] = {"separate_us": sorted(t2), "one_pass_us": sorted(t1),
              "one_pass_GBs_median": round(nbytes / (sorted(t1)[len(t1) // 2] * 1e-6) / 1e9, 1),
              "parts_us": {k: round(v * 1e3, 2) for k, v in parts().items()}}
    print(B, json.dumps(res[B]), flush=True)
