"""Anomaly-map kernels at C2 / 518 shapes, timed as GPU time: `reps` launches captured
into one hipGraph (torch.cuda.CUDAGraph) and replayed between HIP events, so Python /
ctypes launch overhead is not in the number (an eager back-to-back loop of a ~5 us
kernel measures the host, not the GPU).
usage: python tools/map_bench.py [--sizes 336,518] [--batch 32]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import ops  # noqa: E402


def graph_time(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="336,518")
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    out = {}
    for S in [int(v) for v in a.sizes.split(",")]:
        B, g, L = a.batch, S // 14, 4
        P = g * g
        seg = torch.randn(B * P, 5 * 768, device=dev)
        lv = [seg[:, j * 768:(j + 1) * 768] for j in range(L)]
        T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev), dim=0).contiguous()
        ws = torch.zeros(B * P + B, device=dev)
        m = torch.empty(B, S, S, device=dev)
        t_ps = graph_time(lambda: ops.patch_scores(lv, T, ws[:B * P]))
        t_bu = graph_time(lambda: ops.blur_upsample(ws[:B * P].view(B, 1, g, g), m.view(B, 1, S, S), ksize=7, sigma=1.0))
        t_u0 = graph_time(lambda: ops.blur_upsample(ws[:B * P].view(B, 1, g, g), m.view(B, 1, S, S), ksize=0, sigma=0.0))
        t_all = graph_time(lambda: ops.anomaly_map(lv, T, m, ws, g=g, ksize=7, sigma=1.0))
        # predict()'s form: the map + image score from per-(row, 32-column) GEMM partials
        part = torch.rand(B * P, (L + 1) * 4 * ops.SCORE_GROUPS, device=dev) + 0.5
        dws, sc = torch.empty(B * P, device=dev), torch.empty(B, device=dev)
        t_pm = graph_time(lambda: ops.anomaly_map_partials(part, L, m, ws, g=g, ksize=7, sigma=1.0, det_ws=dws, score=sc))
        survey = B * 3.99e6 if S == 336 else None  # SURVEY 8(d) bytes per image at 336 px
        rd = L * B * P * 768 * 4
        wr = B * S * S * 4
        out[S] = {"patch_scores_us": round(t_ps, 2), "patch_scores_TBs": round(rd / t_ps / 1e6, 2),
                  "blur_upsample_us": round(t_bu, 2), "upsample_only_us": round(t_u0, 2), "blur_upsample_TBs": round(wr / t_bu / 1e6, 2),
                  "anomaly_map_us": round(t_all, 2), "anomaly_map_TBs": round((rd + wr) / t_all / 1e6, 2),
                  "partials_map_score_us": round(t_pm, 2),
                  "partials_frac_vs_survey_bytes": round(survey / t_pm / 1e6 / 8.0, 3) if survey else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
