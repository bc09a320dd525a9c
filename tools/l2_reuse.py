"""L2 / fabric traffic of the block GEMMs per tile-order group height.

`run`: launches QKV (N 3072, bias) and c_fc (N 4096, bias + GELU) on the 8-phase kernel
(family 3) at the two-stream chunk shape M = 9232 and the merged M = 18464, for every
tile-order group height in GROUPS (aaclip_set_gemm_variant bits 4-7; the XCD remap is
the same bijective one), REPS launches each, always in the same order -- so the rocprofv3
PMC passes of the same command can be matched dispatch by dispatch.
`summarize DIR`: reads the passes (tools/prof_pmc_l2.sh) and reports per (shape, group):
fabric bytes (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE) vs algorithmic
(A + W read once, C written once), L2 hit rate, MFMA busy.
usage: python tools/l2_reuse.py run | python tools/l2_reuse.py summarize gpurun_out/l2 [--out F.json]"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]

SHAPES = [("qkv", 9232, 3072, 1024), ("c_fc", 9232, 4096, 1024), ("qkv", 18464, 3072, 1024),
          ("c_fc", 18464, 4096, 1024)]
GROUPS = (1, 2, 4, 8, 15)
REPS = 4


def configs():
    return [(name, M, N, K, gm) for (name, M, N, K) in SHAPES for gm in GROUPS]


def run():
    import torch

    from aaclip import _lib, ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    bufs = {}
    for name, M, N, K in SHAPES:
        bufs[(name, M)] = (torch.randn(M, K, device=dev, generator=g).bfloat16(),
                           (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16(),
                           torch.randn(N, device=dev, generator=g) * 0.02,
                           torch.empty(M, N, device=dev, dtype=torch.bfloat16))
    for name, M, N, K, gm in configs():
        a, w, b, out = bufs[(name, M)]
        _lib.call("aaclip_set_gemm_variant", 3 | (gm << 4))
        try:
            for _ in range(REPS):
                ops.gemm(a, w, out, bias=b, gelu=(name == "c_fc"))
        finally:
            _lib.call("aaclip_set_gemm_variant", 0)
    torch.cuda.synchronize()
    print("l2_reuse run ok", len(configs()) * REPS, "launches")


def summarize(root, out=None):
    per_pass = []
    for f in sorted(glob.glob(os.path.join(root, "pmc*", "*counter_collection.csv"))):
        rows = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if "gemm_bf16_8ph" not in r["Kernel_Name"]:
                continue
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        per_pass.append([rows[k] for k in sorted(rows)])
    cfg = configs()
    n = len(cfg) * REPS
    merged = [dict() for _ in range(n)]
    for p in per_pass:
        if len(p) != n:
            raise SystemExit(f"expected {n} GEMM dispatches per pass, found {len(p)}")
        for i, d in enumerate(p):
            merged[i].update(d)
    res = []
    for c, (name, M, N, K, gm) in enumerate(cfg):
        ds = merged[c * REPS + 1:(c + 1) * REPS]  # first launch of a config: cold, dropped
        avg = {k: sum(d[k] for d in ds) / len(ds) for k in ds[0]}
        alg = (M * K + N * K + M * N) * 2
        rd = avg.get("FETCH_SIZE", 0) * 1024 * 2
        wr = avg.get("WRITE_SIZE", 0) * 1024
        e = {"shape": name, "M": M, "N": N, "K": K, "group_m": gm, "algorithmic_MB": round(alg / 1e6, 1),
             "fabric_read_MB": round(rd / 1e6, 1), "write_MB": round(wr / 1e6, 1),
             "traffic_over_algorithmic": round((rd + wr) / alg, 3),
             "input_reads_over_algorithmic": round(rd / ((M * K + N * K) * 2), 3)}
        if avg.get("TCC_HIT_sum", 0) + avg.get("TCC_MISS_sum", 0) > 0:
            e["l2_hit_rate"] = round(avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]), 4)
        if avg.get("GRBM_GUI_ACTIVE"):
            e["mfma_busy_frac"] = round(avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (avg["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
        res.append(e)
        print(f"{name:5s} M={M:6d} group_m={gm:2d}  traffic {e['traffic_over_algorithmic']:.2f}x alg "
              f"(reads {e['input_reads_over_algorithmic']:.2f}x inputs)  l2hit {e.get('l2_hit_rate', 0):.3f}  "
              f"mfma {e.get('mfma_busy_frac', 0):.3f}")
    if out:
        open(out, "w").write(json.dumps({"source": f"rocprofv3 --pmc passes over `python tools/l2_reuse.py run` ({root}); "
                                                   "read = FETCH_SIZE*1024*2, write = WRITE_SIZE*1024; "
                                                   "FETCH_SIZE counts L2 misses served by the 256 MB MALL too",
                                         "configs": res}, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("run", "summarize"))
    ap.add_argument("root", nargs="?")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.mode == "run":
        run()
    else:
        summarize(a.root, a.out)
