"""Clock and MFMA-busy per block GEMM under load: launches each C2 block GEMM (real
epilogue) 10 times eagerly, meant to run under
  rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv
then `python tools/gemm_clock.py --summarise DIR` joins counters with the trace:
effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md,
DVFS give-back), MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM/8 * 1024 SIMDs).
usage: python tools/gemm_clock.py [--M 18464]"""
import argparse
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]


def run(M):
    import torch
    from aaclip import ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (N, K, name) in ((3072, 1024, "qkv"), (1024, 1024, "out"), (4096, 1024, "fc"), (1024, 4096, "proj")):
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
        bias = torch.randn(N, device=dev, generator=g)
        if name in ("out", "proj"):
            out = torch.randn(M, N, device=dev, generator=g)
            for _ in range(10):
                ops.gemm(x, w, out, bias=bias, residual=out)
        else:
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            for _ in range(10):
                ops.gemm(x, w, out, bias=bias, gelu=name == "fc")
        torch.cuda.synchronize()


def summarise(d):
    cnt = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            cnt[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            cnt[int(r["Dispatch_Id"])]["name"] = r["Kernel_Name"]
            cnt[int(r["Dispatch_Id"])]["grid"] = int(r["Grid_Size"])
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = collections.defaultdict(list)
    for i, c in cnt.items():
        if "gemm" not in c["name"] or i not in dur:
            continue
        agg[(c["name"].split("(")[0].replace("(anonymous namespace)::", ""), c["grid"])].append(
            (dur[i], c.get("GRBM_GUI_ACTIVE", 0), c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)))
    for (name, grid), v in sorted(agg.items()):
        t = sum(x[0] for x in v) / len(v)
        grbm = sum(x[1] for x in v) / len(v)
        busy = sum(x[2] for x in v) / len(v)
        clk = grbm / 8 / t / 1e9
        print(f"{name[:48]:48s} grid={grid:7d} n={len(v):2d} {t * 1e6:8.1f} us  clock {clk:5.2f} GHz  "
              f"MFMA busy {busy / (grbm / 8 * 1024):.3f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=18464)
    ap.add_argument("--summarise")
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a.M)
