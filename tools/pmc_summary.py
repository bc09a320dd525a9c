"""Summarise rocprofv3 PMC passes (tools/prof_pmc.sh output) per kernel and
grid size, with the gfx950 corrections of MI355X_MICROARCH.md §HBM:
  read bytes  = FETCH_SIZE [KB] * 1024 * 2   (FETCH_SIZE reports half of a wide
                                              coalesced stream on gfx950)
  write bytes = WRITE_SIZE [KB] * 1024        (exact for 16-B/lane stores)
  MFMA busy   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
usage: python tools/pmc_summary.py PMC_DIR [--out FILE.json]"""
import argparse
import collections
import csv
import glob
import json
import os


def summarise(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip(), int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = []
    for (name, grid), cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"kernel": name, "grid_size": grid, "dispatches": max(len(v) for v in cs.values()), "counters": m}
        if "FETCH_SIZE" in m:
            e["hbm_read_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            e["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m and m["TCC_HIT_sum"] + m["TCC_MISS_sum"] > 0:
            e["l2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            e["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
        if m.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"]
        out.append(e)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out")
    ap.add_argument("--traffic-out", help="write the bench roofline traffic file (C2 shapes)")
    a = ap.parse_args()
    s = summarise(a.root)
    if a.traffic_out:
        # C2 (B=32, M = 18464): QKV and c_fc launches of 512-thread workgroups, on the
        # 320x256 kernel (58 x 12 / 58 x 16 tiles) or the 8-phase 256x256 one (73 x 12 / 73 x 16)
        grids = {696 * 512, 928 * 512, 876 * 512, 1168 * 512}
        gemm = [e for e in s if "gemm_bf16" in e["kernel"] and e["grid_size"] in grids and "hbm_bytes" in e]
        # the map as predict() runs it since round 4: partial_scores + blur_upsample_score
        # (the row form, patch_scores + blur_upsample, when a summary holds only that)
        mp = [e for e in s if "partial_scores" in e["kernel"] and "hbm_bytes" in e]
        bu = [e for e in s if "blur_upsample_score" in e["kernel"] and "hbm_bytes" in e]
        if not mp:
            mp = [e for e in s if "patch_scores" in e["kernel"] and "hbm_bytes" in e]
            bu = [e for e in s if "blur_upsample" in e["kernel"] and "hbm_bytes" in e]
        t = {"source": f"rocprofv3 --pmc passes (tools/prof_pmc.sh) summarised by tools/pmc_summary.py from {a.root}; "
                       "read = FETCH_SIZE*1024*2 (gfx950 half-count correction), write = WRITE_SIZE*1024"}
        if gemm:
            t["gemm"] = {"bytes_per_launch": sum(e["hbm_bytes"] for e in gemm) / len(gemm),
                         "per_shape": {str(e["grid_size"] // 512): e["hbm_bytes"] for e in gemm},
                         "l2_hit_rate": sum(e.get("l2_hit_rate", 0) for e in gemm) / len(gemm),
                         "mfma_busy_frac": sum(e.get("mfma_busy_frac", 0) for e in gemm) / len(gemm)}
        if mp:  # the anomaly map as one operation: stage 1 (patch scores) + stage 2 (blur + upsample)
            t["map"] = {"bytes_per_launch": mp[0]["hbm_bytes"] + (bu[0]["hbm_bytes"] if bu else 0),
                        "stage1_bytes": mp[0]["hbm_bytes"], "stage2_bytes": bu[0]["hbm_bytes"] if bu else None,
                        "l2_hit_rate": mp[0].get("l2_hit_rate")}
        open(a.traffic_out, "w").write(json.dumps(t, indent=1))
    txt = json.dumps(s, indent=1)
    if a.out:
        open(a.out, "w").write(txt)
    for e in s:
        print(f'{e["kernel"][:48]:48s} grid={e["grid_size"]:8d} n={e["dispatches"]:3d} '
              f'hbm={e.get("hbm_bytes", 0)/1e6:9.1f} MB l2hit={e.get("l2_hit_rate", 0):.2f} '
              f'mfma={e.get("mfma_busy_frac", 0):.3f} wait={e.get("wait_frac", 0):.2f}')
