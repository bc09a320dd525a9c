"""Effective shader clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT
run (MI355X_MICROARCH.md, DVFS give-back: clock ~= GRBM_GUI_ACTIVE / 8 XCDs / wall).
usage: python tools/clock_summary.py RUN_counter_collection.csv [--last N]"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--last", type=int, default=400, help="only the last N dispatches (the timed steps)")
a = ap.parse_args()
disp = collections.defaultdict(dict)
for r in csv.DictReader(open(a.csv)):
    d = disp[int(r["Dispatch_Id"])]
    d[r["Counter_Name"]] = float(r["Counter_Value"])
    d["name"] = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]
    d["grid"] = int(r["Grid_Size"])
    d["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
ids = sorted(disp)[-a.last:]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for i in ids:
    d = disp[i]
    k = (d["name"], d["grid"])
    agg[k][0] += 1
    agg[k][1] += d["dur"]
    agg[k][2] += d.get("GRBM_GUI_ACTIVE", 0.0)
for (n, g), (c, dur, act) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:14]:
    print(f"{n:40s} grid={g:8d} calls={c:4d} avg={dur / c:8.1f} us  clock={act / 8 / (dur * 1e3):.3f} GHz")
