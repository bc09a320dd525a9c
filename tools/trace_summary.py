"""Per-(kernel, grid size) dispatch statistics from a rocprofv3 --kernel-trace
CSV: lets the HIP-event `avg_launch_us` of one GEMM shape in bench.py be checked
against the profiler (the --stats summary averages all shapes of a kernel).
usage: python tools/trace_summary.py RUN_kernel_trace.csv [--out FILE.json]"""
import argparse
import collections
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--out")
a = ap.parse_args()
d = collections.defaultdict(list)
for r in csv.DictReader(open(a.trace)):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip()
    grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
    d[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = []
for (name, grid), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    rows.append({"kernel": name, "grid_size": grid, "calls": len(v), "avg_us": sum(v) / len(v),
                 "min_us": min(v), "max_us": max(v), "total_us": sum(v)})
if a.out:
    open(a.out, "w").write(json.dumps(rows, indent=1))
for r in rows[:25]:
    print(f'{r["kernel"][:55]:55s} grid={r["grid_size"]:8d} calls={r["calls"]:5d} avg={r["avg_us"]:9.2f} us')
