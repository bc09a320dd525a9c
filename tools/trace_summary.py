"""Per-(kernel, grid size) dispatch statistics from a rocprofv3 --kernel-trace
CSV: lets the HIP-event `avg_launch_us` of one GEMM shape in bench.py be checked
against the profiler (the --stats summary averages all shapes of a kernel).
--timeline: from the first to the last run of library kernels longer than 1 ms (the
warm-up + timed steps; setup and parity legs fall outside), the union of
kernel intervals -> GPU idle time, mean concurrency and the largest idle gaps.
usage: python tools/trace_summary.py RUN_kernel_trace.csv [--out FILE.json] [--timeline]"""
import argparse
import collections
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--out")
ap.add_argument("--timeline", action="store_true")
a = ap.parse_args()
d = collections.defaultdict(list)
ivs = []
for r in csv.DictReader(open(a.trace)):
    ivs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
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

if a.timeline:
    ivs.sort()
    # window: the longest run of library kernels not interrupted by a torch/copy kernel
    # (the warm-up + timed steps; setup, RNG and parity legs fall outside it)
    runs, cur = [], []
    for iv in ivs:
        if "anonymous namespace" in iv[2]:
            cur.append(iv)
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    big = [r for r in runs if max(e for _, e, _ in r) - r[0][0] > 1_000_000]  # > 1 ms: steps
    lo, hi = big[0][0][0], max(e for _, e, _ in big[-1])
    w = [iv for iv in ivs if iv[0] >= lo and iv[0] < hi]
    t0, t1 = w[0][0], max(e for _, e, _ in w)
    busy, cur_s, cur_e, gaps, work = 0, None, None, [], 0
    for st, en, _ in w:
        work += en - st
        if cur_e is None or st > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((st - cur_e, cur_e - t0))
            cur_s, cur_e = st, en
        else:
            cur_e = max(cur_e, en)
    busy += cur_e - cur_s
    span = t1 - t0
    print(f"timeline: {len(w)} kernels over {span/1e3:.1f} us, busy {busy/1e3:.1f} us ({busy/span:.1%}), "
          f"idle {(span-busy)/1e3:.1f} us, mean concurrency while busy {work/busy:.2f}")
    for g, at in sorted(gaps, reverse=True)[:10]:
        print(f"  gap {g/1e3:7.2f} us at +{at/1e3:9.1f} us")
