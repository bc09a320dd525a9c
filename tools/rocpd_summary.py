"""Kernel statistics from a rocprofv3 --kernel-trace run stored as a rocpd SQLite
database (ROCm 7 default output): the --stats table (per kernel: calls, total,
average, share) and the per-(kernel, grid) breakdown of tools/trace_summary.py.

usage: python tools/rocpd_summary.py RUN.db [--stats-csv FILE] [--grid-json FILE] [--skip-first N]
--skip-first drops the first N dispatches of each (kernel, grid) (warm-up / graph capture).
"""
import argparse
import collections
import csv
import json
import sqlite3


def clean(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--stats-csv")
    ap.add_argument("--grid-json")
    ap.add_argument("--skip-first", type=int, default=0)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, grid_x * grid_y * grid_z, start, end from kernels order by start").fetchall()
    by_grid = collections.defaultdict(list)
    for name, grid, t0, t1 in rows:
        by_grid[(clean(name), grid)].append((t1 - t0) / 1e3)
    by_name = collections.defaultdict(list)
    for (name, grid), v in by_grid.items():
        by_name[name].extend(v[a.skip_first:])
    total = sum(sum(v) for v in by_name.values())
    stats = sorted(((n, len(v), sum(v), sum(v) / len(v), min(v), max(v)) for n, v in by_name.items() if v),
                   key=lambda r: -r[2])
    print(f"{'kernel':60s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s} {'pct':>6s}")
    for n, k, tot, avg, lo, hi in stats:
        print(f"{n[:60]:60s} {k:6d} {tot / 1e3:9.2f} {avg:9.2f} {100 * tot / total:6.2f}")
    if a.stats_csv:
        with open(a.stats_csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for n, k, tot, avg, lo, hi in stats:
                w.writerow([n, k, round(tot * 1e3), round(avg * 1e3), round(100 * tot / total, 4),
                            round(lo * 1e3), round(hi * 1e3)])
    if a.grid_json:
        out = []
        for (name, grid), v in sorted(by_grid.items(), key=lambda kv: -sum(kv[1])):
            v = v[a.skip_first:] or v
            out.append({"kernel": name, "grid_size": grid, "calls": len(v), "avg_us": sum(v) / len(v),
                        "min_us": min(v), "max_us": max(v), "total_us": sum(v)})
        open(a.grid_json, "w").write(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
