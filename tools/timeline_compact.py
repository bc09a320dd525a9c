"""Compact a raw step-timeline record (tools/timeline.py output) into its summary: the
per-op table, CU-busy / gap statistics and clocks, without the per-2-us busy-CU bins.
usage: python tools/timeline_compact.py RAW.json OUT.json"""
import json
import sys


def compact(d: dict) -> dict:
    out = {k: v for k, v in d.items() if k != "replays"}
    reps = []
    for r in d.get("replays", []):
        r = dict(r)
        b = r.get("busy_cus_over_time")
        if isinstance(b, dict):
            r["busy_cus_over_time"] = {k: v for k, v in b.items() if k != "bins"}
            r["busy_cus_over_time"]["n_bins"] = len(b.get("bins", []))
        reps.append(r)
    out["replays"] = reps
    out["note"] = "summary of the raw per-wave timeline (per-2-us busy-CU bins dropped; raw file kept in gpurun_out/)"
    return out


if __name__ == "__main__":
    src, dst = sys.argv[1], sys.argv[2]
    with open(src) as f:
        d = json.load(f)
    with open(dst, "w") as f:
        json.dump(compact(d), f, indent=1)
