"""Idle CU time of a traced C2 step attributed to op transitions: for every CU, each gap
between the end of the op that last held it and the start of its next wave is charged
to (that op -> the next wave's op). Input: the npz `tools/timeline.py --raw` writes.
usage: python tools/timeline_transitions.py gpurun_out/r05d/raw_2s.npz [top]"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import timeline as tl  # noqa: E402


def main():
    d = np.load(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    t0 = d["t0"].astype(np.float64) / 100
    t1 = d["t1"].astype(np.float64) / 100
    slot = d["slot"].astype(np.int64)
    ut, inv = np.unique(d["tag"], return_inverse=True)
    names = sorted({tl.op_of(int(t)) for t in ut})
    opid = np.array([names.index(tl.op_of(int(t))) for t in ut])[inv]
    agg, cnt = collections.Counter(), collections.Counter()
    cus = np.unique(slot)
    for c in cus:
        m = slot == c
        o = np.argsort(t0[m])
        s, e, op = t0[m][o], t1[m][o], opid[m][o]
        best, holder = -1.0, -1
        for i in range(len(s)):
            if i and s[i] > best:
                key = (names[holder], names[op[i]])
                agg[key] += s[i] - best
                cnt[key] += 1
            if e[i] >= best:
                best, holder = e[i], op[i]
    n = len(cus)
    print(f"window {t1.max() / 1e3:.3f} ms, {n} CUs, idle between waves {sum(agg.values()) / n / 1e3:.3f} ms per CU")
    for k, v in agg.most_common(top):
        print(f"{k[0]:>12s} -> {k[1]:<12s} {v / n / 1e3:7.3f} ms/CU  gaps {cnt[k]:6d}  mean {v / cnt[k]:6.1f} us")


if __name__ == "__main__":
    main()
