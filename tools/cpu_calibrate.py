"""CPU-baseline calibration: time the REFERENCE's own
CPU path beside the CPU restatements on the same host, same synthetic weights and
images, so bench.py's `cpu_baseline` (which cannot run the reference on the GPU
box) carries a measured reference/port ratio.

Build container only (imports /root/reference with tests/golden/stubs, like
tests/golden/make_golden.py):

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_calibrate.py [--seconds 12] [--threads 4,8]

Per leg: bs = 1 images at 336 px through forward + 4-level anomaly map + image
score (reference: AdaptedCLIP.forward, calculate_similarity_map per level, the
test.py:83-93 sum and score), 2 warm-up images, then the reference and the torch port
alternate in 3 slices each (2 x --seconds per candidate in all); the numpy port once.
Run it on an otherwise idle host: anything else on the cores skews the ratio.
Writes profiles/r03/cpu_calibration.json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True


def _legs(fn, n_pool, seconds, warmup=2):
    for i in range(warmup):
        fn(i % n_pool)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn((warmup + n) % n_pool)
        n += 1
    dt = time.perf_counter() - t0
    return {"images_per_sec": round(n / dt, 4), "images": n, "seconds": round(dt, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--threads", default="4,8")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03", "cpu_calibration.json"))
    args = ap.parse_args()
    import numpy as np
    import torch
    from threadpoolctl import threadpool_limits

    import make_golden as mg
    from oracle import aaclip_np as R
    from oracle import aaclip_torch as RT
    from oracle import synth

    clip, model, sd, ia, _ = mg.build_reference()
    import forward_utils as fu  # the reference's module (on sys.path via make_golden)
    pool = 8
    x = synth.images(111, pool, 336)
    T = np.linalg.qr(np.random.default_rng(0).standard_normal((768, 2)))[0].astype(np.float32)
    Tt = torch.from_numpy(T)
    xt = torch.from_numpy(x)
    tw = RT.prepare(sd, ia)

    @torch.no_grad()
    def ref_one(i):
        feats, det = model(xt[i:i + 1])
        pred = (det @ Tt)
        _ = ((pred[:, 1] + 1) / 2).numpy()
        maps = [fu.calculate_similarity_map(f, Tt, 336, test=True, domain="Industrial") for f in feats]
        return torch.cat(maps, 1).sum(1).numpy()

    def np_one(i):
        seg, det = R.visual_forward(sd, ia, x[i:i + 1])
        R.anomaly_map(seg, T, 336, "Industrial")
        R.image_score(det, T)

    @torch.no_grad()
    def torch_one(i):
        seg, det = RT.visual_forward(tw, xt[i:i + 1])
        RT.anomaly_map(seg, Tt, 336, "Industrial")
        RT.image_score(det, Tt)

    # same outputs first (the timed legs must be the same computation)
    ref_map = ref_one(0)
    seg, det = R.visual_forward(sd, ia, x[:1])
    np_map = R.anomaly_map(seg, T, 336, "Industrial")
    with torch.no_grad():
        s2, d2 = RT.visual_forward(tw, xt[:1])
        t_map = RT.anomaly_map(s2, Tt, 336, "Industrial").numpy()
    out = {"host": {"nproc": os.cpu_count(), "torch": torch.__version__, "numpy": np.__version__},
           "workload": "bs=1 synthetic 336 px images, forward + 4-level anomaly map + image score, fp32; "
                       "2 warm-up images each, then reference and torch port alternating in 3 slices "
                       "(%.0f s each in all), numpy port %.0f s" % (2 * args.seconds, args.seconds / 2),
           "map_max_abs_diff_vs_reference": {"numpy_port": float(np.abs(np_map - ref_map).max()),
                                             "torch_port": float(np.abs(t_map - ref_map).max())},
           "legs": {}}

    def interleaved(fns, seconds, rounds=3):
        """Alternate the candidates in `rounds` slices of seconds/rounds each (slow drift
        in the host's clock or load then hits all of them alike)."""
        tot = {k: [0, 0.0] for k in fns}
        for k, f in fns.items():  # warm-up
            for i in range(2):
                f(i % pool)
        for r in range(rounds):
            for k, f in fns.items():
                leg = _legs(f, pool, seconds / rounds, warmup=0)
                tot[k][0] += leg["images"]
                tot[k][1] += leg["seconds"]
        return {k: {"images_per_sec": round(n / t, 4), "images": n, "seconds": round(t, 2)} for k, (n, t) in
                tot.items()}

    for th in [int(v) for v in args.threads.split(",")]:
        torch.set_num_threads(th)
        with threadpool_limits(limits=th):
            leg = interleaved({"reference": ref_one, "torch_port": torch_one}, 2 * args.seconds)
            leg["numpy_port"] = _legs(np_one, pool, args.seconds / 2)
        r = leg["reference"]["images_per_sec"]
        leg["ratio_numpy_port_over_reference"] = round(leg["numpy_port"]["images_per_sec"] / r, 4)
        leg["ratio_torch_port_over_reference"] = round(leg["torch_port"]["images_per_sec"] / r, 4)
        out["legs"][f"threads_{th}"] = leg
        print(th, json.dumps(leg), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
