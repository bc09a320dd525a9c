"""Config C4 on synthetic data (GPU): the MVTec-AD eval flow — 15 classes, each
class's ensemble prompts through the adapted text tower, per-class batches of
images through forward + 4-level map + image score, per-class metrics_eval
(pixel/image AUROC + AP) — on the drop-in API (model.adapter / forward_utils,
test.py:185-236), with synthetic weights (oracle/synth.py) and seeded synthetic
images/masks (dataset "synthetic_mvtec"). MVTec images and the OpenAI/AA-CLIP
checkpoints are absent here, so the absolute AUROCs mean nothing; what this
measures is the whole-eval rate and the parity of every per-class metric with
the CPU reference (numpy oracle + sklearn) on the same inputs.

usage: python tools/c4_synthetic.py [--n 32] [--cpu-n 8] [--out FILE]
  --n      images per class on the GPU (timed flow, bf16)
  --cpu-n  images per class in the parity subset (first cpu-n of each class:
           normal + anomalous), run through the oracle and through the GPU in
           fp32 and bf16; metrics compared per class. With fewer than 4 images
           of each label per class the image AUROC/AP can only take a few values
           (2 images: 0 or 100), so such rows are flagged degenerate in the JSON
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from dataset import DOMAINS, get_dataset  # noqa: E402
from forward_utils import _sentences, get_adapted_text_embedding, metrics_eval, metrics_eval_deferred  # noqa: E402,E501
from model.adapter import AdaptedCLIP  # noqa: E402
from model.clip import create_model  # noqa: E402
from model.tokenizer import tokenize  # noqa: E402
from dataset.constants import REAL_NAMES  # noqa: E402
from oracle import aaclip_np as R  # noqa: E402
from oracle import aaclip_torch as RT  # noqa: E402
from oracle import synth  # noqa: E402

DS = "synthetic_mvtec"


def build(dev, dtype):
    clip = create_model("ViT-L-14-336", 336, pretrained=None, device=dev)
    clip.load_state_dict({k: torch.from_numpy(v) for k, v in synth.clip_state_dict(111).items()}, strict=True)
    m = AdaptedCLIP(clip, relu=False, compute_dtype=dtype).to(dev).eval()
    ia, ta = synth.adapter_state_dicts(111)
    m.image_adapter.load_state_dict({k: torch.from_numpy(v) for k, v in ia.items()})
    m.text_adapter.load_state_dict({k: torch.from_numpy(v) for k, v in ta.items()})
    return m


def class_batches(ds, n, bs, pin=False):
    """The DataLoader's batches of one class (dicts as test.py's loop reads them), pinned
    host memory like DataLoader(pin_memory=True)."""
    out = []
    for b0 in range(0, n, bs):
        items = [ds[i] for i in range(b0, min(n, b0 + bs))]
        img = torch.stack([it["image"] for it in items])
        msk = torch.stack([it["mask"] for it in items])
        out.append({"image": img.pin_memory() if pin else img, "mask": msk.pin_memory() if pin else msk,
                    "label": torch.tensor([it["label"] for it in items]),
                    "class_name": [it["class_name"] for it in items], "file_name": [it["file_name"] for it in items]})
    return out


def gpu_eval(model, datasets, dev, batches):
    """test.py:185-236 for every class through the harness's own get_predictions (copy
    stream prefetch of batch k+1 under batch k, maps / masks kept on the device) and
    the device metrics_eval; returns per-class metrics, maps, scores."""
    import test as harness
    dom = DOMAINS[DS]
    out = {}
    with torch.no_grad():
        T = get_adapted_text_embedding(model, DS, dev)
        for c in datasets:
            masks, labels, preds, scores, _ = harness.get_predictions(model, T[c], batches[c], dev, 336,
                                                                      dataset=DS, streams=2)
            out[c] = (metrics_eval_deferred(masks, labels, preds, scores, c, domain=dom), preds, scores, masks,
                      labels)
    return T, {c: (v[0](),) + v[1:] for c, v in out.items()}  # read every class's metrics after the last


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--cpu-n", type=int, default=8)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    datasets = get_dataset(DS, 336, None, -1, "test", synthetic_n=a.n)
    # host-side batches prepared once (pinned), as the DataLoader workers would
    pinned = {c: class_batches(ds, a.n, a.bs, pin=True) for c, ds in datasets.items()}
    res = {"workload": f"C4-synthetic: 15 MVTec classes x {a.n} synthetic 336px images, ensemble prompts "
                       f"(adapted text tower), batch {a.bs}, 4 levels, metrics_eval per class, 1 GPU",
           "data": "synthetic weights (oracle/synth.py) and seeded synthetic images/masks (dataset synthetic_mvtec)"}
    model = build(dev, torch.bfloat16)
    gpu_eval(model, datasets, dev, pinned)  # warm-up: engines, workspaces, graphs
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, out16 = gpu_eval(model, datasets, dev, pinned)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_img = a.n * len(datasets)
    res["bf16_whole_eval"] = {"seconds": round(dt, 4), "images": n_img, "images_per_sec": round(n_img / dt, 1),
                              "includes": "H2D copies of the pinned batches, 15 text anchors (240 prompts), "
                                          "forward + map + score, per-class device metrics"}
    # where the whole-eval time goes (each phase alone, synchronised; not the timed flow)
    import test as harness

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / reps

    with torch.no_grad():
        Tall = get_adapted_text_embedding(model, DS, dev)
        c0 = next(iter(datasets))
        x0 = pinned[c0][0]["image"].to(dev)
        res["breakdown_seconds"] = {
            "text_anchors_240_prompts": round(timed(lambda: get_adapted_text_embedding(model, DS, dev)), 4),
            "predict_b32_eager_x15": round(15 * timed(lambda: model.predict(x0, Tall[c0], DOMAINS[DS], streams=2)), 4),
            "get_predictions_x15": round(15 * timed(lambda: harness.get_predictions(
                model, Tall[c0], pinned[c0], dev, 336, dataset=DS, streams=2)), 4),
            "metrics_eval_x15": round(15 * timed(lambda: metrics_eval(out16[c0][3], out16[c0][4], out16[c0][1],
                                                                        out16[c0][2], c0, domain=DOMAINS[DS])), 4)}
        eng = model.visual_engine()
        run = eng.graphed_predict(x0.shape[0], 336, DOMAINS[DS], streams=2)
        res["breakdown_seconds"]["predict_b32_graph_x15"] = round(15 * timed(lambda: run(x0, Tall[c0])), 4)
        del run
    print(json.dumps(res["breakdown_seconds"]), flush=True)
    mean = {k: float(np.mean([out16[c][0][k] for c in out16])) for k in ("pixel AUC", "pixel AP", "image AUC",
                                                                        "image AP")}
    res["bf16_mean_metrics"] = mean
    del model
    torch.cuda.empty_cache()

    # parity subset: first cpu-n images of each class through the oracle and the GPU (fp32, bf16)
    if a.cpu_n > 0:
        sd = synth.clip_state_dict(111)
        ia, ta = synth.adapter_state_dicts(111)
        tw = RT.prepare(sd, ia)
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
        par = {}
        t0 = time.perf_counter()
        ref = {}
        for c, ds in datasets.items():
            sn, sa = _sentences(REAL_NAMES[DS][c])
            Tc = R.class_anchor(sd, ta, tokenize(sn).numpy(), tokenize(sa).numpy())
            bt = class_batches(ds, a.cpu_n, a.cpu_n)[0]
            with torch.no_grad():  # the torch-CPU oracle (same arithmetic as the numpy one, ATen speed)
                seg, det = RT.visual_forward(tw, bt["image"])
                Tt = torch.from_numpy(Tc)
                maps = RT.anomaly_map(seg, Tt, 336, DOMAINS[DS]).numpy()
                sc = RT.image_score(det, Tt).numpy()
            ref[c] = (Tc, R.metrics_eval(bt["mask"].numpy()[:, 0], bt["label"].numpy(), maps, sc, c, DOMAINS[DS]),
                      maps, sc)
            print(f"cpu reference: class {c} done ({time.perf_counter() - t0:.0f} s)", file=sys.stderr, flush=True)
        cpu_dt = time.perf_counter() - t0
        for tag, dt_ in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
            model = build(dev, dt_)
            sub = {c: class_batches(ds, a.cpu_n, a.cpu_n) for c, ds in datasets.items()}
            T, out = gpu_eval(model, datasets, dev, sub)
            rows = {}
            for c in datasets:
                g, r = out[c][0], ref[c][1]
                rows[c] = {k: round(abs(float(g[k]) - float(r[k])), 4) for k in ("pixel AUC", "pixel AP",
                                                                                  "image AUC", "image AP")}
                rows[c]["anchor_max_abs_err"] = float(np.abs(T[c].cpu().numpy() - ref[c][0]).max())
                m = out[c][1].cpu().numpy()
                rows[c]["map_max_abs_err"] = float(np.abs(m - ref[c][2]).max())
                rows[c]["map_frac_within_tol"] = float((np.abs(m - ref[c][2]) <= 1e-3 + 1e-2 * np.abs(ref[c][2])).mean())
            par[tag] = {"max_metric_abs_diff_pct_points": max(max(v[k] for k in ("pixel AUC", "pixel AP", "image AUC",
                                                                                 "image AP")) for v in rows.values()),
                        "max_anchor_abs_err": max(v["anchor_max_abs_err"] for v in rows.values()),
                        "max_map_abs_err": max(v["map_max_abs_err"] for v in rows.values()),
                        "min_map_frac_within_tol": min(v["map_frac_within_tol"] for v in rows.values()),
                        "per_class": rows}
            del model
            torch.cuda.empty_cache()
        res["parity"] = {"images_per_class": a.cpu_n, "reference": "CPU oracle (text anchors: numpy oracle; visual "
                                                                  "path: torch-CPU oracle) + sklearn, same weights/inputs",
                         "image_metrics_degenerate": a.cpu_n < 8,
                         "cpu_seconds": round(cpu_dt, 1), **par}
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
