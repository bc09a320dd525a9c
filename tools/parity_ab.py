"""A/B of bf16 map numerics against the fp32 parity mode (itself pinned to the CPU
oracle) on the bench's synthetic weights: frac of pixels inside the north_star
contract, max/rel-L2 map error, pixel-AUROC difference.
usage: python tools/parity_ab.py [n_images]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from sklearn.metrics import roc_auc_score  # noqa: E402

from aaclip.engine import VisualEngine  # noqa: E402
from oracle import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda:0")
    sd = synth.clip_state_dict(111)
    ia, _ = synth.adapter_state_dicts(111)
    x = torch.from_numpy(synth.images(111, n, 336)).to(dev)
    lab = synth.masks(111, n, 336)[:, 0].reshape(-1) > 0
    T = torch.from_numpy(np.linalg.qr(np.random.default_rng(0).standard_normal((768, 2)))[0].astype(np.float32)).to(dev)
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    iad = {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}
    ref = VisualEngine(vp, iad, dtype=torch.float32).predict(x, T, "Industrial")[0].cpu().numpy()
    auc_ref = roc_auc_score(lab, ref.reshape(-1))
    tol = 1e-3 + 1e-2 * np.abs(ref)
    for name, kw in (("bf16 fold", dict(dtype=torch.bfloat16)),
                     ("bf16 no-fold", dict(dtype=torch.bfloat16, fold_q_scale=False))):
        m = VisualEngine(vp, iad, **kw).predict(x, T, "Industrial")[0].cpu().numpy()
        e = np.abs(m - ref)
        print(f"{name:14s} within={float((e <= tol).mean()):.6f} max={e.max():.4g} "
              f"relL2={np.linalg.norm(m - ref) / np.linalg.norm(ref):.4g} "
              f"dAUC={abs(roc_auc_score(lab, m.reshape(-1)) - auc_ref):.3g}")


if __name__ == "__main__":
    main()
