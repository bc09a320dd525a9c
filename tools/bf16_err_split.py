"""Where does the bf16 mode's anomaly-map error come from? (GPU diagnostic)

Reference = the fp32 parity engine (within 1e-5 of the CPU oracle). Variants
recompute the level projections seg_l = tap_l . W_seg,l^T in torch (fp32
accumulate) from the engine's ln_post taps, with chosen operands rounded to
bf16, and run the same map kernel:
  tapW32     fp32 taps, fp32 W        (sanity: ~= reference)
  tap16      bf16(tap), fp32 W        (tap rounding only)
  W16        fp32 tap, bf16(W)        (seg weight rounding only)
  tap16W16   both                     (what the bf16 engine does after the taps)
  blocks16   taps from the bf16 engine (24 bf16 blocks + tap rounding), fp32 W
  bf16       the bf16 engine end to end
usage: python tools/bf16_err_split.py [n_images]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip import ops  # noqa: E402
from aaclip.engine import EMBED, VisualEngine  # noqa: E402
from oracle import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda:0")
    sd = synth.clip_state_dict(111)
    ia, _ = synth.adapter_state_dicts(111)
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    iad = {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}
    x = torch.from_numpy(synth.images(111, n, 336)).to(dev)
    T = torch.from_numpy(np.linalg.qr(np.random.default_rng(0).standard_normal((768, 2)))[0].astype(np.float32)).to(dev)
    e32 = VisualEngine(vp, iad, dtype=torch.float32)
    e16 = VisualEngine(vp, iad, dtype=torch.bfloat16)
    ref = e32.predict(x, T, "Industrial")[0].clone()
    full16 = e16.predict(x, T, "Industrial")[0].clone()
    _, _, ws32 = e32.forward_raw(x)
    taps32 = [t.clone() for t in ws32["taps"]]
    _, _, ws16 = e16.forward_raw(x)
    taps16 = [t.float().clone() for t in ws16["taps"]]
    W32 = [w.float() for w in e32.w_seg]

    def bf(t):
        return t.bfloat16().float()

    def map_from(taps, rt, rw):
        sb = ws32["segbuf"].clone()
        segs = []
        for j, (tap, w) in enumerate(zip(taps, W32)):
            a = bf(tap) if rt else tap
            b = bf(w) if rw else w
            s = (a.double() @ b.double().T).float()[:, :EMBED]
            sb[:, j * EMBED:(j + 1) * EMBED] = s
            segs.append(sb[:, j * EMBED:(j + 1) * EMBED])
        out = torch.empty_like(ref)
        ops.anomaly_map(segs, T, out, ws32["grid"], g=ws32["g"], ksize=7, sigma=1.0)
        return out

    variants = {
        "tapW32": map_from(taps32, False, False),
        "tap16": map_from(taps32, True, False),
        "W16": map_from(taps32, False, True),
        "tap16W16": map_from(taps32, True, True),
        "blocks16": map_from(taps16, False, False),
        "blocks16W16": map_from(taps16, False, True),
        "bf16": full16,
    }
    torch.cuda.synchronize()
    r = ref.double()
    tol = 1e-3 + 1e-2 * r.abs()
    for k, m in variants.items():
        e = (m.double() - r).abs()
        print(f"{k:12s} max {e.max().item():.3e}  mean {e.mean().item():.3e}  rel-L2 "
              f"{(e.norm() / r.norm()).item():.3e}  within-tol {(e <= tol).double().mean().item():.6f}")


if __name__ == "__main__":
    main()
