"""Run-to-run determinism of the visual engine: the default path twice, then the
deferred-residual path, on the library AACLIP_LIB points at; prints which outputs
differ and by how much. usage: python tools/det_check.py [bf16|fp16|fp32]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
from aaclip.engine import VisualEngine  # noqa: E402
from oracle import synth  # noqa: E402


def main():
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[sys.argv[1] if len(sys.argv) > 1 else "bf16"]
    dev = torch.device("cuda:0")
    sd = synth.clip_state_dict(111)
    ia, _ = synth.adapter_state_dicts(111)
    sd = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    ia = {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}
    eng = VisualEngine(sd, ia, dtype=dt)
    g = torch.Generator(device=dev).manual_seed(8)
    x = torch.randn(3, 3, 336, 336, device=dev, generator=g)
    outs = []
    for defer in (False, False, True):
        eng.defer_resid = defer
        eng._ws.clear()
        seg, det = eng.forward(x)
        outs.append(([s.clone() for s in seg], det.clone()))
    for i, name in ((1, "default again"), (2, "deferred")):
        d = [float((a - b).abs().max()) for a, b in zip(outs[0][0], outs[i][0])]
        print(f"{name}: seg max diffs {d}, det {float((outs[0][1] - outs[i][1]).abs().max())}")


if __name__ == "__main__":
    main()
