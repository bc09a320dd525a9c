"""Diagnostic: two-stream predict at B=32 vs one stream (bits, NaN), fp16 and bf16."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aa-clip_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from aaclip.engine import VisualEngine  # noqa: E402
from bench import synthetic_visual_weights  # noqa: E402

dev = torch.device("cuda:0")
if os.environ.get("WEIGHTS") == "synth":
    from oracle import synth
    sd = synth.clip_state_dict(111)
    ia, _ = synth.adapter_state_dicts(111)
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    ad = {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}
else:
    vp, ad = synthetic_visual_weights(dev)
tag = os.environ.get("TAG", "")
for dt in (torch.float16, torch.bfloat16):
    eng = VisualEngine(vp, ad, dtype=dt)
    eng.poison = os.environ.get("POISON") == "1"
    g = torch.Generator(device=dev).manual_seed(5)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    x = torch.randn(32, 3, 336, 336, device=dev, generator=g)
    m1, s1 = (t.clone() for t in eng.predict(x, T, "Industrial", streams=1))
    res = []
    for rep in range(4):
        m2, s2 = eng.predict(x, T, "Industrial", streams=2)
        torch.cuda.synchronize()
        nan_imgs = torch.isnan(m2).flatten(1).any(1).nonzero().flatten().tolist()
        res.append((bool(torch.equal(m1, m2)), nan_imgs[:4], len(nan_imgs)))
    print(tag, dt, "one-stream nan:", int(torch.isnan(m1).sum()), res, flush=True)
    del eng
    torch.cuda.empty_cache()
