"""The trace build of the library (`make -C aa-clip_amd/csrc trace` ->
libaaclip_hip_trace.so, -DAACLIP_TRACE) that the round-5 step timelines
(tools/timeline.py, profiles/r05/timeline_*.json) come from computes the same bits as
the product library: the same two-stream graphed C2-shaped step (8 images) runs in one
child process per library -- the trace build with its per-wave record buffer armed --
and the maps and image scores are compared bit for bit. Each library loads in its own
process (the ctypes loader binds one library per process, AACLIP_LIB)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACE_LIB = os.path.join(ROOT, "aa-clip_amd", "aaclip", "libaaclip_hip_trace.so")

CHILD = r"""
import os, sys
import numpy as np
import torch
root, out, armed = sys.argv[1], sys.argv[2], sys.argv[3] == "1"
sys.path[:0] = [root, os.path.join(root, "aa-clip_amd")]
from aaclip import _lib
from aaclip.engine import VisualEngine
from bench import synthetic_visual_weights
dev = torch.device("cuda:0")
B, S = 8, 336
vp, ad = synthetic_visual_weights(dev, n_tok=(S // 14) ** 2 + 1)
eng = VisualEngine(vp, ad, dtype=torch.bfloat16)
g = torch.Generator(device=dev).manual_seed(5)
x = torch.randn(B, 3, S, S, device=dev, generator=g)
T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
run = eng.graphed_predict(B, S, "Industrial", streams=2)
n_rec = 0
if armed:
    recs = torch.zeros(2048, 4096, 8, device=dev, dtype=torch.int32)
    cnt = torch.zeros(2048, 16, device=dev, dtype=torch.int32)
    _lib.call("aaclip_trace_buffer", recs.data_ptr(), cnt.data_ptr(), 4096)
maps, score = run(x, T)
torch.cuda.synchronize()
if armed:
    n_rec = int(cnt[:, 0].sum())
    assert int(cnt[:, 0].max()) <= 4096
    _lib.call("aaclip_trace_buffer", None, None, 0)
np.savez(out, maps=maps.cpu().numpy(), score=score.cpu().numpy(), n_rec=n_rec)
"""


def _run(lib, out, armed, tmp_path):
    env = dict(os.environ, AACLIP_LIB=lib)
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    r = subprocess.run([sys.executable, str(script), ROOT, str(out), "1" if armed else "0"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return np.load(out)


@pytest.mark.skipif(not os.path.exists(TRACE_LIB), reason="trace build not present (make -C aa-clip_amd/csrc trace)")
def test_trace_build_same_bits(tmp_path):
    prod = _run(os.path.join(ROOT, "aa-clip_amd", "aaclip", "libaaclip_hip.so"), tmp_path / "p.npz", False, tmp_path)
    trace = _run(TRACE_LIB, tmp_path / "t.npz", True, tmp_path)
    assert int(trace["n_rec"]) > 1000  # the waves did record
    assert np.isfinite(prod["maps"]).all()
    assert np.array_equal(prod["maps"], trace["maps"])
    assert np.array_equal(prod["score"], trace["score"])
