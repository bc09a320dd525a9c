"""Weight-load path vs the REAL reference: the same synthetic
OpenAI-layout checkpoint (oracle/synth.py:write_openai_checkpoint) through
create_model(..., pretrained='openai') must give a bit-identical fp32 state dict to
the reference's (tests/golden/golden_load.json, tests/golden/make_load_golden.py):
fp16 effective-weight rounding of the OpenAI-cast tensors, dropped metadata entries,
and the bicubic+antialias positional-embedding resize 24x24 -> 32x32 at 448 px and
-> 37x37 at 518 px (the reference's default size).
Both checkpoint formats: plain state dict and TorchScript archive (the OpenAI release
format). CPU only (~850 MB temporary checkpoint per format)."""
import json
import os

import pytest

from oracle import synth

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", params=["state_dict", "torchscript"])
def checkpoint(request, tmp_path_factory):
    """Both checkpoint formats: a plain state dict, and the OpenAI release format -- a
    TorchScript archive (the reference reads it with torch.jit.load, model/openai.py:56-59;
    model/clip.py's load_openai_state_dict takes its jit branch for it)."""
    path = str(tmp_path_factory.mktemp("ckpt") / "ViT-L-14-336px.pt")
    writer = synth.write_openai_checkpoint if request.param == "state_dict" else synth.write_openai_torchscript
    writer(path, 111)
    yield request.param, path
    os.remove(path)


@pytest.mark.parametrize("size", [336, 448, 518])
def test_openai_checkpoint_load_matches_reference(checkpoint, size, monkeypatch):
    import torch

    import model.clip as clip
    fmt, path = checkpoint
    key = str(size) if fmt == "state_dict" else f"torchscript_{size}"
    golden = json.load(open(os.path.join(HERE, "golden", "golden_load.json")))[key]
    assert golden["reference_branch"] == ("torch.jit.load" if fmt == "torchscript" else "torch.load")
    monkeypatch.setitem(clip._MODEL_CKPT_PATHS, "ViT-L-14-336", path)
    jit_calls = []
    real = torch.jit.load
    monkeypatch.setattr(torch.jit, "load", lambda *a, **k: jit_calls.append(1) or real(*a, **k))
    m = clip.create_model("ViT-L-14-336", size, pretrained="openai")
    assert len(jit_calls) == (1 if fmt == "torchscript" else 0)  # the branch the format needs was taken
    sd = m.state_dict()
    assert list(sd["visual.positional_embedding"].shape) == golden["pos_shape"]
    assert sd["visual.positional_embedding"][:3, :8].tolist() == golden["pos_rows"]
    assert len(sd) == golden["n_keys"]
    assert synth.torch_state_checksum(sd) == golden["sha256"]


def test_missing_checkpoint_raises(monkeypatch, tmp_path):
    import model.clip as clip
    monkeypatch.setitem(clip._MODEL_CKPT_PATHS, "ViT-L-14-336", str(tmp_path / "absent.pt"))
    with pytest.raises(RuntimeError, match="not found"):
        clip.create_model("ViT-L-14-336", 336, pretrained="openai")


def test_corrupt_checkpoint_keeps_its_error(monkeypatch, tmp_path):
    """A file that is neither a weights-only state dict nor a TorchScript archive is
    not handed to torch.jit.load: the weights-only loader's own error surfaces."""
    import model.clip as clip
    bad = tmp_path / "ViT-L-14-336px.pt"
    bad.write_bytes(b"\x00not a checkpoint" * 64)
    monkeypatch.setitem(clip._MODEL_CKPT_PATHS, "ViT-L-14-336", str(bad))
    with pytest.raises(Exception) as e:
        clip.create_model("ViT-L-14-336", 336, pretrained="openai")
    assert "jit" not in type(e.value).__module__ and "TorchScript" not in str(e.value)
