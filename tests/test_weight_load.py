"""Weight-load path vs the REAL reference: the same synthetic
OpenAI-layout checkpoint (oracle/synth.py:write_openai_checkpoint) through
create_model(..., pretrained='openai') must give a bit-identical fp32 state dict to
the reference's (tests/golden/golden_load.json, tests/golden/make_load_golden.py):
fp16 effective-weight rounding of the OpenAI-cast tensors, dropped metadata entries,
and the bicubic+antialias positional-embedding resize 24x24 -> 32x32 at 448 px and
-> 37x37 at 518 px (the reference's default size).
CPU only (~850 MB temporary checkpoint)."""
import json
import os

import pytest

from oracle import synth

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checkpoint(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("ckpt") / "ViT-L-14-336px.pt")
    synth.write_openai_checkpoint(path, 111)
    return path


@pytest.mark.parametrize("size", [336, 448, 518])
def test_openai_checkpoint_load_matches_reference(checkpoint, size, monkeypatch):
    import model.clip as clip
    golden = json.load(open(os.path.join(HERE, "golden", "golden_load.json")))[str(size)]
    monkeypatch.setitem(clip._MODEL_CKPT_PATHS, "ViT-L-14-336", checkpoint)
    m = clip.create_model("ViT-L-14-336", size, pretrained="openai")
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
