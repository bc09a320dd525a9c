"""Host-side logic of the drop-in API (CPU only, no kernel launches):
state-dict compatibility with the reference, tokenizer table vs the reference
tokenizer's golden output, dataset tables, error conventions, metrics."""
import json

import numpy as np
import pytest
import torch

from oracle import synth


def test_clip_and_adapter_state_dicts_load_strict():
    from model.adapter import AdaptedCLIP
    from model.clip import create_model
    m = create_model("ViT-L-14-336", 336, pretrained=None)
    sd = synth.clip_state_dict(111)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    for relu in (False, True):
        a = AdaptedCLIP(m, relu=relu)
        ia, ta = synth.adapter_state_dicts(111, relu=relu)
        a.image_adapter.load_state_dict({k: torch.from_numpy(v) for k, v in ia.items()}, strict=True)
        a.text_adapter.load_state_dict({k: torch.from_numpy(v) for k, v in ta.items()}, strict=True)
        assert a.levels == [6, 12, 18, 24] and a.i_w == 0.1 and a.t_w == 0.1
    # 6-level variant (config C5)
    a6 = AdaptedCLIP(m, levels=[4, 8, 12, 16, 20, 24], relu=False)
    assert len(a6.image_adapter["seg_proj"]) == 6


def test_create_model_error_conventions():
    from model.clip import create_model
    with pytest.raises(RuntimeError, match="not found"):
        create_model("ViT-B-99", 336)
    with pytest.raises(RuntimeError, match="required"):
        create_model("ViT-L-14-336", 336, pretrained=None, require_pretrained=True)
    m = create_model("ViT-L-14-336", 448, pretrained=None, force_image_size=448)
    assert m.visual.positional_embedding.shape == (1025, 1024)


def test_create_model_quick_gelu_and_jit(monkeypatch):
    """force_quick_gelu builds QuickGELU towers on the non-OpenAI branch only (reference
    clip.py:151-153; the OpenAI branch builds from the config, clip.py:107-142); the
    engines read the activation off the modules. jit=True is accepted (the hipGraph of
    predict_cached is the compiled path) and returns the model."""
    import model.clip as clip
    from model.adapter import AdaptedCLIP
    m = clip.create_model("ViT-L-14-336", 336, pretrained=None, force_quick_gelu=True, jit=True)
    assert isinstance(m, clip.CLIP) and m.quick_gelu
    assert m.visual.transformer.quick_gelu and m.transformer.quick_gelu
    assert isinstance(m.visual.transformer.resblocks[5].mlp.gelu, clip.QuickGELU)
    x = torch.linspace(-6, 6, 101)
    torch.testing.assert_close(m.transformer.resblocks[0].mlp.gelu(x), x * torch.sigmoid(1.702 * x))
    sd = synth.clip_state_dict(111)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)  # same parameter names
    assert AdaptedCLIP(m, relu=False).image_encoder.transformer.quick_gelu
    plain = clip.create_model("ViT-L-14-336", 336, pretrained=None)
    assert not plain.quick_gelu and not plain.visual.transformer.quick_gelu
    monkeypatch.setattr(clip, "load_openai_state_dict", lambda path: {k: torch.from_numpy(v) for k, v in sd.items()})
    o = clip.create_model("ViT-L-14-336", 336, pretrained="openai", force_quick_gelu=True)
    assert not o.visual.transformer.quick_gelu and not o.transformer.quick_gelu


def test_adapted_clip_modality_error():
    from model.adapter import AdaptedCLIP
    from model.clip import create_model
    a = AdaptedCLIP(create_model("ViT-L-14-336", 336), relu=False)
    with pytest.raises(ValueError):
        a.forward_original(None, modality="text")


def test_tokenizer_matches_reference(golden):
    from model.tokenizer import tokenize
    t = golden["text"]
    from forward_utils import _sentences
    from dataset.constants import REAL_NAMES
    for cls, real in (("bottle", REAL_NAMES["MVTec"]["bottle"]), ("brain", REAL_NAMES["Brain"]["Brain"])):
        normal, abnormal = _sentences(real)
        assert np.array_equal(tokenize(normal).numpy(), t[f"{cls}_tok_normal"])
        assert np.array_equal(tokenize(abnormal).numpy(), t[f"{cls}_tok_abnormal"])
    # outside the prompt ensemble the BPE restatement tokenises (pinned by tests/test_bpe.py)
    assert tokenize(["a sentence outside the prompt ensemble"])[0, 0] == 49406


def test_prompt_table_covers_every_class():
    from dataset.constants import CLASS_NAMES, REAL_NAMES
    from forward_utils import _sentences
    from model.tokenizer import tokenize
    for ds, classes in CLASS_NAMES.items():
        for c in classes:
            real = REAL_NAMES[ds][c] if c in REAL_NAMES.get(ds, {}) else None
            for name in ([real] if real else []) + ["object"]:
                for s in _sentences(name):
                    tok = tokenize(s)
                    assert (tok.argmax(-1) == (tok != 0).sum(-1) - 1).all()  # EOT is the argmax


def test_unknown_class_asserts():
    from forward_utils import get_adapted_single_class_text_embedding
    with pytest.raises(AssertionError):
        get_adapted_single_class_text_embedding(None, "MVTec", "not_a_class", "cpu")


def test_dataset_tables_and_synthetic():
    from dataset import DOMAINS, get_dataset
    assert DOMAINS["MVTec"] == "Industrial" and DOMAINS["Brain"] == "Medical"
    ds = get_dataset("synthetic", 336, None, stage="test", synthetic_n=6)["bottle"]
    a, b = ds[3], ds[3]
    assert torch.equal(a["image"], b["image"]) and a["label"] == 1 and ds[2]["label"] == 0
    frac = a["mask"].mean().item()
    assert 0.005 < frac < 0.12
    with pytest.raises(AssertionError):
        get_dataset("NoSuchSet", 336, None, stage="test")


def test_metrics_eval_has_no_cpu_path():
    """forward_utils.metrics_eval runs on the device kernel only (the golden check is
    tests/test_metrics_gpu.py::test_forward_utils_metrics_golden)."""
    from forward_utils import metrics_eval
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        metrics_eval(np.zeros((1, 4, 4)), np.zeros(1), np.zeros((1, 4, 4)), np.zeros(1), "c", "Industrial")


def test_metadata_root_env(monkeypatch, tmp_path):
    """Without ./dataset/metadata in the working directory the jsonl lists are looked up
    under $AACLIP_METADATA_ROOT (the reference checkout's dataset/metadata)."""
    import dataset
    monkeypatch.chdir(tmp_path)
    monkeypatch.delenv("AACLIP_METADATA_ROOT", raising=False)
    assert dataset.metadata_root() == "./dataset/metadata"
    monkeypatch.setenv("AACLIP_METADATA_ROOT", "/some/reference/dataset/metadata")
    assert dataset.metadata_root() == "/some/reference/dataset/metadata"
    (tmp_path / "dataset" / "metadata").mkdir(parents=True)
    assert dataset.metadata_root() == "./dataset/metadata"
