"""BPE restatement (aa-clip_amd/model/bpe.py, §8(f)-4) vs the REAL reference
tokenizer's ids (model/tokenizer.py:150-185): the 624 prompt-ensemble sentences
(model/prompt_tokens.json) and 26 ASCII strings covering the pre-tokeniser
(tests/golden/bpe_extra.json). CPU only."""
import json
import os

import pytest
import torch

from model.bpe import EOT, SOT, default_bpe
from model.tokenizer import tokenize

HERE = os.path.dirname(os.path.abspath(__file__))
TABLE = os.path.join(HERE, "..", "aa-clip_amd", "model", "prompt_tokens.json")
EXTRA = os.path.join(HERE, "golden", "bpe_extra.json")


@pytest.mark.parametrize("path", [TABLE, EXTRA])
def test_bpe_matches_reference_ids(path):
    bpe = default_bpe()
    table = json.load(open(path))["tokens"]
    for text, ids in table.items():
        assert [bpe.ids[SOT]] + bpe.encode(text) + [bpe.ids[EOT]] == ids, text


def test_tokenize_contract():
    t = tokenize(["a photo of a flawless bottle.", "a"])
    assert t.dtype == torch.int32 and tuple(t.shape) == (2, 77)
    assert t[0, 0] == 49406 and (t[1, :3] == torch.tensor([49406, 320, 49407], dtype=torch.int32)).all()
    assert (t[1, 3:] == 0).all()
    long = " ".join(["word"] * 100)
    with pytest.raises(RuntimeError):
        tokenize(long)
    tt = tokenize(long, truncate=True)
    assert tt[0, -1] == 49407 and (tt[0] != 0).all()


def test_bpe_roundtrip_decode():
    bpe = default_bpe()
    s = "a cropped photo of the metal nut with a bent part."
    assert bpe.decode(bpe.encode(s)).strip().replace(" .", ".") == s
