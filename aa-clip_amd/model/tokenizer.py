"""tokenize() for the AA-CLIP prompts — same signature and output as reference
model/tokenizer.py:150-185 (int32 [n, context_length], SOT 49406 ... EOT 49407,
zero padded; RuntimeError when a text is longer than the context).

The reference runs CLIP's BPE over bpe_simple_vocab_16e6.txt.gz. The path only
ever tokenises the prompt-ensemble sentences built from dataset/constants
(forward_utils.py:147-153), so this module serves them from prompt_tokens.json
— every such sentence tokenised by the REAL reference tokenizer
(tests/golden/make_golden.py). A sentence outside that table raises KeyError
(a BPE restatement is the §8(f)-4 "next" row).
"""
from __future__ import annotations

import json
import os
from functools import lru_cache
from typing import List, Union

import torch

_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "prompt_tokens.json")


@lru_cache()
def _table():
    with open(_TABLE) as f:
        return json.load(f)


def encode_ids(text: str) -> list:
    t = _table()["tokens"]
    if text not in t:
        raise KeyError(f"no token ids for {text!r}: only the AA-CLIP prompt ensemble is tabulated "
                       f"({len(t)} sentences, model/prompt_tokens.json)")
    return t[text]


def tokenize(texts: Union[str, List[str]], context_length: int = 77, truncate: bool = False) -> torch.IntTensor:
    if isinstance(texts, str):
        texts = [texts]
    eot = _table()["eot"]
    result = torch.zeros(len(texts), context_length, dtype=torch.int)
    for i, text in enumerate(texts):
        tokens = encode_ids(text)
        if len(tokens) > context_length:
            if truncate:
                tokens = tokens[:context_length]
                tokens[-1] = eot
            else:
                raise RuntimeError(f"Input {text} is too long for context length {context_length}")
        result[i, :len(tokens)] = torch.tensor(tokens)
    return result
