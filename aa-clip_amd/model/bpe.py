"""CLIP byte-level BPE (the §8(f)-4 row): the algorithm of reference
model/tokenizer.py:22-147 (SimpleTokenizer) restated for prompts outside the
committed token table.

Pipeline per text (tokenizer.py:60-71, :138-143): clean (html-unescape twice,
strip; ftfy.fix_text is applied first in the reference — ftfy is not installed
here, and it is the identity on the ASCII prompts of this path, so only text that
ftfy would rewrite can differ), collapse whitespace, lower-case; split with the
CLIP pre-tokeniser pattern; map each UTF-8 byte to its printable stand-in
(GPT-2 byte table, tokenizer.py:27-47); greedy BPE over each piece (the lowest-rank
adjacent pair is merged everywhere, left to right, until no ranked pair is left;
the last symbol carries '</w>'); look the symbols up in the vocabulary
[256 bytes, 256 bytes+'</w>', 48894 merges, SOT, EOT].

Data: model/data/bpe_simple_vocab_16e6.txt.gz, the CLIP merge list the reference
ships (tokenizer.py:24) — a data file, read with gzip.
"""
from __future__ import annotations

import gzip
import html
import os
from functools import lru_cache

import regex

VOCAB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "bpe_simple_vocab_16e6.txt.gz")
N_MERGES = 49152 - 256 - 2  # tokenizer.py:77: lines 1 .. 48894 of the file
SOT, EOT = "<|startoftext|>", "<|endoftext|>"
_PIECES = regex.compile(r"<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+",
                        regex.IGNORECASE)


_PRINTABLE = list(range(0x21, 0x7F)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))


@lru_cache()
def byte_alphabet() -> list:
    """byte value -> printable stand-in character (printable Latin-1 bytes map to
    themselves, the other 68 to U+0100 + running index), as tokenizer.py:27-47."""
    keep = set(_PRINTABLE)
    table, extra = [None] * 256, 0
    for b in range(256):
        if b in keep:
            table[b] = chr(b)
        else:
            table[b] = chr(256 + extra)
            extra += 1
    return table


def vocab_order() -> list:
    """The 256 base symbols in vocabulary-id order: printable bytes first, then the
    remapped ones (the insertion order of the reference's byte table)."""
    table = byte_alphabet()
    rest = [b for b in range(256) if b not in set(_PRINTABLE)]
    return [table[b] for b in _PRINTABLE + rest]


class BPE:
    def __init__(self, path: str = VOCAB_PATH):
        with gzip.open(path, "rt", encoding="utf-8") as f:
            lines = f.read().split("\n")[1:N_MERGES + 1]
        merges = [tuple(line.split()) for line in lines]
        base = vocab_order()
        symbols = base + [c + "</w>" for c in base] + ["".join(m) for m in merges] + [SOT, EOT]
        self.ids = {s: i for i, s in enumerate(symbols)}
        self.rank = {m: r for r, m in enumerate(merges)}
        self._memo = {}

    def _merge(self, piece: str) -> list:
        if piece in self._memo:
            return self._memo[piece]
        syms = list(piece[:-1]) + [piece[-1] + "</w>"]
        while len(syms) > 1:
            best, best_rank = None, None
            for pair in zip(syms, syms[1:]):
                r = self.rank.get(pair)
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = pair, r
            if best is None:
                break
            out, i = [], 0
            while i < len(syms):
                if i + 1 < len(syms) and syms[i] == best[0] and syms[i + 1] == best[1]:
                    out.append(best[0] + best[1])
                    i += 2
                else:
                    out.append(syms[i])
                    i += 1
            syms = out
        self._memo[piece] = syms
        return syms

    @staticmethod
    def clean(text: str) -> str:
        text = html.unescape(html.unescape(text)).strip()
        return " ".join(text.split()).lower()

    def encode(self, text: str) -> list:
        alphabet = byte_alphabet()
        out = []
        for piece in _PIECES.findall(self.clean(text)):
            if piece in (SOT, EOT):  # literal special tokens map to their ids (tokenizer.py:85)
                out.append(self.ids[piece])
                continue
            mapped = "".join(alphabet[b] for b in piece.encode("utf-8"))
            out.extend(self.ids[s] for s in self._merge(mapped))
        return out

    def decode(self, ids) -> str:
        inv = {v: k for k, v in self.ids.items()}
        back = {c: b for b, c in enumerate(byte_alphabet())}
        text = "".join(inv[i] for i in ids)
        return bytearray(back[c] for c in text).decode("utf-8", errors="replace").replace("</w>", " ")


@lru_cache()
def default_bpe() -> BPE:
    return BPE()
