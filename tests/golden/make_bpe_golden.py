"""Golden token ids for the BPE restatement (aa-clip_amd/model/bpe.py) beyond the
prompt table: runs the REAL reference tokenizer (model/tokenizer.py:150-185) from
/root/reference with the import-only stubs of tests/golden/stubs (ftfy.fix_text =
identity, torchvision unused by tokenize) on ASCII strings that exercise the
pre-tokeniser pattern, contractions, digits, punctuation runs, HTML entities and
whitespace. Non-ASCII text stays unpinned: ftfy (the reference's first cleaning
step) is not installed, and the stub is only faithful on ASCII. Build container only:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_bpe_golden.py
Writes tests/golden/bpe_extra.json ({text: ids} with SOT/EOT, unpadded)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "stubs"))
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

TEXTS = [
    "a photo of a flawless bottle.", "A PHOTO OF A DAMAGED Bottle!!", "it's the cat's toy, isn't it?",
    "we'll see; they'd've gone", "I'm here and you're there", "3 cracks, 12 holes and 2048 scratches",
    "pi is 3.14159", "hello---world...", "  lots   of \t whitespace \n here  ", "tom &amp; jerry &lt;3",
    "&amp;amp; double escaped", "email: foo@bar.com (see http://x.y/z?q=1)", "<|startoftext|> literal tokens <|endoftext|>",
    "hyphen-ated and under_scored words", "MIXED case WoRdS", "a", "", "!!!", "1234567890",
    "transistor with misplaced lead", "zipper with fabric interior broken teeth",
    "a cropped photo of the [c] with a defect", "metal_nut", "screw, bent; pill: faulty_imprint",
    "the quick brown fox jumps over the lazy dog", "supercalifragilisticexpialidocious antidisestablishmentarianism",
]


def main():
    prev = os.getcwd()
    os.chdir("/root/reference")
    try:
        from model.tokenizer import _tokenizer
    finally:
        os.chdir(prev)
    sot, eot = _tokenizer.encoder["<|startoftext|>"], _tokenizer.encoder["<|endoftext|>"]
    out = {t: [sot] + _tokenizer.encode(t) + [eot] for t in TEXTS}
    with open(os.path.join(HERE, "bpe_extra.json"), "w") as f:
        json.dump({"generated_by": "tests/golden/make_bpe_golden.py (reference model/tokenizer.py, ftfy stub)",
                   "tokens": out}, f, indent=0, ensure_ascii=False)
    print(len(out), "strings")


if __name__ == "__main__":
    main()
