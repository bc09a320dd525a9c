"""ftfy stub: fix_text is the identity on the pure-ASCII AA-CLIP prompts
(verified for all 688 prompts)."""
def fix_text(s):
    assert all(ord(c) < 128 for c in s), "ftfy stub only valid for ASCII prompts"
    return s
