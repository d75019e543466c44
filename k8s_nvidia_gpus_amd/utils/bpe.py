"""Byte-level BPE helpers shared by the CLIP (SD1.5) and Qwen2 (LLM) tokenizers."""
from __future__ import annotations

from typing import Dict


def bytes_to_unicode() -> Dict[int, str]:
    """GPT-2's byte → printable-unicode table (the alphabet of byte-level BPE vocabularies): the
    188 printable Latin-1 bytes map to themselves, the other 68 to code points 256…323."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) \
        + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))
