"""CLIP byte-level BPE tokenizer (SD1.5's ``tokenizer/vocab.json`` + ``merges.txt``).

Same behaviour as transformers' ``CLIPTokenizer`` without ftfy (whitespace clean-up, lower-casing,
CLIP's pre-tokenisation regex, byte→unicode table, ``</w>`` word ends, BOS/EOS, pad/truncate to 77)
— the CPU tests compare the two on the same vocabulary.  ``HashTokenizer`` is the offline stand-in
used with random-init weights when no vocabulary files exist (no network for checkpoints here);
it is never used when a model directory provides ``tokenizer/``.
"""
from __future__ import annotations

import functools
import json
import os
import zlib
from typing import Dict, List, Sequence, Tuple

from ...utils.bpe import bytes_to_unicode

import regex

_PAT = regex.compile(
    r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
    regex.IGNORECASE)


@functools.lru_cache()


def _pairs(word: Tuple[str, ...]):
    return {(a, b) for a, b in zip(word, word[1:])}


class CLIPTokenizer:
    def __init__(self, vocab_file: str, merges_file: str, max_length: int = 77):
        with open(vocab_file, encoding="utf-8") as f:
            self.encoder: Dict[str, int] = json.load(f)
        with open(merges_file, encoding="utf-8") as f:
            lines = f.read().strip().split("\n")
        merges = [tuple(m.split()) for m in lines[1:] if m and not m.startswith("#version")]
        merges = [m for m in merges if len(m) == 2]
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.byte_encoder = bytes_to_unicode()
        self.max_length = max_length
        self.bos_id = self.encoder["<|startoftext|>"]
        self.eos_id = self.encoder["<|endoftext|>"]
        self.pad_id = self.eos_id
        self.unk_id = self.encoder.get("<|endoftext|>")
        self.cache = {"<|startoftext|>": "<|startoftext|>", "<|endoftext|>": "<|endoftext|>"}

    @classmethod
    def from_dir(cls, path: str) -> "CLIPTokenizer":
        return cls(os.path.join(path, "vocab.json"), os.path.join(path, "merges.txt"))

    def bpe(self, token: str) -> str:
        if token in self.cache:
            return self.cache[token]
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        pairs = _pairs(word)
        if not pairs:
            return token + "</w>"
        while True:
            bigram = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if bigram not in self.bpe_ranks:
                break
            first, second = bigram
            new: List[str] = []
            i = 0
            while i < len(word):
                try:
                    j = word.index(first, i)
                except ValueError:
                    new.extend(word[i:])
                    break
                new.extend(word[i:j])
                i = j
                if word[i] == first and i < len(word) - 1 and word[i + 1] == second:
                    new.append(first + second)
                    i += 2
                else:
                    new.append(word[i])
                    i += 1
            word = tuple(new)
            if len(word) == 1:
                break
            pairs = _pairs(word)
        out = " ".join(word)
        self.cache[token] = out
        return out

    def tokenize(self, text: str) -> List[int]:
        text = regex.sub(r"\s+", " ", text).strip().lower()
        ids: List[int] = []
        for tok in regex.findall(_PAT, text):
            tok = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder.get(p, self.unk_id) for p in self.bpe(tok).split(" "))
        return ids

    def __call__(self, texts: Sequence[str]) -> List[List[int]]:
        """Padded, truncated ids ``[len(texts), max_length]`` (``padding="max_length"``)."""
        out = []
        for t in texts:
            ids = [self.bos_id] + self.tokenize(t)[: self.max_length - 2] + [self.eos_id]
            out.append(ids + [self.pad_id] * (self.max_length - len(ids)))
        return out


class HashTokenizer:
    """Offline stand-in (no vocabulary files): words → stable CRC32 buckets, BOS/EOS, pad to 77."""

    def __init__(self, vocab_size: int, bos_id: int, eos_id: int, max_length: int = 77):
        self.vocab_size, self.bos_id, self.eos_id = vocab_size, bos_id, eos_id
        self.pad_id = eos_id
        self.max_length = max_length

    def tokenize(self, text: str) -> List[int]:
        words = regex.findall(_PAT, regex.sub(r"\s+", " ", text).strip().lower())
        span = self.vocab_size - 2
        return [zlib.crc32(w.encode("utf-8")) % span for w in words]

    def __call__(self, texts: Sequence[str]) -> List[List[int]]:
        out = []
        for t in texts:
            ids = [self.bos_id] + self.tokenize(t)[: self.max_length - 2] + [self.eos_id]
            out.append(ids + [self.pad_id] * (self.max_length - len(ids)))
        return out
