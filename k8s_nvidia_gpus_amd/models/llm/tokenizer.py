"""Byte-level BPE tokenizer built from a GGUF file's ``tokenizer.ggml.*`` metadata, and the
ChatML prompt format of Qwen2.5-Instruct (the fallback when a file carries no chat template).

llama.cpp reads the vocabulary from the model file (``tokenizer.ggml.model = gpt2``, ``tokens``,
``merges``, ``token_type``, ``pre``); so does this engine, through the ``tokenizers`` library's BPE
model with the pre-tokenisation regex ``tokenizer.ggml.pre`` names (chat_template.py; unknown
pre-types are refused) and a byte-level decoder.  Control tokens (``token_type == 3``:
``<|im_start|>``, ``<|im_end|>``, ``<|endoftext|>`` …) are registered as special tokens so they are
matched whole in prompts.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

from ...utils.bpe import bytes_to_unicode

import numpy as np

from .chat_template import QWEN2 as QWEN2_PATTERN, QWEN25_TEMPLATE, pre_tokenizer_pattern
CONTROL = 3
DEFAULT_SYSTEM = "You are Qwen, created by Alibaba Cloud. You are a helpful assistant."


class Tokenizer:
    def __init__(self, tokens: Sequence[str], merges: Sequence[str],
                 token_types: Optional[Sequence[int]] = None, eos_id: Optional[int] = None,
                 bos_id: Optional[int] = None, add_bos: bool = False, pattern: str = QWEN2_PATTERN):
        from tokenizers import AddedToken, Regex, decoders, models, pre_tokenizers
        from tokenizers import Tokenizer as HFTokenizer

        vocab = {t: i for i, t in enumerate(tokens)}
        pairs = []
        for m in merges:
            a, _, b = m.partition(" ")
            if a in vocab and b in vocab:
                pairs.append((a, b))
        bpe = models.BPE(vocab=vocab, merges=pairs, ignore_merges=False)
        tk = HFTokenizer(bpe)
        tk.pre_tokenizer = pre_tokenizers.Sequence([
            pre_tokenizers.Split(Regex(pattern), behavior="isolated", invert=False),
            pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
        tk.decoder = decoders.ByteLevel()
        types = list(token_types) if token_types is not None else [1] * len(tokens)
        special = [AddedToken(t, special=True, normalized=False)
                   for t, ty in zip(tokens, types) if ty == CONTROL]
        if special:
            tk.add_special_tokens(special)
        self._tk = tk
        self.tokens = list(tokens)
        self.special_ids = {i for i, ty in enumerate(types) if ty == CONTROL}
        self.eos_id = eos_id
        self.bos_id = bos_id
        self.add_bos = add_bos
        self.vocab = vocab
        from .chat_template import ChatFormatter

        # prompt format of /v1/chat/completions: the file's own template once from_gguf ran
        self.formatter = ChatFormatter(None, default_system=DEFAULT_SYSTEM)

    @classmethod
    def from_gguf(cls, meta: Dict) -> "Tokenizer":
        model = meta.get("tokenizer.ggml.model", "gpt2")
        if model != "gpt2":
            raise ValueError(f"tokenizer model {model!r}: only byte-level BPE (gpt2) is supported")
        from .chat_template import ChatFormatter

        pattern = pre_tokenizer_pattern(meta)
        formatter = ChatFormatter.from_gguf(meta, meta["tokenizer.ggml.tokens"])  # parses or raises
        types = meta.get("tokenizer.ggml.token_type")
        t = cls(list(meta["tokenizer.ggml.tokens"]), list(meta.get("tokenizer.ggml.merges", [])),
                   None if types is None else [int(x) for x in np.asarray(types)],
                   eos_id=meta.get("tokenizer.ggml.eos_token_id"),
                   bos_id=meta.get("tokenizer.ggml.bos_token_id"),
                   add_bos=bool(meta.get("tokenizer.ggml.add_bos_token", False)), pattern=pattern)
        t.formatter = formatter
        return t

    def encode(self, text: str) -> List[int]:
        ids = self._tk.encode(text, add_special_tokens=False).ids
        if self.add_bos and self.bos_id is not None:
            ids = [self.bos_id] + ids
        return ids

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        return self._tk.decode(list(ids), skip_special_tokens=skip_special)

    def token_bytes(self) -> List[bytes]:
        """The bytes every token id stands for (control tokens: ``b""``, as :meth:`decode` skips
        them), in the byte-level decoder's rule: a token whose characters are all in the byte
        alphabet maps through it, any other token to its own UTF-8.  Built once, on first use."""
        tb = getattr(self, "_token_bytes", None)
        if tb is None:
            inv = {c: b for b, c in bytes_to_unicode().items()}
            tb = []
            for i, t in enumerate(self.tokens):
                if i in self.special_ids:
                    tb.append(b"")
                elif all(c in inv for c in t):
                    tb.append(bytes(inv[c] for c in t))
                else:
                    tb.append(t.encode("utf-8"))
            self._token_bytes = tb
        return tb

    def stream(self) -> "StreamDecoder":
        return StreamDecoder(self)

    def token_id(self, text: str) -> Optional[int]:
        return self.vocab.get(text)

    def stop_ids(self) -> List[int]:
        ids = set()
        if self.eos_id is not None:
            ids.add(int(self.eos_id))
        for t in ("<|im_end|>", "<|endoftext|>"):
            i = self.vocab.get(t)
            if i is not None:
                ids.add(i)
        return sorted(ids)


def chatml(messages: Sequence[Dict[str, str]], default_system: Optional[str] = DEFAULT_SYSTEM,
           add_generation_prompt: bool = True) -> str:
    """Qwen2.5-Instruct's chat template (ChatML)."""
    from .chat_template import message_text

    out = []
    if default_system and (not messages or messages[0].get("role") != "system"):
        out.append(f"<|im_start|>system\n{default_system}<|im_end|>\n")
    for m in messages:
        out.append(f"<|im_start|>{m.get('role', 'user')}\n{message_text(m.get('content', ''))}<|im_end|>\n")
    if add_generation_prompt:
        out.append("<|im_start|>assistant\n")
    return "".join(out)


def synthetic_vocab(size: int, corpus: str = "") -> Dict:
    """A byte-level BPE vocabulary of ``size`` entries for synthetic models: the 256 byte symbols,
    merges learned greedily from ``corpus`` (most frequent adjacent pair first), and the three
    Qwen2 control tokens at the end.  Returns GGUF tokenizer metadata."""
    b2u = bytes_to_unicode()
    specials = ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]
    tokens = [b2u[b] for b in range(256)]
    merges: List[str] = []
    text = corpus or ("the quick brown fox jumps over the lazy dog. a cozy cabin in the woods. "
                      "hello world, you are a helpful assistant. ") * 4
    words = [[b2u[b] for b in w.encode("utf-8")] for w in text.split(" ")]
    budget = size - len(tokens) - len(specials)
    while len(merges) < budget:
        counts: Dict[tuple, int] = {}
        for w in words:
            for a, b in zip(w, w[1:]):
                counts[(a, b)] = counts.get((a, b), 0) + 1
        if not counts:
            break
        (a, b), _ = max(counts.items(), key=lambda kv: (kv[1], kv[0]))
        merges.append(f"{a} {b}")
        tokens.append(a + b)
        new = []
        for w in words:
            out, i = [], 0
            while i < len(w):
                if i + 1 < len(w) and w[i] == a and w[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(w[i])
                    i += 1
            new.append(out)
        words = new
    while len(tokens) < size - len(specials):
        tokens.append(f"<|pad{len(tokens)}|>")
    types = [1] * len(tokens) + [CONTROL] * len(specials)
    tokens += specials
    return {"tokenizer.ggml.model": "gpt2", "tokenizer.ggml.pre": "qwen2",
            "tokenizer.ggml.tokens": tokens, "tokenizer.ggml.merges": merges,
            "tokenizer.ggml.token_type": types,
            "tokenizer.ggml.eos_token_id": tokens.index("<|im_end|>"),
            "tokenizer.ggml.padding_token_id": tokens.index("<|endoftext|>"),
            "tokenizer.ggml.bos_token_id": tokens.index("<|endoftext|>"),
            "tokenizer.ggml.add_bos_token": False,
            "tokenizer.chat_template": QWEN25_TEMPLATE}


class StreamDecoder:
    """Incremental detokenisation for streaming: each pushed token costs its own bytes, whatever
    the length of the text so far.  An incomplete UTF-8 sequence at the end is carried into the
    next push; ``flush`` ends it as U+FFFD, so the concatenated pieces equal
    ``Tokenizer.decode`` of the whole sequence (CPU test ``test_stream_decoder_equals_decode``)."""

    def __init__(self, tok: Tokenizer):
        import codecs

        self._tb = tok.token_bytes()
        self._dec = codecs.getincrementaldecoder("utf-8")("replace")

    def push(self, tok_id: int) -> str:
        return self._dec.decode(self._tb[tok_id])

    def flush(self) -> str:
        return self._dec.decode(b"", final=True)
