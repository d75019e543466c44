"""Token sampling with llama-server's request parameters.

The reference's LLM pod is upstream ``llama-server`` (reference cluster-config/apps/llm/
deployment.yaml:61,76-84); its clients may send, besides temperature / top_k / top_p:
``min_p``, ``repeat_penalty`` + ``repeat_last_n``, ``presence_penalty``, ``frequency_penalty`` and
``logit_bias``.  This module applies them in llama.cpp's default sampler-chain order:

    logit bias → penalties → top-k → top-p → min-p → temperature → draw

(penalties count the last ``repeat_last_n`` tokens of prompt + generation, like llama.cpp's
sampler, which is fed the prompt tokens too).  ``temperature <= 0`` is greedy over the biased and
penalised logits.  All maths is one fp32 vector of the vocabulary on the logits' device; only the
drawn token id crosses to the host.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Dict, Mapping, Optional, Sequence

import torch


@dataclass
class SamplingParams:
    temperature: float = 0.0
    top_k: int = 0
    top_p: float = 1.0
    min_p: float = 0.0
    repeat_penalty: float = 1.0
    repeat_last_n: int = 64
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    logit_bias: Dict[int, float] = field(default_factory=dict)

    @property
    def penalised(self) -> bool:
        return self.repeat_last_n != 0 and (self.repeat_penalty != 1.0 or self.presence_penalty != 0.0
                                            or self.frequency_penalty != 0.0)

    @property
    def plain_greedy(self) -> bool:
        """argmax of the raw logits (the batched fast path applies)."""
        return self.temperature <= 0.0 and not self.penalised and not self.logit_bias

    @classmethod
    def from_request(cls, body: Mapping[str, Any], vocab: Optional[int] = None) -> "SamplingParams":
        """llama-server / OpenAI request fields → params (llama-server's defaults)."""
        def num(key, default, cast=float, lo=None, hi=None, lo_open=False):
            v = body.get(key)
            if v is None:
                return default
            if isinstance(v, bool) or not isinstance(v, (int, float, str)):
                raise ValueError(f"{key} must be a number")
            try:
                x = cast(v)
            except (TypeError, ValueError):
                raise ValueError(f"{key} must be a number, got {v!r}") from None
            if not math.isfinite(x):
                raise ValueError(f"{key} must be finite")
            if lo is not None and (x <= lo if lo_open else x < lo):
                raise ValueError(f"{key} = {x} must be {'>' if lo_open else '>='} {lo}")
            if hi is not None and x > hi:
                raise ValueError(f"{key} = {x} must be <= {hi}")
            return x

        # out-of-range values are rejected here (HTTP 400) instead of turning logits into inf/NaN
        # inside the shared decode loop
        return cls(temperature=num("temperature", 0.8), top_k=num("top_k", 40, int),
                   top_p=num("top_p", 0.95, lo=0.0, hi=1.0), min_p=num("min_p", 0.05, lo=0.0, hi=1.0),
                   repeat_penalty=num("repeat_penalty", 1.0, lo=0.0, lo_open=True),
                   repeat_last_n=num("repeat_last_n", 64, int, lo=-1),
                   presence_penalty=num("presence_penalty", 0.0),
                   frequency_penalty=num("frequency_penalty", 0.0),
                   logit_bias=parse_logit_bias(body.get("logit_bias"), vocab))


def parse_logit_bias(raw, vocab: Optional[int] = None) -> Dict[int, float]:
    """OpenAI form ``{"123": -5}`` or llama.cpp form ``[[123, -5], [456, false]]`` (false = ban)."""
    if not raw:
        return {}
    items = raw.items() if isinstance(raw, Mapping) else raw
    out: Dict[int, float] = {}
    for entry in items:
        if not isinstance(entry, (list, tuple)) or len(entry) != 2:
            raise ValueError(f"logit_bias entry {entry!r}: expected [token, bias]")
        tok, b = int(entry[0]), entry[1]
        if vocab is not None and not 0 <= tok < vocab:
            raise ValueError(f"logit_bias token {tok} outside the vocabulary ({vocab})")
        if b is False:
            out[tok] = -float("inf")
            continue
        bias = float(b)
        if math.isnan(bias) or bias == float("inf"):
            raise ValueError(f"logit_bias for token {tok} must be finite (or false to ban it)")
        out[tok] = bias
    if vocab is not None and sum(1 for v in out.values() if v == -float("inf")) >= vocab:
        raise ValueError("logit_bias bans every token of the vocabulary")
    return out


class NoTokenLeft(ValueError):
    """Every token was filtered out (e.g. the request's biases ban all that remain)."""


def _penalise(x: torch.Tensor, p: SamplingParams, history: Sequence[int]) -> torch.Tensor:
    n = len(history) if p.repeat_last_n < 0 else min(p.repeat_last_n, len(history))
    if n == 0:
        return x
    recent = torch.tensor(list(history[len(history) - n:]), dtype=torch.long, device=x.device)
    counts = torch.zeros_like(x).index_add_(0, recent, torch.ones(n, dtype=x.dtype, device=x.device))
    seen = counts > 0
    if p.repeat_penalty != 1.0:
        x = torch.where(seen, torch.where(x > 0, x / p.repeat_penalty, x * p.repeat_penalty), x)
    return x - counts * p.frequency_penalty - seen.to(x.dtype) * p.presence_penalty


def _one_hot(like: torch.Tensor, tok: int) -> torch.Tensor:
    d = torch.zeros(like.numel(), dtype=torch.float32, device=like.device)
    d[tok] = 1.0
    return d


def sample_token(logits: torch.Tensor, p: SamplingParams, history: Sequence[int] = (),
                 generator: Optional[torch.Generator] = None,
                 dist_out: Optional[dict] = None) -> int:
    """One token from fp logits [vocab] under ``p``; ``history`` = prompt + generated ids.
    ``dist_out``: receives ``"probs"``, the distribution the token was drawn from (after the whole
    sampler chain; one-hot when greedy) — llama-server's ``post_sampling_probs``."""
    if p.plain_greedy:
        tok = int(torch.argmax(logits).item())
        if dist_out is not None:
            dist_out["probs"] = _one_hot(logits, tok)
        return tok
    x = logits.float().clone()
    for tok, b in p.logit_bias.items():
        x[tok] += b
    if p.penalised:
        x = _penalise(x, p, history)
        # extreme (valid) penalties may overflow: keep the order, never produce inf/NaN logits
        x = torch.nan_to_num(x, nan=-float("inf"), posinf=torch.finfo(x.dtype).max)
    if p.temperature <= 0.0:
        if not torch.isfinite(x.max()):
            raise NoTokenLeft("no token left to sample (every candidate was banned)")
        tok = int(torch.argmax(x).item())
        if dist_out is not None:
            dist_out["probs"] = _one_hot(x, tok)
        return tok
    if p.top_k and p.top_k > 0:
        kth = torch.topk(x, min(p.top_k, x.numel())).values[-1]
        x = x.masked_fill(x < kth, -float("inf"))
    if p.top_p < 1.0:
        sx, idx = torch.sort(x, descending=True)
        pr = torch.softmax(sx, -1)
        drop = pr.cumsum(-1) - pr > p.top_p       # keep the smallest prefix reaching top_p
        x = torch.full_like(x, -float("inf")).scatter(0, idx, sx.masked_fill(drop, -float("inf")))
    if p.min_p > 0.0:
        # keep tokens whose probability is >= min_p x the most likely one's (before temperature)
        x = x.masked_fill(x < x.max() + torch.log(torch.tensor(p.min_p)), -float("inf"))
    top = x.max()
    if not torch.isfinite(top):
        raise NoTokenLeft("no token left to sample (every candidate was banned or filtered)")
    # shift before scaling: a tiny temperature sends the others to -inf, never the maximum to +inf
    probs = torch.softmax((x - top) / p.temperature, -1)
    if generator is not None and generator.device != probs.device:
        probs = probs.to(generator.device)
    if dist_out is not None:
        dist_out["probs"] = probs
    return int(torch.multinomial(probs, 1, generator=generator).item())
