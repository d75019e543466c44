"""Sequence parallelism for the Wan2.1 DiT across GPUs (Ulysses-style all-to-all over RCCL/xGMI).

A 512×320×16-frame job is 2560 tokens per sample; a 720p 81-frame job is 75 600.  Everything in a
Wan block except self-attention is token-local (AdaLN, q/k RMSNorm + RoPE, cross-attention to the
per-rank copy of the text K/V, FFN), so each of P ranks keeps L/P tokens of the residual stream for
the whole forward.  Self-attention needs every token: two ``all_to_all_single`` per block turn
``[L/P tokens × all heads]`` into ``[all tokens × H/P heads]`` and back (the DeepSpeed-Ulysses
exchange), each rank running the flash-attention kernel on its head group over the full sequence.
Per block a rank sends 3 + 1 activations of L/P × C·(P−1)/P elements — point-to-point traffic that
xGMI's full mesh (every GPU pair directly linked) carries without a ring's per-hop serialisation.
The head's output is all-gathered so every rank holds the full velocity and the sampler state
stays identical on all ranks (same seed, same noise).

Constraints: P divides the head count (1.3B: 12 heads → P ∈ {2, 3, 4, 6}; 14B: 40 → 2, 4, 5, 8)
and the token count per sample.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class SequenceParallel:
    world: int
    rank: int
    group: Optional[object] = None

    @classmethod
    def from_env(cls, group=None) -> "SequenceParallel":
        return cls(dist.get_world_size(group), dist.get_rank(group), group)

    def check(self, tokens: int, heads: int) -> None:
        if heads % self.world or tokens % self.world:
            raise ValueError(f"sequence parallel over {self.world} ranks needs heads ({heads}) and "
                             f"tokens ({tokens}) divisible by it")

    def shard(self, t: torch.Tensor, dim: int = 1) -> torch.Tensor:
        n = t.shape[dim] // self.world
        return t.narrow(dim, self.rank * n, n).contiguous()

    def gather(self, t: torch.Tensor, dim: int = 1) -> torch.Tensor:
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, dim)

    def _a2a(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty_like(t)
        dist.all_to_all_single(out, t, group=self.group)
        return out

    def attention(self, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int, attn_fn):
        """q/k/v: this rank's ``[B, L/P, H·d]`` rows → its rows of softmax(qkᵀ/√d)v over all L."""
        b, ls, c = q.shape
        w = self.world
        hp = heads // w
        cw = c // w                                    # one rank's head group: hp·d channels

        def to_heads(t):                               # [b, ls, w, cw] → all tokens, my heads
            t = t.reshape(b, ls, w, cw).permute(2, 0, 1, 3).contiguous()
            return self._a2a(t).permute(1, 0, 2, 3).reshape(b, w * ls, cw)

        o = attn_fn(to_heads(q), to_heads(k), to_heads(v), hp)          # [b, L, cw]
        t = o.reshape(b, w, ls, cw).permute(1, 0, 2, 3).contiguous()   # chunk j → rank j
        return self._a2a(t).permute(1, 2, 0, 3).reshape(b, ls, c)
