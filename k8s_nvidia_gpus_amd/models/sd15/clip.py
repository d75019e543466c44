"""CLIP ViT-L/14 text encoder (SD1.5's ``text_encoder``), parameter names of transformers'
``CLIPTextModel`` (``text_model.encoder.layers.{i}.self_attn.q_proj`` …).

Runs once per request on 77 tokens: causal self-attention, quick-GELU MLP, final LayerNorm; the
last hidden state is the UNet's cross-attention context (reference: diffusers
``StableDiffusionPipeline._encode_prompt``).  On the CPU this is plain PyTorch, which the CPU tests
check bit for bit against ``transformers.CLIPTextModel`` with the same weights.  On the GPU
(:meth:`CLIPTextModel.native`) the projections run on the in-tree fp16 GEMMs with q|k|v fused into
one launch, the causal attention on the flash kernel of ``ops/csrc/attn_d128.hip``, residual
add + LayerNorm on the fused kernel, and the whole encoder is replayed from a HIP graph per batch
size: eager PyTorch spent 5.7 ms of a 223 ms request here, 2.6 % of it, mostly launching ~200
small library kernels (VERDICT r5 "Next round" 7).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .config import CLIPTextConfig


class CLIPAttention(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        d = cfg.hidden_size
        self.heads = cfg.num_heads
        self.q_proj = nn.Linear(d, d)
        self.k_proj = nn.Linear(d, d)
        self.v_proj = nn.Linear(d, d)
        self.out_proj = nn.Linear(d, d)

    def forward(self, x):
        n, l, d = x.shape
        h = self.heads

        def split(t):
            return t.reshape(n, l, h, d // h).transpose(1, 2)

        o = F.scaled_dot_product_attention(split(self.q_proj(x)), split(self.k_proj(x)),
                                           split(self.v_proj(x)), is_causal=True)
        return self.out_proj(o.transpose(1, 2).reshape(n, l, d))


class CLIPMLP(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.fc1 = nn.Linear(cfg.hidden_size, cfg.intermediate_size)
        self.fc2 = nn.Linear(cfg.intermediate_size, cfg.hidden_size)

    def forward(self, x):
        x = self.fc1(x)
        return self.fc2(x * torch.sigmoid(1.702 * x))   # quick_gelu


class CLIPEncoderLayer(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.self_attn = CLIPAttention(cfg)
        self.layer_norm1 = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.mlp = CLIPMLP(cfg)
        self.layer_norm2 = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)

    def forward(self, x):
        x = x + self.self_attn(self.layer_norm1(x))
        return x + self.mlp(self.layer_norm2(x))


class _Embeddings(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.token_embedding = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.position_embedding = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size)
        self.register_buffer("position_ids", torch.arange(cfg.max_position_embeddings)[None],
                             persistent=False)

    def forward(self, ids):
        return self.token_embedding(ids) + self.position_embedding(self.position_ids[:, :ids.shape[1]])


class _Encoder(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.layers = nn.ModuleList([CLIPEncoderLayer(cfg) for _ in range(cfg.num_layers)])

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x


class _TextTransformer(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.embeddings = _Embeddings(cfg)
        self.encoder = _Encoder(cfg)
        self.final_layer_norm = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)

    def forward(self, ids):
        return self.final_layer_norm(self.encoder(self.embeddings(ids)))


class CLIPTextModel(nn.Module):
    def __init__(self, cfg: CLIPTextConfig = CLIPTextConfig()):
        super().__init__()
        self.cfg = cfg
        self.text_model = _TextTransformer(cfg)
        self._fused = None
        self._graphs: dict = {}

    def forward(self, input_ids: torch.Tensor) -> torch.Tensor:
        """``input_ids`` [N, 77] → last hidden state [N, 77, hidden]."""
        return self.text_model(input_ids)

    # ------------------------------------------------------------------ GPU path
    def _prepare(self) -> list:
        if self._fused is None:
            fused = []
            for L in self.text_model.encoder.layers:
                a = L.self_attn
                fused.append((torch.cat([a.q_proj.weight, a.k_proj.weight, a.v_proj.weight]).contiguous(),
                              torch.cat([a.q_proj.bias, a.k_proj.bias, a.v_proj.bias]).contiguous()))
            self._fused = fused
        return self._fused

    def _native_body(self, ids: torch.Tensor) -> torch.Tensor:
        from k8s_nvidia_gpus_amd.ops import gemm_epi as GE
        from k8s_nvidia_gpus_amd.ops import sd_kernels as SK

        tm = self.text_model
        c = tm.final_layer_norm.normalized_shape[0]
        heads = self.cfg.num_heads
        scale = (c // heads) ** -0.5
        h = tm.embeddings(ids)                                   # [N, L, C] in the model dtype
        layers = tm.encoder.layers
        y = SK.add_layernorm(h, None, layers[0].layer_norm1.weight, layers[0].layer_norm1.bias,
                             layers[0].layer_norm1.eps)
        for i, (L, (wqkv, bqkv)) in enumerate(zip(layers, self._prepare())):
            qkv = GE.linear(y, wqkv, bqkv)                       # [N, L, 3C], one launch
            o = SK.attention_causal(qkv[..., :c], qkv[..., c:2 * c], qkv[..., 2 * c:], heads, scale)
            d = GE.linear(o, L.self_attn.out_proj.weight, L.self_attn.out_proj.bias)
            h, y = SK.add_layernorm(h, d, L.layer_norm2.weight, L.layer_norm2.bias,
                                    L.layer_norm2.eps)         # h += attn; y = LN2(h)
            t = GE.linear(y, L.mlp.fc1.weight, L.mlp.fc1.bias)
            t = t * torch.sigmoid(1.702 * t)                     # quick_gelu
            d = GE.linear(t, L.mlp.fc2.weight, L.mlp.fc2.bias)
            nxt = layers[i + 1].layer_norm1 if i + 1 < len(layers) else tm.final_layer_norm
            h, y = SK.add_layernorm(h, d, nxt.weight, nxt.bias, nxt.eps)
        return y                                                  # final LayerNorm of the last h

    def native_supported(self) -> bool:
        """Shapes the in-tree kernels take (SD1.5's 768 / 3072 / 12 heads of 64 do; the miniature
        test configs do not and stay on the PyTorch forward)."""
        c, f, h = self.cfg.hidden_size, self.cfg.intermediate_size, self.cfg.num_heads
        return (c % 64 == 0 and f % 64 == 0 and c % h == 0 and c // h in (40, 64, 80, 128, 160)
                and c % 8 == 0 and c // 8 <= 256)

    @torch.no_grad()
    def native(self, input_ids: torch.Tensor, use_graph: bool = True) -> torch.Tensor:
        """The GPU forward (see the module docstring); ``input_ids`` [N, 77] on the GPU."""
        if not self.native_supported():
            return self(input_ids)
        if not use_graph:
            return self._native_body(input_ids)
        key = tuple(input_ids.shape)
        st = self._graphs.get(key)
        if st is None:
            ids = input_ids.clone()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                self._native_body(ids)                           # warm-up outside the capture
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = self._native_body(ids)
            st = self._graphs[key] = {"ids": ids, "out": out, "graph": g}
            while len(self._graphs) > 8:                          # client-chosen batch sizes
                self._graphs.pop(next(iter(self._graphs)))["graph"].reset()
        st["ids"].copy_(input_ids)
        st["graph"].replay()
        return st["out"].clone()
