"""Load SD1.5 checkpoints in the diffusers directory layout (safetensors only — never pickle).

``<model_dir>/unet/diffusion_pytorch_model[.fp16].safetensors``,
``<model_dir>/vae/diffusion_pytorch_model[.fp16].safetensors``,
``<model_dir>/text_encoder/model[.fp16].safetensors``, ``<model_dir>/tokenizer/{vocab,merges}``
— the files ``StableDiffusionPipeline.from_pretrained`` reads in the reference
(sd15-api/configmap.yaml:41-47, HF cache on the PVC per deployment.yaml:49-50).  Parameter names
match the in-tree modules directly; the only translation is the VAE attention's legacy names
(``query/key/value/proj_attn`` with 1×1-conv shaped weights in older exports).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, Optional, Tuple

import torch

_VAE_LEGACY = {"query": "to_q", "key": "to_k", "value": "to_v", "proj_attn": "to_out.0"}


def find_file(d: str, stems: Iterable[str]) -> Optional[str]:
    for stem in stems:
        for suffix in (".safetensors", ".fp16.safetensors"):
            p = os.path.join(d, stem + suffix)
            if os.path.exists(p):
                return p
    return None


def read_safetensors(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    return load_file(path)


def convert_vae_keys(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in sd.items():
        if k.startswith(("encoder.", "quant_conv.")):
            continue   # text-to-image decodes only
        parts = k.split(".")
        if "attentions" in parts and len(parts) >= 2 and parts[-2] in _VAE_LEGACY:
            parts[-2] = _VAE_LEGACY[parts[-2]]
            k = ".".join(parts)
        if ".attentions." in k and k.endswith(".weight") and v.dim() == 4 and "group_norm" not in k:
            v = v[:, :, 0, 0]
        out[k] = v
    return out


def load_into(module: torch.nn.Module, sd: Dict[str, torch.Tensor],
              ignore_prefixes: Tuple[str, ...] = ()) -> None:
    """Strict load: every parameter must be present with the right shape (buffers excepted)."""
    own = module.state_dict()
    sd = {k: v for k, v in sd.items() if not k.startswith(ignore_prefixes)}
    missing = [k for k in own if k not in sd and not k.endswith("position_ids")]
    unexpected = [k for k in sd if k not in own]
    bad = [k for k in own if k in sd and tuple(sd[k].shape) != tuple(own[k].shape)]
    if missing or unexpected or bad:
        raise ValueError(f"checkpoint mismatch for {type(module).__name__}: missing {missing[:5]} "
                         f"({len(missing)}), unexpected {unexpected[:5]} ({len(unexpected)}), "
                         f"shape {bad[:5]}")
    with torch.no_grad():
        for k, t in own.items():
            if k in sd:
                t.copy_(sd[k].to(t.dtype))


def load_pipeline_weights(model_dir: str, unet, vae, text_encoder) -> None:
    u = find_file(os.path.join(model_dir, "unet"), ["diffusion_pytorch_model"])
    v = find_file(os.path.join(model_dir, "vae"), ["diffusion_pytorch_model"])
    t = find_file(os.path.join(model_dir, "text_encoder"), ["model"])
    if not (u and v and t):
        raise FileNotFoundError(f"{model_dir}: need unet/, vae/, text_encoder/ safetensors "
                                f"(found unet={u}, vae={v}, text_encoder={t})")
    load_into(unet, read_safetensors(u))
    load_into(vae, convert_vae_keys(read_safetensors(v)))
    load_into(text_encoder, read_safetensors(t), ignore_prefixes=("text_model.embeddings.position_ids",))
