"""SD1.5 model family on CPU: architecture (published parameter counts, checkpoint key names),
parity of the CLIP encoder / tokenizer with transformers, scheduler maths, checkpoint round trip,
and the pipeline's batching/seeding contract (reference sd15-api/configmap.yaml:41-121)."""
import json
import os

import pytest
import torch

from k8s_nvidia_gpus_amd.models.sd15 import StableDiffusion, tiny
from k8s_nvidia_gpus_amd.models.sd15 import functional as SF
from k8s_nvidia_gpus_amd.models.sd15.clip import CLIPTextModel
from k8s_nvidia_gpus_amd.models.sd15.config import SD15, SchedulerConfig
from k8s_nvidia_gpus_amd.models.sd15.schedulers import (DDIMScheduler, EulerDiscreteScheduler,
                                                        PNDMScheduler, alphas_cumprod)
from k8s_nvidia_gpus_amd.models.sd15.unet import UNet2DConditionModel
from k8s_nvidia_gpus_amd.models.sd15.vae import AutoencoderKLDecoder


def _count(m):
    return sum(p.numel() for p in m.parameters())


def test_full_size_parameter_counts_match_published_sd15():
    with torch.device("meta"):
        unet, clip, vae = UNet2DConditionModel(SD15.unet), CLIPTextModel(SD15.text), \
            AutoencoderKLDecoder(SD15.vae)
    assert _count(unet) == 859_520_964      # runwayml/stable-diffusion-v1-5 unet
    assert _count(clip) == 123_060_480      # openai/clip-vit-large-patch14 text tower
    assert _count(vae) == 49_490_199        # AutoencoderKL decoder half + post_quant_conv
    keys = set(unet.state_dict())
    for k in ("conv_in.weight", "time_embedding.linear_2.bias",
              "down_blocks.0.attentions.1.transformer_blocks.0.attn2.to_k.weight",
              "down_blocks.1.downsamplers.0.conv.weight", "mid_block.resnets.1.conv2.weight",
              "up_blocks.3.attentions.2.transformer_blocks.0.ff.net.0.proj.weight",
              "up_blocks.0.upsamplers.0.conv.weight", "up_blocks.1.resnets.2.conv_shortcut.weight",
              "conv_norm_out.weight", "conv_out.bias"):
        assert k in keys, k
    assert not any("up_blocks.3.upsamplers" in k for k in keys)
    assert not any(k.startswith("down_blocks.3.attentions") for k in keys)


def test_unet_shapes_and_skip_wiring_tiny():
    cfg = tiny()
    torch.manual_seed(0)
    unet = UNet2DConditionModel(cfg.unet).eval()
    x = torch.randn(2, 4, 16, 24)
    ctx = torch.randn(2, 77, cfg.unet.cross_attention_dim)
    with torch.no_grad():
        y = unet(x, torch.tensor([10, 900]), ctx)
    assert y.shape == x.shape and torch.isfinite(y).all()


def test_fused_qkv_equals_separate_projections():
    cfg = tiny()
    torch.manual_seed(1)
    unet = UNet2DConditionModel(cfg.unet).eval()
    x, ctx, t = torch.randn(1, 4, 16, 16), torch.randn(1, 77, 32), torch.tensor([500])
    with torch.no_grad():
        ref = unet(x, t, ctx)
        unet.prepare()
        fused = unet(x, t, ctx)
    torch.testing.assert_close(fused, ref, rtol=1e-5, atol=1e-5)


def _hf_clip(cfg):
    transformers = pytest.importorskip("transformers")
    hcfg = transformers.CLIPTextConfig(
        vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
        intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_layers,
        num_attention_heads=cfg.num_heads, max_position_embeddings=cfg.max_position_embeddings,
        hidden_act="quick_gelu", layer_norm_eps=cfg.layer_norm_eps, bos_token_id=cfg.bos_token_id,
        eos_token_id=cfg.eos_token_id, pad_token_id=1)
    return transformers.CLIPTextModel(hcfg).eval()


def test_clip_text_encoder_matches_transformers():
    cfg = tiny().text
    torch.manual_seed(2)
    hf = _hf_clip(cfg)
    mine = CLIPTextModel(cfg).eval()
    sd = hf.state_dict()
    prefix = "" if any(k.startswith("text_model.") for k in sd) else "text_model."
    mine.load_state_dict({prefix + k: v for k, v in sd.items() if "position_ids" not in k},
                         strict=False)
    ids = torch.randint(0, cfg.vocab_size - 2, (2, 77))
    with torch.no_grad():
        ref = hf(input_ids=ids).last_hidden_state
        got = mine(ids)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def _write_vocab(tmp_path):
    from k8s_nvidia_gpus_amd.models.sd15.tokenizer import bytes_to_unicode

    chars = sorted(set(bytes_to_unicode().values()))
    vocab = {}
    for c in chars:
        vocab[c] = len(vocab)
    for c in chars:
        vocab[c + "</w>"] = len(vocab)
    merges = [("c", "a"), ("ca", "t</w>"), ("d", "o"), ("do", "g</w>"), ("t", "h"), ("th", "e</w>"),
              ("a", "n"), ("i", "n"), ("in", "g</w>")]
    for a, b in merges:
        vocab[a + b] = len(vocab)
    vocab["<|startoftext|>"] = len(vocab)
    vocab["<|endoftext|>"] = len(vocab)
    (tmp_path / "vocab.json").write_text(json.dumps(vocab))
    (tmp_path / "merges.txt").write_text("#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges))
    return str(tmp_path)


def test_tokenizer_matches_transformers_clip_tokenizer(tmp_path):
    transformers = pytest.importorskip("transformers")
    from k8s_nvidia_gpus_amd.models.sd15.tokenizer import CLIPTokenizer

    d = _write_vocab(tmp_path)
    mine = CLIPTokenizer.from_dir(d)
    hf = transformers.CLIPTokenizer(os.path.join(d, "vocab.json"), os.path.join(d, "merges.txt"),
                                    pad_token="<|endoftext|>")
    texts = ["The cat and the DOG", "a cozy cabin, 4k!  photo's", "singing dogs " * 40]
    ref = hf(texts, padding="max_length", max_length=77, truncation=True)["input_ids"]
    assert mine(texts) == ref


def test_scheduler_timesteps_match_sd15_pndm_and_ddim():
    p = PNDMScheduler(SchedulerConfig())
    p.set_timesteps(30)
    assert len(p.timesteps) == 31 and p.timesteps[:4] == [958, 925, 925, 892] and p.timesteps[-1] == 1
    d = DDIMScheduler(SchedulerConfig())
    d.set_timesteps(50)
    assert d.timesteps[0] == 981 and d.timesteps[-1] == 1 and len(d.timesteps) == 50
    acp = alphas_cumprod(SchedulerConfig())
    assert abs(float(acp[0]) - 0.99915) < 1e-5 and abs(float(acp[-1]) - 0.0047) < 2e-4


@pytest.mark.parametrize("cls", [PNDMScheduler, DDIMScheduler, EulerDiscreteScheduler])
def test_schedulers_denoise_exactly_with_an_oracle_noise_prediction(cls):
    """With ε = the true noise, every sampler must land on x0 (the deterministic fixed point)."""
    torch.manual_seed(3)
    s = cls(SchedulerConfig())
    s.set_timesteps(20)
    x0 = torch.randn(2, 4, 8, 8, dtype=torch.float64)
    eps = torch.randn_like(x0)
    acp = s.alphas_cumprod
    if cls is EulerDiscreteScheduler:
        x = x0 + s.sigmas[0] * eps            # σ-space sample
        for t in s.timesteps:
            x = s.step(eps, t, x)
    else:
        t0 = s.timesteps[0]
        x = acp[t0].sqrt() * x0 + (1 - acp[t0]).sqrt() * eps
        for t in s.timesteps:
            x = s.step(eps, t, x)
        a_end = s._acp(-1)
        x = (x - (1 - a_end) ** 0.5 * eps) / a_end ** 0.5
    torch.testing.assert_close(x, x0, rtol=1e-6, atol=1e-6)


def _tiny_pipe(**kw):
    return StableDiffusion(device="cpu", cfg=tiny(), **kw)


def test_pipeline_batched_equals_single_and_is_seeded():
    pipe = _tiny_pipe()
    gens = [torch.Generator().manual_seed(s) for s in (11, 12)]
    out = pipe(["a cat", "a dog"], num_inference_steps=3, width=64, height=64, generator=gens)
    assert [im.size for im in out.images] == [(64, 64), (64, 64)]
    solo = pipe(["a dog"], num_inference_steps=3, width=64, height=64,
                generator=[torch.Generator().manual_seed(12)], output_type="latent")
    torch.testing.assert_close(solo.latents[0], out.latents[1], rtol=1e-3, atol=1e-3)
    again = pipe(["a cat", "a dog"], num_inference_steps=3, width=64, height=64,
                 generator=[torch.Generator().manual_seed(s) for s in (11, 12)],
                 output_type="latent")
    torch.testing.assert_close(again.latents, out.latents, rtol=0, atol=0)


def test_pipeline_rejects_bad_sizes_and_negative_prompt_count():
    pipe = _tiny_pipe()
    with pytest.raises(ValueError):
        pipe("x", width=60, height=64, num_inference_steps=1)
    with pytest.raises(ValueError):
        pipe(["a", "b"], negative_prompt=["n"], width=64, height=64, num_inference_steps=1)


def test_checkpoint_round_trip_in_diffusers_layout(tmp_path):
    safetensors = pytest.importorskip("safetensors.torch")
    cfg = tiny()
    src = StableDiffusion(device="cpu", cfg=cfg, init_seed=5)
    for sub, m, name in (("unet", src.unet, "diffusion_pytorch_model"),
                         ("text_encoder", src.text_encoder, "model")):
        (tmp_path / sub).mkdir()
        sd = {k: v.contiguous() for k, v in m.state_dict().items() if "position_ids" not in k}
        safetensors.save_file(sd, str(tmp_path / sub / f"{name}.safetensors"))
    # VAE in the legacy attention naming with 1x1-conv shaped weights + encoder tensors to skip
    (tmp_path / "vae").mkdir()
    vsd = {}
    for k, v in src.vae.state_dict().items():
        for new, old in (("to_q", "query"), ("to_k", "key"), ("to_v", "value"),
                         ("to_out.0", "proj_attn")):
            if f".attentions.0.{new}." in k:
                k = k.replace(f".attentions.0.{new}.", f".attentions.0.{old}.")
                if k.endswith("weight"):
                    v = v[:, :, None, None]
        vsd[k] = v.contiguous()
    vsd["encoder.conv_in.weight"] = torch.zeros(3)
    safetensors.save_file(vsd, str(tmp_path / "vae" / "diffusion_pytorch_model.safetensors"))
    dst = StableDiffusion(model_dir=str(tmp_path), device="cpu", cfg=cfg, init_seed=99)
    a = src(["x"], num_inference_steps=2, width=64, height=64,
            generator=[torch.Generator().manual_seed(0)], output_type="tensor")
    b = dst(["x"], num_inference_steps=2, width=64, height=64,
            generator=[torch.Generator().manual_seed(0)], output_type="tensor")
    torch.testing.assert_close(b.images, a.images, rtol=0, atol=0)


def test_functional_reference_ops_match_torch():
    torch.manual_seed(4)
    q, k, v = torch.randn(2, 10, 16), torch.randn(2, 7, 16), torch.randn(2, 7, 16)
    o = SF.attention(q, k, v, 4)
    w = torch.softmax((q.view(2, 10, 4, 4).transpose(1, 2) @ k.view(2, 7, 4, 4).permute(0, 2, 3, 1))
                      / 2.0, -1)
    ref = (w @ v.view(2, 7, 4, 4).transpose(1, 2)).transpose(1, 2).reshape(2, 10, 16)
    torch.testing.assert_close(o, ref, rtol=1e-5, atol=1e-5)
    x = torch.randn(3, 5, 8)
    torch.testing.assert_close(SF.geglu(x), x[..., :4] * torch.nn.functional.gelu(x[..., 4:]))


def test_unet_handles_sizes_that_are_not_multiples_of_64():
    """a 520x512 request (latent 65x64) — the upsamplers follow the skips' sizes
    (65 → 33 → 17 → 9 and back), as diffusers' forward_upsample_size does."""
    cfg = tiny()
    torch.manual_seed(0)
    unet = UNet2DConditionModel(cfg.unet).eval()
    ctx = torch.randn(1, 77, cfg.unet.cross_attention_dim)
    for h, w in ((65, 64), (17, 23), (9, 40)):
        x = torch.randn(1, 4, h, w)
        with torch.no_grad():
            y = unet(x, torch.tensor([10]), ctx)
        assert y.shape == x.shape and torch.isfinite(y).all()
    pipe = _tiny_pipe()
    out = pipe("a cabin", num_inference_steps=1, width=72, height=520 // 4 // 2 * 8,
               generator=[torch.Generator().manual_seed(1)])
    assert out.images[0].size == (72, 520 // 4 // 2 * 8)


def test_unet_graph_cache_is_bounded():
    from k8s_nvidia_gpus_amd.models.sd15.pipeline import UNetRunner

    class _G:
        was_reset = False

        def reset(self):
            self.was_reset = True

    r = UNetRunner(UNet2DConditionModel(tiny().unet), torch.float32, use_graphs=True, max_graphs=2)
    graphs = {}
    for key in [(1, 64, 64), (1, 64, 72), (2, 64, 64)]:
        graphs[key] = _G()
        r._graphs[key] = {"graph": graphs[key]}
        r._evict()
    assert list(r._graphs) == [(1, 64, 72), (2, 64, 64)]
    assert graphs[(1, 64, 64)].was_reset and not graphs[(2, 64, 64)].was_reset
