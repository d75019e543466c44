"""Wan2.1 model family on CPU: DiT vs the upstream-semantics forward, VAE whole-sequence decode vs
the upstream chunked algorithm, umT5 vs Hugging Face transformers' UMT5 encoder, samplers on an
analytic denoiser, tokenizer, checkpoint loading and the end-to-end pipeline."""
import os

import pytest
import torch

from k8s_nvidia_gpus_amd.models.wan import functional as WF
from k8s_nvidia_gpus_amd.models.wan import sampler as S
from k8s_nvidia_gpus_amd.models.wan.config import (UMT5Config, WanDiTConfig, WanVAEConfig,
                                                   latent_frames)
from k8s_nvidia_gpus_amd.models.wan.dit import WanDiT, reference_forward
from k8s_nvidia_gpus_amd.models.wan.pipeline import WanPipeline, dit_config_from_state
from k8s_nvidia_gpus_amd.models.wan.t5 import UMT5Encoder, UMT5Tokenizer, clean_prompt
from k8s_nvidia_gpus_amd.models.wan.vae import WanVAE, reference_decode


def _perturb(m, scale=0.02, seed=0):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(torch.randn(p.shape, generator=g) * scale)
    return m


def test_dit_forward_matches_upstream_semantics():
    torch.manual_seed(0)
    cfg = WanDiTConfig.tiny()
    m = _perturb(WanDiT(cfg))
    x = torch.randn(2, 16, 3, 8, 12)
    t = torch.tensor([900.0, 900.0])
    ctx = torch.randn(2, 7, cfg.text_dim)
    y = m(x, t, m.text_kv(m.embed_text(ctx)))
    ref = reference_forward(m, x, t, ctx)
    assert y.shape == x.shape
    torch.testing.assert_close(y, ref, rtol=1e-3, atol=1e-3)


def test_patchify_roundtrip_and_rope_sections():
    m = WanDiT(WanDiTConfig.tiny())
    x = torch.randn(1, 16, 2, 6, 10)
    rows = m.patchify(x)
    assert rows.shape == (1, 2 * 3 * 5, 64)
    # the head emits (pt, ph, pw, c) per token; re-order the patch rows the same way and invert
    y = rows.reshape(1, 30, 16, 1, 2, 2).permute(0, 1, 3, 4, 5, 2).reshape(1, 30, 64)
    torch.testing.assert_close(m.unpatchify(y, m.grid(x.shape)), x)
    cos, sin = WF.rope_table((2, 3, 5), 128)
    assert cos.shape == (30, 64)
    # token (f=1, h=0, w=0): only the 22 frame pairs rotate
    ang = torch.atan2(sin[15], cos[15])
    assert torch.all(ang[22:] == 0) and torch.all(ang[:22] != 0)


def test_vae_whole_sequence_equals_upstream_chunked_decode():
    torch.manual_seed(1)
    v = WanVAE(WanVAEConfig.tiny())
    with torch.no_grad():
        for n, p in v.named_parameters():
            if n.endswith("bias") or "gamma" in n:
                p.add_(torch.randn_like(p) * 0.1)
    z = torch.randn(1, 16, 4, 4, 6) * 0.3
    out = v.decode(z)
    ref = reference_decode(v, z)
    assert out.shape == (1, 3, 1 + 4 * 3, 32, 48) == ref.shape
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


def test_umt5_matches_transformers():
    transformers = pytest.importorskip("transformers")
    hcfg = transformers.UMT5Config(vocab_size=300, d_model=64, d_kv=16, d_ff=128, num_layers=2,
                                   num_heads=4, relative_attention_num_buckets=8,
                                   relative_attention_max_distance=16,
                                   feed_forward_proj="gated-gelu", dropout_rate=0.0)
    torch.manual_seed(2)
    hf = transformers.UMT5EncoderModel(hcfg).eval()
    ours = UMT5Encoder(UMT5Config(vocab=300, dim=64, ffn_dim=128, heads=4, head_dim=16, layers=2,
                                  buckets=8, max_distance=16))
    sd = {k: v for k, v in hf.state_dict().items() if k != "encoder.embed_tokens.weight"}
    ours.load_state_dict(sd, strict=True)
    ids = torch.randint(2, 300, (1, 37))
    with torch.no_grad():
        ref = hf(input_ids=ids).last_hidden_state
    torch.testing.assert_close(ours(ids), ref, rtol=1e-4, atol=1e-4)


def test_schedules_follow_comfy_flow_conventions():
    s = S.schedule("simple", 25, 8.0)
    assert len(s) == 26 and s[0] == 1.0 and s[-1] == 0.0
    assert torch.all(s[:-1] > s[1:])
    assert abs(float(S.training_sigmas(8.0)[-1]) - 1.0) < 1e-12
    assert len(S.schedule("normal", 10, 8.0)) == 11
    part = S.schedule("simple", 10, 8.0, denoise=0.5)
    assert len(part) == 11 and part[0] < 1.0
    with pytest.raises(ValueError):
        S.schedule("karras-ish", 10, 8.0)


@pytest.mark.parametrize("name", S.SAMPLERS)
def test_samplers_recover_point_mass_and_gaussian(name):
    x0 = torch.randn(64)
    sig = S.schedule("simple", 8, 8.0)
    out = S.sample(name, lambda x, s: x0, torch.randn(64) * float(sig[0]), sig)
    torch.testing.assert_close(out, x0, rtol=1e-5, atol=1e-5)
    mu = 2.0

    def gauss(x, s):                       # exact E[x0 | x_s] for x0 ~ N(mu, 1)
        a = 1 - s
        return mu + a / (a * a + s * s) * (x - a * mu)

    sig = S.schedule("simple", 25, 8.0)
    e = torch.randn(50000, generator=torch.Generator().manual_seed(3))
    out = S.sample(name, gauss, e * float(sig[0]), sig)
    assert abs(out.mean().item() - mu) < 0.02
    target = 0.85 if name == "euler" else 0.95       # UniPC's order-2 corrector is markedly closer
    assert out.std().item() > target


def test_initial_noise_is_comfy_cpu_seeded():
    a = S.initial_noise(42, (1, 16, 2, 4, 4), 1.0)
    torch.manual_seed(42)
    torch.testing.assert_close(a, torch.randn(1, 16, 2, 4, 4))
    assert latent_frames(16) == 4 and latent_frames(1) == 1 and latent_frames(17) == 5


def _train_spm(tmp_path):
    spm = pytest.importorskip("sentencepiece")
    corpus = tmp_path / "corpus.txt"
    corpus.write_text("\n".join(["a panda riding a motorbike", "a cat on a neon street at night",
                                 "blurry low quality artifacts", "cinematic video of the sea"] * 50))
    prefix = str(tmp_path / "sp")
    spm.SentencePieceTrainer.train(input=str(corpus), model_prefix=prefix, vocab_size=32, hard_vocab_limit=False,
                                   pad_id=0, eos_id=1, unk_id=2, bos_id=-1,
                                   minloglevel=2)
    return prefix + ".model"


def test_tokenizer_appends_eos_and_cleans(tmp_path):
    model = _train_spm(tmp_path)
    tok = UMT5Tokenizer(model, max_len=8)
    ids = tok.encode("a  panda&amp;riding\n a motorbike, a cat on a neon street")
    assert ids[-1] == UMT5Tokenizer.EOS and len(ids) == 8
    assert clean_prompt(" a \t b&amp;c ") == "a b&c"
    blob = open(model, "rb").read()
    assert UMT5Tokenizer.from_proto(blob).encode("a panda") == UMT5Tokenizer(model).encode("a panda")


def _tiny_pipe(seed=0):
    p = WanPipeline.synthetic("cpu", WanDiTConfig.tiny(), UMT5Config.tiny(vocab=60),
                              WanVAEConfig.tiny(), seed=seed)
    p.dtype = torch.float32
    p.dit.float()
    p.t5.float()
    p.vae.float()
    return p


def test_pipeline_end_to_end_tiny_cpu():
    p = _tiny_pipe()
    r1 = p.generate("a panda riding a motorbike", "blurry", width=64, height=48, frames=9, steps=3,
                    cfg=6.0, seed=5)
    assert r1.frames.shape == (9, 48, 64, 3) and r1.frames.dtype == torch.uint8
    assert r1.latent.shape == (1, 16, 3, 6, 8)
    r2 = p.generate("a panda riding a motorbike", "blurry", width=64, height=48, frames=9, steps=3,
                    cfg=6.0, seed=5)
    assert torch.equal(r1.frames, r2.frames)
    r3 = p.generate("a panda riding a motorbike", "blurry", width=64, height=48, frames=9, steps=3,
                    cfg=1.0, seed=5, sampler="euler")
    assert not torch.equal(r1.latent, r3.latent)
    with pytest.raises(ValueError):
        p.generate("x", width=60, height=48)


def test_checkpoint_files_roundtrip(tmp_path):
    from safetensors.torch import save_file

    p = _tiny_pipe(seed=3)
    unet = tmp_path / "wan2.1_t2v_1.3B_bf16.safetensors"
    clip = tmp_path / "umt5_xxl_fp16.safetensors"
    vae = tmp_path / "wan_2.1_vae.safetensors"
    save_file({"model.diffusion_model." + k: v.contiguous() for k, v in p.dit.state_dict().items()},
              str(unet))
    tsd = {k: v.contiguous() for k, v in p.t5.state_dict().items()}
    tsd["encoder.embed_tokens.weight"] = tsd["shared.weight"].clone()
    save_file(tsd, str(clip))
    vsd = {k: v.contiguous() for k, v in p.vae.state_dict().items()}
    vsd["encoder.conv1.weight"] = torch.zeros(1)          # encoder tensors are ignored
    save_file(vsd, str(vae))
    model = _train_spm(tmp_path)
    q = WanPipeline.from_files(str(unet), str(clip), str(vae), tokenizer=model, device="cpu")
    assert dit_config_from_state(p.dit.state_dict()).layers == 2
    q.dtype = torch.float32
    q.dit.float()
    q.t5.float()
    q.vae.float()
    p.tokenizer = q.tokenizer
    a = p.generate("a cat", "blurry", width=32, height=32, frames=5, steps=2, seed=1)
    b = q.generate("a cat", "blurry", width=32, height=32, frames=5, steps=2, seed=1)
    torch.testing.assert_close(a.latent, b.latent)
    with pytest.raises(ValueError):
        from k8s_nvidia_gpus_amd.models.wan.pipeline import load_strict
        load_strict(WanDiT(WanDiTConfig.tiny()), {"bogus": torch.zeros(1)})
    assert os.path.exists(unet)
