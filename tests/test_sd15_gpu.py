"""SD1.5 model family on MI355X: HIP kernels vs PyTorch fp32 references, native UNet vs the torch
path, and HIP-graph replay vs eager (same numbers)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from k8s_nvidia_gpus_amd.ops import kernels

    kernels.library()  # the in-tree .so — no fallback
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def SK(dev):
    from k8s_nvidia_gpus_amd.ops import sd_kernels

    return sd_kernels


def _gn_ref(x, w, b, g, eps, silu):
    y = torch.nn.functional.group_norm(x.float(), g, w.float(), b.float(), eps)
    return torch.nn.functional.silu(y) if silu else y


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape,groups", [((2, 320, 64, 64), 32), ((2, 2560, 8, 8), 32),
                                          ((4, 960, 32, 32), 32), ((1, 128, 128, 128), 32),
                                          ((3, 32, 5, 7), 8)])
@pytest.mark.parametrize("silu", [False, True])
@pytest.mark.parametrize("fused", [2, 0])           # single-launch group-set form / two launches
def test_group_norm_nhwc_vs_fp32(SK, dev, dtype, shape, groups, silu, fused):
    SK.set_group_norm_fused(fused)
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(shape, generator=g, device=dev) * 3 + 1.5).to(dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    w = (torch.rand(shape[1], generator=g, device=dev) + 0.5).to(dtype)
    b = (torch.randn(shape[1], generator=g, device=dev) * 0.1).to(dtype)
    y = SK.group_norm_nhwc(x, w, b, groups, 1e-5, silu)
    assert y.is_contiguous(memory_format=torch.channels_last)
    ref = _gn_ref(x, w, b, groups, 1e-5, silu)
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    SK.set_group_norm_fused(-1)
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("fused", [2, 0])
def test_group_norm_large_mean_both_forms(SK, dev, fused):
    """Mean 200, unit variance: the single-launch form's per-thread (n, mean, M2) + Chan merges keep
    the variance that a whole-image sum of squares would lose in fp32."""
    SK.set_group_norm_fused(fused)
    g = torch.Generator(device=dev).manual_seed(4)
    x = (torch.randn(2, 640, 32, 32, generator=g, device=dev) + 200.0).half()
    x = x.contiguous(memory_format=torch.channels_last)
    w = torch.ones(640, device=dev).half()
    b = torch.zeros(640, device=dev).half()
    y = SK.group_norm_nhwc(x, w, b, 32, 1e-5, True)
    SK.set_group_norm_fused(-1)
    torch.testing.assert_close(y.float(), _gn_ref(x, w, b, 32, 1e-5, True), rtol=2e-2, atol=2e-2)


def test_group_norm_rows_layout_and_determinism(SK, dev):
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(2, 4096, 640, generator=g, device=dev).half()
    w = torch.ones(640, device=dev).half()
    b = torch.zeros(640, device=dev).half()
    y1 = SK.group_norm_nhwc(x, w, b, 32, 1e-6, False)
    y2 = SK.group_norm_nhwc(x, w, b, 32, 1e-6, False)
    assert torch.equal(y1, y2)   # no float atomics: bit-reproducible
    ref = _gn_ref(x.permute(0, 2, 1), w, b, 32, 1e-6, False).permute(0, 2, 1)
    torch.testing.assert_close(y1.float(), ref, rtol=4e-3, atol=4e-3)


def test_group_norm_large_mean_is_stable(SK, dev):
    g = torch.Generator(device=dev).manual_seed(2)
    x = (torch.randn(2, 320, 64, 64, generator=g, device=dev) + 200.0).half()
    x = x.contiguous(memory_format=torch.channels_last)
    w = torch.ones(320, device=dev).half()
    b = torch.zeros(320, device=dev).half()
    y = SK.group_norm_nhwc(x, w, b, 32, 1e-5, False)
    torch.testing.assert_close(y.float(), _gn_ref(x, w, b, 32, 1e-5, False), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_geglu_vs_fp32(SK, dev, dtype):
    g = torch.Generator(device=dev).manual_seed(3)
    x = (torch.randn(2, 4096, 2 * 1280, generator=g, device=dev) * 2).to(dtype)
    y = SK.geglu(x)
    h, gate = x.float().chunk(2, dim=-1)
    ref = h * torch.nn.functional.gelu(gate)
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


def _tiny_pipe(dev, dtype=torch.float16, graphs=False):
    from k8s_nvidia_gpus_amd.models.sd15 import StableDiffusion, tiny

    return StableDiffusion(device=dev, dtype=dtype, cfg=tiny(), use_graphs=graphs)


def test_tiny_unet_native_matches_torch_path(dev):
    from k8s_nvidia_gpus_amd.models.sd15 import functional as SF

    pipe = _tiny_pipe(dev)
    g = torch.Generator(device=dev).manual_seed(4)
    lat = torch.randn(2, 4, 32, 32, generator=g, device=dev)
    ctx = pipe.encode_prompt(["a", "b"], ["", ""])
    try:
        SF.set_backend("torch")
        ref = pipe.runner.eager(lat, 500, ctx, 7.5)
        SF.set_backend("native")
        out = pipe.runner.eager(lat, 500, ctx, 7.5)
    finally:
        SF.set_backend("auto")
    torch.testing.assert_close(out, ref, rtol=3e-2, atol=3e-2)


def test_hip_graph_replay_equals_eager(dev):
    pipe = _tiny_pipe(dev, graphs=True)
    g = torch.Generator(device=dev).manual_seed(5)
    lat = torch.randn(1, 4, 32, 32, generator=g, device=dev)
    ctx = pipe.encode_prompt(["x"], [""])
    eager = pipe.runner.eager(lat, 321, ctx, 5.0)
    # library GEMM/conv solvers may differ between the eager call and the captured one (MIOpen /
    # hipBLASLt pick per call), so replay is compared to fp16 rounding, not bit-for-bit
    for t in (321, 321, 654):   # capture, replay, replay with a new timestep
        out = pipe.runner(lat, t, ctx, 5.0)
        if t == 321:
            torch.testing.assert_close(out, eager, rtol=2e-2, atol=2e-2)
    assert pipe.runner.captures == 1
    torch.testing.assert_close(out, pipe.runner.eager(lat, 654, ctx, 5.0), rtol=2e-2, atol=2e-2)
    assert not torch.allclose(out, eager, rtol=1e-3, atol=1e-3)   # the timestep really changed


def test_tiny_pipeline_end_to_end_png(dev):
    pipe = _tiny_pipe(dev, graphs=True)
    gens = [torch.Generator(device=dev).manual_seed(i) for i in range(3)]
    out = pipe(["a", "b", "c"], num_inference_steps=4, width=64, height=64, generator=gens)
    assert len(out.images) == 3 and out.images[0].size == (64, 64)
    solo = pipe(["b"], num_inference_steps=4, width=64, height=64,
                generator=[torch.Generator(device=dev).manual_seed(1)], output_type="latent")
    # batch 3 vs batch 1 may run different GEMM/conv solvers: equal to fp16 noise over 4 steps
    torch.testing.assert_close(solo.latents[0], out.latents[1], rtol=5e-2, atol=5e-2)


def _attn_ref(q, k, v, heads, scale):
    n, lq, c = q.shape
    d = c // heads

    def split(t):
        return t.float().reshape(n, t.shape[1], heads, d).transpose(1, 2)

    o = torch.nn.functional.scaled_dot_product_attention(split(q), split(k), split(v), scale=scale)
    return o.transpose(1, 2).reshape(n, lq, c)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("n,heads,lq,lk,d,fused", [
    (2, 8, 4096, 4096, 40, True),     # 64x64 self-attention, q|k|v slices of one projection
    (2, 8, 1024, 1024, 80, True),     # 32x32
    (2, 8, 256, 256, 160, True),      # 16x16
    (2, 8, 64, 64, 160, True),        # mid block 8x8
    (2, 8, 4096, 77, 40, False),      # cross-attention over 77 text tokens
    (2, 8, 1024, 77, 80, False),
    (1, 3, 100, 33, 64, False),       # ragged query and key counts
    (1, 2, 130, 200, 128, True),
    (2, 12, 2560, 2560, 128, True),   # Wan2.1 self-attention (attn_d128.hip)
    (2, 12, 2560, 512, 128, False),   # Wan2.1 cross-attention over the 512-token text context
    (1, 3, 1000, 777, 128, False),    # ragged d = 128
])
def test_attention_vs_fp32(SK, dev, dtype, n, heads, lq, lk, d, fused):
    g = torch.Generator(device=dev).manual_seed(lq + lk + d)
    c = heads * d
    if fused:
        qkv = torch.randn(n, lq, 3 * c, generator=g, device=dev).to(dtype)
        q, k, v = qkv[..., :c], qkv[..., c:2 * c], qkv[..., 2 * c:]
    else:
        q = torch.randn(n, lq, c, generator=g, device=dev).to(dtype)
        kv = torch.randn(n, lk, 2 * c, generator=g, device=dev).to(dtype)
        k, v = kv[..., :c], kv[..., c:]
    q = q * 2   # sharper softmax than unit scores
    assert SK.attention_supported(q, k, v, heads)
    scale = d ** -0.5
    o = SK.attention(q, k, v, heads, scale)
    ref = _attn_ref(q, k, v, heads, scale)
    tol = 2e-2 if dtype == torch.bfloat16 else 5e-3
    torch.testing.assert_close(o.float(), ref, rtol=tol, atol=tol)


def test_attention_extreme_scores_are_finite(SK, dev):
    g = torch.Generator(device=dev).manual_seed(9)
    q = (torch.randn(1, 256, 320, generator=g, device=dev) * 30).half()
    k = (torch.randn(1, 256, 320, generator=g, device=dev) * 30).half()
    v = torch.randn(1, 256, 320, generator=g, device=dev).half()
    o = SK.attention(q, k, v, 8, 40 ** -0.5)
    assert torch.isfinite(o).all()
    torch.testing.assert_close(o.float(), _attn_ref(q, k, v, 8, 40 ** -0.5), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_group_norm_with_addend_and_add3(SK, dev, dtype):
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(2, 640, 32, 32, generator=g, device=dev).to(dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    w = (torch.rand(640, generator=g, device=dev) + 0.5).to(dtype)
    b = torch.randn(640, generator=g, device=dev).to(dtype)
    big = torch.randn(2, 3000, generator=g, device=dev).to(dtype) * 4
    add = big[:, 1000:1640]                       # strided slice of the stacked temb GEMM output
    y = SK.group_norm_nhwc(x, w, b, 32, 1e-5, True, add)
    ref = _gn_ref(x.float() + add.float()[:, :, None, None], w, b, 32, 1e-5, True)
    tol = 3e-2 if dtype == torch.bfloat16 else 6e-3
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    bias = torch.randn(640, generator=g, device=dev).to(dtype)
    y0 = SK.group_norm_nhwc(x, w, b, 32, 1e-5, False, bias.expand(2, -1))   # row stride 0
    torch.testing.assert_close(y0.float(), _gn_ref(x.float() + bias.float()[:, None, None], w, b, 32,
                                                   1e-5, False), rtol=tol, atol=tol)
    z = torch.randn(2, 640, 32, 32, generator=g, device=dev).to(dtype)
    z = z.contiguous(memory_format=torch.channels_last)
    s = SK.add3(x, z, bias)
    torch.testing.assert_close(s.float(), x.float() + z.float() + bias.float()[:, None, None],
                               rtol=tol, atol=tol)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("c", [320, 640, 1280, 2048])
def test_add_layernorm_vs_fp32(SK, dev, dtype, c):
    g = torch.Generator(device=dev).manual_seed(c)
    x = (torch.randn(2, 1000, c, generator=g, device=dev) * 2 + 1).to(dtype)
    dl = torch.randn(2, 1000, c, generator=g, device=dev).to(dtype)
    w = (torch.rand(c, generator=g, device=dev) + 0.5).to(dtype)
    b = torch.randn(c, generator=g, device=dev).to(dtype)
    tol = 3e-2 if dtype == torch.bfloat16 else 6e-3
    y = SK.add_layernorm(x, None, w, b, 1e-5)
    ref = torch.nn.functional.layer_norm(x.float(), (c,), w.float(), b.float(), 1e-5)
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    xs, y2 = SK.add_layernorm(x, dl, w, b, 1e-5)
    assert torch.equal(xs, x + dl)
    ref2 = torch.nn.functional.layer_norm((x + dl).float(), (c,), w.float(), b.float(), 1e-5)
    torch.testing.assert_close(y2.float(), ref2, rtol=tol, atol=tol)


@pytest.mark.parametrize("growing", [True, False])
def test_attention_deferred_rescale_branch(SK, dev, growing):
    """Scores whose row max grows tile after tile (rescale taken at many tiles) or only shrinks
    (never taken after the first tile): both must match the fp32 reference."""
    g = torch.Generator(device=dev).manual_seed(21)
    lk = 1024
    q = torch.randn(1, 512, 320, generator=g, device=dev)
    k = torch.randn(1, lk, 320, generator=g, device=dev)
    ramp = torch.linspace(0.2, 6.0, lk, device=dev)
    k = k * (ramp if growing else ramp.flip(0))[None, :, None]
    v = torch.randn(1, lk, 320, generator=g, device=dev)
    q, k, v = q.half(), k.half(), v.half()
    o = SK.attention(q, k, v, 8, 40 ** -0.5)
    torch.testing.assert_close(o.float(), _attn_ref(q, k, v, 8, 40 ** -0.5), rtol=6e-3, atol=6e-3)


@pytest.mark.parametrize("variant,nw", [(0, 0), (2, 4), (2, 8)])
@pytest.mark.parametrize("lq,lk", [(333, 1000), (2560, 2560)])
@pytest.mark.parametrize("d", [40, 64, 80, 128, 160])
def test_attention_m32_kernels_agree(SK, dev, variant, nw, lq, lk, d):
    """Every head dim of the 32x32x16 kernel (4 and 8 waves) and the legacy transposed kernel
    against fp32, on fused q|k|v column views with ragged lengths."""
    g = torch.Generator(device=dev).manual_seed(lq * 7 + lk + d)
    heads = 4
    c = heads * d
    q = torch.randn(2, lq, c, generator=g, device=dev).bfloat16() * 2
    kv = torch.randn(2, lk, 3 * c, generator=g, device=dev).bfloat16()
    k, v = kv[..., c:2 * c], kv[..., 2 * c:]
    SK.attention_set_variant(variant)
    SK.attention_d128_set_nw(nw)
    try:
        o = SK.attention(q, k, v, heads, d ** -0.5)
    finally:
        SK.attention_set_variant(-1)
        SK.attention_d128_set_nw(0)
    torch.testing.assert_close(o.float(), _attn_ref(q, k, v, heads, d ** -0.5), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("d", [40, 80, 160])
def test_attention_m32_fp16_sd_shapes(SK, dev, d):
    """fp16 (the SD1.5 service's dtype) through the 32x32x16 kernel at the UNet head dims."""
    g = torch.Generator(device=dev).manual_seed(d)
    heads, lq = 8, {40: 4096, 80: 1024, 160: 256}[d]
    qkv = torch.randn(2, lq, 3 * heads * d, generator=g, device=dev).half()
    c = heads * d
    q, k, v = qkv[..., :c] * 2, qkv[..., c:2 * c], qkv[..., 2 * c:]
    o = SK.attention(q, k, v, heads, d ** -0.5)
    torch.testing.assert_close(o.float(), _attn_ref(q, k, v, heads, d ** -0.5), rtol=6e-3, atol=6e-3)


@pytest.mark.parametrize("growing", [True, False])
def test_attention_d128_deferred_rescale_branch(SK, dev, growing):
    g = torch.Generator(device=dev).manual_seed(23)
    lk = 1024
    q = torch.randn(1, 512, 256, generator=g, device=dev)
    k = torch.randn(1, lk, 256, generator=g, device=dev)
    ramp = torch.linspace(0.2, 6.0, lk, device=dev)
    k = k * (ramp if growing else ramp.flip(0))[None, :, None]
    v = torch.randn(1, lk, 256, generator=g, device=dev)
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    o = SK.attention(q, k, v, 2, 128 ** -0.5)
    torch.testing.assert_close(o.float(), _attn_ref(q, k, v, 2, 128 ** -0.5), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("d,L,heads", [(64, 77, 12), (64, 130, 4), (128, 300, 2), (40, 65, 3)])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_causal_attention_vs_fp32(SK, dev, d, L, heads, dtype):
    """The flash kernel's causal form (CLIP's text self-attention) against the fp32 softmax with a
    causal mask; q/k/v are strided views of one fused q|k|v tensor, as the encoder passes them."""
    g = torch.Generator(device=dev).manual_seed(d + L)
    c = heads * d
    qkv = torch.randn(2, L, 3 * c, generator=g, device=dev).to(dtype)
    q, k, v = qkv[..., :c], qkv[..., c:2 * c], qkv[..., 2 * c:]
    o = SK.attention_causal(q, k, v, heads, d ** -0.5)

    def split(t):
        return t.float().reshape(2, L, heads, d).transpose(1, 2)

    s = split(q) @ split(k).transpose(-1, -2) * d ** -0.5
    s = s.masked_fill(torch.ones(L, L, dtype=torch.bool, device=dev).triu(1), float("-inf"))
    ref = (torch.softmax(s, -1) @ split(v)).transpose(1, 2).reshape(2, L, c)
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    torch.testing.assert_close(o.float(), ref, rtol=tol, atol=tol)


def test_clip_text_encoder_native_matches_torch(dev):
    """SD1.5's CLIP text encoder on the in-tree kernels (fused q|k|v GEMM, causal flash attention,
    residual + LayerNorm kernel), eager and replayed from its HIP graph, against the PyTorch
    forward of the same fp16 weights."""
    from k8s_nvidia_gpus_amd.models.sd15.clip import CLIPTextModel
    from k8s_nvidia_gpus_amd.models.sd15.config import CLIPTextConfig

    torch.manual_seed(0)
    m = CLIPTextModel(CLIPTextConfig()).to(dev, torch.float16).eval()
    assert m.native_supported()
    ids = torch.randint(0, 49408, (4, 77), device=dev)
    with torch.no_grad():
        ref = m(ids).float()
        eager = m.native(ids, use_graph=False).float()
        graphed = m.native(ids).float()
        again = m.native(ids[:2]).float()             # another batch size: its own graph
    assert torch.isfinite(eager).all()
    torch.testing.assert_close(eager, ref, rtol=3e-2, atol=3e-2)
    assert torch.equal(graphed, eager)
    torch.testing.assert_close(again, eager[:2], rtol=1e-2, atol=1e-2)   # other M: other GEMM plan
    cos = torch.nn.functional.cosine_similarity(eager.flatten(), ref.flatten(), dim=0)
    assert cos > 0.9999
