"""Fused-epilogue bf16 GEMM (csrc/gemm_bf16_epi.hip) against fp32 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def GE():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from k8s_nvidia_gpus_amd.ops import gemm_epi

    return gemm_epi


def _ref(x, w, b):
    y = x.float().reshape(-1, x.shape[-1]) @ w.float().t()
    return y + b.float() if b is not None else y


@pytest.mark.parametrize("m,n,k", [(5120, 1536, 1536), (5120, 4608, 1536), (333, 1536, 1536),
                                   (1, 128, 64), (5120, 1536, 8960), (1000, 256, 4096),
                                   (8192, 320, 320), (8192, 960, 320), (500, 72, 768)])
@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_linear_vs_fp32(GE, m, n, k, bias, dtype):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    x = torch.randn(m, k, generator=g, device=dev).to(dtype)
    w = (torch.randn(n, k, generator=g, device=dev) / k ** 0.5).to(dtype)
    b = torch.randn(n, generator=g, device=dev).to(dtype) if bias else None
    assert GE.supported(x, w)
    y = GE.linear(x, w, b)
    assert y.dtype == dtype
    ref = _ref(x, w, b)
    tol = 2e-2 if dtype == torch.bfloat16 else 5e-3
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


def test_linear_gelu_and_batched_rows(GE):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(2, 2560, 1536, generator=g, device=dev).bfloat16()
    w = (torch.randn(8960, 1536, generator=g, device=dev) / 40).bfloat16()
    b = torch.randn(8960, generator=g, device=dev).bfloat16()
    y = GE.linear_gelu(x, w, b)
    ref = F.gelu(_ref(x, w, b), approximate="tanh").view(2, 2560, 8960)
    assert y.shape == (2, 2560, 8960)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("gated", [True, False])
@pytest.mark.parametrize("L", [2560, 999])
def test_linear_residual_in_place(GE, gated, L):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(L)
    x = torch.randn(2, L, 8960, generator=g, device=dev).bfloat16()
    w = (torch.randn(1536, 8960, generator=g, device=dev) / 95).bfloat16()
    b = torch.randn(1536, generator=g, device=dev).bfloat16()
    res = torch.randn(2, L, 1536, generator=g, device=dev)
    mods = torch.randn(2, 6, 1536, generator=g, device=dev)
    gate = mods[:, 5] if gated else None            # strided per-sample gate view
    want = res + (_ref(x, w, b).view(2, L, 1536) * (gate[:, None, :] if gated else 1.0))
    out = GE.linear_residual_(res, x, w, b, gate)
    assert out.data_ptr() == res.data_ptr()
    torch.testing.assert_close(res, want, rtol=1e-2, atol=2e-2)


def test_strided_input_rows(GE):
    """A column slice of a wider activation (the DiT's fused q|k|v output) as the A operand."""
    dev = torch.device("cuda")
    big = torch.randn(700, 3 * 1536, device=dev).bfloat16()
    x = big[:, 1536:3072]
    w = (torch.randn(1536, 1536, device=dev) / 40).bfloat16()
    torch.testing.assert_close(GE.linear(x, w).float(), _ref(x, w, None), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("m", [5120, 5000, 65520])
@pytest.mark.parametrize("gelu", [False, True])
def test_wide_projection_on_w4a(GE, m, gelu):
    """Wide bf16 projections take the 256x256 w4a kernel (bias / GELU store epilogue, M tail)."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(m)
    n, k = 4608, 1536
    assert GE.use_w4a(m, n, k, torch.bfloat16)
    x = torch.randn(m, k, generator=g, device=dev).bfloat16()
    w = (torch.randn(n, k, generator=g, device=dev) / 40).bfloat16()
    b = torch.randn(n, generator=g, device=dev).bfloat16()
    y = GE.linear(x, w, b, gelu=gelu)
    ref = _ref(x, w, b)
    if gelu:
        ref = F.gelu(ref, approximate="tanh")
    torch.testing.assert_close(y.float(), ref, rtol=3e-2, atol=3e-2)
    # w4a wrote only rows < M: the row after the output is untouched
    big = torch.full((m + 256, n), 7.0, device=dev).bfloat16()
    GE._w4a(2 if gelu else 1, x, w, b, big[:m])
    assert bool((big[m:] == 7.0).all())


@pytest.mark.parametrize("tile", [0, 1, 2, 3])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_every_tile_variant(GE, tile, dtype):
    """Each wave-grid block tile (256×128, 128×128, 128×64, 64×64) with M / N tails: store, GELU
    and the gated residual epilogue."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(tile)
    m, n, k = 777, 328, 192
    x = torch.randn(m, k, generator=g, device=dev).to(dtype)
    w = (torch.randn(n, k, generator=g, device=dev) / k ** 0.5).to(dtype)
    b = torch.randn(n, generator=g, device=dev).to(dtype)
    ref = _ref(x, w, b)
    tol = 2e-2 if dtype == torch.bfloat16 else 5e-3
    GE.set_tile(tile)
    try:
        assert GE.plan(m, n, k) == (GE.TILES[tile], 1)
        torch.testing.assert_close(GE.linear(x, w, b).float(), ref, rtol=tol, atol=tol)
        torch.testing.assert_close(GE.linear_gelu(x, w, b).float(),
                                   F.gelu(ref, approximate="tanh"), rtol=tol, atol=tol)
        res = torch.randn(1, m, n, generator=g, device=dev)
        gate = torch.randn(1, n, generator=g, device=dev)
        want = res + ref.view(1, m, n) * gate[:, None, :]
        GE.linear_residual_(res, x.view(1, m, k), w, b, gate)
        torch.testing.assert_close(res, want, rtol=tol, atol=2 * tol)
    finally:
        GE.set_tile(-1)
    assert GE.plan(8192, 1536, 1536) == ((256, 128), 1) and GE.plan(128, 1280, 1280) == ((64, 64), 2)
    assert GE.plan(8192, 320, 2880) == ((128, 128), 1)       # SD 64² conv: 192 tiles, unsplit
    assert GE.plan(2048, 640, 5760) == ((256, 128), 5)       # 40 tiles x 5 splits


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("gated", [True, False])
def test_w4a_gated_residual(GE, dtype, gated):
    """The w4a 256x256 kernel's RESID epilogue: x += gate · (A·Bᵀ + b) with per-sample gate rows
    that do not align with the 256-row tiles (2 × 2500 rows), M tail, bf16 and fp16."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(11)
    L, n, k = 2500, 4608, 1536
    assert GE.use_w4a(2 * L, n, k, dtype)
    x = torch.randn(2, L, k, generator=g, device=dev).to(dtype)
    w = (torch.randn(n, k, generator=g, device=dev) / 40).to(dtype)
    b = torch.randn(n, generator=g, device=dev).to(dtype)
    res = torch.randn(2, L, n, generator=g, device=dev)
    mods = torch.randn(2, 6, n, generator=g, device=dev)
    gate = mods[:, 2] if gated else None
    y = _ref(x, w, None).to(dtype).float().view(2, L, n) + b.float()   # 16-bit rounded product
    want = res + y * (gate[:, None, :] if gated else 1.0)
    GE.linear_residual_(res, x, w, b, gate)
    torch.testing.assert_close(res, want, rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("gelu", [False, True])
def test_w4a_fp16_epilogue(GE, gelu):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    m, n, k = 8192, 2560, 320                 # SD1.5 GEGLU projection at 64² latents, CFG batch
    assert GE.use_w4a(m, n, k, torch.float16)
    x = torch.randn(m, k, generator=g, device=dev).half()
    w = (torch.randn(n, k, generator=g, device=dev) / 18).half()
    b = torch.randn(n, generator=g, device=dev).half()
    ref = _ref(x, w, b)
    if gelu:
        ref = F.gelu(ref, approximate="tanh")
    torch.testing.assert_close(GE.linear(x, w, b, gelu=gelu).float(), ref, rtol=5e-3, atol=5e-3)


@pytest.mark.parametrize("mode", ["s1", "s2", "up2"])
@pytest.mark.parametrize("shape", [(2, 64, 9, 13, 40), (2, 320, 64, 64, 320), (1, 128, 17, 6, 264),
                                   (3, 640, 8, 8, 1280)])
@pytest.mark.parametrize("add", [False, True])
def test_conv3x3_implicit_gemm_vs_fp32(GE, mode, shape, add):
    """Implicit-GEMM 3×3 conv (pad 1) on channels-last fp16 against F.conv2d in fp32: stride 1,
    stride 2 (odd sizes), nearest-2× upsample folded into the addressing, bias, residual add."""
    dev = torch.device("cuda")
    n, cin, h, w, cout = shape
    g = torch.Generator(device=dev).manual_seed(cin + h + w)
    x = torch.randn(n, cin, h, w, generator=g, device=dev).half().contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, 3, 3, generator=g, device=dev) / (3 * cin ** 0.5)).half()
    b = torch.randn(cout, generator=g, device=dev).half()
    xin = x.float()
    if mode == "up2":
        xin = F.interpolate(xin, scale_factor=2.0, mode="nearest")
    ref = F.conv2d(xin, wt.float(), b.float(), stride=2 if mode == "s2" else 1, padding=1)
    r = None
    if add:
        r = torch.randn(ref.shape, generator=g, device=dev).half().contiguous(memory_format=torch.channels_last)
        ref = ref + r.float()
    m = {"s1": GE.CONV_S1, "s2": GE.CONV_S2, "up2": GE.CONV_UP2}[mode]
    y = GE.conv3x3(x, GE.conv_weight(wt), b, mode=m, r=r)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)


def test_linear_add_in_place(GE):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn(3000, 640, generator=g, device=dev).half()
    w = (torch.randn(320, 640, generator=g, device=dev) / 25).half()
    b = torch.randn(320, generator=g, device=dev).half()
    r = torch.randn(3000, 320, generator=g, device=dev).half()
    want = _ref(x, w, b) + r.float()
    out = GE.linear_add(x, w, b, r, out=r)
    assert out.data_ptr() == r.data_ptr()
    torch.testing.assert_close(r.float(), want, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("epi", ["store", "gelu", "add"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_split_k_small_grid(GE, epi, dtype):
    """Problems whose tile grid cannot fill the chip (SD1.5 deep levels: M = 128, K = 5120) run
    split-K: fp32 atomics into a workspace + a finalize pass with the same epilogue."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    m, n, k = 128, 1280, 5120
    assert GE.splits(m, n, k) > 1
    x = torch.randn(m, k, generator=g, device=dev).to(dtype)
    w = (torch.randn(n, k, generator=g, device=dev) / k ** 0.5).to(dtype)
    b = torch.randn(n, generator=g, device=dev).to(dtype)
    ref = _ref(x, w, b)
    tol = 2e-2 if dtype == torch.bfloat16 else 5e-3
    if epi == "store":
        y = GE.linear(x, w, b)
    elif epi == "gelu":
        y = GE.linear_gelu(x, w, b)
        ref = F.gelu(ref, approximate="tanh")
    else:
        r = torch.randn(m, n, generator=g, device=dev).to(dtype)
        ref = ref.to(dtype).float() + r.float()
        y = GE.linear_add(x, w, b, r)
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=2 * tol)


@pytest.mark.parametrize("gated", [False, True])
def test_split_k_gated_residual(GE, gated):
    """The LLM prefill's ffn_down shape (512 tokens, N 3584, K 18944): split-K with the fp32
    (gated) residual update in the finalize pass."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(9)
    m, n, k = 512, 3584, 18944
    assert GE.splits(m, n, k) > 1
    x = torch.randn(1, m, k, generator=g, device=dev).half()
    w = (torch.randn(n, k, generator=g, device=dev) / k ** 0.5).half()
    res = torch.randn(1, m, n, generator=g, device=dev)
    gate = torch.randn(1, n, generator=g, device=dev) if gated else None
    want = res + _ref(x, w, None).view(1, m, n) * (gate[:, None, :] if gated else 1.0)
    GE.linear_residual_(res, x, w, None, gate)
    torch.testing.assert_close(res, want, rtol=5e-3, atol=5e-3)


@pytest.mark.parametrize("m,n,k", [(512, 37888, 3584), (256, 76800, 1024), (300, 40960, 2048)])
@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_w4a_partial_last_wave_split_over_k(GE, m, n, k, bias, dtype):
    """a 256×256 grid filling the chip 1 < waves < 2 times (the LLM gate|up
    prefill GEMM at 512 tokens: 296 tiles on 256 CUs) runs its whole waves plainly and its partial
    last wave split over K on the idle CUs (16-bit partial tiles summed in fp32): the hybrid's
    plan engages and the product equals the fp32 reference."""
    dev = torch.device("cuda")
    na, ks = GE.hybrid_plan(m, n, k, GE._cus(dev))
    assert 0 < na < n and 2 <= ks <= 8, (na, ks)
    g = torch.Generator(device=dev).manual_seed(m + n)
    x = torch.randn(m, k, generator=g, device=dev).to(dtype)
    w = (torch.randn(n, k, generator=g, device=dev) / k ** 0.5).to(dtype)
    b = torch.randn(n, generator=g, device=dev).to(dtype) if bias else None
    y = GE.linear(x, w, b)
    ref = _ref(x, w, b)
    tol = 1e-2 if dtype == torch.bfloat16 else 5e-3
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    prev = GE._HYBRID
    GE._HYBRID = False
    try:
        plain = GE.linear(x, w, b)
    finally:
        GE._HYBRID = prev
    if dtype == torch.bfloat16:                 # bf16 never takes the hybrid
        assert torch.equal(y, plain)
        return
    # the split columns agree with the plain kernel's to fp16 rounding
    torch.testing.assert_close(y[:, na:].float(), plain[:, na:].float(), rtol=3e-3, atol=3e-3)
    assert torch.equal(y[:, :na], plain[:, :na])            # whole waves: the same kernel


@pytest.mark.parametrize("m,f,k", [(512, 18944, 3584), (1024, 6144, 1024), (700, 9472, 512)])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_w4a_swiglu_epilogue_equals_gemm_then_swiglu(GE, m, f, k, dtype):
    """SwiGLU in the 256×256 kernel's epilogue (tile-interleaved gate|up rows; the LLM prefill's
    gate|up at 512 tokens runs it as the hybrid, whose K-split finalize applies it too): the same
    bits as the stored [M, 2F] product followed by the swiglu_f16 pass (fp16), and the fp32
    reference to rounding."""
    from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(m + f)
    x = torch.randn(m, k, generator=g, device=dev).to(dtype)
    wg = (torch.randn(f, k, generator=g, device=dev) / k ** 0.5).to(dtype)
    wu = (torch.randn(f, k, generator=g, device=dev) / k ** 0.5).to(dtype)
    w = LK.gate_up_interleave(wg, wu)
    gate, up = LK.gate_up_split(w.float().t())
    assert torch.equal(gate, wg.float().t()) and torch.equal(up, wu.float().t())
    t = GE.linear_swiglu(x, w)
    assert t is not None and t.shape == (m, f)
    prod = GE.linear(x, w)                       # the same kernel (and plan), stored
    gp, up_ = LK.gate_up_split(prod.float())
    ref16 = (F.silu(gp) * up_)
    ref = F.silu(x.float() @ wg.float().t()) * (x.float() @ wu.float().t())
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-2
    torch.testing.assert_close(t.float(), ref, rtol=tol, atol=tol)
    torch.testing.assert_close(t.float(), ref16, rtol=tol / 4, atol=tol / 4)
    if dtype == torch.float16:                   # bit-equal to the two-pass fp16 path
        t2 = torch.empty_like(t)
        LK.swiglu_f16(prod, t2, 128)
        assert torch.equal(t, t2)
    if m == 512 and dtype == torch.float16:     # the prefill shape takes the hybrid
        assert GE.hybrid_plan(m, 2 * f, k, GE._cus(dev))[1] > 1


def test_swiglu_f16_block_layout_matches_halves(GE):
    """swiglu_f16 on the 128-block interleaved layout gives the bits of the halves layout."""
    from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

    dev = torch.device("cuda")
    p, f = 37, 384
    gate = torch.randn(p, f, device=dev).half()
    up = torch.randn(p, f, device=dev).half()
    halves = torch.cat([gate, up], 1).contiguous()
    inter = LK.gate_up_interleave(gate.t().contiguous(), up.t().contiguous()).t().contiguous()
    a, b = torch.empty(p, f, device=dev).half(), torch.empty(p, f, device=dev).half()
    LK.swiglu_f16(halves, a)
    LK.swiglu_f16(inter, b, 128)
    assert torch.equal(a, b)
    torch.testing.assert_close(a.float(), F.silu(gate.float()) * up.float(), rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("m,n,k", [(512, 4608, 3584), (512, 3584, 3584), (512, 3584, 18944),
                                   (700, 3584, 3584)])
@pytest.mark.parametrize("epi", ["store", "bias", "resid"])
def test_w4a_split_k_every_tile(GE, m, n, k, epi):
    """The LLM prefill chunk's narrow GEMMs (q|k|v, o_proj, ffn_down at 512 tokens: 28-36 tiles of
    256×256) on the 256×256 kernel with every tile split over K (16-bit partial tiles, fp32 sums in
    slice order in the finalize, which applies the epilogue): the planner engages, and store /
    + bias / += into the fp32 residual stream equal the fp32 reference (fp16)."""
    dev = torch.device("cuda")
    ks = GE.splitk_plan(m, n, k, GE._cus(dev))
    assert 2 <= ks <= 8, ks
    g = torch.Generator(device=dev).manual_seed(m * 7 + n + k)
    x = torch.randn(m, k, generator=g, device=dev).half()
    w = (torch.randn(n, k, generator=g, device=dev) / k ** 0.5).half()
    b = torch.randn(n, generator=g, device=dev).half() if epi != "store" else None
    ref = _ref(x, w, b)
    if epi == "resid":
        res = torch.randn(m, n, generator=g, device=dev)
        want = res + ref
        GE.linear_residual_(res, x, w, b)
        torch.testing.assert_close(res, want, rtol=5e-3, atol=5e-3)
        return
    y = GE.linear(x, w, b)
    torch.testing.assert_close(y.float(), ref, rtol=5e-3, atol=5e-3)
    # deterministic: the slices are summed in a fixed order
    assert torch.equal(y, GE.linear(x, w, b))
    # a pinned wave-grid tile keeps the shape off the split form (the A/B contract of set_tile)
    GE.set_tile(0)
    try:
        y2 = GE.linear(x, w, b)
    finally:
        GE.set_tile(-1)
    torch.testing.assert_close(y2.float(), ref, rtol=5e-3, atol=5e-3)


@pytest.mark.parametrize("k", [3584, 18944])
def test_w4a_split_k_residual_with_fused_rmsnorm(GE, k):
    """The prefill chunk's o_proj / ffn_down: the split-K finalize adds the product into the fp32
    residual stream and writes the next RMSNorm's fp16 rows in the same pass — the same bits as
    the residual GEMM followed by rmsnorm_f16."""
    from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

    dev = torch.device("cuda")
    m, n = 512, 3584
    g = torch.Generator(device=dev).manual_seed(k)
    x = torch.randn(m, k, generator=g, device=dev).half()
    w = (torch.randn(n, k, generator=g, device=dev) / k ** 0.5).half()
    res = torch.randn(m, n, generator=g, device=dev)
    nw = torch.rand(n, generator=g, device=dev) + 0.5
    r1, y1 = res.clone(), torch.empty(m, n, device=dev, dtype=torch.float16)
    assert GE.linear_residual_norm_(r1, x, w, nw, 1e-6, y1)
    r2, y2 = res.clone(), torch.empty(m, n, device=dev, dtype=torch.float16)
    GE.linear_residual_(r2, x, w)
    LK.rmsnorm_f16(r2, nw, 1e-6, y2)
    assert torch.equal(r1, r2)
    assert torch.equal(y1, y2)
    want = res + _ref(x, w, None)
    torch.testing.assert_close(r1, want, rtol=5e-3, atol=5e-3)
    # a shape the split form does not take: nothing done, the caller runs the two passes
    big = torch.randn(4096, k, generator=g, device=dev).half()
    rb = torch.zeros(4096, n, device=dev)
    assert not GE.linear_residual_norm_(rb, big, w, nw, 1e-6, torch.empty_like(rb).half())
    assert int(rb.abs().sum()) == 0
