"""Numerics of the hand-written gfx950 kernels against plain PyTorch fp32 references (MI355X)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from k8s_nvidia_gpus_amd.ops import kernels

    kernels.library()  # must load the in-tree .so — no fallback
    return kernels


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda", 0)


def _rand_bf16(shape, gen, dev):
    return (torch.rand(shape, generator=gen, device=dev) * 2 - 1).to(torch.bfloat16)


def test_vector_add_reference_shape(K, dev):
    n = 50000
    a = torch.rand(n, device=dev)
    b = torch.rand(n, device=dev)
    c = K.vector_add(a, b)
    assert K.vector_add_blocks(n) == 196
    torch.testing.assert_close(c, a + b, rtol=0, atol=0)


def test_vector_add_bandwidth_form(K, dev):
    n = 1 << 22
    a = torch.rand(n, device=dev)
    b = torch.rand(n, device=dev)
    c = torch.empty_like(a)
    K.vector_add_bandwidth(a, b, c)
    torch.testing.assert_close(c, a + b, rtol=0, atol=0)


@pytest.mark.parametrize("variant", ["w8", "w4", "w4a", "auto"])
@pytest.mark.parametrize("m,n,k", [
    (256, 256, 64),      # one K-tile: prologue-only path
    (256, 256, 128),     # two K-tiles: tail-only path
    (256, 512, 192),     # three K-tiles: one steady tile
    (512, 768, 320),     # rectangular, odd tile counts
    (768, 256, 1024),
    (1024, 1024, 4096),  # long K: steady-state vmcnt(8) pipeline
    (2304, 1280, 576),   # nwg % 8 != 0: bijective XCD remap + ragged GROUP_M tail
])
def test_gemm_bf16_nt_matches_fp32(K, dev, m, n, k, variant):
    g = torch.Generator(device=dev).manual_seed(m * 131 + n * 7 + k)
    a = _rand_bf16((m, k), g, dev)
    b = _rand_bf16((n, k), g, dev)
    c = K.gemm_bf16_nt(a, b, variant=variant)
    ref = a.float() @ b.float().t()
    # bf16 output rounding (2^-8 relative) + fp32 accumulation-order differences
    torch.testing.assert_close(c.float(), ref, rtol=1e-2, atol=1e-2 * (k ** 0.5) / 8)


@pytest.mark.parametrize("variant", ["w8", "w4", "w4a", "auto"])
def test_gemm_identity_asymmetric(K, dev, variant):
    """A = I with an asymmetric B must return exactly Bᵀ: catches any row/col swap in C."""
    s = 256
    a = torch.eye(s, device=dev, dtype=torch.bfloat16)
    i = torch.arange(s, device=dev, dtype=torch.float32)
    b = ((i[:, None] * 3 + i[None, :] * 0.5) / 64).to(torch.bfloat16)  # asymmetric, exact in bf16
    c = K.gemm_bf16_nt(a, b, variant=variant)
    assert torch.equal(c, b.t().contiguous())
    c2 = K.gemm_bf16_nt(b, a, variant=variant)  # = B · Iᵀ = B
    assert torch.equal(c2, b)


@pytest.mark.parametrize("variant", ["w8", "w4", "w4a", "auto"])
def test_gemm_strided_leading_dims(K, dev, variant):
    g = torch.Generator(device=dev).manual_seed(3)
    big_a = _rand_bf16((512, 640), g, dev)
    big_b = _rand_bf16((256, 704), g, dev)
    a = big_a[:, 64:576]   # lda = 640, K = 512
    b = big_b[:, 128:640]  # ldb = 704
    out = torch.empty((512, 384), device=dev, dtype=torch.bfloat16)[:, :256]
    K.gemm_bf16_nt(a, b, out=out, variant=variant)
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=3e-2)


@pytest.mark.parametrize("variant", ["w8", "w4", "w4a", "auto"])
def test_gemm_deterministic(K, dev, variant):
    g = torch.Generator(device=dev).manual_seed(11)
    a = _rand_bf16((1024, 2048), g, dev)
    b = _rand_bf16((1024, 2048), g, dev)
    c1 = K.gemm_bf16_nt(a, b, variant=variant).clone()
    for _ in range(5):
        assert torch.equal(K.gemm_bf16_nt(a, b, variant=variant), c1)


def test_gemm_variants_agree_bitwise_at_8192(K, dev):
    """All variants accumulate each output in the same K order → identical bits."""
    g = torch.Generator(device=dev).manual_seed(21)
    a = _rand_bf16((2048, 8192), g, dev)
    b = _rand_bf16((2048, 8192), g, dev)
    c8 = K.gemm_bf16_nt(a, b, variant="w8")
    assert torch.equal(c8, K.gemm_bf16_nt(a, b, variant="w4"))
    assert torch.equal(c8, K.gemm_bf16_nt(a, b, variant="w4a"))


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (256, 256, 128), (512, 256, 192),
                                   (768, 512, 1024), (4096, 4096, 640), (8192, 4096, 192)])
def test_gemm_w4a_matches_fp32_and_w4(K, dev, m, n, k):
    """The generated-assembly K-loop against an fp32 reference and bit-for-bit against hipcc's w4
    (T = 1: clamped restage into the read buffer; T = 2/3: odd tail of the parity-unrolled loop;
    4096² and 8192×4096: super-block order), written over a NaN-filled output."""
    g = torch.Generator(device=dev).manual_seed(43 + m + k)
    a = _rand_bf16((m, k), g, dev)
    b = _rand_bf16((n, k), g, dev)
    c = torch.full((m, n), float("nan"), dtype=torch.bfloat16, device=dev)
    K.gemm_bf16_nt(a, b, out=c, variant="w4a")
    assert not torch.isnan(c.float()).any()
    assert torch.equal(c, K.gemm_bf16_nt(a, b, variant="w4"))
    rows, cols = min(m, 512), min(n, 256)
    ref = a[:rows].float() @ b[:cols].float().t()
    torch.testing.assert_close(c[:rows, :cols].float(), ref, rtol=1e-2, atol=1e-2 * (k ** 0.5) / 8)


def test_gemm_auto_picks_generated_assembly_kernel(K):
    assert K.pick_gemm_variant(8192, 8192, 8192) == "w4a"
    assert K.pick_gemm_variant(256, 256, 1 << 22) == "w4"   # panel past 32-bit buffer offsets


def test_gemm_padded_general_shapes(K, dev):
    g = torch.Generator(device=dev).manual_seed(5)
    a = _rand_bf16((300, 100), g, dev)
    w = _rand_bf16((77, 100), g, dev)
    y = K.gemm_bf16(a, w)
    torch.testing.assert_close(y.float(), a.float() @ w.float().t(), rtol=1e-2, atol=2e-2)
    bkn = _rand_bf16((100, 130), g, dev)
    y2 = K.gemm_bf16(a, bkn, b_layout="kn")
    torch.testing.assert_close(y2.float(), a.float() @ bkn.float(), rtol=1e-2, atol=2e-2)


def test_gemm_rejects_bad_shapes(K, dev):
    a = torch.zeros((200, 64), device=dev, dtype=torch.bfloat16)
    b = torch.zeros((256, 64), device=dev, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        K.gemm_bf16_nt(a, b)


def test_sample_check_matches_torch(K, dev):
    g = torch.Generator(device=dev).manual_seed(9)
    a = _rand_bf16((512, 1024), g, dev)
    b = _rand_bf16((256, 1024), g, dev)
    coords = torch.tensor([[0, 0], [511, 255], [17, 200], [300, 3]], dtype=torch.int32)
    ref = K.gemm_sample_check(a, b, coords)
    full = a.float() @ b.float().t()
    exp = full[coords[:, 0].long(), coords[:, 1].long()]
    torch.testing.assert_close(ref, exp, rtol=1e-4, atol=1e-3)


def test_fill_uniform_bf16(K, dev):
    t = torch.empty(1 << 20, device=dev, dtype=torch.bfloat16)
    K.fill_uniform_bf16(t, seed=123)
    f = t.float()
    assert f.min().item() >= -1.0 and f.max().item() <= 1.0
    assert abs(f.mean().item()) < 0.01
    assert 0.3 < f.std().item() < 0.7  # uniform[-1,1) std = 0.577
    t2 = torch.empty_like(t)
    K.fill_uniform_bf16(t2, seed=123)
    assert torch.equal(t, t2)


@pytest.mark.parametrize("superblock", ["1", "0"])
def test_gemm_w4_superblock_order_matches_w8(K, dev, superblock, monkeypatch):
    """4096x4096 tiles (16x16 grid) take the super-block order in w4; output must not change."""
    monkeypatch.setenv("AMDK8S_W4_SUPERBLOCK", superblock)
    g = torch.Generator(device=dev).manual_seed(31)
    a = _rand_bf16((4096, 512), g, dev)
    b = _rand_bf16((4096, 512), g, dev)
    c4 = K.gemm_bf16_nt(a, b, variant="w4")
    c8 = K.gemm_bf16_nt(a, b, variant="w8")
    assert torch.equal(c4, c8)
    ref = a[:512].float() @ b[:256].float().t()
    torch.testing.assert_close(c4[:512, :256].float(), ref, rtol=1e-2, atol=3e-2)


@pytest.mark.parametrize("schedule", ["interleaved", "region"])
@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (256, 256, 128), (512, 256, 192),
                                   (768, 512, 1024), (4096, 4096, 640)])
def test_gemm_w4_schedules_match_fp32_and_w8(K, dev, schedule, m, n, k, monkeypatch):
    """Both w4 schedules (forced) against an fp32 reference and bit-for-bit against w8 (k = 64 is
    a single K-tile — the clamped restage and the unused "tile T" reads —, 192 an odd count)."""
    monkeypatch.setenv("AMDK8S_W4_SCHEDULE", schedule)
    g = torch.Generator(device=dev).manual_seed(41 + m + k)
    a = _rand_bf16((m, k), g, dev)
    b = _rand_bf16((n, k), g, dev)
    c4 = K.gemm_bf16_nt(a, b, variant="w4")
    assert torch.equal(c4, K.gemm_bf16_nt(a, b, variant="w8"))
    rows, cols = min(m, 512), min(n, 256)
    ref = a[:rows].float() @ b[:cols].float().t()
    torch.testing.assert_close(c4[:rows, :cols].float(), ref, rtol=1e-2, atol=1e-2 * (k ** 0.5) / 8)


@pytest.mark.parametrize("schedule", ["region"])
def test_gemm_w4_schedule_repeatable_under_load(K, dev, schedule, monkeypatch):
    """The region schedule's DMA/read phases are ordered only by counted waits + barriers:
    repeat a large grid several times and require identical bits every time (a race shows up as
    drift)."""
    monkeypatch.setenv("AMDK8S_W4_SCHEDULE", schedule)
    g = torch.Generator(device=dev).manual_seed(77)
    a = _rand_bf16((4096, 2048), g, dev)
    b = _rand_bf16((4096, 2048), g, dev)
    c0 = K.gemm_bf16_nt(a, b, variant="w4").clone()
    for _ in range(8):
        assert torch.equal(K.gemm_bf16_nt(a, b, variant="w4"), c0)
    monkeypatch.setenv("AMDK8S_W4_SCHEDULE", "interleaved")
    assert torch.equal(K.gemm_bf16_nt(a, b, variant="w4"), c0)



@pytest.mark.parametrize("m,n,k", [(256, 256, 256), (512, 256, 768), (768, 512, 2048),
                                   (4096, 4096, 512), (2304, 1280, 1024)])
def test_gemm_fp8_matches_fp32(K, dev, m, n, k):
    """fp8 e4m3 GEMM against an fp32 matmul of the same (exactly representable) fp8 values; the
    generated-assembly f8a kernel (default) and the hipcc-scheduled one give identical bits."""
    a = K.uniform_fp8((m, k), seed=m + 3 * k, device=dev)
    b = K.uniform_fp8((n, k), seed=n + 5 * k, device=dev)
    c = torch.full((m, n), float("nan"), dtype=torch.bfloat16, device=dev)
    K.gemm_fp8_nt(a, b, out=c)
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(c.float(), ref, rtol=1e-2, atol=1e-2 * (k ** 0.5) / 8)
    assert torch.equal(K.gemm_fp8_nt(a, b), c)  # deterministic
    assert torch.equal(K.gemm_fp8_nt(a, b, variant="hipcc"), c)


def test_gemm_fp8_identity_asymmetric(K, dev):
    """A = I (exact in e4m3) with an asymmetric small-integer B returns Bᵀ exactly."""
    s = 256
    a = torch.eye(s, device=dev).to(K.FP8_DTYPE)
    i = torch.arange(s, device=dev)
    b = ((i[:, None] * 3 + i[None, :]) % 17 - 8).float().to(K.FP8_DTYPE)  # |v| ≤ 8: exact
    c = K.gemm_fp8_nt(a, b)
    assert torch.equal(c.float(), b.float().t())


def test_gemm_fp8_rejects_bad_shapes(K, dev):
    a = torch.zeros((256, 128), device=dev).to(K.FP8_DTYPE)
    with pytest.raises(ValueError):
        K.gemm_fp8_nt(a, a)  # K % 256 != 0
    with pytest.raises(TypeError):
        K.gemm_fp8_nt(a.float(), a.float())


def test_fill_uniform_fp8_is_ocp_e4m3(K, dev):
    """The device fill's bytes decode (as torch.float8_e4m3fn) to the e4m3 rounding of values in
    [-1, 1): the in-kernel v_cvt_pk_fp8_f32 produces OCP e4m3, the format the GEMM assumes."""
    t = K.uniform_fp8((1024, 1024), seed=5, device=dev)
    f = t.float()
    assert f.min().item() >= -1.0 and f.max().item() <= 1.0
    assert abs(f.mean().item()) < 0.01 and 0.5 < f.std().item() < 0.65
    assert torch.equal(f.to(K.FP8_DTYPE).float(), f)  # every value is an e4m3 value
    assert len(torch.unique(f)) > 100


# ----------------------------------------------------------------------------- load generators
def test_hbm_copy_is_exact_and_read_write_run(K, dev):
    n = (256 << 20) // 4 + 12  # 256 MiB + a 48-B tail past the unrolled body
    src = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)
    dst = torch.zeros_like(src)
    assert K.hbm_stream("copy", src, dst) == 2 * n * 4
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    for variant in [(0, 0, 1, 0), (1, 1, 8, 1), (1, 0, 2, 1), (0, 1, 4, 0)]:
        dst.zero_()
        K.hbm_stream("copy", src, dst, variant=variant)
        torch.cuda.synchronize()
        assert torch.equal(dst, src), variant
    w = torch.zeros_like(src)
    K.hbm_stream("write", None, w)
    torch.cuda.synchronize()
    assert (w != 0).float().mean().item() > 0.99  # the toggling pattern, never zeros
    K.hbm_stream("read", src, None)
    torch.cuda.synchronize()
    assert int(K._sink(dev)[0].item()) == 0  # the keep-alive store never fires


def test_hbm_bandwidth_floors(K, dev):
    nbytes = 2 << 30
    src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    dst = torch.empty_like(src)
    K.hbm_stream("write", None, src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rates = {}
    for mode in ("read", "write", "copy"):
        s, d = (src if mode != "write" else None), (dst if mode != "read" else None)
        for _ in range(3):
            K.hbm_stream(mode, s, d)
        e0.record()
        moved = sum(K.hbm_stream(mode, s, d) for _ in range(10))
        e1.record()
        e1.synchronize()
        rates[mode] = moved / (e0.elapsed_time(e1) * 1e-3) / 1e9
    # measured 6.0-7.1 / 4.4-5.9 / 4.8-5.5 TB/s (profiles/r02_session1/hbm_sweep*.txt); floors at ~70 %
    assert rates["read"] > 4500 and rates["write"] > 3500 and rates["copy"] > 3500, rates


def test_fp32_and_fp64_loads(K, dev):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    K.fp32_fma(dev, iters=2000)
    e0.record()
    flop = sum(K.fp32_fma(dev, iters=5000) for _ in range(5))
    e1.record()
    e1.synchronize()
    tf32 = flop / (e0.elapsed_time(e1) * 1e-3) / 1e12
    K.fp64_mfma(dev, iters=500)
    e0.record()
    flop = sum(K.fp64_mfma(dev, iters=1500) for _ in range(5))
    e1.record()
    e1.synchronize()
    tf64 = flop / (e0.elapsed_time(e1) * 1e-3) / 1e12
    # 157.3 TF fp32 vector / 78.6 TF fp64 matrix peaks; measured 124 / 68 (proftester_all.log)
    assert 80 < tf32 < 160 and 40 < tf64 < 80, (tf32, tf64)
    assert int(K._sink(dev)[0].item()) == 0


def test_proftester_native_protocol():
    import json
    import subprocess

    from k8s_nvidia_gpus_amd.ops import build as B

    p = subprocess.run([str(B.NATIVE_BIN / "amd-proftester"), "-t", "1005,1006,1007,1008,1010,xgmi",
                        "--iters", "5", "--settle-ms", "20", "--hbm-bytes", "1G", "--json"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    docs = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert {d["test"] for d in docs} == {"hbm-copy", "fp64", "fp32", "tensor-fp16", "pcie-h2d", "xgmi"}
    assert all(d["passed"] for d in docs)
    assert p.stdout.rstrip().endswith("Test PASSED\nDone")


@pytest.mark.parametrize("xcds", ["1", "2", "4", "8"])
@pytest.mark.parametrize("m,n,k", [(8192, 4096, 256), (2304, 1280, 320)])  # super-block / GROUP_M grids
def test_gemm_tile_order_per_partition_is_bitwise_identical(K, dev, xcds, m, n, k, monkeypatch):
    """CPX/DPX/QPX tile orders (tile_order.h, forced with AMDK8S_GEMM_XCDS on this SPX device) cover
    every tile exactly once: bit-identical C to the SPX order, for bf16 w4a/w4 and fp8 f8a."""
    g = torch.Generator(device=dev).manual_seed(5)
    a = _rand_bf16((m, k), g, dev)
    b = _rand_bf16((n, k), g, dev)
    monkeypatch.delenv("AMDK8S_GEMM_XCDS", raising=False)
    ref = {v: K.gemm_bf16_nt(a, b, variant=v) for v in ("w4a", "w4")}
    a8 = K.uniform_fp8((m, 512), seed=3, device=dev)
    b8 = K.uniform_fp8((n, 512), seed=4, device=dev)
    ref8 = K.gemm_fp8_nt(a8, b8)
    monkeypatch.setenv("AMDK8S_GEMM_XCDS", xcds)
    for v, r in ref.items():
        out = torch.full((m, n), float("nan"), dtype=torch.bfloat16, device=dev)
        K.gemm_bf16_nt(a, b, out=out, variant=v)
        assert torch.equal(out, r), (v, xcds)
    out8 = torch.full((m, n), float("nan"), dtype=torch.bfloat16, device=dev)
    K.gemm_fp8_nt(a8, b8, out=out8)
    assert torch.equal(out8, ref8), xcds


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (512, 768, 320), (2304, 1280, 1024), (4096, 4096, 4096)])
def test_gemm_f16_matches_fp32(K, dev, m, n, k):
    g = torch.Generator(device=dev).manual_seed(11)
    a = (torch.rand((m, k), generator=g, device=dev) * 2 - 1).half()
    b = (torch.rand((n, k), generator=g, device=dev) * 2 - 1).half()
    out = torch.full((m, n), float("nan"), dtype=torch.float16, device=dev)
    K.gemm_f16_nt(a, b, out=out)
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(out.float(), ref, rtol=2e-3, atol=2e-3 * (k ** 0.5))
    # the fp16 kernel is the bf16 kernel's loop: identical sums, only the operand format differs
    ab, bb = a.to(torch.bfloat16), b.to(torch.bfloat16)
    assert torch.isfinite(K.gemm_bf16_nt(ab, bb, variant="w4a").float()).all()


def test_gemm_f16_rejects_bad_dtype_and_shape(K, dev):
    a = torch.zeros((256, 64), dtype=torch.bfloat16, device=dev)
    with pytest.raises(TypeError):
        K.gemm_f16_nt(a, a)
    h = torch.zeros((256, 96), dtype=torch.float16, device=dev)
    with pytest.raises(ValueError):
        K.gemm_f16_nt(h, h)
