"""CPU tests of the wave-grid GEMM launch planner (``amdk8s_gemm_epi_plan`` in
``ops/csrc/gemm_bf16_epi.hip``) and the wide-projection routing rule (``gemm_epi.use_w4a``).

The planner is host code in the kernel library, so it runs here without a GPU: the tests pin the
measured decisions (profiles/r03/e, h, o — see docs/gemm_tuning.md) on the shapes that motivated
them, and check the native planner against an independent Python statement of its rules over a
grid of shapes, so a change to one without the other fails.
"""
import itertools

import pytest
import torch

from k8s_nvidia_gpus_amd.ops import gemm_epi as GE
from k8s_nvidia_gpus_amd.ops.kernels import KernelLibraryError


@pytest.fixture(scope="module")
def ge():
    try:
        GE.set_tile(-1)
        GE.set_splits(-1)
    except (KernelLibraryError, OSError) as e:  # no toolchain and no prebuilt library
        pytest.skip(f"kernel library unavailable: {e}")
    yield GE
    GE.set_tile(-1)
    GE.set_splits(-1)


def _grid(t, m, n):
    tm, tn = GE.TILES[t]
    return -(-m // tm) * -(-n // tn)


def _model(m, n, k):
    """The planner's rules, restated: 8-/4-wave tile with >= 160 WGs unsplit; else the largest tile
    that reaches 192 WGs with >= 8 K-tiles per split (<= 16 splits); else 64x64, max splits."""
    kt = k // 64
    if m <= 1024 and 2048 <= n <= 8192 and 2048 <= k <= 4096:   # narrow prefill projections
        g = _grid(2, m, n)
        return GE.TILES[2], 1 if g >= 256 else max(1, min(-(-384 // g), 8, kt // 8, 16))
    for t in (0, 1):
        if _grid(t, m, n) >= 160:
            return GE.TILES[t], 1
    for t in range(4):
        need = -(-192 // _grid(t, m, n))
        if need <= 16 and kt // need >= 8:
            return GE.TILES[t], need
    need = -(-192 // _grid(3, m, n))
    return GE.TILES[3], max(1, min(need, kt // 8, 16))


@pytest.mark.parametrize("shape,expect", [
    ((8192, 1536, 1536), ((256, 128), 1)),    # Wan-1.3B o-proj, CFG x 2 x 4096 tokens
    ((128, 1280, 1280), ((64, 64), 2)),       # SD time embedding: tiny M, split K
    ((8192, 320, 2880), ((128, 128), 1)),     # SD 64^2 conv (implicit GEMM), 192 tiles unsplit
    ((2048, 640, 5760), ((256, 128), 5)),     # SD 32^2 conv: 80 big tiles x 5 splits
    ((512, 3584, 18944), ((256, 128), 4)),    # LLM prefill FFN down, 512-token chunk
    ((512, 4608, 3584), ((128, 64), 1)),      # LLM prefill q|k|v, 512-token chunk (r06 sweep)
    ((512, 3584, 3584), ((128, 64), 2)),      # LLM prefill o_proj
    ((128, 4608, 3584), ((128, 64), 6)),      # q|k|v of a 128-token chunk
])
def test_plan_measured_shapes(ge, shape, expect):
    assert ge.plan(*shape) == expect


def test_plan_matches_rules(ge):
    ms = (1, 16, 128, 300, 512, 2048, 5120, 8192, 32768)
    ns = (8, 64, 320, 640, 1280, 1536, 3072, 8960)
    ks = (64, 256, 512, 1536, 5760, 18944)
    for m, n, k in itertools.product(ms, ns, ks):
        assert ge.plan(m, n, k) == _model(m, n, k), (m, n, k)


def test_split_never_below_pipeline_depth(ge):
    # every split keeps >= 8 K-tiles (the 3-stage ring's depth) unless K itself is that short
    for m, n, k in itertools.product((16, 256, 1024), (64, 512, 1280), (512, 1024, 4096, 16384)):
        (_, _), sp = ge.plan(m, n, k)
        assert 1 <= sp <= 16
        if sp > 1:
            assert (k // 64) // sp >= 8


def test_overrides(ge):
    try:
        ge.set_tile(2)
        t, sp = ge.plan(8192, 1536, 1536)
        assert t == (128, 64) and sp == 1            # 1152 WGs: no split needed
        ge.set_splits(3)
        assert ge.plan(8192, 1536, 1536) == ((128, 64), 3)
        ge.set_splits(64)                             # clamped to the number of K-tiles
        assert ge.plan(64, 64, 256)[1] == 4
    finally:
        ge.set_tile(-1)
        ge.set_splits(-1)
    assert ge.plan(8192, 1536, 1536) == ((256, 128), 1)


def test_use_w4a_routing():
    # wide projections with N % 256 and enough 256x256 tiles go to the w4a kernel
    assert GE.use_w4a(5120, 4608, 1536, torch.bfloat16)        # Wan QKV at 2 x 2560 tokens
    assert GE.use_w4a(5120, 4608, 1536, torch.float16)
    assert not GE.use_w4a(5120, 4608, 1536, torch.float32)     # fp32 operands: not this kernel
    assert not GE.use_w4a(5120, 1540, 1536, torch.bfloat16)    # N % 256
    assert not GE.use_w4a(5120, 4608, 1500, torch.bfloat16)    # K % 64
    assert not GE.use_w4a(512, 1536, 1536, torch.bfloat16)     # 2 x 6 tiles: far from filling
    # 3/4 of a wave and up (LLM prefill q|k|v and o_proj at 3584 tokens: 252 / 196 tiles)
    assert GE.use_w4a(3584, 4608, 3584, torch.float16) and GE.use_w4a(3584, 3584, 3584, torch.float16)
    assert not GE.use_w4a(2560, 4608, 3584, torch.float16)     # 10 x 18 = 180 tiles


@pytest.mark.parametrize("shape,ks", [
    ((512, 4608, 3584), 7),      # LLM prefill q|k|v chunk: 36 tiles x 7 slices
    ((512, 3584, 3584), 8),      # o_proj: 28 x 8
    ((512, 3584, 18944), 8),     # ffn_down: 28 x 8
    ((300, 1536, 1536), 1),      # 12 tiles x 4 slices: the split grid would not fill the chip
    ((700, 3584, 3584), 6),      # 42 tiles (M tail) x 6
    ((256, 3584, 18944), 1),     # 14 tiles x 8 = 112 workgroups: the wave-grid family wins
    ((8192, 1536, 1536), 1),     # 192 tiles fill 3/4 of the chip: plain
    ((512, 37888, 3584), 1),     # gate|up: 296 tiles (the hybrid's case)
    ((128, 4608, 3584), 1),      # below one 256-row panel: the wave-grid family
    ((512, 4608, 320), 1),       # 5 K-tiles: nothing to split
])
def test_w4a_splitk_plan(ge, shape, ks):
    """Split-K over every 256×256 tile (amdk8s_gemm_w4a_splitk_plan): slices fill the chip, at
    most 8 (16-bit partial tiles), at least 6 K-tiles each, only when the plain grid is < 3/4 of
    the chip and the split grid >= 3/4."""
    assert ge.splitk_plan(*shape) == ks
