"""CPU-side checks that every native artefact builds for gfx950 and exports its C ABI."""
import json
import os
import subprocess

import pytest

from k8s_nvidia_gpus_amd.ops import build as B

pytestmark = pytest.mark.skipif(not B.toolchain_available(), reason="hipcc not available")


@pytest.fixture(scope="module")
def built():
    B.build_all(jobs=4)
    return True


def _nm(path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_kernel_library_exports(built):
    syms = _nm(B.KERNEL_LIB)
    for s in ["amdk8s_gemm_bf16_nt", "amdk8s_gemm_bf16_nt_sample_check", "amdk8s_vector_add_f32",
              "amdk8s_vector_add_f32_bw", "amdk8s_fill_uniform_bf16", "amdk8s_vector_add_blocks",
              "amdk8s_hbm_stream", "amdk8s_hbm_stream_variant", "amdk8s_fp32_fma", "amdk8s_fp64_mfma",
              "amdk8s_gemm_f16_nt_w4a"]:
        assert s in syms, s


def test_sd_kernel_bindings_resolve_in_the_library(built):
    """Every C symbol the SD1.5 bindings declare (ops/sd_kernels.py) is exported."""
    import re

    syms = _nm(B.KERNEL_LIB)
    src = (B.PKG_DIR / "sd_kernels.py").read_text()
    names = set(re.findall(r"lib\.(amdk8s_\w+)\.argtypes", src))
    assert len(names) >= 8
    assert names <= syms, names - syms


def test_kernel_library_targets_gfx950_only(built):
    blob = B.KERNEL_LIB.read_bytes()
    assert b"gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"gfx1100", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in blob


def test_native_tools_built(built):
    for t in B.NATIVE_TARGETS:
        p = B.NATIVE_BIN / t.name
        assert p.exists() and os.access(p, os.X_OK), p


def test_gemm_kernel_resource_budget(tmp_path):
    """The main loop must fit 2 waves/SIMD (≤256 VGPRs), never spill, and stay within 160 KiB LDS."""
    src = B.CSRC_DIR / "gemm_bf16_gfx950.hip"
    r = subprocess.run([B.HIPCC, *B.HIP_FLAGS, "-c", str(src), "-o", str(tmp_path / "g.o"),
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    text = r.stderr
    block = text.split("Function Name: amdk8s_gemm_bf16_nt_256x256")[1].split("Function Name:")[0]

    def val(key):
        line = [ln for ln in block.splitlines() if key in ln][0]
        return int(line.split(key)[1].split()[0])

    assert val("VGPRs:") <= 256
    assert val("VGPRs Spill:") == 0
    assert val("ScratchSize [bytes/lane]:") == 0
    assert val("LDS Size [bytes/block]:") <= 160 * 1024
    assert val("Occupancy [waves/SIMD]:") >= 2


def test_kfd_probe_help(built):
    r = subprocess.run([str(B.NATIVE_BIN / "kfd-probe"), "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "usage" in r.stdout


def test_kfd_probe_reports_missing_topology(built, tmp_path):
    r = subprocess.run([str(B.NATIVE_BIN / "kfd-probe"), "--sysfs-root", str(tmp_path / "none"),
                        "--dev-root", str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 1
    assert "not ready" in r.stderr


def test_proftester_lists_tests_and_rejects_unknown_without_a_gpu(built):
    exe = str(B.NATIVE_BIN / "amd-proftester")
    p = subprocess.run([exe, "--list"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0
    assert p.stdout.split() == ["tensor", "tensor-fp16", "tensor-fp8", "hbm-read", "hbm-write", "hbm-copy", "fp32",
                                "fp64", "pcie-h2d", "pcie-d2h", "xgmi"]
    p = subprocess.run([exe, "-t", "hbm-copy,bogus"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "unknown test 'bogus'" in p.stderr


def test_loadgen_kernels_use_the_intended_instructions(tmp_path):
    """The fp32 load must be v_pk_fma_f32 (the 157 TF vector path), the fp64 load the f64 MFMA,
    and the streaming kernels 16-B-per-lane accesses, non-temporal where the policy says so."""
    src = B.CSRC_DIR / "loadgen.hip"
    subprocess.run([B.HIPCC, *B.HIP_FLAGS, "--save-temps", "-c", str(src), "-o", str(tmp_path / "l.o")],
                   cwd=tmp_path, check=True, capture_output=True)
    (asm,) = tmp_path.glob("*gfx950*.s")
    text = asm.read_text()
    assert text.count("v_pk_fma_f32") >= 32 and text.count("v_mfma_f64_16x16x4") >= 16
    assert "global_load_dwordx4" in text and "global_store_dwordx4" in text
    assert " nt" in text and "scratch_" not in text


def test_kernel_library_override_is_loaded_as_named(tmp_path, monkeypatch):
    """AMDK8S_KERNEL_LIB (A/B builds of the same sources, e.g. -DAMDK8S_ATTN_PARTS=...) is loaded
    as given — never rebuilt over, and a missing file is an error, not a silent fallback."""
    from k8s_nvidia_gpus_amd.ops import kernels as K

    monkeypatch.setattr(K, "_lib", None)
    monkeypatch.setenv("AMDK8S_KERNEL_LIB", str(tmp_path / "missing.so"))
    calls = []
    monkeypatch.setattr(K._build, "build_kernel_library", lambda *a, **k: calls.append(1))
    with pytest.raises(K.KernelLibraryError):
        K.library()
    assert not calls
    monkeypatch.setattr(K, "_lib", None)


def test_attention_build_knobs_default_to_the_measured_choice():
    """The decode-attention A/B knobs (llm_attn.hip) default to what the round-5 sweeps chose:
    64 partials per head, a 2-deep chunk ring, 4 waves per workgroup, the one-chunk fast path."""
    src = (B.CSRC_DIR / "llm_attn.hip").read_text()
    for knob, val in [("AMDK8S_ATTN_PARTS", "64"), ("AMDK8S_ATTN_RING", "2"),
                      ("AMDK8S_ATTN_WAVES", "4"), ("AMDK8S_ATTN_FAST1", "1"),
                      ("AMDK8S_ATTN_WPE", "1")]:
        assert f"#define {knob} {val}\n" in src, knob
