"""The partition-aware GEMM tile order (ops/csrc/tile_order.h), checked on the host: the real
header compiled by hipcc, its block_tile() run on the CPU for 1/2/4/8-XCD partitions."""
import shutil
import subprocess

import pytest

from k8s_nvidia_gpus_amd.ops import build as B

pytestmark = pytest.mark.skipif(not B.toolchain_available(), reason="hipcc not available")


def test_tile_order_covers_every_tile_once_per_partition(tmp_path):
    exe = tmp_path / "tile_order_check"
    subprocess.run([B.HIPCC, f"--offload-arch={B.OFFLOAD_ARCH}", "-O2", "-std=c++17", f"-I{B.CSRC_DIR}",
                    str(B.NATIVE_DIR / "tests" / "tile_order_check.hip"), "-o", str(exe)],
                   check=True, capture_output=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and p.stdout.strip() == "tile order OK", p.stdout + p.stderr
