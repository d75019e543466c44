#!/usr/bin/env python3
"""Numerics gate for the generated-assembly fp8 kernel (f8a) before timing it.

For each shape: NaN-filled output, bit-equality with the hipcc-scheduled fp8 kernel (same per-lane
MFMA order), and the error against an fp32 matmul of the same e4m3 values.
usage: python tools/gemm_fp8_check.py
"""
import sys

import torch

sys.path.insert(0, ".")
from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402

SHAPES = [(256, 256, 256), (4096, 4096, 256), (8192, 8192, 256), (8192, 4096, 768),
          (768, 512, 2048), (12288, 12288, 1024), (8192, 8192, 8192)]


def main() -> int:
    dev = torch.device("cuda", 0)
    ok = True
    for (m, n, k) in SHAPES:
        a = K.uniform_fp8((m, k), 3, dev)
        b = K.uniform_fp8((n, k), 4, dev)
        c = torch.full((m, n), float("nan"), dtype=torch.bfloat16, device=dev)
        K.gemm_fp8_nt(a, b, out=c, variant="f8a")
        ch = K.gemm_fp8_nt(a, b, variant="hipcc")
        rows, cols = min(m, 1024), min(n, 1024)
        ref = a[:rows].float() @ b[:cols].float().t()
        err = (c[:rows, :cols].float() - ref).abs().max().item()
        same = torch.equal(c, ch)
        nan = bool(torch.isnan(c.float()).any().item())
        good = (not nan) and same and err < 0.05 * (k ** 0.5) / 8 + 0.05
        ok &= good
        print(f"{m}x{n}x{k}: max_abs_err {err:.4f} equal_to_hipcc {same} nan {nan} "
              f"{'ok' if good else 'FAIL'}", flush=True)
    print("ALL OK" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
